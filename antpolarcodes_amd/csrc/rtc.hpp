// rtc.hpp -- plan-specialised kernels compiled at run time (rtc.cpp).
#pragma once
#include "kernels.hpp"
#include "plan.hpp"

#include <string>
#include <vector>

namespace pcg {
// The hiprtc source of a Fast-SSC plan's specialised scq kernel (scq_kernel.hip, PCG_RTC).
std::string scq_rtc_source(const PlanHost& h);
// Compile it (cached per process by source text): 0 and the code object, or -1 and *err.
int scq_rtc_compile(const PlanHost& h, std::vector<char>* code, std::string* err);
// Launch the loaded kernel `scq_rtc_kernel` (grid = a.units, LDS = a.wave_lds_floats).
int scq_rtc_launch(hipFunction_t fn, const KernelArgs& a, hipStream_t stream);
} // namespace pcg
