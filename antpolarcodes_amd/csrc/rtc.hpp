// rtc.hpp -- plan-specialised kernels compiled at run time (rtc.cpp).
#pragma once
#include "kernels.hpp"
#include "plan.hpp"

#include <string>
#include <vector>

namespace pcg {
// The hiprtc source of a Fast-SSC plan's specialised scq kernel (scq_kernel.hip, PCG_RTC;
// kernel scq_rtc_kernel) and of a float list plan's lane-serial kernel with its layout
// (sclls_kernel.hip; kernel scl_rtc_kernel).
std::string scq_rtc_source(const PlanHost& h);
std::string scl_rtc_source(const PlanHost& h, uint32_t lp, uint32_t Sl, uint32_t virt, uint32_t v3, uint32_t sb,
                           uint32_t fuse);
// Compile a source (cached per process and on disk): 0 and the code object, or -1 and *err.
int rtc_compile(const std::string& src, std::vector<char>* code, std::string* err);
// Launch a loaded specialised kernel (grid = a.units, LDS = a.wave_lds_floats).
int rtc_launch(hipFunction_t fn, const KernelArgs& a, hipStream_t stream);
} // namespace pcg
