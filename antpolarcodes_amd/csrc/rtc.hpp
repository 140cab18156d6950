// rtc.hpp -- plan-specialised kernels compiled at run time (rtc.cpp).
#pragma once
#include "kernels.hpp"
#include "plan.hpp"

#include <memory>
#include <string>
#include <vector>

namespace pcg {
// The hiprtc source of a Fast-SSC plan's specialised scq kernel (scq_kernel.hip, PCG_RTC;
// kernel scq_rtc_kernel) and of a float list plan's lane-serial kernel with its layout
// (sclls_kernel.hip; kernel scl_rtc_kernel).  Both carry the compile-time knobs of the
// library's own kernel translation units (sclls_rtc_defines), so a specialised kernel is
// always the interpreter's code with the plan folded in.
std::string scq_rtc_source(const PlanHost& h);
std::string scl_rtc_source(const PlanHost& h, uint32_t lp, uint32_t Sl, uint32_t virt, uint32_t v3, uint32_t sb,
                           uint32_t fuse);
// The 8-bit lane-serial Fast-SSC kernel (sccs_kernel.hip) with the plan's constants and layout
// as literals (kernels sccs_rtc_kernel: int8 LLRs, sccs_rtc_kernel_f32: float LLRs quantised in
// the kernel).
std::string sccs_rtc_source(const PlanHost& h, uint32_t Sl);
// The 8-bit lane-serial list kernel (scl_char_kernel.hip), likewise (scl_char_rtc_kernel[_f32]).
std::string sclc_rtc_source(const PlanHost& h, uint32_t lp, uint32_t Sl);
// sclls_kernel.hip (host part): "#define PCG_LS_... <value>" lines of that translation unit's
// compile-time knobs; *nondefault = a knob differs from the source's default (a dev build)
std::string sclls_rtc_defines(bool* nondefault);

// One compile of one generated source, shared by every plan (and thread) asking for it.
struct RtcJob;
// Start (or join) the compile of `src`: a code object already in the process cache, the
// library's shipped cache (<dir of libpcg.so>/rtc) or the user cache (PCG_RTC_CACHE) makes a
// finished job at once; otherwise hiprtc runs in a detached thread.  Never waits for that
// compile; the first one a process starts is preceded, on the caller's thread and outside any
// lock, by a small warm-up compile that loads hiprtc's compiler (~1-2 s, once per process:
// rtc.cpp warm_and_hook).
std::shared_ptr<RtcJob> rtc_start(const std::string& src);
// A finished job from the caches only, or null (no compile is started).
std::shared_ptr<RtcJob> rtc_lookup(const std::string& src);
bool rtc_done(const RtcJob& j);
// Wait for the job: 0 and the code object, or -1 and *err.
int rtc_result(RtcJob& j, std::vector<char>* code, std::string* err);
// rtc_result(*rtc_start(src)): compile and wait.
int rtc_compile(const std::string& src, std::vector<char>* code, std::string* err);
// hiprtc compiles started by this process (tests: plans of one code share one compile)
int rtc_compiles();
// The cache file name of a generated source (the user cache, and what a compile writes).
std::string rtc_cache_name(const std::string& src);
// The name a lookup in directory `dir` reads for `src`: named by the hiprtc version the
// directory records (its HIPRTC_VERSION file), else this process's (what disk_lookup reads in the
// shipped cache).
std::string rtc_lookup_name(const std::string& src, const std::string& dir);
// The hiprtc version this process compiles with ("major.minor"; "none" without hiprtc).
std::string rtc_version();
// The GPU architecture the specialised kernels are compiled for (the library's ARCH).
const char* rtc_arch();
// Launch a loaded specialised kernel (grid = a.units, LDS = a.wave_lds_floats).
int rtc_launch(hipFunction_t fn, const KernelArgs& a, hipStream_t stream);
} // namespace pcg
