// rtc.cpp -- plan-specialised decoder kernels, compiled at run time with hiprtc.
//
// The reference builds one decoder object tree per code (FastSscAvx::createDecoder,
// fastssc_avx_float.cpp:797-896) and walks it with virtual calls; scq_kernel.hip walks the
// plan's flattened schedule as an interpreter (schedule words through the scalar cache, a
// dispatch branch per op).  A plan-specialised kernel is the same device code compiled with
// the plan's fused schedule as a compile-time array (scq_kernel.hip, PCG_RTC): every op is
// inlined with literal codes, stages and offsets.  The same holds for the lane-serial list
// decoder (sclls_kernel.hip; SclAvx::createDecoder, scl_avx_float.cpp:624-651), whose
// layout constants and path counts become literals as well.  The sources are the kernel
// files and the headers they include, embedded into the library at build time
// (build/rtc_src.inc).
//
// hiprtc is opened with dlopen on first use, so a machine without it still loads libpcg and
// decodes with the interpreter kernel.  Compiled code objects are cached per process by
// source text and on disk (PCG_RTC_CACHE, default $XDG_CACHE_HOME or ~/.cache
// /antpolarcodes_amd/rtc; "0" = off) under a hash of the generated source, the embedded
// sources and the compile options, so other processes of the same build skip the compile;
// each plan loads its own module on its device.
#include "kernels.hpp"
#include "plan.hpp"
#include "rtc.hpp"

#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace pcg {
namespace {

#include "build/rtc_src.inc" // rtc_names[], rtc_srcs[], rtc_nsrcs

struct RtcApi {
    bool ok = false;
    std::string err;
    hiprtcResult (*create)(hiprtcProgram*, const char*, const char*, int, const char**, const char**) = nullptr;
    hiprtcResult (*compile)(hiprtcProgram, int, const char**) = nullptr;
    hiprtcResult (*log_size)(hiprtcProgram, size_t*) = nullptr;
    hiprtcResult (*log)(hiprtcProgram, char*) = nullptr;
    hiprtcResult (*code_size)(hiprtcProgram, size_t*) = nullptr;
    hiprtcResult (*code)(hiprtcProgram, char*) = nullptr;
    hiprtcResult (*destroy)(hiprtcProgram*) = nullptr;
};

RtcApi& api()
{
    static RtcApi a;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"libhiprtc.so", "libhiprtc.so.7", "/opt/rocm/lib/libhiprtc.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr)
                break;
        if (!h) {
            a.err = "hiprtc not found (dlopen libhiprtc.so)";
            return;
        }
        a.create = reinterpret_cast<decltype(a.create)>(dlsym(h, "hiprtcCreateProgram"));
        a.compile = reinterpret_cast<decltype(a.compile)>(dlsym(h, "hiprtcCompileProgram"));
        a.log_size = reinterpret_cast<decltype(a.log_size)>(dlsym(h, "hiprtcGetProgramLogSize"));
        a.log = reinterpret_cast<decltype(a.log)>(dlsym(h, "hiprtcGetProgramLog"));
        a.code_size = reinterpret_cast<decltype(a.code_size)>(dlsym(h, "hiprtcGetCodeSize"));
        a.code = reinterpret_cast<decltype(a.code)>(dlsym(h, "hiprtcGetCode"));
        a.destroy = reinterpret_cast<decltype(a.destroy)>(dlsym(h, "hiprtcDestroyProgram"));
        a.ok = a.create && a.compile && a.log_size && a.log && a.code_size && a.code && a.destroy;
        if (!a.ok)
            a.err = "hiprtc: missing entry points";
    });
    return a;
}

std::mutex g_cache_mu;
std::map<std::string, std::vector<char>> g_cache; // source text -> code object

// the library's own flags (Makefile HIPFLAGS): IEEE fp32, no contraction, denormals kept
const char* const g_opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                              "-fno-gpu-flush-denormals-to-zero", "-fno-fast-math"};
constexpr int g_nopts = (int)(sizeof(g_opts) / sizeof(g_opts[0]));

uint64_t fnv1a(uint64_t h, const char* p, size_t n)
{
    for (size_t i = 0; i < n; ++i)
        h = (h ^ (uint8_t)p[i]) * 0x100000001b3ull;
    return h;
}

// the on-disk cache file of a generated source, or "" when the cache is off
std::string disk_path(const std::string& src)
{
    std::string dir;
    if (const char* e = getenv("PCG_RTC_CACHE")) {
        if (e[0] == '0' && e[1] == 0)
            return "";
        dir = e;
    } else if (const char* x = getenv("XDG_CACHE_HOME")) {
        dir = std::string(x) + "/antpolarcodes_amd/rtc";
    } else if (const char* hm = getenv("HOME")) {
        dir = std::string(hm) + "/.cache/antpolarcodes_amd/rtc";
    } else {
        return "";
    }
    uint64_t h = fnv1a(0xcbf29ce484222325ull, src.data(), src.size());
    for (int i = 0; i < rtc_nsrcs; ++i) {
        h = fnv1a(h, rtc_names[i], strlen(rtc_names[i]));
        h = fnv1a(h, rtc_srcs[i], strlen(rtc_srcs[i]));
    }
    for (int i = 0; i < g_nopts; ++i)
        h = fnv1a(h, g_opts[i], strlen(g_opts[i]));
    for (size_t k = 1; k <= dir.size(); ++k) // mkdir -p
        if (k == dir.size() || dir[k] == '/')
            (void)mkdir(dir.substr(0, k).c_str(), 0755);
    char name[32];
    snprintf(name, sizeof(name), "/pcg_%016llx.co", (unsigned long long)h);
    return dir + name;
}

bool read_file(const std::string& path, std::vector<char>* out)
{
    FILE* f = fopen(path.c_str(), "rb");
    if (!f)
        return false;
    std::vector<char> buf;
    char tmp[65536];
    size_t n;
    while ((n = fread(tmp, 1, sizeof(tmp), f)) > 0)
        buf.insert(buf.end(), tmp, tmp + n);
    fclose(f);
    // an ELF code object (a torn or foreign file is ignored and recompiled)
    if (buf.size() < 64 || buf[0] != 0x7f || buf[1] != 'E' || buf[2] != 'L' || buf[3] != 'F')
        return false;
    *out = std::move(buf);
    return true;
}

void write_file(const std::string& path, const std::vector<char>& code)
{
    const std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f)
        return;
    const bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
    if (fclose(f) == 0 && ok)
        (void)rename(tmp.c_str(), path.c_str()); // atomic: readers see the old or the whole file
    else
        (void)unlink(tmp.c_str());
}

} // namespace

std::string scq_rtc_source(const PlanHost& h)
{
    std::string s = "#define PCG_RTC 1\n";
    s += "#define PCG_RTC_Q " + std::to_string(h.scq_q) + "\n";
    s += "#define PCG_RTC_V " + std::to_string(h.scq_virt ? 1 : 0) + "\n";
    s += "#define PCG_RTC_N " + std::to_string(h.N) + "u\n";
    s += "#define PCG_RTC_LOG2N " + std::to_string(h.log2N) + "u\n";
    s += "#define PCG_RTC_K " + std::to_string(h.K) + "u\n";
    s += "#define PCG_RTC_CRC " + std::to_string(h.crc_kind) + "u\n";
    s += "#define PCG_RTC_SYS " + std::to_string(h.systematic ? 1 : 0) + "\n";
    s += "#define PCG_RTC_OPS";
    for (size_t k = 0; k < h.ops_fused.size(); ++k)
        s += (k ? "," : " ") + std::to_string(h.ops_fused[k]) + "u";
    s += "\n#include \"scq_kernel.hip\"\n";
    return s;
}

std::string scl_rtc_source(const PlanHost& h, uint32_t lp, uint32_t Sl, uint32_t virt, uint32_t v3, uint32_t sb,
                           uint32_t fuse)
{
    std::string s = "#define PCG_RTC 1\n";
    auto def = [&](const char* k, uint32_t v) { s += std::string("#define PCG_RTC_") + k + " " + std::to_string(v) + "u\n"; };
    def("LP", lp);
    def("N", h.N);
    def("LOG2N", h.log2N);
    def("K", h.K);
    def("L", h.L);
    def("CRC", (uint32_t)h.crc_kind);
    s += "#define PCG_RTC_SYS " + std::to_string(h.systematic ? 1 : 0) + "\n";
    def("SL", Sl);
    def("VIRT", virt);
    def("V3", v3);
    def("SB", sb);
    def("FUSE", fuse);
    s += "#define PCG_RTC_OPS";
    for (size_t k = 0; k < h.ops.size(); ++k)
        s += (k ? "," : " ") + std::to_string(h.ops[k]) + "u";
    s += "\n#include \"sclls_kernel.hip\"\n";
    return s;
}

int rtc_compile(const std::string& src, std::vector<char>* code, std::string* err)
{
    if (const char* path = getenv("PCG_RTC_DUMP")) { // development aid: the generated source
        if (FILE* f = fopen(path, "w")) {
            fputs(src.c_str(), f);
            fclose(f);
        }
    }
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        auto it = g_cache.find(src);
        if (it != g_cache.end()) {
            *code = it->second;
            return 0;
        }
    }
    const std::string disk = disk_path(src);
    if (!disk.empty() && read_file(disk, code)) {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        g_cache.emplace(src, *code);
        return 0;
    }
    RtcApi& a = api();
    if (!a.ok) {
        *err = a.err;
        return -1;
    }
    hiprtcProgram prog = nullptr;
    if (a.create(&prog, src.c_str(), "pcg_rtc.hip", rtc_nsrcs, rtc_srcs, rtc_names) != HIPRTC_SUCCESS) {
        *err = "hiprtcCreateProgram failed";
        return -1;
    }
    const hiprtcResult r = a.compile(prog, g_nopts, const_cast<const char**>(g_opts));
    if (r != HIPRTC_SUCCESS) {
        size_t n = 0;
        std::string log;
        if (a.log_size(prog, &n) == HIPRTC_SUCCESS && n > 1) {
            log.resize(n);
            (void)a.log(prog, &log[0]);
        }
        *err = "hiprtc compile failed: " + log.substr(0, 2000);
        (void)a.destroy(&prog);
        return -1;
    }
    size_t n = 0;
    if (a.code_size(prog, &n) != HIPRTC_SUCCESS || n == 0) {
        *err = "hiprtcGetCodeSize failed";
        (void)a.destroy(&prog);
        return -1;
    }
    code->resize(n);
    const hiprtcResult rc = a.code(prog, code->data());
    (void)a.destroy(&prog);
    if (rc != HIPRTC_SUCCESS) {
        *err = "hiprtcGetCode failed";
        return -1;
    }
    if (!disk.empty())
        write_file(disk, *code);
    std::lock_guard<std::mutex> lk(g_cache_mu);
    g_cache.emplace(src, *code);
    return 0;
}

int rtc_launch(hipFunction_t fn, const KernelArgs& a, hipStream_t stream)
{
    const uint64_t grid = a.units;
    if (grid == 0) // no waves for a non-empty batch: an error, never a silent no-op
        return a.F ? -4 : 0;
    KernelArgs args = a;
    void* params[] = {&args};
    const hipError_t e = hipModuleLaunchKernel(fn, (uint32_t)grid, 1, 1, 64, 1, 1, a.wave_lds_floats * 4u, stream,
                                               params, nullptr);
    return e == hipSuccess ? 0 : -3;
}

} // namespace pcg
