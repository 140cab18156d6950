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
// (build/rtc_src.inc), plus the compile-time knobs of the library's own kernel objects.
//
// hiprtc is opened with dlopen on first use, so a machine without it still loads libpcg and
// decodes with the interpreter kernel.  Code objects are looked up, in order, in the
// process cache, the library's shipped cache (<dir of libpcg.so>/rtc: the codes `make
// rtc-cache` compiled at build time) and the user cache (PCG_RTC_CACHE, default
// $XDG_CACHE_HOME or ~/.cache/antpolarcodes_amd/rtc; "0" = off).  Files are named by a hash of
// the generated source, the embedded sources, the compile options, the target architecture
// and the hiprtc version, and end in a trailer (magic, length, checksum) that a torn or foreign
// file fails.  One compile per source runs at a time in the process (plans of the same code on
// several devices share it) in a detached thread that owns its state: a plan destroyed while
// it runs does not wait; process exit waits for it (atexit) rather than tear hiprtc down
// under it.
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

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#ifndef PCG_ARCH
#define PCG_ARCH "gfx950"
#endif

namespace pcg {

struct RtcJob {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    std::vector<char> code;
    std::string err;
};

namespace {

#include "build/rtc_src.inc" // rtc_names[], rtc_srcs[], rtc_nsrcs

struct RtcApi {
    bool ok = false;
    std::string err;
    std::string version; // "major.minor" (cache key)
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
    static RtcApi* a = new RtcApi; // immortal: compile threads may outlive static destruction
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"libhiprtc.so", "libhiprtc.so.7", "/opt/rocm/lib/libhiprtc.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr)
                break;
        if (!h) {
            a->err = "hiprtc not found (dlopen libhiprtc.so)";
            a->version = "none";
            return;
        }
        a->create = reinterpret_cast<decltype(a->create)>(dlsym(h, "hiprtcCreateProgram"));
        a->compile = reinterpret_cast<decltype(a->compile)>(dlsym(h, "hiprtcCompileProgram"));
        a->log_size = reinterpret_cast<decltype(a->log_size)>(dlsym(h, "hiprtcGetProgramLogSize"));
        a->log = reinterpret_cast<decltype(a->log)>(dlsym(h, "hiprtcGetProgramLog"));
        a->code_size = reinterpret_cast<decltype(a->code_size)>(dlsym(h, "hiprtcGetCodeSize"));
        a->code = reinterpret_cast<decltype(a->code)>(dlsym(h, "hiprtcGetCode"));
        a->destroy = reinterpret_cast<decltype(a->destroy)>(dlsym(h, "hiprtcDestroyProgram"));
        auto ver = reinterpret_cast<hiprtcResult (*)(int*, int*)>(dlsym(h, "hiprtcVersion"));
        int mj = 0, mn = 0;
        if (ver && ver(&mj, &mn) == HIPRTC_SUCCESS)
            a->version = std::to_string(mj) + "." + std::to_string(mn);
        else
            a->version = "unknown";
        a->ok = a->create && a->compile && a->log_size && a->log && a->code_size && a->code && a->destroy;
        if (!a->ok)
            a->err = "hiprtc: missing entry points";
    });
    return *a;
}

// Process-wide registry of jobs by source (immortal, like everything a compile thread touches).
struct Registry {
    std::mutex mu;
    std::condition_variable idle;
    std::map<std::string, std::shared_ptr<RtcJob>> jobs;
    int running = 0;
    int started = 0;
};
Registry& reg()
{
    static Registry* r = new Registry;
    return *r;
}

// the library's flags (Makefile HIPFLAGS): IEEE fp32, no contraction, denormals kept
const char* const g_opts[] = {"--offload-arch=" PCG_ARCH, "-O3", "-std=c++17", "-ffp-contract=off",
                              "-fno-gpu-flush-denormals-to-zero", "-fno-fast-math"};
constexpr int g_nopts = (int)(sizeof(g_opts) / sizeof(g_opts[0]));

// development aid: PCG_RTC_XOPTS = extra hiprtc options, separated by spaces or commas (compiler flag A/Bs;
// part of the cache name, and a plan compiled with them reports PCG_DEV_BUILD)
const std::vector<std::string>& extra_opts()
{
    static const std::vector<std::string> v = [] {
        std::vector<std::string> r;
        if (const char* e = getenv("PCG_RTC_XOPTS")) {
            std::string cur;
            for (const char* q = e;; ++q) {
                if (*q == ' ' || *q == ',' || *q == 0) {
                    if (!cur.empty())
                        r.push_back(cur);
                    cur.clear();
                    if (*q == 0)
                        break;
                } else
                    cur += *q;
            }
        }
        return r;
    }();
    return v;
}

uint64_t fnv1a(uint64_t h, const char* p, size_t n)
{
    for (size_t i = 0; i < n; ++i)
        h = (h ^ (uint8_t)p[i]) * 0x100000001b3ull;
    return h;
}

void mkdirs(const std::string& dir)
{
    for (size_t k = 1; k <= dir.size(); ++k) // mkdir -p
        if (k == dir.size() || dir[k] == '/')
            (void)mkdir(dir.substr(0, k).c_str(), 0755);
}

// The cache file name of a generated source: everything that determines the code object
// (ver: the hiprtc version that compiles it -- this process's, or the one the shipped cache
// was built with).
std::string cache_name(const std::string& src, const std::string& ver)
{
    uint64_t h = fnv1a(0xcbf29ce484222325ull, src.data(), src.size());
    for (int i = 0; i < rtc_nsrcs; ++i) {
        h = fnv1a(h, rtc_names[i], strlen(rtc_names[i]) + 1);
        h = fnv1a(h, rtc_srcs[i], strlen(rtc_srcs[i]) + 1);
    }
    for (int i = 0; i < g_nopts; ++i)
        h = fnv1a(h, g_opts[i], strlen(g_opts[i]) + 1);
    for (const std::string& o : extra_opts())
        h = fnv1a(h, o.c_str(), o.size() + 1);
    const std::string tag = std::string(PCG_ARCH) + "|hiprtc " + ver;
    h = fnv1a(h, tag.data(), tag.size());
    char name[40];
    snprintf(name, sizeof(name), "pcg_%016llx.co", (unsigned long long)h);
    return name;
}
std::string cache_name(const std::string& src) { return cache_name(src, api().version); }

// the user cache directory, or "" when it is off
std::string user_dir()
{
    if (const char* e = getenv("PCG_RTC_CACHE")) {
        if (e[0] == '0' && e[1] == 0)
            return "";
        return e;
    }
    if (const char* x = getenv("XDG_CACHE_HOME"))
        return std::string(x) + "/antpolarcodes_amd/rtc";
    if (const char* hm = getenv("HOME"))
        return std::string(hm) + "/.cache/antpolarcodes_amd/rtc";
    return "";
}

// the shipped cache next to the library (read-only use)
std::string shipped_dir()
{
    Dl_info info{};
    if (dladdr(reinterpret_cast<void*>(&shipped_dir), &info) == 0 || !info.dli_fname)
        return "";
    std::string p = info.dli_fname;
    const size_t k = p.rfind('/');
    return k == std::string::npos ? std::string("rtc") : p.substr(0, k) + "/rtc";
}

// A cache directory records the hiprtc version its files were compiled with
// (kVersionFile): the shipped cache is looked up under the build machine's version, so a
// machine without hiprtc (or with another version) still loads the shipped code objects --
// they only need hipModuleLoadData.
constexpr const char* kVersionFile = "HIPRTC_VERSION";
std::string dir_version(const std::string& dir)
{
    std::string v;
    if (FILE* f = fopen((dir + "/" + kVersionFile).c_str(), "r")) {
        char buf[64] = {0};
        if (fgets(buf, sizeof(buf), f))
            v = buf;
        fclose(f);
    }
    while (!v.empty() && (v.back() == '\n' || v.back() == '\r' || v.back() == ' '))
        v.pop_back();
    return v;
}

// File = code object, then a 24-byte trailer: "PCGRTC01", the code length, its FNV-1a hash.
constexpr char kMagic[8] = {'P', 'C', 'G', 'R', 'T', 'C', '0', '1'};

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
    if (buf.size() < 64 + 24)
        return false;
    const char* t = buf.data() + buf.size() - 24;
    uint64_t len = 0, hash = 0;
    memcpy(&len, t + 8, 8);
    memcpy(&hash, t + 16, 8);
    if (memcmp(t, kMagic, 8) != 0 || len != buf.size() - 24 ||
        fnv1a(0xcbf29ce484222325ull, buf.data(), len) != hash || buf[0] != 0x7f || buf[1] != 'E' || buf[2] != 'L' ||
        buf[3] != 'F')
        return false; // torn, truncated or foreign: ignored (and recompiled)
    buf.resize(len);
    *out = std::move(buf);
    return true;
}

void write_file(const std::string& dir, const std::string& name, const std::vector<char>& code)
{
    mkdirs(dir);
    if (dir_version(dir).empty() && api().ok) { // (first writer; every writer of a version agrees)
        if (FILE* f = fopen((dir + "/" + kVersionFile).c_str(), "w")) {
            fprintf(f, "%s\n", api().version.c_str());
            fclose(f);
        }
    }
    std::string tmpl = dir + "/." + name + ".XXXXXX";
    const int fd = mkstemp(&tmpl[0]); // unique per writer: concurrent writers never share a temp file
    if (fd < 0)
        return;
    FILE* f = fdopen(fd, "wb");
    if (!f) {
        close(fd);
        (void)unlink(tmpl.c_str());
        return;
    }
    const uint64_t len = code.size(), hash = fnv1a(0xcbf29ce484222325ull, code.data(), code.size());
    bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
    ok = ok && fwrite(kMagic, 1, 8, f) == 8 && fwrite(&len, 8, 1, f) == 1 && fwrite(&hash, 8, 1, f) == 1;
    (void)fchmod(fd, 0644);
    if (fclose(f) == 0 && ok)
        (void)rename(tmpl.c_str(), (dir + "/" + name).c_str()); // atomic: readers see the old or the whole file
    else
        (void)unlink(tmpl.c_str());
}

// cached code object of a source: shipped, then user cache
bool disk_lookup(const std::string& src, std::vector<char>* code)
{
    const std::string sd = shipped_dir();
    if (!sd.empty()) {
        const std::string sv = dir_version(sd);
        if (read_file(sd + "/" + cache_name(src, sv.empty() ? api().version : sv), code))
            return true;
    }
    const std::string ud = user_dir();
    return !ud.empty() && read_file(ud + "/" + cache_name(src), code);
}

void dump_source(const std::string& src)
{
    if (const char* path = getenv("PCG_RTC_DUMP")) { // development aid: the generated source
        if (FILE* f = fopen(path, "w")) {
            fputs(src.c_str(), f);
            fclose(f);
        }
    }
}

int hiprtc_build(const std::string& src, std::vector<char>* code, std::string* err)
{
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
    std::vector<const char*> opts(g_opts, g_opts + g_nopts);
    for (const std::string& o : extra_opts())
        opts.push_back(o.c_str());
    const hiprtcResult r = a.compile(prog, (int)opts.size(), opts.data());
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
    return 0;
}

// (see rtc_start: the compiler's statics exist before the exit hook is registered)
const char* const kWarmSrc = "extern \"C\" __global__ void pcg_rtc_warm(float* x, int n)\n"
                             "{ float s = 0.f; for (int i = threadIdx.x; i < n; i += 64) s += x[i] * x[i];\n"
                             "  x[threadIdx.x] = __shfl_xor(s, 1); }\n";

void finish(RtcJob& j)
{
    std::lock_guard<std::mutex> lk(j.mu);
    j.done = true;
    j.cv.notify_all();
}

// Process exit waits for compiles still running (their thread is inside hiprtc, whose
// teardown must not run under it).  It says so on stderr when it has to wait, and
// PCG_RTC_EXIT_WAIT=<seconds> bounds the wait: past it the process flushes every stdio stream and
// ends at once (_exit) without running the remaining exit handlers.  An atexit handler cannot
// read the status the program passed to exit(), so that status is REPLACED by
// PCG_RTC_EXIT_STATUS (default 75, EX_TEMPFAIL): never 0, so leaving early never reports a
// failed run as a success.
void wait_running()
{
    Registry& r = reg();
    std::unique_lock<std::mutex> lk(r.mu);
    if (getenv("PCG_RTC_DEBUG"))
        fprintf(stderr, "[pcg] exit: %d compiles running\n", r.running);
    if (r.running > 0)
        fprintf(stderr,
                "[pcg] waiting for %d background kernel compile(s) to finish before exit "
                "(PCG_RTC=0: no automatic compiles; PCG_RTC_EXIT_WAIT=<s>: bound this wait)\n",
                r.running);
    long bound = -1;
    if (const char* e = getenv("PCG_RTC_EXIT_WAIT"))
        bound = atol(e);
    if (bound >= 0) {
        if (!r.idle.wait_for(lk, std::chrono::seconds(bound), [&] { return r.running == 0; })) {
            int status = 75; // EX_TEMPFAIL
            if (const char* e = getenv("PCG_RTC_EXIT_STATUS"))
                status = atoi(e);
            fprintf(stderr,
                    "[pcg] exit: %d compile(s) still running after %ld s; leaving without them, exit status %d "
                    "(PCG_RTC_EXIT_STATUS) replaces the program's\n",
                    r.running, bound, status);
            fflush(nullptr); // every stdio stream: buffered stdout of C / C++ callers too
            _exit(status);
        }
    } else {
        r.idle.wait(lk, [&] { return r.running == 0; });
    }
    if (getenv("PCG_RTC_DEBUG"))
        fprintf(stderr, "[pcg] exit: compiles done\n");
}

// The exit hook must run before the destructors of hiprtc's compiler (comgr, loaded by
// hiprtc's first compile, and the function-local statics that compile creates): exit() runs
// handlers in reverse order of registration, so a small compile runs first, then the hook
// is registered.  Once per process, before the registry lock is taken: the first
// rtc_start of a process blocks its caller for this warm-up (loading comgr, ~1-2 s), never
// another thread's registry access.
void warm_and_hook()
{
    static std::once_flag at;
    std::call_once(at, [] {
        std::vector<char> c;
        std::string e;
        (void)hiprtc_build(kWarmSrc, &c, &e);
        atexit(wait_running);
    });
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

std::string sccs_rtc_source(const PlanHost& h, uint32_t Sl)
{
    std::string s = "#define PCG_RTC 1\n";
    auto def = [&](const char* k, uint32_t v) { s += std::string("#define PCG_RTC_") + k + " " + std::to_string(v) + "u\n"; };
    def("N", h.N);
    def("LOG2N", h.log2N);
    def("K", h.K);
    def("CRC", (uint32_t)h.crc_kind);
    s += "#define PCG_RTC_SYS " + std::to_string(h.systematic ? 1 : 0) + "\n";
    def("SL", Sl);
    def("NOPS", (uint32_t)h.ops.size()); // (the schedule itself stays in the plan's device buffer)
    s += "#include \"sccs_kernel.hip\"\n";
    return s;
}

std::string sclc_rtc_source(const PlanHost& h, uint32_t lp, uint32_t Sl)
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
    def("NOPS", (uint32_t)h.ops.size());
    s += "#include \"scl_char_kernel.hip\"\n";
    return s;
}

std::string scl_rtc_source(const PlanHost& h, uint32_t lp, uint32_t Sl, uint32_t virt, uint32_t v3, uint32_t sb,
                           uint32_t fuse)
{
    bool nd = false;
    std::string s = "#define PCG_RTC 1\n" + sclls_rtc_defines(&nd);
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

const char* rtc_arch() { return PCG_ARCH; }

std::string rtc_cache_name(const std::string& src) { return cache_name(src); }

std::string rtc_lookup_name(const std::string& src, const std::string& dir)
{
    const std::string v = dir_version(dir);
    return cache_name(src, v.empty() ? api().version : v);
}

std::string rtc_version() { return api().version; }

int rtc_compiles()
{
    std::lock_guard<std::mutex> lk(reg().mu);
    return reg().started;
}

std::shared_ptr<RtcJob> rtc_lookup(const std::string& src)
{
    Registry& r = reg();
    {
        std::lock_guard<std::mutex> lk(r.mu);
        auto it = r.jobs.find(src);
        if (it != r.jobs.end()) {
            if (rtc_done(*it->second))
                return it->second;
            return nullptr;
        }
    }
    std::vector<char> code;
    if (!disk_lookup(src, &code))
        return nullptr;
    auto j = std::make_shared<RtcJob>();
    j->code = std::move(code);
    j->done = true;
    std::lock_guard<std::mutex> lk(r.mu);
    auto ins = r.jobs.emplace(src, j);
    return ins.first->second;
}

std::shared_ptr<RtcJob> rtc_start(const std::string& src)
{
    dump_source(src);
    if (auto j = rtc_lookup(src))
        return j;
    Registry& r = reg();
    warm_and_hook();
    std::shared_ptr<RtcJob> j;
    {
        std::lock_guard<std::mutex> lk(r.mu);
        auto it = r.jobs.find(src);
        if (it != r.jobs.end())
            return it->second; // another plan's compile of the same source: share it
        j = std::make_shared<RtcJob>();
        r.jobs.emplace(src, j);
        ++r.running;
        ++r.started;
    }
    std::thread([j, src] {
        std::vector<char> code;
        std::string err;
        if (hiprtc_build(src, &code, &err) == 0) {
            const std::string ud = user_dir();
            if (!ud.empty())
                write_file(ud, cache_name(src), code);
            j->code = std::move(code);
        } else {
            j->err = err;
        }
        finish(*j);
        Registry& rr = reg();
        std::lock_guard<std::mutex> lk(rr.mu);
        if (!j->err.empty()) // a failed compile is retried by the next request
            rr.jobs.erase(src);
        if (--rr.running == 0)
            rr.idle.notify_all();
    }).detach();
    return j;
}

bool rtc_done(const RtcJob& j)
{
    std::lock_guard<std::mutex> lk(const_cast<std::mutex&>(j.mu));
    return j.done;
}

int rtc_result(RtcJob& j, std::vector<char>* code, std::string* err)
{
    std::unique_lock<std::mutex> lk(j.mu);
    j.cv.wait(lk, [&] { return j.done; });
    if (j.code.empty()) {
        *err = j.err.empty() ? std::string("hiprtc: no code object") : j.err;
        return -1;
    }
    *code = j.code;
    return 0;
}

int rtc_compile(const std::string& src, std::vector<char>* code, std::string* err)
{
    return rtc_result(*rtc_start(src), code, err);
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
