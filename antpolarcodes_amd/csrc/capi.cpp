// capi.cpp -- the C ABI of include/pcg.h on top of the HIP kernels.
#include "../../include/pcg.h"

#include "frames.hpp"
#include "kernels.hpp"
#include "plan.hpp"
#include "rtc.hpp"

#include <hip/hip_runtime.h>
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

struct HostPipe;
struct pcg_plan {
    pcg::PlanHost host;
    int device = 0;
    uint32_t* d_ops = nullptr;
    uint16_t* d_info_pos = nullptr;
    uint32_t* d_crc_m = nullptr;
    uint32_t wave_lds_floats = 0;
    uint32_t lds_stage_limit = 0;
    uint32_t scl_virt = 0;
    uint32_t scl_fuse = 7;
    uint32_t scl_lp = 0;          // lane-serial SCL: lanes per codeword (0 = list_pow2(L))
    uint32_t scl_v3 = 0;          // lane-serial SCL: stage 3 recomputed from stage 4 (sclls_layout)
    uint32_t scl_sb = 0;          // lane-serial SCL: bit buffers below this stage in LDS (0: codeword rows)
    uint64_t scratch_floats = 0;  // per scratch unit (lane-serial wave)
    float* d_scratch = nullptr;   // grown stream-ordered (hipMallocAsync) when a launch needs more waves
    uint64_t scratch_cap = 0;     // capacity in elements (units x per-unit floats / dwords)
    // persistent-wave caps of this plan's kernel on its device (float / int8 channel input),
    // evaluated once at plan creation
    uint64_t wave_cap = 0;
    uint64_t wave_cap_i8 = 0;
    uint32_t* d_queue = nullptr;  // lane-serial SCL work queue: one counter, zeroed on the launch stream
    const char* kernel = "";      // name of the decode kernel (pcg_plan_kernel_name)
    // developer switches, read from the environment once at plan creation
    uint32_t dev_flags = 0;
    bool dev_opprof = false;
    float metric0 = 0.0f;         // initial path-0 metric (pcg_plan_set_initial_metric)
    // host-pointer path staging
    float* d_llr = nullptr;
    uint8_t* d_info = nullptr;
    uint8_t* d_ok = nullptr;
    float* d_met = nullptr;
    uint64_t stage_frames = 0;
    // host-pointer pipeline (pcg_decode_f32_host / _i8_host): two chunk slots, each with device
    // buffers and pinned host staging, a copy stream and a decode stream (HostPipe below)
    struct HostPipe* pipe = nullptr;
    // pcg_decode_punctured_f32: depunctured LLRs (F x N), reused across calls
    float* d_dep = nullptr;
    uint64_t dep_frames = 0;
    // adaptive plans (pcg_plan_create_adaptive): the Fast-SSC first stage and the
    // failed-frame list of the SCL second stage ([0] = count, then indices)
    pcg_plan* fast = nullptr;
    uint32_t* d_fmap = nullptr;
    uint8_t* d_okbuf = nullptr;
    uint64_t fmap_frames = 0;
    // pcg_decode_f32_soft_host staging (the float staging above holds the LLRs)
    float* d_soft = nullptr;
    uint64_t soft_frames = 0;
    // Stream ordering of the plan's buffers (scratch, queue, staging, frame map): the
    // event is recorded after every decode on the stream it ran on, and a decode on a
    // different stream first waits for it, so launches of one plan never overlap whatever
    // streams callers use; pcg_plan_destroy waits for it before freeing.
    hipEvent_t last_ev = nullptr;
    hipStream_t last_stream = nullptr;
    bool has_last = false;
    uint32_t dev_overrides = 0;   // PCG_DEV_* bits: developer switches that changed this plan
    // plan-specialised kernel (rtc.cpp; Fast-SSC float plans on the scq kernel): rtc_mode 0 =
    // never, 1 = compile at the first decode and wait for it, 2 = compile in the background
    // from the first decode of >= RTC_AUTO_FRAMES frames, switching once it is ready
    // (PCG_RTC=0/1, default 2); rtc_state 0 = not tried, 2 = compiling (rtc_job), 1 = loaded,
    // -1 = failed (rtc_err)
    int rtc_mode = 2;
    int rtc_state = 0;
    bool walk_latency = false; // an adaptive plan's list stage
    bool rtc_scl = true;       // list plans specialise too (PCG_RTC_SCL=0: not)
    bool rtc_probed = false;   // the caches were asked for this plan's code object (mode 2)
    std::shared_ptr<pcg::RtcJob> rtc_job; // the compile this plan waits for (shared, never joined by destroy)
    std::string rtc_err;
    hipModule_t rtc_mod = nullptr;
    hipFunction_t rtc_fn = nullptr;
    hipFunction_t rtc_fn_i8 = nullptr; // 8-bit plans: the kernel for int8 channel LLRs (rtc_fn: float LLRs)
};

// The host-pointer pipeline of pcg_decode_f32_host / pcg_decode_i8_host: chunks of the
// caller's batch alternate between two slots, so chunk i+1's host staging and H2D copy (copy
// stream) run while chunk i decodes (decode stream) and chunk i-1's outputs come back.
struct HostPipe {
    hipStream_t copy = nullptr, dec = nullptr;
    uint64_t frames = 0; // capacity of a slot in frames
    size_t in_fb = 0;    // input bytes per frame the slots were sized for
    uint32_t L = 0;
    uint64_t kb = 0;
    void* d_in[2] = {nullptr, nullptr};
    uint8_t* d_info[2] = {nullptr, nullptr};
    uint8_t* d_ok[2] = {nullptr, nullptr};
    float* d_met[2] = {nullptr, nullptr};
    void* h_in[2] = {nullptr, nullptr};     // pinned input staging (mode 2)
    uint8_t* h_out[2] = {nullptr, nullptr}; // pinned outputs of one chunk: info | ok | metrics
    hipEvent_t ev_h2d[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
};

namespace {

thread_local std::string g_last_error;
unsigned long long* g_prof = nullptr; // dev-only op profiler buffer (PCG_OPPROF=1)

int fail(int code, const std::string& msg)
{
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what)
{
    return fail(PCG_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// The largest V such that no SCL leaf or size-8 subtree op sits at stage >= top-V: the
// recomputed top stages may go that deep (sclls_layout, virt = V).
uint32_t scl_leaf_free_levels(const std::vector<uint32_t>& ops, uint32_t top)
{
    uint32_t hi = 0; // highest leaf stage
    for (size_t k = 0; k < ops.size(); ++k) {
        const uint32_t c = pcg::op_code(ops[k]), s = pcg::op_stage(ops[k]);
        if (c >= pcg::OP_S_R0 && c <= pcg::OP_S_ST8 && s > hi)
            hi = s;
        if (c == pcg::OP_S_ST8)
            ++k; // its descriptor word
    }
    return hi + 1u < top ? top - 1u - hi : 0u;
}

struct DeviceGuard {
    int prev = 0;
    bool ok = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && hipSetDevice(dev) == hipSuccess)
            ok = true;
    }
    ~DeviceGuard()
    {
        if (ok)
            (void)hipSetDevice(prev);
    }
};

void free_pipe(HostPipe* q)
{
    if (!q)
        return;
    for (hipStream_t st : {q->copy, q->dec})
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    for (int b = 0; b < 2; ++b) {
        (void)hipFree(q->d_in[b]);
        (void)hipFree(q->d_info[b]);
        (void)hipFree(q->d_ok[b]);
        (void)hipFree(q->d_met[b]);
        if (q->h_in[b])
            (void)hipHostFree(q->h_in[b]);
        if (q->h_out[b])
            (void)hipHostFree(q->h_out[b]);
        if (q->ev_h2d[b])
            (void)hipEventDestroy(q->ev_h2d[b]);
        if (q->ev_done[b])
            (void)hipEventDestroy(q->ev_done[b]);
    }
    delete q;
}

void free_plan_device(pcg_plan* p)
{
    // everything queued on the plan's buffers has finished once its last event has
    if (p->has_last)
        (void)hipEventSynchronize(p->last_ev);
    free_pipe(p->pipe);
    p->pipe = nullptr;
    (void)hipFree(p->d_ops);
    (void)hipFree(p->d_info_pos);
    (void)hipFree(p->d_crc_m);
    if (p->d_scratch) { // stream-ordered allocation (idle now): return it to the pool
        (void)hipFreeAsync(p->d_scratch, nullptr);
        (void)hipStreamSynchronize(nullptr);
    }
    (void)hipFree(p->d_soft);
    if (p->last_ev)
        (void)hipEventDestroy(p->last_ev);
    p->last_ev = nullptr;
    p->has_last = false;
    (void)hipFree(p->d_queue);
    (void)hipFree(p->d_llr);
    (void)hipFree(p->d_info);
    (void)hipFree(p->d_ok);
    (void)hipFree(p->d_met);
    (void)hipFree(p->d_dep);
    (void)hipFree(p->d_fmap);
    (void)hipFree(p->d_okbuf);
    if (p->rtc_mod)
        (void)hipModuleUnload(p->rtc_mod);
    p->rtc_mod = nullptr;
    p->rtc_fn = nullptr;
    p->rtc_fn_i8 = nullptr;
}

// Batches from this size on specialise a Fast-SSC plan's kernel at their first decode (the
// hiprtc compile takes seconds once per code and process; smaller batches are latency work).
constexpr uint64_t RTC_AUTO_FRAMES = 8192;

// Plans with a specialised kernel: Fast-SSC float plans on the LDS-resident kernel (the walk
// unrolled), float list plans (their layout and plan constants as literals, the schedule
// loop kept: a fully unrolled walk -- 280 schedule words for config 3, each op inlining path
// selection and the leaf decoders -- had not compiled after 20 minutes, against 34 s for
// config 2's 60 fused Fast-SSC ops; PCG_RTC_SCL=0 keeps list plans on the interpreter), the
// 8-bit lane-serial kernels, and both stages of adaptive plans; never with the op profiler.
bool rtc_capable(const pcg_plan* p)
{
    if (p->dev_opprof)
        return false;
    if (p->host.fixed) // the 8-bit lane-serial kernels (sccs, scl_char)
        return p->host.L > 1 || p->host.sc_kind == 0;
    return p->host.L == 1 ? p->host.sc_kind == 2 : p->rtc_scl;
}

// the specialised kernel's name (float-LLR kernel of an 8-bit plan: + "_f32")
const char* rtc_kernel_name(const pcg_plan* p)
{
    if (p->host.fixed)
        return p->host.L == 1 ? "sccs_rtc_kernel" : "scl_char_rtc_kernel";
    return p->host.L == 1 ? "scq_rtc_kernel" : "scl_rtc_kernel";
}

uint32_t list_pow2(uint32_t L);

std::string rtc_source(const pcg_plan* p)
{
    if (p->host.fixed)
        return p->host.L == 1 ? pcg::sccs_rtc_source(p->host, p->lds_stage_limit)
                              : pcg::sclc_rtc_source(p->host, list_pow2(p->host.L), p->lds_stage_limit);
    if (p->host.L == 1)
        return pcg::scq_rtc_source(p->host);
    return pcg::scl_rtc_source(p->host, p->scl_lp, p->lds_stage_limit, p->scl_virt, p->scl_v3, p->scl_sb,
                               p->scl_fuse);
}

// Load the finished job's code object into the plan (a device plan: its module and kernel);
// on failure the plan keeps the interpreter kernel and remembers why.
int rtc_load(pcg_plan* p)
{
    std::vector<char> code;
    std::string err;
    const int r = pcg::rtc_result(*p->rtc_job, &code, &err);
    p->rtc_job.reset();
    if (r != 0) {
        p->rtc_state = -1;
        p->rtc_err = "plan specialisation: " + err;
        return fail(PCG_E_HIP, p->rtc_err);
    }
    const char* fn = rtc_kernel_name(p);
    if (p->device < 0) { // host-only plan: the source compiles; nothing to load
        p->rtc_state = 0;
        p->kernel = fn;
        return PCG_OK;
    }
    // the code objects are built for the library's architecture: refuse another device
    hipDeviceProp_t prop{};
    if (hipGetDeviceProperties(&prop, p->device) == hipSuccess) {
        const std::string an = prop.gcnArchName, want = pcg::rtc_arch();
        if (an.compare(0, want.size(), want) != 0 || (an.size() > want.size() && an[want.size()] != ':')) {
            p->rtc_state = -1;
            p->rtc_err = "plan specialisation: device architecture " + an + " is not the library's " + want;
            return fail(PCG_E_UNSUPPORTED, p->rtc_err);
        }
    }
    hipError_t e = hipModuleLoadData(&p->rtc_mod, code.data());
    if (e == hipSuccess && p->host.fixed) {
        e = hipModuleGetFunction(&p->rtc_fn_i8, p->rtc_mod, fn);
        if (e == hipSuccess)
            e = hipModuleGetFunction(&p->rtc_fn, p->rtc_mod, (std::string(fn) + "_f32").c_str());
        // the specialised kernel's own occupancy (the grid-stride assignment is static)
        int n = 0, cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->device);
        if (e == hipSuccess &&
            hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, p->rtc_fn_i8, 64, p->wave_lds_floats * 4u) ==
                hipSuccess &&
            n > 0)
            p->wave_cap_i8 = (uint64_t)cus * (uint64_t)std::min(n, 16);
        if (e == hipSuccess &&
            hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&n, p->rtc_fn, 64, p->wave_lds_floats * 4u) ==
                hipSuccess &&
            n > 0)
            p->wave_cap = (uint64_t)cus * (uint64_t)std::min(n, 16);
    } else if (e == hipSuccess) {
        e = hipModuleGetFunction(&p->rtc_fn, p->rtc_mod, fn);
    }
    if (e != hipSuccess) {
        if (p->rtc_mod)
            (void)hipModuleUnload(p->rtc_mod);
        p->rtc_mod = nullptr;
        p->rtc_fn = nullptr;
        p->rtc_fn_i8 = nullptr;
        p->rtc_state = -1;
        p->rtc_err = std::string("plan specialisation: module load: ") + hipGetErrorString(e);
        return fail(PCG_E_HIP, p->rtc_err);
    }
    p->rtc_state = 1;
    p->kernel = fn;
    return PCG_OK;
}

// Start the plan's specialisation (a cached code object makes it finish at once; otherwise
// hiprtc compiles in a background thread shared by every plan of the code) and, with wait, load
// it -- or, without, load it only if it is ready (a later call loads it otherwise).
int specialize(pcg_plan* p, bool wait = true)
{
    if (p->rtc_state == 1)
        return PCG_OK;
    if (p->rtc_state == -1)
        return fail(PCG_E_HIP, p->rtc_err);
    if (p->rtc_state == 0) {
        p->rtc_job = pcg::rtc_start(rtc_source(p));
        p->rtc_state = 2;
    }
    if (!wait && !pcg::rtc_done(*p->rtc_job))
        return PCG_OK; // still compiling: the interpreter kernel runs meanwhile
    return rtc_load(p);
}

// At a decode of F frames (rtc_mode, DESIGN.md "Plan-specialised kernels"): mode 1 specialises
// and waits; mode 2 uses a cached code object of the plan's code at once (shipped with the
// library or compiled before), starts a background compile from the first decode of >=
// RTC_AUTO_FRAMES frames, and switches once it is ready.
void auto_specialize(pcg_plan* p, uint64_t F)
{
    if (p->rtc_mode == 0 || p->rtc_state == 1 || p->rtc_state == -1 || !rtc_capable(p))
        return;
    if (p->rtc_state == 2) {
        (void)specialize(p, p->rtc_mode == 1);
        return;
    }
    if (p->rtc_mode == 1) {
        (void)specialize(p, true);
        return;
    }
    if (!p->rtc_probed) {
        p->rtc_probed = true;
        if (auto j = pcg::rtc_lookup(rtc_source(p))) {
            p->rtc_job = j;
            p->rtc_state = 2;
            (void)rtc_load(p);
            return;
        }
    }
    if (F >= RTC_AUTO_FRAMES)
        (void)specialize(p, false);
}

// lanes per codeword of an adaptive plan's SCL stage, 0 = list_pow2(L).  Measured on
// AdaptiveFloat L = 8 (profiles/r02ae_adaptive8_lp_sweep.txt): 8 lanes 6.0e7 cw/s, 16 lanes
// 5.2e7, 32 lanes 3.3e7 -- wider groups shorten F/G but not the leaves and path selection,
// and halve the codewords per launch round, so the list-sized group stays the default.
constexpr uint32_t ADAPT_SCL_LP = 0;

// LP: the list size rounded up to a power of two (>= 2), the lane-serial kernels' template
uint32_t list_pow2(uint32_t L)
{
    uint32_t lp = 2;
    while (lp < L)
        lp <<= 1;
    return lp;
}

const char* kernel_name(const pcg::PlanHost& h, uint32_t scl_lp = 0)
{
    static const char* const sclls[] = {"sclls_kernel<2>", "sclls_kernel<4>", "sclls_kernel<8>",
                                        "sclls_kernel<16>", "sclls_kernel<32>"};
    static const char* const sclc[] = {"scl_char_kernel<2>", "scl_char_kernel<4>", "scl_char_kernel<8>",
                                       "scl_char_kernel<16>", "scl_char_kernel<32>"};
    if (h.L == 1) {
        if (h.fixed)
            return h.sc_kind == 0 ? "sccs_kernel" : "sc_char_kernel";
        return h.sc_kind == 2 ? (h.scq_q == 8 ? "scq_kernel<8>" : h.scq_q == 32 ? "scq_kernel<32>" : "scq_kernel<16>")
                              : (h.sc_kind == 0 ? "scs_kernel" : "sc_kernel");
    }
    const uint32_t lp = std::max(list_pow2(h.L), scl_lp);
    const int i = __builtin_ctz(lp) - 1;
    return h.fixed ? sclc[i] : sclls[i];
}

// Grow the plan's scratch to `units` waves of `per` elements each (default: the plan's
// per-wave scratch), in stream order (no device-wide sync).
int grow_scratch(pcg_plan* p, uint64_t units, size_t elem, hipStream_t s, uint64_t per = 0)
{
    const uint64_t need = units * (per ? per : p->scratch_floats);
    if (need == 0 || need <= p->scratch_cap)
        return PCG_OK;
    if (p->d_scratch)
        (void)hipFreeAsync(p->d_scratch, s);
    p->d_scratch = nullptr;
    p->scratch_cap = 0;
    void* ptr = nullptr;
    hipError_t e = hipMallocAsync(&ptr, need * elem, s);
    if (e != hipSuccess)
        return hip_fail(e, "hipMallocAsync(scratch)");
    p->d_scratch = static_cast<float*>(ptr);
    p->scratch_cap = need;
    return PCG_OK;
}

// Order a decode on `s` after the plan's previous decode (on whatever stream that ran).
int order_on(pcg_plan* p, hipStream_t s)
{
    if (p->has_last && p->last_stream != s) {
        hipError_t e = hipStreamWaitEvent(s, p->last_ev, 0);
        if (e != hipSuccess)
            return hip_fail(e, "hipStreamWaitEvent(plan order)");
    }
    return PCG_OK;
}

// Record the end of a decode on `s`.
int mark_done(pcg_plan* p, hipStream_t s)
{
    if (!p->last_ev)
        return PCG_OK;
    hipError_t e = hipEventRecord(p->last_ev, s);
    if (e != hipSuccess)
        return hip_fail(e, "hipEventRecord(plan order)");
    p->last_stream = s;
    p->has_last = true;
    return PCG_OK;
}

} // namespace

namespace pcg {
int set_error(int code, const std::string& msg) { return fail(code, msg); }
} // namespace pcg

extern "C" {

const char* pcg_last_error(void) { return g_last_error.c_str(); }

// Development aid, not part of include/pcg.h: with PCG_OPPROF=1 in the environment
// the kernels accumulate s_memtime cycles and counts per op code; this copies the
// 64 x {cycles, count} table out and clears it.
// (pcg_dev_opprof_fetch_n: the first n <= kProfN entries -- the list kernel's profiler keeps
// requested global read / write bytes per op bucket in entries 64-127 / 128-191, and a
// -DPCG_LS_PROF_POS build the cycles of schedule position k in entry 256 + k.)
constexpr int kProfN = 4096;
int pcg_dev_opprof_fetch_n(unsigned long long* out, int n)
{
    if (n < 0 || n > kProfN)
        return fail(PCG_E_ARG, "opprof: n > 4096");
    if (!g_prof) {
        std::memset(out, 0, (size_t)n * sizeof(unsigned long long));
        return PCG_OK;
    }
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, g_prof, (size_t)n * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(PCG_E_HIP, "opprof copy failed");
    (void)hipMemset(g_prof, 0, kProfN * sizeof(unsigned long long));
    return PCG_OK;
}
int pcg_dev_opprof_fetch(unsigned long long* out128) { return pcg_dev_opprof_fetch_n(out128, 128); }

// Development aid, not part of include/pcg.h: the cache file name of the plan's specialised
// kernel (antpolarcodes_amd/rtc_warm.py keeps the shipped cache to the listed codes).
int pcg_dev_rtc_cache_name(const pcg_plan* p, char* out, size_t n)
{
    if (!p || !out || n == 0)
        return fail(PCG_E_ARG, "null argument");
    std::string name;
    for (const pcg_plan* q : {(const pcg_plan*)p->fast, p}) // an adaptive plan: both stages' files
        if (q && rtc_capable(q))
            name += (name.empty() ? "" : " ") + pcg::rtc_cache_name(rtc_source(q));
    if (name.empty())
        return fail(PCG_E_UNSUPPORTED, "no plan-specialised kernel for this plan");
    snprintf(out, n, "%s", name.c_str());
    return PCG_OK;
}

// Development aid, not part of include/pcg.h: the name a lookup in directory `dir` reads for the
// plan's specialised kernel (the shipped cache is read under the version its HIPRTC_VERSION file
// records; rtc_warm.py checks that this is the name it wrote).
int pcg_dev_rtc_lookup_name(const pcg_plan* p, const char* dir, char* out, size_t n)
{
    if (!p || !dir || !out || n == 0)
        return fail(PCG_E_ARG, "null argument");
    std::string name;
    for (const pcg_plan* q : {(const pcg_plan*)p->fast, p})
        if (q && rtc_capable(q))
            name += (name.empty() ? "" : " ") + pcg::rtc_lookup_name(rtc_source(q), dir);
    if (name.empty())
        return fail(PCG_E_UNSUPPORTED, "no plan-specialised kernel for this plan");
    snprintf(out, n, "%s", name.c_str());
    return PCG_OK;
}

// Development aid, not part of include/pcg.h: the hiprtc version this process compiles with (the
// shipped cache's HIPRTC_VERSION, which rtc_warm.py rewrites when it differs).
int pcg_dev_rtc_version(char* out, size_t n)
{
    if (!out || n == 0)
        return fail(PCG_E_ARG, "null argument");
    snprintf(out, n, "%s", pcg::rtc_version().c_str());
    return PCG_OK;
}

// Development aid, not part of include/pcg.h: the plan's flattened op schedule (n words at most;
// returns the count) -- tools/ls_prof_pos.py names the per-position cycles with it.
int pcg_dev_plan_ops(const pcg_plan* p, uint32_t* out, int n)
{
    if (!p || !out || n < 0)
        return fail(PCG_E_ARG, "null argument");
    const auto& ops = p->host.ops;
    for (int k = 0; k < n && k < (int)ops.size(); ++k)
        out[k] = ops[k];
    return (int)ops.size();
}

// Development aid, not part of include/pcg.h: hiprtc compiles this process started.
int pcg_dev_rtc_compiles(void) { return pcg::rtc_compiles(); }

int pcg_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

static int plan_create_impl(pcg_plan** out,
                            uint32_t N,
                            uint32_t L,
                            const uint32_t* frozen,
                            uint32_t n_frozen,
                            int systematic,
                            int crc_kind,
                            int device,
                            int fixed,
                            uint32_t scl_lp = 0,
                            bool walk_latency = false)
{
    if (!out)
        return fail(PCG_E_ARG, "plan output pointer is null");
    *out = nullptr;
    auto* p = new pcg_plan();
    std::string err;
    int rc = pcg::build_plan(p->host, N, L, frozen, n_frozen, systematic, crc_kind, &err, fixed);
    if (rc != 0) {
        delete p;
        return fail(rc, err);
    }
    if (fixed && L == 1 && p->host.sc_kind == 2)
        p->host.sc_kind = 0; // the 8-bit decoder has no LDS-resident variant: lane-serial first
    if (!fixed && L == 1 && p->host.sc_kind == 2) {
        // LDS-resident Fast-SSC: Q lanes per codeword (PCG_SCQ_Q dev override), while a
        // wave's state fits a CU and leaves room for several waves
        uint32_t q = 16;
        if (const char* e = getenv("PCG_SCQ_Q")) {
            q = (uint32_t)atoi(e);
            p->dev_overrides |= PCG_DEV_SCQ;
        }
        bool v = true; // the root's children recomputed from the channel (half the LDS)
        if (const char* e = getenv("PCG_SCQ_VIRT")) {
            v = e[0] != '0';
            p->dev_overrides |= PCG_DEV_SCQ;
        }
        // ... only F / G / G0 / ROne read them (leaves and fused size-16 ops read stored stages)
        const auto& fo = p->host.ops_fused;
        for (size_t k = 0; k < fo.size(); ++k) {
            const uint32_t c = pcg::op_code(fo[k]), st = pcg::op_stage(fo[k]) & 15u;
            // the stage an op reads: its own, or its parent's (size 32) for Q16F / Q16G
            const uint32_t rs = (c == pcg::OP_Q16F || c == pcg::OP_Q16G) ? st + 1 : st;
            if (rs == p->host.log2N - 1 && c != pcg::OP_F && c != pcg::OP_G && c != pcg::OP_G0 &&
                c != pcg::OP_RONE && c != pcg::OP_COMB && c != pcg::OP_COPY0)
                v = false;
            if (pcg::op_has_desc(c))
                ++k; // descriptor word
        }
        const uint32_t d = N <= 4096 ? pcg::scq_layout(N, q, v) : 0u;
        if (d != 0) {
            p->host.scq_q = q;
            p->host.scq_virt = v ? 1 : 0;
            p->wave_lds_floats = d;
            p->scratch_floats = 0;
        } else {
            p->host.sc_kind = 0;
        }
    }
    if (!fixed && L == 1 && p->host.sc_kind == 2) {
        // (layout chosen above)
    } else if (fixed && L == 1 && p->host.sc_kind == 0 &&
        pcg::sccs_layout(N, &p->wave_lds_floats, &p->lds_stage_limit, &p->scratch_floats) == 0) {
        // lane-serial 8-bit Fast-SSC
    } else if (fixed && L == 1) {
        p->host.sc_kind = 1; // one codeword per wave (sc_char_kernel.hip)
        p->scratch_floats = 0;
        p->wave_lds_floats = pcg::sc_wave_lds_floats(N);
    } else if (fixed) {
        uint64_t sd = 0;
        rc = pcg::sclc_layout(N, L, &p->wave_lds_floats, &p->lds_stage_limit, &sd);
        if (rc != 0) {
            delete p;
            return fail(rc, "8-bit list decoding layout unsupported for this N/L");
        }
        p->scratch_floats = sd;
    } else if (L == 1 && p->host.sc_kind == 0 &&
               pcg::scs_layout(N, &p->wave_lds_floats, &p->lds_stage_limit, &p->scratch_floats) == 0) {
        // lane-serial Fast-SSC (its per-lane bit rows fit the LDS up to N = 8192)
    } else if (L == 1) {
        p->host.sc_kind = 1; // one codeword per wave (sc_kernel.hip)
        p->scratch_floats = 0;
        p->wave_lds_floats = pcg::sc_wave_lds_floats(N);
    } else {
        // lanes per codeword: the caller's request, else the PCG_SCL_LP dev override; used
        // when it is a power of two between list_pow2(L) and 32
        if (const char* e = getenv("PCG_SCL_LP"); e && scl_lp == 0) {
            scl_lp = (uint32_t)strtoul(e, nullptr, 10);
            p->dev_overrides |= PCG_DEV_SCL_LP;
        }
        p->scl_lp = list_pow2(L);
        if (scl_lp > p->scl_lp && scl_lp <= 32 && (scl_lp & (scl_lp - 1)) == 0)
            p->scl_lp = scl_lp;
        if (const char* e = getenv("PCG_SCL_FUSE")) {
            p->scl_fuse = (uint32_t)atoi(e);
            p->dev_overrides |= PCG_DEV_SCL_FUSE;
        }
        // (an adaptive plan's list stage is one walk over a few frames: its latency, not its
        // traffic, counts -- the root's children only: 6.18e7 vs 5.99e7 cw/s for AdaptiveFloat
        // L = 8, profiles/r03p_adaptive_virt_sweep.txt)
        const uint32_t vleaf = (p->scl_fuse & 5u) == 5u && !walk_latency
                                   ? scl_leaf_free_levels(p->host.ops, p->host.log2N)
                                   : 0u;
        rc = pcg::sclls_layout(N, L, p->scl_lp, vleaf, &p->wave_lds_floats, &p->lds_stage_limit,
                               &p->scratch_floats, &p->scl_virt, &p->scl_v3, &p->scl_sb);
        if (rc != 0) {
            delete p;
            return fail(rc, "list decoding layout unsupported for this N/L");
        }
    }
    p->kernel = kernel_name(p->host, p->scl_lp);
    p->walk_latency = walk_latency;
    if (!fixed && L > 1) {
        bool nd = false;
        (void)pcg::sclls_rtc_defines(&nd);
        if (nd) // a dev build of the list kernel (tools/build_dev_lib.sh -D...)
            p->dev_overrides |= PCG_DEV_BUILD;
    }
    if (getenv("PCG_RTC_XOPTS")) // extra compiler options for the specialised kernels
        p->dev_overrides |= PCG_DEV_BUILD;
    if (const char* e = getenv("PCG_RTC_SCL"); e && e[0] == '0') {
        p->rtc_scl = false;
        p->dev_overrides |= PCG_DEV_LAYOUT;
    }
    if (const char* e = getenv("PCG_RTC")) // 0: interpreter only, 1: specialise at the first decode
        p->rtc_mode = e[0] == '0' ? 0 : (e[0] == '1' ? 1 : 2);
    p->dev_opprof = getenv("PCG_OPPROF") != nullptr;
    if (p->dev_opprof)
        p->dev_overrides |= PCG_DEV_OPPROF;
    if (const char* fl = getenv("PCG_FLAGS")) {
        p->dev_flags = (uint32_t)strtoul(fl, nullptr, 0);
        if (p->dev_flags)
            p->dev_overrides |= PCG_DEV_FLAGS;
    }
    for (const char* v : {"PCG_SC_KERNEL", "PCG_SCL_V3", "PCG_SCL_LDS_KB", "PCG_SCL_STAGE_LIMIT", "PCG_SCL_VIRT", "PCG_SCL_QUEUE",
                          "PCG_SCQ_WPC", "PCG_SCS_WPC", "PCG_SCL_WPC", "PCG_SCCS_WPC", "PCG_SCLC_WPC",
                          "PCG_SCS_LDS_KB", "PCG_SCS_SL", "PCG_SCCS_LDS_KB", "PCG_SCCS_SL", "PCG_SCLC_LDS_KB",
                          "PCG_SCLC_SL"})
        if (getenv(v))
            p->dev_overrides |= PCG_DEV_LAYOUT;
    if (device < 0) { // host-only plan: classification / validation without a GPU
        p->device = -1;
        *out = p;
        return PCG_OK;
    }
    int ndev = pcg_device_count();
    if (ndev <= 0) {
        delete p;
        return fail(PCG_E_NODEVICE, "no HIP device available");
    }
    if (device >= ndev) {
        delete p;
        return fail(PCG_E_ARG, "device index out of range");
    }
    p->device = device;
    DeviceGuard g(device);
    if (!g.ok) {
        delete p;
        return fail(PCG_E_HIP, "hipSetDevice failed");
    }
    const auto& h = p->host;
    hipError_t e;
    if ((e = hipEventCreateWithFlags(&p->last_ev, hipEventDisableTiming)) != hipSuccess) {
        p->last_ev = nullptr;
        delete p;
        return hip_fail(e, "hipEventCreate(plan order)");
    }
    if ((e = hipMalloc(&p->d_ops, 4 * std::max<size_t>(1, h.ops.size() + h.ops_fused.size()))) != hipSuccess ||
        // info positions padded to whole 16-byte groups (scq_kernel.hip reads 8 at once)
        (e = hipMalloc(&p->d_info_pos, 2 * (h.info_pos.size() + 16))) != hipSuccess ||
        (e = hipMalloc(&p->d_crc_m, 4 * (h.crc_m.size() + h.crc_rows.size() + 1))) != hipSuccess) {
        free_plan_device(p);
        delete p;
        return hip_fail(e, "hipMalloc(plan)");
    }
    // wave caps (hipOccupancy) of the lane-serial kernels, once per plan
    if (h.fixed && h.L == 1 && h.sc_kind == 0) {
        p->wave_cap = pcg::sccs_wave_cap(p->wave_lds_floats, false);
        p->wave_cap_i8 = pcg::sccs_wave_cap(p->wave_lds_floats, true);
    } else if (h.fixed && h.L > 1) {
        p->wave_cap = pcg::sclc_wave_cap(h.L, p->wave_lds_floats, false);
        p->wave_cap_i8 = pcg::sclc_wave_cap(h.L, p->wave_lds_floats, true);
    } else if (!h.fixed && h.L == 1 && h.sc_kind == 2) {
        p->wave_cap = pcg::scq_wave_cap(h.scq_q, h.scq_virt != 0, p->wave_lds_floats);
    } else if (!h.fixed && h.L == 1 && h.sc_kind == 0) {
        p->wave_cap = pcg::scs_wave_cap(p->wave_lds_floats);
    } else if (!h.fixed && h.L > 1) {
        p->wave_cap = pcg::sclls_wave_cap(p->scl_lp, p->wave_lds_floats);
        const char* q = getenv("PCG_SCL_QUEUE"); // dev switch: 0 = static grid stride
        if (!(q && q[0] == '0')) {
            if ((e = hipMalloc(&p->d_queue, sizeof(uint32_t))) != hipSuccess) {
                free_plan_device(p);
                delete p;
                return hip_fail(e, "hipMalloc(work queue)");
            }
        }
    }
    if ((e = hipMemcpy(p->d_ops, h.ops.data(), 4 * h.ops.size(), hipMemcpyHostToDevice)) != hipSuccess ||
        (!h.ops_fused.empty() && (e = hipMemcpy(p->d_ops + h.ops.size(), h.ops_fused.data(), 4 * h.ops_fused.size(),
                                                hipMemcpyHostToDevice)) != hipSuccess) ||
        (!h.info_pos.empty() &&
         (e = hipMemcpy(p->d_info_pos, h.info_pos.data(), 2 * h.info_pos.size(), hipMemcpyHostToDevice)) !=
             hipSuccess) ||
        (!h.crc_m.empty() &&
         (e = hipMemcpy(p->d_crc_m, h.crc_m.data(), 4 * h.crc_m.size(), hipMemcpyHostToDevice)) != hipSuccess) ||
        (!h.crc_rows.empty() &&
         (e = hipMemcpy(p->d_crc_m + h.crc_m.size(), h.crc_rows.data(), 4 * h.crc_rows.size(),
                        hipMemcpyHostToDevice)) != hipSuccess)) {
        free_plan_device(p);
        delete p;
        return hip_fail(e, "hipMemcpy(plan)");
    }
    *out = p;
    return PCG_OK;
}

int pcg_plan_create(pcg_plan** out,
                    uint32_t N,
                    uint32_t L,
                    const uint32_t* frozen,
                    uint32_t n_frozen,
                    int systematic,
                    int crc_kind,
                    int device)
{
    return plan_create_impl(out, N, L, frozen, n_frozen, systematic, crc_kind, device, 0);
}

int pcg_plan_create_char(pcg_plan** out,
                         uint32_t N,
                         uint32_t L,
                         const uint32_t* frozen,
                         uint32_t n_frozen,
                         int systematic,
                         int crc_kind,
                         int device)
{
    return plan_create_impl(out, N, L, frozen, n_frozen, systematic, crc_kind, device, 1);
}

static int plan_create_adaptive_impl(pcg_plan** out,
                                     uint32_t N,
                                     uint32_t L,
                                     const uint32_t* frozen,
                                     uint32_t n_frozen,
                                     int systematic,
                                     int crc_kind,
                                     int device,
                                     int fixed)
{
    if (L < 2) // makeDecoder with listSize 1 builds the plain Fast-SSC decoder (decoder.cpp:60-68)
        return plan_create_impl(out, N, L, frozen, n_frozen, systematic, crc_kind, device, fixed);
    // The SCL stage decodes only the Fast-SSC failures: a few frames per launch at useful
    // SNRs, so its time is about one walk's latency.  PCG_ADAPT_LP (dev override) runs it
    // with wider lane groups, the lanes beyond the list sharing every F/G.
    uint32_t lp = ADAPT_SCL_LP;
    const char* lpe = getenv("PCG_ADAPT_LP");
    if (lpe)
        lp = (uint32_t)strtoul(lpe, nullptr, 10);
    int rc = plan_create_impl(out, N, L, frozen, n_frozen, systematic, crc_kind, device, fixed, fixed ? 0 : lp, true);
    if (rc != 0)
        return rc;
    if (lpe)
        (*out)->dev_overrides |= PCG_DEV_SCL_LP;
    pcg_plan* fast = nullptr;
    // the Fast-SSC stage rejects what its constructor rejects (invalid_argument)
    rc = plan_create_impl(&fast, N, 1, frozen, n_frozen, systematic, crc_kind, device, fixed);
    if (rc != 0) {
        std::string msg = g_last_error;
        pcg_plan_destroy(*out);
        *out = nullptr;
        return fail(rc, msg);
    }
    (*out)->fast = fast;
    return PCG_OK;
}

int pcg_plan_create_adaptive(pcg_plan** out,
                             uint32_t N,
                             uint32_t L,
                             const uint32_t* frozen,
                             uint32_t n_frozen,
                             int systematic,
                             int crc_kind,
                             int device)
{
    return plan_create_adaptive_impl(out, N, L, frozen, n_frozen, systematic, crc_kind, device, 0);
}

int pcg_plan_create_adaptive_char(pcg_plan** out,
                                  uint32_t N,
                                  uint32_t L,
                                  const uint32_t* frozen,
                                  uint32_t n_frozen,
                                  int systematic,
                                  int crc_kind,
                                  int device)
{
    return plan_create_adaptive_impl(out, N, L, frozen, n_frozen, systematic, crc_kind, device, 1);
}

int pcg_plan_set_initial_metric(pcg_plan* p, float metric0)
{
    if (!p)
        return fail(PCG_E_ARG, "null plan");
    p->metric0 = metric0;
    return PCG_OK;
}

const char* pcg_plan_kernel_name(const pcg_plan* p)
{
    if (!p)
        return "";
    return p->kernel;
}

int pcg_plan_describe(const pcg_plan* p, pcg_plan_desc* d)
{
    if (!p || !d)
        return fail(PCG_E_ARG, "null argument");
    d->block_length = p->host.N;
    d->info_length = p->host.K;
    d->list_size = p->host.L;
    d->node_count = p->host.node_count;
    d->op_count = (uint32_t)p->host.ops.size();
    d->lds_bytes = p->wave_lds_floats * 4;
    d->scratch_bytes = p->scratch_floats * 4;
    d->crc_kind = p->host.crc_kind;
    d->systematic = p->host.systematic;
    d->lanes_per_codeword = p->host.L > 1 && !p->host.fixed ? p->scl_lp
                          : (p->host.L == 1 && p->host.sc_kind == 2 ? p->host.scq_q : 0);
    d->dev_overrides = p->dev_overrides | (p->fast ? p->fast->dev_overrides : 0u);
    d->recomputed_stages = p->host.L > 1 && !p->host.fixed ? p->scl_virt : 0u;
    // every stage that has a specialised kernel runs it (an adaptive plan: both stages, float
    // and 8-bit alike)
    {
        bool any = false, all = true;
        for (const pcg_plan* q : {(const pcg_plan*)p->fast, p})
            if (q && rtc_capable(q)) {
                any = any || q->rtc_state == 1;
                all = all && q->rtc_state == 1;
            }
        d->specialized = any && all ? 1u : 0u;
    }
    return PCG_OK;
}

static int plan_specialize(pcg_plan* p, bool wait)
{
    if (!p)
        return fail(PCG_E_ARG, "null plan");
    if (p->fast) { // adaptive plans: both stages (the list stage: float plans only)
        const int rc = plan_specialize(p->fast, wait);
        if (rc != 0 || !rtc_capable(p))
            return rc;
    }
    if (!rtc_capable(p))
        return fail(PCG_E_UNSUPPORTED, "no plan-specialised kernel for this plan (not with PCG_OPPROF; the "
                                       "8-bit Fast-SSC decoder on its one-codeword-per-wave kernel has none)");
    if (p->device < 0)
        return specialize(p, wait);
    DeviceGuard g(p->device);
    if (!g.ok)
        return fail(PCG_E_HIP, "hipSetDevice failed");
    return specialize(p, wait);
}

int pcg_plan_specialize(pcg_plan* p) { return plan_specialize(p, true); }

int pcg_plan_specialize_async(pcg_plan* p) { return plan_specialize(p, false); }

static int decode_impl(pcg_plan* p,
                       const float* llr,
                       uint64_t F,
                       uint8_t* info,
                       uint8_t* ok,
                       float* metrics,
                       void* stream,
                       const uint32_t* fmap,
                       const uint32_t* fcount,
                       const int8_t* llr8 = nullptr,
                       float* soft = nullptr,
                       const int32_t* pmap = nullptr,
                       uint32_t in_stride = 0);

static int decode_adaptive(pcg_plan* p, const float* llr, uint64_t F, uint8_t* info, uint8_t* ok, float* metrics,
                           void* stream, const int8_t* llr8 = nullptr)
{
    // AdaptiveFloat::decode (adaptive_float.cpp:33-45): Fast-SSC for every frame, then SCL
    // for the frames whose check failed, whose SCL output (and ok) replaces the SC one.
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipError_t e;
    int rc = order_on(p, s); // d_fmap / d_okbuf are reused: after the previous call's readers
    if (rc != 0)
        return rc;
    if (p->fmap_frames < F) {
        (void)hipFree(p->d_fmap);
        (void)hipFree(p->d_okbuf);
        p->d_fmap = nullptr;
        p->d_okbuf = nullptr;
        p->fmap_frames = 0;
        if ((e = hipMalloc(&p->d_fmap, 4 * (F + 1))) != hipSuccess || (e = hipMalloc(&p->d_okbuf, F)) != hipSuccess)
            return hip_fail(e, "hipMalloc(adaptive)");
        p->fmap_frames = F;
    }
    uint8_t* okb = ok ? ok : p->d_okbuf;
    rc = decode_impl(p->fast, llr, F, info, okb, nullptr, stream, nullptr, nullptr, llr8);
    if (rc != 0)
        return rc;
    if (metrics && (e = hipMemsetAsync(metrics, 0, F * p->host.L * sizeof(float), s)) != hipSuccess)
        return hip_fail(e, "hipMemsetAsync(metrics)");
    if (pcg::launch_compact_failed(okb, F, p->d_fmap + 1, p->d_fmap, s) != 0)
        return fail(PCG_E_HIP, std::string("compaction launch failed: ") + hipGetErrorString(hipGetLastError()));
    return decode_impl(p, llr, F, info, okb, metrics, stream, p->d_fmap + 1, p->d_fmap, llr8);
}

int pcg_decode_f32(pcg_plan* p,
                   const float* llr,
                   uint64_t F,
                   uint8_t* info,
                   uint8_t* ok,
                   float* metrics,
                   void* stream)
{
    if (!p)
        return fail(PCG_E_ARG, "null plan");
    if (F == 0)
        return PCG_OK;
    if (!llr || !info)
        return fail(PCG_E_ARG, "null llr/info buffer");
    if (p->device < 0)
        return fail(PCG_E_NODEVICE, "host-only plan (created with device < 0)");
    if (F > 0xFFFFFFFFull)
        return fail(PCG_E_ARG, "at most 2^32 - 1 frames per call");
    DeviceGuard g(p->device);
    if (p->fast)
        return decode_adaptive(p, llr, F, info, ok, metrics, stream);
    return decode_impl(p, llr, F, info, ok, metrics, stream, nullptr, nullptr);
}

static int decode_impl(pcg_plan* p,
                       const float* llr,
                       uint64_t F,
                       uint8_t* info,
                       uint8_t* ok,
                       float* metrics,
                       void* stream,
                       const uint32_t* fmap,
                       const uint32_t* fcount,
                       const int8_t* llr8,
                       float* soft,
                       const int32_t* pmap,
                       uint32_t in_stride)
{
    const auto& h = p->host;
    pcg::KernelArgs a{};
    a.llr = llr;
    a.F = F;
    a.ops = p->d_ops;
    a.nops = (uint32_t)h.ops.size();
    a.N = h.N;
    a.log2N = h.log2N;
    a.K = h.K;
    a.kb = (h.K + 7) / 8;
    a.L = h.L;
    a.info_pos = p->d_info_pos;
    a.crc_m = p->d_crc_m;
    a.crc_bits = (uint32_t)h.crc_kind;
    a.crc_rows = p->d_crc_m + h.crc_m.size();
    a.crc_c0 = h.crc_c0;
    a.systematic = h.systematic;
    a.info = info;
    a.ok = ok;
    a.metrics = metrics;
    a.wave_lds_floats = p->wave_lds_floats;
    a.lds_stage_limit = p->lds_stage_limit;
    a.scl_virt = p->scl_virt;
    a.scl_v3 = p->scl_v3;
    a.scl_sb = p->scl_sb;
    a.scl_fuse = p->scl_fuse;
    a.scratch_floats = p->scratch_floats;
    a.fmap = fmap;
    a.fcount = fcount;
    a.llr8 = llr8;
    a.metric0 = p->metric0;
    if (p->dev_opprof) {
        if (!g_prof && hipMalloc(&g_prof, kProfN * sizeof(unsigned long long)) == hipSuccess)
            (void)hipMemset(g_prof, 0, kProfN * sizeof(unsigned long long));
        a.prof = g_prof;
    }
    a.flags = p->dev_flags;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool i8 = llr8 != nullptr;
    int rc = order_on(p, s);
    if (rc != 0)
        return rc;
    if (soft) { // soft codeword: the one-codeword-per-wave Fast-SSC kernel (float plans, L = 1)
        a.soft = soft;
        a.wave_lds_floats = pcg::sc_wave_lds_floats(h.N);
        rc = pcg::launch_sc(a, s);
    } else if (h.fixed && h.L == 1 && h.sc_kind == 0) {
        auto_specialize(p, F); // (before the grid: a loaded kernel brings its own occupancy)
        a.units = (uint32_t)pcg::wave_units(F, 64, i8 ? p->wave_cap_i8 : p->wave_cap);
        if ((rc = grow_scratch(p, a.units, sizeof(uint32_t), s)) != 0)
            return rc;
        a.scratch = p->d_scratch;
        rc = p->rtc_state == 1 ? pcg::rtc_launch(i8 ? p->rtc_fn_i8 : p->rtc_fn, a, s) : pcg::launch_sccs(a, s);
    } else if (h.fixed && h.L == 1) {
        rc = pcg::launch_sc_char(a, s);
    } else if (h.fixed) {
        auto_specialize(p, F); // (before the grid: a loaded kernel brings its own occupancy)
        a.units = (uint32_t)pcg::wave_units(F, 64 / list_pow2(h.L), i8 ? p->wave_cap_i8 : p->wave_cap);
        if ((rc = grow_scratch(p, a.units, sizeof(uint32_t), s)) != 0)
            return rc;
        a.scratch = p->d_scratch;
        rc = p->rtc_state == 1 ? pcg::rtc_launch(i8 ? p->rtc_fn_i8 : p->rtc_fn, a, s) : pcg::launch_scl_char(a, s);
    } else if (h.L == 1 && h.sc_kind == 2) {
        a.units = (uint32_t)pcg::wave_units(F, 64 / h.scq_q, p->wave_cap);
        a.ops = p->d_ops + h.ops.size(); // the fused schedule (plan.cpp fuse_sc16)
        a.nops = (uint32_t)h.ops_fused.size();
        auto_specialize(p, F); // on failure the interpreter runs (rtc_err says why)
        rc = p->rtc_state == 1 ? pcg::rtc_launch(p->rtc_fn, a, s) : pcg::launch_scq(a, h.scq_q, h.scq_virt != 0, s);
    } else if (h.L == 1 && h.sc_kind == 0) {
        a.units = (uint32_t)pcg::wave_units(F, 64, p->wave_cap);
        if ((rc = grow_scratch(p, a.units, sizeof(float), s)) != 0)
            return rc;
        a.scratch = p->d_scratch;
        rc = pcg::launch_scs(a, s);
    } else if (h.L == 1) {
        rc = pcg::launch_sc(a, s);
    } else {
        a.scl_lp = p->scl_lp;
        a.units = (uint32_t)pcg::wave_units(F, 64 / p->scl_lp, p->wave_cap);
        if (pmap) { // punctured frames: each wave depunctures its group into its scratch
            a.pmap = pmap;
            a.in_stride = in_stride;
            a.scratch_floats = p->scratch_floats + (uint64_t)(64 / p->scl_lp) * h.N;
        }
        if ((rc = grow_scratch(p, a.units, sizeof(float), s, a.scratch_floats)) != 0)
            return rc;
        a.scratch = p->d_scratch;
        a.queue = p->d_queue;
        if (a.queue) { // the work-queue counter starts at 0 for every launch, in stream order
            hipError_t e = hipMemsetAsync(a.queue, 0, sizeof(uint32_t), s);
            if (e != hipSuccess)
                return hip_fail(e, "hipMemsetAsync(work queue)");
        }
        auto_specialize(p, F);
        rc = p->rtc_state == 1 ? pcg::rtc_launch(p->rtc_fn, a, s) : pcg::launch_sclls(a, s);
    }
    if (rc != 0)
        return fail(rc, std::string("kernel launch failed: ") + hipGetErrorString(hipGetLastError()));
    return mark_done(p, s);
}

int pcg_decode_i8(pcg_plan* p,
                  const int8_t* llr,
                  uint64_t F,
                  uint8_t* info,
                  uint8_t* ok,
                  float* metrics,
                  void* stream)
{
    if (!p)
        return fail(PCG_E_ARG, "null plan");
    if (!p->host.fixed)
        return fail(PCG_E_ARG, "int8 LLRs need an 8-bit plan (pcg_plan_create_char)");
    if (F == 0)
        return PCG_OK;
    if (!llr || !info)
        return fail(PCG_E_ARG, "null llr/info buffer");
    if (p->device < 0)
        return fail(PCG_E_NODEVICE, "host-only plan (created with device < 0)");
    if (F > 0xFFFFFFFFull)
        return fail(PCG_E_ARG, "at most 2^32 - 1 frames per call");
    DeviceGuard g(p->device);
    if (p->fast)
        return decode_adaptive(p, nullptr, F, info, ok, metrics, stream, llr);
    return decode_impl(p, nullptr, F, info, ok, metrics, stream, nullptr, nullptr, llr);
}

// ---- host-pointer decodes: the overlapped pipeline ----------------------------------------
// Reference callers: Decoder::decode_vector (decoder.cpp:154-181), pypolar decode on numpy
// arrays (python/bindings/decoder_python.cc:41-75), the simulator's block loop
// (simulator.cpp:920-937) -- all hand over host buffers.  The batch is cut into chunks that
// alternate between two slots (HostPipe): the host stages chunk i+1 and the copy stream
// moves it to the device while the decode stream decodes chunk i, whose (small) outputs come
// back on the decode stream into pinned memory and are handed to the caller when the slot
// is reused.  PCG_HOST_PIPE selects the staging (development A/B; default 2):
//   0  serial: blocking pageable copies, then the decode, chunk by chunk (no overlap);
//   1  the caller's pageable buffer copied by the runtime on the copy stream (the host thread
//      blocks in the copy while the previous chunk decodes);
//   2  plan-owned pinned staging filled by PCG_HOST_THREADS host threads (default 8; with
//      non-temporal stores, PCG_HOST_NT=0: plain memcpy), then a DMA copy on the copy stream;
//   3  each chunk's whole pages page-locked in place for its copy (hipHostRegister, overlapped
//      with the previous chunk's copy), the partial end pages staged as in 2.
// A caller buffer that is already pinned (hipHostMalloc / hipHostRegister) is copied from
// directly in modes 1 and 2.  PCG_HOST_CHUNK overrides the chunk size in frames (default:
// 64 MB of input, between 4096 and 65536 frames).
static int env_int(const char* name, int dflt)
{
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

// A copy into the pinned staging with non-temporal 16-byte stores: the destination is only read
// by the DMA engine, so its lines need not be fetched into the cache first (ordinary stores read
// each line before writing it: a third of the host memory traffic of the staging copy).
static void nt_memcpy(void* dst, const void* src, size_t bytes)
{
    char* d = (char*)dst;
    const char* s = (const char*)src;
    size_t head = (16 - ((uintptr_t)d & 15)) & 15;
    if (head > bytes)
        head = bytes;
    memcpy(d, s, head);
    d += head;
    s += head;
    bytes -= head;
    size_t i = 0;
    for (; i + 64 <= bytes; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i*)(s + i)), b = _mm_loadu_si128((const __m128i*)(s + i + 16)),
                      c = _mm_loadu_si128((const __m128i*)(s + i + 32)), e = _mm_loadu_si128((const __m128i*)(s + i + 48));
        _mm_stream_si128((__m128i*)(d + i), a);
        _mm_stream_si128((__m128i*)(d + i + 16), b);
        _mm_stream_si128((__m128i*)(d + i + 32), c);
        _mm_stream_si128((__m128i*)(d + i + 48), e);
    }
    memcpy(d + i, s + i, bytes - i);
    _mm_sfence();
}

static void par_memcpy(void* dst, const void* src, size_t bytes, int threads, bool nt)
{
    auto cp = nt ? nt_memcpy : [](void* d, const void* s, size_t n) { memcpy(d, s, n); };
    const size_t per = size_t(4) << 20; // at least 4 MB per thread
    int t = (int)std::min<size_t>((size_t)std::max(threads, 1), (bytes + per - 1) / per);
    if (t <= 1) {
        cp(dst, src, bytes);
        return;
    }
    const size_t part = ((bytes + t - 1) / t + 4095) & ~size_t(4095);
    std::vector<std::thread> th;
    for (int k = 1; k < t; ++k) {
        const size_t o = part * k;
        if (o >= bytes)
            break;
        th.emplace_back([=] { cp((char*)dst + o, (const char*)src + o, std::min(part, bytes - o)); });
    }
    cp(dst, src, std::min(part, bytes));
    for (auto& x : th)
        x.join();
}

// Stage `bytes` of pageable input into the pinned buffer `h` and copy it to `d` on `st`, piece by
// piece: the host threads (started once) each copy their share of piece k and count it done; the
// calling thread issues piece k's DMA as soon as every share has landed, while the threads go on
// with piece k+1.
static hipError_t staged_copy(void* h, void* d, const char* src, size_t bytes, size_t piece0, size_t piece,
                              int threads, bool nt, hipStream_t st)
{
    if (piece >= bytes || threads <= 1) {
        par_memcpy(h, src, bytes, threads, nt);
        return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st);
    }
    // piece i = [off(i), off(i + 1)): the first one piece0 long (the copy engine starts sooner),
    // then piece
    piece0 = std::min(piece0, piece);
    auto off = [&](size_t i) { return i == 0 ? size_t(0) : std::min(bytes, piece0 + (i - 1) * piece); };
    const size_t np = 1 + (bytes > piece0 ? (bytes - piece0 + piece - 1) / piece : 0);
    auto cp = nt ? nt_memcpy : [](void* dd, const void* ss, size_t n) { memcpy(dd, ss, n); };
    std::vector<std::atomic<int>> done(np);
    for (auto& x : done)
        x.store(0, std::memory_order_relaxed);
    const int t = threads;
    auto work = [&](int k) {
        for (size_t i = 0; i < np; ++i) {
            const size_t o = off(i), pb = off(i + 1) - o;
            const size_t part = ((pb + t - 1) / t + 4095) & ~size_t(4095), a = part * (size_t)k;
            if (a < pb)
                cp((char*)h + o + a, src + o + a, std::min(part, pb - a));
            done[i].fetch_add(1, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    for (int k = 0; k < t; ++k)
        th.emplace_back(work, k);
    hipError_t e = hipSuccess;
    for (size_t i = 0; i < np && e == hipSuccess; ++i) {
        while (done[i].load(std::memory_order_acquire) < t)
            std::this_thread::yield();
        const size_t o = off(i);
        e = hipMemcpyAsync((char*)d + o, (const char*)h + o, off(i + 1) - o, hipMemcpyHostToDevice, st);
    }
    for (auto& x : th)
        x.join();
    return e;
}

static int pipe_alloc(pcg_plan* p, uint64_t frames, size_t in_fb, bool pinned_in)
{
    HostPipe* q = p->pipe;
    const auto& h = p->host;
    if (q && q->frames >= frames && q->in_fb >= in_fb && (!pinned_in || q->h_in[0]))
        return PCG_OK;
    if (q) { // grow: everything queued on the old buffers finishes first
        frames = std::max(frames, q->frames);
        in_fb = std::max(in_fb, q->in_fb);
        pinned_in = pinned_in || q->h_in[0];
        free_pipe(q);
        p->pipe = nullptr;
    }
    q = new HostPipe;
    p->pipe = q;
    q->frames = frames;
    q->in_fb = in_fb;
    q->L = h.L;
    q->kb = std::max<uint64_t>((h.K + 7) / 8, 1);
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&q->copy, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipStreamCreateWithFlags(&q->dec, hipStreamNonBlocking)) != hipSuccess)
        return hip_fail(e, "hipStreamCreate(host pipeline)");
    const size_t out_b = frames * (q->kb + 1 + h.L * sizeof(float));
    for (int b = 0; b < 2; ++b) {
        if ((e = hipMalloc(&q->d_in[b], frames * in_fb)) != hipSuccess ||
            (e = hipMalloc(&q->d_info[b], frames * q->kb)) != hipSuccess ||
            (e = hipMalloc(&q->d_ok[b], frames)) != hipSuccess ||
            (e = hipMalloc(&q->d_met[b], frames * h.L * sizeof(float))) != hipSuccess)
            return hip_fail(e, "hipMalloc(host pipeline)");
        if ((e = hipHostMalloc(&q->h_out[b], out_b, hipHostMallocDefault)) != hipSuccess)
            return hip_fail(e, "hipHostMalloc(host pipeline outputs)");
        if (pinned_in && (e = hipHostMalloc(&q->h_in[b], frames * in_fb, hipHostMallocDefault)) != hipSuccess)
            return hip_fail(e, "hipHostMalloc(host pipeline staging)");
        if ((e = hipEventCreateWithFlags(&q->ev_h2d[b], hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&q->ev_done[b], hipEventDisableTiming)) != hipSuccess)
            return hip_fail(e, "hipEventCreate(host pipeline)");
    }
    return PCG_OK;
}

// the caller's buffer is page-locked host memory the DMA engines can read directly
static bool host_pinned(const void* ptr)
{
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, ptr) != hipSuccess) {
        (void)hipGetLastError(); // (pageable memory: not an error worth keeping)
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

static int decode_host_serial(pcg_plan* p, const void* llr, size_t elem, uint64_t F, uint8_t* info, uint8_t* ok,
                              float* metrics, uint64_t chunk)
{
    const auto& h = p->host;
    const uint64_t kb = (h.K + 7) / 8;
    const size_t fb = h.N * elem;
    int rc = pipe_alloc(p, chunk, fb, false);
    if (rc != 0)
        return rc;
    HostPipe* q = p->pipe;
    hipError_t e;
    for (uint64_t f0 = 0; f0 < F; f0 += chunk) {
        const uint64_t n = std::min(chunk, F - f0);
        if ((e = hipMemcpy(q->d_in[0], (const char*)llr + f0 * fb, n * fb, hipMemcpyHostToDevice)) != hipSuccess)
            return hip_fail(e, "hipMemcpy(H2D)");
        rc = elem == 1 ? pcg_decode_i8(p, (const int8_t*)q->d_in[0], n, q->d_info[0], ok ? q->d_ok[0] : nullptr,
                                       metrics ? q->d_met[0] : nullptr, nullptr)
                       : pcg_decode_f32(p, (const float*)q->d_in[0], n, q->d_info[0], ok ? q->d_ok[0] : nullptr,
                                        metrics ? q->d_met[0] : nullptr, nullptr);
        if (rc != 0)
            return rc;
        if ((e = hipMemcpy(info + f0 * kb, q->d_info[0], n * kb, hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "hipMemcpy(D2H info)");
        if (ok && (e = hipMemcpy(ok + f0, q->d_ok[0], n, hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "hipMemcpy(D2H ok)");
        if (metrics &&
            (e = hipMemcpy(metrics + f0 * h.L, q->d_met[0], n * h.L * sizeof(float), hipMemcpyDeviceToHost)) !=
                hipSuccess)
            return hip_fail(e, "hipMemcpy(D2H metrics)");
    }
    return PCG_OK;
}

static int decode_host(pcg_plan* p, const void* llr, size_t elem, uint64_t F, uint8_t* info, uint8_t* ok,
                       float* metrics)
{
    const auto& h = p->host;
    const uint64_t kb = (h.K + 7) / 8;
    const size_t fb = h.N * elem;
    const int mode = env_int("PCG_HOST_PIPE", 2);
    uint64_t chunk = (uint64_t)env_int("PCG_HOST_CHUNK", 0);
    if (chunk == 0)
        chunk = std::min<uint64_t>(65536, std::max<uint64_t>(4096, (64ull << 20) / fb));
    chunk = std::min<uint64_t>(chunk, F);
    if (mode == 0)
        return decode_host_serial(p, llr, elem, F, info, ok, metrics, chunk);
    const bool direct = host_pinned(llr);
    const bool stage = (mode == 2 || mode == 3) && !direct;
    const bool reg = mode == 3 && !direct;
    const int threads = env_int("PCG_HOST_THREADS", 8);
    const bool nt = env_int("PCG_HOST_NT", 1) != 0;
    // staging piece (PCG_HOST_PIECE_MB, default 16 MB; 0: the whole chunk at once, round 5).
    // Measured on config 3 (profiles/r06d_host_pieces.txt, 8 threads, chunk 16384 frames = 64 MB):
    // whole chunk 1.008e7 cw/s, pieces of 4 / 8 / 16 MB 1.029e7 / 1.068e7 / 1.079e7 (a page-locked
    // caller buffer, no staging: 1.127e7)
    const int piece_mb = env_int("PCG_HOST_PIECE_MB", 16);
    const size_t piece = piece_mb > 0 ? (size_t)piece_mb << 20 : ~size_t(0);
    // the batch's first piece is shorter (PCG_HOST_FIRST_KB, default 2048): nothing overlaps its staging
    const size_t piece_first = (size_t)std::max(env_int("PCG_HOST_FIRST_KB", 2048), 64) << 10;
    int rc = pipe_alloc(p, chunk, fb, stage);
    if (rc != 0)
        return rc;
    HostPipe* q = p->pipe;
    hipError_t e;
    // mode 3: each chunk's whole pages are page-locked in place (hipHostRegister, while the
    // previous chunk's copy runs) and copied from directly; the partial pages at its ends go
    // through the staging buffer.  Every registration ends once its copy has completed (and on
    // any error return, after the copy stream has drained).
    struct Reg {
        void* p = nullptr;
    } regs[2];
    struct RegGuard {
        HostPipe* q;
        Reg* r;
        ~RegGuard()
        {
            if (!r[0].p && !r[1].p)
                return;
            (void)hipStreamSynchronize(q->copy);
            for (int k = 0; k < 2; ++k)
                if (r[k].p)
                    (void)hipHostUnregister(r[k].p);
        }
    } guard{q, regs};
    auto unreg = [&](int b) {
        if (regs[b].p) {
            (void)hipHostUnregister(regs[b].p);
            regs[b].p = nullptr;
        }
    };
    // the slots' buffers are reused after the plan's previous decodes, whatever stream ran them
    if ((rc = order_on(p, q->copy)) != 0)
        return rc;
    struct Pending {
        uint64_t f0 = 0, n = 0;
        bool live = false;
    } pend[2];
    const size_t o_ok = chunk * kb, o_met = o_ok + chunk;
    auto retire = [&](int b) -> int {
        if (!pend[b].live)
            return PCG_OK;
        pend[b].live = false;
        hipError_t x = hipEventSynchronize(q->ev_done[b]);
        if (x != hipSuccess)
            return hip_fail(x, "hipEventSynchronize(host pipeline)");
        unreg(b); // (its copy has completed)
        const uint64_t f0 = pend[b].f0, n = pend[b].n;
        memcpy(info + f0 * kb, q->h_out[b], n * kb);
        if (ok)
            memcpy(ok + f0, q->h_out[b] + o_ok, n);
        if (metrics)
            memcpy(metrics + f0 * h.L, q->h_out[b] + o_met, n * h.L * sizeof(float));
        return PCG_OK;
    };
    uint64_t i = 0;
    for (uint64_t f0 = 0; f0 < F; f0 += chunk, ++i) {
        const int b = (int)(i & 1u);
        const uint64_t n = std::min(chunk, F - f0);
        // chunk i-2 leaves slot b: its decode (and so its input copy) is complete
        if ((rc = retire(b)) != 0)
            return rc;
        const char* src = (const char*)llr + f0 * fb;
        const size_t nb = n * fb;
        bool done = false;
        if (reg) {
            const uintptr_t a = (uintptr_t)src, z = a + nb, pg = 4096;
            const uintptr_t pa = (a + pg - 1) & ~(pg - 1), pz = z & ~(pg - 1);
            if (pz > pa && hipHostRegister((void*)pa, pz - pa, hipHostRegisterDefault) == hipSuccess) {
                regs[b].p = (void*)pa;
                char* d = (char*)q->d_in[b];
                char* hs = (char*)q->h_in[b];
                memcpy(hs, src, pa - a);
                memcpy(hs + (pz - a), (const char*)pz, z - pz);
                if ((pa > a && (e = hipMemcpyAsync(d, hs, pa - a, hipMemcpyHostToDevice, q->copy)) != hipSuccess) ||
                    (e = hipMemcpyAsync(d + (pa - a), (const void*)pa, pz - pa, hipMemcpyHostToDevice, q->copy)) !=
                        hipSuccess ||
                    (z > pz &&
                     (e = hipMemcpyAsync(d + (pz - a), hs + (pz - a), z - pz, hipMemcpyHostToDevice, q->copy)) !=
                         hipSuccess))
                    return hip_fail(e, "hipMemcpyAsync(H2D)");
                done = true;
            } else {
                (void)hipGetLastError(); // (not registrable: staged like mode 2)
            }
        }
        if (!done && stage) {
            // staged in pieces, each copied as soon as it is staged: the DMA of piece k overlaps
            // the staging of piece k+1, so the copy engine starts after one piece (not one whole
            // chunk) and the pipeline's fill is a piece long
            if ((e = staged_copy(q->h_in[b], q->d_in[b], src, nb, i == 0 ? piece_first : piece, piece, threads, nt,
                                 q->copy)) != hipSuccess)
                return hip_fail(e, "hipMemcpyAsync(H2D)");
        } else if (!done) {
            if ((e = hipMemcpyAsync(q->d_in[b], src, nb, hipMemcpyHostToDevice, q->copy)) != hipSuccess)
                return hip_fail(e, "hipMemcpyAsync(H2D)");
        }
        if ((e = hipEventRecord(q->ev_h2d[b], q->copy)) != hipSuccess ||
            (e = hipStreamWaitEvent(q->dec, q->ev_h2d[b], 0)) != hipSuccess)
            return hip_fail(e, "host pipeline event");
        rc = elem == 1 ? pcg_decode_i8(p, (const int8_t*)q->d_in[b], n, q->d_info[b], ok ? q->d_ok[b] : nullptr,
                                       metrics ? q->d_met[b] : nullptr, q->dec)
                       : pcg_decode_f32(p, (const float*)q->d_in[b], n, q->d_info[b], ok ? q->d_ok[b] : nullptr,
                                        metrics ? q->d_met[b] : nullptr, q->dec);
        if (rc != 0)
            return rc;
        if ((e = hipMemcpyAsync(q->h_out[b], q->d_info[b], n * kb, hipMemcpyDeviceToHost, q->dec)) != hipSuccess ||
            (ok && (e = hipMemcpyAsync(q->h_out[b] + o_ok, q->d_ok[b], n, hipMemcpyDeviceToHost, q->dec)) !=
                       hipSuccess) ||
            (metrics && (e = hipMemcpyAsync(q->h_out[b] + o_met, q->d_met[b], n * h.L * sizeof(float),
                                            hipMemcpyDeviceToHost, q->dec)) != hipSuccess))
            return hip_fail(e, "hipMemcpyAsync(D2H)");
        if ((e = hipEventRecord(q->ev_done[b], q->dec)) != hipSuccess)
            return hip_fail(e, "hipEventRecord(host pipeline)");
        pend[b] = {f0, n, true};
    }
    // the last two chunks, in order
    const int last = (int)((i - 1) & 1u);
    if ((rc = retire(last ^ 1)) != 0 || (rc = retire(last)) != 0)
        return rc;
    return PCG_OK;
}

int pcg_decode_i8_host(pcg_plan* p, const int8_t* llr, uint64_t F, uint8_t* info, uint8_t* ok, float* metrics)
{
    if (!p)
        return fail(PCG_E_ARG, "null plan");
    if (!p->host.fixed)
        return fail(PCG_E_ARG, "int8 LLRs need an 8-bit plan (pcg_plan_create_char)");
    if (F == 0)
        return PCG_OK;
    if (!llr || !info)
        return fail(PCG_E_ARG, "null llr/info buffer");
    if (p->device < 0)
        return fail(PCG_E_NODEVICE, "host-only plan (created with device < 0)");
    DeviceGuard g(p->device);
    return decode_host(p, llr, 1, F, info, ok, metrics);
}

int pcg_decode_f32_host(pcg_plan* p, const float* llr, uint64_t F, uint8_t* info, uint8_t* ok, float* metrics)
{
    if (!p)
        return fail(PCG_E_ARG, "null plan");
    if (F == 0)
        return PCG_OK;
    if (!llr || !info)
        return fail(PCG_E_ARG, "null llr/info buffer");
    if (p->device < 0)
        return fail(PCG_E_NODEVICE, "host-only plan (created with device < 0)");
    DeviceGuard g(p->device);
    return decode_host(p, llr, sizeof(float), F, info, ok, metrics);
}

static int soft_supported(const pcg_plan* p)
{
    if (!p)
        return fail(PCG_E_ARG, "null plan");
    if (p->host.L != 1 || p->host.fixed || p->fast)
        return fail(PCG_E_UNSUPPORTED, "soft codewords: Fast-SSC float plans only (FastSscAvxFloat)");
    if (pcg::sc_soft_lds_bytes(p->host.N) == 0)
        return fail(PCG_E_UNSUPPORTED, "soft codewords: block length too large for one wave's LDS");
    return PCG_OK;
}

int pcg_decode_f32_soft(pcg_plan* p,
                        const float* llr,
                        uint64_t F,
                        uint8_t* info,
                        uint8_t* ok,
                        float* soft,
                        void* stream)
{
    int rc = soft_supported(p);
    if (rc != 0)
        return rc;
    if (F == 0)
        return PCG_OK;
    if (!llr || !info || !soft)
        return fail(PCG_E_ARG, "null llr/info/soft buffer");
    if (p->device < 0)
        return fail(PCG_E_NODEVICE, "host-only plan (created with device < 0)");
    if (F > 0xFFFFFFFFull)
        return fail(PCG_E_ARG, "at most 2^32 - 1 frames per call");
    DeviceGuard g(p->device);
    return decode_impl(p, llr, F, info, ok, nullptr, stream, nullptr, nullptr, nullptr, soft);
}

int pcg_decode_f32_soft_host(pcg_plan* p, const float* llr, uint64_t F, uint8_t* info, uint8_t* ok, float* soft)
{
    int rc = soft_supported(p);
    if (rc != 0)
        return rc;
    if (F == 0)
        return PCG_OK;
    if (!llr || !info || !soft)
        return fail(PCG_E_ARG, "null llr/info/soft buffer");
    if (p->device < 0)
        return fail(PCG_E_NODEVICE, "host-only plan (created with device < 0)");
    DeviceGuard g(p->device);
    const uint64_t N = p->host.N, kb = (p->host.K + 7) / 8;
    hipError_t e;
    // staging kept in the plan (pcg_decode_f32_host's buffers + a soft-codeword buffer);
    // the null-stream copies below are ordered after the plan's previous decode
    if ((rc = order_on(p, nullptr)) != 0)
        return rc;
    // (the shared LLR / info / ok staging grows to F when smaller; the soft buffer follows the
    // largest soft call alone, so a single frame after a large host batch costs N floats)
    if (p->stage_frames < F || p->soft_frames < F) {
        if ((e = hipStreamSynchronize(nullptr)) != hipSuccess)
            return hip_fail(e, "hipStreamSynchronize");
    }
    if (p->stage_frames < F) {
        (void)hipFree(p->d_llr);
        (void)hipFree(p->d_info);
        (void)hipFree(p->d_ok);
        (void)hipFree(p->d_met);
        p->d_llr = nullptr;
        p->d_info = nullptr;
        p->d_ok = nullptr;
        p->d_met = nullptr;
        p->stage_frames = 0;
        if ((e = hipMalloc(&p->d_llr, F * N * sizeof(float))) != hipSuccess ||
            (e = hipMalloc(&p->d_info, F * std::max<uint64_t>(kb, 1))) != hipSuccess ||
            (e = hipMalloc(&p->d_ok, F)) != hipSuccess ||
            (e = hipMalloc(&p->d_met, F * p->host.L * sizeof(float))) != hipSuccess)
            return hip_fail(e, "hipMalloc(soft staging)");
        p->stage_frames = F;
    }
    if (p->soft_frames < F) {
        (void)hipFree(p->d_soft);
        p->d_soft = nullptr;
        p->soft_frames = 0;
        if ((e = hipMalloc(&p->d_soft, F * N * sizeof(float))) != hipSuccess)
            return hip_fail(e, "hipMalloc(soft codewords)");
        p->soft_frames = F;
    }
    if ((e = hipMemcpy(p->d_llr, llr, F * N * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy(H2D)");
    if ((rc = pcg_decode_f32_soft(p, p->d_llr, F, p->d_info, p->d_ok, p->d_soft, nullptr)) != 0)
        return rc;
    if ((e = hipMemcpy(info, p->d_info, F * kb, hipMemcpyDeviceToHost)) != hipSuccess ||
        (e = hipMemcpy(soft, p->d_soft, F * N * sizeof(float), hipMemcpyDeviceToHost)) != hipSuccess ||
        (ok && (e = hipMemcpy(ok, p->d_ok, F, hipMemcpyDeviceToHost)) != hipSuccess))
        return hip_fail(e, "hipMemcpy(D2H)");
    return PCG_OK;
}

int pcg_decode_punctured_f32(pcg_plan* p,
                             const pcg_puncturer* punc,
                             const float* llr,
                             uint64_t F,
                             uint8_t* info,
                             uint8_t* ok,
                             float* metrics,
                             void* stream)
{
    if (!p || !punc)
        return fail(PCG_E_ARG, "null plan/puncturer");
    if (punc->N != p->host.N)
        return fail(PCG_E_ARG, "puncturer parent length != decoder block length");
    if (F == 0)
        return PCG_OK;
    if (!llr || !info)
        return fail(PCG_E_ARG, "null llr/info buffer");
    if (p->device < 0 || punc->device < 0)
        return fail(PCG_E_NODEVICE, "host-only plan or puncturer");
    if (p->device != punc->device)
        return fail(PCG_E_ARG, "plan and puncturer live on different devices");
    DeviceGuard g(p->device);
    const auto& h = p->host;
    const uint64_t kb = (h.K + 7) / 8;
    if (h.L > 1 && !h.fixed && !p->fast) {
        // float list plans depuncture inside the kernel (each wave its codeword group, into its
        // scratch slab: sclls_kernel.hip ls_depuncture) -- one launch, no staging buffer
        if (F > 0xFFFFFFFFull)
            return fail(PCG_E_ARG, "at most 2^32 - 1 frames per call");
        return decode_impl(p, llr, F, info, ok, metrics, stream, nullptr, nullptr, nullptr, nullptr, punc->d_src,
                           punc->E);
    }
    // d_dep is reused: the depuncture below runs after the plan's previous decode
    if (int rc = order_on(p, reinterpret_cast<hipStream_t>(stream)); rc != 0)
        return rc;
    // depunctured staging: at most 256 MB per chunk
    const uint64_t chunk = std::min<uint64_t>(F, std::max<uint64_t>(1, (1ull << 26) / h.N));
    if (p->dep_frames < chunk) {
        (void)hipFree(p->d_dep);
        p->d_dep = nullptr;
        p->dep_frames = 0;
        hipError_t e = hipMalloc(&p->d_dep, chunk * h.N * sizeof(float));
        if (e != hipSuccess)
            return hip_fail(e, "hipMalloc(depuncture staging)");
        p->dep_frames = chunk;
    }
    for (uint64_t f0 = 0; f0 < F; f0 += chunk) {
        const uint64_t n = std::min(chunk, F - f0);
        int rc = pcg_depuncture_f32(punc, llr + f0 * punc->E, n, p->d_dep, stream);
        if (rc != 0)
            return rc;
        rc = pcg_decode_f32(p, p->d_dep, n, info + f0 * kb, ok ? ok + f0 : nullptr,
                            metrics ? metrics + f0 * h.L : nullptr, stream);
        if (rc != 0)
            return rc;
    }
    return PCG_OK;
}

void pcg_plan_destroy(pcg_plan* p)
{
    if (!p)
        return;
    pcg_plan_destroy(p->fast);
    if (p->device >= 0) {
        DeviceGuard g(p->device);
        free_plan_device(p);
    }
    delete p;
}

} // extern "C"
