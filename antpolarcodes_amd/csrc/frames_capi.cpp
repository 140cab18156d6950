// frames_capi.cpp -- C ABI (include/pcg.h) of the puncturer, the encoder and the frame
// source around the decoder.  Host-side table building + launches of frames_kernel.hip.
#include "../../include/pcg.h"

#include "crc_host.hpp"
#include "frames.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <random>
#include <string>
#include <vector>

// pcg_last_error's storage lives in capi.cpp
namespace pcg {
int set_error(int code, const std::string& msg);
}

namespace {

using pcg::set_error;

int hip_error(hipError_t e, const char* what)
{
    return set_error(PCG_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DevGuard {
    int prev = 0;
    bool ok = false;
    explicit DevGuard(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && hipSetDevice(dev) == hipSuccess)
            ok = true;
    }
    ~DevGuard()
    {
        if (ok)
            (void)hipSetDevice(prev);
    }
};

} // namespace

struct pcg_encoder {
    pcg::EncodeArgs a{};
    int device = -1;
    int crc_kind = 0;
    void* d_mem = nullptr; // one allocation holding every table
};

namespace pcg {

int build_puncturer(uint32_t E, const uint32_t* frozen, uint32_t nf, uint32_t* N, std::vector<uint32_t>* pos,
                    const char** err)
{
    // round_up_power_of_two (puncturer.cpp:23-33, the 32-bit bit trick)
    uint32_t v = E - 1;
    v |= v >> 1;
    v |= v >> 2;
    v |= v >> 4;
    v |= v >> 8;
    v |= v >> 16;
    const uint32_t parent = v + 1;
    const uint32_t np = parent - E;
    if (np > nf) {
        *err = "Number of required puncturing positions exceeds frozen bit positions!";
        return -1;
    }
    // inverse_set_difference: the std::set_difference merge of iota(parent) and the
    // first np frozen entries (puncturer.cpp:35-49)
    pos->clear();
    uint32_t j = 0;
    for (uint32_t x = 0; x < parent;) {
        if (j == np || x < frozen[j]) {
            pos->push_back(x++);
        } else {
            if (!(frozen[j] < x))
                ++x;
            ++j;
        }
    }
    *N = parent;
    return 0;
}

} // namespace pcg

extern "C" {

int pcg_puncturer_create(pcg_puncturer** out, uint32_t E, const uint32_t* frozen, uint32_t n_frozen, int device)
{
    if (!out)
        return set_error(PCG_E_ARG, "puncturer output pointer is null");
    *out = nullptr;
    if (E == 0 || E > (1u << 31))
        return set_error(PCG_E_ARG, "punctured block length must be in [1, 2^31]");
    if (n_frozen && !frozen)
        return set_error(PCG_E_ARG, "null frozen list");
    auto* p = new pcg_puncturer();
    const char* err = nullptr;
    if (pcg::build_puncturer(E, frozen, n_frozen, &p->N, &p->pos, &err) != 0) {
        delete p;
        return set_error(PCG_E_ARG, err);
    }
    p->E = E;
    if ((uint32_t)p->pos.size() != E) {
        // only reachable with frozen lists that are not ascending / contain duplicates
        delete p;
        return set_error(PCG_E_ARG, "frozen positions must be ascending and unique");
    }
    if (device < 0) {
        *out = p;
        return PCG_OK;
    }
    int ndev = pcg_device_count();
    if (device >= ndev) {
        delete p;
        return set_error(ndev <= 0 ? PCG_E_NODEVICE : PCG_E_ARG, "device index out of range / no HIP device");
    }
    DevGuard g(device);
    std::vector<int32_t> src(p->N, -1);
    for (uint32_t k = 0; k < E; ++k)
        src[p->pos[k]] = (int32_t)k;
    hipError_t e;
    if ((e = hipMalloc(&p->d_pos, 4ull * E)) != hipSuccess || (e = hipMalloc(&p->d_src, 4ull * p->N)) != hipSuccess ||
        (e = hipMemcpy(p->d_pos, p->pos.data(), 4ull * E, hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(p->d_src, src.data(), 4ull * p->N, hipMemcpyHostToDevice)) != hipSuccess) {
        (void)hipFree(p->d_pos);
        (void)hipFree(p->d_src);
        delete p;
        return hip_error(e, "puncturer tables");
    }
    p->device = device;
    *out = p;
    return PCG_OK;
}

int pcg_puncturer_describe(const pcg_puncturer* p, uint32_t* E, uint32_t* N, uint32_t* positions)
{
    if (!p)
        return set_error(PCG_E_ARG, "null puncturer");
    if (E)
        *E = p->E;
    if (N)
        *N = p->N;
    if (positions)
        std::memcpy(positions, p->pos.data(), 4ull * p->E);
    return PCG_OK;
}

static int punc_ready(const pcg_puncturer* p)
{
    if (!p)
        return set_error(PCG_E_ARG, "null puncturer");
    if (p->device < 0)
        return set_error(PCG_E_NODEVICE, "host-only puncturer (created with device < 0)");
    return PCG_OK;
}

int pcg_depuncture_f32(const pcg_puncturer* p, const float* in, uint64_t F, float* out, void* stream)
{
    if (int rc = punc_ready(p))
        return rc;
    if (F == 0)
        return PCG_OK;
    if (!in || !out)
        return set_error(PCG_E_ARG, "null buffer");
    if (p->N % 4)
        return set_error(PCG_E_UNSUPPORTED, "device depuncturing needs N >= 4");
    DevGuard g(p->device);
    if (pcg::launch_depuncture(in, F, p->E, p->N, p->d_src, out, reinterpret_cast<hipStream_t>(stream)))
        return hip_error(hipGetLastError(), "depuncture launch");
    return PCG_OK;
}

int pcg_puncture_f32(const pcg_puncturer* p, const float* in, uint64_t F, float* out, void* stream)
{
    if (int rc = punc_ready(p))
        return rc;
    if (F == 0)
        return PCG_OK;
    if (!in || !out)
        return set_error(PCG_E_ARG, "null buffer");
    DevGuard g(p->device);
    if (pcg::launch_puncture(in, F, p->N, p->E, p->d_pos, out, reinterpret_cast<hipStream_t>(stream)))
        return hip_error(hipGetLastError(), "puncture launch");
    return PCG_OK;
}

int pcg_puncture_packed(const pcg_puncturer* p, const uint8_t* in, uint64_t F, uint8_t* out, void* stream)
{
    if (int rc = punc_ready(p))
        return rc;
    if (F == 0)
        return PCG_OK;
    if (!in || !out)
        return set_error(PCG_E_ARG, "null buffer");
    if (p->E % 8 || p->N % 8) // puncturer.cpp:73-74 asserts
        return set_error(PCG_E_ARG, "packed puncturing needs E and N to be multiples of 8");
    DevGuard g(p->device);
    if (pcg::launch_puncture_packed(in, F, p->N, p->E, p->d_pos, out, reinterpret_cast<hipStream_t>(stream)))
        return hip_error(hipGetLastError(), "puncture_packed launch");
    return PCG_OK;
}

void pcg_puncturer_destroy(pcg_puncturer* p)
{
    if (!p)
        return;
    if (p->device >= 0) {
        DevGuard g(p->device);
        (void)hipFree(p->d_pos);
        (void)hipFree(p->d_src);
    }
    delete p;
}

// ---------------------------------------------------------------------------- encoder
int pcg_encoder_create(pcg_encoder** out,
                       uint32_t N,
                       const uint32_t* frozen,
                       uint32_t nf,
                       int systematic,
                       int crc_kind,
                       int device)
{
    if (!out)
        return set_error(PCG_E_ARG, "encoder output pointer is null");
    *out = nullptr;
    if (N < 8 || N > 32768 || (N & (N - 1)))
        return set_error(PCG_E_ARG, "block length must be a power of two in [8, 32768]");
    if (nf > N || (nf && !frozen))
        return set_error(PCG_E_ARG, "bad frozen-bit count");
    for (uint32_t i = 0; i < nf; ++i)
        if (frozen[i] >= N || (i && frozen[i] <= frozen[i - 1]))
            return set_error(PCG_E_ARG, "frozen bits must be strictly ascending indices < N");
    if (crc_kind != 0 && crc_kind != 8 && crc_kind != 11 && crc_kind != 16 && crc_kind != 32)
        return set_error(PCG_E_ARG, "CRC INVALID SIZE!");
    const uint32_t K = N - nf, kb = (K + 7) / 8, nwords = (N + 31) / 32;
    // the detector runs over K/8 bytes (butterfly_fip_packed.cpp:47)
    const int gbytes = (int)(K / 8);
    if (crc_kind && gbytes * 8 < crc_kind)
        return set_error(PCG_E_ARG, "information length too small for the detector");

    std::vector<uint16_t> rank(N, 0xFFFF), info_pos;
    std::vector<uint32_t> infomask(nwords, 0u);
    {
        std::vector<uint8_t> isf(N, 0);
        for (uint32_t i = 0; i < nf; ++i)
            isf[frozen[i]] = 1;
        for (uint32_t i = 0; i < N; ++i)
            if (!isf[i]) {
                rank[i] = (uint16_t)info_pos.size();
                info_pos.push_back((uint16_t)i);
                infomask[i >> 5] |= 1u << (i & 31);
            }
    }
    // generate() as an affine map on the K-bit message: the trailer T = bits generate()
    // may change; delta_j = generate(e_j) ^ generate(0) restricted to T.
    std::vector<uint16_t> trail;
    std::vector<uint32_t> delta(K, 0u);
    uint32_t g0 = 0;
    if (crc_kind) {
        std::vector<uint8_t> z(kb + 8, 0), m(kb + 8, 0);
        pcg::crc_generate(crc_kind, z.data(), gbytes);
        std::vector<uint8_t> touched(K, 0);
        auto bit = [](const std::vector<uint8_t>& v, uint32_t j) { return (v[j >> 3] >> (7 - (j & 7))) & 1u; };
        std::vector<std::vector<uint8_t>> outs(K);
        for (uint32_t j = 0; j < K; ++j) {
            std::fill(m.begin(), m.end(), 0);
            m[j >> 3] = (uint8_t)(0x80u >> (j & 7));
            pcg::crc_generate(crc_kind, m.data(), gbytes);
            for (uint32_t i = 0; i < K; ++i)
                if (bit(m, i) != ((i == j) ? 1u : 0u) || bit(z, i))
                    touched[i] = 1;
            outs[j] = m;
        }
        for (uint32_t i = 0; i < K; ++i)
            if (touched[i])
                trail.push_back((uint16_t)i);
        if (trail.size() > 32)
            return set_error(PCG_E_UNSUPPORTED, "detector writes more than 32 bits");
        for (size_t t = 0; t < trail.size(); ++t) {
            g0 |= bit(z, trail[t]) << t;
            for (uint32_t j = 0; j < K; ++j)
                if (bit(outs[j], trail[t]) ^ bit(z, trail[t]))
                    delta[j] |= 1u << t;
        }
        // self-check the model on random messages
        std::mt19937 rng(777);
        for (int r = 0; r < 16; ++r) {
            for (uint32_t i = 0; i < kb; ++i)
                m[i] = (uint8_t)rng();
            if (K % 8)
                m[kb - 1] &= (uint8_t)(0xFFu << (8 - K % 8));
            uint32_t acc = g0;
            for (uint32_t j = 0; j < K; ++j)
                if (bit(m, j))
                    acc ^= delta[j];
            pcg::crc_generate(crc_kind, m.data(), gbytes);
            for (size_t t = 0; t < trail.size(); ++t)
                if (bit(m, trail[t]) != ((acc >> t) & 1u))
                    return set_error(PCG_E_UNSUPPORTED, "internal: detector generate() is not affine");
        }
    }
    auto* e = new pcg_encoder();
    e->crc_kind = crc_kind;
    auto& a = e->a;
    a.N = N;
    a.K = K;
    a.kb = kb;
    a.nwords = nwords;
    a.systematic = systematic ? 1 : 0;
    a.ntrail = (uint32_t)trail.size();
    a.g0 = g0;
    if (device < 0) {
        *out = e;
        return PCG_OK;
    }
    int ndev = pcg_device_count();
    if (device >= ndev) {
        delete e;
        return set_error(ndev <= 0 ? PCG_E_NODEVICE : PCG_E_ARG, "device index out of range / no HIP device");
    }
    DevGuard g(device);
    // one allocation: rank | info_pos | trail (u16, padded) | infomask | delta (u32)
    const size_t n16 = N + K + trail.size() + 8;
    const size_t bytes = ((2 * n16 + 15) & ~size_t(15)) + 4ull * (nwords + K + 1);
    hipError_t he = hipMalloc(&e->d_mem, bytes);
    if (he != hipSuccess) {
        delete e;
        return hip_error(he, "encoder tables");
    }
    std::vector<uint8_t> host(bytes, 0);
    uint16_t* h16 = reinterpret_cast<uint16_t*>(host.data());
    std::memcpy(h16, rank.data(), 2ull * N);
    std::memcpy(h16 + N, info_pos.data(), 2ull * K);
    if (!trail.empty())
        std::memcpy(h16 + N + K, trail.data(), 2 * trail.size());
    uint32_t* h32 = reinterpret_cast<uint32_t*>(host.data() + ((2 * n16 + 15) & ~size_t(15)));
    std::memcpy(h32, infomask.data(), 4ull * nwords);
    if (K)
        std::memcpy(h32 + nwords, delta.data(), 4ull * K);
    if ((he = hipMemcpy(e->d_mem, host.data(), bytes, hipMemcpyHostToDevice)) != hipSuccess) {
        (void)hipFree(e->d_mem);
        delete e;
        return hip_error(he, "encoder tables");
    }
    const uint16_t* d16 = reinterpret_cast<const uint16_t*>(e->d_mem);
    const uint32_t* d32 =
        reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(e->d_mem) + ((2 * n16 + 15) & ~size_t(15)));
    a.rank = d16;
    a.info_pos = d16 + N;
    a.trail = d16 + N + K;
    a.infomask = d32;
    a.delta = d32 + nwords;
    e->device = device;
    *out = e;
    return PCG_OK;
}

int pcg_encode(pcg_encoder* e, uint8_t* info, uint64_t F, uint8_t* code, void* stream)
{
    if (!e)
        return set_error(PCG_E_ARG, "null encoder");
    if (e->device < 0)
        return set_error(PCG_E_NODEVICE, "host-only encoder (created with device < 0)");
    if (F == 0)
        return PCG_OK;
    if (!info || !code)
        return set_error(PCG_E_ARG, "null buffer");
    DevGuard g(e->device);
    pcg::EncodeArgs a = e->a;
    a.F = F;
    a.info = info;
    a.code = code;
    const int rc = pcg::launch_encode(a, reinterpret_cast<hipStream_t>(stream));
    if (rc == -4)
        return set_error(PCG_E_UNSUPPORTED, "block length too large for the device encoder");
    if (rc)
        return hip_error(hipGetLastError(), "encode launch");
    return PCG_OK;
}

void pcg_encoder_destroy(pcg_encoder* e)
{
    if (!e)
        return;
    if (e->device >= 0) {
        DevGuard g(e->device);
        (void)hipFree(e->d_mem);
    }
    delete e;
}

int pcg_random_info(uint8_t* info, uint64_t F, uint32_t K, uint64_t seed, void* stream)
{
    if (F == 0 || K == 0)
        return PCG_OK;
    if (!info)
        return set_error(PCG_E_ARG, "null buffer");
    if (pcg::launch_random_info(info, F, K, seed, reinterpret_cast<hipStream_t>(stream)))
        return hip_error(hipGetLastError(), "random_info launch");
    return PCG_OK;
}

int pcg_bpsk_awgn_f32(const uint8_t* code, uint64_t F, uint32_t n, float sigma, uint64_t seed, float* llr,
                      void* stream)
{
    if (F == 0)
        return PCG_OK;
    if (!code || !llr)
        return set_error(PCG_E_ARG, "null buffer");
    if (n == 0 || n % 8)
        return set_error(PCG_E_ARG, "symbols per frame must be a positive multiple of 8");
    if (pcg::launch_bpsk_awgn(code, F, n, sigma, seed, llr, reinterpret_cast<hipStream_t>(stream)))
        return hip_error(hipGetLastError(), "bpsk_awgn launch");
    return PCG_OK;
}

} // extern "C"
