// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (oracle/_ref).
//
// A thin extern "C" shim over the *reference* library's public C++ API
// (/root/reference, compiled from its own sources by oracle/Makefile into
// oracle/_ref/libpolarref.so).  It is used
//   * in this container to pin oracle/polar_oracle.c and to generate the
//     golden fixtures under tests/golden/ (tests/golden/make_golden.py), and
//   * on the GPU box as bench.py's `cpu_baseline` leg (kind "reference"):
//     the reference AVX2 decoder timed on the host cores.
// Nothing in the product (antpolarcodes_amd/) links or loads this file.
//
// Reference entry points used (paths relative to /root/reference):
//   Decoding::create                 src/polarcode/decoding/decoder.cpp:26-52
//   Decoder::decode_vector           src/polarcode/decoding/decoder.cpp:154-167
//   Decoder::getSoftCodeword         src/polarcode/decoding/decoder.cpp:147
//   ErrorDetection::create           src/polarcode/errordetection/errordetector.cpp:23-67
//   Construction::frozen_bits        src/polarcode/construction/constructor.cpp:41-63
//   Encoding::ButterflyFipPacked     src/polarcode/encoding/butterfly_fip_packed.cpp:45-70
//   SclAvx::PathList / createDecoder src/polarcode/decoding/scl_avx_float.cpp:21-171,624-651
//   Puncturer                        src/polarcode/puncturer.cpp:51-89, puncturer.h:60-99
//   Decoding::create(..., "char")    FastSscFipChar / SclFipChar (decoder.cpp:37-38, 62-80)
//   Decoder::decode_vector(char*)    src/polarcode/decoding/decoder.cpp:169-181
//   SclFip::PathList / createDecoder src/polarcode/decoding/scl_fip_char.cpp:21-171, 729-752
//   CharContainer::insertLlr         src/polarcode/bitcontainer.cpp:505-516

#include <polarcode/construction/constructor.h>
#include <polarcode/decoding/decoder.h>
#include <polarcode/decoding/scl_avx_float.h>
#include <polarcode/decoding/scl_fip_char.h>
#include <polarcode/bitcontainer.h>
#include <polarcode/encoding/butterfly_fip_packed.h>
#include <polarcode/errordetection/errordetector.h>
#include <polarcode/puncturer.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

using namespace PolarCode;

namespace {

std::string g_err;

std::vector<unsigned> to_vec(const uint32_t* f, uint32_t nf)
{
    return std::vector<unsigned>(f, f + nf);
}

// crc < 0: keep the CRC-8 that makeDecoder installs (decoder.cpp:85)
Decoding::Decoder* make_dec(uint32_t N,
                            uint32_t L,
                            const std::vector<unsigned>& fr,
                            int systematic,
                            int crc,
                            const char* type = "float")
{
    Decoding::Decoder* d = Decoding::create(N, L, fr, type);
    d->setSystematic(systematic != 0);
    if (crc >= 0)
        d->setErrorDetection(ErrorDetection::create((unsigned)crc, "crc"));
    return d;
}

} // namespace

extern "C" {

const char* ref_last_error() { return g_err.c_str(); }

// Puncturer(E, frozen): parent length into *N, the kept positions into pos (E entries);
// returns E or -1 (std::out_of_range text in ref_last_error).
int ref_puncturer(uint32_t E, const uint32_t* frozen, uint32_t nf, uint32_t* N, uint32_t* pos)
{
    try {
        Puncturer p(E, to_vec(frozen, nf));
        *N = (uint32_t)p.parentBlockLength();
        auto v = p.blockOutputPositions();
        for (size_t i = 0; i < v.size(); ++i)
            pos[i] = v[i];
        return (int)v.size();
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Puncturer::depuncture<float> / puncture<float> / puncturePacked on one frame.
int ref_punc_apply(uint32_t E, const uint32_t* frozen, uint32_t nf, int op, const void* in, void* out)
{
    try {
        Puncturer p(E, to_vec(frozen, nf));
        if (op == 0)
            p.depuncture<float>(static_cast<float*>(out), static_cast<const float*>(in));
        else if (op == 1)
            p.puncture<float>(static_cast<float*>(out), static_cast<const float*>(in));
        else
            p.puncturePacked(static_cast<unsigned char*>(out), static_cast<const unsigned char*>(in));
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

int ref_frozen_bits(uint32_t N, uint32_t K, float dsnr, const char* type, uint32_t* out)
{
    try {
        auto v = Construction::frozen_bits((int)N, (int)K, dsnr, std::string(type));
        for (size_t i = 0; i < v.size(); ++i)
            out[i] = v[i];
        return (int)v.size();
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Decode F frames through the reference "float" decoder (Fast-SSC for L=1, SCL for
// L>=2).  info: F x ceil(K/8) bytes, ok: F bytes (may be null),
// softcw: F x N floats of the SC soft codeword (may be null, L=1 only).
int ref_decode(uint32_t N,
               uint32_t L,
               const uint32_t* frozen,
               uint32_t nf,
               int systematic,
               int crc,
               const float* llr,
               uint64_t F,
               uint8_t* info,
               uint8_t* ok,
               float* softcw)
{
    try {
        auto fr = to_vec(frozen, nf);
        Decoding::Decoder* d = make_dec(N, L, fr, systematic, crc);
        const size_t kb = (N - nf + 7) / 8;
        for (uint64_t f = 0; f < F; ++f) {
            bool r = d->decode_vector(llr + f * N, info + f * kb);
            if (ok)
                ok[f] = r ? 1 : 0;
            if (softcw && L == 1)
                d->getSoftCodeword(softcw + f * N);
        }
        delete d;
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Drive the SCL internals (the public SclAvx namespace) to expose the final
// ordered path list: metrics[F][L], path count[F], and per-path hard codeword
// bits (sign bits of the stage-log2N Bit buffer) packed MSB-first [F][L][N/8].
int ref_scl_paths(uint32_t N,
                  uint32_t L,
                  const uint32_t* frozen,
                  uint32_t nf,
                  const float* llr,
                  uint64_t F,
                  float* metrics,
                  uint32_t* pathcount,
                  uint8_t* pathbits)
{
    try {
        auto fr = to_vec(frozen, nf);
        const unsigned stages = __builtin_ctz(N) + 1;
        Decoding::SclAvx::datapool_t pool;
        Decoding::SclAvx::PathList pl(L, stages, &pool);
        Decoding::SclAvx::Node base(N, L, &pool, &pl);
        Decoding::SclAvx::Node* root = Decoding::SclAvx::createDecoder(fr, &base);
        std::vector<float> buf(N < 8 ? 8 : N);
        for (uint64_t f = 0; f < F; ++f) {
            memcpy(buf.data(), llr + f * N, 4 * N);
            pl.clear();
            pl.setFirstPath(buf.data());
            root->decode();
            unsigned pc = pl.PathCount();
            pathcount[f] = pc;
            for (unsigned p = 0; p < L; ++p) {
                metrics[f * L + p] = p < pc ? pl.Metric(p) : 0.0f;
                uint8_t* pb = pathbits + (f * L + p) * (N / 8);
                memset(pb, 0, N / 8);
                if (p < pc) {
                    const uint32_t* b =
                        reinterpret_cast<const uint32_t*>(pl.Bit(p, stages - 1));
                    for (unsigned i = 0; i < N; ++i)
                        if (b[i] & 0x80000000u)
                            pb[i / 8] |= (uint8_t)(0x80u >> (i % 8));
                }
            }
            pl.clear();
        }
        delete root;
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Encode F frames of packed info bytes (ceil(K/8) each) into packed codewords (N/8).
// crc: detector generated over the info bytes before encoding (0 = none).
int ref_encode(uint32_t N,
               const uint32_t* frozen,
               uint32_t nf,
               int systematic,
               int crc,
               const uint8_t* info,
               uint64_t F,
               uint8_t* code)
{
    try {
        auto fr = to_vec(frozen, nf);
        Encoding::ButterflyFipPacked enc(N, fr);
        enc.setSystematic(systematic != 0);
        ErrorDetection::Detector* det = ErrorDetection::create((unsigned)crc, "crc");
        enc.setErrorDetection(det);
        const size_t kb = (N - nf + 7) / 8;
        std::vector<uint8_t> tmp(kb + 32);
        for (uint64_t f = 0; f < F; ++f) {
            memcpy(tmp.data(), info + f * kb, kb);
            enc.encode_vector(tmp.data(), code + f * (N / 8));
        }
        delete det;
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Detector check/generate over `bytes` bytes (in place for generate).
int ref_crc(int crc, int generate, uint8_t* data, int bytes)
{
    try {
        ErrorDetection::Detector* det = ErrorDetection::create((unsigned)crc, "crc");
        int r = 0;
        if (generate)
            det->generate(data, bytes);
        else
            r = det->check(data, bytes) ? 1 : 0;
        delete det;
        return r;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Throughput of the reference decoder: `threads` workers, one decoder each,
// each decoding frames [t*F/threads, (t+1)*F/threads) `reps` times.
// Returns codewords/s (decoder time only, as pcbench/pcsim time it).
double ref_bench(uint32_t N,
                 uint32_t L,
                 const uint32_t* frozen,
                 uint32_t nf,
                 int systematic,
                 int crc,
                 const float* llr,
                 uint64_t F,
                 int threads,
                 int reps)
{
    try {
        auto fr = to_vec(frozen, nf);
        if (threads < 1)
            threads = 1;
        std::vector<Decoding::Decoder*> decs;
        for (int t = 0; t < threads; ++t)
            decs.push_back(make_dec(N, L, fr, systematic, crc));
        const size_t kb = (N - nf + 7) / 8;
        std::atomic<int> ready{ 0 };
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) {
            pool.emplace_back([&, t]() {
                std::vector<uint8_t> out(kb + 32);
                uint64_t lo = F * t / threads, hi = F * (t + 1) / threads;
                for (int r = 0; r < reps; ++r)
                    for (uint64_t f = lo; f < hi; ++f)
                        decs[t]->decode_vector(llr + f * N, out.data());
                ready++;
            });
        }
        for (auto& th : pool)
            th.join();
        double s =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (auto* d : decs)
            delete d;
        return (double)F * reps / s;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1.0;
    }
}

// ---- 8-bit ("char") decoders: FastSscFipChar (L = 1) / SclFipChar (L >= 2) -------------

// CharContainer::insertLlr(const float*) on F frames of N floats.
int ref_f32_to_i8(uint32_t N, const float* in, uint64_t F, int8_t* out)
{
    try {
        CharContainer c(N);
        for (uint64_t f = 0; f < F; ++f) {
            c.insertLlr(in + f * N);
            memcpy(out + f * N, c.data(), N);
        }
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Decode F frames through create(N, L, frozen, "char").  llr_i8 != 0: llr is F x N int8
// (decode_vector(const char*)), else F x N float (decode_vector(const float*)).
// softcw: F x N int8 of getSoftCodeword (L = 1 only, nullable).
int ref_decode_char(uint32_t N,
                    uint32_t L,
                    const uint32_t* frozen,
                    uint32_t nf,
                    int systematic,
                    int crc,
                    int llr_i8,
                    const void* llr,
                    uint64_t F,
                    uint8_t* info,
                    uint8_t* ok,
                    int8_t* softcw)
{
    try {
        auto fr = to_vec(frozen, nf);
        Decoding::Decoder* d = make_dec(N, L, fr, systematic, crc, "char");
        const size_t kb = (N - nf + 7) / 8;
        for (uint64_t f = 0; f < F; ++f) {
            bool r = llr_i8 ? d->decode_vector(static_cast<const char*>(llr) + f * N, info + f * kb)
                            : d->decode_vector(static_cast<const float*>(llr) + f * N, info + f * kb);
            if (ok)
                ok[f] = r ? 1 : 0;
            if (softcw && L == 1)
                d->getSoftCodeword(softcw + f * N);
        }
        delete d;
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// SclFip internals on int8 frames, a fresh path list per frame: ordered metrics
// [F][L] (int64), path count [F], per-path hard codeword bits [F][L][N/8] MSB-first.
int ref_sclc_paths(uint32_t N,
                   uint32_t L,
                   const uint32_t* frozen,
                   uint32_t nf,
                   const int8_t* llr,
                   uint64_t F,
                   int64_t* metrics,
                   uint32_t* pathcount,
                   uint8_t* pathbits)
{
    try {
        auto fr = to_vec(frozen, nf);
        const unsigned stages = __builtin_ctz(N) + 1;
        std::vector<char> buf(N < 32 ? 32 : N);
        for (uint64_t f = 0; f < F; ++f) {
            Decoding::SclFip::datapool_t pool;
            Decoding::SclFip::PathList pl(L, stages, &pool);
            Decoding::SclFip::Node base(N, L, &pool, &pl);
            Decoding::SclFip::Node* root = Decoding::SclFip::createDecoder(fr, &base);
            memcpy(buf.data(), llr + f * N, N);
            pl.clear();
            pl.setFirstPath(buf.data());
            root->decode();
            unsigned pc = pl.PathCount();
            pathcount[f] = pc;
            for (unsigned p = 0; p < L; ++p) {
                metrics[f * L + p] = p < pc ? (int64_t)pl.Metric(p) : 0;
                uint8_t* pb = pathbits + (f * L + p) * (N / 8);
                memset(pb, 0, N / 8);
                if (p < pc) {
                    const uint8_t* b = reinterpret_cast<const uint8_t*>(pl.Bit(p, stages - 1));
                    for (unsigned i = 0; i < N; ++i)
                        if (b[i] & 0x80u)
                            pb[i / 8] |= (uint8_t)(0x80u >> (i % 8));
                }
            }
            pl.clear();
            delete root;
        }
        return 0;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

// Throughput of the reference char decoder on int8 frames (as ref_bench).
double ref_bench_char(uint32_t N,
                      uint32_t L,
                      const uint32_t* frozen,
                      uint32_t nf,
                      int systematic,
                      int crc,
                      const int8_t* llr,
                      uint64_t F,
                      int threads,
                      int reps)
{
    try {
        auto fr = to_vec(frozen, nf);
        if (threads < 1)
            threads = 1;
        std::vector<Decoding::Decoder*> decs;
        for (int t = 0; t < threads; ++t)
            decs.push_back(make_dec(N, L, fr, systematic, crc, "char"));
        const size_t kb = (N - nf + 7) / 8;
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) {
            pool.emplace_back([&, t]() {
                std::vector<uint8_t> out(kb + 32);
                uint64_t lo = F * t / threads, hi = F * (t + 1) / threads;
                for (int r = 0; r < reps; ++r)
                    for (uint64_t f = lo; f < hi; ++f)
                        decs[t]->decode_vector(reinterpret_cast<const char*>(llr) + f * N, out.data());
            });
        }
        for (auto& th : pool)
            th.join();
        double s =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (auto* d : decs)
            delete d;
        return (double)F * reps / s;
    } catch (std::exception& e) {
        g_err = e.what();
        return -1.0;
    }
}

} // extern "C"
