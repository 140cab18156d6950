// plan.cpp -- build the flattened decoder schedule (see plan.hpp).
#include "plan.hpp"

#include "crc_host.hpp"

#include <cstdlib>
#include <random>

namespace pcg {

namespace {

struct Err {
    int code;
    std::string msg;
};

void split(const std::vector<uint32_t>& f,
           uint32_t half,
           std::vector<uint32_t>& l,
           std::vector<uint32_t>& r)
{
    l.clear();
    r.clear();
    for (uint32_t v : f) {
        if (v < half)
            l.push_back(v);
        else
            r.push_back(v - half);
    }
}

uint32_t ilog2(uint32_t n) { return (uint32_t)__builtin_ctz(n); }

uint32_t mkop(uint32_t code, uint32_t n, uint32_t off)
{
    return code | (ilog2(n) << 8) | (off << 16);
}

std::string fmt_frozen(const std::vector<uint32_t>& f)
{
    std::string s = "[";
    for (size_t i = 0; i < f.size(); ++i) {
        if (i)
            s += ", ";
        s += std::to_string(f[i]);
    }
    return s + "]";
}

// FastSscAvx::createDecoder (fastssc_avx_float.cpp:797-896), emitted in decode order:
//   RateR : F, <left>, G, <right>, COMB        (RateRNode::decode :148-155; ShortRateRNode
//           :178-185 has the same observable semantics on packed sign bits)
//   ROne  : F, <left>, RONE                    (:198-219)
//   ZeroR : G0, <right>, COPY0                 (:232-237)
void sc_emit(PlanHost& p, const std::vector<uint32_t>& f, uint32_t n, uint32_t off)
{
    const uint32_t nf = (uint32_t)f.size();
    p.node_count++;
    auto leaf = [&](uint32_t code) {
        p.node_types.push_back((int)code);
        p.ops.push_back(mkop(code, n, off));
    };
    if (nf == n) return leaf(OP_L_R0);
    if (nf == 0) return leaf(OP_L_R1);
    if (nf == n - 1) return leaf(OP_L_REP);
    if (nf == 1) return leaf(OP_L_SPC);
    if (nf == n - 2) {
        for (uint32_t i = 0; i < nf; ++i)
            if (f[i] != i)
                throw Err{ -2, fmt_frozen(f) };
        if (n < 4)
            throw Err{ -2, "Minimum block length for double Repetition code is 4!" };
        return leaf(OP_L_DREP);
    }
    if (nf == 2 && f[0] == 0 && f[1] == 1)
        return leaf(n == 8 ? OP_L_DSPC8 : OP_L_DSPC);
    if (nf == n - 3 && n > 8 && f[nf - 1] == n - 4) {
        for (uint32_t i = 0; i < nf; ++i)
            if (f[i] != i)
                throw Err{ -2, fmt_frozen(f) };
        return leaf(OP_L_TREP);
    }
    if (nf == n - 4 && f[nf - 1] == n - 4 && f[nf - 2] == n - 6)
        return leaf(OP_L_TYPE5);
    if (n == 8 && nf == 3 && f[0] == 0 && f[1] == 1 && f[2] == 2)
        return leaf(OP_L_REPR1);
    if (n == 8 && nf == 5 && f[nf - 1] == n - 4 && f[nf - 2] == n - 5)
        return leaf(OP_L_ZSPC8);

    const uint32_t h = n / 2;
    std::vector<uint32_t> lf, rf;
    split(f, h, lf, rf);
    p.node_types.push_back(0);
    if (n <= 8) { // ShortRateRNode
        p.ops.push_back(mkop(OP_F, n, off));
        sc_emit(p, lf, h, off);
        p.ops.push_back(mkop(OP_G, n, off));
        sc_emit(p, rf, h, off + h);
        p.ops.push_back(mkop(OP_COMB, n, off));
        return;
    }
    if (lf.size() == h && rf.size() == 1) { // ZeroSpcDecoder (a leaf kind)
        p.node_types.back() = OP_L_ZSPC;
        p.ops.push_back(mkop(OP_L_ZSPC, n, off));
        return;
    }
    if (rf.empty()) { // ROneNode: the right child is an unused dummy Node
        p.ops.push_back(mkop(OP_F, n, off));
        sc_emit(p, lf, h, off);
        p.ops.push_back(mkop(OP_RONE, n, off));
        return;
    }
    if (lf.size() == h) { // ZeroRNode: the left child is an unused dummy Node
        p.ops.push_back(mkop(OP_G0, n, off));
        sc_emit(p, rf, h, off + h);
        p.ops.push_back(mkop(OP_COPY0, n, off));
        return;
    }
    p.ops.push_back(mkop(OP_F, n, off));
    sc_emit(p, lf, h, off);
    p.ops.push_back(mkop(OP_G, n, off));
    sc_emit(p, rf, h, off + h);
    p.ops.push_back(mkop(OP_COMB, n, off));
}

// scq_kernel.hip's schedule: [F 4 o][leaf 3 o][G 4 o][leaf 3 o+8][COMB 4 o] -> [Q16 4 o][desc],
// [F 4 o][leaf 3 o][RONE 4 o] -> [Q16R 4 o][desc] (size-8 leaves of the Fast-SSC tree).
void fuse_sc16(PlanHost& p)
{
    const auto& v = p.ops;
    auto is8 = [&](size_t k, uint32_t o) {
        return k < v.size() && op_code(v[k]) >= OP_L_R0 && op_code(v[k]) <= OP_L_ZSPC && op_stage(v[k]) == 3 &&
               op_off(v[k]) == o;
    };
    auto is = [&](size_t k, uint32_t code, uint32_t o) {
        return k < v.size() && op_code(v[k]) == code && op_stage(v[k]) == 4 && op_off(v[k]) == o;
    };
    std::vector<uint32_t> out;
    for (size_t k = 0; k < v.size();) {
        const uint32_t o = op_off(v[k]);
        if (is(k, OP_F, o) && is8(k + 1, o) && is(k + 2, OP_G, o) && is8(k + 3, o + 8) && is(k + 4, OP_COMB, o)) {
            out.push_back(mkop(OP_Q16, 16, o));
            out.push_back(op_code(v[k + 1]) | (op_code(v[k + 3]) << 8));
            k += 5;
        } else if (is(k, OP_F, o) && is8(k + 1, o) && is(k + 2, OP_RONE, o)) {
            out.push_back(mkop(OP_Q16R, 16, o));
            out.push_back(op_code(v[k + 1]));
            k += 3;
        } else {
            out.push_back(v[k]);
            ++k;
        }
    }
    // The size-32 parent's F / G folded into a fused size-16 child (the child's 16 LLRs are
    // then computed in registers from the parent's 32): [F 5 o][Q16* 4 o][d] -> [Q16F 4 o][d'],
    // [G 5 o][Q16* 4 o+16][d] -> [Q16G 4 o+16][d'], d' = d | (child is Q16R) << 16.
    {
        std::vector<uint32_t> o2;
        for (size_t k = 0; k < out.size(); ++k) {
            const uint32_t w = out[k], c = op_code(w);
            if ((c == OP_F || c == OP_G) && op_stage(w) == 5 && k + 2 < out.size()) {
                const uint32_t nx = out[k + 1], nc = op_code(nx);
                const uint32_t oc = op_off(w) + (c == OP_G ? 16u : 0u);
                if ((nc == OP_Q16 || nc == OP_Q16R) && op_off(nx) == oc) {
                    o2.push_back(mkop(c == OP_F ? OP_Q16F : OP_Q16G, 16, oc));
                    o2.push_back(out[k + 2] | (nc == OP_Q16R ? 1u << 16 : 0u));
                    k += 2;
                    continue;
                }
                // a size-16 leaf child: descriptor = leaf code | 1 << 17
                if (nc >= OP_L_R0 && nc <= OP_L_ZSPC && nc != OP_L_DSPC8 && nc != OP_L_ZSPC8 && nc != OP_L_REPR1 &&
                    op_stage(nx) == 4 && op_off(nx) == oc) {
                    o2.push_back(mkop(c == OP_F ? OP_Q16F : OP_Q16G, 16, oc));
                    o2.push_back(nc | (1u << 17));
                    k += 1;
                    continue;
                }
            }
            o2.push_back(w);
            if (op_has_desc(c))
                o2.push_back(out[++k]);
        }
        out.swap(o2);
    }
    // Second pass: a parent's COMB right after the last op of its right child's subtree is
    // folded into that op as a count of combine levels in the stage byte (stage | levels << 4):
    // after the op, the kernel applies COMB at stages s+1 .. s+levels going up the right
    // spine.  `end` tracks the subtree each emitted op completes.
    p.ops_fused.clear();
    size_t last = SIZE_MAX;           // index of the last op word (not a descriptor)
    uint32_t end_s = 0, end_o = 0;    // the subtree it completes
    for (size_t k = 0; k < out.size(); ++k) {
        const uint32_t w = out[k], c = op_code(w), s = op_stage(w), o = op_off(w);
        if (c == OP_COMB && last != SIZE_MAX && end_s + 1 == s && end_o == o + (1u << (s - 1)) &&
            (op_stage(p.ops_fused[last]) >> 4) < 15) {
            p.ops_fused[last] += 1u << 12; // one more level (bits 12..15 of the word)
            end_s = s;
            end_o = o;
            continue;
        }
        last = p.ops_fused.size();
        p.ops_fused.push_back(w);
        end_s = s;
        end_o = o;
        if (op_has_desc(c))
            p.ops_fused.push_back(out[++k]); // descriptor
    }
}

// SCL classification of a small node (n <= 4) as an ST8 descriptor kind.
uint32_t scl_small_kind(const std::vector<uint32_t>& f, uint32_t n, PlanHost& p, uint32_t* sub)
{
    const uint32_t nf = (uint32_t)f.size();
    p.node_count++;
    if (nf == 0) return ST_R1;
    if (nf == n) return ST_R0;
    if (nf == n - 1 && n < 8) return ST_REP;
    if (nf == 1) return ST_SPC;
    // ShortRateRNode (n == 4): two size-2 children (R0 / R1 / Rep only)
    std::vector<uint32_t> lf, rf;
    split(f, n / 2, lf, rf);
    uint32_t d0 = 0, d1 = 0;
    const uint32_t k0 = scl_small_kind(lf, n / 2, p, &d0), k1 = scl_small_kind(rf, n / 2, p, &d1);
    *sub = k0 | (k1 << 2);
    return ST_RATER;
}

// SclAvx::createDecoder (scl_avx_float.cpp:624-651), RateRNode::decode order (:229-263).
void scl_emit(PlanHost& p, const std::vector<uint32_t>& f, uint32_t n, uint32_t off)
{
    const uint32_t nf = (uint32_t)f.size();
    p.node_count++;
    auto leaf = [&](uint32_t code) {
        p.node_types.push_back((int)code);
        p.ops.push_back(mkop(code, n, off));
    };
    if (nf == 0) return leaf(OP_S_R1);
    if (nf == n) return leaf(OP_S_R0);
    if (nf == n - 1 && n < 8) return leaf(OP_S_REP);
    if (nf == 1) return leaf(OP_S_SPC);
    const uint32_t h = n / 2;
    std::vector<uint32_t> lf, rf;
    split(f, h, lf, rf);
    p.node_types.push_back(0);
    if (n == 8 && p.scl_st8) { // ShortRateRNode of size 8: one lane-serial subtree op
        uint32_t desc = 0;
        for (uint32_t c = 0; c < 2; ++c) {
            uint32_t sub = 0;
            const uint32_t kind = scl_small_kind(c ? rf : lf, 4, p, &sub);
            desc |= (kind | (sub << 3)) << (8 * c);
        }
        p.ops.push_back(mkop(OP_S_ST8, n, off));
        p.ops.push_back(desc);
        return;
    }
    p.ops.push_back(mkop(OP_F, n, off));
    scl_emit(p, lf, h, off);
    p.ops.push_back(mkop(OP_G, n, off));
    scl_emit(p, rf, h, off + h);
    p.ops.push_back(mkop(OP_COMB, n, off));
}

// FastSscFip::createDecoder (fastssc_fip_char.cpp:496-580).  Short (n <= 32) and long
// variants of RateR / ROne / ZeroR have the same effect on sign bits; the leaves differ.
void sc_char_emit(PlanHost& p, const std::vector<uint32_t>& f, uint32_t n, uint32_t off)
{
    constexpr uint32_t BV = 32; // BYTESPERVECTOR of the AVX2 build
    const uint32_t nf = (uint32_t)f.size();
    p.node_count++;
    auto leaf = [&](uint32_t code) {
        p.node_types.push_back((int)code);
        p.ops.push_back(mkop(code, n, off));
    };
    if (nf == n) return leaf(OP_C_R0);
    if (nf == 0) return leaf(OP_C_R1);
    if (nf == n - 1) return leaf(n <= BV ? OP_C_REPS : OP_C_REP);
    if (nf == 1) return leaf(n <= BV ? OP_C_SPCS : OP_C_SPC);
    if (nf == n - 2 && n >= BV) return leaf(OP_C_DREP);
    const uint32_t h = n / 2;
    std::vector<uint32_t> lf, rf;
    split(f, h, lf, rf);
    if (n <= BV) {
        if (lf.size() == h && rf.empty()) return leaf(OP_C_ZONES);
        if (lf.size() == h && rf.size() == 1) return leaf(OP_C_ZSPCS);
    } else if (lf.size() == h && rf.size() == 1) {
        return leaf(OP_C_ZSPC);
    }
    p.node_types.push_back(0);
    // (Short)ROneNode / (Short)ZeroRNode construct both children (RateRNode's constructor,
    // fastssc_fip_char.cpp:81-94) but decode only one: count the other, emit nothing
    auto count_only = [&](const std::vector<uint32_t>& cf) {
        PlanHost tmp;
        sc_char_emit(tmp, cf, h, 0);
        p.node_count += tmp.node_count;
    };
    if (rf.empty()) { // (Short)ROneNode
        p.ops.push_back(mkop(OP_F, n, off));
        sc_char_emit(p, lf, h, off);
        count_only(rf);
        p.ops.push_back(mkop(OP_RONE, n, off));
        return;
    }
    if (lf.size() == h) { // (Short)ZeroRNode
        count_only(lf);
        p.ops.push_back(mkop(OP_G0, n, off));
        sc_char_emit(p, rf, h, off + h);
        p.ops.push_back(mkop(OP_COPY0, n, off));
        return;
    }
    p.ops.push_back(mkop(OP_F, n, off)); // (Short)RateRNode
    sc_char_emit(p, lf, h, off);
    p.ops.push_back(mkop(OP_G, n, off));
    sc_char_emit(p, rf, h, off + h);
    p.ops.push_back(mkop(OP_COMB, n, off));
}

// SclFip::createDecoder (scl_fip_char.cpp:729-752); RateRNode::decode order (:315-349).
void scl_char_emit(PlanHost& p, const std::vector<uint32_t>& f, uint32_t n, uint32_t off)
{
    const uint32_t nf = (uint32_t)f.size();
    p.node_count++;
    auto leaf = [&](uint32_t code) {
        p.node_types.push_back((int)code);
        p.ops.push_back(mkop(code, n, off));
    };
    if (nf == n) return leaf(OP_CS_R0);
    if (nf == 0) return leaf(OP_CS_R1);
    if (nf == n - 1) return leaf(OP_CS_REP);
    if (nf == 1) return leaf(OP_CS_SPC);
    const uint32_t h = n / 2;
    std::vector<uint32_t> lf, rf;
    split(f, h, lf, rf);
    p.node_types.push_back(0);
    p.ops.push_back(mkop(OP_F, n, off));
    scl_char_emit(p, lf, h, off);
    p.ops.push_back(mkop(OP_G, n, off));
    scl_char_emit(p, rf, h, off + h);
    p.ops.push_back(mkop(OP_COMB, n, off));
}

} // namespace

int build_plan(PlanHost& p,
               uint32_t N,
               uint32_t L,
               const uint32_t* frozen,
               uint32_t nf,
               int systematic,
               int crc_kind,
               std::string* err,
               int fixed)
{
    p = PlanHost();
    // Fast-SSC float plans run codes down to N = 2 (the reference's own Repetition /
    // SPC KATs start there, decodingtest.cpp:185-195); the lane-serial list and 8-bit
    // kernels need N >= 8
    const uint32_t nmin = (L == 1 && !fixed) ? 2u : 8u;
    if (N < nmin || N > 32768 || (N & (N - 1))) {
        *err = nmin == 2 ? "block length must be a power of two in [2, 32768]"
                         : "block length must be a power of two in [8, 32768]";
        return -1;
    }
    if (L < 1 || L > 32) {
        *err = "list size must be in [1, 32]";
        return -1;
    }
    if (nf > N || (nf > 0 && frozen == nullptr)) {
        *err = "bad frozen-bit count";
        return -1;
    }
    for (uint32_t i = 0; i < nf; ++i) {
        if (frozen[i] >= N || (i > 0 && frozen[i] <= frozen[i - 1])) {
            *err = "frozen bits must be strictly ascending indices < N";
            return -1;
        }
    }
    if (crc_kind != 0 && crc_kind != 8 && crc_kind != 11 && crc_kind != 16 && crc_kind != 32) {
        *err = "CRC INVALID SIZE!"; // errordetector.cpp:33-35
        return -1;
    }
    p.N = N;
    p.L = L;
    p.log2N = ilog2(N);
    p.K = N - nf;
    p.systematic = systematic ? 1 : 0;
    p.crc_kind = crc_kind;
    p.frozen.assign(frozen, frozen + nf);
    p.fixed = fixed ? 1 : 0;
    {
        const char* k = getenv("PCG_SC_KERNEL"); // dev switch: "wave" = sc_kernel.hip
        // "wave" = sc_kernel.hip, "scs" = lane-serial scs_kernel.hip, default: the float
        // decoder's LDS-resident scq_kernel.hip where it fits (capi.cpp), else scs
        p.sc_kind = (k && std::string(k) == "wave") ? 1 : ((k && std::string(k) == "scs") ? 0 : 2);
    }
    try {
        if (p.fixed && L == 1)
            sc_char_emit(p, p.frozen, N, 0);
        else if (p.fixed)
            scl_char_emit(p, p.frozen, N, 0);
        else if (L == 1)
        {
            sc_emit(p, p.frozen, N, 0);
            fuse_sc16(p);
        }
        else
            scl_emit(p, p.frozen, N, 0);
    } catch (Err& e) {
        *err = e.msg;
        return e.code;
    }

    // information-bit LUT (BitContainer::calculateLUT, bitcontainer.cpp:68-84)
    std::vector<uint8_t> isf(N, 0);
    for (uint32_t v : p.frozen)
        isf[v] = 1;
    for (uint32_t i = 0; i < N; ++i)
        if (!isf[i])
            p.info_pos.push_back((uint16_t)i);

    // Affine GF(2) syndrome of the detector over the K info bits, packed MSB-first
    // into ceil(K/8) bytes exactly as getPackedInformationBits lays them out:
    //   syndrome(b) = c0 ^ XOR_{j: b_j = 1} m_j ;  check() passes <=> syndrome == 0.
    const uint32_t K = p.K, kb = (K + 7) / 8;
    std::vector<uint8_t> msg(kb + 4, 0);
    uint32_t s0 = 0;
    crc_syndrome(crc_kind, msg.data(), (int)kb, &s0);
    p.crc_c0 = s0;
    p.crc_m.assign(K, 0);
    for (uint32_t j = 0; j < K; ++j) {
        std::fill(msg.begin(), msg.end(), 0);
        msg[j / 8] = (uint8_t)(0x80u >> (j % 8));
        uint32_t s = 0;
        crc_syndrome(crc_kind, msg.data(), (int)kb, &s);
        p.crc_m[j] = s ^ s0;
    }
    // the same model in codeword coordinates: row r marks the info positions whose
    // column has syndrome bit r set
    {
        const uint32_t W = N >= 32 ? N / 32 : 1;
        const uint32_t cb = (uint32_t)crc_kind;
        const uint32_t hi = cb >= 32 ? 0u : ~((1u << cb) - 1u);
        bool narrow = (p.crc_c0 & hi) == 0;
        for (uint32_t j = 0; j < K; ++j)
            narrow = narrow && (p.crc_m[j] & hi) == 0;
        if (!narrow) {
            *err = "internal: detector syndrome wider than its check bits";
            return -4;
        }
        p.crc_rows.assign((size_t)cb * W, 0u);
        for (uint32_t j = 0; j < K; ++j)
            for (uint32_t r = 0; r < cb; ++r)
                if ((p.crc_m[j] >> r) & 1u)
                    p.crc_rows[r * W + (p.info_pos[j] >> 5)] |= 1u << (p.info_pos[j] & 31u);
    }
    // self-check of the affine model on random messages
    std::mt19937 rng(12345);
    for (int t = 0; t < 8 && K > 0; ++t) {
        uint32_t acc = s0;
        std::fill(msg.begin(), msg.end(), 0);
        for (uint32_t j = 0; j < K; ++j)
            if (rng() & 1) {
                msg[j / 8] |= (uint8_t)(0x80u >> (j % 8));
                acc ^= p.crc_m[j];
            }
        uint32_t s = 0;
        crc_syndrome(crc_kind, msg.data(), (int)kb, &s);
        if (s != acc) {
            *err = "internal: detector is not affine over GF(2)";
            return -4;
        }
    }
    return 0;
}

} // namespace pcg
