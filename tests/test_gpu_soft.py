"""Soft codewords on the GPU (Decoder::getSoftCodeword / getSoftInformation) and the SCL
metric carry of a reused decoder instance.

The soft-codeword KATs restate the reference's own tests through the GPU path
(test/polarcode/decodingtest.cpp:159-411: Repetition, DoubleRepetition, SPC, DoubleSPC,
TypeFive and RepRateOne8 codes as a single root node, non-systematic, soft output checked
to 1e-7).  Where the reference computes its expectation with its own helper
(decode_double_spc / decode_type_five_generic / decode_repone_generic_8) the oracle's
restatement stands in for it, and the inputs are numpy normal(10, 20) draws instead of the
test's std::mt19937_64 stream (its generator is not reproducible outside libstdc++).
Beyond the KATs, whole codes are compared word for word with the oracle's soft codeword
(itself pinned to the reference's getSoftCodeword, tests/test_oracle.py)."""
import numpy as np
import pytest

from helpers import LLR_KINDS, llr_kinds, node_cover_sets

pytestmark = pytest.mark.gpu


def _dec(N, frozen):
    from antpolarcodes_amd import pypolar
    d = pypolar.PolarDecoder(N, 1, list(frozen), "gpu")
    d.setSystematic(False)
    return d


def _soft(N, frozen, signal):
    d = _dec(N, frozen)
    d.decode_vector(np.asarray(signal, np.float32))
    return d.getSoftCodeword()


@pytest.mark.parametrize("N", [2, 4, 8, 16, 32, 64, 128])
def test_kat_repetition(N):  # decodingtest.cpp:159-195
    sig = np.arange(N, dtype=np.float32)
    out = _soft(N, range(N - 1), sig)
    np.testing.assert_allclose(out, np.full(N, sig.sum(dtype=np.float32)), atol=1e-7)


@pytest.mark.parametrize("N", [4, 8, 16, 32, 64, 128, 256])
def test_kat_double_repetition(N):  # decodingtest.cpp:198-240
    sig = np.arange(N, dtype=np.float32)
    out = _soft(N, range(N - 2), sig)
    r0, r1 = np.float32(0), np.float32(0)
    for i in range(0, N, 2):
        r0 += sig[i]
        r1 += sig[i + 1]
    np.testing.assert_allclose(out[0::2], r0, atol=1e-7)
    np.testing.assert_allclose(out[1::2], r1, atol=1e-7)


@pytest.mark.parametrize("N", [4, 8, 16, 32, 64, 128, 256])
def test_kat_spc(N):  # decodingtest.cpp:244-282
    sig = (np.arange(N) - 2.9).astype(np.float32)
    exp = sig.copy()
    exp[3] *= -1.0
    np.testing.assert_allclose(_soft(N, [0], sig), exp, atol=1e-7)


@pytest.mark.parametrize("kind,N", [("dspc", 8), ("dspc", 16), ("dspc", 32), ("dspc", 64),
                                    ("type5", 8), ("type5", 16), ("type5", 32), ("type5", 64),
                                    ("repr1", 8)])
def test_kat_generic_leaves(oracle, kind, N):  # decodingtest.cpp:284-411
    rng = np.random.default_rng(N)
    sig = rng.normal(10.0, 20.0, N).astype(np.float32)
    if kind == "dspc":
        fr = [0, 1]
    elif kind == "type5":
        fr = list(range(N - 5)) + [N - 4]
    else:
        fr = [0, 1, 2]
    out = _soft(N, fr, sig)
    _, _, exp = oracle.sc_decode(N, fr, sig[None, :], systematic=False, soft=True)
    np.testing.assert_allclose(out, exp[0], atol=1e-7)
    assert np.array_equal(out.view(np.uint32), exp[0].view(np.uint32))


def test_soft_codewords_bit_exact_vs_oracle(oracle):
    """Every Fast-SSC node kind at the root and inside BB codes, LLR families with ties,
    +-0 and wide ranges: the soft codeword equals the oracle's word for word."""
    from antpolarcodes_amd._native import PCG_E_FROZEN, PcgError, Plan
    rng = np.random.default_rng(5)
    cases = [(N, fr) for N, fr in node_cover_sets()]
    for N in (64, 256, 1024):
        cases.append((N, oracle.frozen_bits_bb(N, N // 2, 0.0)))
    for N, fr in cases:
        try:
            p = Plan(N, 1, fr, systematic=False, crc=0, device=0)
        except PcgError as e:  # frozen patterns the reference rejects (invalid_argument)
            assert e.code == PCG_E_FROZEN
            continue
        for kind in LLR_KINDS:
            llr = llr_kinds(rng, 16, N, kind)
            info, ok, soft = _decode_soft(p, llr)
            oi, _, osoft = oracle.sc_decode(N, fr, llr, systematic=False, crc=0, soft=True)
            assert np.array_equal(info, oi), (N, kind)
            bad = np.nonzero(~(soft.view(np.uint32) == osoft.view(np.uint32)).all(axis=1))[0]
            assert bad.size == 0, f"N={N} {kind}: soft codeword differs in frames {bad[:4]}"


def _decode_soft(plan, llr):
    import torch
    F = llr.shape[0]
    d_llr = torch.from_numpy(np.ascontiguousarray(llr)).cuda()
    info = torch.zeros((F, plan.kb), dtype=torch.uint8, device="cuda")
    ok = torch.zeros(F, dtype=torch.uint8, device="cuda")
    soft = torch.zeros((F, plan.N), dtype=torch.float32, device="cuda")
    plan.decode_soft_device(d_llr, info, ok, soft)
    torch.cuda.synchronize()
    hi, hok, hs = plan.decode_soft_host(llr)  # the host-buffer entry point agrees
    assert np.array_equal(hi, info.cpu().numpy()) and np.array_equal(hs.view(np.uint32),
                                                                      soft.cpu().numpy().view(np.uint32))
    return info.cpu().numpy(), ok.cpu().numpy(), soft.cpu().numpy()


def test_soft_information_and_unsupported(oracle):
    from antpolarcodes_amd import pypolar
    N, K = 256, 128
    fr = oracle.frozen_bits_bb(N, K, 0.0)
    sig = np.random.default_rng(1).normal(0.5, 1.0, N).astype(np.float32)
    d = _dec(N, fr)
    d.decode_vector(sig)
    sc = d.getSoftCodeword()
    info_pos = np.setdiff1d(np.arange(N), fr)
    assert np.array_equal(d.getSoftInformation().view(np.uint32), sc[info_pos].view(np.uint32))



def test_soft_outputs_of_list_char_and_adaptive_decoders(oracle):
    """List, 8-bit and adaptive GPU decoders return the selected path's signed hard decisions
    from getSoftCodeword / getSoftInformation (the reference copies the selected path's bit
    buffer into mBitContainer, scl_avx_float.cpp:711-750, and returns it, decoder.cpp:147-151;
    only its signs are observable): signs = the oracle's selected-path codeword, the soft
    information = the codeword at the information positions."""
    from antpolarcodes_amd import frames, pypolar
    N, K = 256, 128
    fr = oracle.frozen_bits_bb(N, K, 0.0)
    info_pos = np.setdiff1d(np.arange(N), fr)
    llr, _, _ = frames.awgn_frames(N, fr, 12, 1.0, seed=3, crc=8)
    x8 = np.clip(np.rint(llr * 10.0), -128, 127).astype(np.int8)
    cases = [("gpu", 8, llr, oracle.scl_decode(N, 8, fr, llr, crc=8, carry=True)[0]),
             ("char", 8, x8, oracle.sclc_decode(N, 8, fr, x8, crc=8, carry=True)[0]),
             ("char", 1, x8, oracle.scc_decode(N, fr, x8, crc=8)[0])]
    sc_i, sc_k = oracle.sc_decode(N, fr, llr, crc=8)
    scl_i = oracle.scl_decode(N, 8, fr, llr, crc=8)[0]
    ad = sc_i.copy()
    ad[sc_k == 0] = scl_i[sc_k == 0]
    cases.append(("mixed", 8, llr, ad))
    for typ, L, x, exp_info in cases:
        d = pypolar.PolarDecoder(N, L, fr, typ)
        d.setErrorDetection(8)
        exp_cw = np.asarray(oracle.encode(N, fr, exp_info, systematic=True, crc=0))
        for f in range(x.shape[0]):
            assert np.array_equal(d.decode_vector(x[f]), exp_info[f]), (typ, L, f)
            soft = d.getSoftCodeword()
            assert soft.shape == (N,)
            neg = soft < 0 if soft.dtype == np.int8 else np.signbit(soft)
            assert np.array_equal(np.packbits(neg.astype(np.uint8)), exp_cw[f]), (typ, L, f)
            si = d.getSoftInformation()
            assert np.array_equal(si.view(np.uint8), soft[info_pos].view(np.uint8)), (typ, L, f)


def test_scl_metric_carry_q8_fixture(oracle):
    """48 successive decode_vector calls on ONE SCL-8 decoder reproduce the reference's
    carried-metric run (tests/golden/reference_fixtures.npz scl8_*_carry, made with one
    reused reference decoder) and the oracle's carried path metrics bit for bit."""
    import os
    from antpolarcodes_amd import pypolar
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.npz"))
    llr = fx["scl8_llr"]
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    dec = pypolar.PolarDecoder(1024, 8, fr, "gpu")  # makeDecoder installs CRC-8 (Q5)
    _, _, om, _, _ = oracle.scl_decode(1024, 8, fr, llr, crc=8, carry=True, paths=True)
    got = []
    for f in range(llr.shape[0]):
        assert dec.carriedMetric() == (0.0 if f == 0 else om[f - 1, 0])
        got.append(dec.decode_vector(llr[f]))
    assert np.array_equal(np.array(got), fx["scl8_info_carry"])
    assert np.float32(dec.carriedMetric()).view(np.uint32) == om[-1, 0].view(np.uint32)
    # a batch keeps fresh-decoder semantics and leaves the carried metric alone
    carried = dec.carriedMetric()
    assert np.array_equal(dec.decode_batch(llr), fx["scl8_info"])
    assert dec.carriedMetric() == carried


def test_scl_metric_carry_char(oracle):
    """The same carry through the 8-bit list decoder (SclFipChar), against the oracle."""
    from antpolarcodes_amd import pypolar
    N = 256
    fr = oracle.frozen_bits_bb(N, 128, 0.0)
    rng = np.random.default_rng(9)
    x8 = np.clip(np.rint(rng.normal(3, 12, (24, N))), -128, 127).astype(np.int8)
    dec = pypolar.PolarDecoder(N, 8, fr, "char")
    oi, _, om, _, _ = oracle.sclc_decode(N, 8, fr, x8, crc=8, carry=True, paths=True)
    got = np.array([dec.decode_vector(x8[f]) for f in range(x8.shape[0])])
    assert np.array_equal(got, oi)
    assert dec.carriedMetric() == om[-1, 0]
