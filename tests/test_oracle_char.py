"""Pin the int8 oracle (oracle/polar_oracle_char.c) to the reference (CPU, no GPU).

1. tests/golden/char_fixtures.npz: outputs of the reference's FastSscFipChar /
   SclFipChar / CharContainer compiled from /root/reference (make_golden_char.py).
2. The reference's own known-answer tests for the 8-bit path, restated as data:
   test/polarcode/decodingtest.cpp:77-155 (Rep / DoubleRep soft outputs),
   testGeneralDecodingFunctionsAvx2 (F, G, CombineBitsShort vectors) and the
   `'char'` case of python/qa_pypolar_decoder.py:77-113.
3. Where oracle/_ref exists (this container), directly against the reference on
   fresh random inputs.
"""
import os

import numpy as np
import pytest

from pyoracle import Reference

from antpolarcodes_amd import frames
from antpolarcodes_amd.construction import frozen_bits

GOLD = os.path.join(os.path.dirname(__file__), "golden", "char_fixtures.npz")


@pytest.fixture(scope="module")
def fx():
    return np.load(GOLD, allow_pickle=False)


def i8_families(rng, F, N):
    out = [
        np.clip(np.rint(rng.normal(8, 20, (F, N))), -128, 127),
        rng.integers(-3, 4, (F, N)),
        rng.choice(np.array([-128, -127, 127, 126, -1, 0, 1]), (F, N)),
        rng.integers(-128, 128, (F, N)),
    ]
    return np.concatenate(out).astype(np.int8)


# ---------------------------------------------------------------- known answers
def test_kat_fip_functions(oracle):
    # decodingtest.cpp testGeneralDecodingFunctionsAvx2: _mm256_set_epi8 lists lanes 31..0
    l0 = np.array([0, 1, 2, 3, 4, 5, 6, -7, 8, 9, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9,
                   0, 1][::-1], np.int8)
    l1 = np.array([-1, 2, 3, -4, 5, 6, -7, 8, 9, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 0,
                   1, 2][::-1], np.int8)
    f_exp = np.array([-1, 1, 2, -3, 4, 5, -6, -7, 8, 1, 1, 1, 2, 3, 4, 5, 6, 7, 8, 1, 1, 1, 2, 3, 4, 5, 6, 7, 8,
                      1, 1, 1][::-1], np.int8)
    assert np.array_equal(oracle.fip_f(l0, l1), f_exp)
    bits = np.zeros(32, np.int8)
    bits[[31 - 3, 31 - 6, 31 - 7]] = -128
    g_exp = np.array([-1, 3, 5, -7, 9, 11, -13, 15, 17, 9, 1, 3, 5, 7, 9, 11, 13, 15, 17, 9, 1, 3, 5, 7, 9, 11,
                      13, 15, 17, 9, 1, 3][::-1], np.int8)
    assert np.array_equal(oracle.fip_g(l0, l1, bits), g_exp)
    out = oracle.fip_combine_short([127] * 8 + [0] * 24, [-128] * 8 + [0] * 24, 8)
    assert np.all(out[:16] < 0) and np.all(out[16:] >= 0)  # testBitVectors: signs only
    # extended combine test: sign(out[0]) = sign(l) ^ sign(r) for h = 1
    for l in (-128, -5, 0, 77, 127):
        for r in (-128, -1, 0, 3, 127):
            o = oracle.fip_combine_short([l] + [0] * 31, [r] + [0] * 31, 1)
            assert (o[0] < 0) == ((l < 0) != (r < 0))


@pytest.mark.parametrize("n", [32, 64])
def test_kat_repetition_soft(oracle, n):
    # decodingtest.cpp:83-111 / 118-155: FastSscFipChar(n, {0..n-2}) resp. {0..n-3},
    # non-systematic, signal = iota(-n/2 - 1)
    sig = (np.arange(n) - n // 2 - 1).astype(np.int8)[None]
    _, _, soft = oracle.scc_decode(n, list(range(n - 1)), sig, systematic=False, crc=0, soft=True)
    assert np.all(soft[0] == np.int8(max(-128, min(127, int(sig.astype(int).sum())))))
    _, _, soft = oracle.scc_decode(n, list(range(n - 2)), sig, systematic=False, crc=0, soft=True)
    r0 = max(-128, min(127, int(sig[0, 0::2].astype(int).sum())))
    r1 = max(-128, min(127, int(sig[0, 1::2].astype(int).sum())))
    assert np.all(soft[0, 0::2] == r0) and np.all(soft[0, 1::2] == r1)


@pytest.mark.parametrize("n", [7, 8, 9, 10])
def test_kat_qa_pypolar_char(oracle, n):
    # qa_pypolar_decoder.py:77-113 ('char', L = 1): CRC-8, llr = 1 - 2b + U(-0.2, 0.2)
    rng = np.random.default_rng(n)
    N = 1 << n
    for K in (N * 3 // 4, N // 2, N // 4, N // 8):
        fr = frozen_bits(N, K, -1.0)
        info = frames.crc_generate(8, rng.integers(0, 256, (10, K // 8)).astype(np.uint8))
        b = frames.encode(N, fr, info, systematic=True, crc=0).astype(np.float32)
        llr = (1.0 - 2.0 * b + rng.uniform(-0.2, 0.2, b.shape)).astype(np.float32)
        got, ok = oracle.scc_decode(N, fr, llr, crc=8)
        assert np.array_equal(got, info) and ok.all()


# ---------------------------------------------------------------- reference fixtures
@pytest.mark.parametrize("N", [8, 16, 32, 64])
def test_fixture_quantisation(oracle, fx, N):
    assert np.array_equal(oracle.f32_to_i8(fx[f"q{N}_in"], N), fx[f"q{N}_out"])


def test_fixture_fastssc_char(oracle, fx):
    fo = lo = io = oo = 0
    for i, N in enumerate(fx["sc_N"]):
        N = int(N)
        nf = int(fx["sc_len"][i])
        fr = fx["sc_frozen"][fo:fo + nf].astype(np.uint32)
        fo += nf
        F = 8 if N <= 256 else 4
        llr = fx["sc_llr"][lo:lo + F * N].reshape(F, N)
        lo += F * N
        kb = (N - nf + 7) // 8
        info, ok, soft = oracle.scc_decode(N, fr, llr, bool(fx["sc_sys"][i]), int(fx["sc_crc"][i]), soft=True)
        assert np.array_equal(info.ravel(), fx["sc_info"][io:io + F * kb]), (N, nf)
        assert np.array_equal(ok, fx["sc_ok"][oo:oo + F]), (N, nf)
        oo += F
        assert np.array_equal(soft.ravel(), fx["sc_soft"][lo - F * N:lo]), (N, nf)
        io += F * kb


def test_fixture_float_input(oracle, fx):
    fr = fx["fin_frozen"].astype(np.uint32)
    info, ok = oracle.scc_decode(1024, fr, fx["fin_llr"], crc=8)
    assert np.array_equal(info, fx["fin_sc_info"]) and np.array_equal(ok, fx["fin_sc_ok"])
    info, ok = oracle.sclc_decode(1024, 8, fr, fx["fin_llr"], crc=8)
    assert np.array_equal(info, fx["fin_scl8_info"]) and np.array_equal(ok, fx["fin_scl8_ok"])


@pytest.mark.parametrize("j", range(10))
def test_fixture_scl_char(oracle, fx, j):
    k = f"scl{j}"
    N, K, L, crc = (int(v) for v in fx[k + "_meta"])
    fr = fx[k + "_frozen"].astype(np.uint32)
    info, ok, met, pc, pb = oracle.sclc_decode(N, L, fr, fx[k + "_llr"], crc=crc, paths=True)
    assert np.array_equal(info, fx[k + "_info"]) and np.array_equal(ok, fx[k + "_ok"])
    assert np.array_equal(met, fx[k + "_met"])
    assert np.array_equal(pc, fx[k + "_pc"])
    assert np.array_equal(pb, fx[k + "_pb"])


def test_fixture_scl_char_carry_and_nonsystematic(oracle, fx):
    fr = fx["carry_frozen"].astype(np.uint32)
    info, ok = oracle.sclc_decode(256, 8, fr, fx["carry_llr"], crc=8, carry=True)
    assert np.array_equal(info, fx["carry_info"]) and np.array_equal(ok, fx["carry_ok"])
    fresh, _ = oracle.sclc_decode(256, 8, fr, fx["carry_llr"], crc=8)
    assert np.array_equal(fresh, info)  # integer metrics: the carried offset changes no decision
    info, ok = oracle.sclc_decode(256, 8, fr, fx["carry_llr"], systematic=False, crc=8)
    assert np.array_equal(info, fx["nsys_info"]) and np.array_equal(ok, fx["nsys_ok"])


# ---------------------------------------------------------------- live reference
needs_ref = pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built here")


@needs_ref
@pytest.mark.parametrize("seed", range(6))
def test_live_reference_char(oracle, seed):
    R = Reference()
    rng = np.random.default_rng(1000 + seed)
    for _ in range(12):
        N = int(rng.choice([8, 16, 32, 64, 128, 256, 512]))
        K = int(rng.integers(1, N))
        fr = sorted(rng.choice(N, N - K, replace=False).tolist()) if rng.random() < 0.5 else frozen_bits(N, K, 0.0)
        llr = i8_families(rng, 1, N)
        sysm = N < 256 or bool(rng.integers(0, 2))
        L = int(rng.choice([1, 2, 4, 8, 32]))
        if L == 1:
            a = oracle.scc_decode(N, fr, llr, sysm, 0, soft=True)
            b = R.decode_char(N, 1, fr, llr, sysm, 0, soft=True)
            for x, y in zip(a, b):
                assert np.array_equal(x, y), (N, K, L)
        else:
            a = oracle.sclc_decode(N, L, fr, llr, sysm, 0, paths=True)
            b = R.decode_char(N, L, fr, llr, sysm, 0, fresh=True)
            m, pc, pb = R.sclc_paths(N, L, fr, llr)
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), (N, K, L)
            assert np.array_equal(a[2], m) and np.array_equal(a[3], pc) and np.array_equal(a[4], pb)
