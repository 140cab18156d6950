"""Pin the oracle (oracle/polar_oracle.c) to the reference (CPU, no GPU).

1. Against tests/golden/reference_fixtures.npz: outputs of the reference library
   compiled from /root/reference (tests/golden/make_golden.py).
2. Against the reference's own known-answer tests (test/polarcode/decodingtest.cpp,
   python/qa_pypolar_detector.py), restated here as data.
3. Where oracle/_ref/libpolarref.so exists (this container), directly against the
   reference on fresh random inputs.
"""
import os

import numpy as np
import pytest

from pyoracle import Reference

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.npz")


@pytest.fixture(scope="module")
def fx():
    return np.load(GOLD, allow_pickle=False)


def bits_u32(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


# ---------------------------------------------------------------- known answers
def test_kat_f_g_combine(oracle):
    # decodingtest.cpp:462-494 (_mm256_set_ps lists lanes 7..0)
    l0 = np.array([0, 1, 2, 3, 4, 5, 6, -7][::-1], np.float32)
    l1 = np.array([1, 2, 3, -4, 5, 6, -7, 8][::-1], np.float32)
    assert np.array_equal(oracle.f(l0, l1), np.array([0, 1, 2, -3, 4, 5, -6, -7][::-1], np.float32))
    l1 = np.array([-1, 2, 3, -4, 5, 6, -7, 8][::-1], np.float32)
    bits = np.array([0, 0, 0, -128, 0, 0, -128, -128][::-1], np.float32)
    assert np.array_equal(oracle.g(l0, l1, bits), np.array([-1, 3, 5, -7, 9, 11, -13, 15][::-1], np.float32))
    out = oracle.combine_short(np.array([1, 1, 1, 1, 0, 0, 0, 0], np.float32),
                               np.array([-1, -1, -1, -1, 0, 0, 0, 0], np.float32), 4)
    assert np.all(np.signbit(out))  # testBitVectors: all sign bits set


def test_kat_list_decoder_n8(oracle):
    # decodingtest.cpp:1128-1177: SclAvxFloat(8, 4, {0,1,2,4}) on {-5,-6,-4,1,-4,-5,-7,2}
    llr = np.array([[-5, -6, -4, 1, -4, -5, -7, 2]], np.float32)
    info, _ = oracle.scl_decode(8, 4, [0, 1, 2, 4], llr, crc=0)
    assert (info[0, 0] & 0xF0) == 0xF0


@pytest.mark.parametrize("msg,ref", [("TestFooB", 0xC2), ("FooBarPolar", 0xA1)])
def test_kat_crc8_generate(oracle, msg, ref):
    # qa_pypolar_detector.py:33-51
    d = np.array([ord(c) for c in msg] + [0], np.uint8)
    assert oracle.crc(8, d, generate=True)[-1] == ref


@pytest.mark.parametrize("msg,ref", [("ChaoticLama", 0x67), ("NeverListenToTheVoid!", 0x69)])
def test_kat_crc8_check(oracle, msg, ref):
    d = [ord(c) for c in msg]
    assert oracle.crc(8, d + [ref])
    assert not oracle.crc(8, d + [42])


@pytest.mark.parametrize("msg,ref", [("Test", [0x8C, 0x2D, 0xE2, 0x19]), ("FooBarPolarT", [0x38, 0xAC, 0x62, 0xC9])])
def test_kat_crc32_generate(oracle, msg, ref):
    # qa_pypolar_detector.py:73-103
    d = np.array([ord(c) for c in msg] + [0, 0, 0, 0], np.uint8)
    assert list(oracle.crc(32, d, generate=True)[-4:]) == ref


def test_kat_crc32_check(oracle):
    d = [ord(c) for c in "DisgustinRoastedWhip"] + [0xD0, 0x0B, 0xD6, 0xFE]
    assert oracle.crc(32, d)
    for i in range(len(d)):
        e = list(d)
        e[i] = 0
        assert not oracle.crc(32, e)


@pytest.mark.parametrize("msg,ref", [("Test", [0x28, 0x88]), ("RIPloPTiger", [0x69, 0x6F])])
def test_kat_crc16_generate(oracle, msg, ref):
    # qa_pypolar_detector.py:142-168
    d = np.array([ord(c) for c in msg] + [0, 0], np.uint8)
    assert list(oracle.crc(16, d, generate=True)[-2:]) == ref


def test_kat_crc16_check(oracle):
    d = [ord(c) for c in "DisgustinRoastedWhip"] + [0xA3, 0x2B]
    assert oracle.crc(16, d)
    for i in range(len(d)):
        e = list(d)
        e[i] = 0
        assert not oracle.crc(16, e)


# ---------------------------------------------------------------- reference fixtures
def test_fixture_construction(oracle, fx):
    from antpolarcodes_amd.construction import frozen_bits
    off = 0
    for N, K, d, n in zip(fx["cons_N"], fx["cons_K"], fx["cons_dsnr"], fx["cons_len"]):
        exp = [int(v) for v in fx["cons_frozen"][off:off + n]]
        off += n
        assert oracle.frozen_bits_bb(int(N), int(K), float(d)) == exp
        assert frozen_bits(int(N), int(K), float(d)) == exp


def test_fixture_crc_generate(oracle, fx):
    for kind in (8, 16, 32):
        for row in fx[f"crc{kind}_gen"]:
            msg = row.copy()
            msg[-(kind // 8):] = 0
            assert np.array_equal(oracle.crc(kind, msg, generate=True), row)
            assert oracle.crc(kind, row)


def test_fixture_encoder(oracle, fx):
    from antpolarcodes_amd import frames
    fr = [int(v) for v in fx["sc_frozen"]]
    for sysm in (0, 1):
        for crc in (0, 8, 32):
            exp = fx[f"enc_s{sysm}_c{crc}"]
            assert np.array_equal(oracle.encode(1024, fr, fx["enc_info"], bool(sysm), crc), exp)
            got = np.packbits(frames.encode(1024, fr, fx["enc_info"], bool(sysm), crc), axis=1)
            assert np.array_equal(got, exp)


def test_fixture_fastssc(oracle, fx):
    fr = [int(v) for v in fx["sc_frozen"]]
    for sysm in (0, 1):
        info, ok, cw = oracle.sc_decode(1024, fr, fx["sc_llr"], systematic=bool(sysm), crc=8, soft=True)
        assert np.array_equal(info, fx[f"sc_info_s{sysm}"])
        assert np.array_equal(ok, fx[f"sc_ok_s{sysm}"])
        if sysm:
            assert np.array_equal(np.packbits((bits_u32(cw) >> 31).astype(np.uint8), axis=1), fx["sc_softcw_sign"])
            assert np.array_equal(bits_u32(cw)[:8], fx["sc_softcw_bits"])  # whole float words


def test_fixture_fastssc_node_kinds(oracle, fx):
    fo = lo = so = 0
    for N, nf, F in fx["kinds_meta"]:
        fr = [int(v) for v in fx["kinds_frozen"][fo:fo + nf]]
        llr = fx["kinds_llr"][lo:lo + F * N].reshape(F, N)
        exp = fx["kinds_softcw"][so:so + F * N].reshape(F, N)
        fo, lo, so = fo + nf, lo + F * N, so + F * N
        _, _, cw = oracle.sc_decode(int(N), fr, llr, crc=0, soft=True)
        assert np.array_equal(bits_u32(cw), exp), (N, fr)


def test_fixture_q1_zerospc(oracle, fx):
    # Q1: ZeroSpcDecoder decides from the right half only -> all 16 signs negative
    _, _, cw = oracle.sc_decode(16, list(range(9)), fx["q1_llr"], crc=0, soft=True)
    assert np.array_equal(bits_u32(cw), fx["q1_softcw"])
    assert np.all(np.signbit(cw))


def test_fixture_scl8(oracle, fx):
    fr = [int(v) for v in fx["sc_frozen"]]
    info, ok, met, pc, pb = oracle.scl_decode(1024, 8, fr, fx["scl8_llr"], crc=8, paths=True)
    assert np.array_equal(info, fx["scl8_info"])
    assert np.array_equal(ok, fx["scl8_ok"])
    assert np.array_equal(bits_u32(met), bits_u32(fx["scl8_metrics"]))
    assert np.array_equal(pc, fx["scl8_pathcount"])
    assert np.array_equal(pb, fx["scl8_pathbits"])
    info, ok = oracle.scl_decode(1024, 8, fr, fx["scl8_llr"], systematic=False, crc=8)
    assert np.array_equal(info, fx["scl8_info_nonsys"])
    assert np.array_equal(ok, fx["scl8_ok_nonsys"])


def test_fixture_scl8_metric_carry_q8(oracle, fx):
    """Q8: one reference decoder instance carries path 0's metric from frame to frame."""
    fr = [int(v) for v in fx["sc_frozen"]]
    info, ok = oracle.scl_decode(1024, 8, fr, fx["scl8_llr"], crc=8, carry=True)
    assert np.array_equal(info, fx["scl8_info_carry"])
    assert np.array_equal(ok, fx["scl8_ok_carry"])


def test_fixture_scl32_n4096(oracle, fx):
    fr = [int(v) for v in fx["scl32_frozen"]]
    info, ok, met, pc, _ = oracle.scl_decode(4096, 32, fr, fx["scl32_llr"], crc=8, paths=True)
    assert np.array_equal(info, fx["scl32_info"])
    assert np.array_equal(ok, fx["scl32_ok"])
    assert np.array_equal(bits_u32(met), bits_u32(fx["scl32_metrics"]))
    assert np.array_equal(pc, fx["scl32_pathcount"])


def test_fixture_scl_small_all_list_sizes(oracle, fx):
    fo = lo = mo = po = bo = 0
    for N, L, nf, F in fx["sclsmall_meta"]:
        N, L, nf, F = int(N), int(L), int(nf), int(F)
        fr = [int(v) for v in fx["sclsmall_frozen"][fo:fo + nf]]
        llr = fx["sclsmall_llr"][lo:lo + F * N].reshape(F, N)
        em = fx["sclsmall_metrics"][mo:mo + F * L].reshape(F, L)
        ep = fx["sclsmall_pathcount"][po:po + F]
        eb = fx["sclsmall_pathbits"][bo:bo + F * L * N // 8].reshape(F, L, N // 8)
        fo, lo, mo, po, bo = fo + nf, lo + F * N, mo + F * L, po + F, bo + F * L * N // 8
        _, _, met, pc, pb = oracle.scl_decode(N, L, fr, llr, crc=0, paths=True)
        assert np.array_equal(bits_u32(met), bits_u32(em)), (N, L)
        assert np.array_equal(pc, ep) and np.array_equal(pb, eb), (N, L)


# ---------------------------------------------------------------- live reference
ref_only = pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built here")


@ref_only
def test_live_reference_fastssc_random(oracle):
    R = Reference()
    rng = np.random.default_rng(1)
    for t in range(150):
        N = int(2 ** rng.integers(3, 9))
        fr = sorted(rng.choice(N, int(rng.integers(0, N + 1)), replace=False).tolist())
        x = rng.integers(-3, 4, (3, N)).astype(np.float32) if t % 2 else rng.normal(0, 2, (3, N)).astype(np.float32)
        try:
            _, _, rc = R.decode(N, 1, fr, x, crc=0, soft=True)
        except ValueError:
            with pytest.raises(ValueError):
                oracle.sc_decode(N, fr, x, crc=0)
            continue
        _, _, oc = oracle.sc_decode(N, fr, x, crc=0, soft=True)
        assert np.array_equal(bits_u32(rc), bits_u32(oc))


@ref_only
def test_live_reference_scl_random(oracle):
    R = Reference()
    rng = np.random.default_rng(2)
    for t in range(60):
        N = int(2 ** rng.integers(3, 8))
        L = int(2 ** rng.integers(1, 6))
        fr = sorted(rng.choice(N, int(rng.integers(0, N + 1)), replace=False).tolist())
        x = rng.integers(-2, 3, (2, N)).astype(np.float32) if t % 2 else rng.normal(0, 2, (2, N)).astype(np.float32)
        rm, rp, rb = R.scl_paths(N, L, fr, x)
        _, _, om, op, ob = oracle.scl_decode(N, L, fr, x, crc=0, paths=True)
        assert np.array_equal(bits_u32(rm), bits_u32(om)) and np.array_equal(rp, op) and np.array_equal(rb, ob)


@ref_only
def test_live_reference_scl_non_power_of_two_lists(oracle):
    """SCL with L not a power of two (the reference accepts any L): ordered metrics, path
    counts and path codewords equal the reference's, and so do info/ok with CRC-8."""
    R = Reference()
    rng = np.random.default_rng(3)
    for L in (3, 5, 6, 7, 12, 24):
        for t in range(12):
            N = int(2 ** rng.integers(3, 9))
            fr = sorted(rng.choice(N, int(rng.integers(0, N + 1)), replace=False).tolist())
            x = rng.integers(-2, 3, (2, N)).astype(np.float32) if t % 2 else rng.normal(0, 2, (2, N)).astype(np.float32)
            rm, rp, rb = R.scl_paths(N, L, fr, x)
            _, _, om, op, ob = oracle.scl_decode(N, L, fr, x, crc=0, paths=True)
            assert np.array_equal(bits_u32(rm), bits_u32(om)) and np.array_equal(rp, op) and np.array_equal(rb, ob)
        fr = oracle.frozen_bits_bb(1024, 512, 0.0)
        x = rng.normal(1.0, 1.2, (8, 1024)).astype(np.float32)
        ri, rk = R.decode(1024, L, fr, x, crc=8, fresh=True)
        oi, ok = oracle.scl_decode(1024, L, fr, x, crc=8)
        assert np.array_equal(ri, oi) and np.array_equal(rk, ok)


def test_oracle_matches_reference_digests_full_size(oracle):
    """The full-size batches the GPU tests decode (2^16 config-2 frames, config 4's 2048
    depunctured frames) give the reference's outputs through the oracle too -- the digests
    of tests/golden/reference_digests.json (made from oracle/_ref by make_digests.py)."""
    import importlib.util
    from helpers import reference_digest, sha256
    spec = importlib.util.spec_from_file_location(
        "make_digests", os.path.join(os.path.dirname(__file__), "golden", "make_digests.py"))
    md = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(md)
    for name in ("config2_sc", "config4_nr_scl8"):
        c = md.CASES[name]
        d = reference_digest(name)
        fr, llr = md.case_frames(c)
        assert sha256(llr) == d["llr"], name
        if c["L"] == 1:
            info, ok = oracle.sc_decode(c["N"], fr, llr, crc=c["crc"])
        else:
            info, ok, met, _, _ = oracle.scl_decode(c["N"], c["L"], fr, llr, crc=c["crc"], paths=True)
            assert sha256(met) == d["metrics"], name
        assert sha256(info) == d["info"] and sha256(ok) == d["ok"], name
