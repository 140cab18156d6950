"""GPU parity of the 8-bit decoders (FastSscFipChar / SclFipChar on MI355X) against the
int8 oracle (oracle/polar_oracle_char.c, pinned to the reference by
tests/test_oracle_char.py): decoded bytes, ok flags and integer SCL path metrics
bit-exact, for int8 frames (pcg_decode_i8) and float frames quantised in the kernel
(pcg_decode_f32 on an 8-bit plan, CharContainer::insertLlr semantics)."""
import numpy as np
import pytest

from antpolarcodes_amd import frames
from antpolarcodes_amd.construction import frozen_bits

pytestmark = pytest.mark.gpu


def i8_kinds(rng, F, N, kind):
    if kind == "normal":
        return np.clip(np.rint(rng.normal(8, 20, (F, N))), -128, 127).astype(np.int8)
    if kind == "ints":  # ties and zeros everywhere
        return rng.integers(-3, 4, (F, N)).astype(np.int8)
    if kind == "sat":   # saturation, -128, +-0
        return rng.choice(np.array([-128, -127, 127, 126, -1, 0, 1], np.int8), (F, N))
    if kind == "full":
        return rng.integers(-128, 128, (F, N)).astype(np.int8)
    raise ValueError(kind)


KINDS = ("normal", "ints", "sat", "full")


def _plan(N, L, fr, systematic=True, crc=8):
    from antpolarcodes_amd._native import Plan
    return Plan(N, L, fr, systematic=systematic, crc=crc, device=0, fixed=True)


def _check(oracle, N, L, fr, llr, systematic=True, crc=8):
    p = _plan(N, L, fr, systematic, crc)
    if llr.dtype == np.int8:
        gi, gok, gm = p.decode_host_i8(llr, want_metrics=L > 1)
    else:
        gi, gok, gm = p.decode_host(llr, want_metrics=L > 1)
    if L == 1:
        oi, ook = oracle.scc_decode(N, fr, llr, systematic, crc)
    else:
        oi, ook, om, _, _ = oracle.sclc_decode(N, L, fr, llr, systematic, crc, paths=True)
        assert np.array_equal(gm, om.astype(np.float32)), f"N={N} L={L}: path metrics differ"
    bad = np.nonzero(~(gi == oi).all(axis=1))[0]
    assert bad.size == 0, f"N={N} K={N - len(fr)} L={L}: info mismatch in frames {bad[:8]}"
    assert np.array_equal(gok, ook)


def cover_codes():
    from antpolarcodes_amd.rtc_codes import char_cover_codes
    return char_cover_codes()


# ------------------------------------------------------------------ FastSscFipChar
@pytest.mark.parametrize("N", [8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096])
def test_scc_bb_codes(oracle, N):
    rng = np.random.default_rng(N)
    for K in sorted({N // 8, N // 4, N // 2, 3 * N // 4, N - 8}):
        if K < 8:
            continue
        for dsnr in (-2.0, 0.0, 3.0):
            fr = frozen_bits(N, K, dsnr)
            for kind in KINDS:
                _check(oracle, N, 1, fr, i8_kinds(rng, 16, N, kind), crc=8 if K % 8 == 0 else 0)


def test_scc_node_kinds_and_random_sets(oracle):
    rng = np.random.default_rng(11)
    codes = cover_codes()
    for _ in range(120):
        N = int(2 ** rng.integers(3, 10))
        codes.append((N, sorted(rng.choice(N, int(rng.integers(0, N + 1)), replace=False).tolist())))
    for N, fr in codes:
        for kind in KINDS:
            _check(oracle, N, 1, fr, i8_kinds(rng, 8, N, kind), crc=0)


@pytest.mark.parametrize("systematic", [True, False])
@pytest.mark.parametrize("crc", [0, 8, 16, 32])
def test_scc_crc_systematic(oracle, systematic, crc):
    rng = np.random.default_rng(7 + crc)
    for N, K in ((64, 32), (256, 128), (1024, 512)):
        fr = frozen_bits(N, K, 0.0)
        _check(oracle, N, 1, fr, i8_kinds(rng, 64, N, "normal"), systematic, crc)


@pytest.mark.parametrize("N", [8, 16, 32, 256, 1024])
def test_scc_float_input_quantised_in_kernel(oracle, N):
    rng = np.random.default_rng(100 + N)
    x = (rng.normal(0, 60, (64, N)) * 10.0 ** rng.uniform(-1, 1.5, (64, N))).astype(np.float32)
    x[0, :4] = [np.nan, 3e9, -3e9, np.inf]
    x[1, :4] = [126.5, 127.5, -128.5, 0.5]
    _check(oracle, N, 1, frozen_bits(N, N // 2, 0.0), x)


@pytest.mark.parametrize("F", [1, 3, 63, 64, 65, 1000])
def test_scc_batch_sizes(oracle, F):
    rng = np.random.default_rng(F)
    _check(oracle, 1024, 1, frozen_bits(1024, 512, 0.0), i8_kinds(rng, F, 1024, "normal"))


# ------------------------------------------------------------------ SclFipChar
@pytest.mark.parametrize("L", [2, 4, 8, 16, 32])
def test_sclc_list_sizes(oracle, L):
    rng = np.random.default_rng(L)
    for N, K in ((8, 4), (16, 8), (32, 16), (64, 32), (128, 64), (256, 128), (1024, 512)):
        fr = frozen_bits(N, K, 0.0)
        for kind in KINDS:
            _check(oracle, N, L, fr, i8_kinds(rng, 16, N, kind), crc=8 if K % 8 == 0 else 0)


def test_sclc_random_sets(oracle):
    rng = np.random.default_rng(99)
    for _ in range(60):
        N = int(2 ** rng.integers(3, 10))
        fr = sorted(rng.choice(N, int(rng.integers(0, N + 1)), replace=False).tolist())
        L = int(rng.choice([2, 4, 8, 16, 32]))
        _check(oracle, N, L, fr, i8_kinds(rng, 8, N, KINDS[_ % 4]), crc=0)


@pytest.mark.parametrize("systematic", [True, False])
@pytest.mark.parametrize("crc", [0, 8, 16, 32])
def test_sclc_crc_systematic(oracle, systematic, crc):
    rng = np.random.default_rng(3 + crc)
    fr = frozen_bits(1024, 512, 0.0)
    _check(oracle, 1024, 8, fr, i8_kinds(rng, 128, 1024, "normal"), systematic, crc)


def test_sclc_float_input_and_awgn_batch(oracle):
    """Config-3 shape through the 8-bit decoder: AWGN LLRs scaled into the int8 range,
    quantised in the kernel; every frame matches the oracle."""
    fr = frozen_bits(1024, 512, 0.0)
    llr, info, _ = frames.awgn_frames(1024, fr, 4096, 2.0, seed=5, crc=8)
    x = (llr * 4.0).astype(np.float32)
    _check(oracle, 1024, 8, fr, x)
    p = _plan(1024, 8, fr)
    got, ok, _ = p.decode_host(x)
    assert (got == info).all(axis=1).mean() > 0.99


def test_sclc_n4096_l32(oracle):
    rng = np.random.default_rng(4096)
    _check(oracle, 4096, 32, frozen_bits(4096, 2048, 0.0), i8_kinds(rng, 8, 4096, "normal"))


# ------------------------------------------------------------------ host APIs
def test_pypolar_char_decode_vector_and_batch(oracle):
    from antpolarcodes_amd import pypolar
    N, K = 256, 128
    fr = frozen_bits(N, K, 0.0)
    rng = np.random.default_rng(1)
    x8 = i8_kinds(rng, 32, N, "normal")
    for L in (1, 8):
        dec = pypolar.PolarDecoder(N, L, fr, "char")
        dec.setErrorDetection(8)
        exp = oracle.scc_decode(N, fr, x8, crc=8)[0] if L == 1 else oracle.sclc_decode(N, L, fr, x8, crc=8)[0]
        assert np.array_equal(dec.decode_batch(x8), exp)
        for f in range(4):
            assert np.array_equal(dec.decode_vector(x8[f]), exp[f])
            assert np.array_equal(dec.decode_vector(x8[f].astype(np.float32)), exp[f])


def test_torch_device_path_i8(oracle):
    import torch
    from antpolarcodes_amd._native import Plan
    N, L = 1024, 8
    fr = frozen_bits(N, 512, 0.0)
    rng = np.random.default_rng(2)
    x8 = i8_kinds(rng, 512, N, "normal")
    p = Plan(N, L, fr, device=0, fixed=True)
    d = torch.from_numpy(x8).cuda()
    info = torch.empty((512, p.kb), dtype=torch.uint8, device="cuda")
    ok = torch.empty(512, dtype=torch.uint8, device="cuda")
    p.decode_device_i8(d, info, ok)
    torch.cuda.synchronize()
    oi, ook = oracle.sclc_decode(N, L, fr, x8, crc=8)
    assert np.array_equal(info.cpu().numpy(), oi) and np.array_equal(ok.cpu().numpy(), ook)


@pytest.mark.parametrize("F", [1, 63, 65, 1000])
def test_scc_lane_serial_batch_edges(oracle, F):
    rng = np.random.default_rng(F)
    _check(oracle, 256, 1, frozen_bits(256, 128, 0.0), i8_kinds(rng, F, 256, "sat"))


def test_scc_wave_kernel_switch(oracle, monkeypatch):
    """The one-codeword-per-wave 8-bit kernel (PCG_SC_KERNEL=wave) stays bit-exact."""
    monkeypatch.setenv("PCG_SC_KERNEL", "wave")
    rng = np.random.default_rng(5)
    for N in (32, 256, 1024):
        _check(oracle, N, 1, frozen_bits(N, N // 2, 0.0), i8_kinds(rng, 64, N, "normal"))


def test_sclc_layout_variants(oracle, monkeypatch):
    """Every stage placement (LDS budget) of the 8-bit SCL kernel decodes identically."""
    rng = np.random.default_rng(9)
    fr = frozen_bits(1024, 512, 0.0)
    x8 = i8_kinds(rng, 64, 1024, "normal")
    for kb in ("9", "10", "12", "20", "40", "80"):
        monkeypatch.setenv("PCG_SCLC_LDS_KB", kb)
        _check(oracle, 1024, 8, fr, x8)


@pytest.mark.parametrize("kernel", ["interp", "rtc"])
@pytest.mark.parametrize("crc", [8, 16])
def test_adaptive_char_matches_oracle(oracle, crc, kernel):
    """AdaptiveChar (adaptive_char.cpp:33-45): FastSscFipChar, SclFipChar for the failures --
    on the interpreter kernels and on both stages' specialised kernels."""
    from antpolarcodes_amd._native import Plan
    N, L = 1024, 8
    fr = frozen_bits(N, 512, 0.0)
    llr, _, _ = frames.awgn_frames(N, fr, 3000, 1.5, seed=crc, crc=crc)
    x8 = np.clip(np.rint(llr * 10.0), -128, 127).astype(np.int8)
    si, sok = oracle.scc_decode(N, fr, x8, crc=crc)
    li, lok = oracle.sclc_decode(N, L, fr, x8, crc=crc)
    exp = np.where(sok[:, None] == 1, si, li)
    eok = np.where(sok == 1, sok, lok)
    assert (sok == 0).sum() > 10  # the list stage runs
    p = Plan(N, L, fr, crc=crc, device=0, fixed=True, adaptive=True)
    if kernel == "rtc":
        p.specialize()
        assert p.describe()["specialized"] == 1 and p.kernel_name() == "scl_char_rtc_kernel"
    gi, gok, _ = p.decode_host_i8(x8)
    assert np.array_equal(gi, exp) and np.array_equal(gok, eok)
    gi, gok, _ = p.decode_host(llr * 10.0)  # float frames, quantised in the kernels
    assert np.array_equal(gi, exp) and np.array_equal(gok, eok)


# ------------------------------------------------------------------ specialised FastSscFipChar
def rtc_char_codes():
    """(N, frozen, systematic, crc) the specialised 8-bit Fast-SSC kernel is checked on (their
    code objects ship with the library: antpolarcodes_amd/rtc_codes.py)."""
    from antpolarcodes_amd.rtc_codes import char_rtc_codes
    return char_rtc_codes()


def test_scc_rtc_kernel(oracle):
    """The 8-bit Fast-SSC decoder on its plan-specialised kernel (sccs_rtc_kernel: the plan's
    constants and layout as literals): int8 frames of every family and float frames quantised in the
    kernel, bit-exact against the oracle, over BB codes, every 8-bit node kind at n = 64 and the
    detector / systematic variants."""
    from antpolarcodes_amd._native import Plan
    rng = np.random.default_rng(77)
    for N, fr, sysm, crc in rtc_char_codes():
        p = Plan(N, 1, fr, systematic=sysm, crc=crc, device=0, fixed=True)
        p.specialize()
        assert p.kernel_name() == "sccs_rtc_kernel" and p.describe()["specialized"] == 1
        for kind in KINDS:
            x = i8_kinds(rng, 96, N, kind)
            gi, gok, _ = p.decode_host_i8(x)
            oi, ook = oracle.scc_decode(N, fr, x, sysm, crc)
            assert np.array_equal(gi, oi) and np.array_equal(gok, ook), (N, kind, sysm, crc)
        x = (rng.normal(0, 60, (64, N)) * 10.0 ** rng.uniform(-1, 1.5, (64, N))).astype(np.float32)
        gi, gok, _ = p.decode_host(x)
        oi, ook = oracle.scc_decode(N, fr, x, sysm, crc)
        assert np.array_equal(gi, oi) and np.array_equal(gok, ook), (N, "float", sysm, crc)


def test_scc_rtc_config_batch(oracle):
    """sc_char's bench code (N=1024 K=512 CRC-8) on 2^16 int8 AWGN frames through the
    specialised kernel, against the oracle and the interpreter kernel."""
    from antpolarcodes_amd._native import Plan
    fr = frozen_bits(1024, 512, 0.0)
    llr, _, _ = frames.awgn_frames(1024, fr, 1 << 16, 2.0, seed=8, crc=8)
    x = np.clip(np.rint(llr * 8.0), -128, 127).astype(np.int8)
    p = Plan(1024, 1, fr, crc=8, device=0, fixed=True)
    gi0, gok0, _ = p.decode_host_i8(x)
    p.specialize()
    assert p.kernel_name() == "sccs_rtc_kernel"
    gi, gok, _ = p.decode_host_i8(x)
    oi, ook = oracle.scc_decode(1024, fr, x, True, 8)
    assert np.array_equal(gi, oi) and np.array_equal(gok, ook)
    assert np.array_equal(gi0, oi) and np.array_equal(gok0, ook)


@pytest.mark.parametrize("N,K,L,crc,systematic", [(256, 128, 2, 8, True), (1024, 512, 8, 8, True),
                                                  (512, 256, 4, 16, False), (1024, 512, 16, 32, True),
                                                  (1024, 512, 32, 8, True), (1024, 512, 6, 0, True)])
def test_sclc_rtc_kernel(oracle, N, K, L, crc, systematic):
    """The 8-bit list decoder on its plan-specialised kernel (scl_char_rtc_kernel: constants
    and layout as literals): int8 frames of every family and float frames quantised in the
    kernel -- info, ok and the integer path metrics bit-exact against the oracle."""
    from antpolarcodes_amd._native import Plan
    rng = np.random.default_rng(N + L)
    fr = frozen_bits(N, K, 0.0)
    p = Plan(N, L, fr, systematic=systematic, crc=crc, device=0, fixed=True)
    p.specialize()
    assert p.kernel_name() == "scl_char_rtc_kernel" and p.describe()["specialized"] == 1
    for kind in KINDS:
        x = i8_kinds(rng, 48, N, kind)
        gi, gok, gm = p.decode_host_i8(x, want_metrics=True)
        oi, ook, om, _, _ = oracle.sclc_decode(N, L, fr, x, systematic, crc, paths=True)
        assert np.array_equal(gi, oi) and np.array_equal(gok, ook), kind
        assert np.array_equal(gm, om.astype(np.float32)), kind
    llr, _, _ = frames.awgn_frames(N, fr, 256, 1.5, seed=L, crc=crc, systematic=systematic)
    gi, gok, gm = p.decode_host(llr, want_metrics=True)
    oi, ook, om, _, _ = oracle.sclc_decode(N, L, fr, llr, systematic, crc, paths=True)
    assert np.array_equal(gi, oi) and np.array_equal(gok, ook) and np.array_equal(gm, om.astype(np.float32))
