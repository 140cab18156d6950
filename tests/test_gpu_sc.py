"""GPU parity of the batched Fast-SSC kernel against the oracle (bit-exact).

The oracle (oracle/polar_oracle.c) is pinned to the reference by tests/test_oracle.py.
"""
import numpy as np
import pytest

from helpers import KERNELS, LLR_KINDS, gpu_plan, llr_kinds, node_cover_sets, reference_digest, sha256

pytestmark = pytest.mark.gpu


def _plan(N, L, frozen, systematic=True, crc=8):
    from antpolarcodes_amd._native import Plan
    return Plan(N, L, frozen, systematic=systematic, crc=crc, device=0)


def _bb(oracle, N, K, dsnr=0.0):
    return oracle.frozen_bits_bb(N, K, dsnr)


def _check_sc(oracle, N, frozen, llr, systematic=True, crc=8):
    p = _plan(N, 1, frozen, systematic, crc)
    gi, gok, _ = p.decode_host(llr)
    oi, ook = oracle.sc_decode(N, frozen, llr, systematic=systematic, crc=crc)
    bad = np.nonzero(~(gi == oi).all(axis=1))[0]
    assert bad.size == 0, f"N={N} K={N-len(frozen)} info mismatch in frames {bad[:8]}"
    assert np.array_equal(gok, ook)


@pytest.mark.parametrize("N", [8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096])
def test_sc_bb_codes(oracle, N):
    rng = np.random.default_rng(N)
    for K in sorted({N // 8, N // 4, N // 2, 3 * N // 4, N - 8}):
        if K < 8:
            continue
        for dsnr in (-2.0, 0.0, 3.0):
            fr = _bb(oracle, N, K, dsnr)
            for kind in LLR_KINDS:
                llr = llr_kinds(rng, 16, N, kind)
                _check_sc(oracle, N, fr, llr)


@pytest.mark.parametrize("systematic", [True, False])
@pytest.mark.parametrize("crc", [0, 8, 16, 32])
def test_sc_crc_and_systematic(oracle, systematic, crc):
    rng = np.random.default_rng(7)
    for N, K in ((256, 128), (1024, 512), (1024, 768)):
        fr = _bb(oracle, N, K)
        llr = llr_kinds(rng, 64, N, "normal")
        _check_sc(oracle, N, fr, llr, systematic, crc)


def test_sc_node_kinds(oracle):
    """Every Fast-SSC leaf kind (incl. the ZeroSpc quirk Q1) at several sizes."""
    rng = np.random.default_rng(11)
    for N, fr in node_cover_sets():
        try:
            oracle.sc_tree(N, fr)
        except ValueError:
            continue  # rejected by the reference too (see test_plan_errors)
        K = N - len(fr)
        for kind in LLR_KINDS:
            llr = llr_kinds(rng, 32, N, kind)
            p = _plan(N, 1, fr, True, 0)
            gi, _, _ = p.decode_host(llr)
            oi, _ = oracle.sc_decode(N, fr, llr, crc=0)
            assert np.array_equal(gi, oi), (N, fr, kind)
            # the packed codeword itself: decode with every bit as info (non-frozen view)
            del p


def test_sc_random_frozen_sets(oracle):
    rng = np.random.default_rng(5)
    tested = 0
    for t in range(400):
        N = int(2 ** rng.integers(3, 9))
        nf = int(rng.integers(0, N + 1))
        fr = sorted(rng.choice(N, nf, replace=False).tolist())
        try:
            oracle.sc_tree(N, fr)
        except ValueError:
            continue
        llr = llr_kinds(rng, 8, N, LLR_KINDS[t % len(LLR_KINDS)])
        _check_sc(oracle, N, fr, llr, crc=0)
        tested += 1
    assert tested > 100


@pytest.mark.parametrize("kernel", KERNELS)
def test_sc_awgn_batch_config2(oracle, kernel):
    """Config 2 shape: N=1024 K=512 BB(0 dB) AWGN Eb/N0 = 2 dB, 2^16 frames, through the
    interpreter kernel and through the plan-specialised kernel the library and bench run."""
    from antpolarcodes_amd import frames
    fr = _bb(oracle, 1024, 512)
    llr, info, _ = frames.awgn_frames(1024, fr, 1 << 16, 2.0, seed=2, crc=8)
    p = gpu_plan(1024, 1, fr, kernel, crc=8)
    gi, gok, _ = p.decode_host(llr)
    oi, ook = oracle.sc_decode(1024, fr, llr, crc=8)
    bad = np.nonzero(~(gi == oi).all(axis=1))[0]
    assert bad.size == 0, f"info mismatch in frames {bad[:8]}"
    assert np.array_equal(gok, ook)
    # ... and the whole batch against the reference itself (tests/golden/make_digests.py)
    d = reference_digest("config2_sc")
    assert sha256(llr) == d["llr"], "frame generator changed: regenerate the digests"
    assert sha256(gi) == d["info"] and sha256(gok) == d["ok"]


def test_sc_device_path_torch(oracle):
    import torch
    from antpolarcodes_amd import frames
    fr = _bb(oracle, 1024, 512)
    llr, _, _ = frames.awgn_frames(1024, fr, 4096, 1.5, seed=3, crc=8)
    p = _plan(1024, 1, fr)
    d_llr = torch.from_numpy(llr).cuda()
    d_info = torch.zeros((4096, 64), dtype=torch.uint8, device="cuda")
    d_ok = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    p.decode_device(d_llr, d_info, d_ok)
    torch.cuda.synchronize()
    oi, ook = oracle.sc_decode(1024, fr, llr)
    assert np.array_equal(d_info.cpu().numpy(), oi)
    assert np.array_equal(d_ok.cpu().numpy(), ook)


@pytest.mark.parametrize("N", [8192, 16384])
def test_sc_large_blocks(oracle, N):
    """Lane-serial Fast-SSC with large per-lane bit rows (64 KB / 128 KB of LDS per wave)."""
    rng = np.random.default_rng(N)
    fr = _bb(oracle, N, N // 2)
    _check_sc(oracle, N, fr, llr_kinds(rng, 70, N, "normal"))


@pytest.mark.parametrize("F", [1, 63, 64, 65, 129, 1000])
def test_sc_batch_edges(oracle, F):
    """Partial last wave of the lane-serial kernel (64 frames per wave)."""
    rng = np.random.default_rng(F)
    fr = _bb(oracle, 1024, 512)
    _check_sc(oracle, 1024, fr, llr_kinds(rng, F, 1024, "zeros"))


def test_sc_wave_kernel_switch(oracle, monkeypatch):
    """The one-codeword-per-wave kernel (dev switch PCG_SC_KERNEL=wave) stays bit-exact."""
    monkeypatch.setenv("PCG_SC_KERNEL", "wave")
    rng = np.random.default_rng(3)
    for N, K in ((64, 32), (1024, 512)):
        fr = _bb(oracle, N, K)
        _check_sc(oracle, N, fr, llr_kinds(rng, 100, N, "ints"))
