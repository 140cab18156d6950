"""GPU parity of the batched SCL kernel against the oracle.

Decoded bytes and the ok flag must be identical; the final ordered path metrics
are compared bit-for-bit too (stricter than the north star's 1e-5 relative).
Oracle semantics: a freshly constructed reference decoder per frame (Q8).
"""
import numpy as np
import pytest

from helpers import LLR_KINDS, llr_kinds

pytestmark = pytest.mark.gpu


def _plan(N, L, frozen, systematic=True, crc=8):
    from antpolarcodes_amd._native import Plan
    return Plan(N, L, frozen, systematic=systematic, crc=crc, device=0)


def _check_scl(oracle, N, L, frozen, llr, systematic=True, crc=8):
    p = _plan(N, L, frozen, systematic, crc)
    gi, gok, gm = p.decode_host(llr, want_metrics=True)
    oi, ook, om, opc, _ = oracle.scl_decode(N, L, frozen, llr, systematic=systematic, crc=crc, paths=True)
    bad = np.nonzero(~(gi == oi).all(axis=1))[0]
    assert bad.size == 0, f"N={N} L={L} K={N-len(frozen)}: info mismatch in frames {bad[:8]}"
    assert np.array_equal(gok, ook)
    mb = np.nonzero(~(gm.view(np.uint32) == om.view(np.uint32)).all(axis=1))[0]
    assert mb.size == 0, f"metrics differ in frames {mb[:8]}: gpu {gm[mb[0]]} oracle {om[mb[0]]}"


@pytest.mark.parametrize("L", [2, 4, 8, 16, 32])
@pytest.mark.parametrize("N", [8, 16, 64, 256, 1024])
def test_scl_bb_codes(oracle, N, L):
    rng = np.random.default_rng(N * 100 + L)
    for K in sorted({N // 4, N // 2, 3 * N // 4}):
        if K < 8:
            continue
        fr = oracle.frozen_bits_bb(N, K, 0.0)
        for kind in LLR_KINDS:
            llr = llr_kinds(rng, 8, N, kind)
            _check_scl(oracle, N, L, fr, llr)


@pytest.mark.parametrize("systematic", [True, False])
@pytest.mark.parametrize("crc", [0, 8, 16, 32])
def test_scl_crc_and_systematic(oracle, systematic, crc):
    from antpolarcodes_amd import frames
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    llr, _, _ = frames.awgn_frames(1024, fr, 96, 1.0, seed=crc + systematic, crc=crc, systematic=systematic)
    _check_scl(oracle, 1024, 8, fr, llr, systematic, crc)


def test_scl_random_frozen_sets(oracle):
    rng = np.random.default_rng(9)
    for t in range(120):
        N = int(2 ** rng.integers(3, 8))
        nf = int(rng.integers(0, N + 1))
        fr = sorted(rng.choice(N, nf, replace=False).tolist())
        L = int(2 ** rng.integers(1, 6))
        llr = llr_kinds(rng, 4, N, LLR_KINDS[t % len(LLR_KINDS)])
        _check_scl(oracle, N, L, fr, llr, crc=0)


def test_scl_awgn_batch_config3(oracle):
    """Config 3 shape: SCL L=8, N=1024 K=512, CRC-8, 2^16 AWGN frames at 2 dB."""
    from antpolarcodes_amd import frames
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    llr, info, _ = frames.awgn_frames(1024, fr, 1 << 16, 2.0, seed=4, crc=8)
    _check_scl(oracle, 1024, 8, fr, llr)


def test_scl_n4096_l32(oracle):
    """Config 5 shape on a small batch: N=4096 K=2048, L=32 (global-scratch stages)."""
    from antpolarcodes_amd import frames
    fr = oracle.frozen_bits_bb(4096, 2048, 0.0)
    llr, _, _ = frames.awgn_frames(4096, fr, 64, 1.5, seed=5, crc=8)
    _check_scl(oracle, 4096, 32, fr, llr)
