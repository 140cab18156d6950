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


def test_scl32_config5_shard(oracle):
    """Config 5 at its per-GPU shard size: 2^17 frames of N=4096 K=2048 SCL-32 (one of the
    8 contiguous shards of the 2^20-frame batch), frames made on the device; a strided subset
    is checked against the oracle (info, ok and path metrics bit for bit), every frame against
    the transmitted information where the CRC passed."""
    import torch
    from antpolarcodes_amd._native import Encoder, Plan, bpsk_awgn_device, random_info_device
    N, K, L, F = 4096, 2048, 32, 1 << 17
    fr = oracle.frozen_bits_bb(N, K, 0.0)
    info = torch.empty((F, K // 8), dtype=torch.uint8, device="cuda:0")
    code = torch.empty((F, N // 8), dtype=torch.uint8, device="cuda:0")
    llr = torch.empty((F, N), dtype=torch.float32, device="cuda:0")
    random_info_device(info, K, seed=17)
    Encoder(N, fr, crc=8, device=0).encode_device(info, code)
    esn0 = 10 ** 0.15 * K / N  # Eb/N0 1.5 dB
    bpsk_awgn_device(code, N, float(1 / np.sqrt(2 * esn0)), 23, llr)
    del code
    p = Plan(N, L, fr, crc=8, device=0)
    out = torch.empty_like(info)
    ok = torch.empty(F, dtype=torch.uint8, device="cuda:0")
    met = torch.empty((F, L), dtype=torch.float32, device="cuda:0")
    p.decode_device(llr, out, ok, met)
    torch.cuda.synchronize()
    okh = ok.cpu().numpy().astype(bool)
    good = (out == info).all(dim=1).cpu().numpy()
    assert okh.mean() > 0.9 and good[okh].mean() > 0.999
    idx = np.arange(0, F, F // 48)
    sub = llr[idx].cpu().numpy()
    oi, ook, om, _, _ = oracle.scl_decode(N, L, fr, sub, crc=8, paths=True)
    assert np.array_equal(out[idx].cpu().numpy(), oi)
    assert np.array_equal(okh[idx].astype(np.uint8), ook)
    assert np.array_equal(met[idx].cpu().numpy().view(np.uint32), om.view(np.uint32))


@pytest.mark.parametrize("fuse", ["0", "1", "2", "3", "5", "7"])
@pytest.mark.parametrize("lds_kb", ["8", "24"])
def test_scl_fused_and_shared_fg(oracle, monkeypatch, fuse, lds_kb):
    """The F/G + child-F fusion (bit 0) and idle-lane sharing (bit 1) of sclls_kernel,
    each on and off, with a small LDS budget that puts more stages in the global slab
    (more fused pairs).  PCG_SCL_FUSE / PCG_SCL_LDS_KB are read at plan creation."""
    from antpolarcodes_amd import frames
    monkeypatch.setenv("PCG_SCL_FUSE", fuse)
    monkeypatch.setenv("PCG_SCL_LDS_KB", lds_kb)
    rng = np.random.default_rng(int(fuse) * 10 + int(lds_kb))
    for N, L in [(256, 4), (1024, 8), (2048, 16)]:
        fr = oracle.frozen_bits_bb(N, N // 2, 0.0)
        llr, _, _ = frames.awgn_frames(N, fr, 48, 1.5, seed=int(rng.integers(1 << 30)), crc=8)
        _check_scl(oracle, N, L, fr, llr)


@pytest.mark.parametrize("lp", ["16", "32"])
@pytest.mark.parametrize("fuse", ["3", "7"])
def test_scl_wide_lane_groups(oracle, monkeypatch, lp, fuse):
    """Lists decoded in lane groups wider than the list (PCG_SCL_LP; the adaptive
    decoder's SCL stage runs this way): the lanes beyond the list share every F/G.
    Bit-exact vs the oracle over the tie-heavy LLR families and AWGN frames."""
    from antpolarcodes_amd import frames
    monkeypatch.setenv("PCG_SCL_LP", lp)
    monkeypatch.setenv("PCG_SCL_FUSE", fuse)
    rng = np.random.default_rng(int(lp) + int(fuse))
    for N, L in [(64, 2), (256, 4), (1024, 8), (1024, 16)]:
        if L >= int(lp):
            continue
        fr = oracle.frozen_bits_bb(N, N // 2, 0.0)
        llr, _, _ = frames.awgn_frames(N, fr, 64, 1.0, seed=int(rng.integers(1 << 30)), crc=8)
        _check_scl(oracle, N, L, fr, llr)
        for kind in LLR_KINDS:
            _check_scl(oracle, N, L, fr, llr_kinds(rng, 8, N, kind))
