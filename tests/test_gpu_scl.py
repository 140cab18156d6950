"""GPU parity of the batched SCL kernel against the oracle.

Decoded bytes and the ok flag must be identical; the final ordered path metrics
are compared bit-for-bit too (stricter than the north star's 1e-5 relative).
Oracle semantics: a freshly constructed reference decoder per frame (Q8).
"""
import numpy as np
import pytest

from helpers import KERNELS, LLR_KINDS, gpu_plan, llr_kinds, reference_digest, sha256

pytestmark = pytest.mark.gpu

_ORACLE = {}  # oracle outputs of the large batches, shared by the kernel parametrizations


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


@pytest.mark.parametrize("virt", [1, 2, 3])
@pytest.mark.parametrize("L", [2, 8, 16, 32])
def test_scl_recomputed_top_stages(oracle, monkeypatch, virt, L):
    """The top LLR stages recomputed from the channel where read (sclls layout):
    virt 1 = the root's children, 2 = also its grandchildren (the codeword's quarters),
    3 = also the eighths (LP >= 16); the deepest allowed by the leaves is the default.  All
    against the oracle, systematic and not, with the deepest nodes' F/G fused (N = 2048) and
    unfused (leaf children, BB(1024, 512))."""
    from antpolarcodes_amd import frames
    monkeypatch.setenv("PCG_SCL_VIRT", str(virt))
    rng = np.random.default_rng(31 * L + virt)
    for N, K in ((1024, 512), (2048, 1024), (512, 256)):
        fr = oracle.frozen_bits_bb(N, K, 0.0)
        p = _plan(N, L, fr)
        got = p.describe()["recomputed_stages"]
        assert 1 <= got <= virt, got
        if N == 1024 and virt >= 2:
            assert got == 2, got  # BB(1024, 512) has leaves at stage 7: the quarters, not the eighths
        if N == 2048 and virt == 3 and L >= 16:
            assert got == 3, got
        for kind in LLR_KINDS[:4]:
            _check_scl(oracle, N, L, fr, llr_kinds(rng, 4, N, kind))
        llr, _, _ = frames.awgn_frames(N, fr, 64, 1.5, seed=N + L, crc=8, systematic=False)
        _check_scl(oracle, N, L, fr, llr, systematic=False)


@pytest.mark.parametrize("kernel", KERNELS)
def test_scl_awgn_batch_config3(oracle, kernel):
    """Config 3 shape: SCL L=8, N=1024 K=512, CRC-8, 2^16 AWGN frames at 2 dB, through the
    interpreter and through the plan-specialised kernel (scl_rtc_kernel) the bench runs: every
    frame's info, ok and ordered path metrics against the oracle and the reference's digest."""
    from antpolarcodes_amd import frames
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    llr, info, _ = frames.awgn_frames(1024, fr, 1 << 16, 2.0, seed=4, crc=8)
    p = gpu_plan(1024, 8, fr, kernel, crc=8)
    gi, gok, gm = p.decode_host(llr, want_metrics=True)
    if "config3" not in _ORACLE:  # (one oracle run serves both kernels)
        _ORACLE["config3"] = oracle.scl_decode(1024, 8, fr, llr, crc=8, paths=True)
    oi, ook, om, _, _ = _ORACLE["config3"]
    bad = np.nonzero(~(gi == oi).all(axis=1))[0]
    assert bad.size == 0, f"info mismatch in frames {bad[:8]}"
    assert np.array_equal(gok, ook)
    assert np.array_equal(gm.view(np.uint32), om.view(np.uint32))
    _check_digest("config3_scl8", llr, gi, gok, gm)


def _check_digest(name, llr, gi, gok, gm):
    """The whole batch against the reference itself (tests/golden/make_digests.py)."""
    d = reference_digest(name)
    assert sha256(llr) == d["llr"], "frame generator changed: regenerate the digests"
    assert sha256(gi) == d["info"] and sha256(gok) == d["ok"]
    assert sha256(gm) == d["metrics"]


@pytest.mark.parametrize("kernel", KERNELS)
def test_scl32_reference_digest(oracle, kernel):
    """Config 5's code (N=4096 K=2048 L=32, CRC-8) on 4096 host frames: info, ok and the
    ordered path metrics of every frame equal the reference's (by digest), on both kernels."""
    from antpolarcodes_amd import frames
    fr = oracle.frozen_bits_bb(4096, 2048, 0.0)
    llr, _, _ = frames.awgn_frames(4096, fr, 4096, 1.5, seed=55, crc=8)
    gi, gok, gm = gpu_plan(4096, 32, fr, kernel, crc=8).decode_host(llr, want_metrics=True)
    _check_digest("config5_scl32", llr, gi, gok, gm)


def test_scl_n4096_l32(oracle):
    """Config 5 shape on a small batch: N=4096 K=2048, L=32 (global-scratch stages)."""
    from antpolarcodes_amd import frames
    fr = oracle.frozen_bits_bb(4096, 2048, 0.0)
    llr, _, _ = frames.awgn_frames(4096, fr, 64, 1.5, seed=5, crc=8)
    _check_scl(oracle, 4096, 32, fr, llr)


@pytest.mark.parametrize("kernel", KERNELS)
def test_scl32_config5_shard(oracle, kernel):
    """Config 5 at its per-GPU shard size: 2^17 frames of N=4096 K=2048 SCL-32 (one of the
    8 contiguous shards of the 2^20-frame batch), frames made on the device; a strided subset
    is checked against the oracle (info, ok and path metrics bit for bit), every frame against
    the transmitted information where the CRC passed."""
    import torch
    from antpolarcodes_amd._native import Encoder, bpsk_awgn_device, random_info_device
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
    p = gpu_plan(N, L, fr, kernel, crc=8)
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


@pytest.mark.parametrize("L", [3, 5, 6, 7, 12, 24])
def test_scl_non_power_of_two_lists(oracle, L):
    """List sizes that are not powers of two (the reference accepts any L; the kernel runs
    them in a group of list_pow2(L) lanes with the spare lanes idle): info, ok and the
    ordered metrics bit for bit over every LLR family and AWGN frames, N <= 1024."""
    from antpolarcodes_amd import frames
    rng = np.random.default_rng(700 + L)
    for N in (16, 64, 256, 1024):
        for K in sorted({N // 4, N // 2, 3 * N // 4}):
            fr = oracle.frozen_bits_bb(N, K, 0.0)
            for kind in LLR_KINDS:
                _check_scl(oracle, N, L, fr, llr_kinds(rng, 6, N, kind), crc=0)
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    llr, _, _ = frames.awgn_frames(1024, fr, 256, 1.0, seed=L, crc=8)
    _check_scl(oracle, 1024, L, fr, llr)


def test_plan_across_streams_and_destroy(oracle):
    """One plan decoding on two non-blocking torch streams back to back (no host sync in
    between), then again after a rejected call, then destroyed right after an asynchronous
    decode: every launch is ordered after the plan's previous one (its scratch, work-queue
    counter and staging are shared), so every output matches the oracle."""
    import torch
    from antpolarcodes_amd import frames
    from antpolarcodes_amd._native import Plan
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    F = 4096
    llr_a, _, _ = frames.awgn_frames(1024, fr, F, 1.0, seed=31, crc=8)
    llr_b, _, _ = frames.awgn_frames(1024, fr, F, 1.5, seed=32, crc=8)
    ea, oka, ma, _, _ = oracle.scl_decode(1024, 8, fr, llr_a[:512], crc=8, paths=True)
    eb, okb, mb, _, _ = oracle.scl_decode(1024, 8, fr, llr_b[:512], crc=8, paths=True)
    dev = torch.device("cuda:0")
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    p = Plan(1024, 8, fr, crc=8, device=0)
    xa, xb = torch.from_numpy(llr_a).to(dev), torch.from_numpy(llr_b).to(dev)
    torch.cuda.synchronize()
    outs = []
    for rnd in range(2):
        ia = torch.empty((F, 64), dtype=torch.uint8, device=dev)
        ib = torch.empty_like(ia)
        ka = torch.empty(F, dtype=torch.uint8, device=dev)
        kb = torch.empty_like(ka)
        mta = torch.empty((F, 8), dtype=torch.float32, device=dev)
        mtb = torch.empty_like(mta)
        xa.record_stream(s1)
        xb.record_stream(s2)
        p.decode_device(xa, ia, ka, mta, stream=s1.cuda_stream)
        p.decode_device(xb, ib, kb, mtb, stream=s2.cuda_stream)
        outs.append((ia, ka, mta, ib, kb, mtb))
        if rnd == 0:  # a rejected call (wrong info shape) leaves the plan usable
            with pytest.raises(ValueError):
                p.decode_device(xa, torch.empty((F, 63), dtype=torch.uint8, device=dev), stream=s1.cuda_stream)
            with pytest.raises(ValueError):  # a frame of the wrong length never reaches the GPU
                p.decode_host(np.zeros((1, 1000), np.float32))
    torch.cuda.synchronize()
    for ia, ka, mta, ib, kb, mtb in outs:
        assert np.array_equal(ia[:512].cpu().numpy(), ea) and np.array_equal(ka[:512].cpu().numpy(), oka)
        assert np.array_equal(ib[:512].cpu().numpy(), eb) and np.array_equal(kb[:512].cpu().numpy(), okb)
        assert np.array_equal(mta[:512].cpu().numpy().view(np.uint32), ma.view(np.uint32))
        assert np.array_equal(mtb[:512].cpu().numpy().view(np.uint32), mb.view(np.uint32))
        # the two streams' results are also consistent over the whole batch
        assert torch.equal(ia, outs[0][0]) and torch.equal(ib, outs[0][3])
    # destroy right after an asynchronous decode on a non-blocking stream: destroy waits
    last = torch.empty((F, 64), dtype=torch.uint8, device=dev)
    lk = torch.empty(F, dtype=torch.uint8, device=dev)
    p.decode_device(xa, last, lk, stream=s2.cuda_stream)
    p.close()
    p2 = Plan(1024, 8, fr, crc=8, device=0)  # a new plan reuses the freed memory
    junk = torch.empty((F, 64), dtype=torch.uint8, device=dev)
    p2.decode_device(xb, junk, stream=s1.cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(last[:512].cpu().numpy(), ea) and np.array_equal(lk[:512].cpu().numpy(), oka)
    assert np.array_equal(junk[:512].cpu().numpy(), eb)
    p2.close()
