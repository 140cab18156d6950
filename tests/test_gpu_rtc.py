"""GPU parity of the plan-specialised Fast-SSC kernel (rtc.cpp, pcg_plan_specialize) against
the oracle, bit-exact: the same device code as the interpreter kernel compiled with the plan's
schedule as literals, so every leaf kind, stage size, detector and the non-systematic
re-encode must give the interpreter's (= the oracle's) bits."""
import numpy as np
import pytest

from helpers import LLR_KINDS, llr_kinds, node_cover_sets

pytestmark = pytest.mark.gpu


def _spec_plan(N, frozen, systematic=True, crc=8):
    from antpolarcodes_amd._native import Plan
    p = Plan(N, 1, frozen, systematic=systematic, crc=crc, device=0)
    p.specialize()
    assert p.describe()["specialized"] == 1
    assert p.kernel_name() == "scq_rtc_kernel"
    return p


def _check(oracle, p, N, frozen, llr, systematic=True, crc=8):
    gi, gok, _ = p.decode_host(llr)
    oi, ook = oracle.sc_decode(N, frozen, llr, systematic=systematic, crc=crc)
    bad = np.nonzero(~(gi == oi).all(axis=1))[0]
    assert bad.size == 0, f"N={N} K={N - len(frozen)} info mismatch in frames {bad[:8]}"
    assert np.array_equal(gok, ook)


@pytest.mark.parametrize("N", [8, 32, 128, 512, 1024])  # (N >= 2048: minutes of compile per code)
def test_rtc_bb_codes(oracle, N):
    rng = np.random.default_rng(100 + N)
    K = max(8, N // 2)
    fr = oracle.frozen_bits_bb(N, K, 0.0)
    p = _spec_plan(N, fr)
    for kind in LLR_KINDS:
        _check(oracle, p, N, fr, llr_kinds(rng, 96, N, kind))


@pytest.mark.parametrize("systematic", [True, False])
@pytest.mark.parametrize("crc", [0, 16, 32])
def test_rtc_crc_and_systematic(oracle, systematic, crc):
    rng = np.random.default_rng(5)
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    p = _spec_plan(1024, fr, systematic, crc)
    _check(oracle, p, 1024, fr, llr_kinds(rng, 256, 1024, "normal"), systematic, crc)


def test_rtc_node_kinds(oracle):
    """Every Fast-SSC leaf kind (incl. the ZeroSpc quirk Q1) through specialised kernels."""
    rng = np.random.default_rng(13)
    done = 0
    for N, fr in node_cover_sets():
        try:
            oracle.sc_tree(N, fr)
        except ValueError:
            continue
        p = _spec_plan(N, fr)
        for kind in ("normal", "ints", "zeros"):
            _check(oracle, p, N, fr, llr_kinds(rng, 64, N, kind))
        done += 1
    assert done > 0


def test_rtc_auto_large_batch_config2(oracle, monkeypatch):
    """Config 2 (N=1024, K=512, CRC-8): a batch of >= 8192 frames starts the plan's
    specialisation in the background (the interpreter kernel decodes meanwhile); once it is
    loaded the same batch decodes through it.  Both match the oracle."""
    import torch
    from antpolarcodes_amd import frames
    from antpolarcodes_amd._native import Plan
    monkeypatch.setenv("PCG_RTC", "2")  # the library default (tests/conftest.py turns it off)
    N, K = 1024, 512
    fr = oracle.frozen_bits_bb(N, K, 0.0)
    llr, _, _ = frames.awgn_frames(N, fr, 8192, 2.0, seed=21, crc=8)
    p = Plan(N, 1, fr, crc=8, device=0)
    assert p.describe()["specialized"] == 0
    x = torch.from_numpy(np.ascontiguousarray(llr, dtype=np.float32)).cuda()
    oi, ook = oracle.sc_decode(N, fr, llr, crc=8)
    for rnd in range(2):
        info = torch.zeros((x.shape[0], p.kb), dtype=torch.uint8, device="cuda")
        ok = torch.zeros(x.shape[0], dtype=torch.uint8, device="cuda")
        p.decode_device(x, info, ok)
        torch.cuda.synchronize()
        assert np.array_equal(info.cpu().numpy(), oi), f"round {rnd}"
        assert np.array_equal(ok.cpu().numpy(), ook), f"round {rnd}"
        p.specialize()  # waits for the background compile
        assert p.describe()["specialized"] == 1
        assert p.kernel_name() == "scq_rtc_kernel"


@pytest.mark.parametrize("N,K,L,crc,systematic,kind", [
    (256, 128, 4, 16, True, "BB"), (1024, 512, 8, 8, True, "BB"), (512, 256, 6, 32, False, "BB"),
    (4096, 2048, 32, 8, True, "BB"), (1024, 512, 12, 8, True, "BB"), (1024, 512, 8, 0, True, "BB"),
    (1024, 512, 8, 11, True, "5G"), (1024, 512, 8, 0, True, "5G")])
def test_rtc_list_plans(oracle, N, K, L, crc, systematic, kind):
    """Specialised list plans (scl_rtc_kernel: the lane-serial kernel with the plan's layout and
    constants as literals): info, ok and the ordered path metrics bit-exact -- BB codes, a list
    size that is not a power of two, no detector, and config 4's 5G reliability-list code with
    CRC-11 and with the Dummy detector."""
    from antpolarcodes_amd._native import Plan
    from antpolarcodes_amd.construction import frozen_bits
    rng = np.random.default_rng(N + L)
    fr = oracle.frozen_bits_bb(N, K, 0.0) if kind == "BB" else frozen_bits(N, K, 0.0, "5G")
    p = Plan(N, L, fr, systematic=systematic, crc=crc, device=0)
    p.specialize()
    assert p.describe()["specialized"] == 1 and p.kernel_name() == "scl_rtc_kernel"
    for kind in LLR_KINDS if N <= 1024 else ("normal", "ints"):
        llr = llr_kinds(rng, 64 if N <= 1024 else 16, N, kind)
        gi, gok, gm = p.decode_host(llr, want_metrics=True)
        oi, ook, om, _, _ = oracle.scl_decode(N, L, fr, llr, systematic=systematic, crc=crc, paths=True)
        assert np.array_equal(gi, oi), kind
        assert np.array_equal(gok, ook), kind
        assert np.array_equal(gm.view(np.uint32), om.view(np.uint32)), kind


def test_rtc_list_random_frozen_sets(oracle):
    """The specialised list kernel on random frozen sets (the catalogue's random list codes,
    antpolarcodes_amd/rtc_codes.py: N = 32 .. 256, L = 3, 8, 32, any number of frozen
    positions): the reference's SCL classifier (scl_avx_float.cpp:624-651) meets R0 / R1 / Rep /
    SPC nodes and size-8 subtrees of every shape, and the layout (recomputed top stages, LDS /
    slab split) varies with the tree.  Info, ok and ordered path metrics bit-exact against the
    oracle, on every LLR family."""
    from antpolarcodes_amd._native import Plan
    from antpolarcodes_amd.rtc_codes import random_list_codes
    rng = np.random.default_rng(404)
    for N, L, fr in random_list_codes():
        p = Plan(N, L, fr, crc=0, device=0)
        p.specialize()
        assert p.describe()["specialized"] == 1 and p.kernel_name() == "scl_rtc_kernel"
        for kind in LLR_KINDS:
            llr = llr_kinds(rng, 64, N, kind)
            gi, gok, gm = p.decode_host(llr, want_metrics=True)
            oi, ook, om, _, _ = oracle.scl_decode(N, L, fr, llr, crc=0, paths=True)
            assert np.array_equal(gi, oi), (N, L, len(fr), kind)
            assert np.array_equal(gok, ook), (N, L, len(fr), kind)
            assert np.array_equal(gm.view(np.uint32), om.view(np.uint32)), (N, L, len(fr), kind)


def test_rtc_default_mode_list_plan(oracle, monkeypatch):
    """The library default (PCG_RTC=2) on list plans: a code whose specialised kernel is in the
    shipped cache (config 3) runs it from its first decode; a code that is not (N=1024 K=600
    L=4) decodes on the interpreter while its compile runs in the background (started by a
    batch of >= 8192 frames) and switches once it is loaded.  Every output matches the oracle."""
    import torch
    from antpolarcodes_amd import frames
    from antpolarcodes_amd._native import Plan
    monkeypatch.setenv("PCG_RTC", "2")
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    llr, _, _ = frames.awgn_frames(1024, fr, 64, 1.5, seed=3, crc=8)
    p = Plan(1024, 8, fr, crc=8, device=0)
    gi, gok, gm = p.decode_host(llr, want_metrics=True)
    assert p.kernel_name() == "scl_rtc_kernel"
    oi, ook, om, _, _ = oracle.scl_decode(1024, 8, fr, llr, crc=8, paths=True)
    assert np.array_equal(gi, oi) and np.array_equal(gok, ook)
    assert np.array_equal(gm.view(np.uint32), om.view(np.uint32))
    fr = oracle.frozen_bits_bb(1024, 600, 0.0)
    llr, _, _ = frames.awgn_frames(1024, fr, 8192, 2.5, seed=4, crc=16)
    x = torch.from_numpy(llr).cuda()
    oi, ook = oracle.scl_decode(1024, 4, fr, llr[:1024], crc=16)
    q = Plan(1024, 4, fr, crc=16, device=0)
    for rnd in range(2):
        info = torch.zeros((8192, q.kb), dtype=torch.uint8, device="cuda")
        ok = torch.zeros(8192, dtype=torch.uint8, device="cuda")
        q.decode_device(x, info, ok)
        torch.cuda.synchronize()
        assert np.array_equal(info[:1024].cpu().numpy(), oi), q.kernel_name()
        assert np.array_equal(ok[:1024].cpu().numpy(), ook), q.kernel_name()
        q.specialize()  # waits for the background compile
        assert q.kernel_name() == "scl_rtc_kernel"
