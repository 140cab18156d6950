"""The 8-bit ("char") decoders on CPU (no GPU): C-ABI plans classify the reference's
FastSscFip / SclFip trees exactly as the pinned oracle, the pypolar / C++ factories map
"char" as decoder.cpp:26-87 does, and decoding without a GPU fails loudly."""
import numpy as np
import pytest

from antpolarcodes_amd.construction import frozen_bits


def _nat():
    from antpolarcodes_amd import _native
    return _native


def test_char_plan_node_counts_match_oracle(oracle):
    nat = _nat()
    rng = np.random.default_rng(5)
    for _ in range(300):
        N = int(2 ** rng.integers(3, 11))
        K = int(rng.integers(0, N + 1))
        fr = sorted(rng.choice(N, N - K, replace=False).tolist()) if rng.random() < 0.5 else frozen_bits(N, max(K, 1), 0.0)
        for L in (1, 8):
            t, _ = oracle.char_tree(N, fr, L=L)
            d = nat.Plan(N, L, fr, fixed=True, device=-1).describe()
            assert d["node_count"] == len(t), (N, K, L)


def test_char_config_trees(oracle):
    nat = _nat()
    fr = frozen_bits(1024, 512, 0.0)
    for L in (1, 8, 32):
        t, _ = oracle.char_tree(1024, fr, L=L)
        assert nat.Plan(1024, L, fr, fixed=True, device=-1).describe()["node_count"] == len(t)


def test_char_plan_host_only_fails_loudly():
    nat = _nat()
    p = nat.Plan(256, 8, frozen_bits(256, 128, 0.0), fixed=True, device=-1)
    with pytest.raises(nat.PcgError) as e:
        p.decode_host_i8(np.zeros((2, 256), np.int8))
    assert e.value.code == nat.PCG_E_NODEVICE
    with pytest.raises(nat.PcgError) as e:
        p.decode_host(np.zeros((2, 256), np.float32))
    assert e.value.code == nat.PCG_E_NODEVICE


def test_int8_on_float_plan_is_an_argument_error():
    nat = _nat()
    p = nat.Plan(256, 1, frozen_bits(256, 128, 0.0), device=-1)
    with pytest.raises(nat.PcgError) as e:
        p.decode_host_i8(np.zeros((2, 256), np.int8))
    assert e.value.code == nat.PCG_E_ARG


def test_char_layout_fits_lds():
    nat = _nat()
    for N, L in ((1024, 8), (4096, 32), (256, 2), (8, 4), (1024, 32)):
        d = nat.Plan(N, L, frozen_bits(N, N // 2, 0.0), fixed=True, device=-1).describe()
        assert 0 < d["lds_bytes"] <= 160 * 1024


def test_pypolar_char_factory_without_gpu():
    """create(..., "char") builds FastSscFipChar / SclFipChar (decoder.cpp:37-38, 62-80); the
    plan is validated at construction (host-only), decoding needs the GPU."""
    from antpolarcodes_amd import pypolar
    fr = frozen_bits(256, 128, 0.0)
    for L in (1, 4):
        dec = pypolar.PolarDecoder(256, L, fr, "char")
        assert dec.isFixedPoint() and dec.listSize() == L
        assert dec.getErrorDetectionMode() == "CRC-8"
    assert not pypolar.PolarDecoder(256, 4, fr, "float").isFixedPoint()
    assert not pypolar.PolarDecoder(256, 1, fr, "mixed").isFixedPoint()  # L < 2: float Fast-SSC
    with pytest.raises(Exception):
        pypolar.PolarDecoder(256, 4, fr, "scan")
    with pytest.raises(Exception, match="Unknown PolarDecoder type"):
        pypolar.PolarDecoder(256, 4, fr, "bogus")


def test_adaptive_char_plan_host_only():
    """AdaptiveChar (adaptive_char.cpp:14-45) builds both 8-bit stages; L < 2 is plain
    FastSscFipChar (makeDecoder's listSize-1 branch)."""
    nat = _nat()
    fr = frozen_bits(256, 128, 0.0)
    d = nat.Plan(256, 8, fr, adaptive=True, fixed=True, device=-1).describe()
    assert d["list_size"] == 8
    assert nat.Plan(256, 1, fr, adaptive=True, fixed=True, device=-1).describe()["list_size"] == 1
