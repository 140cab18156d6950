"""The C-ABI boundary on CPU (no GPU needed): the library loads, exports every
symbol include/pcg.h declares, validates arguments like the reference, and
classifies decoder trees exactly as the oracle (and hence the reference) does.
Decoding through a host-only plan must fail loudly (no CPU fallback)."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _native():
    from antpolarcodes_amd import _native
    return _native


def test_library_exports_every_header_symbol():
    nat = _native()
    lib = nat.lib()
    hdr = open(os.path.join(ROOT, "include", "pcg.h")).read()
    names = re.findall(r"^(?:int|void|const char\*)\s+(pcg_\w+)\s*\(", hdr, re.M)
    assert len(names) >= 7
    for n in names:
        assert hasattr(lib, n), n


def test_host_only_plan_and_loud_failure():
    nat = _native()
    fr = list(range(512))
    p = nat.Plan(1024, 1, fr, device=-1)
    d = p.describe()
    assert d["block_length"] == 1024 and d["info_length"] == 512 and d["list_size"] == 1
    with pytest.raises(nat.PcgError) as e:
        p.decode_host(np.zeros((2, 1024), np.float32))
    assert e.value.code == nat.PCG_E_NODEVICE


@pytest.mark.parametrize("args,code", [
    ((1000, 1, [0]), -1),            # N not a power of two
    ((1024, 64, [0]), -1),           # list size above 32
    ((64, 1, [5, 3]), -1),           # frozen bits not ascending
    ((64, 1, [70]), -1),             # frozen index out of range
])
def test_argument_errors(args, code):
    nat = _native()
    with pytest.raises(nat.PcgError) as e:
        nat.Plan(*args, device=-1)
    assert e.value.code == code


def test_crc_size_error():
    nat = _native()
    with pytest.raises(nat.PcgError) as e:
        nat.Plan(64, 4, list(range(32)), crc=7, device=-1)
    assert e.value.code == nat.PCG_E_ARG and "CRC INVALID SIZE" in str(e.value)


def test_fastssc_classification_matches_oracle(oracle):
    """pcg_plan_create(L=1) rejects exactly the frozen sets the reference's
    FastSscAvx::createDecoder rejects with std::invalid_argument, and builds a tree
    with the same node count otherwise."""
    nat = _native()
    rng = np.random.default_rng(3)
    seen_err = seen_ok = 0
    for _ in range(600):
        N = int(2 ** rng.integers(3, 9))
        fr = sorted(rng.choice(N, int(rng.integers(0, N + 1)), replace=False).tolist())
        try:
            t, _ = oracle.sc_tree(N, fr)
        except ValueError:
            with pytest.raises(nat.PcgError) as e:
                nat.Plan(N, 1, fr, device=-1)
            assert e.value.code == nat.PCG_E_FROZEN
            seen_err += 1
            continue
        d = nat.Plan(N, 1, fr, device=-1).describe()
        assert d["node_count"] == len(t)
        seen_ok += 1
    assert seen_err > 20 and seen_ok > 100


def test_config_trees():
    """Node / op counts of the configs' trees (88 Fast-SSC nodes for
    BB(1024,512); 189 SCL nodes)."""
    nat = _native()
    from antpolarcodes_amd.construction import frozen_bits
    fr = frozen_bits(1024, 512, 0.0)
    assert nat.Plan(1024, 1, fr, device=-1).describe()["node_count"] == 88
    assert nat.Plan(1024, 8, fr, device=-1).describe()["node_count"] == 189
    assert nat.Plan(4096, 1, frozen_bits(4096, 2048, 0.0), device=-1).describe()["node_count"] == 265
