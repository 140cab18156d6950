"""Plan-specialised kernels on the CPU: the generated hiprtc source compiles for
gfx950 (a host-only plan compiles without loading; no GPU needed) and the API refuses plans
that have no specialised kernel."""
import time

import pytest


@pytest.fixture(autouse=True)
def _rtc_cache(tmp_path, monkeypatch):
    monkeypatch.setenv("PCG_RTC_CACHE", str(tmp_path / "rtc"))


def _host_plan(oracle, N, K, L=1, crc=8, systematic=True, fixed=False):
    from antpolarcodes_amd._native import Plan
    return Plan(N, L, oracle.frozen_bits_bb(N, K, 0.0), systematic=systematic, crc=crc, device=-1, fixed=fixed)


def test_specialize_compiles_config2(oracle, tmp_path, monkeypatch):
    p = _host_plan(oracle, 1024, 512)
    assert p.kernel_name().startswith("scq_kernel")
    t = time.time()
    p.specialize()
    first = time.time() - t
    assert p.kernel_name() == "scq_rtc_kernel"
    t = time.time()
    _host_plan(oracle, 1024, 512).specialize()  # same code: the process cache
    assert time.time() - t < max(0.5, first / 4)
    files = list((tmp_path / "rtc").glob("pcg_*.co"))  # and the disk cache, for other processes
    assert len(files) == 1 and files[0].read_bytes()[:4] == b"\x7fELF"


@pytest.mark.parametrize("N,K,crc,systematic", [(64, 32, 0, True), (256, 128, 32, False)])
def test_specialize_compiles_other_codes(oracle, N, K, crc, systematic):
    _host_plan(oracle, N, K, crc=crc, systematic=systematic).specialize()


def test_specialize_compiles_list_plan(oracle):
    """Float list plans: the lane-serial kernel with the plan's layout and constants."""
    p = _host_plan(oracle, 128, 64, L=4, crc=16)
    assert p.kernel_name() == "sclls_kernel<4>"
    p.specialize()
    assert p.kernel_name() == "scl_rtc_kernel"


def test_specialize_unsupported_plans(oracle):
    from antpolarcodes_amd._native import PcgError, PCG_E_UNSUPPORTED
    for kw in ({"fixed": True}, {"fixed": True, "L": 8}):
        with pytest.raises(PcgError) as e:
            _host_plan(oracle, 256, 128, **kw).specialize()
        assert e.value.code == PCG_E_UNSUPPORTED
