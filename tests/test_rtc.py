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


def test_specialize_compiles_a_new_code(oracle, tmp_path, monkeypatch):
    """A code the shipped cache does not hold: compiled once, then from the process cache and,
    for other processes, the user cache."""
    p = _host_plan(oracle, 512, 200)
    assert p.kernel_name().startswith("scq_kernel")
    t = time.time()
    p.specialize()
    first = time.time() - t
    assert p.kernel_name() == "scq_rtc_kernel"
    t = time.time()
    _host_plan(oracle, 512, 200).specialize()  # same code: the process cache
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


def test_specialize_8bit_and_unsupported_plans(oracle, monkeypatch):
    """The 8-bit decoders specialise too (their constants and layout as literals:
    sccs_rtc_kernel / scl_char_rtc_kernel for int8 LLRs, *_f32 for float ones); a plan built
    with the op profiler has no specialised kernel."""
    from antpolarcodes_amd._native import PcgError, PCG_E_UNSUPPORTED
    p = _host_plan(oracle, 256, 128, fixed=True)
    assert p.kernel_name() == "sccs_kernel"
    p.specialize()
    assert p.kernel_name() == "sccs_rtc_kernel"
    p = _host_plan(oracle, 256, 128, L=8, fixed=True)
    assert p.kernel_name() == "scl_char_kernel<8>"
    p.specialize()
    assert p.kernel_name() == "scl_char_rtc_kernel"
    monkeypatch.setenv("PCG_OPPROF", "1")
    with pytest.raises(PcgError) as e:
        _host_plan(oracle, 256, 128).specialize()
    assert e.value.code == PCG_E_UNSUPPORTED


def _run(code, env_extra, timeout=600):
    """A fresh process (its own process cache) running `code` with the repo on sys.path."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if not k.startswith("PCG_")}
    env.update(env_extra)
    pre = ("import sys, time, ctypes; sys.path.insert(0, %r)\n"
           "from antpolarcodes_amd._native import Plan, lib\n"
           "from antpolarcodes_amd.construction import frozen_bits\n" % root)
    r = subprocess.run([sys.executable, "-c", pre + code], env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


# a code no shipped cache holds (antpolarcodes_amd/rtc_warm.py): compiles in a few seconds
_SMALL = "p = Plan(16, 1, frozen_bits(16, 8, 0.0, 'BB'), systematic=False, crc=0, device=-1)\n"


def test_corrupt_or_foreign_cache_files_are_recompiled(tmp_path):
    """A torn, truncated or foreign file under a cache name is never loaded: the code is
    compiled again and the file rewritten whole (trailer: magic, length, checksum)."""
    env = {"PCG_RTC_CACHE": str(tmp_path)}
    _run(_SMALL + "p.specialize()\n", env)
    files = list(tmp_path.glob("pcg_*.co"))
    assert len(files) == 1
    good = files[0].read_bytes()
    assert good[:4] == b"\x7fELF" and good[-24:-16] == b"PCGRTC01"
    for bad in (good[:-30], good[:len(good) // 2], b"\x7fELF" + b"\0" * 4096, good[:-1] + bytes([good[-1] ^ 1])):
        files[0].write_bytes(bad)
        out = _run(_SMALL + "p.specialize()\nprint('compiles', lib().pcg_dev_rtc_compiles())\n", env)
        assert "compiles 1" in out  # recompiled, not loaded
        assert files[0].read_bytes() == good
    out = _run(_SMALL + "p.specialize()\nprint('compiles', lib().pcg_dev_rtc_compiles())\n", env)
    assert "compiles 0" in out  # the valid file is used
    assert not list(tmp_path.glob(".pcg_*"))  # no temp files left behind


def test_destroy_during_compile_and_shared_compile(tmp_path):
    """Two plans of one code share one hiprtc compile; destroying a plan whose compile is
    still running returns at once (the detached compile finishes on its own), and the process
    exits cleanly after it."""
    code = (_SMALL + "q = Plan(16, 1, frozen_bits(16, 8, 0.0, 'BB'), systematic=False, crc=0, device=-1)\n"
            "p.specialize(wait=False); q.specialize(wait=False)\n"
            "t = time.time(); p.close(); dt = time.time() - t\n"
            "assert dt < 0.5, dt\n"
            "q.specialize()\n"
            "assert q.kernel_name() == 'scq_rtc_kernel'\n"
            "print('compiles', lib().pcg_dev_rtc_compiles())\n"
            "r = Plan(16, 1, frozen_bits(16, 8, 0.0, 'BB'), systematic=False, crc=0, device=-1)\n"
            "r.specialize(wait=False); del r\n")  # a finished job: nothing left to wait for at exit
    out = _run(code, {"PCG_RTC_CACHE": str(tmp_path)})
    assert "compiles 1" in out
    # exit while a compile of another code is still running: the process waits for it
    code = ("p = Plan(32, 1, frozen_bits(32, 16, 0.0, 'BB'), systematic=False, crc=16, device=-1)\n"
            "p.specialize(wait=False); p.close()\n")
    _run(code, {"PCG_RTC_CACHE": str(tmp_path / "b")})
    assert len(list((tmp_path / "b").glob("pcg_*.co"))) == 1


# catalogue entries whose frozen sets the Fast-SSC classifier rejects (PCG_E_FROZEN, as the
# reference's createDecoder throws): listed so that a code that stops constructing fails the test
_REJECTED_CATALOGUE_ENTRIES = 2


def test_shipped_cache_holds_the_catalogue():
    """The build (antpolarcodes_amd/rtc_warm.py) ships the specialised kernels of the whole
    catalogue (antpolarcodes_amd/rtc_codes.py: the benchmark configurations and the validation
    codes the GPU tests use) next to the library, with the hiprtc version they were built by:
    every code that constructs has its file there, under the name a lookup reads, and loads
    without any compile."""
    import os
    from antpolarcodes_amd import rtc_warm
    from antpolarcodes_amd.rtc_codes import codes
    assert os.path.isfile(os.path.join(rtc_warm.CACHE, "HIPRTC_VERSION"))
    code = ("from antpolarcodes_amd.rtc_codes import codes\n"
            "from antpolarcodes_amd._native import PcgError\n"
            "from antpolarcodes_amd import rtc_warm\n"
            "n, rej, missing = 0, 0, []\n"
            "b = ctypes.create_string_buffer(256)\n"
            "for N, L, (kind, arg), crc, sysm, *ad in codes():\n"
            "    fr = list(arg) if kind == 'set' else frozen_bits(N, arg, 0.0, kind)\n"
            "    try:\n"
            "        p = Plan(N, L, fr, systematic=sysm, crc=crc, device=-1,\n"
            "                 adaptive=ad[:1] in (['adaptive'], ['adaptive_char']),\n"
            "                 fixed=ad[:1] in (['char'], ['adaptive_char']))\n"
            "    except PcgError:\n"
            "        rej += 1\n"
            "        continue\n"
            "    assert lib().pcg_dev_rtc_lookup_name(p._h, rtc_warm.CACHE.encode(), b, 256) == 0\n"
            "    missing += [f for f in b.value.decode().split() if not os.path.isfile(os.path.join(rtc_warm.CACHE, f))]\n"
            "    p.specialize()\n"
            "    n += 1\n"
            "print('codes', n, 'rejected', rej, 'missing', missing, 'compiles', lib().pcg_dev_rtc_compiles())\n")
    out = _run("import os\n" + code, {"PCG_RTC_CACHE": "0"}, timeout=300)
    assert "compiles 0" in out, out
    assert "missing []" in out, out
    assert "codes %d rejected %d " % (len(codes()) - _REJECTED_CATALOGUE_ENTRIES, _REJECTED_CATALOGUE_ENTRIES) in out, out


def test_warm_names_follow_the_cache_version(tmp_path):
    """A cache directory recorded under another hiprtc version (a build machine whose compiler
    changed): rtc_warm rewrites its HIPRTC_VERSION to the running version, so the files it writes
    are named exactly as a lookup in that directory reads them, and prunes the stale entries."""
    from antpolarcodes_amd import rtc_warm
    d = tmp_path / "shipped"
    d.mkdir()
    (d / "HIPRTC_VERSION").write_text("0.0\n")
    (d / "pcg_0000000000000000.co").write_bytes(b"stale")
    code = (16, 1, ("BB", 8), 0, False)
    keep = rtc_warm.warm(quiet=True, cache=str(d), todo=[code])
    assert (d / "HIPRTC_VERSION").read_text().strip() == rtc_warm.hiprtc_version() != "0.0"
    assert len(keep) == 1 and sorted(f.name for f in d.glob("*.co")) == sorted(keep)
    _, rc, err, written, lookups = rtc_warm._one(code, str(d))
    assert rc == 0 and written == lookups == sorted(keep), err


def test_exit_wait_bound_keeps_a_failure_status(tmp_path):
    """PCG_RTC_EXIT_WAIT: a process leaving while a compile still runs never reports success
    (the status it asked for is replaced by PCG_RTC_EXIT_STATUS, 75)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prog = ("import sys; sys.path.insert(0, %r)\n"
            "from antpolarcodes_amd._native import Plan\n"
            "from antpolarcodes_amd.construction import frozen_bits\n"
            "p = Plan(64, 1, frozen_bits(64, 20, 0.0, 'BB'), systematic=False, crc=32, device=-1)\n"
            "p.specialize(wait=False)\n" % root)
    env = {k: v for k, v in os.environ.items() if not k.startswith("PCG_")}
    env.update({"PCG_RTC_CACHE": str(tmp_path), "PCG_RTC_EXIT_WAIT": "0"})
    r = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=300)
    if r.returncode == 0:  # the compile finished before exit: nothing was cut short
        assert "still running" not in r.stderr
        return
    assert r.returncode == 75 and "still running" in r.stderr, (r.returncode, r.stderr[-2000:])


def test_dev_build_knobs_reach_the_specialised_source():
    """The specialised list kernel is compiled with the library's own compile-time knobs
    (sclls_rtc_defines), and a plan of a default build reports no development override."""
    code = ("p = Plan(1024, 8, frozen_bits(1024, 512, 0.0, 'BB'), crc=8, device=-1)\n"
            "print('dev', p.describe()['dev_overrides'])\n")
    assert "dev 0" in _run(code, {})


def test_extra_compiler_options_are_a_dev_build(tmp_path):
    """PCG_RTC_XOPTS (extra hiprtc options, a development aid) changes the cache name -- a
    code object built with them is never taken for the default one -- and marks the plan's
    results as a development build (PCG_DEV_BUILD)."""
    code = _SMALL + "p.specialize()\nprint('dev', p.describe()['dev_overrides'])\n"
    out = _run(code, {"PCG_RTC_CACHE": str(tmp_path / "a")})
    assert "dev 0" in out
    out = _run(code, {"PCG_RTC_CACHE": str(tmp_path / "b"), "PCG_RTC_XOPTS": "-mllvm,-amdgpu-schedule-metric-bias=0"})
    assert "dev %d" % 0x40 in out
    a = [f.name for f in (tmp_path / "a").glob("pcg_*.co")]
    b = [f.name for f in (tmp_path / "b").glob("pcg_*.co")]
    assert len(a) == 1 and len(b) == 1 and a != b
