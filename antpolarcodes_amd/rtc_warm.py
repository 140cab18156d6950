"""Fill the library's shipped cache of plan-specialised kernels (antpolarcodes_amd/lib/rtc/).

A plan's specialised kernel (rtc.cpp, pcg_plan_specialize) is looked up in this directory
before the user cache and before any hiprtc compile, so the codes listed here -- the
benchmark configurations and the codes the GPU tests specialise --
load at once on a fresh machine.  It is a build step (`__graft_entry__.build()`, or
`python -m antpolarcodes_amd.rtc_warm`): each code is compiled by a host-only plan
(device = -1, no GPU needed) in its own process, several in parallel.  The cache files are
named by everything that determines the code object (generated source, embedded kernel
sources, options, architecture, hiprtc version), so a stale entry is never loaded -- it is
simply not found, and the build compiles the current one.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CACHE = os.path.join(HERE, "lib", "rtc")


def bench_codes():
    """(N, L, frozen spec, crc, systematic): the configurations bench.py decodes."""
    return [
        (1024, 1, ("BB", 512), 8, True),     # config 2
        (1024, 8, ("BB", 512), 8, True),     # config 3
        (1024, 8, ("BB", 512), 8, True, "adaptive"),  # config 3 with AdaptiveFloat (both stages)
        (1024, 8, ("5G", 512), 11, True),    # config 4
        (4096, 32, ("BB", 2048), 8, True),   # config 5
        (1024, 1, ("BB", 512), 8, True, "char"),      # sc_char
        (1024, 8, ("BB", 512), 8, True, "char"),      # scl8_char
        (1024, 8, ("BB", 512), 8, True, "adaptive_char"),  # adaptive8_char (both stages)
    ]


def test_codes():
    """The codes the GPU tests run through specialised kernels (tests/test_gpu_rtc.py and the
    specialised variants of the full-size parity tests)."""
    out = []
    for N in (8, 32, 128, 512, 1024):                      # test_rtc_bb_codes
        out.append((N, 1, ("BB", max(8, N // 2)), 8, True))
    for sysm in (True, False):                            # test_rtc_crc_and_systematic
        for crc in (0, 16, 32):
            out.append((1024, 1, ("BB", 512), crc, sysm))
    try:                                                  # test_rtc_node_kinds
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
        from helpers import node_cover_sets
        for N, fr in node_cover_sets():
            out.append((N, 1, ("set", tuple(fr)), 8, True))
    except ImportError:
        pass
    for N, K, L, crc, sysm in ((256, 128, 4, 16, True), (1024, 512, 8, 8, True), (512, 256, 6, 32, False),
                               (4096, 2048, 32, 8, True), (1024, 512, 12, 8, True), (1024, 512, 8, 0, True)):
        out.append((N, L, ("BB", K), crc, sysm))          # test_rtc_list_plans
    out.append((1024, 8, ("5G", 512), 0, True))           # config 4's decoder core with the Dummy detector
    out.append((1024, 1, ("5G", 512), 11, True))          # config 4 through Fast-SSC
    for crc in (8, 16, 32):                               # test_adaptive_matches_oracle: both stages
        out.append((1024, 8, ("BB", 512), crc, True, "adaptive"))
    try:                                                  # test_gpu_char.py::test_scc_rtc_kernel
        from test_gpu_char import rtc_char_codes
        for N, fr, sysm, crc in rtc_char_codes():
            out.append((N, 1, ("set", tuple(int(v) for v in fr)), crc, sysm, "char"))
    except ImportError:
        pass
    for N, K, L, crc, sysm in ((256, 128, 2, 8, True), (1024, 512, 8, 8, True), (512, 256, 4, 16, False),
                               (1024, 512, 16, 32, True), (1024, 512, 32, 8, True), (1024, 512, 6, 0, True)):
        out.append((N, L, ("BB", K), crc, sysm, "char"))  # test_gpu_char.py::test_sclc_rtc_kernel
    for crc in (8, 16):                                   # test_adaptive_char_matches_oracle
        out.append((1024, 8, ("BB", 512), crc, True, "adaptive_char"))
    return out


def _key(c):
    return tuple(c[:2]) + tuple(c[2]) + tuple(c[3:])


def codes():
    seen, out = set(), []
    for c in bench_codes() + test_codes():
        if _key(c) not in seen:
            seen.add(_key(c))
            out.append(c)
    return out


def _one(c):
    """Compile one code in a child process (hiprtc state stays out of the caller)."""
    N, L, (kind, arg), crc, sysm = c[:5]
    adaptive = len(c) > 5 and c[5] in ("adaptive", "adaptive_char")
    fixed = len(c) > 5 and c[5] in ("char", "adaptive_char")
    prog = (
        "import sys; sys.path.insert(0, %r)\n"
        "from antpolarcodes_amd._native import Plan, PcgError\n"
        "from antpolarcodes_amd.construction import frozen_bits\n"
        "kind, arg = %r, %r\n"
        "fr = list(arg) if kind == 'set' else frozen_bits(%d, arg, 0.0, kind)\n"
        "try:\n"
        "    p = Plan(%d, %d, fr, systematic=%r, crc=%d, device=-1, adaptive=%r, fixed=%r)\n"
        "except PcgError:\n"
        "    sys.exit(0)  # a frozen set the decoder rejects: nothing to compile\n"
        "p.specialize()\n"
        "import ctypes\n"
        "from antpolarcodes_amd._native import lib\n"
        "b = ctypes.create_string_buffer(128)\n"
        "lib().pcg_dev_rtc_cache_name(p._h, b, 128)\n"
        "print('RTCFILE', b.value.decode())\n" % (os.path.dirname(HERE), kind, arg, N, N, L, sysm, crc, adaptive, fixed))
    env = {k: v for k, v in os.environ.items() if not k.startswith("PCG_")}  # the default layouts
    env["PCG_RTC_CACHE"] = CACHE
    r = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True)
    names = [n for ln in r.stdout.splitlines() if ln.startswith("RTCFILE ") for n in ln.split()[1:]]
    return c, r.returncode, r.stderr[-2000:], names


def warm(jobs=None, quiet=False):
    os.makedirs(CACHE, exist_ok=True)
    todo = codes()
    jobs = jobs or min(8, os.cpu_count() or 1)
    bad, keep = [], set()
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for c, rc, err, names in ex.map(_one, todo):
            if rc != 0:
                bad.append((c, err))
            keep.update(names)
    if not bad:  # entries no listed code produces any more (older sources) are dropped
        for f in os.listdir(CACHE):
            if f not in keep:
                os.remove(os.path.join(CACHE, f))
    if not quiet:
        print(f"rtc cache: {len(todo)} codes, {len(os.listdir(CACHE))} files in {CACHE}")
    if bad:
        raise RuntimeError("rtc cache: %d codes failed to compile, first: %s\n%s" % (len(bad), bad[0][0], bad[0][1]))


if __name__ == "__main__":
    warm()
