"""Fill the library's shipped cache of plan-specialised kernels (antpolarcodes_amd/lib/rtc/).

A plan's specialised kernel (rtc.cpp, pcg_plan_specialize) is looked up in this directory
before the user cache and before any hiprtc compile, so the codes of the catalogue
(antpolarcodes_amd/rtc_codes.py: the benchmark configurations, SURVEY.md configs 2-5, and a
validation catalogue covering every node kind) load at once on a fresh machine.  It is a build step (`__graft_entry__.build()`, or
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


def codes():
    """The shipped catalogue (antpolarcodes_amd/rtc_codes.py)."""
    from antpolarcodes_amd import rtc_codes
    return rtc_codes.codes()


def _one(c, cache=None):
    """Compile one code in a child process (hiprtc state stays out of the caller).  Returns the
    file names the compile wrote and the names a lookup in `cache` reads (they must agree)."""
    cache = cache or CACHE
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
        "b = ctypes.create_string_buffer(256)\n"
        "lib().pcg_dev_rtc_cache_name(p._h, b, 256)\n"
        "print('RTCFILE', b.value.decode())\n"
        "lib().pcg_dev_rtc_lookup_name(p._h, %r.encode(), b, 256)\n"
        "print('RTCLOOKUP', b.value.decode())\n" % (os.path.dirname(HERE), kind, arg, N, N, L, sysm, crc, adaptive,
                                                    fixed, cache))
    env = {k: v for k, v in os.environ.items() if not k.startswith("PCG_")}  # the default layouts
    env["PCG_RTC_CACHE"] = cache
    r = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True)

    def names(tag):
        return [n for ln in r.stdout.splitlines() if ln.startswith(tag + " ") for n in ln.split()[1:]]
    return c, r.returncode, r.stderr[-2000:], names("RTCFILE"), names("RTCLOOKUP")


def hiprtc_version():
    """The hiprtc version the compiles of this machine run with (a child process: the
    caller never loads hiprtc)."""
    prog = ("import sys, ctypes; sys.path.insert(0, %r)\n"
            "from antpolarcodes_amd._native import lib\n"
            "b = ctypes.create_string_buffer(64)\n"
            "lib().pcg_dev_rtc_version(b, 64)\n"
            "print('HIPRTC', b.value.decode())\n" % os.path.dirname(HERE))
    r = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True, check=True)
    return [ln.split()[1] for ln in r.stdout.splitlines() if ln.startswith("HIPRTC ")][0]


def dir_version(cache):
    try:
        with open(os.path.join(cache, "HIPRTC_VERSION")) as f:
            return f.read().strip()
    except OSError:
        return ""


def warm(jobs=None, quiet=False, strict=True, cache=None, todo=None):
    """Compile the catalogue into the shipped cache.  strict=False (the build step): codes that
    fail to compile are reported as a warning -- the library runs without them (their plans
    compile on first use or keep the interpreter kernel), as it does without hiprtc.

    The cache is read under the hiprtc version its HIPRTC_VERSION file records (rtc.cpp
    disk_lookup) and written under the running one, so the file is set to the running version
    first: after a compiler change every entry is rebuilt under the new names (and the old ones
    pruned), and the names written are checked to be the names a lookup reads."""
    cache = cache or CACHE
    os.makedirs(cache, exist_ok=True)
    todo = codes() if todo is None else todo
    try:
        ver = hiprtc_version()
    except (subprocess.CalledProcessError, IndexError, OSError) as e:  # (the library does not load here)
        ver = None
        print(f"WARNING: rtc cache: hiprtc version unknown ({e}); {cache}/HIPRTC_VERSION left as it is",
              file=sys.stderr)
    if ver and ver != "none" and dir_version(cache) != ver:
        with open(os.path.join(cache, "HIPRTC_VERSION"), "w") as f:
            f.write(ver + "\n")
    jobs = jobs or min(8, os.cpu_count() or 1)
    bad, keep = [], set()
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for c, rc, err, names, lookups in ex.map(lambda c: _one(c, cache), todo):
            if rc == 0 and names != lookups:
                rc, err = 1, "written %s but a lookup reads %s" % (names, lookups)
            if rc == 0 and any(not os.path.isfile(os.path.join(cache, n)) for n in names):
                rc, err = 1, "%s not written to %s" % (names, cache)
            if rc != 0:
                bad.append((c, err))
            keep.update(names)
    if not bad:  # entries no listed code produces any more (older sources) are dropped
        for f in os.listdir(cache):
            if f not in keep and f != "HIPRTC_VERSION":
                os.remove(os.path.join(cache, f))
    if not quiet:
        print(f"rtc cache: {len(todo)} codes, {len(os.listdir(cache))} files in {cache}")
    if bad:
        msg = "rtc cache: %d codes failed to compile, first: %s\n%s" % (len(bad), bad[0][0], bad[0][1])
        if strict:
            raise RuntimeError(msg)
        print("WARNING: " + msg, file=sys.stderr)
    return keep


if __name__ == "__main__":
    warm(strict="--warn" not in sys.argv[1:])
