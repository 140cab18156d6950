"""Compile the specialised kernel of one bench configuration under the CURRENT environment
(PCG_DEV_LIB variant, layout knobs such as PCG_SCL_LDS_KB) into a dev cache directory, so an
A/B sweep on the GPU box loads it instead of compiling there (development aid).
    PCG_DEV_LIB=lib_dev/libpcg_x.so [PCG_...] python tools/warm_dev.py <cache dir> <mode> ...
modes: the bench_codes() entries of antpolarcodes_amd/rtc_codes.py by bench mode name.
On the box: PCG_RTC_CACHE=<cache dir> with the same PCG_* settings."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antpolarcodes_amd.rtc_codes import bench_codes  # noqa: E402

MODES = dict(zip(["sc", "scl8", "adaptive8", "nr5g", "scl32", "sc_char", "scl8_char", "adaptive8_char"],
                 bench_codes()))


def main():
    cache = os.path.abspath(sys.argv[1])
    os.makedirs(cache, exist_ok=True)
    for m in sys.argv[2:]:
        c = MODES[m]
        N, L, (kind, arg), crc, sysm = c[:5]
        adaptive = len(c) > 5 and c[5] in ("adaptive", "adaptive_char")
        fixed = len(c) > 5 and c[5] in ("char", "adaptive_char")
        prog = (
            "import sys; sys.path.insert(0, %r)\n"
            "from antpolarcodes_amd._native import Plan\n"
            "from antpolarcodes_amd.construction import frozen_bits\n"
            "p = Plan(%d, %d, frozen_bits(%d, %r, 0.0, %r), systematic=%r, crc=%d, device=-1, adaptive=%r, fixed=%r)\n"
            "p.specialize()\n" % (ROOT, N, L, N, arg, kind, sysm, crc, adaptive, fixed))
        env = dict(os.environ, PCG_RTC_CACHE=cache)
        r = subprocess.run([sys.executable, "-c", prog], env=env)
        if r.returncode:
            sys.exit(r.returncode)
        print(m, "ok")


if __name__ == "__main__":
    main()
