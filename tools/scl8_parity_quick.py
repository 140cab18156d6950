"""Quick bit-exact check of a (dev) SCL library against the oracle: every LLR family at
N = 8 ... 2048 and AWGN frames, one list size (dev libraries built with PCG_LS_ONLY=L).
    PCG_DEV_LIB=lib_dev/libpcg_<tag>.so python tools/scl8_parity_quick.py [L]"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
from helpers import LLR_KINDS, llr_kinds  # noqa: E402
from pyoracle import Oracle  # noqa: E402
from antpolarcodes_amd import frames  # noqa: E402
from antpolarcodes_amd._native import Plan  # noqa: E402

LIST = int(sys.argv[1]) if len(sys.argv) > 1 else 8
orc = Oracle()
rng = np.random.default_rng(123)
bad = 0
cases = 0
for N in (8, 16, 64, 256, 1024, 2048):
    for K in sorted({N // 4, N // 2, 3 * N // 4}):
        fr = orc.frozen_bits_bb(N, K, 0.0)
        for kind in LLR_KINDS:
            llr = llr_kinds(rng, 32, N, kind)
            for crc in (0, 8) if K >= 16 else (0,):
                gi, gk, gm = Plan(N, LIST, fr, crc=crc, device=0).decode_host(llr, want_metrics=True)
                oi, ok, om, _, _ = orc.scl_decode(N, LIST, fr, llr, crc=crc, paths=True)
                cases += 1
                if not (np.array_equal(gi, oi) and np.array_equal(gk, ok) and
                        np.array_equal(gm.view(np.uint32), om.view(np.uint32))):
                    bad += 1
                    print("MISMATCH", N, K, kind, crc, flush=True)
fr = orc.frozen_bits_bb(1024, 512, 0.0)
llr, _, _ = frames.awgn_frames(1024, fr, 8192 if LIST <= 8 else 1024, 1.5, seed=9, crc=8)
gi, gk, gm = Plan(1024, LIST, fr, crc=8, device=0).decode_host(llr, want_metrics=True)
oi, ok, om, _, _ = orc.scl_decode(1024, LIST, fr, llr, crc=8, paths=True)
cases += 1
if not (np.array_equal(gi, oi) and np.array_equal(gk, ok) and np.array_equal(gm.view(np.uint32), om.view(np.uint32))):
    bad += 1
    print("MISMATCH awgn", flush=True)
if LIST >= 16:  # the config-5 shape: eighths recomputed (virt 3)
    fr = orc.frozen_bits_bb(4096, 2048, 0.0)
    llr, _, _ = frames.awgn_frames(4096, fr, 128, 1.5, seed=5, crc=8)
    p = Plan(4096, LIST, fr, crc=8, device=0)
    print("N=4096 recomputed stages:", p.describe()["recomputed_stages"], flush=True)
    gi, gk, gm = p.decode_host(llr, want_metrics=True)
    oi, ok, om, _, _ = orc.scl_decode(4096, LIST, fr, llr, crc=8, paths=True)
    cases += 1
    if not (np.array_equal(gi, oi) and np.array_equal(gk, ok) and np.array_equal(gm.view(np.uint32), om.view(np.uint32))):
        bad += 1
        print("MISMATCH config5", flush=True)
print(f"scl{LIST} quick parity: {cases - bad}/{cases} cases bit-exact ({os.environ.get('PCG_DEV_LIB', 'in-tree')})")
sys.exit(1 if bad else 0)
