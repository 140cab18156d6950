"""Quick bit-exact check of a (dev) SCL-8 library against the oracle: every LLR family at
N = 8 ... 1024 and AWGN frames, L = 8 only (dev libraries built with PCG_LS_ONLY=8).
    PCG_DEV_LIB=lib_dev/libpcg_<tag>.so python tools/scl8_parity_quick.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
from helpers import LLR_KINDS, llr_kinds  # noqa: E402
from pyoracle import Oracle  # noqa: E402
from antpolarcodes_amd import frames  # noqa: E402
from antpolarcodes_amd._native import Plan  # noqa: E402

orc = Oracle()
rng = np.random.default_rng(123)
bad = 0
cases = 0
for N in (8, 16, 64, 256, 1024):
    for K in sorted({N // 4, N // 2, 3 * N // 4}):
        fr = orc.frozen_bits_bb(N, K, 0.0)
        for kind in LLR_KINDS:
            llr = llr_kinds(rng, 32, N, kind)
            for crc in (0, 8) if K >= 16 else (0,):
                gi, gk, gm = Plan(N, 8, fr, crc=crc, device=0).decode_host(llr, want_metrics=True)
                oi, ok, om, _, _ = orc.scl_decode(N, 8, fr, llr, crc=crc, paths=True)
                cases += 1
                if not (np.array_equal(gi, oi) and np.array_equal(gk, ok) and
                        np.array_equal(gm.view(np.uint32), om.view(np.uint32))):
                    bad += 1
                    print("MISMATCH", N, K, kind, crc, flush=True)
fr = orc.frozen_bits_bb(1024, 512, 0.0)
llr, _, _ = frames.awgn_frames(1024, fr, 8192, 1.5, seed=9, crc=8)
gi, gk, gm = Plan(1024, 8, fr, crc=8, device=0).decode_host(llr, want_metrics=True)
oi, ok, om, _, _ = orc.scl_decode(1024, 8, fr, llr, crc=8, paths=True)
cases += 1
if not (np.array_equal(gi, oi) and np.array_equal(gk, ok) and np.array_equal(gm.view(np.uint32), om.view(np.uint32))):
    bad += 1
    print("MISMATCH awgn", flush=True)
print(f"scl8 quick parity: {cases - bad}/{cases} cases bit-exact ({os.environ.get('PCG_DEV_LIB', 'in-tree')})")
sys.exit(1 if bad else 0)
