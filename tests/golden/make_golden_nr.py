#!/usr/bin/env python3
"""Golden fixtures for the rate-matching / construction rows from the
REFERENCE itself (oracle/_ref/libpolarref.so, built from /root/reference's sources).

Writes tests/golden/nr_fixtures.npz (data only):
  * Construction::frozen_bits "5G" (fiveGList.cpp) and "BE" (betaexpansion.cpp)
  * Puncturer(E, frozen) kept positions, depuncture / puncture / puncturePacked outputs
  * the 5G NR config-4 decoder core: FiveGList(1024, 512) frozen set, frames punctured
    to E = 896, depunctured (+0.0 at the 128 punctured positions, so SCL sort ties are
    certain), decoded by the reference Fast-SSC and SCL-8 (Dummy detector: the output is
    ordered path 0) + the reference's ordered SCL-8 path metrics and path codewords.
CRC-11 itself has no reference: "parity unpinned"; the decoder core is
pinned through the ordered path list, the CRC-11 selection on top by the oracle.

    python tests/golden/make_golden_nr.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

from pyoracle import Reference  # noqa: E402

from antpolarcodes_amd import frames  # noqa: E402


def main():
    R = Reference()
    rng = np.random.default_rng(20261016)
    fx = {}

    # construction "5G" (N <= 1024) and "BE"
    for kind, Ns in (("5G", range(3, 11)), ("BE", range(3, 13))):
        rows = []
        for n in Ns:
            N = 1 << n
            for K in sorted({0, 1, N // 8, N // 4, N // 2, 3 * N // 4, N - 1, N}):
                rows.append((N, K, R.frozen_bits(N, K, 0.0, kind)))
        fx[f"cons{kind}_N"] = np.array([r[0] for r in rows], np.int32)
        fx[f"cons{kind}_K"] = np.array([r[1] for r in rows], np.int32)
        fx[f"cons{kind}_len"] = np.array([len(r[2]) for r in rows], np.int32)
        fx[f"cons{kind}_frozen"] = np.concatenate([np.array(r[2], np.uint16) for r in rows])

    # puncturer: (E, frozen) cases incl. non-multiple-of-8 E and E = parent
    cases = []
    for N, K, E, kind in ((64, 32, 48, "BB"), (64, 32, 56, "BB"), (64, 32, 64, "BB"), (128, 64, 100, "BB"),
                          (256, 128, 200, "5G"), (1024, 512, 896, "5G"), (1024, 512, 600, "5G"),
                          (32, 16, 17, "BB"), (2048, 1024, 1600, "BB")):
        fr = R.frozen_bits(N, K, 0.0, kind)
        parent, pos = R.puncturer(E, fr)
        x = rng.normal(0, 2, E).astype(np.float32)
        dep = R.punc_apply(E, fr, 0, x)
        y = rng.normal(0, 2, parent).astype(np.float32)
        pun = R.punc_apply(E, fr, 1, y)
        if E % 8 == 0:
            b = rng.integers(0, 256, parent // 8, dtype=np.uint8)
            pp = R.punc_apply(E, fr, 2, b)
        else:
            b = np.zeros(0, np.uint8)
            pp = np.zeros(0, np.uint8)
        cases.append((E, parent, fr, pos, x, dep, y, pun, b, pp))
    for i, (E, parent, fr, pos, x, dep, y, pun, b, pp) in enumerate(cases):
        fx[f"punc{i}_E"] = np.int32(E)
        fx[f"punc{i}_N"] = np.int32(parent)
        fx[f"punc{i}_frozen"] = np.array(fr, np.uint16)
        fx[f"punc{i}_pos"] = pos.astype(np.uint16)
        fx[f"punc{i}_x"], fx[f"punc{i}_dep"] = x, dep
        fx[f"punc{i}_y"], fx[f"punc{i}_pun"] = y, pun
        fx[f"punc{i}_b"], fx[f"punc{i}_pp"] = b, pp
    fx["punc_cases"] = np.int32(len(cases))
    # too few frozen positions -> std::out_of_range
    try:
        R.puncturer(40, list(range(10)))
        fx["punc_err"] = np.array(b"")
    except ValueError as e:
        fx["punc_err"] = np.array(str(e).encode())

    # config-4 decoder core on depunctured frames
    N, K, E = 1024, 512, 896
    llr_e, info, fr, pos = frames.nr_frames(E, K, 24, 1.5, seed=5, crc=11)
    dep = np.zeros((llr_e.shape[0], N), np.float32)
    dep[:, pos] = llr_e
    fx["nr_frozen"] = np.array(fr, np.uint16)
    fx["nr_llr"] = dep
    fx["nr_info_tx"] = info
    sc_info, _ = R.decode(N, 1, fr, dep, crc=0, fresh=True)
    fx["nr_sc_info"] = sc_info
    scl_info, _ = R.decode(N, 8, fr, dep, crc=0, fresh=True)
    fx["nr_scl8_info"] = scl_info
    met, pc, pb = R.scl_paths(N, 8, fr, dep, fresh=True)
    fx["nr_scl8_met"], fx["nr_scl8_pc"], fx["nr_scl8_pb"] = met, pc, pb

    out = os.path.join(HERE, "nr_fixtures.npz")
    np.savez_compressed(out, **fx)
    print(f"wrote {out} ({os.path.getsize(out) / 1024:.0f} KiB)")


if __name__ == "__main__":
    main()
