#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only where the reference library was built from /root/reference's sources
(`make -C oracle ref` -> oracle/_ref/libpolarref.so).  Every expected output in
the fixtures comes from the reference decoder/encoder/detector/constructor; the
inputs are seeded synthetic data.  The fixtures are data only (inputs + expected
outputs); tests/test_oracle.py pins oracle/polar_oracle.c against them and the GPU
tests check the HIP kernels against the pinned oracle.

    python tests/golden/make_golden.py
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


def llr_kinds(rng, F, N):
    """A mix of AWGN-like, tie-heavy and signed-zero inputs."""
    out = []
    out.append(rng.normal(1.0, 1.5, (F, N)))
    out.append(rng.integers(-3, 4, (F, N)))
    x = rng.normal(0.0, 2.0, (F, N))
    x[rng.random((F, N)) < 0.2] = -0.0
    x[rng.random((F, N)) < 0.2] = 0.0
    out.append(x)
    out.append(np.sign(rng.normal(0, 1, (F, N))) * rng.integers(0, 2, (F, N)))
    return np.concatenate(out).astype(np.float32)


def main():
    R = Reference()
    rng = np.random.default_rng(20261015)
    fx = {}

    # --- construction (Construction::frozen_bits, "BB") -----------------------------
    cons = []
    for n in range(3, 13):
        N = 1 << n
        for K in sorted({1, N // 8, N // 4, N // 2, 3 * N // 4, N - 1}):
            for d in (-2.0, 0.0, 2.5):
                cons.append((N, K, d, R.frozen_bits(N, K, d)))
    fx["cons_N"] = np.array([c[0] for c in cons], np.int32)
    fx["cons_K"] = np.array([c[1] for c in cons], np.int32)
    fx["cons_dsnr"] = np.array([c[2] for c in cons], np.float32)
    fx["cons_frozen"] = np.concatenate([np.array(c[3], np.uint16) for c in cons])
    fx["cons_len"] = np.array([len(c[3]) for c in cons], np.int32)

    # --- detectors: random messages, reference generate() ----------------------------
    for kind in (8, 16, 32):
        msgs = rng.integers(0, 256, (16, 24), dtype=np.uint8)
        gen = np.stack([R.crc(kind, m, generate=True) for m in msgs])
        fx[f"crc{kind}_gen"] = gen

    # --- encoder (ButterflyFipPacked), systematic and not, with CRC -----------------
    fr = R.frozen_bits(1024, 512, 0.0)
    info = rng.integers(0, 256, (8, 64), dtype=np.uint8)
    for sysm in (0, 1):
        for crc in (0, 8, 32):
            fx[f"enc_s{sysm}_c{crc}"] = R.encode(1024, fr, info, systematic=bool(sysm), crc=crc)
    fx["enc_info"] = info

    # --- Fast-SSC (config 1/2 shape): AWGN + quirk inputs, systematic and not ---------
    llr_awgn, _, _ = frames.awgn_frames(1024, fr, 48, 2.0, seed=7, crc=8)
    llr_sc = np.concatenate([llr_awgn, llr_kinds(rng, 4, 1024)])
    fx["sc_frozen"] = np.array(fr, np.uint16)
    fx["sc_llr"] = llr_sc
    for sysm in (0, 1):
        info, ok, cw = R.decode(1024, 1, fr, llr_sc, systematic=bool(sysm), crc=8, soft=True)
        fx[f"sc_info_s{sysm}"] = info
        fx[f"sc_ok_s{sysm}"] = ok
        if sysm:
            fx["sc_softcw_sign"] = np.packbits((cw.view(np.uint32) >> 31).astype(np.uint8), axis=1)
            fx["sc_softcw_bits"] = cw.view(np.uint32)[:8]  # full float words of 8 frames

    # --- Fast-SSC node kinds: one small code per leaf type (+ Q1 ZeroSpc) -------------
    sets = [(8, [0, 1]), (8, [0, 1, 2]), (8, [0, 1, 2, 3, 4]), (8, [0, 1, 2, 4]),
            (16, [0, 1]), (16, list(range(13))), (16, sorted(set(range(10)) | {10, 12})),
            (32, list(range(17))), (32, list(range(15))), (64, list(range(30)) + [32])]
    kinds_llr, kinds_info, kinds_soft, kinds_meta = [], [], [], []
    for N, f in sets:
        x = llr_kinds(rng, 2, N)
        info, ok, cw = R.decode(N, 1, f, x, crc=0, soft=True)
        kinds_llr.append(x.ravel())
        kinds_soft.append(cw.view(np.uint32).ravel())
        kinds_meta.append((N, len(f), x.shape[0]))
    fx["kinds_meta"] = np.array(kinds_meta, np.int32)
    fx["kinds_frozen"] = np.concatenate([np.array(f, np.uint16) for _, f in sets])
    fx["kinds_llr"] = np.concatenate(kinds_llr)
    fx["kinds_softcw"] = np.concatenate(kinds_soft)
    # Q1: ZeroSpcDecoder outputs the right half to both halves
    q1_fr = list(range(9))
    q1_llr = np.array([[5, 6, 7, 8, 9, 10, 11, 12, -1, -1.1, -1.2, -1.3, -1.4, -1.5, -1.6, -1.7]], np.float32)
    _, _, q1cw = R.decode(16, 1, q1_fr, q1_llr, crc=0, soft=True)
    fx["q1_llr"] = q1_llr
    fx["q1_softcw"] = q1cw.view(np.uint32)

    # --- SCL (config 3 shape), fresh decoder per frame -------------------------------
    llr_awgn, _, _ = frames.awgn_frames(1024, fr, 40, 1.5, seed=8, crc=8)
    llr_scl = np.concatenate([llr_awgn, llr_kinds(rng, 2, 1024)])
    fx["scl8_llr"] = llr_scl
    info, ok = R.decode(1024, 8, fr, llr_scl, crc=8, fresh=True)
    met, pc, pb = R.scl_paths(1024, 8, fr, llr_scl, fresh=True)
    fx["scl8_info"], fx["scl8_ok"] = info, ok
    fx["scl8_metrics"], fx["scl8_pathcount"], fx["scl8_pathbits"] = met, pc, pb
    info_ns, ok_ns = R.decode(1024, 8, fr, llr_scl, systematic=False, crc=8, fresh=True)
    fx["scl8_info_nonsys"], fx["scl8_ok_nonsys"] = info_ns, ok_ns
    # Q8: the reference carries path 0's metric across frames in one decoder instance
    info_c, ok_c = R.decode(1024, 8, fr, llr_scl, crc=8, fresh=False)
    fx["scl8_info_carry"], fx["scl8_ok_carry"] = info_c, ok_c

    # --- SCL L=32, N=4096 K=2048 (config 5 shape) -------------------------------------
    fr4 = R.frozen_bits(4096, 2048, 0.0)
    llr4, _, _ = frames.awgn_frames(4096, fr4, 4, 1.5, seed=9, crc=8)
    fx["scl32_frozen"] = np.array(fr4, np.uint16)
    fx["scl32_llr"] = llr4
    fx["scl32_info"], fx["scl32_ok"] = R.decode(4096, 32, fr4, llr4, crc=8, fresh=True)
    fx["scl32_metrics"], fx["scl32_pathcount"], _ = R.scl_paths(4096, 32, fr4, llr4, fresh=True)

    # --- small SCL codes, every list size ---------------------------------------------
    small = []
    for N in (8, 16, 32, 64):
        for L in (2, 4, 8, 16, 32):
            f = R.frozen_bits(N, N // 2, 0.0)
            x = llr_kinds(rng, 1, N)
            met, pc, pb = R.scl_paths(N, L, f, x, fresh=True)
            small.append((N, L, f, x, met, pc, pb))
    fx["sclsmall_meta"] = np.array([(N, L, len(f), x.shape[0]) for N, L, f, x, *_ in small], np.int32)
    fx["sclsmall_frozen"] = np.concatenate([np.array(f, np.uint16) for _, _, f, *_ in small])
    fx["sclsmall_llr"] = np.concatenate([x.ravel() for *_, x, _, _, _ in small])
    fx["sclsmall_metrics"] = np.concatenate([m.ravel() for *_, m, _, _ in small])
    fx["sclsmall_pathcount"] = np.concatenate([p.ravel() for *_, p, _ in small])
    fx["sclsmall_pathbits"] = np.concatenate([b.ravel() for *_, b in small])

    out = os.path.join(HERE, "reference_fixtures.npz")
    np.savez_compressed(out, **fx)
    print(f"wrote {out} ({os.path.getsize(out) / 1024:.0f} KiB, {len(fx)} arrays)")


if __name__ == "__main__":
    main()
