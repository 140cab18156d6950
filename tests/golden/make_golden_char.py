#!/usr/bin/env python3
"""Generate tests/golden/char_fixtures.npz from the REFERENCE's 8-bit decoders.

Runs only where oracle/_ref/libpolarref.so was built from /root/reference's sources
(`make -C oracle ref`).  Every expected output comes from the reference library
(Decoding::create(..., "char") = FastSscFipChar / SclFipChar, CharContainer::insertLlr,
the SclFip path list); inputs are seeded synthetic data.  Data only: inputs and
expected outputs.  tests/test_oracle_char.py pins oracle/polar_oracle_char.c to these
fixtures; the GPU tests check the HIP int8 kernels against the pinned oracle.

    python tests/golden/make_golden_char.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

from pyoracle import Oracle, Reference  # noqa: E402

from antpolarcodes_amd.construction import frozen_bits  # noqa: E402


def i8_families(rng, F, N):
    """int8 LLR families: AWGN-like, tie-heavy small ints, saturated, full range."""
    out = [
        np.clip(np.rint(rng.normal(8, 20, (F, N))), -128, 127),
        rng.integers(-3, 4, (F, N)),
        rng.choice(np.array([-128, -127, 127, 126, -1, 0, 1]), (F, N)),
        rng.integers(-128, 128, (F, N)),
    ]
    return np.concatenate(out).astype(np.int8)


def cover_codes():
    """(N, frozen) sets whose FastSscFip trees hold every node type at several sizes."""
    out = []
    for n in (8, 16, 32, 64, 128, 256):
        h = n // 2
        out.append((n, list(range(n - 1))))                   # Rep / ShortRep
        out.append((n, [0]))                                  # Spc / ShortSpc
        out.append((n, list(range(n - 2))))                   # DoubleRep (n >= 32)
        out.append((n, list(range(h))))                       # ZeroOne (short) / ZeroR+R1
        out.append((n, list(range(h)) + [h]))                 # ZeroSpc / ShortZeroSpc
        out.append((n, list(range(h - 1))))                   # ROne at the root
        out.append((n, list(range(h)) + [h, h + 1, h + 3]))   # ZeroR at the root
        out.append((n, [0, 1, 2, 4, h, h + 1]))               # RateR with mixed children
    return [(n, sorted(set(f))) for n, f in out]


def main():
    R = Reference()
    O = Oracle()
    rng = np.random.default_rng(20261016)
    fx = {}

    # --- float -> int8 quantisation (CharContainer::insertLlr) ---------------------
    for N in (8, 16, 32, 64):
        x = (rng.normal(0, 60, (4, N)) * 10.0 ** rng.uniform(-1, 1.5, (4, N))).astype(np.float32)
        edge = np.array([np.nan, 3e9, -3e9, np.inf, -np.inf, 126.5, 127.5, -128.5, -127.5, 0.5, -0.5,
                         1.5, 2.5, -2.5, 127.49, -128.49], np.float32)
        x[0, :min(N, len(edge))] = edge[:N]
        fx[f"q{N}_in"] = x
        fx[f"q{N}_out"] = R.f32_to_i8(x, N)

    # --- FastSscFipChar: node-type cover + BB codes, int8 input -----------------------
    codes = cover_codes()
    for N, K in ((64, 32), (256, 128), (1024, 512), (1024, 256), (128, 96)):
        codes.append((N, frozen_bits(N, K, 0.0)))
    for _ in range(12):
        N = int(rng.choice([16, 32, 64, 128, 256]))
        K = int(rng.integers(1, N))
        codes.append((N, sorted(rng.choice(N, N - K, replace=False).tolist())))
    sc_frozen, sc_len, sc_N, sc_llr, sc_info, sc_ok, sc_soft, sc_crc, sc_sys = [], [], [], [], [], [], [], [], []
    for i, (N, fr) in enumerate(codes):
        F = 2 if N <= 256 else 1
        llr = i8_families(rng, F, N)
        K = N - len(fr)
        crc = 8 if K % 8 == 0 and K >= 8 else 0
        sysm = True if N < 256 else bool(i % 2)  # non-systematic char output is undefined for N < 256 (Q9)
        info, ok, soft = R.decode_char(N, 1, fr, llr, sysm, crc, soft=True)
        sc_frozen.append(np.array(fr, np.uint16))
        sc_len.append(len(fr))
        sc_N.append(N)
        sc_llr.append(llr.ravel())
        sc_info.append(info.ravel())
        sc_ok.append(ok.ravel())
        sc_soft.append(soft.ravel())
        sc_crc.append(crc)
        sc_sys.append(int(sysm))
    fx["sc_N"] = np.array(sc_N, np.int32)
    fx["sc_len"] = np.array(sc_len, np.int32)
    fx["sc_crc"] = np.array(sc_crc, np.int32)
    fx["sc_sys"] = np.array(sc_sys, np.int32)
    fx["sc_frozen"] = np.concatenate(sc_frozen)
    fx["sc_llr"] = np.concatenate(sc_llr)
    fx["sc_info"] = np.concatenate(sc_info)
    fx["sc_ok"] = np.concatenate(sc_ok)
    fx["sc_soft"] = np.concatenate(sc_soft)

    # --- FastSscFipChar / SclFipChar on float input (decode_vector(const float*)) -----
    N, K = 1024, 512
    fr = frozen_bits(N, K, 0.0)
    xf = (rng.normal(1.0, 1.0, (8, N)) * 12.0).astype(np.float32)
    fx["fin_frozen"] = np.array(fr, np.uint16)
    fx["fin_llr"] = xf
    fx["fin_sc_info"], fx["fin_sc_ok"] = R.decode_char(N, 1, fr, xf, True, 8)
    fx["fin_scl8_info"], fx["fin_scl8_ok"] = R.decode_char(N, 8, fr, xf, True, 8, fresh=True)

    # --- SclFipChar: ordered int64 metrics, path counts, path codewords ---------------
    scl_cases = [(1024, 512, 8, 4), (256, 128, 8, 4), (256, 128, 2, 2), (256, 128, 4, 2),
                 (128, 64, 16, 2), (64, 40, 32, 2), (32, 16, 8, 2), (16, 8, 4, 2), (8, 4, 4, 2),
                 (1024, 512, 32, 1)]
    for j, (N, K, L, F) in enumerate(scl_cases):
        fr = frozen_bits(N, K, 0.0) if j % 3 else sorted(rng.choice(N, N - K, replace=False).tolist())
        llr = i8_families(rng, F, N)
        crc = 8 if K % 8 == 0 else 0
        info, ok = R.decode_char(N, L, fr, llr, True, crc, fresh=True)
        met, pc, pb = R.sclc_paths(N, L, fr, llr)
        key = f"scl{j}"
        fx[key + "_meta"] = np.array([N, K, L, crc], np.int32)
        fx[key + "_frozen"] = np.array(fr, np.uint16)
        fx[key + "_llr"] = llr
        fx[key + "_info"] = info
        fx[key + "_ok"] = ok
        fx[key + "_met"] = met
        fx[key + "_pc"] = pc
        fx[key + "_pb"] = pb
    # one decoder for a run of frames (metric carried, decisions unchanged) + non-systematic N >= 256
    N, K, L = 256, 128, 8
    fr = frozen_bits(N, K, 0.0)
    llr = i8_families(rng, 3, N)
    fx["carry_frozen"] = np.array(fr, np.uint16)
    fx["carry_llr"] = llr
    fx["carry_info"], fx["carry_ok"] = R.decode_char(N, L, fr, llr, True, 8, fresh=False)
    fx["nsys_info"], fx["nsys_ok"] = R.decode_char(N, L, fr, llr, False, 8, fresh=True)

    # sanity: the oracle reproduces what was recorded (the tests re-check this)
    assert np.array_equal(O.sclc_decode(N, L, fr, llr, True, 8, carry=True)[0], fx["carry_info"])
    out = os.path.join(HERE, "char_fixtures.npz")
    np.savez_compressed(out, **fx)
    print(f"wrote {out} ({os.path.getsize(out) // 1024} KiB)")


if __name__ == "__main__":
    main()
