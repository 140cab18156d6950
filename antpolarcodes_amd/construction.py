"""Frozen-set construction (host side), mirroring Construction::frozen_bits
(src/polarcode/construction/constructor.cpp:41-63).

* "BB": Bhattacharyya bounds (bhattacharrya.cpp:39-82): float initial parameter
  exp(-2 * 10^(dSNR/10) * K/N), double-precision recursion, stable descending sort
  (trackingSorter::stableSortDescending, arrayfuncs.cpp:93-107), the N-K least
  reliable channels frozen, returned ascending.
"""
import numpy as np


def _bhattacharyya(N, K, dsnr):
    lin = np.float32(10.0 ** (np.float64(dsnr) / 10.0))
    init = np.float32(np.exp(-2.0 * np.float64(lin) * K / N))
    z = np.zeros(N, np.float64)
    z[0] = np.float64(init)
    stage = int(np.log2(N)) - 1
    while stage >= 0:
        B = 1 << stage
        for j in range(0, N, 2 * B):
            T = z[j]
            z[j + B] = T * T
            z[j] = 2 * T - z[j + B]
        stage -= 1
    order = np.argsort(-z, kind="stable")  # descending, ties keep index order
    return sorted(int(v) for v in order[:N - K])


def frozen_bits(blockLength, infoLength, designSNR=0.0, constructorType="BB"):
    N, K = int(blockLength), int(infoLength)
    if N < 1 or (N & (N - 1)) or K < 0 or K > N:
        raise ValueError("block length must be a power of two and 0 <= K <= N")
    t = constructorType.lower()
    if "be" in t or "5g" in t:
        raise NotImplementedError(f"construction '{constructorType}' is not part of this build yet")
    return _bhattacharyya(N, K, float(designSNR))
