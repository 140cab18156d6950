#!/usr/bin/env python3
"""SHA-256 digests of the REFERENCE's outputs on the full-size GPU test batches.

The GPU tests compare the HIP kernels with the oracle frame by frame; these digests pin
the same batches to the reference itself (oracle/_ref/libpolarref.so, built from the
reference's sources by `make -C oracle ref`), so the 2^16-frame runs are pinned directly,
not only through the oracle.  Frames come from the build's seeded numpy generator
(antpolarcodes_amd/frames.py) with exactly the seeds the GPU tests use; only the digests
(and the generation parameters) are committed, in reference_digests.json.

Digest = sha256 over the C-contiguous bytes of the array: info (F x ceil(K/8) uint8), ok
(F uint8), metrics (F x L float32, little endian; ordered path metrics of a freshly
constructed decoder per frame, unused slots 0).

    python tests/golden/make_digests.py          # ~1 min on 8 CPUs
"""
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

# name: generation parameters = the GPU test's own call (file::test)
CASES = {
    # tests/test_gpu_sc.py::test_sc_awgn_batch_config2
    "config2_sc": dict(kind="awgn", N=1024, K=512, L=1, F=1 << 16, ebn0=2.0, seed=2, crc=8),
    # tests/test_gpu_scl.py::test_scl_awgn_batch_config3
    "config3_scl8": dict(kind="awgn", N=1024, K=512, L=8, F=1 << 16, ebn0=2.0, seed=4, crc=8),
    # tests/test_gpu_nr.py::test_decode_punctured_matches_oracle[8]: the decoder core on the
    # depunctured frames (the reference has no CRC-11: metrics, and info/ok with Dummy)
    "config4_nr_scl8": dict(kind="nr", N=1024, K=512, L=8, F=1 << 16, E=896, ebn0=1.25, seed=48, crc=0),
    # tests/test_gpu_scl.py::test_scl32_reference_digest (config 5 code, host frames)
    "config5_scl32": dict(kind="awgn", N=4096, K=2048, L=32, F=4096, ebn0=1.5, seed=55, crc=8),
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def case_frames(c):
    """(frozen, F x N float32 LLRs) of a case, as the GPU test builds them."""
    from antpolarcodes_amd import frames
    from antpolarcodes_amd.construction import frozen_bits
    if c["kind"] == "nr":
        llr, _, fr, _ = frames.nr_frames(c["E"], c["K"], c["F"], c["ebn0"], seed=c["seed"])
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from pyoracle import Oracle
        return list(fr), Oracle().depuncture(c["E"], fr, llr)
    fr = frozen_bits(c["N"], c["K"], 0.0)
    llr, _, _ = frames.awgn_frames(c["N"], fr, c["F"], c["ebn0"], seed=c["seed"], crc=c["crc"])
    return list(fr), llr


def _ref_chunk(args):
    N, L, fr, x, crc = args
    from pyoracle import Reference
    R = Reference()
    info, ok = R.decode(N, L, fr, x, crc=crc, fresh=True)
    met = R.scl_paths(N, L, fr, x, fresh=True)[0] if L > 1 else None
    return info, ok, met


def reference_outputs(N, L, fr, llr, crc, workers=8):
    parts = np.array_split(np.arange(llr.shape[0]), workers * 4)
    with ProcessPoolExecutor(workers) as ex:
        res = list(ex.map(_ref_chunk, [(N, L, fr, llr[p], crc) for p in parts]))
    info = np.concatenate([r[0] for r in res])
    ok = np.concatenate([r[1] for r in res])
    met = np.concatenate([r[2] for r in res]) if L > 1 else None
    return info, ok, met


def main():
    out = {"_doc": "sha256 of the reference's outputs (oracle/_ref) on the GPU tests' full-size batches; "
                   "made by tests/golden/make_digests.py", "cases": {}}
    for name, c in CASES.items():
        fr, llr = case_frames(c)
        info, ok, met = reference_outputs(c["N"], c["L"], fr, llr, c["crc"])
        d = dict(c, info=sha(info), ok=sha(ok), frames_ok=int(ok.sum()), llr=sha(llr))
        if met is not None:
            d["metrics"] = sha(met.astype(np.float32))
        out["cases"][name] = d
        print(name, d["frames_ok"], "/", c["F"], "ok", flush=True)
    path = os.path.join(HERE, "reference_digests.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
