"""Host-buffer decode rate (pcg_decode_f32_host) across the pipeline's staging modes, host
threads and chunk sizes (capi.cpp decode_host; the variables are read per call), for a
resident numpy batch of config 3 (SCL-8, N=1024, 2^16 frames) -- and from a page-locked
caller buffer, which the pipeline copies from directly.
    python tools/host_pipe_sweep.py [mode: scl8|sc] [pieces]
`pieces`: only the pinned-staging mode over staging piece sizes (PCG_HOST_PIECE_MB), staging
threads and chunk sizes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from antpolarcodes_amd import frames  # noqa: E402
from antpolarcodes_amd._native import Plan  # noqa: E402
from antpolarcodes_amd.construction import frozen_bits  # noqa: E402

L = 1 if len(sys.argv) > 1 and sys.argv[1] == "sc" else 8
N, K, F = 1024, 512, 1 << 16
fr = frozen_bits(N, K, 0.0)
llr, _, _ = frames.awgn_frames(N, fr, F, 2.0, seed=5, crc=8)
p = Plan(N, L, fr, crc=8, device=0)
p.specialize()
ref, _, _ = p.decode_host(llr)


def rate(x, fresh=False, **env):
    """best of 3 timed calls; fresh: every call on a newly written copy of the batch (a caller
    whose buffer the library has never seen)"""
    for k, v in env.items():
        os.environ[k] = str(v)
    try:
        gi, _, _ = p.decode_host(x)
        assert np.array_equal(gi, ref)
        best = 0.0
        for _ in range(3):
            y = x.copy() if fresh else x
            t0 = time.perf_counter()
            gi, _, _ = p.decode_host(y)
            best = max(best, F / (time.perf_counter() - t0))
            assert np.array_equal(gi, ref)
        return best
    finally:
        for k in env:
            del os.environ[k]


# device-resident rate for reference
d = torch.from_numpy(llr).cuda()
info = torch.empty((F, p.kb), dtype=torch.uint8, device="cuda")
p.decode_device(d, info)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    p.decode_device(d, info)
torch.cuda.synchronize()
print(f"device-resident {5 * F / (time.perf_counter() - t0):.4g} cw/s")
t0 = time.perf_counter()
h = d.cpu()
print(f"D2H of the batch (torch, pageable) {llr.nbytes / (time.perf_counter() - t0) / 1e9:.1f} GB/s")
pinned = torch.from_numpy(llr).pin_memory()
t0 = time.perf_counter()
d.copy_(pinned, non_blocking=True)
torch.cuda.synchronize()
print(f"H2D of the batch (torch, pinned) {llr.nbytes / (time.perf_counter() - t0) / 1e9:.1f} GB/s")
print(f"serial (PCG_HOST_PIPE=0) {rate(llr, PCG_HOST_PIPE=0):.4g} cw/s")
if "pieces" in sys.argv[1:]:
    for chunk in (16384, 32768):
        print(f"page-locked caller buffer, chunk {chunk}: {rate(pinned.numpy(), PCG_HOST_CHUNK=chunk):.4g} cw/s")
    for thr in (8, 12):
        for chunk in (8192, 16384):
            for pmb in (0, 8, 16):
                for fkb in ((16384, 2048, 256) if pmb else (2048,)):
                    r = rate(llr, PCG_HOST_PIPE=2, PCG_HOST_THREADS=thr, PCG_HOST_CHUNK=chunk, PCG_HOST_PIECE_MB=pmb,
                             PCG_HOST_FIRST_KB=fkb)
                    print(f"pinned staging (2), {thr} threads, chunk {chunk}, piece {pmb} MB, first piece {fkb} KB: "
                          f"{r:.4g} cw/s", flush=True)
    sys.exit(0)
for chunk in (16384, 32768):
    print(f"pageable runtime copies (1), chunk {chunk}: {rate(llr, PCG_HOST_PIPE=1, PCG_HOST_CHUNK=chunk):.4g} cw/s")
for thr in (8, 16):
    for chunk in (8192, 16384, 32768):
        r = rate(llr, PCG_HOST_PIPE=2, PCG_HOST_THREADS=thr, PCG_HOST_CHUNK=chunk)
        rf = rate(llr, fresh=True, PCG_HOST_PIPE=2, PCG_HOST_THREADS=thr, PCG_HOST_CHUNK=chunk)
        print(f"pinned staging (2), {thr} threads, chunk {chunk}: {r:.4g} cw/s, fresh buffers {rf:.4g}")
for chunk in (8192, 16384, 32768):
    r = rate(llr, PCG_HOST_PIPE=3, PCG_HOST_CHUNK=chunk)
    rf = rate(llr, fresh=True, PCG_HOST_PIPE=3, PCG_HOST_CHUNK=chunk)
    print(f"pages locked in place per chunk (3), chunk {chunk}: {r:.4g} cw/s, fresh buffers {rf:.4g}")
for chunk in (8192, 16384, 32768):
    print(f"page-locked caller buffer, chunk {chunk}: {rate(pinned.numpy(), PCG_HOST_CHUNK=chunk):.4g} cw/s")

# the price of page-locking the caller's buffer per call (hipHostRegister / hipHostUnregister,
# through torch's runtime bindings: the process has one HIP runtime)
rt = torch.cuda.cudart()
x = np.ascontiguousarray(llr)
for _ in range(2):
    t0 = time.perf_counter()
    rc = rt.cudaHostRegister(x.ctypes.data, x.nbytes, 0)
    t1 = time.perf_counter()
    rc2 = rt.cudaHostUnregister(x.ctypes.data)
    t2 = time.perf_counter()
    print(f"hipHostRegister {x.nbytes >> 20} MiB: rc {rc}, {1e3 * (t1 - t0):.2f} ms; unregister rc {rc2}, "
          f"{1e3 * (t2 - t1):.2f} ms")
