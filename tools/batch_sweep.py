"""Decode time against batch size for one code on the resident-frame path (pcg_decode_f32 on the
specialised kernel): time(F) = fixed + F / rate separates the per-launch cost (launch, queue reset,
the tail of waves finishing their last codeword group) from the steady-state rate.
    python tools/batch_sweep.py [N K L]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from antpolarcodes_amd import frames  # noqa: E402
from antpolarcodes_amd._native import Plan  # noqa: E402
from antpolarcodes_amd.construction import frozen_bits  # noqa: E402

N, K, L = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (1024, 512, 8)
fr = frozen_bits(N, K, 0.0)
Fmax = 1 << 18
llr, _, _ = frames.awgn_frames(N, fr, 1 << 16, 2.0, seed=9, crc=8)
d = torch.from_numpy(np.tile(llr, (Fmax >> 16, 1))).cuda()
p = Plan(N, L, fr, crc=8, device=0)
p.specialize()
info = torch.empty((Fmax, p.kb), dtype=torch.uint8, device="cuda")
rows = []
for lg in range(12, 19):
    F = 1 << lg
    x, o = d[:F], info[:F]
    for _ in range(2):
        p.decode_device(x, o)
    torch.cuda.synchronize()
    reps = max(3, min(20, (1 << 20) // F))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        p.decode_device(x, o)
        b.record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    rows.append((F, ms))
    print(f"F = 2^{lg:2d}: {ms:8.3f} ms per launch, {F / ms * 1e3:.4g} cw/s", flush=True)
# least squares over the batches of >= 4 rounds of groups
A = np.array([[1.0, F] for F, ms in rows if F >= 1 << 15])
y = np.array([ms for F, ms in rows if F >= 1 << 15])
fixed, per = np.linalg.lstsq(A, y, rcond=None)[0]
print(f"fit over F >= 2^15: fixed {fixed:.3f} ms per launch + {per * 1e6:.3f} ns per frame "
      f"(steady state {1e3 / per:.4g} cw/s)")
