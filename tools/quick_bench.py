"""Quick device-resident throughput probe (development aid, not the contract bench)."""
import argparse
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from antpolarcodes_amd import frames
from antpolarcodes_amd._native import Plan

ap = argparse.ArgumentParser()
ap.add_argument("--N", type=int, default=1024)
ap.add_argument("--K", type=int, default=512)
ap.add_argument("--L", type=int, default=1)
ap.add_argument("--F", type=int, default=1 << 16)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
sys.path.insert(0, "oracle")
from pyoracle import Oracle
fr = Oracle().frozen_bits_bb(a.N, a.K, 0.0)
llr, info, _ = frames.awgn_frames(a.N, fr, a.F, 2.0, seed=1, crc=8)
p = Plan(a.N, a.L, fr, crc=8)
print(p.describe())
d_llr = torch.from_numpy(llr).cuda()
d_info = torch.zeros((a.F, p.kb), dtype=torch.uint8, device="cuda")
d_ok = torch.zeros(a.F, dtype=torch.uint8, device="cuda")
for _ in range(3):
    p.decode_device(d_llr, d_info, d_ok)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.reps):
    p.decode_device(d_llr, d_info, d_ok)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.reps
cw = a.F / (ms * 1e-3)
print(f"N={a.N} K={a.K} L={a.L} F={a.F}: {ms:.3f} ms/launch  {cw:.3e} cw/s  {cw*(4*a.N+a.K/8)/1e9:.1f} GB/s  ok={d_ok.float().mean().item():.4f}")
