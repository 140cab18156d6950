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

if os.environ.get("PCG_OPPROF"):
    import ctypes as C
    from antpolarcodes_amd import _native
    buf = (C.c_ulonglong * 128)()
    _native.lib().pcg_dev_opprof_fetch(buf)
    names = {1: "F", 2: "G", 3: "G0", 4: "COMB", 5: "COPY0", 6: "RONE", 16: "L_R0", 17: "L_R1", 18: "L_REP", 19: "L_SPC",
             20: "L_DREP", 21: "L_DSPC", 22: "L_DSPC8", 23: "L_TREP", 24: "L_TYPE5", 25: "L_REPR1", 26: "L_ZSPC8",
             27: "L_ZSPC", 40: "S_R0", 41: "S_R1", 42: "S_REP", 43: "S_SPC", 44: "S_ST8",
             48: "~weak", 49: "~cand", 50: "~sort", 51: "~commit"}
    tot = sum(buf[2 * c] for c in range(48))
    frames_done = a.F * (a.reps + 3)
    for c in range(64):
        cyc, cnt = buf[2 * c], buf[2 * c + 1]
        if c >= 48 and cyc:
            print(f"  phase {names.get(c, c):8s} cycles/frame {cyc / frames_done:9.0f}")
        elif cnt:
            print(f"  op {names.get(c, c):8s} count/frame {cnt / frames_done:7.1f}  cycles/op {cyc / cnt:9.0f}  share {100 * cyc / tot:5.1f}%  cycles/frame {cyc / frames_done:9.0f}")
    print(f"  total op cycles per frame (per wave): {tot / frames_done:.0f}")
