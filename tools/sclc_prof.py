"""Per-phase cycle profile of the int8 SCL kernel (development aid).
Build altlib/libpcg_prof.so with -DPCG_SCLC_PROF (tools/build_prof.sh), then run with
PCG_DEV_LIB=altlib/libpcg_prof.so PCG_OPPROF=1 python tools/sclc_prof.py"""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from antpolarcodes_amd import frames, _native
from antpolarcodes_amd._native import Plan
from antpolarcodes_amd.construction import frozen_bits
N, K, L, F = 1024, 512, 8, 1 << 16
fz = frozen_bits(N, K, 0.0, "BB")
llr, info, _ = frames.awgn_frames(N, fz, F, 2.0, seed=1, crc=8)
x8 = np.clip(np.rint(llr * 10), -128, 127).astype(np.int8)
p = Plan(N, L, fz, crc=8, fixed=True)
d = torch.from_numpy(x8).cuda()
di = torch.zeros((F, p.kb), dtype=torch.uint8, device="cuda")
do = torch.zeros(F, dtype=torch.uint8, device="cuda")
for _ in range(2):
    p.decode_device_i8(d, di, do)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 128)()
_native.lib().pcg_dev_opprof_fetch(buf)
names = {1: "F", 2: "G", 4: "COMB", 16: "R0", 17: "R1 cand", 18: "Rep cand", 19: "SPC cand", 20: "pruning",
         21: "survivors", 22: "final"}
groups = max(buf[62], 1)
tot = buf[61]
print(f"groups {buf[62]}  cycles/group {tot / groups:.0f}")
for b in range(61):
    if buf[b]:
        print(f"  {names.get(b, b):10s} {buf[b] / groups:10.0f} cycles/group  {100 * buf[b] / tot:5.1f}%")
