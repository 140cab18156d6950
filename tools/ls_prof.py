"""Per-op-class cycle profile of the lane-serial SCL kernel (build with -DPCG_LS_PROF;
run with PCG_OPPROF=1).  Development aid."""
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
p = Plan(N, L, fz, crc=8)
d = torch.from_numpy(llr).cuda()
di = torch.zeros((F, p.kb), dtype=torch.uint8, device="cuda")
do = torch.zeros(F, dtype=torch.uint8, device="cuda")
reps = 3
for _ in range(reps):
    p.decode_device(d, di, do)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 128)()
_native.lib().pcg_dev_opprof_fetch(buf)
names = {1: "F lds", 2: "G lds", 9: "F gl->gl", 10: "G gl->gl", 17: "F virt", 18: "G virt", 25: "F gl->lds",
         26: "G gl->lds", 4: "COMB", 40: "R0", 41: "R1", 43: "SPC", 44: "ST8", 60: "final", 50: "~select", 51: "~dup", 52: "~st8 move", 53: "~weak"}
groups = buf[62]
tot = buf[61]
print(f"groups {groups}  cycles/group {tot / max(groups, 1):.0f}")
for b in range(61):
    if buf[b]:
        print(f"  {names.get(b, b):10s} {buf[b] / groups:10.0f} cycles/group  {100 * buf[b] / tot:5.1f}%")
