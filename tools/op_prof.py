"""Per-op-code cycle profile of a decode kernel (PCG_OPPROF=1 must be set before the plan
is created).  Development aid: python tools/op_prof.py [L] (defaults to Fast-SSC)."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PCG_OPPROF"] = "1"
import torch  # noqa: E402
from antpolarcodes_amd import frames, _native  # noqa: E402
from antpolarcodes_amd._native import Plan  # noqa: E402
from antpolarcodes_amd.construction import frozen_bits  # noqa: E402
L = int(sys.argv[1]) if len(sys.argv) > 1 else 1
N, K, F = 1024, 512, 1 << 16
fz = frozen_bits(N, K, 0.0, "BB")
llr, info, _ = frames.awgn_frames(N, fz, F, 2.0, seed=1, crc=8)
p = Plan(N, L, fz, crc=8)
d = torch.from_numpy(llr).cuda()
di = torch.zeros((F, p.kb), dtype=torch.uint8, device="cuda")
do = torch.zeros(F, dtype=torch.uint8, device="cuda")
buf = (C.c_ulonglong * 128)()
p.decode_device(d, di, do)
torch.cuda.synchronize()
_native.lib().pcg_dev_opprof_fetch(buf)  # discard the first launch
p.decode_device(d, di, do)
torch.cuda.synchronize()
_native.lib().pcg_dev_opprof_fetch(buf)
names = {1: "F", 2: "G", 3: "G0", 4: "COMB", 5: "COPY0", 6: "RONE", 16: "R0", 17: "R1", 18: "REP", 19: "SPC",
         20: "DREP", 21: "DSPC", 22: "DSPC8", 23: "TREP", 24: "TYPE5", 25: "REPR1", 26: "ZSPC8", 27: "ZSPC",
         15: "output", 30: "Q16F", 31: "Q16G", 28: "Q16", 29: "Q16R"}
tot = sum(buf[2 * b] for b in range(64))
print(f"kernel {p.kernel_name()}: total {tot:.3e} wave-cycles")
rows = []
for b in range(64):
    if buf[2 * b]:
        nm = names.get(b & 31, str(b & 31)) + (" (s>=8)" if b >= 32 else "")
        rows.append((buf[2 * b], nm, buf[2 * b + 1]))
for cyc, nm, cnt in sorted(rows, reverse=True):
    print(f"  {nm:14s} {100 * cyc / tot:5.1f}%  {cyc / max(cnt, 1):8.0f} cycles/op  ({cnt} ops)")
