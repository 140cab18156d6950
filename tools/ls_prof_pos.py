"""Per-schedule-position cycle profile of sclls_kernel (development aid).  Needs a libpcg built
with -DPCG_LS_PROF -DPCG_LS_PROF_POS (tools/build_dev_lib.sh ls_pos sclls_kernel.hip -DPCG_LS_PROF
-DPCG_LS_PROF_POS) selected by PCG_DEV_LIB:
    PCG_DEV_LIB=lib_dev/libpcg_ls_pos.so python tools/ls_prof_pos.py [L [N [F [char]]]]
The 8-bit list kernel (scl_char_kernel.hip) likewise, from a build with -DPCG_SCLC_PROF
-DPCG_SCLC_PROF_POS and the trailing argument `char` (int8 frames, x10 amplification as bench.py).
Prints every op of the schedule (code, stage, offset) with its wave-cycles per codeword group,
its share of the walk, and the cumulative share, then the positions sorted by cost."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PCG_OPPROF"] = "1"
import torch  # noqa: E402
from antpolarcodes_amd import frames, _native  # noqa: E402
from antpolarcodes_amd._native import Plan  # noqa: E402
from antpolarcodes_amd.construction import frozen_bits  # noqa: E402

NAMES = {1: "F", 2: "G", 3: "G0", 4: "COMB", 40: "R0", 41: "R1", 42: "REP", 43: "SPC", 44: "ST8",
         80: "R0", 81: "R1", 82: "REP", 83: "SPC"}
L = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
F = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 16
CHAR = len(sys.argv) > 4 and sys.argv[4] == "char"
fz = frozen_bits(N, N // 2, 0.0, "BB")
llr, info, _ = frames.awgn_frames(N, fz, F, 2.0, seed=1, crc=8)
if CHAR:  # (bench.py CHAR_AMP)
    import numpy as np
    llr = np.clip(np.rint(llr * 10.0), -128, 127).astype(np.int8)
p = Plan(N, L, fz, crc=8, fixed=CHAR)
lib = _native.lib()
ops = (C.c_uint32 * 4096)()
nops = lib.pcg_dev_plan_ops(p._h, ops, 4096)
d = torch.from_numpy(llr).cuda()
di = torch.zeros((F, p.kb), dtype=torch.uint8, device="cuda")
do = torch.zeros(F, dtype=torch.uint8, device="cuda")
buf = (C.c_ulonglong * 4096)()
dec = p.decode_device_i8 if CHAR else p.decode_device
dec(d, di, do)
torch.cuda.synchronize()
lib.pcg_dev_opprof_fetch_n(buf, 4096)  # discard the first launch
dec(d, di, do)
torch.cuda.synchronize()
lib.pcg_dev_opprof_fetch_n(buf, 4096)
groups = max(buf[62], 1)
walk = buf[61] / groups
print(f"kernel {p.kernel_name()}: {walk:.0f} wave-cycles per codeword group walk, {groups} groups, {nops} words")
rows, cum = [], 0.0
for k in range(min(nops, 3840)):
    cyc = buf[256 + k] / groups
    if cyc == 0:
        continue
    w = ops[k]
    code, st, off = w & 0xFF, (w >> 8) & 0xFF, w >> 16
    cum += cyc
    nm = NAMES.get(code, str(code))
    rows.append((cyc, k, nm, st, off))
    print(f"  [{k:4d}] {nm:5s} s={st:2d} o={off:5d} {cyc:9.0f} cyc {100 * cyc / walk:5.2f} %  cum {100 * cum / walk:6.2f} %")
print("most expensive positions:")
for cyc, k, nm, st, off in sorted(rows, reverse=True)[:40]:
    print(f"  [{k:4d}] {nm:5s} s={st:2d} o={off:5d} {cyc:9.0f} cyc {100 * cyc / walk:5.2f} %")
