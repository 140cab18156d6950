"""Per-op cycle profile of sclls_kernel (development aid).  Needs a libpcg built with
-DPCG_LS_PROF (tools/build_dev_lib.sh ls_prof -DPCG_LS_PROF) selected by PCG_DEV_LIB:
    PCG_DEV_LIB=lib_dev/libpcg_ls_prof.so python tools/ls_prof.py [L [N [F]]]
Buckets (sclls_kernel.hip, PCG_LS_PROF): op code, +8 for a global-slab source stage,
+16 for a recomputed (root child) source stage, +24 for an LDS source feeding a global
output; 60 = extractBestPath + output.  Sub-buckets, also counted inside their op's
bucket: 50 = path selection (ls_select, sort + merge rounds / bitonic merge), 51 = path
duplication (ls_dup: slot row + codeword prefix copy), 52 = survivor register shuffle
inside size-8 subtrees (st8_branch), 53 = weak-LLR search of Rate-1 / SPC leaves n >= 8
(weak_fast, ls_weak on ties).  Beside the cycles: the global bytes each op bucket requests
(loads, LDS DMA and stores through the slab / channel / D-region accessors, per codeword) --
what the L1 asks of L2, against which the measured HBM traffic (FETCH_SIZE + WRITE_SIZE) of
the bench line is the L2 / MALL-filtered part."""
import ctypes as C
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PCG_OPPROF"] = "1"
import torch  # noqa: E402
from antpolarcodes_amd import frames, _native  # noqa: E402
from antpolarcodes_amd._native import Plan  # noqa: E402
from antpolarcodes_amd.construction import frozen_bits  # noqa: E402
L = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
F = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 16
K = N // 2
fz = frozen_bits(N, K, 0.0, "BB")
llr, info, _ = frames.awgn_frames(N, fz, F, 2.0, seed=1, crc=8)
p = Plan(N, L, fz, crc=8)
d = torch.from_numpy(llr).cuda()
di = torch.zeros((F, p.kb), dtype=torch.uint8, device="cuda")
do = torch.zeros(F, dtype=torch.uint8, device="cuda")
buf = (C.c_ulonglong * 256)()
p.decode_device(d, di, do)
torch.cuda.synchronize()
_native.lib().pcg_dev_opprof_fetch_n(buf, 256)  # discard the first launch
p.decode_device(d, di, do)
torch.cuda.synchronize()
_native.lib().pcg_dev_opprof_fetch_n(buf, 256)
base = {1: "F", 2: "G", 4: "COMB", 40: "R0", 41: "R1", 42: "REP", 43: "SPC", 44: "ST8", 60: "output",
        50: "  [path selection]", 51: "  [path duplication]", 52: "  [st8 survivor shuffle]",
        53: "  [weak-LLR search]"}
cls = {0: "", 8: " (global src)", 16: " (root child)", 24: " (LDS src, global dst)"}
whole = buf[61]
print(f"kernel {p.kernel_name()}: {whole:.3e} wave-cycles over {buf[62]} codeword groups")
rows = []
for b in range(60):
    if buf[b]:
        if b < 32 and (b & 7) in (1, 2):
            nm = base[b & 7] + cls[b & 24]
        else:
            nm = base.get(b, str(b))
        rows.append((buf[b], nm))
rows.append((buf[60], "output"))
for cyc, nm in sorted(rows, reverse=True):
    print(f"  {nm:20s} {100 * cyc / max(whole, 1):5.1f}%")
# requested global bytes per codeword and op bucket (G = 64 / LP codewords per group)
lp = 1
while lp < L:
    lp <<= 1
ncw = max(buf[62], 1) * (64 // lp)
print(f"requested global bytes per codeword by op bucket (loads incl. LDS DMA / stores), {ncw} codewords:")
tr = tw = 0
brow = []
for b in range(60):
    r, w = buf[64 + b], buf[128 + b]
    if r or w:
        nm = base[b & 7] + cls[b & 24] if b < 32 and (b & 7) in (1, 2) else base.get(b, str(b))
        brow.append((r + w, nm, r, w))
        tr += r
        tw += w
for _, nm, r, w in sorted(brow, reverse=True):
    print(f"  {nm:24s} read {r / ncw:9.0f} B  write {w / ncw:9.0f} B  ({100 * (r + w) / max(tr + tw, 1):5.1f}%)")
print(f"  {'total':24s} read {tr / ncw:9.0f} B  write {tw / ncw:9.0f} B")
