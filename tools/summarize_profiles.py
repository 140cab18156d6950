"""Collect a gpurun_out/<tag> profile run into profiles/ (committed evidence).

HBM bytes per launch from FETCH_SIZE / WRITE_SIZE (rocprofv3, KB units), corrected
per MI355X_MICROARCH.md §HBM: FETCH_SIZE reads exactly 1/2 of the bytes of wide
coalesced streaming reads on gfx950 -> doubled; WRITE_SIZE taken as is."""
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
kern = sys.argv[2] if len(sys.argv) > 2 else "scl_kernel"
src = os.path.join("gpurun_out", tag)
dst = "profiles"
os.makedirs(dst, exist_ok=True)


def counter(path, name):
    vals = []
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == name:
            vals.append(float(r["Counter_Value"]))
    return vals


fetch = counter(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
write = counter(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
bench = json.load(open(os.path.join(src, "bench_scl8.json")))
F = bench["config"]["frames_per_step_per_gpu"]
fb = 2 * 1024 * fetch[-1]
wb = 1024 * write[-1]
tr = {"kernel": kern, "launch_frames": F, "fetch_size_kb_raw": fetch[-1], "write_size_kb_raw": write[-1],
      "hbm_read_bytes_per_launch": fb, "hbm_write_bytes_per_launch": wb,
      "hbm_bytes_per_launch": fb + wb, "hbm_bytes_per_codeword": (fb + wb) / F,
      "algorithmic_bytes_per_codeword": bench["roofline"]["algorithmic_bytes_per_codeword"],
      "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount, MI355X_MICROARCH.md HBM)"}
json.dump(tr, open(os.path.join(dst, "traffic_scl8.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "stats", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_scl8_kernel_stats.csv"))
shutil.copy(os.path.join(src, "bench_scl8.json"), os.path.join(dst, f"{tag}_bench_scl8.json"))
shutil.copy(os.path.join(src, "bench_sc.json"), os.path.join(dst, f"{tag}_bench_sc.json"))
sq = {}
for r in csv.DictReader(open(os.path.join(src, "sq", "run_counter_collection.csv"))):
    if kern in r["Kernel_Name"]:
        sq[r["Counter_Name"]] = float(r["Counter_Value"])
sq["frames_per_launch"] = F
json.dump(sq, open(os.path.join(dst, f"{tag}_scl8_sq_counters.json"), "w"), indent=1)
print(json.dumps(tr, indent=1))
