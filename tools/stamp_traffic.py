"""Write profiles/traffic_<mode>.json from a bench.py JSON line whose roofline carries a
measured traffic figure, stamped with the kernel name and the source digest of the run
(bench.py only reuses such a file for the same kernel and sources)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(mode, bench_json):
    with open(bench_json) as fh:
        d = json.loads([ln for ln in fh if ln.startswith("{")][-1])
    r = d["roofline"]
    if r.get("traffic") is None:
        sys.exit(f"{bench_json}: no measured traffic")
    out = {"kernel": r["kernel"], "src_digest": d["src_digest"], "git_head": d.get("git_head"),
           "frames_per_launch": r["frames_per_launch"], "bytes_per_codeword": r["traffic_bytes_per_codeword"],
           "bytes_per_launch": r["traffic"], "algorithmic_bytes_per_codeword": r["algorithmic_bytes_per_codeword"],
           "kernel_ms": r["kernel_ms"], "source_run": os.path.basename(bench_json),
           "correction": "FETCH_SIZE x1024 x2 (gfx950), WRITE_SIZE x1024"}
    with open(os.path.join(ROOT, "profiles", f"traffic_{mode}.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
