"""Reconcile a rocprofv3 kernel trace with bench lines (evidence aid).

    python tools/reconcile_profile.py <kernel_trace.csv> <kernel> <warmup> <profiled.json> [<bench.json>]

The profiled run is `bench.py ... --warmup W` under `rocprofv3 --kernel-trace --stats`: its first
W launches of <kernel> are the warm-up, the rest are the timed steps.  Prints the trace's average
over the timed launches beside (a) the profiled run's own kernel_ms (HIP events on the launch
stream, same launches: must agree) and (b) an unprofiled bench line's kernel_ms (another run: the
chip's clock under the profiler differs), and the roofline fraction recomputed from each."""
import csv
import json
import sys


def line(path):
    return json.loads([ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1])


def main():
    trace, kernel, warm = sys.argv[1], sys.argv[2], int(sys.argv[3])
    base = kernel.split("<")[0]  # ("sclls_kernel<8>": rocprof names "...sclls_kernel<8>(pcg::KernelArgs)")
    rows = [r for r in csv.DictReader(open(trace)) if base in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]
    timed = durs[warm:]
    avg = sum(timed) / len(timed)
    print(f"{kernel}: {len(durs)} launches in the trace, {len(timed)} timed (after {warm} warm-up): "
          f"average {avg:.4f} ms, min {min(timed):.4f}, max {max(timed):.4f}; all launches {sum(durs) / len(durs):.4f}")
    for tag, path in zip(("profiled run", "bench line"), sys.argv[4:6]):
        d = line(path)
        r = d["roofline"]
        fpl, bpc, peak = r["frames_per_launch"], r["algorithmic_bytes_per_codeword"], r["peak"]
        frac_trace = fpl * bpc / (avg * 1e-3) / 1e9 / peak
        if r.get("kernel_ms_scope"):  # adaptive modes: the events bracket more than this kernel
            print(f"  ({tag}: kernel_ms is {r['kernel_ms_scope']} -- not this kernel's own time)")
        print(f"  {tag:12s} kernel_ms {r['kernel_ms']:.4f} (trace/events {avg / r['kernel_ms']:.3f}), "
              f"ms_per_step {d['ms_per_step']:.4f}, frac {r['frac']:.5f} vs {frac_trace:.5f} from the trace "
              f"({100 * (frac_trace / r['frac'] - 1):+.1f} %)")


if __name__ == "__main__":
    main()
