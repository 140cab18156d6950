#!/usr/bin/env python3
"""bench.py -- headline benchmark: batched CRC-aided SCL (L=8) polar decoding,
N=1024 K=512 (BASELINE.json metric; config 3), on 1..8 MI355X.

A "step" is one decode of a resident batch of synthetic BPSK-AWGN frames (Eb/N0 =
2 dB, Bhattacharyya construction at 0 dB, CRC-8 appended by the encoder and checked
by the decoder) through the C ABI (pcg_decode_f32) on the GPU.  Frames are
independent, so ranks shard with no data-path collective; the barrier and the
max-over-ranks timing go through gloo on the host.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--mode MODE]
  --gpus N > 1 without a torch.distributed.run environment: this process starts N
  rank processes itself (it never touches the GPU), relays rank 0's JSON line and
  fails if any rank fails.
Prints ONE JSON line on rank 0.

roofline: `achieved`/`frac` use the algorithmic bytes (LLRs in, info bytes + ok flag
[+ metrics] out) over the decode time measured with HIP events on the launch
stream; `traffic` is the FETCH_SIZE/WRITE_SIZE bytes per launch of the same kernel,
measured by rocprofv3 child runs of this script (--traffic, default at N=1) or read
from profiles/traffic_<mode>.json only when that file names the same kernel and the
same source digest.
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODES = {
    # name: (N, K, L, frames per step (per GPU; global for *_strong), workload text)
    "scl8": (1024, 512, 8, 1 << 16, "config 3: CRC-aided SCL L=8, N=1024 K=512, 2^16 AWGN frames"),
    "sc": (1024, 512, 1, 1 << 16, "config 2: batched Fast-SSC, N=1024 K=512, 2^16 AWGN frames"),
    "scl32": (4096, 2048, 32, 1 << 17, "config 5 per-GPU shard: SCL L=32, N=4096 K=2048, 2^17 frames per GPU "
                                       "(= 2^20 / 8), weak scaling"),
    "scl32_strong": (4096, 2048, 32, 1 << 20, "config 5: SCL L=32, N=4096 K=2048, one 2^20-frame batch split "
                                              "into contiguous shards over the ranks (strong scaling)"),
    "nr5g": (1024, 512, 8, 1 << 16, "config 4: 5G NR uplink, FiveGList N=1024 K=512 (501 + CRC-11), "
                                     "punctured to E=896, device depuncture + SCL L=8, 2^16 frames"),
    "adaptive8": (1024, 512, 8, 1 << 16, "config 3 with the adaptive decoder (AdaptiveFloat): Fast-SSC, "
                                         "then SCL L=8 for CRC-8 failures, N=1024 K=512, 2^16 frames"),
    "sc_char": (1024, 512, 1, 1 << 16, "config 2 through the 8-bit decoder (FastSscFipChar): int8 LLRs "
                                       "(amplification 10, pcsim's amp-fixed), N=1024 K=512, 2^16 frames"),
    "scl8_char": (1024, 512, 8, 1 << 16, "config 3 through the 8-bit decoder (SclFipChar): int8 LLRs "
                                         "(amplification 10, pcsim's amp-fixed), N=1024 K=512, 2^16 frames"),
    "adaptive8_char": (1024, 512, 8, 1 << 16, "config 3 with pcsim's 8-bit list decoder (AdaptiveChar): "
                                              "FastSscFipChar, then SclFipChar L=8 for CRC-8 failures, int8 LLRs "
                                              "(amplification 10), N=1024 K=512, 2^16 frames"),
}
HEADLINE_METRIC = "codewords/s + info-bits/s, N=1024 K=512 SCL L=8, 1/2/4/8 MI355X"
CHAR_AMP = 10.0  # src/simulation/setup.cpp:58 "amp-fixed" (8-bit pre-quantisation scaling)
NR_E = 896
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
FETCH_CORRECTION = 2.0  # MI355X_MICROARCH.md (HBM): FETCH_SIZE counts half the bytes of 16 B/lane reads
SRC_DIRS = ("antpolarcodes_amd/csrc",)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--mode", default="scl8", choices=sorted(MODES))
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (0: the job's CPU share, OMP_NUM_THREADS, else every "
                         "CPU in this process's affinity mask)")
    ap.add_argument("--traffic", dest="traffic", action="store_true", default=None,
                    help="measure FETCH/WRITE bytes with rocprofv3 child runs (default on at N=1)")
    ap.add_argument("--no-traffic", dest="traffic", action="store_false")
    ap.add_argument("--no-host-rate", action="store_true", help="skip the PCIe-inclusive host-buffer rate")
    ap.add_argument("--no-copy-bw", action="store_true", help="skip the device copy-bandwidth probe")
    ap.add_argument("--in-flight", action="store_true",
                    help="also time the same steps with a second batch in flight (second plan and stream): "
                         "reported as roofline.throughput_2_in_flight_cw_per_s, never as value (off by default: "
                         "its overlapping launches would skew a profiler's per-launch average)")
    ap.add_argument("--no-in-flight", dest="single_stream", action="store_true",
                    help="one batch at a time: no second-batch figure, and one stream for every mode (profiling "
                         "and traffic runs: per-launch kernel statistics without overlapping launches)")
    ap.add_argument("--streams", type=int, default=0,
                    help="batches in flight: S plans on S HIP streams, step i on stream i %% S (default: 2 for "
                         "the adaptive modes, whose latency-bound list stage then overlaps the next batch's "
                         "Fast-SSC stage; 1 otherwise)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / reduction plumbing only: no GPU, no decode (CPU tests)")
    a = ap.parse_args(argv)
    if a.single_stream:
        a.in_flight = False
    return a


# --------------------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """--gpus N outside torch.distributed.run: start N rank processes of this script
    (subprocess, no exec; this parent never initialises the GPU), relay rank 0's
    stdout, return the first non-zero exit code of any rank."""
    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(),
                                      text=True))
    out = procs[0].communicate()[0]
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    if out:
        sys.stdout.write(out)
        sys.stdout.flush()
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        print(f"[bench] rank exit codes {rcs}", file=sys.stderr)
        return bad[0] if bad[0] > 0 else 1
    return 0


# --------------------------------------------------------------------------- evidence
def src_digest():
    """sha256 over the native sources (the GPU box has no .git: this stamps a build)."""
    h = hashlib.sha256()
    for d in SRC_DIRS:
        for p in sorted(glob.glob(os.path.join(ROOT, d, "**", "*"), recursive=True)):
            if os.path.isfile(p) and p.endswith((".hip", ".cpp", ".hpp", ".h", ".inc", "Makefile")):
                h.update(os.path.relpath(p, ROOT).encode())
                with open(p, "rb") as fh:
                    h.update(fh.read())
    with open(os.path.join(ROOT, "include", "pcg.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def git_head():
    try:
        return subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                              text=True, timeout=10).stdout.strip() or None
    except Exception:
        return None


def _counter_rows(outdir):
    rows = []
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def specialize(plan):
    """Plan-specialised kernels (pcg_plan_specialize: hiprtc, float Fast-SSC and list plans,
    both stages of a float adaptive plan; the shipped cache holds the benchmark codes) before
    the warmup, so a compile is never timed and the kernel name is the one that runs.
    PCG_RTC=0 keeps the interpreter kernels."""
    from antpolarcodes_amd._native import PCG_E_UNSUPPORTED, PcgError
    if os.environ.get("PCG_RTC") == "0":
        return
    try:
        plan.specialize()
    except PcgError as e:
        if e.code != PCG_E_UNSUPPORTED:
            raise


def measure_traffic(args, kernel, frames):
    """FETCH_SIZE and WRITE_SIZE (one rocprofv3 --pmc pass each, as the guide requires)
    of the decode kernel over child runs of this script; per-launch median."""
    rocprof = shutil.which("rocprofv3")
    if not rocprof or not kernel:
        return None, "rocprofv3 not found" if not rocprof else "no kernel name"
    # "sclls_kernel<8>" matches rocprof's "...sclls_kernel<8>(pcg::KernelArgs)" and
    # "scq_kernel<16>" its "...scq_kernel<16, true, false>(...)": name + first template argument
    base = kernel.split("<")[0]
    targ = kernel[len(base) + 1:-1] if "<" in kernel else ""
    pats = (f"{base}<{targ}>", f"{base}<{targ},") if targ else (base,)
    vals = {}
    with tempfile.TemporaryDirectory(prefix="pcg_traffic_", dir="/tmp") as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            od = os.path.join(td, ctr)
            cmd = [rocprof, "--pmc", ctr, "-d", od, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--mode", args.mode, "--steps", "2", "--warmup", "1",
                   "--ebn0", str(args.ebn0), "--no-cpu-baseline", "--no-traffic", "--no-host-rate", "--no-copy-bw",
                   "--no-in-flight"]
            env = dict(os.environ, TMPDIR="/tmp")
            for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
                env.pop(k, None)
            # own process group, so a pass that overruns is killed with the application it profiles
            pr = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env,
                                  start_new_session=True)
            try:
                _, err = pr.communicate(timeout=240)
            except subprocess.TimeoutExpired:
                os.killpg(pr.pid, 9)
                pr.communicate()
                return None, f"rocprofv3 {ctr} pass timed out"
            if pr.returncode != 0:
                return None, f"rocprofv3 {ctr} pass failed (rc {pr.returncode}): {err[-300:]}"
            per = [float(row["Counter_Value"]) for row in _counter_rows(od)
                   if row.get("Counter_Name") == ctr and any(q in row.get("Kernel_Name", "") for q in pats)]
            if not per:
                return None, f"no {ctr} rows for {kernel}"
            per.sort()
            vals[ctr] = per[len(per) // 2]
    rd = vals["FETCH_SIZE"] * 1024.0 * FETCH_CORRECTION
    wr = vals["WRITE_SIZE"] * 1024.0
    return {"kernel": kernel, "frames_per_launch": frames, "fetch_size_kb_raw": vals["FETCH_SIZE"],
            "write_size_kb_raw": vals["WRITE_SIZE"], "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
            "bytes_per_launch": rd + wr, "bytes_per_codeword": (rd + wr) / frames,
            "correction": "FETCH_SIZE x1024 x2 (gfx950 16 B/lane read undercount, MI355X_MICROARCH.md HBM), "
                          "WRITE_SIZE x1024", "source": "measured now (rocprofv3 --pmc child runs)"}, None


def stamped_traffic(mode, kernel, digest):
    tfile = os.path.join(ROOT, "profiles", f"traffic_{mode}.json")
    if not os.path.exists(tfile):
        return None, "no measurement"
    try:
        with open(tfile) as fh:
            t = json.load(fh)
    except Exception as e:  # noqa: BLE001
        return None, f"unreadable {tfile}: {e}"
    if t.get("kernel") != kernel or t.get("src_digest") != digest:
        return None, (f"{os.path.basename(tfile)} is for kernel {t.get('kernel')!r} / sources "
                      f"{t.get('src_digest')!r}, this build runs {kernel!r} / {digest!r}: not used")
    t["source"] = f"profiles/traffic_{mode}.json (same kernel and source digest)"
    return t, None


def copy_bandwidth(torch, dev):
    """Device-to-device copy of 2 GiB, best of 5 (read + write bytes / time)."""
    n = 1 << 29
    a = torch.empty(n, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    best = 0.0
    for _ in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        best = max(best, 2 * 4 * n / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del a, b
    torch.cuda.empty_cache()
    return best


def cpu_threads(args):
    if args.cpu_threads > 0:
        return args.cpu_threads
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        return int(share)
    return len(os.sched_getaffinity(0))


def cpu_baseline(mode, N, L, frozen, llr, threads):
    """Reference AVX2 decoder (oracle/_ref, compiled from the reference sources) timed on
    this host on a bounded sample of the same frames; falls back to the C restatement
    (oracle/liboracle.so) if absent.  For nr5g the LLRs are the depunctured frames and the
    reference keeps the CRC-8 its makeDecoder installs (it has no CRC-11)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    fixed = mode.endswith("_char")
    visible = len(os.sched_getaffinity(0))
    note = (f"{threads} threads = this job's CPU share (OMP_NUM_THREADS) of {visible} CPUs visible"
            if os.environ.get("OMP_NUM_THREADS") else f"{threads} threads of {visible} CPUs visible")
    try:
        from pyoracle import Reference
        ref = Reference()
        F = llr.shape[0]

        def timed(nthreads, target):
            """a bounded sample of about `target` s: first a probe, then enough frames / repeats"""
            def go(reps, x):
                if fixed:
                    return ref.bench_char(N, L, frozen, x, threads=nthreads, reps=reps, crc=8)
                return ref.bench(N, L, frozen, x, threads=nthreads, reps=reps, crc=8)
            probe = llr[:min(F, max(nthreads * 4, 64 if nthreads == 1 else 256))]
            t0 = time.time()
            go(1, probe)
            per_frame = (time.time() - t0) / probe.shape[0]
            nfr = int(min(F, max(probe.shape[0], target / max(per_frame, 1e-9))))
            x = llr[:nfr]
            reps = 1
            if nfr == F and per_frame * F < target:
                reps = int(min(200, max(1, round(target / max(per_frame * F, 1e-6)))))
            t0 = time.time()
            cw = go(reps, x)
            return cw, nfr, reps, time.time() - t0

        cw, nfr, reps, wall = timed(threads, 8.0)
        # and one thread (all of the job's host cores and 1 thread)
        cw1, nfr1, reps1, wall1 = timed(1, 4.0)
        return {"value": cw, "unit": "codewords/s", "cores": threads, "kind": "reference",
                "host_cpus_visible": visible,
                "sample": f"{nfr} frames of the same workload x {reps} pass(es), one reference decoder per "
                          f"thread, {note} ({wall:.1f} s wall)",
                "single_thread": {"value": cw1, "unit": "codewords/s", "cores": 1,
                                  "sample": f"{nfr1} frames x {reps1} pass(es), one reference decoder "
                                            f"({wall1:.1f} s wall)"}}
    except FileNotFoundError:
        from pyoracle import Oracle
        orc = Oracle()
        F = min(llr.shape[0], 4096 if L > 1 else 65536)
        if fixed:  # the int8 restatement, timed directly
            t0 = time.time()
            if L > 1:
                orc.sclc_decode(N, L, frozen, llr[:F], crc=8)
            else:
                orc.scc_decode(N, frozen, llr[:F], crc=8)
            cw = F / (time.time() - t0)
        else:
            cw = orc.bench(N, L, frozen, llr[:F], reps=1)
        return {"value": cw, "unit": "codewords/s", "cores": 1, "kind": "port", "host_cpus_visible": visible,
                "sample": f"{F} frames of the same workload, 1 thread (oracle restatement)"}


# --------------------------------------------------------------------------- frames
def device_frames(torch, N, frozen, F, ebn0, seed, crc, dev):
    """Frames generated on the device (config 5 sizes: 2^17 x 4096 LLRs = 2 GiB per GPU):
    Philox info bits -> detector generate + systematic ButterflyFipPacked encode ->
    BPSK-AWGN LLRs (pcg_random_info / pcg_encode / pcg_bpsk_awgn_f32)."""
    from antpolarcodes_amd._native import Encoder, bpsk_awgn_device, random_info_device
    K = N - len(frozen)
    kb = (K + 7) // 8
    info = torch.empty((F, kb), dtype=torch.uint8, device=dev)
    code = torch.empty((F, N // 8), dtype=torch.uint8, device=dev)
    llr = torch.empty((F, N), dtype=torch.float32, device=dev)
    random_info_device(info, K, seed)
    enc = Encoder(N, frozen, systematic=True, crc=crc, device=dev.index)
    enc.encode_device(info, code)
    esn0 = 10.0 ** (ebn0 / 10.0) * K / N
    sigma = 1.0 / (2.0 * esn0) ** 0.5
    bpsk_awgn_device(code, N, sigma, seed ^ 0x5DEECE66D, llr)
    torch.cuda.synchronize()
    enc.close()
    del code
    return llr, info


# --------------------------------------------------------------------------- main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    N, K, L, F_mode, workload = MODES[args.mode]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: WORLD_SIZE={world} but --gpus={args.gpus}; reporting n_gpus={world}", file=sys.stderr)
    strong = args.mode.endswith("_strong")
    if strong:
        from antpolarcodes_amd.distributed import shard_bounds
        lo, hi = shard_bounds(F_mode, world, rank)
        F = hi - lo
    else:
        lo, F = 0, F_mode

    import numpy as np
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    digest = src_digest()
    measure = args.traffic if args.traffic is not None else (world == 1 and not args.dry_run)

    from antpolarcodes_amd._native import Plan
    from antpolarcodes_amd.construction import frozen_bits

    crc = 11 if args.mode == "nr5g" else 8
    fixed = args.mode.endswith("_char")
    adaptive = args.mode.startswith("adaptive")
    frozen = frozen_bits(1024, K, 0.0, "5G") if args.mode == "nr5g" else frozen_bits(N, K, 0.0, "BB")

    S = 1  # batches in flight (--streams)
    in_flight2 = None
    if args.dry_run:
        # plumbing only: a host-only plan (classification, no GPU), a sleep as the step
        plan = Plan(N, L, frozen, systematic=True, crc=crc, device=-1, adaptive=adaptive, fixed=fixed)
        kernel = plan.kernel_name()
        for _ in range(args.warmup):
            time.sleep(0.001)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            time.sleep(0.002)
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        kern_ms, fer, ok_rate, dev = wall / max(args.steps, 1) * 1e3, None, None, None
    else:
        # traffic passes first: child processes, while this one has not touched the GPU
        traffic, traffic_note = None, None
        if measure and rank == 0:
            probe = Plan(N, L, frozen, systematic=True, crc=crc, device=-1, adaptive=adaptive, fixed=fixed)
            # adaptive plans: the list stage's kernel (the dominant one, r02af stats: 61 % of the
            # step) -- its FETCH/WRITE per launch, over the CRC failures it decodes
            specialize(probe)
            traffic, traffic_note = measure_traffic(args, probe.kernel_name(), F)
            probe.close()
        torch.cuda.set_device(local)
        dev = torch.device(f"cuda:{local}")
        punc = None
        host_llr = None
        if args.mode == "nr5g":
            from antpolarcodes_amd import frames
            from antpolarcodes_amd._native import Puncturer
            host_llr, info_h, frozen, pos = frames.nr_frames(NR_E, K, F, args.ebn0, seed=1000 + rank, crc=crc)
            punc = Puncturer(NR_E, frozen, device=local)
            d_llr = torch.from_numpy(host_llr).to(dev)
            d_ref = torch.from_numpy(info_h).to(dev)
        elif N > 1024:
            d_llr, d_ref = device_frames(torch, N, frozen, F, args.ebn0, 1000 + lo + 7919 * rank, crc, dev)
        else:
            from antpolarcodes_amd import frames
            host_llr, info_h, _ = frames.awgn_frames(N, frozen, F, args.ebn0, seed=1000 + rank, crc=crc)
            if fixed:  # pcsim's Scale(amplification) then CharContainer::insertLlr (host side, once)
                host_llr = np.clip(np.rint(host_llr * CHAR_AMP), -128, 127).astype(np.int8)
            d_llr = torch.from_numpy(host_llr).to(dev)
            d_ref = torch.from_numpy(info_h).to(dev)
        # S batches in flight (--streams): one plan, output buffers and HIP stream each; every
        # step decodes the whole resident batch on stream i % S
        S = args.streams if args.streams > 0 else (2 if adaptive and not args.single_stream else 1)
        plans = [Plan(N, L, frozen, systematic=True, crc=crc, device=local, adaptive=adaptive, fixed=fixed)
                 for _ in range(S)]
        for q in plans:
            specialize(q)
        plan = plans[0]
        kernel = plan.kernel_name()
        kb = plan.kb
        outs = [(torch.empty((F, kb), dtype=torch.uint8, device=dev), torch.empty(F, dtype=torch.uint8, device=dev),
                 torch.empty((F, L), dtype=torch.float32, device=dev) if L > 1 else None) for _ in range(S)]
        d_info, d_ok, d_met = outs[0]
        streams = [torch.cuda.current_stream()] + [torch.cuda.Stream(device=dev) for _ in range(S - 1)]
        stream = streams[0]

        def step(i=0):
            q, st = plans[i % S], streams[i % S].cuda_stream
            oi, ok, om = outs[i % S]
            if punc is not None:
                q.decode_punctured_device(punc, d_llr, oi, ok, om, stream=st)
            elif fixed:
                q.decode_device_i8(d_llr, oi, ok, om, stream=st)
            else:
                q.decode_device(d_llr, oi, ok, om, stream=st)

        for i in range(max(args.warmup, S)):
            step(i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
        t0 = time.perf_counter()
        for i in range(args.steps):
            ev[i][0].record(streams[i % S])
            step(i)
            ev[i][1].record(streams[i % S])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        # one stream: the mean decode time from events on the launch stream; S > 1 streams: the
        # decodes overlap, so the per-batch time is the wall time per step (the event spans are
        # each decode's latency, reported beside it)
        lat_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if args.steps else 0.0
        kern_ms = lat_ms if S == 1 else wall / max(args.steps, 1) * 1e3
        # correctness spot check of the last step (decoded == transmitted fraction)
        fer = float((d_info != d_ref).any(dim=1).float().mean().item())
        ok_rate = float(d_ok.float().mean().item())
        # (one stream) the same steps with a second batch in flight on a second stream and plan:
        # reported beside `value`, never as it -- a launch ends with a tail of waves finishing
        # their last codeword group, which the next batch's waves fill
        in_flight2 = None
        if S == 1 and world == 1 and args.steps and args.in_flight:
            q2 = Plan(N, L, frozen, systematic=True, crc=crc, device=local, adaptive=adaptive, fixed=fixed)
            specialize(q2)
            plans.append(q2)
            outs.append((torch.empty_like(d_info), torch.empty_like(d_ok),
                         torch.empty_like(d_met) if d_met is not None else None))
            streams.append(torch.cuda.Stream(device=dev))
            S = 2
            for i in range(2):
                step(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                step(i)
            torch.cuda.synchronize()
            in_flight2 = F * args.steps / (time.perf_counter() - t0)
            S = 1

    from antpolarcodes_amd.distributed import reduce_stats
    st = reduce_stats({"wall": (wall, "max"), "frames": (F * args.steps, "sum")})
    wall_max = st["wall"]
    total_frames = int(st["frames"])
    value = total_frames / wall_max if wall_max > 0 else 0.0

    if rank == 0:
        # LLRs in (E per frame for nr5g), info bytes + ok flag out (+ metrics below)
        bytes_per_cw = (1 if fixed else 4) * (NR_E if args.mode == "nr5g" else N) + (K + 7) // 8 + 1
        if L > 1:
            bytes_per_cw += 4 * L
        achieved = F * bytes_per_cw / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": kernel, "kernel_ms": kern_ms,
                "frames_per_launch": F, "algorithmic_bytes_per_codeword": bytes_per_cw}
        if adaptive:  # the events bracket the whole adaptive decode, not the list kernel alone
            roof["kernel_ms_scope"] = ("the whole adaptive decode: the Fast-SSC stage, the compaction of its CRC "
                                       f"failures and {kernel} (rocprof gives each kernel's own average)")
        if in_flight2 is not None:
            roof["throughput_2_in_flight_cw_per_s"] = in_flight2
        if S > 1:
            roof["kernel_ms_scope"] = (f"{S} batches in flight on {S} streams: wall time per batch; one decode's "
                                       f"latency (events on its stream) is decode_latency_ms")
            roof["decode_latency_ms"] = lat_ms
        line = {
            "metric": HEADLINE_METRIC if args.mode == "scl8" else f"codewords/s ({args.mode})",
            "value": value,
            "unit": "codewords/s",
            "info_bits_per_s": value * K,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / max(args.steps, 1) * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "i8" if fixed else "f32",
            "data": ("synthetic BPSK-AWGN frames (Eb/N0 %.1f dB), " % args.ebn0)
            + ("5G reliability-list frozen set, CRC-11, punctured to E=%d" % NR_E if args.mode == "nr5g"
               else "BB(0 dB) frozen set, CRC-8")
            + (", LLRs x%g quantised to int8" % CHAR_AMP if fixed else "")
            + (", generated on the device (Philox)" if N > 1024 else ""),
            "config": {"workload": workload, "N": N, "K": K, "L": L,
                       ("global_frames" if strong else "frames_per_step_per_gpu"): F_mode,
                       "crc": "CRC-11" if crc == 11 else "CRC-8", "systematic": True,
                       "parallelism": f"{world} independent shard(s), no collective",
                       "streams": S},
            "roofline": roof,
            **({"value_scope": f"{S} batches in flight on {S} HIP streams (plans), step i on stream i % {S}: the "
                               "wall-time throughput of overlapping batches -- not comparable with a one-stream "
                               "value (--no-in-flight / --streams 1)"} if S > 1 else {}),
            "src_digest": digest,
        }
        # developer environment switches that changed the plan (pcg_plan_desc.dev_overrides):
        # 0 = the production kernel and layout
        line["config"]["dev_overrides"] = plan.describe()["dev_overrides"]
        head = git_head()
        if head:
            line["git_head"] = head
        if args.dry_run:
            line["dry_run"] = True
        else:
            line["frame_error_rate"] = fer
            line["crc_ok_rate"] = ok_rate
            if traffic is None:
                traffic, why = stamped_traffic(args.mode, kernel, digest)
                traffic_note = traffic_note or why
                if traffic is not None:
                    traffic_note = None
            if traffic is not None:
                tb = traffic["bytes_per_codeword"] * F
                roof["traffic"] = tb
                roof["traffic_bytes_per_codeword"] = traffic["bytes_per_codeword"]
                if "read_bytes_per_launch" in traffic:
                    roof["traffic_read_bytes_per_codeword"] = traffic["read_bytes_per_launch"] / F
                    roof["traffic_write_bytes_per_codeword"] = traffic["write_bytes_per_launch"] / F
                roof["traffic_frac"] = tb / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if kern_ms > 0 else None
                roof["traffic_source"] = traffic["source"]
                if adaptive:
                    roof["traffic_scope"] = (f"{kernel}: the list stage over the frames whose Fast-SSC CRC check "
                                             f"failed; the Fast-SSC stage is another kernel")
            else:
                roof["traffic_note"] = traffic_note or "not measured"
            if world == 1 and not args.no_copy_bw:
                roof["measured_copy_GBps"] = copy_bandwidth(torch, dev)
                roof["frac_of_measured_copy"] = achieved / roof["measured_copy_GBps"]
            if world == 1 and punc is None and host_llr is not None and not args.no_host_rate:
                # PCIe-inclusive rate (host buffers: H2D + decode + D2H, pcg_decode_*_host), never `value`
                # (the overlapped pipeline of pcg_decode_*_host, and beside it the serial chunk loop
                # it replaced, PCG_HOST_PIPE=0 -- read per call)
                dh = plan.decode_host_i8 if fixed else plan.decode_host

                def host_rate(pipe):
                    old = os.environ.get("PCG_HOST_PIPE")
                    os.environ["PCG_HOST_PIPE"] = pipe
                    try:
                        dh(host_llr)  # (staging allocated outside the timed calls)
                        best = 0.0
                        for _ in range(3):
                            t0 = time.perf_counter()
                            dh(host_llr)
                            best = max(best, F / (time.perf_counter() - t0))
                        return best
                    finally:
                        if old is None:
                            del os.environ["PCG_HOST_PIPE"]
                        else:
                            os.environ["PCG_HOST_PIPE"] = old
                line["host_buffers_cw_per_s"] = host_rate(os.environ.get("PCG_HOST_PIPE", "2"))
                line["host_buffers_serial_cw_per_s"] = host_rate("0")
                # a page-locked caller buffer (e.g. a simulator's reused frame buffer): copied from
                # directly, no staging copy -- the PCIe-bound rate
                pinned = torch.from_numpy(host_llr).pin_memory()
                host_llr_pageable, host_llr = host_llr, pinned.numpy()
                line["host_buffers_pinned_cw_per_s"] = host_rate(os.environ.get("PCG_HOST_PIPE", "2"))
                host_llr = host_llr_pageable
                del pinned
            if not args.no_cpu_baseline and world == 1:
                if host_llr is None:  # device-generated frames: copy a bounded sample back
                    cpu_llr = d_llr[:4096].cpu().numpy()
                elif punc is not None:
                    cpu_llr = np.zeros((host_llr.shape[0], N), np.float32)
                    cpu_llr[:, pos] = host_llr
                else:
                    cpu_llr = host_llr
                line["cpu_baseline"] = cpu_baseline(args.mode, N, L, frozen, cpu_llr, cpu_threads(args))
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
