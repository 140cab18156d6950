"""pcsim -- the reference simulator's BER/BLER/throughput flow on MI355X (config 1 "via pcsim").

Restates `Simulation::Simulator` / `SimulationWorker` (src/simulation/simulator.cpp of
david13pod/antPolarCodes) around the batched GPU decoders:

  * job list: configureSingleRun / CodeLength / DesignSnr / ListLength / Rate /
    Amplification (simulator.cpp:126-285), then snrInflateJobList (:361-379), with the
    reference's float32 arithmetic for the SNR / design-SNR / rate / amplification grids;
  * per job (SimulationWorker::run, :632-672): Bhattacharyya frozen set (:680-697),
    encoder + decoder by precision and list size (setCoders :699-760: L > 1 -> Adaptive
    {Char, Float, Mixed}, L == 1 -> FastSscFipChar / FastSscAvxFloat), CRC-8 / CRC-32 /
    none (setErrorDetector :761-805; "cmac*" is outside this build), BPSK-AWGN at
    Es/N0 = Eb/N0 * BPS * K / N (setChannel :806-824), Scale(amplification) of the
    demodulated symbols (:920-937), warm-up min(blocks / 8, 1000) blocks, then the
    counted blocks: BER over the K decoded bits, block errors, reported (check()) errors
    (countErrors :938-965, calculateStatistics :966-985);
  * results: saveResults' CSV columns and number formatting (:510-545).

GPU-first differences: frames are generated, encoded, transmitted and decoded on the device
in batches of up to `--batch` frames (the reference loops one frame at a time), so the
decode time of a block is the batch's HIP-event time divided by its frames (time min /
max / mean / deviation are over those per-block figures); -t/--threads workers take jobs
from the shared queue like SimThread (:120-131), worker w on GPU w % device_count.  The
channel noise comes from the device Philox generator, not std::mt19937.

Usage: python -m antpolarcodes_amd.pcsim [simtype] [-w BITS] [--snr-min X] [--snr-max X]
       [--snr-count C] [-n N] [-r RATE] [-l L] [-d DSNR] [-e crc8|crc32|none] [-s]
       [-p 8|32|832] [-a AMP] [-o NAME] [-t THREADS] [--batch F]
"""
import argparse
import math
import os
import sys
import threading
import time
from dataclasses import dataclass, field, replace

import numpy as np

SIMTYPES = ("single", "codelength", "designsnr", "listlength", "rate", "amplification", "fixed", "depthfirst",
            "scan", "fastsscan", "ask", "compareall", "getcode")
SUPPORTED = ("single", "codelength", "designsnr", "listlength", "rate", "amplification", "getcode")
CSV_HEADER = ('"N","K","dSNR","C","L","Eb/N0","BPS","BLER","BER","RER","Runs","Errors","Time","Blockspeed",'
              '"Coded Bitrate","Payload Bitrate","Effective Payload Bitrate","Encoder Bitrate","Amplification",'
              '"time min","time max","time mean","time deviation"')
f32 = np.float32


def error_detection_id(s):
    """errorDetectionStringToId (simulator.h:33-52)."""
    return {"crc8": 8, "crc32": 32, "cmac8": 8, "cmac16": 16, "cmac32": 32, "cmac64": 64, "cmac128": 128}.get(s, 0)


def error_detection_type(s):
    """errorDetectionStringToType (simulator.h:55-67)."""
    if s.startswith("crc"):
        return "crc"
    if s.startswith("cmac"):
        return "cmac"
    return "none"


@dataclass
class Job:
    """DataPoint (simulator.h:72-121)."""
    designSNR: float
    N: int
    K: int
    L: int
    errorDetection: int
    errorDetectionType: str
    systematic: bool
    EbN0: float
    BlocksToSimulate: int
    precision: int
    amplification: float
    bitsPerSymbol: int = 1
    name: str = ""
    runs: int = 0
    bits: int = 0
    errors: int = 0
    reportedErrors: int = 0
    biterrors: int = 0
    BLER: float = 0.0
    BER: float = 0.0
    RER: float = 0.0
    time_sum: float = 0.0
    time_min: float = 0.0
    time_max: float = 0.0
    time_mean: float = 0.0
    time_dev: float = 0.0
    blps: float = 0.0
    cbps: float = 0.0
    pbps: float = 0.0
    effectiveRate: float = 0.0
    encTime: float = 0.0
    ebps: float = 0.0
    block_times: list = field(default_factory=list)  # (seconds per block, blocks) per batch


def default_job(a):
    """getDefaultDataPoint (simulator.cpp:133-163)."""
    N = int(a.blocklength)
    return Job(designSNR=float(f32(a.design_snr)), N=N, K=int(f32(N) * f32(a.rate)), L=int(a.pathlimit),
               errorDetection=error_detection_id(a.error_detection),
               errorDetectionType=error_detection_type(a.error_detection), systematic=not a.non_systematic,
               EbN0=float(f32(a.snr_max)), BlocksToSimulate=int(a.workload) // N, precision=int(a.precision),
               amplification=float(f32(a.amplification)))


def _grid(lo, hi, count):
    """float scale = (max - min) / (count - 1); value_i = min + i * scale (float32)."""
    lo, hi = f32(lo), f32(hi)
    scale = f32((hi - lo) / f32(count - 1))
    return [float(f32(lo + f32(i) * scale)) for i in range(count)]


def configure(a):
    """The job template list of one simtype (simulator.cpp:126-285), before SNR inflation."""
    t = default_job(a)
    st = a.simtype
    if st == "single":
        return [t]
    if st == "codelength":
        jobs, n = [], int(a.n_min)
        while n <= int(a.n_max):
            jobs.append(replace(t, N=n, K=int(f32(n) * f32(a.rate)), BlocksToSimulate=int(a.workload) // n))
            n *= 2
        return jobs
    if st == "designsnr":
        return [replace(t, designSNR=d) for d in _grid(a.dsnr_min, a.dsnr_max, int(a.dsnr_count))]
    if st == "listlength":
        jobs, l = [], int(a.l_min)
        while l <= int(a.l_max):
            jobs.append(replace(t, L=l))
            l *= 2
        return jobs
    if st == "rate":
        jobs = []
        for r in _grid(a.r_min, a.r_max, int(a.r_count)):
            K = int(f32(t.N) * f32(r))  # job->K = job->N * rate, then rounded up to a byte
            jobs.append(replace(t, K=(K + 7) // 8 * 8))
        return jobs
    if st == "amplification":
        return [replace(t, amplification=v) for v in _grid(a.amp_min, a.amp_max, int(a.amp_count))]
    raise SystemExit(f"pcsim: simulation type '{st}' is outside this build "
                     f"(supported: {', '.join(SUPPORTED)})")


def snr_inflate(jobs, snr_min, snr_max, snr_count):
    """snrInflateJobList + pushJobsInRange (simulator.cpp:338-379): three SNR ranges
    [min, 0], [0, 2], [2, max] with count/4, count/2, count/4 points, each range's first
    point skipped; float decoding (precision 32) sets amplification = 4 * 10^(Eb/N0 / 10)."""
    out = []
    for job in jobs:
        for lo, hi, c in ((snr_min, 0.0, snr_count // 4), (0.0, 2.0, snr_count // 2),
                          (2.0, snr_max, snr_count // 4)):
            if c < 2:
                continue
            g = _grid(lo, hi, c)
            for i in range(1, c):
                nj = replace(job, EbN0=g[i], block_times=[])
                if nj.precision == 32:
                    nj.amplification = float(f32(4 * math.pow(10.0, g[i] / 10.0)))
                out.append(nj)
    return out


def build_jobs(a):
    return snr_inflate(configure(a), a.snr_min, a.snr_max, int(a.snr_count))


def fmt(x):
    """C++ ostream << float/double with the default precision (6 significant digits)."""
    if isinstance(x, (int, np.integer)):
        return str(int(x))
    if x == 0:
        return "0"
    s = f"{x:.6g}"
    if "e" in s:  # C++ prints at least two exponent digits: 1e-05, 1.5e+07
        m, e = s.split("e")
        sign = e[0]
        digits = e[1:].lstrip("0")
        s = f"{m}e{sign}{digits.zfill(2)}"
    return s


def save_results(jobs, path):
    """saveResults (simulator.cpp:510-545): header, then one line per job."""
    with open(path, "w") as fh:
        fh.write(CSV_HEADER + "\n")
        for j in jobs:
            cols = [j.N, j.K, fmt(j.designSNR), j.errorDetection, j.L, fmt(j.EbN0), j.bitsPerSymbol,
                    fmt(j.BLER) if j.BLER > 0 else "1e-99", fmt(j.BER) if j.BER > 0 else "1e-99",
                    fmt(j.RER) if j.RER > 0 else "1e-99", j.runs, j.errors, fmt(j.time_sum), fmt(j.blps),
                    fmt(j.cbps), fmt(j.pbps), fmt(j.effectiveRate), fmt(j.ebps), fmt(j.amplification),
                    int(j.time_min * 1e9), int(j.time_max * 1e9), int(j.time_mean * 1e9), int(j.time_dev * 1e9)]
            fh.write(",".join(str(c) for c in cols) + "\n")


def calculate_statistics(j):
    """calculateStatistics (simulator.cpp:966-985); the time statistics are over blocks
    (each batch contributes its per-block time once per block it decoded)."""
    if j.block_times:
        t = np.concatenate([np.full(n, s, np.float64) for s, n in j.block_times])
        j.time_sum = float(t.sum())
        j.time_min, j.time_max, j.time_mean = float(t.min()), float(t.max()), float(t.mean())
        j.time_dev = float(t.std())
    runs = max(j.runs, 1)
    j.bits = j.runs * (j.K - j.errorDetection)
    j.BLER = float(f32(j.errors) / f32(runs))
    j.BER = float(j.biterrors / (float(runs) * float(j.K)))
    j.RER = float(f32(j.reportedErrors) / f32(runs))
    ts = j.time_sum if j.time_sum > 0 else float("inf")
    j.blps = j.runs / ts
    j.cbps = j.runs * j.N / ts
    j.pbps = j.bits / ts
    j.ebps = j.runs * j.N / j.encTime if j.encTime > 0 else 0.0
    j.effectiveRate = (j.runs - j.errors) * (j.K - j.errorDetection) / ts


def count_errors(j, sent, got, ok):
    """countErrors (simulator.cpp:938-965) over a batch: bit errors over the K bits,
    erroneous blocks, and blocks whose check() failed (reported errors, decode() :920-937)."""
    nb = j.K // 8
    diff = np.bitwise_xor(sent[:, :nb], got[:, :nb])
    be = np.unpackbits(diff, axis=1).sum(axis=1)
    j.biterrors += int(be.sum())
    j.errors += int((be > 0).sum())
    j.reportedErrors += int((ok == 0).sum())
    j.runs += int(sent.shape[0])


class GpuBackend:
    """One worker's device: frame source (pcg_random_info / pcg_encode / pcg_bpsk_awgn_f32)
    and the decoder setCoders picks, all on one HIP stream."""

    def __init__(self, device=0):
        import torch
        self.torch = torch
        self.device = device
        self.dev = torch.device(f"cuda:{device}")

    def setup(self, job):
        from .construction import frozen_bits
        from ._native import Encoder, Plan
        if job.errorDetection >= job.K:  # setErrorDetector (:763-766)
            job.errorDetection, job.errorDetectionType = 0, "none"
        if job.errorDetectionType == "cmac":
            raise SystemExit("pcsim: CMAC error detection is outside this build (crc8, crc32, none)")
        crc = job.errorDetection if job.errorDetectionType == "crc" and job.errorDetection in (8, 32) else 0
        self.crc = crc
        self.frozen = frozen_bits(job.N, job.K, job.designSNR, "BB")
        self.enc = Encoder(job.N, self.frozen, systematic=job.systematic, crc=crc, device=self.device)
        self.second = None
        if job.L > 1 and job.precision == 832:  # AdaptiveMixed: FastSscFipChar, then SclAvxFloat
            self.plan = Plan(job.N, 1, self.frozen, job.systematic, crc, self.device, fixed=True)
            self.second = Plan(job.N, job.L, self.frozen, job.systematic, crc, self.device)
        elif job.L > 1:  # AdaptiveChar / AdaptiveFloat
            if job.precision not in (8, 32):
                raise SystemExit(f"No decoder present for {job.precision}-bit decoding.")
            self.plan = Plan(job.N, job.L, self.frozen, job.systematic, crc, self.device, adaptive=True,
                             fixed=job.precision == 8)
        else:  # FastSscFipChar (8, 832) / FastSscAvxFloat (32)
            if job.precision not in (8, 32, 832):
                raise SystemExit(f"No decoder present for {job.precision}-bit decoding.")
            self.plan = Plan(job.N, 1, self.frozen, job.systematic, crc, self.device, fixed=job.precision != 32)
        esn0 = 10.0 ** (job.EbN0 / 10.0) * job.bitsPerSymbol * job.K / job.N
        self.sigma = float(np.sqrt(1.0 / (2.0 * esn0)))
        # the device channel returns 2 y / sigma^2; the reference decodes amplification * y
        self.scale = job.amplification * self.sigma * self.sigma / 2.0

    def frames(self, job, F, seed):
        # a worker thread starts on cuda:0: events, streams and syncs must be this worker's GPU's
        with self.torch.cuda.device(self.dev):
            return self._frames(job, F, seed)

    def _frames(self, job, F, seed):
        torch = self.torch
        from ._native import bpsk_awgn_device, random_info_device
        kb = (job.K + 7) // 8
        info = torch.empty((F, kb), dtype=torch.uint8, device=self.dev)
        code = torch.empty((F, job.N // 8), dtype=torch.uint8, device=self.dev)
        llr = torch.empty((F, job.N), dtype=torch.float32, device=self.dev)
        random_info_device(info, job.K, seed)
        st = torch.cuda.current_stream(self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        self.enc.encode_device(info, code)
        e1.record(st)
        bpsk_awgn_device(code, job.N, self.sigma, seed ^ 0x9E3779B97F4A7C15, llr)
        llr.mul_(self.scale)
        torch.cuda.synchronize(self.dev)
        return llr, info, e0.elapsed_time(e1) * 1e-3

    def decode(self, job, llr):
        with self.torch.cuda.device(self.dev):
            return self._decode(job, llr)

    def _decode(self, job, llr):
        torch = self.torch
        F = llr.shape[0]
        out = torch.empty((F, self.plan.kb), dtype=torch.uint8, device=self.dev)
        ok = torch.empty(F, dtype=torch.uint8, device=self.dev)
        st = torch.cuda.current_stream(self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        self.plan.decode_device(llr, out, ok)  # 8-bit plans quantise the floats (insertLlr)
        if self.second is not None:  # AdaptiveMixed: list decoding of the failed frames
            bad = torch.nonzero(ok == 0).flatten()
            if bad.numel():
                sub = llr.index_select(0, bad).contiguous()
                so = torch.empty((bad.numel(), self.plan.kb), dtype=torch.uint8, device=self.dev)
                sk = torch.empty(bad.numel(), dtype=torch.uint8, device=self.dev)
                self.second.decode_device(sub, so, sk)
                out.index_copy_(0, bad, so)
                ok.index_copy_(0, bad, sk)
        e1.record(st)
        torch.cuda.synchronize(self.dev)
        return out.cpu().numpy(), ok.cpu().numpy(), e0.elapsed_time(e1) * 1e-3

    def close(self):
        for p in (getattr(self, "plan", None), getattr(self, "second", None), getattr(self, "enc", None)):
            if p is not None:
                p.close()


def run_job(job, backend, batch, seed=0, log=None):
    """SimulationWorker::run for one job (simulator.cpp:632-672), batched."""
    backend.setup(job)
    blocks = job.BlocksToSimulate
    warm = min(blocks // 8, 1000)
    if warm:
        llr, _, _ = backend.frames(job, warm, seed * 1000003 + 1)
        backend.decode(job, llr)
    done, k = 0, 0
    while done < blocks:
        F = min(batch, blocks - done)
        llr, sent, tenc = backend.frames(job, F, seed * 1000003 + 2 + k)
        got, ok, tdec = backend.decode(job, llr)
        sent = sent.cpu().numpy() if hasattr(sent, "cpu") else np.asarray(sent)
        count_errors(job, sent, got, ok)
        job.encTime += tenc
        job.block_times.append((tdec / F, F))
        done += F
        k += 1
    calculate_statistics(job)
    backend.close()
    if log:
        log(f"N={job.N}, K={job.K}, L={job.L}, dSNR={job.designSNR:g}, ErrorDetector={job.errorDetectionType}"
            f"{job.errorDetection}, SNR={job.EbN0:g}: BLER={job.BLER:g} BER={job.BER:g} "
            f"({job.runs} blocks, {job.blps:.4g} blocks/s)")
    return job


def run(jobs, threads=1, batch=1 << 16, make_backend=None, log=None):
    """Simulator::run (simulator.cpp:86-131): `threads` workers take jobs from the shared
    queue (getJob's atomic counter); worker w decodes on GPU w % device_count."""
    if make_backend is None:
        from ._native import device_count
        ng = max(1, device_count())

        def make_backend(w):
            return GpuBackend(w % ng)
    nxt = [0]
    lock = threading.Lock()
    errors = []

    def worker(w):
        be = make_backend(w)
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= len(jobs):
                return
            if log:
                log(f"[{w + 1}] Jobs in queue: {len(jobs) - i - 1}")
            try:
                run_job(jobs[i], be, batch, seed=i, log=log)
            except BaseException as e:  # noqa: BLE001
                errors.append(e)
                return

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(max(1, threads))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errors:
        raise errors[0]
    return jobs


def print_code(a):
    """getcode (simulator.cpp:478-500): the frozen-bit mask, then the frozen indices."""
    from .construction import frozen_bits
    t = default_job(a)
    fr = frozen_bits(t.N, t.K, t.designSNR, "BB")
    isf = np.zeros(t.N, bool)
    isf[list(fr)] = True
    print("".join("1," if v else "0," for v in isf))
    print()
    print("".join(f"{i}," for i in fr))


def parser():
    ap = argparse.ArgumentParser(prog="pcsim", description="Polar code BER/BLER simulation on MI355X")
    ap.add_argument("simtype", nargs="?", default="single", choices=SIMTYPES)
    ap.add_argument("-w", "--workload", type=int, default=int(1e9), help="bits per simulation run")
    ap.add_argument("--snr-min", type=float, default=-1.59174539)
    ap.add_argument("--snr-max", type=float, default=4.0)
    ap.add_argument("--snr-count", type=int, default=16)
    ap.add_argument("-d", "--design-snr", type=float, default=0.0)
    ap.add_argument("--dsnr-min", type=float, default=-1.59174539)
    ap.add_argument("--dsnr-max", type=float, default=6.0)
    ap.add_argument("--dsnr-count", type=int, default=6)
    ap.add_argument("-n", "--blocklength", type=int, default=1024)
    ap.add_argument("--n-min", type=int, default=128)
    ap.add_argument("--n-max", type=int, default=32768)
    ap.add_argument("-r", "--rate", type=float, default=0.5)
    ap.add_argument("--r-min", type=float, default=0.25)
    ap.add_argument("--r-max", type=float, default=0.9)
    ap.add_argument("--r-count", type=int, default=5)
    ap.add_argument("-l", "--pathlimit", type=int, default=8)
    ap.add_argument("--l-min", type=int, default=1)
    ap.add_argument("--l-max", type=int, default=16)
    ap.add_argument("-e", "--error-detection", default="crc32",
                    choices=("none", "crc8", "crc32", "cmac8", "cmac16", "cmac32", "cmac64", "cmac128"))
    ap.add_argument("-s", "--non-systematic", action="store_true")
    ap.add_argument("-p", "--precision", type=int, default=832)
    ap.add_argument("-a", "--amplification", type=float, default=10.0)
    ap.add_argument("--amp-min", type=float, default=1.0)
    ap.add_argument("--amp-max", type=float, default=128.0)
    ap.add_argument("--amp-count", type=int, default=6)
    ap.add_argument("-o", "--output", default="simulation")
    ap.add_argument("-t", "--threads", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1 << 16, help="frames per GPU launch (this build)")
    return ap


def main(argv=None):
    a = parser().parse_args(argv)
    if a.simtype == "getcode":
        print_code(a)
        return 0
    jobs = build_jobs(a)
    run(jobs, threads=a.threads, batch=a.batch, log=lambda m: print(m, flush=True))
    path = f"{a.output}_{a.simtype}.csv"
    save_results(jobs, path)
    print(f"results: {os.path.abspath(path)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
