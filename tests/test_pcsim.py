"""pcsim-equivalent driver (antpolarcodes_amd/pcsim.py) on CPU: the reference simulator's
job list (configure* + snrInflateJobList, simulator.cpp:126-379), error counting and
statistics (:938-985) and CSV layout (:510-545), with a mocked frame source / decoder."""
import numpy as np
import pytest

from antpolarcodes_amd import pcsim

f32 = np.float32


def _args(*argv):
    return pcsim.parser().parse_args(list(argv))


def _ref_range(lo, hi, c):
    lo, hi = f32(lo), f32(hi)
    sc = f32((hi - lo) / f32(c - 1))
    return [float(f32(lo + f32(i) * sc)) for i in range(1, c)]


def test_single_job_snr_inflation_defaults():
    jobs = pcsim.build_jobs(_args())
    # snr-count 16: 3 + 7 + 3 points (each range's first point skipped)
    exp = _ref_range(-1.59174539, 0.0, 4) + _ref_range(0.0, 2.0, 8) + _ref_range(2.0, 4.0, 4)
    assert [j.EbN0 for j in jobs] == exp and len(jobs) == 13
    j = jobs[0]
    assert (j.N, j.K, j.L, j.errorDetection, j.errorDetectionType, j.systematic, j.precision) == \
        (1024, 512, 8, 32, "crc", True, 832)
    assert j.BlocksToSimulate == int(1e9) // 1024 and j.amplification == pytest.approx(10.0)


def test_float_precision_amplification_and_grids():
    jobs = pcsim.build_jobs(_args("-p", "32", "--snr-count", "8"))
    for j in jobs:  # pushJobsInRange: amplification = 4 * 10^(Eb/N0 / 10) for 32-bit decoding
        assert j.amplification == float(f32(4 * 10 ** (j.EbN0 / 10)))
    cl = pcsim.configure(_args("codelength", "--n-min", "256", "--n-max", "2048", "-w", "1048576"))
    assert [(j.N, j.K, j.BlocksToSimulate) for j in cl] == [(256, 128, 4096), (512, 256, 2048),
                                                              (1024, 512, 1024), (2048, 1024, 512)]
    ll = pcsim.configure(_args("listlength", "--l-min", "1", "--l-max", "32"))
    assert [j.L for j in ll] == [1, 2, 4, 8, 16, 32]
    rt = pcsim.configure(_args("rate"))
    assert all(j.K % 8 == 0 for j in rt) and rt[0].K == 256 and rt[-1].K == 928
    ds = pcsim.configure(_args("designsnr", "--dsnr-min", "0", "--dsnr-max", "5", "--dsnr-count", "6"))
    assert [j.designSNR for j in ds] == [0.0, 1.0, 2.0, 3.0, 4.0, 5.0]
    with pytest.raises(SystemExit):
        pcsim.configure(_args("scan"))


class MockBackend:
    """Frames from the numpy generator; the 'decoder' returns the sent bits with chosen
    frames corrupted (and reports some of them), so the counts are known exactly."""

    def __init__(self, flip_every=7, report_every=2):
        self.flip_every, self.report_every = flip_every, report_every
        self.sent = []

    def setup(self, job):
        self.K = job.K

    def frames(self, job, F, seed):
        rng = np.random.default_rng(seed)
        info = rng.integers(0, 256, (F, job.K // 8), dtype=np.uint8)
        self.sent.append(info)
        return info.copy(), info, 1e-3

    def decode(self, job, llr):
        got = llr.copy()
        ok = np.ones(llr.shape[0], np.uint8)
        for f in range(0, llr.shape[0], self.flip_every):
            got[f, 0] ^= 0x11  # 2 bit errors
            if (f // self.flip_every) % self.report_every == 0:
                ok[f] = 0
        return got, ok, 2e-3

    def close(self):
        pass


def test_worker_counts_statistics_and_csv(tmp_path):
    job = pcsim.build_jobs(_args("-n", "256", "-w", str(256 * 1000), "--snr-count", "8", "-e", "crc8"))[0]
    be = MockBackend()
    pcsim.run_job(job, be, batch=300, seed=3)
    assert job.runs == 1000  # warm-up blocks (min(1000/8, 1000) = 125) are not counted
    per = [len(range(0, F, 7)) for F in (300, 300, 300, 100)]
    assert job.errors == sum(per) and job.biterrors == 2 * sum(per)
    assert job.reportedErrors == sum(len(range(0, F, 14)) for F in (300, 300, 300, 100))
    assert job.BLER == pytest.approx(sum(per) / 1000) and job.BER == pytest.approx(2 * sum(per) / (1000 * 128))
    assert job.time_sum == pytest.approx(4 * 2e-3) and job.blps == pytest.approx(1000 / 8e-3)
    assert job.effectiveRate == pytest.approx((1000 - sum(per)) * (128 - 8) / 8e-3)
    out = tmp_path / "r.csv"
    pcsim.save_results([job], str(out))
    lines = out.read_text().splitlines()
    assert lines[0] == pcsim.CSV_HEADER and len(lines[1].split(",")) == 23
    assert lines[1].startswith("256,128,0,8,8,")


def test_cpp_float_formatting():
    assert [pcsim.fmt(x) for x in (0.5, 1e-5, 1.5e7, 123456.7, 3, 2.0)] == \
        ["0.5", "1e-05", "1.5e+07", "123457", "3", "2"]
