"""pcsim-equivalent driver on the GPU: one job of config 1's chain (BB construction, CRC-8,
systematic encoder, BPSK-AWGN, Scale(amplification)) decoded by the GPU decoders; its block
/ bit / reported error counts must equal the oracle's decisions on the very same frames."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class Recording:
    def __init__(self):
        from antpolarcodes_amd.pcsim import GpuBackend
        self.be = GpuBackend(0)
        self.llr, self.sent = [], []

    def setup(self, job):
        self.be.setup(job)

    def frames(self, job, F, seed):
        llr, info, t = self.be.frames(job, F, seed)
        self.llr.append(llr.cpu().numpy())
        self.sent.append(info.cpu().numpy())
        return llr, info, t

    def decode(self, job, llr):
        return self.be.decode(job, llr)

    def close(self):
        self.frozen = self.be.frozen
        self.be.close()


# (N, L, precision): N = 1024, L = 1, precision 32 is config 1 itself (pcsim -n 1024 -r 0.5 -l 1
# -p 32, FastSscAvxFloat); 832 is pcsim's default AdaptiveMixed (FastSscFipChar, then SclAvxFloat)
@pytest.mark.parametrize("N,L,precision", [(1024, 1, 32), (256, 1, 32), (256, 8, 32), (256, 4, 8), (256, 8, 832),
                                           (1024, 8, 832)])
def test_pcsim_job_matches_oracle(oracle, N, L, precision):
    from antpolarcodes_amd import pcsim
    a = pcsim.parser().parse_args(["-n", str(N), "-r", "0.5", "-l", str(L), "-p", str(precision), "-e", "crc8",
                                   "-w", str(N * 3000), "--snr-min", "1.0", "--snr-max", "2.0",
                                   "--snr-count", "4"])
    job = pcsim.build_jobs(a)[0]
    rec = Recording()
    pcsim.run_job(job, rec, batch=1024, seed=5)
    llr = np.concatenate(rec.llr[1:])  # the first call is the warm-up batch
    sent = np.concatenate(rec.sent[1:])
    assert llr.shape[0] == job.runs == 3000
    assert job.N == N
    fr = rec.frozen
    if precision in (8, 832):  # 8-bit decoders quantise the amplified floats (CharContainer::insertLlr)
        info, ok = oracle.scc_decode(N, fr, llr, crc=8)
    else:
        info, ok = oracle.sc_decode(N, fr, llr, crc=8)
    if L > 1:  # Adaptive*: list decoding of the frames whose check failed (832: the float SCL)
        bad = np.nonzero(ok == 0)[0]
        if bad.size:
            if precision == 8:
                si, sk = oracle.sclc_decode(N, L, fr, llr[bad], crc=8)[:2]
            else:
                si, sk = oracle.scl_decode(N, L, fr, llr[bad], crc=8)
            info[bad], ok[bad] = si, sk
    be = np.unpackbits(np.bitwise_xor(sent, info), axis=1).sum(axis=1)
    assert job.errors == int((be > 0).sum())
    assert job.biterrors == int(be.sum())
    assert job.reportedErrors == int((ok == 0).sum())
    assert 0 < job.BLER < 1


def test_pcsim_worker_on_second_gpu_times_its_own_device():
    """A worker thread on cuda:1 records its timing events on cuda:1's stream (a new thread's
    current device is cuda:0): positive, finite decode times."""
    import threading
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    from antpolarcodes_amd import pcsim
    a = pcsim.parser().parse_args(["-n", "256", "-r", "0.5", "-l", "1", "-p", "32", "-e", "crc8",
                                   "-w", str(256 * 2000), "--snr-min", "2.0", "--snr-max", "2.0"])
    job = pcsim.build_jobs(a)[0]
    res = {}

    def work():
        res["job"] = pcsim.run_job(job, pcsim.GpuBackend(1), batch=512, seed=3)

    t = threading.Thread(target=work)
    t.start()
    t.join()
    j = res["job"]
    times = [tb for tb, _ in j.block_times]
    assert all(np.isfinite(x) and x > 0 for x in times)
    assert j.encTime > 0
