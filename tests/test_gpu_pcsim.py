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


@pytest.mark.parametrize("L,precision", [(1, 32), (8, 32), (4, 8)])
def test_pcsim_job_matches_oracle(oracle, L, precision):
    from antpolarcodes_amd import pcsim
    a = pcsim.parser().parse_args(["-n", "256", "-r", "0.5", "-l", str(L), "-p", str(precision), "-e", "crc8",
                                   "-w", str(256 * 3000), "--snr-min", "1.0", "--snr-max", "2.0",
                                   "--snr-count", "4"])
    job = pcsim.build_jobs(a)[0]
    rec = Recording()
    pcsim.run_job(job, rec, batch=1024, seed=5)
    llr = np.concatenate(rec.llr[1:])  # the first call is the warm-up batch
    sent = np.concatenate(rec.sent[1:])
    assert llr.shape[0] == job.runs == 3000
    N, fr = job.N, rec.frozen
    if precision == 8:  # 8-bit decoders quantise the amplified floats (CharContainer::insertLlr)
        info, ok = oracle.scc_decode(N, fr, llr, crc=8)
    else:
        info, ok = oracle.sc_decode(N, fr, llr, crc=8)
    if L > 1:  # Adaptive*: list decoding of the frames whose check failed
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
