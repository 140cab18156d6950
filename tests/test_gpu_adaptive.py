"""GPU parity of the adaptive decoder (AdaptiveFloat, adaptive_float.cpp:33-45; SURVEY §8f
rank 3): per frame, Fast-SSC's output where its check passes, otherwise the CRC-aided SCL
output and ok flag -- compared with the oracle's SC and SCL decoders frame by frame."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expect(oracle, N, L, fr, llr, crc, systematic=True):
    si, sok = oracle.sc_decode(N, fr, llr, systematic=systematic, crc=crc)
    li, lok, lm, _, _ = oracle.scl_decode(N, L, fr, llr, systematic=systematic, crc=crc, paths=True)
    use_scl = sok == 0
    info = np.where(use_scl[:, None], li, si)
    ok = np.where(use_scl, lok, sok)
    met = np.where(use_scl[:, None], lm, 0.0).astype(np.float32)
    return info, ok, met, use_scl


@pytest.mark.parametrize("kernel", ["interp", "rtc"])
@pytest.mark.parametrize("ebn0", [1.0, 2.5])
@pytest.mark.parametrize("crc", [8, 16, 32])
def test_adaptive_matches_oracle(oracle, ebn0, crc, kernel):
    """AdaptiveFloat frame by frame; "rtc": both stages on their plan-specialised kernels
    (scq_rtc_kernel, then scl_rtc_kernel over the failed frames -- what the library runs for
    the code)."""
    from antpolarcodes_amd import frames
    from helpers import gpu_plan
    N, L = 1024, 8
    fr = oracle.frozen_bits_bb(N, 512, 0.0)
    llr, _, _ = frames.awgn_frames(N, fr, 3000, ebn0, seed=crc, crc=crc)
    p = gpu_plan(N, L, fr, kernel, crc=crc, adaptive=True)
    gi, gok, gm = p.decode_host(llr, want_metrics=True)
    ei, eok, em, use_scl = _expect(oracle, N, L, fr, llr, crc)
    assert 0 < use_scl.sum() < len(use_scl)
    bad = np.nonzero(~(gi == ei).all(axis=1))[0]
    assert bad.size == 0, f"frames {bad[:8]} (scl={use_scl[bad[:8]]})"
    assert np.array_equal(gok, eok)
    assert np.array_equal(gm.view(np.uint32), em.view(np.uint32))


def test_adaptive_device_path_and_pypolar(oracle):
    import torch
    from antpolarcodes_amd import frames, pypolar
    N, L = 256, 4
    fr = oracle.frozen_bits_bb(N, 128, 0.0)
    llr, _, _ = frames.awgn_frames(N, fr, 777, 1.5, seed=3, crc=8)
    ei, eok, _, use_scl = _expect(oracle, N, L, fr, llr, 8)
    dec = pypolar.PolarDecoder(N, L, fr, "mixed")
    dec.setErrorDetection(8)
    assert np.array_equal(dec.decode_batch(llr), ei)
    f = int(np.nonzero(use_scl)[0][0])
    assert np.array_equal(dec.decode_vector(llr[f]), ei[f])
    # no ok buffer requested: the plan's own is used
    from antpolarcodes_amd._native import Plan
    p = Plan(N, L, fr, crc=8, device=0, adaptive=True)
    d_llr = torch.from_numpy(llr).cuda()
    info = torch.empty((777, 16), dtype=torch.uint8, device="cuda:0")
    for _ in range(2):  # reuse of the failed-frame list across calls
        p.decode_device(d_llr, info)
    torch.cuda.synchronize()
    assert np.array_equal(info.cpu().numpy(), ei)
