"""pypolar-compatible API on the GPU: the reference's QA decoder test
(python/qa_pypolar_decoder.py:65-113) restated for decoder type "gpu", plus
decode_batch / decode_device parity with the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pp():
    from antpolarcodes_amd import pypolar
    return pypolar


@pytest.mark.parametrize("N", [128, 256, 512, 1024])
def test_qa_cpp_decoder_impls(pp, N):
    rng = np.random.default_rng(N)
    for K in (int(N * 0.75), N // 2, N // 4, N // 8):
        f = pp.frozen_bits(N, K, -1.0)
        enc = pp.PolarEncoder(N, f)
        enc.setErrorDetection(8)
        for L in (1, 4, 8):
            dec = pp.PolarDecoder(N, L, f, "gpu")
            dec.setErrorDetection(8)
            assert dec.frozenBits() == f
            for _ in range(4):
                u = rng.integers(0, 2, K).astype(np.uint8)
                d = np.packbits(u)
                cw = enc.encode_vector(d)
                d = d.copy()
                d[-1] = pp.Detector(8, "crc").generate(d[:-1])[-1]  # the encoder appended the CRC
                llr = (1.0 - 2.0 * np.unpackbits(cw)).astype(np.float32)
                llr += rng.uniform(-0.2, 0.2, llr.size).astype(np.float32)
                assert np.array_equal(dec.decode_vector(llr), d)


@pytest.mark.parametrize("L", [1, 2, 8, 32])
def test_decode_batch_matches_oracle(pp, oracle, L):
    from antpolarcodes_amd import frames
    N, K = 1024, 512
    f = pp.frozen_bits(N, K, 0.0)
    llr, _, _ = frames.awgn_frames(N, f, 512, 1.5, seed=L, crc=16)
    dec = pp.PolarDecoder(N, L, f, "float")
    dec.setErrorDetection(16)
    info, ok, met = dec.decode_batch(llr, return_ok=True, return_metrics=True)
    if L == 1:
        oi, ook = oracle.sc_decode(N, f, llr, crc=16)
    else:
        oi, ook, om, _, _ = oracle.scl_decode(N, L, f, llr, crc=16, paths=True)
        assert np.array_equal(met.view(np.uint32), om.view(np.uint32))
    assert np.array_equal(info, oi) and np.array_equal(ok, ook)


def test_decode_device_torch(pp, oracle):
    import torch
    from antpolarcodes_amd import frames
    N, K, F = 1024, 512, 2048
    f = pp.frozen_bits(N, K, 0.0)
    llr, _, _ = frames.awgn_frames(N, f, F, 2.0, seed=3, crc=8)
    dec = pp.PolarDecoder(N, 8, f, "gpu")
    x = torch.from_numpy(llr).cuda()
    info = torch.zeros((F, K // 8), dtype=torch.uint8, device="cuda")
    ok = torch.zeros(F, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    dec.decode_device(x.data_ptr(), F, info.data_ptr(), ok.data_ptr(), 0, s.cuda_stream)
    torch.cuda.synchronize()
    oi, ook = oracle.scl_decode(N, 8, f, llr, crc=8)
    assert np.array_equal(info.cpu().numpy(), oi) and np.array_equal(ok.cpu().numpy(), ook)


def test_nonsystematic_and_edge_batches(pp, oracle):
    N = 256
    f = pp.frozen_bits(N, 128, 0.0)
    rng = np.random.default_rng(0)
    for L in (1, 8):
        dec = pp.PolarDecoder(N, L, f, "gpu")
        dec.setSystematic(False)
        for F in (1, 63, 64, 65, 1000):
            llr = rng.normal(0.5, 1.0, (F, N)).astype(np.float32)
            got = dec.decode_batch(llr)
            exp = (oracle.sc_decode(N, f, llr, systematic=False, crc=8)[0] if L == 1 else
                   oracle.scl_decode(N, L, f, llr, systematic=False, crc=8)[0])
            assert np.array_equal(got, exp), (L, F)
        assert dec.decode_batch(np.zeros((0, N), np.float32)).shape == (0, 16)
