"""The host-buffer path (pcg_decode_f32_host / pcg_decode_i8_host): the batch is cut into
chunks that alternate between two slots, so one chunk's H2D copy overlaps the previous
chunk's decode (capi.cpp decode_host).  Reference callers hand over host buffers the same
way: Decoder::decode_vector (decoder.cpp:154-181), pypolar's decode on numpy arrays
(python/bindings/decoder_python.cc:41-75).  Every staging mode, chunk boundaries that do not
divide the batch, pageable and pinned caller buffers and a slot reused across calls must give
the oracle's bits, ok flags and path metrics."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def code(oracle):
    from antpolarcodes_amd import frames
    N, K = 1024, 512
    fr = oracle.frozen_bits_bb(N, K, 0.0)
    llr, _, _ = frames.awgn_frames(N, fr, 3000, 1.5, seed=17, crc=8)
    return N, fr, llr


@pytest.mark.parametrize("mode", ["0", "1", "2", "2p", "3"])
def test_host_pipeline_three_chunks_scl(oracle, monkeypatch, code, mode):
    """SCL-8 over 3000 frames in chunks of 1024 (three chunks, the last one partial): info, ok
    and metrics bit-exact against the oracle, in every staging mode (2p: staged and copied in
    1 MB pieces, the last one partial); then a second call on the same plan (slots reused) and
    a pinned caller buffer (copied from directly)."""
    import torch
    from antpolarcodes_amd._native import Plan
    N, fr, llr = code
    monkeypatch.setenv("PCG_HOST_PIPE", mode[0])
    monkeypatch.setenv("PCG_HOST_PIECE_MB", "1" if mode == "2p" else "0")
    monkeypatch.setenv("PCG_HOST_CHUNK", "1024")
    oi, ook, om, _, _ = oracle.scl_decode(N, 8, fr, llr, crc=8, paths=True)
    p = Plan(N, 8, fr, crc=8, device=0)
    for rnd in range(2):
        gi, gok, gm = p.decode_host(llr, want_metrics=True)
        assert np.array_equal(gi, oi), (mode, rnd)
        assert np.array_equal(gok, ook), (mode, rnd)
        assert np.array_equal(gm.view(np.uint32), om.view(np.uint32)), (mode, rnd)
    pinned = torch.from_numpy(llr).pin_memory()
    gi, gok, _ = p.decode_host(pinned.numpy())
    assert np.array_equal(gi, oi) and np.array_equal(gok, ook), mode


@pytest.mark.parametrize("mode", ["1", "2", "3"])
def test_host_pipeline_sc_and_int8(oracle, monkeypatch, code, mode):
    """Fast-SSC float frames and the 8-bit list decoder on int8 frames through the pipeline
    (odd chunk size: 7 chunks of 448 frames, the last one partial), and a batch smaller than
    one chunk."""
    from antpolarcodes_amd._native import Plan
    N, fr, llr = code
    monkeypatch.setenv("PCG_HOST_PIPE", mode)
    monkeypatch.setenv("PCG_HOST_CHUNK", "448")
    monkeypatch.setenv("PCG_HOST_PIECE_MB", "1")  # (448 frames = 1.75 MB: two pieces per chunk)
    p = Plan(N, 1, fr, crc=8, device=0)
    gi, gok, _ = p.decode_host(llr)
    oi, ook = oracle.sc_decode(N, fr, llr, crc=8)
    assert np.array_equal(gi, oi) and np.array_equal(gok, ook)
    gi, gok, _ = p.decode_host(llr[:5])
    assert np.array_equal(gi, oi[:5]) and np.array_equal(gok, ook[:5])
    x8 = np.clip(np.rint(llr * 8.0), -128, 127).astype(np.int8)
    q = Plan(N, 4, fr, crc=8, device=0, fixed=True)
    gi, gok, gm = q.decode_host_i8(x8, want_metrics=True)
    ei, eok = oracle.sclc_decode(N, 4, fr, x8, crc=8)[:2]
    assert np.array_equal(gi, ei) and np.array_equal(gok, eok)
