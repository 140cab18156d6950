"""The C++ boundary, compiled the way a reference maintainer would use it:

* tests/cpp/subclass_decoder.cpp -- a reference-style Decoder subclass (containers in
  initialize(), decode() over mLlrContainer / mOutputContainer);
* tests/cpp/reference_callers.cpp -- the reference simulator's own call sequences against the
  reference's include paths and class names: the encoder sequence setInformation -> encode ->
  getEncodedData (simulator.cpp:869-875) checked against the reference's encoder fixtures, a
  reference-style Encoder subclass overriding encode(), makeDecoder's default (8-bit)
  decoders, BitContainer formats; and (GPU) the decoder sequence setSignal -> decode ->
  packedOutput of setCoders' decoder classes (simulator.cpp:703-764, 920-937).

Built with g++ against include/ and libpolarcode_amd.so; the CPU parts run here.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "antpolarcodes_amd", "lib")
GOLD = os.path.join(ROOT, "tests", "golden", "reference_fixtures.npz")
needs_gxx = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


def build(tmp_path, name):
    exe = str(tmp_path / name)
    src = os.path.join(ROOT, "tests", "cpp", f"{name}.cpp")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), src, "-o", exe,
                        "-L", LIB, "-lpolarcode_amd", "-lpcg", f"-Wl,-rpath,{LIB}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


@needs_gxx
def test_reference_style_subclass_compiles_and_runs(tmp_path):
    exe = build(tmp_path, "subclass_decoder")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "subclass_decoder ok" in r.stdout


@needs_gxx
def test_reference_callers_api(tmp_path):
    exe = build(tmp_path, "reference_callers")
    r = subprocess.run([exe, "api"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "api ok" in r.stdout


def _encode(exe, tmp_path, N, frozen, info, sys, crc):
    fp, ip = tmp_path / "frozen.txt", tmp_path / "info.bin"
    fp.write_text(" ".join(str(int(v)) for v in frozen))
    ip.write_bytes(np.asarray(info, np.uint8).tobytes())
    r = subprocess.run([exe, "encode", str(N), str(int(sys)), str(crc), str(fp), str(ip)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    code, info_out = r.stdout.split()
    return np.frombuffer(bytes.fromhex(code), np.uint8), np.frombuffer(bytes.fromhex(info_out), np.uint8)


@needs_gxx
def test_simulator_encoder_sequence_matches_reference_fixtures(tmp_path):
    """setInformation -> encode -> getEncodedData (and encode_vector, and the reference-style
    subclass) give the reference's own encoder outputs (make_golden.py enc_* fixtures)."""
    exe = build(tmp_path, "reference_callers")
    fx = np.load(GOLD, allow_pickle=False)
    fr = fx["sc_frozen"]
    for sysm in (0, 1):
        for crc in (0, 8, 32):
            for i, row in enumerate(fx["enc_info"]):
                code, _ = _encode(exe, tmp_path, 1024, fr, row, sysm, crc)
                assert np.array_equal(code, fx[f"enc_s{sysm}_c{crc}"][i]), (sysm, crc, i)


@needs_gxx
def test_simulator_encoder_sequence_small_codes(tmp_path, oracle):
    """Codes below 256 bits live at the end of the PackedContainer's 256-bit buffer (the
    reference's mFakeSize): N = 8 ... 512 against the oracle encoder (pinned to the reference)."""
    exe = build(tmp_path, "reference_callers")
    rng = np.random.default_rng(5)
    for N in (8, 16, 32, 64, 128, 256, 512):
        K = N // 2
        fr = oracle.frozen_bits_bb(N, K, 0.0)
        for sysm in (0, 1):
            for crc in ((0, 8) if K >= 16 else (0,)):
                info = rng.integers(0, 256, (K + 7) // 8, dtype=np.uint8)
                code, info_out = _encode(exe, tmp_path, N, fr, info, sysm, crc)
                exp = oracle.encode(N, fr, info[None, :], systematic=bool(sysm), crc=crc)
                assert np.array_equal(code, np.asarray(exp).reshape(-1)), (N, sysm, crc)


@pytest.mark.gpu
@needs_gxx
def test_simulator_decoder_sequence_on_gpu(tmp_path, oracle):
    """setCoders' decoders (FastSscAvxFloat, AdaptiveFloat, AdaptiveMixed, SclAvxFloat by their
    reference names) through setSignal -> decode -> packedOutput, one frame at a time, equal the
    oracle; outputContainer() holds the decoded codeword and getSoftCodeword's signs are the
    selected path's codeword (the reference's mBitContainer, scl_avx_float.cpp:711-750)."""
    from antpolarcodes_amd import frames
    exe = build(tmp_path, "reference_callers")
    fr = oracle.frozen_bits_bb(1024, 512, 0.0)
    F = 24
    llr, _, _ = frames.awgn_frames(1024, fr, F, 1.25, seed=77, crc=8)
    (tmp_path / "frozen.txt").write_text(" ".join(str(v) for v in fr))
    (tmp_path / "llr.bin").write_bytes(np.ascontiguousarray(llr, np.float32).tobytes())
    r = subprocess.run([exe, "gpu", str(tmp_path / "frozen.txt"), str(tmp_path / "llr.bin"), str(F)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "gpu ok" in r.stdout
    sc_i, sc_k = oracle.sc_decode(1024, fr, llr, crc=8)
    scl_i, scl_k = oracle.scl_decode(1024, 8, fr, llr, crc=8)
    # AdaptiveMixed's first stage is the 8-bit decoder on the quantised floats
    mx_i, mx_k = oracle.scc_decode(1024, fr, llr, crc=8)
    ad_i, ad_k = sc_i.copy(), sc_k.copy()
    bad = sc_k == 0
    ad_i[bad], ad_k[bad] = scl_i[bad], scl_k[bad]
    bad8 = mx_k == 0
    mx_i[bad8], mx_k[bad8] = scl_i[bad8], scl_k[bad8]
    # SclAvxFloat decoded one frame after another by one instance carries path 0's metric (Q8):
    # its expected outputs come from the oracle's carried decode
    cs_i, cs_k = oracle.scl_decode(1024, 8, fr, llr, crc=8, carry=True)[:2]
    exp = {0: (sc_i, sc_k), 1: (ad_i, ad_k), 2: (mx_i, mx_k), 3: (cs_i, cs_k)}
    enc = {k: oracle.encode(1024, fr, v[0], systematic=True, crc=0) for k, v in exp.items()}
    for line in r.stdout.splitlines():
        if line.endswith("ok"):
            continue
        k, f, okv, info, cw, soft = line.split()
        k, f = int(k), int(f)
        assert int(okv) == int(exp[k][1][f]), (k, f)
        assert np.array_equal(np.frombuffer(bytes.fromhex(info), np.uint8), exp[k][0][f]), (k, f)
        assert np.array_equal(np.frombuffer(bytes.fromhex(cw), np.uint8), np.asarray(enc[k])[f]), (k, f)
        # getSoftCodeword's signs: the selected path's codeword (systematic: the encoding of the
        # decoded information), for the soft Fast-SSC codeword and the list / adaptive decoders alike
        assert np.array_equal(np.frombuffer(bytes.fromhex(soft), np.uint8), np.asarray(enc[k])[f]), (k, f)
