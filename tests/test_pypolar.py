"""The pypolar-compatible host API (CPU parts): construction, encoder, detectors,
decoder construction/validation.  Mirrors python/qa_pypolar_{encoder,detector}.py."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_fixtures.npz")


@pytest.fixture(scope="module")
def pp():
    from antpolarcodes_amd import pypolar
    return pypolar


@pytest.fixture(scope="module")
def fx():
    return np.load(GOLD, allow_pickle=False)


def test_frozen_bits_match_reference(pp, fx):
    off = 0
    for N, K, d, n in zip(fx["cons_N"], fx["cons_K"], fx["cons_dsnr"], fx["cons_len"]):
        exp = [int(v) for v in fx["cons_frozen"][off:off + n]]
        off += n
        assert pp.frozen_bits(int(N), int(K), float(d)) == exp


def test_encoder_matches_reference(pp, fx):
    fr = [int(v) for v in fx["sc_frozen"]]
    for sysm in (0, 1):
        for crc in (0, 8, 32):
            enc = pp.PolarEncoder(1024, fr)
            enc.setSystematic(bool(sysm))
            enc.setErrorDetection(crc)
            for i, row in enumerate(fx["enc_info"]):
                assert np.array_equal(enc.encode_vector(row), fx[f"enc_s{sysm}_c{crc}"][i])


def test_detectors_kat(pp):
    d8, d16, d32 = pp.Detector(8, "cRc"), pp.Detector(16, "crc"), pp.Detector(32, "CRC")
    m = lambda s: np.array([ord(c) for c in s], np.uint8)  # noqa: E731
    assert d8.generate(m("TestFooB"))[-1] == 0xC2
    assert d8.check(np.append(m("ChaoticLama"), 0x67)) and not d8.check(np.append(m("ChaoticLama"), 42))
    assert list(d16.generate(m("Test"))[-2:]) == [0x28, 0x88]
    assert list(d32.generate(m("Test"))[-4:]) == [0x8C, 0x2D, 0xE2, 0x19]
    assert d32.check(np.concatenate([m("DisgustinRoastedWhip"), [0xD0, 0x0B, 0xD6, 0xFE]]).astype(np.uint8))
    with pytest.raises(RuntimeError, match="CRC INVALID SIZE"):
        pp.Detector(12, "crc")
    with pytest.raises(RuntimeError, match="Unknown Error detector"):
        pp.Detector(8, "parity")


def test_decoder_construction_and_errors(pp):
    fr = pp.frozen_bits(256, 128, 0.0)
    dec = pp.PolarDecoder(256, 4, fr, "gpu")
    assert dec.blockLength() == 256 and dec.infoLength() == 128 and dec.listSize() == 4
    assert dec.frozenBits() == fr and dec.isSystematic()
    assert dec.getErrorDetectionMode() == "CRC-8"  # makeDecoder installs CRC-8 (Q5)
    dec.setErrorDetection(32)
    assert dec.getErrorDetectionMode() == "CRC-32"
    dec.setErrorDetection()
    assert dec.getErrorDetectionMode() == "DUMMY-0"
    with pytest.raises(RuntimeError, match="Unknown PolarDecoder type"):
        pp.PolarDecoder(256, 4, fr, "quantum")
    with pytest.raises(RuntimeError, match="ONE-dimensional"):
        dec.decode_vector(np.zeros((2, 128), np.float32))
    with pytest.raises(RuntimeError, match="blockSize"):
        dec.decode_vector(np.zeros(100, np.float32))
    # Fast-SSC rejects the frozen patterns the reference rejects (std::invalid_argument)
    with pytest.raises(ValueError):
        pp.PolarDecoder(8, 1, [1, 2, 4], "gpu")


def test_mixed_is_adaptive_float():
    """create(..., "mixed") -> AdaptiveFloat (decoder.cpp:40-41, 75): constructs both stages,
    so frozen patterns Fast-SSC rejects fail for it too, while "float" SCL accepts them."""
    from antpolarcodes_amd import pypolar as pp
    fr = pp.frozen_bits(1024, 512, 0.0)
    dec = pp.PolarDecoder(1024, 8, fr, "Mixed")
    # AdaptiveFloat::setErrorDetection / setSystematic configure its two stages and leave its
    # own members alone (adaptive_float.cpp:47-57), so the CRC-8 makeDecoder installs is not
    # what its getErrorDetectionMode reports
    assert dec.listSize() == 8 and dec.getErrorDetectionMode() == "DUMMY-0" and dec.isSystematic()
    dec.setSystematic(False)
    assert dec.isSystematic()
    assert pp.PolarDecoder(1024, 1, fr, "mixed").listSize() == 1
    pp.PolarDecoder(8, 4, [1, 2, 4], "float")
    with pytest.raises(ValueError):
        pp.PolarDecoder(8, 4, [1, 2, 4], "mixed")
    with pytest.raises(RuntimeError, match="not part of this build"):
        pp.PolarDecoder(1024, 8, fr, "scan")


def test_adaptive_plan_host_only():
    from antpolarcodes_amd import _native as nat
    fr = list(range(32))
    d = nat.Plan(64, 8, fr, adaptive=True, device=-1).describe()
    assert d["list_size"] == 8
    with pytest.raises(nat.PcgError) as e:
        nat.Plan(8, 4, [1, 2, 4], adaptive=True, device=-1)
    assert e.value.code == nat.PCG_E_FROZEN
