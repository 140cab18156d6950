"""Synthetic BPSK-AWGN polar frames (vectorised numpy), for tests and bench.py.

Follows the reference simulator's chain (src/simulation/simulator.cpp:850-937):
uniform info bytes -> detector generate() over the info bytes -> ButterflyFipPacked
systematic encode (transform, clear frozen, transform: butterfly_fip_packed.cpp:45-58)
-> BPSK (bit 0 -> +1, bpsk.cpp:54-80) -> AWGN with Es/N0 = Eb/N0 * K/N
(simulator.cpp:832-838, awgn.cpp:38-43) -> LLR = 2 y / sigma^2.
"""
import numpy as np

_CRC8_TABLE = None


def _crc8_table():
    global _CRC8_TABLE
    if _CRC8_TABLE is None:
        t = np.zeros(256, np.uint8)
        for i in range(256):
            c = i
            for _ in range(8):
                c = ((c << 1) ^ (0x07 if c & 0x80 else 0)) & 0xFF
            t[i] = c
        _CRC8_TABLE = t
    return _CRC8_TABLE


def _crc16_table():
    t = np.zeros(256, np.uint16)
    for i in range(256):
        c = i << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x1021) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
        t[i] = c
    return t


def _crc32c_table():
    t = np.zeros(256, np.uint32)
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
        t[i] = c
    return t


def crc_generate(kind, data):
    """Detector::generate over each row of `data` (F x bytes, modified copy returned)."""
    d = np.array(data, dtype=np.uint8, copy=True)
    F, B = d.shape
    if kind == 0:
        return d
    if kind == 8:
        t = _crc8_table()
        c = np.zeros(F, np.uint8)
        for i in range(B - 1):
            c = t[c ^ d[:, i]]
        d[:, B - 1] = c
    elif kind == 16:
        t = _crc16_table()
        c = np.full(F, 0xFFFF, np.uint16)
        for i in range(B - 2):
            c = (t[((c >> 8) ^ d[:, i]) & 0xFF] ^ (c << 8)).astype(np.uint16)
        d[:, B - 2] = (c >> 8).astype(np.uint8)
        d[:, B - 1] = (c & 0xFF).astype(np.uint8)
    elif kind == 11:
        # 3GPP TS 38.212 gCRC11 over the bit stream, parity in the last 11 bits
        bits = np.unpackbits(d, axis=1)
        nb = B * 8 - 11
        c = np.zeros(F, np.uint32)
        for i in range(nb):
            fb = ((c >> 10) ^ bits[:, i]) & 1
            c = ((c << 1) & 0x7FF) ^ (fb * 0x621).astype(np.uint32)
        for k in range(11):
            bits[:, nb + k] = (c >> (10 - k)) & 1
        d = np.packbits(bits, axis=1)
    elif kind == 32:
        t = _crc32c_table()
        rw = B // 4 - 1
        c = np.zeros(F, np.uint32)
        for i in range(4 * rw):  # byte-wise reflected CRC-32C == the u32 SSE4.2 form on LE words
            c = t[(c ^ d[:, i]) & 0xFF] ^ (c >> 8)
        d[:, 4 * rw:4 * rw + 4] = c.astype("<u4").view(np.uint8).reshape(F, 4)
    else:
        raise ValueError("CRC INVALID SIZE!")
    return d


def polar_transform(x):
    """x (F x N, uint8 0/1) -> x G_N, in place per stage x[i] ^= x[i + 2^s]."""
    x = np.array(x, dtype=np.uint8, copy=True)
    F, N = x.shape
    B = 1
    while B < N:
        v = x.reshape(F, N // (2 * B), 2, B)
        v[:, :, 0, :] ^= v[:, :, 1, :]
        B *= 2
    return x


def encode(N, frozen, info, systematic=True, crc=0):
    """Packed info bytes (F x ceil(K/8)) -> codeword bits (F x N, uint8)."""
    frozen = np.asarray(list(frozen), dtype=np.int64)
    K = N - len(frozen)
    info = np.atleast_2d(np.asarray(info, dtype=np.uint8))
    if crc:
        info = crc_generate(crc, info[:, :K // 8])
    bits = np.unpackbits(info, axis=1)[:, :K]
    isf = np.zeros(N, bool)
    isf[frozen] = True
    u = np.zeros((info.shape[0], N), np.uint8)
    u[:, ~isf] = bits
    x = polar_transform(u)
    if systematic:
        x[:, isf] = 0
        x = polar_transform(x)
    return x


def awgn_frames(N, frozen, F, ebn0_db=2.0, seed=0, crc=8, systematic=True):
    """Returns (llr F x N float32, info F x ceil(K/8) uint8 incl. the CRC, codeword bits)."""
    K = N - len(list(frozen))
    kb = (K + 7) // 8
    rng = np.random.default_rng(seed)
    info = rng.integers(0, 256, size=(F, kb), dtype=np.uint8)
    if K % 8:
        info[:, -1] &= np.uint8((0xFF << (8 - K % 8)) & 0xFF)
    if crc:
        info = crc_generate(crc, info)
    x = encode(N, frozen, info, systematic=systematic, crc=0)
    esn0 = 10.0 ** (ebn0_db / 10.0) * K / N
    sigma = 1.0 / np.sqrt(2.0 * esn0)
    y = (1.0 - 2.0 * x.astype(np.float32)) + sigma * rng.standard_normal((F, N)).astype(np.float32)
    llr = (2.0 / (sigma * sigma) * y).astype(np.float32)
    return llr, info, x


def nr_frames(E, K, F, ebn0_db=2.0, seed=0, crc=11, N=1024):
    """5G NR uplink-style frames (SURVEY config 4): FiveGList(N, K) frozen set, CRC-11
    over the K info bits (K - 11 payload bits), systematic encode, puncture to E
    (Puncturer(E, frozen): the first N - E frozen positions), BPSK-AWGN at
    Es/N0 = Eb/N0 * K/E.  Returns (llr F x E float32, info F x K/8 uint8, frozen, positions)."""
    from .construction import frozen_bits
    frozen = frozen_bits(N, K, 0.0, "5G")
    nf = len(frozen)
    np_ = N - E
    if np_ > nf:
        raise ValueError("Number of required puncturing positions exceeds frozen bit positions!")
    pos = np.setdiff1d(np.arange(N), np.asarray(frozen[:np_], np.int64))
    kb = (K + 7) // 8
    rng = np.random.default_rng(seed)
    info = rng.integers(0, 256, size=(F, kb), dtype=np.uint8)
    if K % 8:
        info[:, -1] &= np.uint8((0xFF << (8 - K % 8)) & 0xFF)
    if crc:
        info = crc_generate(crc, info)
    x = encode(N, frozen, info, systematic=True, crc=0)[:, pos]
    esn0 = 10.0 ** (ebn0_db / 10.0) * K / E
    sigma = 1.0 / np.sqrt(2.0 * esn0)
    y = (1.0 - 2.0 * x.astype(np.float32)) + sigma * rng.standard_normal((F, E)).astype(np.float32)
    llr = (2.0 / (sigma * sigma) * y).astype(np.float32)
    return llr, info, frozen, pos
