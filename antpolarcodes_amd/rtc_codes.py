"""The catalogue of codes whose plan-specialised kernels ship with the library
(antpolarcodes_amd/lib/rtc/, filled by antpolarcodes_amd/rtc_warm.py at build time).

A code outside this catalogue still specialises: its kernel is compiled by hiprtc in the
background on first use (rtc.cpp) and kept in the user cache.  What ships is

  * the benchmark configurations (SURVEY.md configs 2-5, and the adaptive / 8-bit variants
    bench.py decodes), and
  * a validation catalogue: codes chosen so that the specialised kernels meet every node
    kind the reference's decoder trees build (FastSscAvx::createDecoder,
    fastssc_avx_float.cpp:797-896; SclAvx::createDecoder, scl_avx_float.cpp:624-651;
    FastSscFip / SclFip, fastssc_fip_char.cpp, scl_fip_char.cpp), every detector, systematic
    and not, a few list sizes that are not powers of two, and random frozen sets.

The GPU parity tests draw their specialised-kernel codes from this catalogue (so a fresh
machine runs them without compiling); the product never imports the tests.

An entry is (N, L, frozen spec, crc, systematic[, variant]): frozen spec ("BB", K) is the
Bhattacharyya construction at 0 dB design SNR, ("5G", K) the 3GPP reliability sequence,
("set", positions) an explicit frozen set; variant "adaptive", "char" or "adaptive_char".
"""


def bench_codes():
    """(N, L, frozen spec, crc, systematic[, variant]): the configurations bench.py decodes."""
    return [
        (1024, 1, ("BB", 512), 8, True),     # config 2
        (1024, 8, ("BB", 512), 8, True),     # config 3
        (1024, 8, ("BB", 512), 8, True, "adaptive"),  # config 3 with AdaptiveFloat (both stages)
        (1024, 8, ("5G", 512), 11, True),    # config 4
        (4096, 32, ("BB", 2048), 8, True),   # config 5
        (1024, 1, ("BB", 512), 8, True, "char"),      # sc_char
        (1024, 8, ("BB", 512), 8, True, "char"),      # scl8_char
        (1024, 8, ("BB", 512), 8, True, "adaptive_char"),  # adaptive8_char (both stages)
    ]


def node_cover_sets():
    """(N, frozen) pairs whose Fast-SSC trees contain every leaf kind at several sizes."""
    out = []
    # 8-bit specials
    out.append((8, [0, 1]))                 # DoubleSpcShort8
    out.append((8, [0, 1, 2]))              # RepRateOne8
    out.append((8, [0, 1, 2, 3, 4]))        # ZeroSpc8
    out.append((8, [0, 1, 2, 4]))           # TypeFive n=8
    out.append((8, [0, 1, 2, 3, 4, 5]))     # DoubleRep n=8
    for n in (16, 32, 64, 128):
        out.append((n, [0, 1]))                                  # DoubleSpc
        out.append((n, list(range(n - 3))))                      # TripleRep
        out.append((n, sorted(set(range(n - 6)) | {n - 6, n - 4})))  # TypeFive
        out.append((n, list(range(n - 2))))                      # DoubleRep
        out.append((n, list(range(n // 2)) + [n // 2]))          # ZeroSpc (Q1)
        out.append((n, list(range(n // 2 - 1))))                 # ROne at the root
        out.append((n, list(range(n // 2)) + [n // 2, n // 2 + 1]))  # ZeroR at the root
    # ShortRateR with n<8 leaves under it
    out.append((8, [0, 4]))
    out.append((8, [1, 2, 4]))
    out.append((16, [0, 2, 8]))
    return out


def char_cover_codes():
    """(N, frozen) pairs covering the 8-bit Fast-SSC node kinds (FastSscFip*, incl. Short)."""
    out = []
    for n in (8, 16, 32, 64, 128, 256):
        h = n // 2
        out += [(n, list(range(n - 1))), (n, [0]), (n, list(range(n - 2))), (n, list(range(h))),
                (n, list(range(h)) + [h]), (n, list(range(h - 1))),
                (n, sorted(set(list(range(h)) + [h, h + 1, h + 3]))), (n, sorted({0, 1, 2, 4, h, h + 1}))]
    return out


def _xorshift(seed):
    """A 32-bit xorshift stream: the random catalogue entries are the same on every machine
    and Python version."""
    x = seed & 0xFFFFFFFF or 1
    while True:
        x ^= (x << 13) & 0xFFFFFFFF
        x ^= x >> 17
        x ^= (x << 5) & 0xFFFFFFFF
        yield x


def random_list_codes():
    """(N, L, frozen) random frozen sets for the specialised list kernel (scl_rtc_kernel):
    short codes (short compiles), list sizes 3, 8 and 32, any number of frozen positions."""
    g = _xorshift(0x5C1A11)
    out = []
    for N, L in ((32, 3), (64, 8), (128, 32), (256, 3), (256, 8), (128, 8), (64, 32), (256, 32)):
        nf = 1 + next(g) % (N - 1)
        pos = list(range(N))
        for i in range(N - 1, 0, -1):  # Fisher-Yates
            j = next(g) % (i + 1)
            pos[i], pos[j] = pos[j], pos[i]
        out.append((N, L, sorted(pos[:nf])))
    # longer codes: trees whose quarters (stage top-2) are recomputed from the channel inside the
    # staged ops, with a fused / unfused child and both recomputed levels (own stream: the entries
    # above keep their frozen sets and cache files)
    g = _xorshift(0x5C1A12)
    for N, L in ((512, 8), (1024, 8), (1024, 4), (64, 2), (256, 5), (512, 16), (1024, 32), (2048, 8), (1024, 12)):
        nf = N // 4 + next(g) % (N // 2)
        pos = list(range(N))
        for i in range(N - 1, 0, -1):
            j = next(g) % (i + 1)
            pos[i], pos[j] = pos[j], pos[i]
        out.append((N, L, sorted(pos[:nf])))
    return out


def validation_codes():
    """The codes the GPU parity tests run through specialised kernels (tests/test_gpu_rtc.py,
    tests/test_gpu_char.py and the specialised variants of the full-size parity tests)."""
    out = []
    for N in (8, 32, 128, 512, 1024):                      # BB codes, Fast-SSC
        out.append((N, 1, ("BB", max(8, N // 2)), 8, True))
    for sysm in (True, False):                            # detectors, systematic or not
        for crc in (0, 16, 32):
            out.append((1024, 1, ("BB", 512), crc, sysm))
    for N, fr in node_cover_sets():                       # every Fast-SSC leaf kind
        out.append((N, 1, ("set", tuple(fr)), 8, True))
    for N, K, L, crc, sysm in ((256, 128, 4, 16, True), (1024, 512, 8, 8, True), (512, 256, 6, 32, False),
                               (4096, 2048, 32, 8, True), (1024, 512, 12, 8, True), (1024, 512, 8, 0, True)):
        out.append((N, L, ("BB", K), crc, sysm))          # list plans
    for N, L, fr in random_list_codes():                  # list plans on random frozen sets
        out.append((N, L, ("set", tuple(fr)), 0, True))
    out.append((1024, 8, ("5G", 512), 0, True))           # config 4's decoder core with the Dummy detector
    out.append((1024, 1, ("5G", 512), 11, True))          # config 4 through Fast-SSC
    for crc in (8, 16, 32):                               # AdaptiveFloat: both stages
        out.append((1024, 8, ("BB", 512), crc, True, "adaptive"))
    for N, fr, sysm, crc in char_rtc_codes():             # FastSscFipChar
        out.append((N, 1, ("set", tuple(fr)), crc, sysm, "char"))
    for N, K, L, crc, sysm in ((256, 128, 2, 8, True), (1024, 512, 8, 8, True), (512, 256, 4, 16, False),
                               (1024, 512, 16, 32, True), (1024, 512, 32, 8, True), (1024, 512, 6, 0, True)):
        out.append((N, L, ("BB", K), crc, sysm, "char"))  # SclFipChar
    for crc in (8, 16):                                   # AdaptiveChar: both stages
        out.append((1024, 8, ("BB", 512), crc, True, "adaptive_char"))
    return out


def char_rtc_codes():
    """(N, frozen, systematic, crc) of the 8-bit Fast-SSC validation codes."""
    from .construction import frozen_bits
    out = [(N, [int(v) for v in frozen_bits(N, max(8, N // 2), 0.0)], True, 8) for N in (8, 32, 128, 256, 1024)]
    out += [(64, fr, True, 0) for n, fr in char_cover_codes() if n == 64]
    fr = [int(v) for v in frozen_bits(1024, 512, 0.0)]
    out += [(1024, fr, sysm, crc) for sysm in (True, False) for crc in (0, 16, 32)]
    return out


def _key(c):
    return tuple(c[:2]) + tuple(c[2]) + tuple(c[3:])


def codes():
    """The whole catalogue, each code once."""
    seen, out = set(), []
    for c in bench_codes() + validation_codes():
        if _key(c) not in seen:
            seen.add(_key(c))
            out.append(c)
    return out
