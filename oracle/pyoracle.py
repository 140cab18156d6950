"""ctypes bindings for the oracle (TEST INFRASTRUCTURE ONLY).

* ``Oracle``     -> oracle/liboracle.so, the plain-C restatement (polar_oracle.c)
* ``Reference``  -> oracle/_ref/libpolarref.so, the reference library compiled from
                    /root/reference's own sources + ref_harness.cpp (oracle/Makefile)

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  The product package (antpolarcodes_amd) never does.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libpolarref.so")

_P = C.c_void_p
_U32 = C.c_uint32
_U64 = C.c_uint64
_I = C.c_int


def _p(a):
    return None if a is None else a.ctypes.data


def _frozen(frozen):
    return np.ascontiguousarray(np.asarray(frozen, dtype=np.uint32))


class Oracle:
    """CPU restatement of the reference Fast-SSC / SCL decoders (bit-exact)."""

    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle oracle`")
        lib = C.CDLL(path)
        lib.orc_sc_decode.argtypes = [_U32, _P, _U32, _I, _I, _P, _U64, _P, _P, _P]
        lib.orc_scl_decode.argtypes = [_U32, _U32, _P, _U32, _I, _I, _I, _P, _U64, _P, _P, _P, _P, _P]
        lib.orc_encode.argtypes = [_U32, _P, _U32, _I, _I, _P, _U64, _P]
        lib.orc_crc.argtypes = [_I, _I, _P, _I]
        lib.orc_sc_tree.argtypes = [_U32, _P, _U32, _P, _P, _I]
        lib.orc_frozen_bits_bb.argtypes = [_U32, _U32, C.c_float, _P]
        lib.orc_bench.argtypes = [_U32, _U32, _P, _U32, _P, _U64, _I]
        lib.orc_bench.restype = C.c_double
        lib.orc_f.argtypes = [_P, _P, _U32]
        lib.orc_g.argtypes = [_P, _P, _P, _U32]
        lib.orc_combine_short.argtypes = [_P, _P, _P, _U32]
        lib.orc_puncturer.argtypes = [_U32, _P, _U32, _P, _P]
        lib.orc_depuncture.argtypes = [_U32, _U32, _P, _P, _U64, _P]
        lib.orc_depuncture.restype = None
        lib.orc_puncture_packed.argtypes = [_U32, _P, _P, _P]
        lib.orc_puncture_packed.restype = None
        # int8 ("char") decoders, polar_oracle_char.c
        lib.orc_f32_to_i8.argtypes = [_P, _U32, _U64, _P]
        lib.orc_f32_to_i8.restype = None
        lib.orc_scc_decode.argtypes = [_U32, _P, _U32, _I, _I, _P, _U64, _P, _P, _P]
        lib.orc_sclc_decode.argtypes = [_U32, _U32, _P, _U32, _I, _I, _I, _P, _U64, _P, _P, _P, _P, _P]
        lib.orc_scc_tree.argtypes = [_U32, _P, _U32, _P, _P, _I]
        lib.orc_sclc_tree.argtypes = [_U32, _P, _U32, _P, _P, _I]
        for fn, n in (("orc_fip_f", 3), ("orc_fip_g", 4), ("orc_fip_combine_short", 4)):
            getattr(lib, fn).argtypes = [_P] * (n - 1) + [_U32]
            getattr(lib, fn).restype = None
        self.lib = lib

    def f(self, left, right):
        x = np.ascontiguousarray(np.concatenate([left, right]), np.float32)
        out = np.zeros(len(left), np.float32)
        self.lib.orc_f(_p(x), _p(out), len(left))
        return out

    def g(self, left, right, bits):
        x = np.ascontiguousarray(np.concatenate([left, right]), np.float32)
        b = np.ascontiguousarray(bits, np.float32)
        out = np.zeros(len(left), np.float32)
        self.lib.orc_g(_p(x), _p(b), _p(out), len(left))
        return out

    def combine_short(self, left, right, h):
        l8 = np.ascontiguousarray(left, np.float32)
        r8 = np.ascontiguousarray(right, np.float32)
        out = np.zeros(8, np.float32)
        self.lib.orc_combine_short(_p(l8), _p(r8), _p(out), h)
        return out

    def sc_decode(self, N, frozen, llr, systematic=True, crc=-1, soft=False):
        fr = _frozen(frozen)
        llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, N)
        F = llr.shape[0]
        kb = (N - len(fr) + 7) // 8
        info = np.zeros((F, kb), np.uint8)
        ok = np.zeros(F, np.uint8)
        cw = np.zeros((F, N), np.float32) if soft else None
        r = self.lib.orc_sc_decode(N, _p(fr), len(fr), int(systematic), crc, _p(llr), F,
                                   _p(info), _p(ok), _p(cw))
        if r != 0:
            raise ValueError(f"orc_sc_decode failed ({r})")
        return (info, ok, cw) if soft else (info, ok)

    def scl_decode(self, N, L, frozen, llr, systematic=True, crc=-1, carry=False, paths=False):
        fr = _frozen(frozen)
        llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, N)
        F = llr.shape[0]
        kb = (N - len(fr) + 7) // 8
        info = np.zeros((F, kb), np.uint8)
        ok = np.zeros(F, np.uint8)
        met = np.zeros((F, L), np.float32) if paths else None
        pc = np.zeros(F, np.uint32) if paths else None
        pb = np.zeros((F, L, N // 8), np.uint8) if paths else None
        r = self.lib.orc_scl_decode(N, L, _p(fr), len(fr), int(systematic), crc, int(carry),
                                    _p(llr), F, _p(info), _p(ok), _p(met), _p(pc), _p(pb))
        if r != 0:
            raise ValueError(f"orc_scl_decode failed ({r})")
        return (info, ok, met, pc, pb) if paths else (info, ok)

    def encode(self, N, frozen, info, systematic=True, crc=0):
        fr = _frozen(frozen)
        kb = (N - len(fr) + 7) // 8
        info = np.ascontiguousarray(info, dtype=np.uint8).reshape(-1, kb)
        code = np.zeros((info.shape[0], N // 8), np.uint8)
        r = self.lib.orc_encode(N, _p(fr), len(fr), int(systematic), crc, _p(info), info.shape[0], _p(code))
        if r != 0:
            raise ValueError("orc_encode failed")
        return code

    def crc(self, kind, data, generate=False):
        d = np.array(data, dtype=np.uint8).copy()
        r = self.lib.orc_crc(kind, int(generate), _p(d), len(d))
        return d if generate else bool(r > 0)

    def sc_tree(self, N, frozen):
        fr = _frozen(frozen)
        t = np.zeros(4 * N, np.int32)
        s = np.zeros(4 * N, np.int32)
        k = self.lib.orc_sc_tree(N, _p(fr), len(fr), _p(t), _p(s), 4 * N)
        if k < 0:
            raise ValueError(f"invalid frozen set for Fast-SSC ({k})")
        return t[:k], s[:k]

    def puncturer(self, E, frozen):
        """(parent N, kept positions) of Puncturer(E, frozen)."""
        fr = _frozen(frozen)
        pos = np.zeros(2 * E + 8, np.uint32)
        n = np.zeros(1, np.uint32)
        r = self.lib.orc_puncturer(E, _p(fr), len(fr), _p(n), _p(pos))
        if r < 0:
            raise ValueError("Number of required puncturing positions exceeds frozen bit positions!")
        return int(n[0]), pos[:r].copy()

    def depuncture(self, E, frozen, x):
        N, pos = self.puncturer(E, frozen)
        x = np.ascontiguousarray(x, np.float32).reshape(-1, E)
        out = np.zeros((x.shape[0], N), np.float32)
        self.lib.orc_depuncture(E, N, _p(pos), _p(x), x.shape[0], _p(out))
        return out

    def puncture_packed(self, E, frozen, x):
        _, pos = self.puncturer(E, frozen)
        x = np.ascontiguousarray(x, np.uint8)
        out = np.zeros(E // 8, np.uint8)
        self.lib.orc_puncture_packed(E, _p(pos), _p(x), _p(out))
        return out

    def frozen_bits_bb(self, N, K, dsnr):
        out = np.zeros(N, np.uint32)
        n = self.lib.orc_frozen_bits_bb(N, K, dsnr, _p(out))
        return [int(v) for v in out[:n]]

    def bench(self, N, L, frozen, llr, reps=1):
        fr = _frozen(frozen)
        llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, N)
        return self.lib.orc_bench(N, L, _p(fr), len(fr), _p(llr), llr.shape[0], reps)

    # ---- int8 ("char") decoders ------------------------------------------------------
    def f32_to_i8(self, llr, N):
        """CharContainer::insertLlr(const float*) for frames of N floats."""
        x = np.ascontiguousarray(llr, np.float32).reshape(-1, N)
        out = np.zeros(x.shape, np.int8)
        self.lib.orc_f32_to_i8(_p(x), N, x.shape[0], _p(out))
        return out

    def _i8(self, llr, N):
        llr = np.asarray(llr)
        if llr.dtype != np.int8:
            return self.f32_to_i8(llr, N)
        return np.ascontiguousarray(llr).reshape(-1, N)

    def scc_decode(self, N, frozen, llr, systematic=True, crc=-1, soft=False):
        """FastSscFipChar; llr int8 (or float, quantised as insertLlr does)."""
        fr = _frozen(frozen)
        llr = self._i8(llr, N)
        F = llr.shape[0]
        kb = (N - len(fr) + 7) // 8
        info = np.zeros((F, kb), np.uint8)
        ok = np.zeros(F, np.uint8)
        cw = np.zeros((F, N), np.int8) if soft else None
        r = self.lib.orc_scc_decode(N, _p(fr), len(fr), int(systematic), crc, _p(llr), F,
                                    _p(info), _p(ok), _p(cw))
        if r != 0:
            raise ValueError(f"orc_scc_decode failed ({r})")
        return (info, ok, cw) if soft else (info, ok)

    def sclc_decode(self, N, L, frozen, llr, systematic=True, crc=-1, carry=False, paths=False):
        """SclFipChar; metrics are int64."""
        fr = _frozen(frozen)
        llr = self._i8(llr, N)
        F = llr.shape[0]
        kb = (N - len(fr) + 7) // 8
        info = np.zeros((F, kb), np.uint8)
        ok = np.zeros(F, np.uint8)
        met = np.zeros((F, L), np.int64) if paths else None
        pc = np.zeros(F, np.uint32) if paths else None
        pb = np.zeros((F, L, N // 8), np.uint8) if paths else None
        r = self.lib.orc_sclc_decode(N, L, _p(fr), len(fr), int(systematic), crc, int(carry),
                                     _p(llr), F, _p(info), _p(ok), _p(met), _p(pc), _p(pb))
        if r != 0:
            raise ValueError(f"orc_sclc_decode failed ({r})")
        return (info, ok, met, pc, pb) if paths else (info, ok)

    def fip_f(self, left, right):
        x = np.ascontiguousarray(np.concatenate([left, right]), np.int8)
        h = len(left)
        out = np.zeros(max(h, 32), np.int8)
        self.lib.orc_fip_f(_p(x), _p(out), h)
        return out[:h]

    def fip_g(self, left, right, bits):
        x = np.ascontiguousarray(np.concatenate([left, right]), np.int8)
        b = np.ascontiguousarray(bits, np.int8)
        h = len(left)
        out = np.zeros(max(h, 32), np.int8)
        self.lib.orc_fip_g(_p(x), _p(b), _p(out), h)
        return out[:h]

    def fip_combine_short(self, left, right, h):
        l = np.array(left, np.int8)
        r = np.array(right, np.int8)
        out = np.zeros(32, np.int8)
        self.lib.orc_fip_combine_short(_p(l), _p(r), _p(out), h)
        return out

    def char_tree(self, N, frozen, L=1):
        fr = _frozen(frozen)
        t = np.zeros(4 * N, np.int32)
        s = np.zeros(4 * N, np.int32)
        fn = self.lib.orc_scc_tree if L == 1 else self.lib.orc_sclc_tree
        k = fn(N, _p(fr), len(fr), _p(t), _p(s), 4 * N)
        if k < 0:
            raise ValueError(f"invalid frozen set ({k})")
        return t[:k], s[:k]


class Reference:
    """The reference library itself (only where oracle/_ref was built)."""

    def __init__(self, path=REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        lib = C.CDLL(path)
        lib.ref_frozen_bits.argtypes = [_U32, _U32, C.c_float, C.c_char_p, _P]
        lib.ref_decode.argtypes = [_U32, _U32, _P, _U32, _I, _I, _P, _U64, _P, _P, _P]
        lib.ref_scl_paths.argtypes = [_U32, _U32, _P, _U32, _P, _U64, _P, _P, _P]
        lib.ref_encode.argtypes = [_U32, _P, _U32, _I, _I, _P, _U64, _P]
        lib.ref_crc.argtypes = [_I, _I, _P, _I]
        lib.ref_bench.argtypes = [_U32, _U32, _P, _U32, _I, _I, _P, _U64, _I, _I]
        lib.ref_bench.restype = C.c_double
        lib.ref_last_error.restype = C.c_char_p
        lib.ref_puncturer.argtypes = [_U32, _P, _U32, _P, _P]
        lib.ref_punc_apply.argtypes = [_U32, _P, _U32, _I, _P, _P]
        lib.ref_f32_to_i8.argtypes = [_U32, _P, _U64, _P]
        lib.ref_decode_char.argtypes = [_U32, _U32, _P, _U32, _I, _I, _I, _P, _U64, _P, _P, _P]
        lib.ref_sclc_paths.argtypes = [_U32, _U32, _P, _U32, _P, _U64, _P, _P, _P]
        lib.ref_bench_char.argtypes = [_U32, _U32, _P, _U32, _I, _I, _P, _U64, _I, _I]
        lib.ref_bench_char.restype = C.c_double
        self.lib = lib

    @staticmethod
    def available():
        return os.path.exists(REF_SO)

    def frozen_bits(self, N, K, dsnr, kind="BB"):
        out = np.zeros(N, np.uint32)
        n = self.lib.ref_frozen_bits(N, K, dsnr, kind.encode(), _p(out))
        if n < 0:
            raise ValueError(self.lib.ref_last_error().decode())
        return [int(v) for v in out[:n]]

    def decode(self, N, L, frozen, llr, systematic=True, crc=-1, soft=False, fresh=False):
        """fresh=True builds a new decoder per frame (no SCL metric carry, Q8)."""
        fr = _frozen(frozen)
        llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, N)
        F = llr.shape[0]
        kb = (N - len(fr) + 7) // 8
        info = np.zeros((F, kb), np.uint8)
        ok = np.zeros(F, np.uint8)
        cw = np.zeros((F, N), np.float32) if soft else None
        if fresh:
            for f in range(F):
                r = self.lib.ref_decode(N, L, _p(fr), len(fr), int(systematic), crc, _p(llr[f:f + 1]), 1,
                                        _p(info[f:f + 1]), _p(ok[f:f + 1]),
                                        None if cw is None else _p(cw[f:f + 1]))
                if r != 0:
                    raise ValueError(self.lib.ref_last_error().decode())
        else:
            r = self.lib.ref_decode(N, L, _p(fr), len(fr), int(systematic), crc, _p(llr), F,
                                    _p(info), _p(ok), _p(cw))
            if r != 0:
                raise ValueError(self.lib.ref_last_error().decode())
        return (info, ok, cw) if soft else (info, ok)

    def scl_paths(self, N, L, frozen, llr, fresh=True):
        fr = _frozen(frozen)
        llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, N)
        F = llr.shape[0]
        met = np.zeros((F, L), np.float32)
        pc = np.zeros(F, np.uint32)
        pb = np.zeros((F, L, N // 8), np.uint8)
        rng = [(f, f + 1) for f in range(F)] if fresh else [(0, F)]
        for a, b in rng:
            r = self.lib.ref_scl_paths(N, L, _p(fr), len(fr), _p(llr[a:b]), b - a,
                                       _p(met[a:b]), _p(pc[a:b]), _p(pb[a:b]))
            if r != 0:
                raise ValueError(self.lib.ref_last_error().decode())
        return met, pc, pb

    def encode(self, N, frozen, info, systematic=True, crc=0):
        fr = _frozen(frozen)
        kb = (N - len(fr) + 7) // 8
        info = np.ascontiguousarray(info, dtype=np.uint8).reshape(-1, kb)
        code = np.zeros((info.shape[0], N // 8), np.uint8)
        r = self.lib.ref_encode(N, _p(fr), len(fr), int(systematic), crc, _p(info), info.shape[0], _p(code))
        if r != 0:
            raise ValueError(self.lib.ref_last_error().decode())
        return code

    def crc(self, kind, data, generate=False):
        d = np.array(data, dtype=np.uint8).copy()
        r = self.lib.ref_crc(kind, int(generate), _p(d), len(d))
        return d if generate else bool(r > 0)

    def puncturer(self, E, frozen):
        """Puncturer(E, frozen): (parent N, kept positions)."""
        fr = _frozen(frozen)
        pos = np.zeros(2 * E + 8, np.uint32)
        n = np.zeros(1, np.uint32)
        r = self.lib.ref_puncturer(E, _p(fr), len(fr), _p(n), _p(pos))
        if r < 0:
            raise ValueError(self.lib.ref_last_error().decode())
        return int(n[0]), pos[:r].copy()

    def punc_apply(self, E, frozen, op, x):
        """op 0 depuncture (E floats -> N), 1 puncture (N floats -> E), 2 puncturePacked."""
        fr = _frozen(frozen)
        N, _ = self.puncturer(E, frozen)
        if op == 2:
            x = np.ascontiguousarray(x, np.uint8)
            out = np.zeros(E // 8, np.uint8)
        else:
            x = np.ascontiguousarray(x, np.float32)
            out = np.zeros(N if op == 0 else E, np.float32)
        r = self.lib.ref_punc_apply(E, _p(fr), len(fr), op, _p(x), _p(out))
        if r < 0:
            raise ValueError(self.lib.ref_last_error().decode())
        return out

    def bench(self, N, L, frozen, llr, threads=1, reps=1, systematic=True, crc=-1):
        fr = _frozen(frozen)
        llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, N)
        return self.lib.ref_bench(N, L, _p(fr), len(fr), int(systematic), crc, _p(llr), llr.shape[0],
                                  threads, reps)

    # ---- int8 ("char") decoders ------------------------------------------------------
    def f32_to_i8(self, llr, N):
        x = np.ascontiguousarray(llr, np.float32).reshape(-1, N)
        out = np.zeros(x.shape, np.int8)
        if self.lib.ref_f32_to_i8(N, _p(x), x.shape[0], _p(out)) != 0:
            raise ValueError(self.lib.ref_last_error().decode())
        return out

    def decode_char(self, N, L, frozen, llr, systematic=True, crc=-1, soft=False, fresh=False):
        """create(N, L, frozen, "char"): int8 llr -> decode_vector(const char*), float llr ->
        decode_vector(const float*).  fresh=True: one decoder per frame."""
        fr = _frozen(frozen)
        llr = np.asarray(llr)
        is_i8 = llr.dtype == np.int8
        llr = np.ascontiguousarray(llr, dtype=np.int8 if is_i8 else np.float32).reshape(-1, N)
        F = llr.shape[0]
        kb = (N - len(fr) + 7) // 8
        info = np.zeros((F, kb), np.uint8)
        ok = np.zeros(F, np.uint8)
        cw = np.zeros((F, N), np.int8) if soft else None
        rng = [(f, f + 1) for f in range(F)] if fresh else [(0, F)]
        for a, b in rng:
            r = self.lib.ref_decode_char(N, L, _p(fr), len(fr), int(systematic), crc, int(is_i8),
                                         _p(llr[a:b]), b - a, _p(info[a:b]), _p(ok[a:b]),
                                         None if cw is None else _p(cw[a:b]))
            if r != 0:
                raise ValueError(self.lib.ref_last_error().decode())
        return (info, ok, cw) if soft else (info, ok)

    def sclc_paths(self, N, L, frozen, llr):
        """SclFip internals, fresh path list per frame: int64 metrics, counts, path bits."""
        fr = _frozen(frozen)
        llr = np.ascontiguousarray(llr, dtype=np.int8).reshape(-1, N)
        F = llr.shape[0]
        met = np.zeros((F, L), np.int64)
        pc = np.zeros(F, np.uint32)
        pb = np.zeros((F, L, N // 8), np.uint8)
        r = self.lib.ref_sclc_paths(N, L, _p(fr), len(fr), _p(llr), F, _p(met), _p(pc), _p(pb))
        if r != 0:
            raise ValueError(self.lib.ref_last_error().decode())
        return met, pc, pb

    def bench_char(self, N, L, frozen, llr, threads=1, reps=1, systematic=True, crc=-1):
        fr = _frozen(frozen)
        llr = np.ascontiguousarray(llr, dtype=np.int8).reshape(-1, N)
        return self.lib.ref_bench_char(N, L, _p(fr), len(fr), int(systematic), crc, _p(llr),
                                       llr.shape[0], threads, reps)
