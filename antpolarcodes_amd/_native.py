"""ctypes binding of libpcg.so, the C ABI declared in include/pcg.h.

The HIP extension is mandatory: importing this module raises if libpcg.so is
missing, and decoding raises if no GPU is present.  There is no CPU fallback.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PCG_DEV_LIB") or os.path.join(_HERE, "lib", "libpcg.so")  # PCG_DEV_LIB: dev builds

PCG_OK = 0
PCG_E_ARG = -1
PCG_E_FROZEN = -2
PCG_E_HIP = -3
PCG_E_UNSUPPORTED = -4
PCG_E_NODEVICE = -5

CRC_KINDS = (0, 8, 11, 16, 32)


class PcgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"pcg error {code}: {msg}")
        self.code = code


class PlanDesc(C.Structure):
    _fields_ = [
        ("block_length", C.c_uint32),
        ("info_length", C.c_uint32),
        ("list_size", C.c_uint32),
        ("node_count", C.c_uint32),
        ("op_count", C.c_uint32),
        ("lds_bytes", C.c_uint32),
        ("scratch_bytes", C.c_uint64),
        ("crc_kind", C.c_int32),
        ("systematic", C.c_int32),
        ("lanes_per_codeword", C.c_uint32),
        ("dev_overrides", C.c_uint32),  # PCG_DEV_* bits: non-default kernel/layout from dev env switches
        ("recomputed_stages", C.c_uint32),  # lane-serial SCL: top stages recomputed (1 or 2)
        ("specialized", C.c_uint32),  # 1: decodes run the plan-specialised kernel (pcg_plan_specialize)
    ]


_lib = None


def _prefer_torch_hip_runtime():
    """Load PyTorch's bundled HIP runtime first when torch is installed.

    torch ships its own libamdhip64/libhsa-runtime64 (SONAME libamdhip64.so.7) and
    its libraries bind them as "libamdhip64.so".  If libpcg.so were loaded first,
    /opt/rocm's runtime would be mapped and torch would then map a second HSA
    runtime, after which torch sees no GPU.  Loading torch first makes
    libpcg.so's DT_NEEDED libamdhip64.so.7 resolve to the runtime torch already
    holds, so device pointers and streams are shared.
    """
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    global _lib
    if _lib is None:
        _prefer_torch_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build the HIP extension first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.pcg_plan_create.argtypes = [C.POINTER(P), C.c_uint32, C.c_uint32, P, C.c_uint32, C.c_int, C.c_int, C.c_int]
        L.pcg_plan_create_adaptive.argtypes = L.pcg_plan_create.argtypes
        L.pcg_plan_create_char.argtypes = L.pcg_plan_create.argtypes
        L.pcg_plan_create_adaptive_char.argtypes = L.pcg_plan_create.argtypes
        L.pcg_decode_i8.argtypes = [P, P, C.c_uint64, P, P, P, P]
        L.pcg_decode_i8_host.argtypes = [P, P, C.c_uint64, P, P, P]
        L.pcg_decode_f32.argtypes = [P, P, C.c_uint64, P, P, P, P]
        L.pcg_decode_f32_host.argtypes = [P, P, C.c_uint64, P, P, P]
        L.pcg_decode_f32_soft.argtypes = [P, P, C.c_uint64, P, P, P, P]
        L.pcg_decode_f32_soft_host.argtypes = [P, P, C.c_uint64, P, P, P]
        L.pcg_plan_describe.argtypes = [P, C.POINTER(PlanDesc)]
        L.pcg_plan_kernel_name.argtypes = [P]
        L.pcg_plan_kernel_name.restype = C.c_char_p
        L.pcg_plan_set_initial_metric.argtypes = [P, C.c_float]
        L.pcg_plan_specialize.argtypes = [P]
        L.pcg_plan_specialize_async.argtypes = [P]
        L.pcg_plan_destroy.argtypes = [P]
        L.pcg_plan_destroy.restype = None
        L.pcg_last_error.restype = C.c_char_p
        L.pcg_device_count.restype = C.c_int
        L.pcg_puncturer_create.argtypes = [C.POINTER(P), C.c_uint32, P, C.c_uint32, C.c_int]
        L.pcg_puncturer_describe.argtypes = [P, P, P, P]
        L.pcg_depuncture_f32.argtypes = [P, P, C.c_uint64, P, P]
        L.pcg_puncture_f32.argtypes = [P, P, C.c_uint64, P, P]
        L.pcg_puncture_packed.argtypes = [P, P, C.c_uint64, P, P]
        L.pcg_puncturer_destroy.argtypes = [P]
        L.pcg_puncturer_destroy.restype = None
        L.pcg_decode_punctured_f32.argtypes = [P, P, P, C.c_uint64, P, P, P, P]
        L.pcg_encoder_create.argtypes = [C.POINTER(P), C.c_uint32, P, C.c_uint32, C.c_int, C.c_int, C.c_int]
        L.pcg_encode.argtypes = [P, P, C.c_uint64, P, P]
        L.pcg_encoder_destroy.argtypes = [P]
        L.pcg_encoder_destroy.restype = None
        L.pcg_random_info.argtypes = [P, C.c_uint64, C.c_uint32, C.c_uint64, P]
        L.pcg_bpsk_awgn_f32.argtypes = [P, C.c_uint64, C.c_uint32, C.c_float, C.c_uint64, P, P]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise PcgError(rc, lib().pcg_last_error().decode(errors="replace"))


def device_count():
    return lib().pcg_device_count()


def _ptr(t):
    if t is None:
        return None
    return t if isinstance(t, int) else t.data_ptr()


def _check_tensor(name, t, dtype, shape, device):
    """Device-buffer arguments of the decode calls: a torch tensor must have the plan's
    dtype, exact shape, be contiguous and live on the plan's device (a mismatch would let
    the kernel read or write out of bounds); raw integer pointers are taken as given."""
    if t is None or isinstance(t, int):
        return
    import torch
    if t.dtype != dtype:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {tuple(shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    if t.device.type != "cuda" or (t.device.index if t.device.index is not None else torch.cuda.current_device()) \
            != device:
        raise ValueError(f"{name}: on {t.device}, the plan lives on cuda:{device}")


def _stream(stream, t):
    if stream is not None:
        return stream
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream


def _frozen_array(frozen):
    fr = np.ascontiguousarray(np.asarray(list(frozen), dtype=np.uint32))
    return fr, (fr.ctypes.data if fr.size else None)


class Plan:
    """Owns one pcg_plan (decoder tree + device schedule for one device)."""

    def __init__(self, N, L, frozen, systematic=True, crc=8, device=0, adaptive=False, fixed=False):
        """adaptive=True: Fast-SSC first, SCL-L for the frames whose check fails
        (AdaptiveFloat, pcg_plan_create_adaptive).  fixed=True: the reference's 8-bit
        decoders FastSscFipChar / SclFipChar (pcg_plan_create_char); both: AdaptiveChar."""
        fr = np.ascontiguousarray(np.asarray(list(frozen), dtype=np.uint32))
        h = C.c_void_p()
        if adaptive:  # AdaptiveFloat / AdaptiveChar
            create = lib().pcg_plan_create_adaptive_char if fixed else lib().pcg_plan_create_adaptive
        else:
            create = lib().pcg_plan_create_char if fixed else lib().pcg_plan_create
        _check(create(C.byref(h), int(N), int(L), fr.ctypes.data if fr.size else None,
                      int(fr.size), int(bool(systematic)), int(crc), int(device)))
        self._h = h
        self.N, self.L, self.K = int(N), int(L), int(N) - int(fr.size)
        self.kb = (self.K + 7) // 8
        self.device = device
        self.fixed = bool(fixed)

    def kernel_name(self):
        """The decode kernel as rocprofv3 names it (pcg_plan_kernel_name)."""
        return lib().pcg_plan_kernel_name(self._h).decode()

    def specialize(self, wait=True):
        """Compile (or take from a cache) and load the kernel specialised to this plan's code
        (pcg_plan_specialize, hiprtc; float Fast-SSC and list plans).  wait=False starts it in
        the background (pcg_plan_specialize_async).  Raises PcgError if that fails or is
        unsupported."""
        _check(lib().pcg_plan_specialize(self._h) if wait else lib().pcg_plan_specialize_async(self._h))

    def set_initial_metric(self, m):
        """SCL: initial path-0 metric of later decodes (reference metric carry)."""
        _check(lib().pcg_plan_set_initial_metric(self._h, float(m)))

    def _check_io(self, llr, info, ok, metrics, dtype):
        import torch
        F = llr.shape[0] if hasattr(llr, "shape") else None
        if F is None:
            raise ValueError("llr must be a tensor (its first dimension is the frame count)")
        _check_tensor("llr", llr, dtype, (F, self.N), self.device)
        _check_tensor("info", info, torch.uint8, (F, self.kb), self.device)
        _check_tensor("ok", ok, torch.uint8, (F,), self.device)
        _check_tensor("metrics", metrics, torch.float32, (F, self.L), self.device)
        return F

    def describe(self):
        d = PlanDesc()
        _check(lib().pcg_plan_describe(self._h, C.byref(d)))
        return {k: getattr(d, k) for k, _ in PlanDesc._fields_}

    def decode_host(self, llr, want_ok=True, want_metrics=False):
        llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, self.N)
        F = llr.shape[0]
        info = np.zeros((F, self.kb), np.uint8)
        ok = np.zeros(F, np.uint8) if want_ok else None
        met = np.zeros((F, self.L), np.float32) if want_metrics else None
        _check(lib().pcg_decode_f32_host(self._h, llr.ctypes.data, F, info.ctypes.data,
                                         None if ok is None else ok.ctypes.data,
                                         None if met is None else met.ctypes.data))
        return info, ok, met

    def decode_host_i8(self, llr, want_ok=True, want_metrics=False):
        """int8 frames (8-bit plans): pcg_decode_i8_host."""
        llr = np.ascontiguousarray(llr, dtype=np.int8).reshape(-1, self.N)
        F = llr.shape[0]
        info = np.zeros((F, self.kb), np.uint8)
        ok = np.zeros(F, np.uint8) if want_ok else None
        met = np.zeros((F, self.L), np.float32) if want_metrics else None
        _check(lib().pcg_decode_i8_host(self._h, llr.ctypes.data, F, info.ctypes.data,
                                        None if ok is None else ok.ctypes.data,
                                        None if met is None else met.ctypes.data))
        return info, ok, met

    def decode_soft_device(self, llr, info, ok, soft, stream=None):
        """Fast-SSC float plans: decode and write the F x N soft codewords
        (pcg_decode_f32_soft, Decoder::getSoftCodeword)."""
        import torch
        F = self._check_io(llr, info, ok, None, torch.float32)
        _check_tensor("soft", soft, torch.float32, (F, self.N), self.device)
        _check(lib().pcg_decode_f32_soft(self._h, _ptr(llr), F, _ptr(info), _ptr(ok), _ptr(soft),
                                         _stream(stream, llr)))

    def decode_soft_host(self, llr):
        """Host arrays: returns (info, ok, soft codewords) (pcg_decode_f32_soft_host)."""
        llr = np.ascontiguousarray(llr, dtype=np.float32).reshape(-1, self.N)
        F = llr.shape[0]
        info = np.zeros((F, self.kb), np.uint8)
        ok = np.zeros(F, np.uint8)
        soft = np.zeros((F, self.N), np.float32)
        _check(lib().pcg_decode_f32_soft_host(self._h, llr.ctypes.data, F, info.ctypes.data, ok.ctypes.data,
                                              soft.ctypes.data))
        return info, ok, soft

    def decode_device_i8(self, llr, info, ok=None, metrics=None, stream=None):
        """int8 device frames (torch.int8 CUDA tensors F x N): pcg_decode_i8."""
        import torch
        F = self._check_io(llr, info, ok, metrics, torch.int8)
        _check(lib().pcg_decode_i8(self._h, _ptr(llr), F, _ptr(info), _ptr(ok), _ptr(metrics),
                                   _stream(stream, llr)))

    def decode_device(self, llr, info, ok=None, metrics=None, stream=None):
        """Device-resident decode of torch CUDA tensors: llr float32 F x N, info uint8
        F x ceil(K/8), ok uint8 F (or None), metrics float32 F x L (or None)."""
        import torch
        F = self._check_io(llr, info, ok, metrics, torch.float32)
        _check(lib().pcg_decode_f32(self._h, _ptr(llr), F, _ptr(info), _ptr(ok), _ptr(metrics),
                                    _stream(stream, llr)))

    def decode_punctured_device(self, punc, llr, info, ok=None, metrics=None, stream=None):
        """Depuncture (F x E, device) with `punc` and decode, one stream-ordered call."""
        import torch
        F = llr.shape[0]
        _check_tensor("llr", llr, torch.float32, (F, punc.E), self.device)
        _check_tensor("info", info, torch.uint8, (F, self.kb), self.device)
        _check_tensor("ok", ok, torch.uint8, (F,), self.device)
        _check_tensor("metrics", metrics, torch.float32, (F, self.L), self.device)
        _check(lib().pcg_decode_punctured_f32(self._h, punc._h, _ptr(llr), llr.shape[0], _ptr(info), _ptr(ok),
                                              _ptr(metrics), _stream(stream, llr)))

    def close(self):
        if getattr(self, "_h", None):
            lib().pcg_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Puncturer:
    """pcg_puncturer: Puncturer(E, frozen) (puncturer.cpp:51-66) with device tables."""

    def __init__(self, E, frozen, device=0):
        fr, fp = _frozen_array(frozen)
        h = C.c_void_p()
        _check(lib().pcg_puncturer_create(C.byref(h), int(E), fp, int(fr.size), int(device)))
        self._h = h
        e, n = C.c_uint32(), C.c_uint32()
        _check(lib().pcg_puncturer_describe(h, C.byref(e), C.byref(n), None))
        self.E, self.N, self.device = e.value, n.value, device

    def positions(self):
        out = np.zeros(self.E, np.uint32)
        _check(lib().pcg_puncturer_describe(self._h, None, None, out.ctypes.data))
        return out

    def depuncture_device(self, x, out, stream=None):
        _check(lib().pcg_depuncture_f32(self._h, _ptr(x), x.shape[0], _ptr(out), _stream(stream, x)))

    def puncture_device(self, x, out, stream=None):
        _check(lib().pcg_puncture_f32(self._h, _ptr(x), x.shape[0], _ptr(out), _stream(stream, x)))

    def puncture_packed_device(self, x, out, stream=None):
        _check(lib().pcg_puncture_packed(self._h, _ptr(x), x.shape[0], _ptr(out), _stream(stream, x)))

    def close(self):
        if getattr(self, "_h", None):
            lib().pcg_puncturer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Encoder:
    """pcg_encoder: ButterflyFipPacked + Detector::generate on the device."""

    def __init__(self, N, frozen, systematic=True, crc=0, device=0):
        fr, fp = _frozen_array(frozen)
        h = C.c_void_p()
        _check(lib().pcg_encoder_create(C.byref(h), int(N), fp, int(fr.size), int(bool(systematic)), int(crc),
                                        int(device)))
        self._h = h
        self.N, self.K = int(N), int(N) - int(fr.size)
        self.kb = (self.K + 7) // 8
        self.device = device

    def encode_device(self, info, code, stream=None):
        """info (F x kb uint8, check bits written in place) -> code (F x N/8 uint8)."""
        _check(lib().pcg_encode(self._h, _ptr(info), info.shape[0], _ptr(code), _stream(stream, info)))

    def close(self):
        if getattr(self, "_h", None):
            lib().pcg_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def random_info_device(info, K, seed, stream=None):
    _check(lib().pcg_random_info(_ptr(info), info.shape[0], int(K), int(seed) & (2**64 - 1), _stream(stream, info)))


def bpsk_awgn_device(code, n, sigma, seed, llr, stream=None):
    _check(lib().pcg_bpsk_awgn_f32(_ptr(code), code.shape[0], int(n), float(sigma), int(seed) & (2**64 - 1),
                                   _ptr(llr), _stream(stream, code)))
