"""Shared test data: frozen sets, LLR generators, node-type coverage sets."""
import numpy as np


def llr_kinds(rng, F, N, kind):
    """LLR families that stress the reference's quirks (ties, +-0, saturation)."""
    if kind == "normal":
        return rng.normal(1.0, 1.5, (F, N)).astype(np.float32)
    if kind == "ints":  # many exact ties and zeros
        return rng.integers(-3, 4, (F, N)).astype(np.float32)
    if kind == "zeros":  # +0 / -0 heavy
        x = rng.normal(0.0, 2.0, (F, N)).astype(np.float32)
        x[rng.random((F, N)) < 0.2] = -0.0
        x[rng.random((F, N)) < 0.2] = 0.0
        return x
    if kind == "sparse":  # {-1, 0, +1}
        return (np.sign(rng.normal(0, 1, (F, N))) * rng.integers(0, 2, (F, N))).astype(np.float32)
    if kind == "wide":  # large dynamic range
        return (rng.normal(0, 1, (F, N)) * 10.0 ** rng.uniform(-3, 4, (F, N))).astype(np.float32)
    raise ValueError(kind)


LLR_KINDS = ("normal", "ints", "zeros", "sparse", "wide")


def node_cover_sets():
    """(N, frozen) pairs whose Fast-SSC trees contain every leaf kind at several sizes (the
    product's validation catalogue, antpolarcodes_amd/rtc_codes.py)."""
    from antpolarcodes_amd.rtc_codes import node_cover_sets as f
    return f()


def sha256(a):
    """Digest of an output array as tests/golden/make_digests.py computes it."""
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def reference_digest(name):
    """The reference's output digests for a full-size GPU test batch
    (tests/golden/reference_digests.json, made by tests/golden/make_digests.py)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_digests.json")) as fh:
        return json.load(fh)["cases"][name]


KERNELS = ("interp", "rtc")


def gpu_plan(N, L, frozen, kernel="interp", device=0, **kw):
    """A device plan on the interpreter kernel ("interp": tests/conftest.py keeps plans from
    specialising themselves) or on its plan-specialised kernel ("rtc": pcg_plan_specialize,
    loaded from the library's shipped cache: the catalogue antpolarcodes_amd/rtc_codes.py).
    Asserts which kernel the decodes will launch."""
    from antpolarcodes_amd._native import Plan
    p = Plan(N, L, frozen, device=device, **kw)
    if kernel == "rtc":
        p.specialize()
        assert p.describe()["specialized"] == 1
        want = "scq_rtc_kernel" if L == 1 else "scl_rtc_kernel"  # (adaptive: its list stage's)
        assert p.kernel_name() == want, p.kernel_name()
    else:
        assert p.describe()["specialized"] == 0 and "rtc" not in p.kernel_name(), p.kernel_name()
    return p
