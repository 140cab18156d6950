"""Drop-in for the reference's `pypolar` module (python/__init__.py +
python/bindings/*.cc of david13pod/antPolarCodes): PolarDecoder, PolarEncoder,
Detector, Puncturer and frozen_bits with the same names, arguments and errors.

    from antpolarcodes_amd import pypolar
    dec = pypolar.PolarDecoder(1024, 8, pypolar.frozen_bits(1024, 512, 0.0), "gpu")
    dec.setErrorDetection(8)
    bits = dec.decode_vector(llr)            # one frame, as in the reference
    info = dec.decode_batch(llrs)            # (F, N) float32 -> (F, K/8) uint8 on the MI355X

Decoder types "gpu" and "float" run the MI355X kernels (list size < 2 -> Fast-SSC,
else CRC-aided SCL).  The native module is mandatory: there is no CPU fallback.
"""
from ._native import _prefer_torch_hip_runtime

_prefer_torch_hip_runtime()  # share PyTorch's HIP runtime (see _native.py)

from ._pypolar import Detector, PolarDecoder, PolarEncoder, Puncturer, frozen_bits  # noqa: E402

__all__ = ["PolarDecoder", "PolarEncoder", "Detector", "Puncturer", "frozen_bits"]
