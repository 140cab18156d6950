"""antpolarcodes_amd -- MI355X-native batched polar SC/SCL decoding.

Drop-in for the float decoding path of david13pod/antPolarCodes: the reference's
`PolarCode::Decoding::Decoder` family (include/polarcode/ in this repo, C++) and
its `pypolar` Python module (antpolarcodes_amd.pypolar), over the C ABI of
include/pcg.h implemented by hand-written HIP kernels for gfx950.
"""
from . import frames  # noqa: F401

__all__ = ["frames"]
