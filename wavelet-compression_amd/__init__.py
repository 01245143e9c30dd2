"""wavelet-compression_amd — MI355X-native hot path of carsonmw3/wavelet-compression.

The per-box one-level 3-D Haar transform, the keep threshold, the ordered
(run, value) pack, the unpack, the inverse transform and the RMSE run as HIP
kernels for gfx950 behind the C-ABI in include/wavelet_amd.h.  This package is
the Python host side: `capi` binds the C-ABI, `codec` mirrors the reference's
compress()/decompress() interface.  Import it through the root shim `wcamd`
(the directory name is not a Python identifier).
"""
from . import capi  # noqa: F401
from .capi import Context, WaveletError, make_units  # noqa: F401
from .codec import (  # noqa: F401
    CompressedWavelet, calc_adj_loss, calc_rmse_per_box, calc_size, compress, compress_payloads,
    decompress, decompress_payloads, deserialize_compressed_wavelet, inverse_wavelet_decompose,
    serialize_compressed_wavelet, wavelet_decompose,
)

__version__ = "0.1.0"
