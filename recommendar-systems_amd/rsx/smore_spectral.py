"""Fused image/text projection + spectral denoise/fusion (reference smore.py:209-252,256-259)
through the HIP kernel rsx_smore_spectral, with autograd."""
from __future__ import annotations

from . import _lib as L


def spectral_available() -> bool:
    return hasattr(L.lib(), "rsx_smore_spectral_fwd")


def spectral_fused(model):
    raise NotImplementedError
