"""mtrl_amd -- MI355X-native multi-task SAC update engine.

The hot path (replay sample + MTSAC gradient step) runs in ``libmtsac.so``
(hand-written HIP for gfx950, C-ABI in ``include/mtsac.h``); this package is the
host-side mirror of the reference's ``mtrl`` trainer interface on top of it.
"""

from ._lib import MTSACError, MTSACLibraryError  # noqa: F401

__all__ = ["MTSACError", "MTSACLibraryError"]
