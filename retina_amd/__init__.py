"""retina_amd: Retina's packet-stage filter rebuilt for MI355X (gfx950).

The product is the HIP kernel generated per subscription set by the C++ filter compiler and run
through the C ABI in include/retina_pc.h (libretina_pc.so). `pc` is the ctypes binding,
`subscription` the host-side mirror of Retina's Subscription/filter API for this stage.
"""
from . import pc, subscription  # noqa: F401

__all__ = ["pc", "subscription"]
