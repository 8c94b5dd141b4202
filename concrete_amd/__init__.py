"""concrete_amd — MI355X-native (gfx950) backend for the Concrete batched programmable bootstrap.

The product is libconcrete_hip.so (C ABI: include/concrete_hip.h).  This package only loads
it and provides host-side plumbing (concrete_amd.backend) for tests and benchmarks.
"""
from . import _native  # noqa: F401
from .backend import CFG2, CFG4, PbsParams  # noqa: F401

__all__ = ["CFG2", "CFG4", "PbsParams"]
