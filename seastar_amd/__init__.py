"""seastar_amd — MI355X-native batch Internet checksum for a Seastar-style
native network stack.

The product is libsccsum.so (HIP kernels for gfx950 + the C-ABI in
include/sccsum.h + the kept per-packet C++ API).  This Python package is host
plumbing for tests and bench: device memory and streams come from torch,
every checksum is computed by the native library (no CPU fallback).
"""
from . import native  # noqa: F401

__all__ = ["native"]
