"""liberasurecode_amd -- MI355X-native erasure-code backend with the liberasurecode API.

Native pieces (built in-tree into liberasurecode_amd/lib/ by csrc/Makefile):
  libecamd_host.so             GF(2^16) field, generator, decode planning (host C++)
  libecamd.so                  gfx950 HIP kernels + batched device API (include/ecamd.h)
  liberasurecode_rs_vand.so.1  drop-in for the reference's built-in RS codec library
Python modules:
  device   -- device-resident batched encode / decode / reconstruct (ctypes over libecamd)
"""
from . import _lib  # noqa: F401

LIBDIR = _lib.LIBDIR
__all__ = ["LIBDIR"]
