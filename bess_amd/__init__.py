"""bess_amd: MI355X-native implementation of BESS's packet-classification
hot path (ExactMatch, WildcardMatch, IPChecksum, L4Checksum).

The compute lives in libbessgpu.so (hand-written gfx950 HIP kernels behind the
C ABI in include/bessgpu.h). Importing a submodule that needs the library
raises if it has not been built -- there is no CPU fallback.
"""
import os

__version__ = "0.1.0"
ROOT = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(ROOT, "libbessgpu.so")


def lib():
    from . import _lib
    return _lib.lib()
