"""corda_amd — MI355X-native batch signature verification for Corda's transaction path.

The product is ``libcordagpu.so`` (HIP kernels for gfx950 + the C ABI in include/cordagpu.h).
This package holds the Python host mirror of the reference's Crypto API over that ABI
(``crypto``, ``transactions``, ``merkle``) and the batch layout (``batch``).
"""
__version__ = "0.1.0"
