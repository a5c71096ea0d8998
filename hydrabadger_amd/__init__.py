"""hydrabadger_amd — MI355X (gfx950) batch engine for the hbbft RBC-coding +
ThresholdDecrypt hot path driven by VegeBun-csj/hydrabadger.

The product is libhbgpu.so (C ABI: include/hbgpu.h; HIP kernels in csrc/).
``broadcast`` mirrors hbbft's ``Coding`` / ``MerkleTree`` / ``Proof`` /
``send_shards`` / ``decode_from_shards`` over that ABI.  There is no CPU
fallback: compute calls raise when the HIP library or a device is missing.
Importing the package does not touch the GPU.
"""
from . import _lib, broadcast, threshold  # noqa: F401

__all__ = ["_lib", "broadcast", "threshold"]
