"""chunkformer_amd — MI355X-native ChunkFormer encoder hot path.

The compute path is `libcfm.so` (hand-written gfx950 HIP kernels behind the
C-ABI declared in include/cfm.h); this package is the thin host side that
mirrors the reference's `ChunkFormerEncoder` / `ChunkFormerModel` API.
"""
from .config import EncoderConfig, LARGE, SMALL  # noqa: F401

__all__ = ["EncoderConfig", "LARGE", "SMALL"]
