"""StreamOptima on MI355X: the per-block encode path of the StreamOptima block video
encoder (Encoder.py / decoder.py call surface) as hand-written gfx950 HIP kernels behind a
C-ABI library, driven from PyTorch-ROCm device buffers.

    from streamoptima_amd.Encoder import Y_Video_codec
    from streamoptima_amd.decoder import decoder
"""
__version__ = "0.1.0"

from .build import LIB_PATH  # noqa: F401
