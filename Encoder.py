"""Top-level alias for `import Encoder` (the reference's module name, Encoder.py:17)."""
from streamoptima_amd.Encoder import Y_Video_codec  # noqa: F401
