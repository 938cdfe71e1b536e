"""Top-level alias for the reference's `import Y_video_codec as codec` (main.py:4)."""
from streamoptima_amd.Encoder import Y_Video_codec  # noqa: F401
