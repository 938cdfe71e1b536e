"""Module alias so the reference's `import Y_video_codec as codec` (main.py:4) resolves."""
from .Encoder import Y_Video_codec  # noqa: F401
