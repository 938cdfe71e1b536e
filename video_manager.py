"""Top-level alias for the reference's `import video_manager as v_manager` (main.py:3)."""
from streamoptima_amd.video_manager import Video_Manager  # noqa: F401
