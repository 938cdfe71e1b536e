"""Top-level alias for the reference's `import decoder as dec` (main.py:5)."""
from streamoptima_amd.decoder import decoder  # noqa: F401
