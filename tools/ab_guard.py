"""Refuse to run an A/B measurement whose environment knobs the loaded library ignores.

The SO_FUSED / SO_ME_IMPL / SO_SEA_PROBE / SO_RUN_PER_CU / SO_P2LAG / SO_FASTME_* knobs are read
only by libraries built with -DSO_AB (`python -m streamoptima_amd.build --out tools/_ab/x.so -D
SO_AB`); the product library ignores them, so a tool setting one against it would silently time
the default path.  Such builds export so_debug_ab_build()."""
import ctypes
import os

KNOBS = ("SO_FUSED", "SO_ME_IMPL", "SO_SEA_PROBE", "SO_RUN_PER_CU", "SO_P2LAG", "SO_FASTME_SERIAL",
         "SO_FASTME_SEG", "SO_FASTME_WARM", "SO_FASTME_ROUNDS")


def require_ab_build(env=None, lib_path=None):
    env = os.environ if env is None else env
    used = [k for k in KNOBS if env.get(k) not in (None, "")]
    if not used:
        return
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = lib_path or env.get("SO_LIB_PATH") or os.path.join(root, "streamoptima_amd", "libstreamoptima_hip.so")
    if not hasattr(ctypes.CDLL(p), "so_debug_ab_build"):
        raise SystemExit(f"{', '.join(used)} set, but {p} was not built with -DSO_AB and ignores them: build a variant "
                         "with `python -m streamoptima_amd.build --out tools/_ab/x.so -D SO_AB` and pass it by SO_LIB_PATH")
