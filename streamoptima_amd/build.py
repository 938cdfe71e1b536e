"""Build libstreamoptima_hip.so (gfx950) in-tree with hipcc.

The library links against the HIP runtime that PyTorch ships (torch/lib/libamdhip64.so,
soname libamdhip64.so.7) so a process that imported torch first uses ONE HIP runtime.
Device code is compiled with -ffp-contract=off: the FP64 DCT must keep pocketfft's
separate multiply/add roundings to stay bit-exact with the reference (so_dct.h).
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB_NAME = "libstreamoptima_hip.so"
LIB_PATH = os.path.join(PKG, LIB_NAME)
ARCH = os.environ.get("SO_OFFLOAD_ARCH", "gfx950")


def _torch_lib_dir() -> str:
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        raise RuntimeError("PyTorch (ROCm) is required to build against its HIP runtime")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.h")) + [
        os.path.join(os.path.dirname(PKG), "include", "streamoptima.h"), __file__]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines: tuple = ()) -> str:
    """Build the library in-tree.  `out` + `defines` make an A/B or instrumented variant
    (tools/: e.g. -DSO_STAMPS) at another path; the product library is always LIB_PATH."""
    target = out or LIB_PATH
    if out is None and not defines and not force and not _stale():
        return LIB_PATH
    tlib = _torch_lib_dir()
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
             *[f"-D{d}" for d in defines],
             "-I", os.path.join(os.path.dirname(PKG), "include")]
    # one object per translation unit, compiled side by side (each .hip is self-contained:
    # device code is shared only through headers), then one link
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    srcs = sources()
    with tempfile.TemporaryDirectory(prefix="so_build_") as tmp:
        objs = [os.path.join(tmp, os.path.basename(s) + ".o") for s in srcs]
        cmds = [[_hipcc(), *flags, "-c", s, "-o", o] for s, o in zip(srcs, objs)]
        cmds.append([_hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", target + ".tmp", *objs,
                     f"-L{tlib}", "-lamdhip64", f"-Wl,-rpath,{tlib}"])
        jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))

        def run(cmd):
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            return subprocess.run(cmd, capture_output=True, text=True)

        with ThreadPoolExecutor(jobs) as ex:
            results = list(ex.map(run, cmds[:-1]))
        results.append(run(cmds[-1]) if all(r.returncode == 0 for r in results) else None)
        for cmd, r in zip(cmds, results):
            if r is not None and r.returncode != 0:
                raise RuntimeError(f"hipcc failed ({r.returncode}) on {cmd[-3] if '-c' in cmd else 'link'}:\n"
                                   f"{r.stderr[-6000:]}")
            if verbose and r is not None and r.stderr:
                print(r.stderr[-4000:], file=sys.stderr)
    os.replace(target + ".tmp", target)
    return target


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--out", default=None, help="variant library path (A/B, instrumented)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra preprocessor define")
    a = ap.parse_args()
    print(build(force=a.force, verbose=True, out=a.out, defines=tuple(a.defines)))
