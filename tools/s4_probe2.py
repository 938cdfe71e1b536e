"""PCIe copy rate of a pinned host buffer against how its pages are backed (diagnostic).

    python tools/s4_probe2.py

A: torch pinned buffer allocated at process start; B: the same after the process has
allocated, touched and freed 6 GB of host memory in small pieces (as bench.py's records
leave the heap); C: an mmap'd buffer advised MADV_HUGEPAGE, touched, then registered with
hipHostRegister.  For each: H2D / D2H best and median GB/s over 6 copies and the buffer's
AnonHugePages from /proc/self/smaps.
"""
import ctypes
import mmap
import os
import time

import numpy as np
import torch

NB = 248832000


def huge_kb(addr, size):
    """AnonHugePages (kB) summed over the smaps entries overlapping [addr, addr + size)."""
    tot, cur = 0, False
    for line in open("/proc/self/smaps"):
        parts = line.split()
        if "-" in parts[0] and len(parts) >= 5 and all(c in "0123456789abcdef-" for c in parts[0]):
            a, b = (int(x, 16) for x in parts[0].split("-"))
            cur = a < addr + size and b > addr
        elif cur and parts[0] == "AnonHugePages:":
            tot += int(parts[1])
    return tot


def rates(host, dst):
    out = {}
    for name, fn in (("h2d", lambda: dst.copy_(host, non_blocking=True)),
                     ("d2h", lambda: host.copy_(dst, non_blocking=True))):
        ts = []
        for _ in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts = sorted(ts[1:])
        out[name] = (round(NB / ts[0] / 1e9, 2), round(NB / ts[len(ts) // 2] / 1e9, 2))
    return out


def report(tag, host, dst):
    r = rates(host, dst)
    print(f"{tag}: h2d {r['h2d']} d2h {r['d2h']} GB/s (best, median); huge pages "
          f"{huge_kb(host.data_ptr(), NB) // 1024} MB of {NB >> 20} MB", flush=True)


def main():
    torch.cuda.init()
    dst = torch.empty(NB, dtype=torch.uint8, device="cuda")
    a = torch.empty(NB, dtype=torch.uint8, pin_memory=True)
    a.fill_(1)
    report("A pinned at start", a, dst)
    keep = []
    for i in range(6000):            # 6 GB in 1 MB pieces, every other one kept
        x = np.ones(1 << 20, np.uint8)
        if i % 2:
            keep.append(x)
    b = torch.empty(NB, dtype=torch.uint8, pin_memory=True)
    b.fill_(1)
    report("B pinned after 6 GB of small allocations", b, dst)
    del keep
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    m = mmap.mmap(-1, NB + (2 << 20))
    m.madvise(mmap.MADV_HUGEPAGE)
    base = ctypes.addressof(ctypes.c_char.from_buffer(m))
    off = (-base) % (2 << 20)
    arr = np.frombuffer(m, dtype=np.uint8, count=NB, offset=off)
    arr[:] = 1
    rc = hip.hipHostRegister(ctypes.c_void_p(base + off), ctypes.c_size_t(NB), ctypes.c_uint(0))
    c = torch.from_numpy(arr)
    print("hipHostRegister rc", rc, "is_pinned", c.is_pinned())
    report("C mmap + MADV_HUGEPAGE + hipHostRegister", c, dst)
    print("THP setting:", open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip(),
          "| defrag:", open("/sys/kernel/mm/transparent_hugepage/defrag").read().strip())


if __name__ == "__main__":
    main()
