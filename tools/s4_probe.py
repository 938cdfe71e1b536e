"""Why BASELINE.md section 4's region depends on what ran before it: host topology and the
PCIe copy rate of a pinned buffer by the NUMA node it was allocated from.

    python tools/s4_probe.py

Prints the CPUs this process may run on, the NUMA nodes and their CPUs, the GPU's PCI
address and NUMA node, then for each node that holds allowed CPUs: the H2D / D2H rate of a
249 MB pinned buffer allocated and first touched by a thread pinned to that node (best and
median of 6 copies).  A diagnostic; nothing here is product code.
"""
import glob
import os
import time

import torch


def cpulist(s):
    out = set()
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def main():
    allowed = os.sched_getaffinity(0)
    print("allowed cpus", len(allowed), sorted(allowed)[:8], "...")
    nodes = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        nodes[int(d.rsplit("node", 1)[1])] = cpulist(open(os.path.join(d, "cpulist")).read())
    for n, c in nodes.items():
        print(f"node {n}: {len(c)} cpus, {len(c & allowed)} allowed")
    p = torch.cuda.get_device_properties(0)
    bus = getattr(p, "pci_bus_id", None)
    dom = getattr(p, "pci_domain_id", 0)
    dev = getattr(p, "pci_device_id", 0)
    gnode = None
    if bus is not None:
        addr = f"{dom:04x}:{bus:02x}:{dev:02x}.0"
        f = f"/sys/bus/pci/devices/{addr}/numa_node"
        gnode = int(open(f).read()) if os.path.exists(f) else None
        print("gpu pci", addr, "numa_node", gnode)
    nbytes = 248832000
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    for n, c in nodes.items():
        cs = c & allowed
        if not cs:
            continue
        os.sched_setaffinity(0, cs)
        host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        host.fill_(1)
        rates = {}
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
            rates[name] = (round(nbytes / ts[0] / 1e9, 2), round(nbytes / ts[len(ts) // 2] / 1e9, 2))
        print(f"pinned buffer from node {n} (gpu node {gnode}): h2d best/median GB/s {rates['h2d']}, "
              f"d2h {rates['d2h']}", flush=True)
        del host
    os.sched_setaffinity(0, allowed)


if __name__ == "__main__":
    main()
