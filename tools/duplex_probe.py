"""Are host->device and device->host copies on two streams concurrent (PCIe full duplex)?
Times 249 MB up alone, 205 MB down alone, and both at once on two streams, 10 times each,
with per-frame (8.3 / 6.8 MB) copies like hoststream.HostStreamEncoder.
    python tools/duplex_probe.py"""
import json
import time

import torch


def main():
    dev = torch.device("cuda:0")
    f, up_b, dn_b = 30, 3840 * 2160, 6_823_865
    hu = torch.empty((f, up_b), dtype=torch.uint8).pin_memory()
    du = torch.empty((f, up_b), dtype=torch.uint8, device=dev)
    dd = torch.empty((f, dn_b), dtype=torch.uint8, device=dev)
    hd = torch.empty((f, dn_b), dtype=torch.uint8).pin_memory()
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def up():
        with torch.cuda.stream(s1):
            for i in range(f):
                du[i].copy_(hu[i], non_blocking=True)

    def down():
        with torch.cuda.stream(s2):
            for i in range(f):
                hd[i].copy_(dd[i], non_blocking=True)

    out = {}
    for name, fns in (("up", [up]), ("down", [down]), ("both", [up, down])):
        ts = []
        for _ in range(10):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for fn in fns:
                fn()
            torch.cuda.synchronize()
            ts.append(round((time.perf_counter() - t0) * 1e3, 3))
        out[name + "_ms"] = ts
    print(json.dumps(out))


if __name__ == "__main__":
    main()
