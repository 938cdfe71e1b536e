"""Host-side cost of one bench step (Y_Video_codec.encode_device of the 4K GOP with reused
symbol buffers): enqueue time per step without synchronising vs the step's wall time, and a
cProfile of the Python side.  Run on the GPU box: python tools/hostprof_probe.py"""
import cProfile, pstats, sys, time, torch
sys.path.insert(0, ".")
from bench import build_codec, make_frames, parse
from streamoptima_amd.workloads import WORKLOADS
dev = torch.device("cuda:0")
cfg = dict(WORKLOADS["4k"])
codec = build_codec(cfg, parse([]), dev)
eng = codec.engine()
fr = make_frames(cfg, dev, 0)
pre = [eng.new_symbols(0 if i % 30 == 0 else 1) for i in range(30)]
for _ in range(3):
    codec.encode_device(fr, 30, symbols=pre, check=False)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    codec.encode_device(fr, 30, symbols=pre, check=False)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("host enqueue per step ms", (t1 - t0) / 20 * 1e3, "total per step ms", (t2 - t0) / 20 * 1e3)
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    codec.encode_device(fr, 30, symbols=pre, check=False)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(14)
