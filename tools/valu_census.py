"""Dynamic VALU census of the plain persistent run (p_run_kernel<8, 0, false, false>) by phase:
executed marker counts x the static VALU instructions of each phase.  VERDICT r04 "Next 3".

  GPU:  SO_LIB_PATH=tools/_ab/marks.so python tools/valu_census.py count > gpurun_out/marks.json
        (a -DSO_MARKS_COUNT build: every SO_MARK a wave passes adds 1 to an LDS counter, summed
        into g_mark_counts -- executions per phase over REPS launches of the 4K bench P-run)
  host: python tools/valu_census.py table gpurun_out/marks.json [--pmc-valu N]
        static VALU per phase from tools/isa_census.py (-DSO_MARKS, the product code with
        comment markers), x executions per launch, / blocks per launch; the total beside the
        PMC SQ_INSTS_VALU per launch of the product build (profiles/pmc_me_traffic.json).
A phase's static count is the code between its marker and the next one in layout order, so a
cold path laid out inside a phase (the wait's timeout record, an edge case) is counted as if it
ran on every pass of that marker: the table marks those phases, and the residual against the
PMC total is printed."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = ("loop_top stage_cur stage_cur_int stage_cur_edge cur_sums wait poll_iter stage_win stage_win_int "
         "stage_win_edge dense_tile dense_tile_block byte_sums block_top bound umin umin_edge ballots bal_row dense_fallback survivors "
         "sur_one sur_le4 sur_pass search_end decode_keys tq_residual tq_fwd tq_quant tq_tokens tq_qtc_store tq_inv "
         "tq_recon tq_sse_records post done_flag task_end vbs_block vbs_umin vbs_list_a vbs_pass vbs_list_b vbs_final "
         "vbs_dense vbs_fwd vbs_fwd_sub vbs_final_q vbs_inv vbs_inv_split vbs_inv_end wait_w0 keys_tail p1_tq p1_flag "
         "p2_wait p2_sums p2_tq p2_flag").split()


def count():
    import ctypes
    import torch
    from streamoptima_amd import _lib
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    h, w = (int(v) for v in os.environ.get("SO_AB_SIZE", "2160x3840").split("x"))
    f, reps = 30, int(os.environ.get("REPS", "3"))
    dev = torch.device("cuda:0")
    lib = _lib.load()
    buf = torch.zeros(64, dtype=torch.int32, device=dev)
    eng = Engine(h, w, 16, 16, os.environ.get("SO_AB_VBS") == "1", 0.015, dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=0, device=dev, content=os.environ.get("SO_AB_CONTENT", "bench")))
    i0 = eng.encode_i(fr[0], 4)
    outs = [eng.new_symbols(1) for _ in range(f - 1)]
    two = os.environ.get("SO_AB_2PASS") == "1"
    if two:   # configs[4]'s two-pass run: its workload's row-QP schedule, ROI and clamp (bench.py)
        sys.path.insert(0, ROOT)
        import bench
        from streamoptima_amd.workloads import WORKLOADS
        cfg = dict(WORKLOADS["4k_rc2pass"])
        codec = bench.build_codec(cfg, None, dev)
        eng = codec.engine()
        i0 = eng.encode_i(fr[0], 4)
        qs = codec.row_qp_schedule(eng.nby)
        roi = codec.roi_block_offsets()
        kw = dict(qp_row=qs, qp_row_dev=eng.qp_row_tensor(qs),
                  roi_dev=eng.device_const_i32(roi) if roi is not None else None,
                  qp_lo=codec.qp_clamp[0], qp_hi=codec.qp_clamp[1])
        maps = [torch.empty(eng.nb, dtype=torch.int32, device=dev) for _ in range(f - 1)]
        outs = [eng.new_symbols(1) for _ in range(f - 1)]

    def run():
        if two:
            eng.encode_p_run_2pass([fr[i] for i in range(1, f)], i0.recon, codec.const_init_Qp, outs, maps, **kw)
        else:
            eng.encode_p_run([fr[i] for i in range(1, f)], i0.recon, 4, outs)
    run()   # warm (uncounted)
    torch.cuda.synchronize()
    assert lib.so_debug_set_mark_counts(ctypes.c_void_p(buf.data_ptr())) == 0
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    eng.check_run()
    c = [int(x) & 0xFFFFFFFF for x in buf.cpu().tolist()]
    print(json.dumps({"launches": reps, "frames_per_launch": f - 1, "blocks_per_frame": (h // 16) * (w // 16),
                      "size": f"{w}x{h}", "vbs": eng.vbs, "two_pass": two,
                      "content": os.environ.get("SO_AB_CONTENT", "bench"),
                      "counts": {n: c[i] for i, n in enumerate(NAMES)}}))


def table(path, pmc_valu=None):
    d = json.load(open(path))
    kernel = ("p_run_kernel<8, 3, false, false, false, false>" if d.get("two_pass") else
              "p_run_kernel<8, 0, true, false, true, false>" if d.get('vbs') else
              "p_run_kernel<8, 0, false, false, false, false>")
    cen = json.loads(subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_census.py"), "--json",
                                     "--kernel", kernel], capture_output=True, text=True, check=True).stdout)
    per_launch = {k: v / d["launches"] for k, v in d["counts"].items()}
    blocks = d["frames_per_launch"] * d["blocks_per_frame"]
    rows, tot = [], 0.0
    for n in NAMES:
        c = cen.get(n, {})
        k = max(1, c.get("copies", 1))   # a marker the compiler unrolled / duplicated: per copy
        st = c.get("valu", 0) / k
        ex = per_launch.get(n, 0.0)
        dyn = st * ex
        tot += dyn
        rows.append((n, round(st, 1), ex / blocks, dyn / blocks, c.get("fp64", 0) / k * ex / blocks,
                     c.get("sad", 0) / k * ex / blocks, c.get("lane_rw", 0) / k * ex / blocks))
    pro = cen.get("prologue", {}).get("valu", 0)
    print(f"{'phase':18s}{'static VALU':>12s}{'runs/block':>12s}{'VALU/block':>12s}{'FP64/block':>12s}"
          f"{'SAD/block':>12s}{'lane r/w':>10s}")
    for r in rows:
        if r[2] > 0:
            print(f"{r[0]:18s}{r[1]:12.1f}{r[2]:12.4f}{r[3]:12.1f}{r[4]:12.1f}{r[5]:12.1f}{r[6]:10.2f}")
    print(f"{'TOTAL':18s}{'':12s}{'':12s}{tot / blocks:12.1f}   (+ prologue {pro} static per wave, once per launch)")
    if pmc_valu:
        print(f"PMC SQ_INSTS_VALU per launch {pmc_valu:.4g} = {pmc_valu / blocks:.1f} per block; census / PMC = "
              f"{tot / pmc_valu:.3f}")
    return {"phases": {r[0]: {"static_valu": r[1], "runs_per_block": round(r[2], 5), "valu_per_block": round(r[3], 2)}
                       for r in rows if r[2] > 0}, "total_per_block": round(tot / blocks, 2),
            "pmc_per_block": round(pmc_valu / blocks, 2) if pmc_valu else None}


if __name__ == "__main__":
    if sys.argv[1] == "count":
        count()
    else:
        pv = None
        if "--pmc-valu" in sys.argv:
            pv = float(sys.argv[sys.argv.index("--pmc-valu") + 1])
        out = table(sys.argv[2], pv)
        if "--json" in sys.argv:
            print(json.dumps(out))
