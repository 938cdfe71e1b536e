"""The persistent run's waits and counters on the MI355X (so_me.hip run_poll):
a lost done flag is reported with the record of the wait that timed out (which tile, which
flags, that they never arrived), the workspace recovers for the next run, and the
kernel-side SAD operation count (SO_OPT_COUNT_SAD_OPS) is deterministic and leaves the
output unchanged."""
import pytest
import torch

from streamoptima_amd import _lib

pytestmark = pytest.mark.gpu


def _run_setup(dev, h=272, w=640, f=4, seed=5):
    from streamoptima_amd.engine import Engine, alloc_planes
    from streamoptima_amd.synth import synth_sequence_torch
    eng = Engine(h, w, 16, 16, False, 0.015, dev)
    fr = alloc_planes(f, h, w, dev)
    fr.copy_(synth_sequence_torch(f, h, w, seed=seed, device=dev))
    i0 = eng.encode_i(fr[0], 4)
    outs = [eng.new_symbols(1) for _ in range(f - 1)]
    return eng, fr, i0, outs


def test_lost_flag_is_reported_with_its_record(gpu):
    """Task 12 (frame 0, tile 12 of the 5 x 9 tiles of a 640 x 272 frame) never sets its done
    flag: the tiles of frame 1 around it time out after 50 ms of polling, Engine.check_run raises
    naming a frame-1 tile waiting on dep 0 whose flag value for tile 12 is not the epoch and
    never arrived; the run after it (no loss) is clean and equals a fresh encode."""
    from streamoptima_amd.digest import symbols_digest
    eng, fr, i0, outs = _run_setup(gpu)
    curs = [fr[i] for i in range(1, fr.shape[0])]
    eng.encode_p_run(curs, i0.recon, 4, outs)
    eng.check_run()
    exp = [symbols_digest(s) for s in outs]
    with _lib.option(_lib.OPT_TEST_LOSE_FLAG, 13):
        eng.encode_p_run(curs, i0.recon, 4, outs)
        torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match=r"timed out.*frame 1 on dep 0.*never arrived"):
        eng.check_run()
    rec = eng.wait_health.records[-1]
    assert rec["mode"] == "one GPU" and rec["frame"] == 1 and rec["dep"] == 0
    tx, ty = rec["tile"] % 5, rec["tile"] // 5
    assert abs(tx - 12 % 5) <= 1 and abs(ty - 12 // 5) <= 1          # a neighbour of the lost tile
    lane = (12 % 5 - tx + 1) + 3 * (12 // 5 - ty + 1)                    # the lane that polled tile 12
    assert rec["flag_values"][lane] != rec["epoch"]
    assert all(v == rec["epoch"] for k, v in rec["flag_values"].items() if k != lane)
    assert rec["poll_us"] >= 50000 and rec["flags_arrived_after_timeout_us"] is None
    assert rec["grid"] > 0 and 0 <= rec["xcc_id"] < 8
    eng.encode_p_run(curs, i0.recon, 4, outs)            # the same workspace, next epoch: clean
    eng.check_run()
    assert [symbols_digest(s) for s in outs] == exp


def test_sad_op_count_is_deterministic_and_output_neutral(gpu):
    """SO_OPT_COUNT_SAD_OPS: the searches' executed SAD byte operations (words 66..67) are the
    same on every run of the same frames, lie between the bound pass alone (73 x 256 per block)
    and the dense scan of every block, and counting changes no symbol."""
    from streamoptima_amd.digest import symbols_digest
    eng, fr, i0, outs = _run_setup(gpu, h=1088, w=1920, f=4, seed=0)
    curs = [fr[i] for i in range(1, fr.shape[0])]
    eng.encode_p_run(curs, i0.recon, 4, outs)
    eng.check_run()
    assert eng.take_sad_ops() == 0                         # off by default
    exp = [symbols_digest(s) for s in outs]
    counts = []
    for _ in range(2):
        with _lib.option(_lib.OPT_COUNT_SAD_OPS, 1):
            eng.encode_p_run(curs, i0.recon, 4, outs)
            torch.cuda.synchronize()
        eng.check_run()
        counts.append(eng.take_sad_ops())
        assert [symbols_digest(s) for s in outs] == exp
    assert counts[0] == counts[1]
    blocks = eng.nb * len(curs)
    assert 73 * 256 * blocks < counts[0] < 1152 * 256 * blocks


def test_frame_pipeline_two_pass_lost_handoff_reports_and_does_not_fault(gpu):
    """The frame-pipeline two-pass run (kRunFPipe2P) whose reference never arrives: rank 1 of two
    is launched alone, so the I-frame push from rank 0 into its landing slot 0 never happens.
    Its first pass-1 wait times out after 2 s and records itself (frame 0 on dep -1, the landing
    flags never arrived); every later wait then returns at once, so pass-2 units can run before
    their row's pass 1 and read motion records nobody wrote.  Those records are poisoned here
    (dx = dy = 0x7F7F): read unclamped they addressed ~125 MB past the reference plane -- the
    round-5 hipErrorIllegalAddress.  The run must end without a device fault, check() must
    raise with the record, and a one-GPU encode on the same device afterwards must be exact."""
    from streamoptima_amd.digest import symbols_digest
    from streamoptima_amd.engine import Engine
    from streamoptima_amd.pipeline import FramePipeRank
    eng0, fr, i0, outs = _run_setup(gpu, seed=7)
    curs = [fr[i] for i in range(1, fr.shape[0])]
    eng0.encode_p_run(curs, i0.recon, 4, outs)
    eng0.check_run()
    exp = [symbols_digest(s) for s in outs]
    h, w, nf = fr.shape[1], fr.shape[2], fr.shape[0]
    engines = [Engine(h, w, 16, 16, False, 0.015, gpu) for _ in range(2)]
    ranks = [FramePipeRank(engines[r], 2, r, nf, max_wg=96) for r in range(2)]
    torch.cuda.synchronize()
    for r in range(2):
        ranks[r].connect(ranks[(r + 1) % 2].info(), ranks[(r - 1) % 2].info())
    qp_row = [4] * (h // 16)
    syms, _ = ranks[1].prepare(nf, qp_row, True)
    for s in syms.values():
        s.mv.view(torch.uint8).fill_(0x7F)
    torch.cuda.synchronize()
    ranks[1].encode(fr, nf, 4, qp_row=qp_row, two_pass=True, qp_clamp=(0, 12))
    torch.cuda.synchronize()                        # a device fault would raise here
    with pytest.raises(RuntimeError, match=r"frame pipeline, two-pass wait \(pass [12]\).*frame 0 on dep -[12]"):
        ranks[1].check()
    # the first record is the landing wait of pass 1 (flags from rank 0, never set) or, as both
    # start together and time out after the same 2 s, a pass-2 wait on that pass 1
    rec = ranks[1].wait_health.records[-1]
    assert rec["mode"] == "frame pipeline, two-pass" and rec["frame"] == 0 and rec["poll_us"] >= 2e6
    if rec["pass"] == 1:
        assert rec["dep"] == -1 and rec["lanes_remote"] != 0 and rec["flags_arrived_after_timeout_us"] is None
    else:
        assert rec["pass"] == 2 and rec["dep"] == -2
    for r in ranks:
        r.close()
    eng0.encode_p_run(curs, i0.recon, 4, outs)      # the device is healthy: same symbols as before
    eng0.check_run()
    assert [symbols_digest(s) for s in outs] == exp
