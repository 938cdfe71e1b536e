"""Host side of the persistent run's wait health (streamoptima_amd/runhealth.py), the
process-wide options (so_set_option) and the device-constant cache -- no GPU needed."""
import collections

import pytest
import torch

from streamoptima_amd import _lib, runhealth


def _record_words(**kw):
    w = [0] * 32
    w[0] = runhealth.DIAG_MAGIC
    vals = dict(task=4711, frame=3, dep=2, tile=17, epoch=9, gop_epoch=0, mode=0 | (1 << 8) | (1 << 12),
                lanes_waited=0b111111111 & ~(1 << 0), lanes_remote=0, poll_ticks=5_000_001, wall_ticks=9_000_000,
                descheduled_ticks=4_000_000, arrival_ticks=0xFFFFFFFF, hw_id=0x1234, xcc_id=5, block=77, grid=768,
                lanes_set_by_atomic_read=0)
    vals.update(kw)
    for i, k in enumerate(runhealth.FIELDS):
        if k in vals:
            w[i] = vals[k] & 0xFFFFFFFF
    for lane in range(12):
        w[20 + lane] = 8 if lane != 4 else 9
    return w


def test_decode_record_fields():
    rec = runhealth.decode_record(_record_words(dep=-1))
    assert rec["task"] == 4711 and rec["frame"] == 3 and rec["dep"] == -1 and rec["tile"] == 17
    assert rec["mode"] == "one GPU" and rec["pass"] == 1 and rec["escalated_to_atomic_reads"]
    assert rec["poll_us"] == 50000.01 and rec["descheduled_us"] == 40000.0
    assert rec["flags_arrived_after_timeout_us"] is None
    assert rec["flag_values"] == {lane: (9 if lane == 4 else 8) for lane in range(1, 9)}
    assert "never arrived" in runhealth.describe(rec)
    rec = runhealth.decode_record(_record_words(arrival_ticks=1234, mode=2 | (2 << 8)))
    assert rec["mode"] == "frame pipeline" and rec["pass"] == 2
    assert "arrived 12.34 us after" in runhealth.describe(rec)
    assert runhealth.decode_record([0] * 32) is None


def test_check_raises_with_the_record_and_clears():
    ws = torch.zeros(256, dtype=torch.int32)
    log = runhealth.HealthLog()
    runhealth.check(ws, log, "p_run_kernel")            # nothing: no raise, nothing logged
    assert log.as_dict()["timeouts"] == 0
    ws[runhealth.GAP_WORD] = 3
    runhealth.check(ws, log, "p_run_kernel")            # a non-fatal count only
    assert (log.stale_reads, log.descheduled_polls) == (0, 3)
    assert int(ws[runhealth.GAP_WORD]) == 0
    ws[runhealth.STALE_WORD] = 2                        # a stale read: counted, cleared, and fatal
    with pytest.raises(RuntimeError, match=r"2 dependency wait\(s\) read a done flag only through an atomic read"):
        runhealth.check(ws, log, "p_run_kernel")
    assert (log.stale_reads, log.descheduled_polls) == (2, 3)
    assert int(ws[runhealth.STALE_WORD]) == 0
    ws[runhealth.TIMEOUT_WORD] = 4
    ws[runhealth.CLAIM_WORD] = 4
    words = _record_words()
    ws[runhealth.DIAG_WORD:runhealth.DIAG_WORD + 32] = torch.tensor([x - (1 << 32) if x >= 1 << 31 else x
                                                                      for x in words], dtype=torch.int32)
    with pytest.raises(RuntimeError, match=r"4 dependency wait\(s\) timed out.*task 4711, frame 3 on dep 2, tile 17"):
        runhealth.check(ws, log, "p_run_kernel")
    assert int(ws[runhealth.TIMEOUT_WORD:runhealth.CLAIM_WORD + 1].abs().sum()) == 0
    assert int(ws[runhealth.DIAG_WORD:].abs().sum()) == 0
    assert log.timeouts == 4 and log.records[0]["tile"] == 17


def test_take_u64():
    ws = torch.zeros(128, dtype=torch.int32)
    v = (5 << 32) | 0x89ABCDEF
    ws[runhealth.SAD_OPS_WORD] = 0x89ABCDEF - (1 << 32)
    ws[runhealth.SAD_OPS_WORD + 1] = 5
    assert runhealth.take_u64(ws, runhealth.SAD_OPS_WORD) == v
    assert runhealth.take_u64(ws, runhealth.SAD_OPS_WORD) == 0


def test_header_words_match_the_host_constants():
    import os
    from conftest import ROOT
    txt = open(os.path.join(ROOT, "include", "streamoptima.h")).read()
    for name, val in (("SO_P_RUN_TIMEOUT_WORD", runhealth.TIMEOUT_WORD), ("SO_P_RUN_STALE_WORD", runhealth.STALE_WORD),
                      ("SO_P_RUN_GAP_WORD", runhealth.GAP_WORD), ("SO_P_RUN_FALLBACK_WORD", runhealth.FALLBACK_WORD),
                      ("SO_P_RUN_SAD_OPS_WORD", runhealth.SAD_OPS_WORD), ("SO_P_RUN_DIAG_WORD", runhealth.DIAG_WORD)):
        assert f"#define {name} {val}\n" in txt, name
    assert f"#define SO_P_RUN_DIAG_MAGIC 0x{runhealth.DIAG_MAGIC:08X}u\n" in txt


def test_set_option_validates_and_round_trips():
    lib = _lib.load()
    assert lib.so_get_option(_lib.OPT_FASTME_SEGMENT) == 32 and lib.so_get_option(_lib.OPT_FASTME_WARMUP) == 32
    assert lib.so_get_option(_lib.OPT_RUN_2PASS_FUSED) == 1 and lib.so_get_option(_lib.OPT_FASTME_SERIAL) == 0
    with _lib.option(_lib.OPT_FASTME_SEGMENT, 8):
        assert lib.so_get_option(_lib.OPT_FASTME_SEGMENT) == 8
    assert lib.so_get_option(_lib.OPT_FASTME_SEGMENT) == 32
    assert lib.so_get_option(_lib.OPT_COUNT_SAD_OPS) == 0
    for opt, bad in ((_lib.OPT_RUN_2PASS_FUSED, 2), (_lib.OPT_FASTME_SEGMENT, 0), (_lib.OPT_FASTME_WARMUP, -1),
                     (_lib.OPT_COUNT_SAD_OPS, 2), (99, 0), (0, 0)):
        assert lib.so_set_option(opt, bad) == _lib.SO_E_INVALID
        assert b"so_set_option" in lib.so_last_error()


class _ConstHost:
    """The Engine fields device_const_i32 uses, on the CPU."""
    MAX_CONSTS = 3

    def __init__(self):
        self.device = torch.device("cpu")
        self._consts = collections.OrderedDict()
        self._pinned_consts = set()
        self._pin_depth = 0


def test_device_consts_are_lru_bounded_not_fatal():
    from streamoptima_amd.engine import Engine
    h = _ConstHost()
    get = lambda v: Engine.device_const_i32(h, v)   # noqa: E731
    a = get([1, 2])
    assert get([1, 2]) is a                         # uploaded once per content
    for k in range(3, 10):
        get([k])                                    # past MAX_CONSTS: evicts, never raises
    assert len(h._consts) == 3
    h._pinned_consts.add(((1,), torch.tensor([9], dtype=torch.int32).numpy().tobytes()))
    for k in range(20, 30):
        get([k])
    assert ((1,), torch.tensor([9], dtype=torch.int32).numpy().tobytes()) in h._consts   # pinned: kept
    Engine.release_consts(h)
    assert not h._consts and not h._pinned_consts
    with Engine.pinned_consts(h):                   # fetched ahead of a capture: pinned explicitly
        get([77])
    for k in range(40, 50):
        get([k])
    assert ((1,), torch.tensor([77], dtype=torch.int32).numpy().tobytes()) in h._consts and h._pin_depth == 0
