"""The persistent run's wait health words and timeout record (include/streamoptima.h,
SO_P_RUN_TIMEOUT_WORD .. SO_P_RUN_DIAG_WORD; DESIGN.md section 4, "Waits").

Every consumer of a run workspace (Engine, the stripe and frame-pipeline ranks) reads the
words 32..127 in ONE device-to-host copy, raises with the decoded record of the first wait
that timed out, raises as well when a wait found its flag only through an atomic read (a
stale read: the consumer protocol failed, even though that wait completed), and keeps the
non-fatal count of descheduled poll intervals for the bench line.
"""
from __future__ import annotations

import torch

TIMEOUT_WORD = 32
STALE_WORD = 33
GAP_WORD = 34
CLAIM_WORD = 35
FALLBACK_WORD = 64
SAD_OPS_WORD = 66       # uint64 (words 66, 67)
DIAG_WORD = 96
DIAG_MAGIC = 0x534F0001
TICK_US = 0.01          # s_memrealtime: 100 MHz

MODES = {0: "one GPU", 1: "stripe", 2: "frame pipeline", 3: "two-pass", 4: "frame pipeline, two-pass"}
FIELDS = ("magic", "task", "frame", "dep", "tile", "epoch", "gop_epoch", "mode", "lanes_waited",
          "lanes_remote", "poll_ticks", "wall_ticks", "descheduled_ticks", "_13", "arrival_ticks", "hw_id",
          "xcc_id", "block", "grid", "lanes_set_by_atomic_read")


def decode_record(words) -> dict | None:
    """The 32-word record at DIAG_WORD (list of ints), or None if no wait timed out."""
    w = [int(x) & 0xFFFFFFFF for x in words]
    if w[0] != DIAG_MAGIC:
        return None
    rec = {k: w[i] for i, k in enumerate(FIELDS) if not k.startswith("_") and k != "magic"}
    for k in ("dep",):
        if rec[k] >= 1 << 31:
            rec[k] -= 1 << 32
    m = rec.pop("mode")
    rec["mode"] = MODES.get(m & 15, str(m & 15))
    rec["vbs"] = bool(m & 16)
    rec["pass"] = (m >> 8) & 15
    rec["escalated_to_atomic_reads"] = bool(m & (1 << 12))
    waited = rec["lanes_waited"]
    rec["flag_values"] = {lane: w[20 + lane] for lane in range(12) if waited >> lane & 1}
    for k in ("poll_ticks", "wall_ticks", "descheduled_ticks"):
        rec[k.replace("_ticks", "_us")] = round(rec.pop(k) * TICK_US, 2)
    a = rec.pop("arrival_ticks")
    rec["flags_arrived_after_timeout_us"] = None if a == 0xFFFFFFFF else round(a * TICK_US, 2)
    return rec


def describe(rec: dict) -> str:
    """One line naming the wait: what it waited for, for how long, and what the flags held."""
    if rec is None:
        return "no record"
    arrived = rec["flags_arrived_after_timeout_us"]
    fate = (f"the flags arrived {arrived} us after the timeout (a slow holder)" if arrived is not None
            else "the flags never arrived within 50 ms more (lost or never set)")
    return (f"{rec['mode']} wait (pass {rec['pass']}): task {rec['task']}, frame {rec['frame']} on dep {rec['dep']}, "
            f"tile {rec['tile']}, epoch {rec['epoch']} (GOP epoch {rec['gop_epoch']}); polled "
            f"{rec['poll_us']} us of {rec['wall_us']} us wall ({rec['descheduled_us']} us descheduled); flag values "
            f"{rec['flag_values']}; XCC {rec['xcc_id']}, HW_ID {rec['hw_id']:#x}, workgroup {rec['block']} of "
            f"{rec['grid']}; {fate}")


def read(ws: torch.Tensor) -> dict:
    """Words 32..127 of a run workspace in one copy (synchronises)."""
    w = ws[TIMEOUT_WORD:DIAG_WORD + 32].cpu().tolist()
    at = lambda k: w[k - TIMEOUT_WORD] & 0xFFFFFFFF   # noqa: E731
    return {"timeouts": at(TIMEOUT_WORD), "stale_reads": at(STALE_WORD), "descheduled_polls": at(GAP_WORD),
            "record": decode_record(w[DIAG_WORD - TIMEOUT_WORD:])}


def clear(ws: torch.Tensor) -> None:
    """Zero the timeout, health and claim words and the record (on the current stream)."""
    ws[TIMEOUT_WORD:CLAIM_WORD + 1].zero_()
    ws[DIAG_WORD:DIAG_WORD + 32].zero_()


class HealthLog:
    """Accumulates the non-fatal counts of a workspace over checks (reported by bench.py)."""

    def __init__(self):
        self.stale_reads = 0
        self.descheduled_polls = 0
        self.timeouts = 0
        self.records: list = []

    def as_dict(self) -> dict:
        return {"timeouts": self.timeouts, "stale_reads_repaired": self.stale_reads,
                "descheduled_polls": self.descheduled_polls, "records": self.records[:4]}


def check(ws: torch.Tensor | None, log: HealthLog | None, what: str) -> None:
    """Read and clear the words; raise RuntimeError naming the first timed-out wait."""
    if ws is None:
        return
    h = read(ws)
    if not (h["timeouts"] or h["stale_reads"] or h["descheduled_polls"] or h["record"]):
        return
    clear(ws)
    if log is not None:
        log.stale_reads += h["stale_reads"]
        log.descheduled_polls += h["descheduled_polls"]
        log.timeouts += h["timeouts"]
        if h["record"]:
            log.records.append(h["record"])
    if h["timeouts"]:
        raise RuntimeError(f"{what}: {h['timeouts']} dependency wait(s) timed out; the symbols are unreliable. "
                           f"First: {describe(h['record'])}")
    if h["stale_reads"]:
        # the consumer protocol (relaxed polls + one agent acquire) kept missing a flag that was
        # set: the wait completed through atomic reads, but the hand-off rule the run's
        # correctness argument rests on did not hold, so the run is not trusted either
        raise RuntimeError(f"{what}: {h['stale_reads']} dependency wait(s) read a done flag only through an atomic "
                           "read after 1 ms of relaxed polls (a stale cached copy): the hand-off protocol failed, "
                           "the run is not trusted")


def timed_out(ws: torch.Tensor | None) -> bool:
    return ws is not None and int(ws[TIMEOUT_WORD].item()) != 0


def take_u64(ws: torch.Tensor, word: int) -> int:
    """A uint64 counter at words (word, word + 1), then cleared."""
    lo, hi = (int(x) & 0xFFFFFFFF for x in ws[word:word + 2].cpu().tolist())
    ws[word:word + 2].zero_()
    return lo | hi << 32
