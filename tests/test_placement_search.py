"""CPU: the pi-state placement search's loop (engine.placement_search) with scripted timings --
when it stops, what it holds, which set it keeps (the device side: tests/test_gpu_placement.py)."""
import pytest

from scdna_replication_tools_amd import engine
from scdna_replication_tools_amd.engine import placement_search

GB = 1 << 30
PATTERN = 6.0e12 * 1e-3          # bytes that stream in 1 ms at 6 TB/s: fast below ~1.034 ms


class Script:
    """Sets are integers 0, 1, 2, ...; ``ms[i]`` is set i's pattern time."""

    def __init__(self, ms, free=1000 * GB):
        self.ms = list(ms)
        self.made = 0
        self.spacers = []
        self.free = free

    def time_set(self, s):
        return self.ms[s]

    def alloc(self, spacer):
        self.made += 1
        sp = ["spacer{}".format(self.made)] if spacer else []
        self.spacers.extend(sp)
        return self.made, sp

    def free_bytes(self):
        return self.free


def run(script, set_bytes=9 * GB, candidates=24):
    return placement_search(0, script.time_set, script.alloc, script.free_bytes, set_bytes, PATTERN, candidates)


def test_top_rate_first_set_stops_at_once():
    sc = Script([0.95, 0.9])                     # 6.3 TB/s: the upper of the two fast rates
    best, times, held = run(sc)
    assert times == [0.95] and best == 0 and sc.made == 0 and held == []


def test_fast_first_set_tries_until_a_top_rate_set():
    sc = Script([1.0, 0.99, 1.01, 0.96, 0.5])
    best, times, held = run(sc)
    # 1.0 ms (6.0 TB/s) is fast, not top; 0.96 ms (6.25 TB/s) is top: the search stops there
    assert times == [1.0, 0.99, 1.01, 0.96] and best == 3
    assert sorted(held) == [0, 1, 2]


def test_slow_sets_until_fast_then_the_extra_budget():
    sc = Script([1.2, 1.2, 1.19, 1.0, 0.99, 1.01, 1.0, 1.0, 1.0, 0.5])
    best, times, held = run(sc, set_bytes=9 * GB)
    # fast first seen at try 4 (1.0 ms: 6.0 TB/s), then PLACEMENT_EXTRA more sets (at most
    # PLACEMENT_EXTRA_BYTES of them)
    n_extra = min(engine.PLACEMENT_EXTRA, engine.PLACEMENT_EXTRA_BYTES // (9 * GB))
    assert times == sc.ms[:4 + n_extra] and best == 4
    assert set(held) == set(range(4 + n_extra)) - {4}


def test_big_sets_stop_at_the_extra_bytes():
    sc = Script([1.0] * 10)
    best, times, held = run(sc, set_bytes=30 * GB)
    assert len(times) == 1 + engine.PLACEMENT_EXTRA_BYTES // (30 * GB) and best == 0


def test_never_fast_stops_at_the_candidate_cap():
    sc = Script([1.2] * 40)
    best, times, held = run(sc, candidates=5)
    assert len(times) == 5 and best == 0 and sc.made == 4


def test_small_sets_walk_with_spacers_and_respect_the_held_cap():
    sc = Script([1.3] * 100)
    set_bytes = 1 * GB
    best, times, held = run(sc, set_bytes=set_bytes)
    step = set_bytes + (engine.PLACEMENT_STRIDE - set_bytes)
    assert sc.made == min(engine.PLACEMENT_CANDIDATES - 1, engine.PLACEMENT_MAX_HELD // step)
    assert len(sc.spacers) == sc.made and all(sp in held for sp in sc.spacers)


def test_low_free_memory_keeps_the_first_set():
    sc = Script([1.3, 0.9], free=20 * GB)
    best, times, held = run(sc, set_bytes=9 * GB)
    assert best == 0 and times == [1.3] and held == []


@pytest.mark.parametrize("ms,want", [([1.2, 1.1, 1.1], 1), ([1.2, 1.25, 1.2], 0)])
def test_ties_keep_the_earlier_set(ms, want):
    sc = Script(ms)
    best, times, held = run(sc, candidates=3)
    assert best == want
