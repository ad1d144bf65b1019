"""GPU: the pi-state placement search (PertShard.choose_pi_placement).

The search moves z / m / v into the fastest of several allocations before the fit starts; it
must change nothing but the addresses: the state after the move equals the state before it, the
library is handed the new pointers, and a fit from a searched shard is bit-identical to the same
fit from the first allocation.  The size threshold is lowered so a test-sized shard is searched
(the rate test then never stops the search early: a small launch is far from the fast rate).
"""
import numpy as np
import pytest
import torch

from tests._problems import KIND_OF, init_constrained, make_problem

pytestmark = pytest.mark.gpu


def _shard(kind, kw, z, placement):
    from scdna_replication_tools_amd.engine import PertShard
    sh = PertShard(KIND_OF[kind], init=init_constrained(kind, z), device="cuda", placement=0, **kw)
    sh.set_unconstrained({k: v.numpy() for k, v in z.items()})
    before = sh.z_pi.clone(), sh.m_pi.clone(), sh.v_pi.clone()
    if placement > 1:
        sh.choose_pi_placement(placement)
    return sh, before


@pytest.mark.parametrize("kind,fused", [("step2", False), ("step2", True), ("step3", True)])
def test_placement_search_changes_nothing_but_addresses(kind, fused):
    prob, kw, z = make_problem(kind, seed=6)
    kw = dict(kw, fused=fused)
    ref, _ = _shard(kind, kw, z, 0)
    sh, before = _shard(kind, kw, z, 3)
    rec = sh.placement
    assert rec is not None and 1 <= len(rec["candidates_ms"]) <= 3
    assert 0 <= rec["chosen"] < len(rec["candidates_ms"])
    assert min(rec["candidates_ms"]) == rec["candidates_ms"][rec["chosen"]]
    # the library is handed the arrays the shard now holds, with the state moved unchanged
    st = sh._state
    assert (st.z_pi, st.m_pi, st.v_pi) == (sh.z_pi.data_ptr(), sh.m_pi.data_ptr(), sh.v_pi.data_ptr())
    for now, was in zip((sh.z_pi, sh.m_pi, sh.v_pi), before):
        assert torch.equal(now, was)
    # the same fit from either placement: identical losses and parameters, bit for bit
    la, _ = ref.run_svi(60, 10 ** 9, 0.0)
    lb, _ = sh.run_svi(60, 10 ** 9, 0.0)
    assert np.array_equal(np.asarray(la), np.asarray(lb))
    assert torch.equal(ref.params, sh.params)
    assert torch.equal(ref.z_pi, sh.z_pi)
    assert torch.equal(ref.v_pi, sh.v_pi)


def test_placement_default_applies_to_large_shards_only():
    from scdna_replication_tools_amd import engine
    prob, kw, z = make_problem("step2", seed=6)
    from scdna_replication_tools_amd.engine import PertShard
    sh = PertShard(KIND_OF["step2"], init=init_constrained("step2", z), device="cuda", **kw)
    assert sh.z_pi.numel() < engine.PLACEMENT_MIN_FLOATS and sh.placement is None


def test_placement_search_out_of_memory_keeps_the_first_set(monkeypatch):
    """An allocation failure inside the search (another allocation on the device took the room)
    leaves the shard on its first set, with the state and the library's pointers unchanged,
    instead of failing the fit."""
    from scdna_replication_tools_amd import engine
    prob, kw, z = make_problem("step2", seed=6)
    ref, _ = _shard("step2", kw, z, 0)
    sh, before = _shard("step2", kw, z, 0)
    ptrs = (sh.z_pi.data_ptr(), sh.m_pi.data_ptr(), sh.v_pi.data_ptr())

    def failing(first, time_set, alloc, free_bytes, set_bytes, pattern_bytes, candidates):
        time_set(first)
        cand, _ = alloc(0)
        time_set(cand)                     # the library now points at the try
        raise torch.cuda.OutOfMemoryError("simulated")
    monkeypatch.setattr(engine, "placement_search", failing)
    rec = sh.choose_pi_placement(3)
    assert rec["candidates_ms"] is None and "OutOfMemoryError" in rec["error"]
    st = sh._state
    assert (st.z_pi, st.m_pi, st.v_pi) == ptrs == (sh.z_pi.data_ptr(), sh.m_pi.data_ptr(), sh.v_pi.data_ptr())
    for now, was in zip((sh.z_pi, sh.m_pi, sh.v_pi), before):
        assert torch.equal(now, was)
    la, _ = ref.run_svi(30, 10 ** 9, 0.0)
    lb, _ = sh.run_svi(30, 10 ** 9, 0.0)
    assert np.array_equal(np.asarray(la), np.asarray(lb))
