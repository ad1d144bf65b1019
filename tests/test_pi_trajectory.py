"""CPU: step 1's canonical pi trajectory shipped with the package
(scdna_replication_tools_amd/data/pi_trajectory.npz, tools/make_pi_trajectory.py) equals the
live computation (engine.CanonicalPiBlock: fp32 torch autograd + Adam) bit for bit, every step's
log pi~ and (z, m, v); and a block reads it for the defaults only."""
import numpy as np

from scdna_replication_tools_amd import engine


def test_shipped_trajectory_equals_live_computation():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "make_pi_trajectory", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "make_pi_trajectory.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    key, live = mk.live(T=2000)
    shipped = engine._shipped_trajectory(key)
    assert shipped is not None
    assert len(shipped["lp"]) == len(live["lp"]) == 2000
    np.testing.assert_array_equal(np.array(shipped["lp"]), np.array(live["lp"]))
    for a, b in zip(shipped["state"], live["state"]):
        for x, y in zip(a, b):
            assert x.dtype == y.dtype == np.float32
            np.testing.assert_array_equal(x, y)


def test_shipped_trajectory_only_for_its_key():
    assert engine._shipped_trajectory((13, 0.05, 0.8, 0.99, 1e-8)) is not None
    assert engine._shipped_trajectory((12, 0.05, 0.8, 0.99, 1e-8)) is None
    assert engine._shipped_trajectory((13, 0.01, 0.8, 0.99, 1e-8)) is None


def test_block_extends_past_the_shipped_steps():
    blk = engine.CanonicalPiBlock(13, 0.05)
    lp = blk.trajectory(1, 2100)                      # 100 steps past the table, computed on
    assert lp.shape == (2100,) and np.isfinite(lp).all()
