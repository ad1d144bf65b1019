"""Write scdna_replication_tools_amd/data/pi_trajectory.npz: step 1's canonical pi trajectory
(engine.CanonicalPiBlock, computed live: fp32 torch autograd + Adam) for the defaults P = 13,
lr 0.05, betas (0.8, 0.99), eps 1e-8, T steps (default 2,000: max_iter_step1 up to 2,000).

    python tools/make_pi_trajectory.py [--steps 2000]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def live(P=13, lr=0.05, betas=(0.8, 0.99), eps=1e-8, T=2000):
    from scdna_replication_tools_amd import engine
    blk = engine.CanonicalPiBlock(P, lr, betas, eps)
    with engine._PI_LOCK:
        key = (blk.P, float(blk.lr), float(blk.b1), float(blk.b2), float(blk.eps))
        engine._PI_TRAJECTORIES.pop(key, None)
        c = blk._cache_locked(T, shipped=False)
        engine._PI_TRAJECTORIES.pop(key, None)
    return key, c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    key, c = live(T=a.steps)
    st = c["state"]
    from scdna_replication_tools_amd.engine import PI_TRAJECTORY_FILE
    np.savez(PI_TRAJECTORY_FILE, key=np.array([float(k) for k in key]), lp=np.array(c["lp"], dtype=np.float64),
             z=np.stack([s[0] for s in st]), m=np.stack([s[1] for s in st]), v=np.stack([s[2] for s in st]))
    print("wrote", PI_TRAJECTORY_FILE, len(c["lp"]), "steps")


if __name__ == "__main__":
    main()
