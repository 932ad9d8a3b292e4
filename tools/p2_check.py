"""Pipeline-2 parity under back-to-back hz_play calls (no host sync between
them): K calls, each call's final states copied on the stream, then every
episode checked against the C oracle.  Usage: p2_check.py [max_plies] [K] [n]"""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import oracle  # noqa: E402
from hzamd.env import BatchedEnv  # noqa: E402
from hzamd.state import unpack_ref  # noqa: E402

mp = int(sys.argv[1]) if len(sys.argv) > 1 else 96
K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
n = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
base = 12345
env = BatchedEnv(n, seed_base=base, device="cuda")
env.set_pipeline(2)
snaps, steps = [], []
g = torch.zeros(n, dtype=torch.int32, device="cuda")
for k in range(K):
    s = torch.zeros(n, dtype=torch.int32, device="cuda")
    env.rollout(mp, games_done=g, steps_done=s, reset=True)
    snaps.append(env.export_state().clone())
    steps.append(s)
torch.cuda.synchronize()
bad = {}
for ep in range(K):
    _, finals, plies, _ = oracle.play_rule_games(n, base, nthreads=8, episode=ep)  # (rule games end by ply 72)
    got = snaps[ep].cpu().numpy()
    wrong = [b for b in range(n) if not (unpack_ref(got[:, b]) == finals[b]).all()]
    st_wrong = int((steps[ep].cpu().numpy() != plies).sum())
    if wrong or st_wrong:
        bad[ep] = (len(wrong), wrong[:5], st_wrong)
print("max_plies", mp, "calls", K, "bad episodes:", bad if bad else "none")
