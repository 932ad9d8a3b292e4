"""hz_play launches only (k_play2 at 4096 boards), for PMC passes:
20 untimed launches to fill the pipeline, then `n` more.
Usage (GPU box): python tools/p2_prog.py [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import torch  # noqa: E402

from hzamd.env import BatchedEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
env = BatchedEnv(4096, device="cuda")
env.set_pipeline(2)
for _ in range(20 + n):
    env.rollout(200, reset=True)
torch.cuda.synchronize()
env.check_errors()
print("ok")
