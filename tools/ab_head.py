"""Same-box A/B of the leaf-eval head inside config-3 self-play: moves of one
4096-board x 200-sim game alternate between the fused head (hz_heads_fc) and
hz_heads + PyTorch linear layers + softmax, so both see the same positions'
cost trend and the same clock/power state.  Prints one JSON line.
Usage (GPU box): python tools/ab_head.py [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd.infer import FoldedNet  # noqa: E402
from hzamd.mcts import BatchedPredictor  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402
from hzamd.selfplay import SelfPlay  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dev = "cuda:0"
torch.manual_seed(0)
net = HarmoniesNet().to(dev).eval()
pred = BatchedPredictor(net)
variants = {"fused": FoldedNet(net), "split": FoldedNet(net, fused_head=False)}
cfg = {"num_simulations": 200, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
       "turns_until_tau0": 15, "testing": False}
sp = SelfPlay(4096, pred, cfg, seed_base=0, device=dev)
sp.env.reset()
ply = 0
for _ in range(2):
    sp.move(ply)
    ply += 1
ms = {k: [] for k in variants}
for r in range(rounds):
    for name in (("fused", "split") if r % 2 == 0 else ("split", "fused")):
        pred.fast = variants[name]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sp.move(ply)
        torch.cuda.synchronize()
        ms[name].append((time.perf_counter() - t0) * 1e3)
        ply += 1
out = {k: {"ms_per_move": v, "mean": sum(v) / len(v)} for k, v in ms.items()}
out["saving_ms_per_move"] = out["split"]["mean"] - out["fused"]["mean"]
print(json.dumps(out))
