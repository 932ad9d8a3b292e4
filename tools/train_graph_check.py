"""Per-batch losses of the default network's training phase: eager twice
and with the full batches replayed as a HIP graph, same data and seeds;
shows whether graph-vs-eager differences are within the eager run-to-run
spread.  Usage (GPU box): python tools/train_graph_check.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd.manager import ModelManager  # noqa: E402
from hzamd.net import DEFAULT  # noqa: E402
from hzamd.train import GraphedStep, TensorSource  # noqa: E402

tcfg = {"device": "cuda:0", "optimizer_type": "Adam", "learning_rate": 0.001, "weight_decay": 1e-4,
        "value_loss_weight": 1.0, "policy_loss_weight": 1.0, "batch_size": 64}
g = torch.Generator().manual_seed(3)
M, B = 64 * 12, 64
src = TensorSource((torch.rand(M, 38, 5, 7, generator=g) > 0.8).float().cuda(), torch.rand(M, 42, generator=g).cuda(),
                   torch.softmax(torch.rand(M, 143, generator=g), 1).cuda(),
                   torch.randint(-1, 2, (M,), generator=g).float().cuda())
runs = {}
for name in ("eager1", "eager2", "graph"):
    torch.manual_seed(0)
    mgr = ModelManager(dict(DEFAULT), tcfg)
    step = GraphedStep(mgr) if name == "graph" else None
    losses = []
    for s in range(0, M, B):
        idx = torch.arange(s, s + B, device="cuda")
        b, gl, pi, z = src.batch(idx)
        t, p, v = step.step(b, gl, pi, z) if step else mgr.train_step_async(b, gl, pi, z)
        losses.append([float(t), float(p), float(v)])
    runs[name] = losses
print(json.dumps(runs))
