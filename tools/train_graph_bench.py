"""Config-5 training phase timing: the reference's default buffer (50,000
examples), batch 64, default network and Adam (config.py:37-48), one epoch,
eager steps vs full batches replayed as a captured HIP graph
(hzamd.train.GraphedStep).  Prints one JSON line.
Usage (GPU box): python tools/train_graph_bench.py [examples]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd.manager import ModelManager  # noqa: E402
from hzamd.net import DEFAULT  # noqa: E402
from hzamd.train import TensorSource, training_phase  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
tcfg = {"device": "cuda:0", "optimizer_type": "Adam", "learning_rate": 0.001, "weight_decay": 1e-4,
        "value_loss_weight": 1.0, "policy_loss_weight": 1.0, "batch_size": 64, "use_scheduler": True,
        "scheduler_type": "StepLR", "scheduler_step_size": 30, "scheduler_gamma": 0.5}
g = torch.Generator(device="cuda").manual_seed(0)
src = TensorSource((torch.rand(M, 38, 5, 7, device="cuda", generator=g) > 0.8).float(),
                   torch.rand(M, 42, device="cuda", generator=g),
                   torch.softmax(torch.rand(M, 143, device="cuda", generator=g), 1),
                   torch.randint(-1, 2, (M,), device="cuda", generator=g).float())
out = {"examples": M, "batch": 64}
CL = os.environ.get("HZ_TRAIN_CL") == "1"  # channels_last model and inputs (MIOpen NHWC kernels)
if CL:
    src = TensorSource(src.t[0].contiguous(memory_format=torch.channels_last), *src.t[1:])
out["channels_last"] = CL
for graph in (False, True, False, True):
    torch.manual_seed(0)
    mgr = ModelManager(dict(DEFAULT), tcfg)
    if CL:
        mgr.model.to(memory_format=torch.channels_last)
    training_phase(mgr, TensorSource(*(t[:640] for t in src.t)), 1, 64, graph=graph)  # warm the kernels
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = training_phase(mgr, src, 1, 64, generator=torch.Generator(device="cuda").manual_seed(1), graph=graph)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out["graph" if graph else "eager"] = {"s": dt, "ms_per_batch": dt * 1e3 / res["batches"], "loss": res["loss"]}
print(json.dumps(out))
