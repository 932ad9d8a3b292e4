"""Time ModelManager.train_step (batch 64, default 128x8 net) variants."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import torch
from hzamd.manager import ModelManager
from hzamd.net import DEFAULT
dev = "cuda:0"
res = {}
for name, bench, cl in [("nchw_bench", True, False), ("nchw_nobench", False, False), ("nhwc_bench", True, True)]:
    torch.backends.cudnn.benchmark = bench
    torch.manual_seed(0)
    mm = ModelManager(DEFAULT, {"device": dev, "optimizer_type": "Adam", "learning_rate": 1e-3, "weight_decay": 1e-4,
                                "value_loss_weight": 1.0, "policy_loss_weight": 1.0, "batch_size": 64})
    if cl:
        mm.model = mm.model.to(memory_format=torch.channels_last)
    B = 64
    b = (torch.rand(B, 38, 5, 7, device=dev) > 0.8).float()
    if cl:
        b = b.to(memory_format=torch.channels_last)
    g = torch.rand(B, 42, device=dev)
    pi = torch.softmax(torch.rand(B, 143, device=dev), 1)
    z = torch.rand(B, 1, device=dev) * 2 - 1
    for _ in range(10):
        mm.train_step_async(b, g, pi, z)
    torch.cuda.synchronize()
    t = time.perf_counter()
    R = 50
    for _ in range(R):
        mm.train_step_async(b, g, pi, z)
    torch.cuda.synchronize()
    res[name] = (time.perf_counter() - t) / R * 1e3
print(json.dumps(res))
