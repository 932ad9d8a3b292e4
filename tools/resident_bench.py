"""FoldedNet.predict (default net) at small batches: the tower as one
resident launch (hz_tower_x6_resident) vs the layered per-conv launches.
Prints one JSON line of microseconds per predict.
Usage (GPU box): python tools/resident_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd.infer import FoldedNet, split_max_batch  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

torch.manual_seed(0)
fnet = FoldedNet(HarmoniesNet().eval().cuda())
out = {}
cap = split_max_batch(torch.device("cuda:0"))  # the split tower's co-residency limit on this device
for batch in [int(b) for b in sys.argv[1:]] or (1, 16, 64, 256, 384, 512, 768, 1024):
    board = (torch.rand(batch, 38, 5, 7, device="cuda") > 0.8).float()
    glob = torch.rand(batch, 42, device="cuda")
    row = {}
    for name, rmax, smax in (("split", 1 << 30, batch), ("resident", 1 << 30, 0), ("layered", 0, 0)):
        if name == "split" and batch > cap:
            continue
        fnet.resident_max, fnet.split_max = rmax, smax
        for _ in range(5):
            fnet.predict(board, glob)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            fnet.predict(board, glob)
        e1.record()
        torch.cuda.synchronize()
        row[name] = round(e0.elapsed_time(e1) * 1e3 / n, 1)
    out[batch] = row
print(json.dumps({"split_max_batch": cap, "us_per_predict": out}))
