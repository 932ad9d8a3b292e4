"""Where the complete-game leg's network time goes by batch size.
(1) One complete game on 4096 boards (config 3: 200 sims, the default net,
torch.manual_seed(0)), recording the row bound every leaf evaluation is
launched with (the active-board count: the launches are sized by it) and
HIP-event times per call.  (2) The forward alone against the row count, for
the default dispatch (resident tower up to 1,024 rows) and with the
eight-state forms forced (resident_max = split_max = 0).
Usage (GPU box): python tools/rows_dist.py out.json [sims]"""
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

out_path = sys.argv[1]
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = torch.device("cuda:0")
torch.manual_seed(0)
net = HarmoniesNet().to(dev).eval()
pred = BatchedPredictor(net)


class Rec:
    device_rows = True
    capturable = False
    row_independent = True

    def __init__(self):
        self.calls = []

    def __call__(self, board, glob, rows=None, count=None):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = pred(board, glob, rows, count)
        e1.record()
        self.calls.append((board.shape[0], e0, e1, count))
        return r


rec = Rec()
cfg = {"num_simulations": sims, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
       "turns_until_tau0": 15, "testing": False}
sp = SelfPlay(4096, rec, cfg, seed_base=0, device=dev)
t0 = time.time()
live = []
game = sp.play()
torch.cuda.synchronize()
wall = time.time() - t0
calls = [(b, e0.elapsed_time(e1)) for b, e0, e1, _ in rec.calls]
print(json.dumps({"game_s": wall, "plies": game["plies"], "calls": len(calls)}), flush=True)
hist = {}
for b, ms in calls:
    k = min(4096, (b + 255) // 256 * 256)
    h = hist.setdefault(k, [0, 0.0])
    h[0] += 1
    h[1] += ms
active = game["valid"].sum(1).tolist()

# (2) forward alone vs rows
f = pred.fast
g = torch.Generator(device="cuda").manual_seed(0)
NB = 4096
board = (torch.rand(NB, 38, 5, 7, device="cuda", generator=g) > 0.8).float()
board[:, 37] = torch.randint(1, 3, (NB, 1, 1), device="cuda", generator=g).float() / 3.0
glob = torch.rand(NB, 42, device="cuda", generator=g)


def timed(R, reps=10):
    for _ in range(3):
        f.predict(board[:R], glob[:R])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f.predict(board[:R], glob[:R])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


sweep = {}
rows = [32, 64, 128, 256, 384, 512, 640, 768, 896, 1024, 1280, 1536, 1792, 2048, 2056, 2304, 2560, 2816,
        3072, 3584, 4096]
rm, sm = f.resident_max, f.split_max
for R in rows:
    d = {"default": timed(R)}
    f.resident_max, f.split_max = 0, 0  # the eight-state tower at any size
    d["eight_state"] = timed(R)
    f.resident_max, f.split_max = rm, sm
    sweep[R] = d
    print(R, json.dumps(d), flush=True)
json.dump({"sims": sims, "game_s": wall, "plies": game["plies"], "active_per_ply": active,
           "calls_by_rows_256": {k: {"calls": v[0], "ms": v[1]} for k, v in sorted(hist.items())},
           "forward_ms_by_rows": sweep}, open(out_path, "w"), indent=1)
