"""What the bench's per-call HIP event pairs cost a self-play move: the
config-3 per-move leg (4096 boards x 200 sims, default network) timed with
bench.py's TimedEvaluator (an event pair around every leaf evaluation) and
with the bare predictor, alternating, same positions (the env restored from
an exported state before every timed move)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from hzamd.mcts import BatchedPredictor  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402
from hzamd.selfplay import SelfPlay  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
net = HarmoniesNet().to(dev).eval()
pred = BatchedPredictor(net)
timed = bench.TimedEvaluator(pred, dev)
cfg = {"num_simulations": 200, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
       "turns_until_tau0": 15, "testing": False}
sp = SelfPlay(4096, timed, cfg, seed_base=0, device=dev)
timed.attach(sp.mcts)
sp.env.reset()
for w in range(2):
    sp.move(w)
torch.cuda.synchronize()
st, mt, idx = sp.env.export_state(with_mt=True)
res = {"timed": [], "bare": []}
for rep in range(3):
    for mode in ("timed", "bare"):
        sp.evaluator = timed if mode == "timed" else pred
        sp.env.import_state(st, mt, idx)
        sp.step_counter = 2
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sp.move(2)
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) * 1e3)
sp.check_steps()
print(json.dumps({k: sorted(v) for k, v in res.items()}))
