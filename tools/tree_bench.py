"""Config-3 moves for kernel profiling: 4096 boards x `sims` simulations with
the default network (x6 kernels), `moves` moves from the game start, then
`moves` more from mid-game positions reached by rule play; prints ms per move.
Run under rocprofv3 --kernel-trace --stats for per-kernel averages
(k_select, k_gather, k_expand_backup, the NN kernels)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]
import torch  # noqa: E402

from hzamd.mcts import BatchedPredictor  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402
from hzamd.selfplay import SelfPlay  # noqa: E402

sims = int(sys.argv[1]) if len(sys.argv) > 1 else 200
moves = int(sys.argv[2]) if len(sys.argv) > 2 else 4
torch.manual_seed(0)
net = HarmoniesNet().cuda().eval()
sp = SelfPlay(4096, BatchedPredictor(net), {"num_simulations": sims}, seed_base=5, device="cuda")
out = {}
for phase, skip in (("start", 0), ("mid", 30)):
    sp.env.reset()
    for p in range(skip):  # rule plies to reach mid-game positions
        mask, count = sp.env.legal_mask()
        sp.env.step(sp.env.rule_actions(mask, count))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(moves):
        sp.move(skip + k)
    torch.cuda.synchronize()
    out[phase] = (time.perf_counter() - t0) / moves * 1e3
print(json.dumps({"sims": sims, "ms_per_move": out}))
