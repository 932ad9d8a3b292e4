"""Config-5 evaluation arena in isolation (diagnostic): n games x `sims`
simulations, MctsAgent vs MctsAgent on one env, (a) stub evaluators, then
(b) two random-init default networks through BatchedPredictor (the x6
kernels on small gathered batches).  Prints one line per stage."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]
import torch  # noqa: E402

from hzamd.arena import MctsAgent, play_games, summarize  # noqa: E402
from hzamd.mcts import BatchedPredictor, stub_evaluator  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
sims = int(sys.argv[2]) if len(sys.argv) > 2 else 200
stage = sys.argv[3] if len(sys.argv) > 3 else "ab"
if "a" in stage:
    t = time.time()
    out, _, plies = play_games(MctsAgent(stub_evaluator, {"num_simulations": sims}),
                               MctsAgent(stub_evaluator, {"num_simulations": sims}), n, seed_base=10**9)
    torch.cuda.synchronize()
    print("stub", summarize(out), plies, f"{time.time() - t:.1f}s", flush=True)
if "b" in stage:
    torch.manual_seed(1)
    a = HarmoniesNet().cuda().eval()
    b = HarmoniesNet().cuda().eval()
    for graph in (False, True):  # eager simulations, then each search's simulations replayed as a HIP graph
        t = time.time()
        out, _, plies = play_games(MctsAgent(BatchedPredictor(a), {"num_simulations": sims}, graph=graph),
                                   MctsAgent(BatchedPredictor(b), {"num_simulations": sims}, graph=graph), n,
                                   seed_base=10**9)
        torch.cuda.synchronize()
        print("nets", "graph" if graph else "eager", summarize(out), plies, f"{time.time() - t:.1f}s", flush=True)
