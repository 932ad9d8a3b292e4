"""Debug aid: MCTS (stub evaluator) vs greedy, ply by ply against the C
oracle; prints the first ply where the GPU's search result differs (visits,
tree sizes) for each board.  Usage: python tools/dbg_arena.py [graph 0/1] [n]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "harmonies-alphazero_amd"))
import oracle  # noqa: E402
from hzamd.env import BatchedEnv  # noqa: E402
from hzamd.mcts import BatchedMCTS, stub_evaluator  # noqa: E402
from hzamd.state import unpack_ref  # noqa: E402

SIMS = 8
graph = len(sys.argv) > 1 and sys.argv[1] == "1"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
base = 400
dev = "cuda:0"
env = BatchedEnv(n, seed_base=base, device=dev)
env.reset()
ms = [oracle.mt_seed(base + g) for g in range(n)]
ss = [oracle.reset(m) for m in ms]
mcts = BatchedMCTS(env, SIMS)
bad = set()
for ply in range(200):
    done = env.done().cpu().numpy()
    if done.all():
        break
    st = env.export_state()
    fin = st.cpu().numpy()
    for g in range(n):
        if g in bad or oracle.is_game_over(ss[g]):
            continue
        if not (unpack_ref(fin[:, g]) == ss[g]).all():
            print(f"ply {ply} board {g}: state diverged")
            bad.add(g)
    to_move = ((st[5] >> 41) & 1).cpu().numpy()
    a_is_p0 = (np.arange(n) % 2) == 0
    a_turn = ((to_move == 0) == a_is_p0) & ~done
    act = np.full(n, -1, np.int64)
    if a_turn.any():
        mask = torch.from_numpy(a_turn).to(dev)
        v = mcts.search(stub_evaluator, 2.0, active=mask, noise=None, eps=0.0, testing=True, graph=graph)
        v = v.cpu().numpy()
        stats = mcts.stats().cpu().numpy()
        for g in np.nonzero(a_turn)[0]:
            act[g] = int(np.argmax(v[g]))
            if g in bad:
                continue
            a, ov, nn, ne = oracle.mcts_search(ss[g], ms[g], SIMS, 2.0, eps=0.0, testing=True, tau0=0, ply=ply)
            if not (ov == v[g]).all() or stats[g, 0] != nn or stats[g, 1] != ne:
                print(f"ply {ply} board {g}: visits gpu {dict((i, int(x)) for i, x in enumerate(v[g]) if x)} "
                      f"oracle {dict((i, int(x)) for i, x in enumerate(ov) if x)} nodes {stats[g, :2]} vs {nn},{ne} "
                      f"overflow {stats[g, 3]}")
                bad.add(g)
            ss[g] = oracle.step(ss[g], a, ms[g])[1]
    b_turn = ~a_turn & ~done
    if b_turn.any():
        ga = env.greedy_actions(sel=torch.from_numpy(b_turn).to(dev)).cpu().numpy()
        for g in np.nonzero(b_turn)[0]:
            act[g] = ga[g]
            if g not in bad:
                ss[g] = oracle.step(ss[g], oracle.greedy_move(ss[g], ms[g]), ms[g])[1]
    status = env.step(torch.from_numpy(np.where(done, -1, act)).to(dev).to(torch.int16)).cpu().numpy()
    for g in np.nonzero(~done & (status != 0))[0]:
        print(f"ply {ply} board {g}: step status {status[g]} action {act[g]}")
        bad.add(g)
print("graph", graph, "boards diverged:", sorted(bad))
