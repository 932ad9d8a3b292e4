"""Cross-move leaf hit rate of config-3 self-play.

For every simulation's gathered leaf batch, each live row's encoded input
(board f32[38,5,7] + glob f32[42], i.e. everything the network sees) is
hashed on the device together with its board id.  A row of move m + 1 is a
"hit" when the same board evaluated the same input during move m's search
(the previous move's tree), and an "any" hit when it did during any earlier
move of the game.  Since each network row is a function of its input row
alone (FoldedNet, test_predict_rows_do_not_depend_on_batch_size), a hit's
network output is already known: the share of hits is what an exact-input
output cache could skip.

usage: python tools/hit_rate.py [boards] [sims] [out.json]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))

import torch  # noqa: E402

from bench import load_selfplay_model  # noqa: E402
from hzamd.mcts import BatchedPredictor  # noqa: E402
from hzamd.selfplay import SelfPlay  # noqa: E402


class HashRows:
    device_rows = True
    capturable = False
    row_independent = True

    def __init__(self, pred, n, dev):
        self.pred = pred
        g = torch.Generator(device="cpu").manual_seed(99)
        self.cb = torch.randint(-2**62, 2**62, (38 * 35,), generator=g, dtype=torch.int64).to(dev) | 1
        self.cg = torch.randint(-2**62, 2**62, (42,), generator=g, dtype=torch.int64).to(dev) | 1
        self.mix = torch.tensor(-7046029254386353131, dtype=torch.int64, device=dev)  # 0x9E37...
        self.keys = []   # this move's [k] int64 keys per simulation
        self.rows = 0

    def __call__(self, board, glob, rows, count):
        out = self.pred(board, glob, rows, count)
        k = int(count.item())
        if k:
            b = board[:k].reshape(k, -1).contiguous().view(torch.int32).to(torch.int64)
            gl = glob[:k].contiguous().view(torch.int32).to(torch.int64)
            h = (b * self.cb).sum(1) + (gl * self.cg).sum(1)
            h = h ^ (rows[:k].to(torch.int64) * self.mix)
            self.keys.append(h)
            self.rows += k
        return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    sims = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    out_path = sys.argv[3] if len(sys.argv) > 3 else None
    dev = torch.device("cuda:0")

    class A:
        checkpoint = None
    net, _ = load_selfplay_model(A(), dev)
    ev = HashRows(BatchedPredictor(net), n, dev)
    cfg = {"num_simulations": sims, "cpuct": 2, "dirichlet_alpha": 0.4, "dirichlet_epsilon": 0.25,
           "turns_until_tau0": 15, "testing": False}
    sp = SelfPlay(n, ev, cfg, seed_base=0, device=dev)
    sp.env.reset()
    prev = None
    seen = torch.empty(0, dtype=torch.int64, device=dev)
    per_ply = []
    tot = {"rows": 0, "hit_prev": 0, "hit_any": 0, "dup_within": 0}
    done = sp.env.done()
    t0 = time.time()
    for ply in range(200):
        nact = int((~done).sum())
        if nact == 0:
            break
        sp._n_active, sp._n_active_epoch = nact, sp.env.epoch
        ev.keys.clear()
        sp.move(ply, done, _bound=nact)
        keys = torch.cat(ev.keys) if ev.keys else torch.empty(0, dtype=torch.int64, device=dev)
        uniq = torch.unique(keys)
        r = keys.numel()
        hp = int(torch.isin(keys, prev).sum()) if prev is not None else 0
        ha = int(torch.isin(keys, seen).sum()) if seen.numel() else 0
        per_ply.append({"ply": ply, "active": nact, "rows": r, "hit_prev": hp, "hit_any": ha,
                        "dup_within": r - uniq.numel()})
        tot["rows"] += r
        tot["hit_prev"] += hp
        tot["hit_any"] += ha
        tot["dup_within"] += r - uniq.numel()
        prev = uniq
        seen = torch.unique(torch.cat([seen, uniq]))
        done = sp.env.done()
        print(f"ply {ply}: active {nact} rows {r} hit_prev {hp / max(1, r):.3f} hit_any {ha / max(1, r):.3f} "
              f"({time.time() - t0:.0f} s)", flush=True)
    sp.check_steps()
    res = {"boards": n, "sims": sims, "plies": len(per_ply), **tot,
           "hit_prev_frac": tot["hit_prev"] / max(1, tot["rows"]),
           "hit_any_frac": tot["hit_any"] / max(1, tot["rows"]), "per_ply": per_ply,
           "basis": "a row hits when the same board's previous move (hit_prev) or any earlier move of the game "
                    "(hit_any) evaluated the same encoded input; keys = 64-bit linear hash of the row's f32 bit "
                    "patterns xor board id"}
    print(json.dumps({k: v for k, v in res.items() if k != "per_ply"}))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
