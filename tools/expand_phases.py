"""Phase timing of k_expand_backup from the stamped diagnostic build
(tools/libhz_diag.so, -DHZ_DIAG): self-play positions at 4096 boards (stub
evaluator), one search of `sims` simulations; the stamps of the last
simulation's expansion, per board: start, after the leaf's legal mask, after
the turn-end chance replay, after the children, after the transposition
probes, after the sibling dedup/ids, after the node/edge writes, after the
backup; then the next simulation's select, the row-slot barriers and the
leaf's encode.  The stamps are the last fused launch's (k_expand_backup with
Sel: simulations 1..S-1; the search's final expansion does not stamp).  Prints medians / 95th percentiles / maxima in cycles, by kind of
expansion, and the span of the launch.
Usage (GPU box, repo root): HZ_LIB=tools/libhz_diag.so python tools/expand_phases.py [sims] [moves]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hzamd._native as nat  # noqa: E402
from hzamd.mcts import stub_evaluator  # noqa: E402
from hzamd.selfplay import SelfPlay  # noqa: E402

sims = int(sys.argv[1]) if len(sys.argv) > 1 else 200
moves = int(sys.argv[2]) if len(sys.argv) > 2 else 6
n = 4096
L = nat.lib()
L.hz_mcts_diag_stamps.argtypes = [ctypes.c_void_p]
sp = SelfPlay(n, stub_evaluator, {"num_simulations": sims, "testing": False}, seed_base=123, device="cuda")
sp.env.reset()
for k in range(moves):
    sp.move(k)
torch.cuda.synchronize()
# one more search; keep the stamps of its last simulation
done = sp.env.done()
sp.mcts.search(stub_evaluator, 2.0, active=~done, testing=True)
torch.cuda.synchronize()
st = np.zeros((16384, 16), dtype=np.uint64)
assert L.hz_mcts_diag_stamps(st.ctypes.data) == 0
st = st[:n].astype(np.int64)
flag = st[:, 10]
expanded = (flag & 1) == 1
turn_end = (flag & 2) == 2
nl = flag >> 8
t0 = st[:, 0].min()
res = {"boards": n, "sims": sims, "moves_before": moves, "expanded": int(expanded.sum()),
       "turn_end": int((expanded & turn_end).sum()), "span_cycles": int(st[:, 7].max() - t0),
       "wave_cycles": {}}
names = ["start->legal", "legal->chance", "chance->children", "children->probes", "probes->dedup",
         "dedup->writes", "writes->backup_done"]


def summ(x):
    return {"median": float(np.median(x)), "p95": float(np.quantile(x, 0.95)), "max": float(x.max())}


for kind, sel in (("turn_end", expanded & turn_end), ("other_expand", expanded & ~turn_end),
                  ("no_expand", ~expanded & (st[:, 7] > 0))):
    if not sel.any():
        continue
    s = st[sel]
    d = {"count": int(sel.sum()), "total": summ(s[:, 7] - s[:, 0]), "nl": summ(nl[sel])}
    if kind != "no_expand":
        for i, nm in enumerate(names[:-1]):
            d[nm] = summ(s[:, i + 1] - s[:, i])
        d[names[-1]] = summ(s[:, 7] - s[:, 6])
    if kind == "turn_end":  # inside legal->chance: stream copy-in, draws, write-back
        d["copy_in"] = summ(s[:, 8] - s[:, 1])
        d["draws"] = summ(s[:, 9] - s[:, 8])
        d["write_back"] = summ(s[:, 2] - s[:, 9])
    d["backup->select"] = summ(s[:, 12] - s[:, 7])
    d["select->slot_barriers"] = summ(s[:, 14] - s[:, 12])
    d["slot_barriers->encoded"] = summ(s[:, 13] - s[:, 14])
    d["whole_wave"] = summ(s[:, 13] - s[:, 0])
    res["wave_cycles"][kind] = d
# s_memtime counters are per XCD (not synchronised across them): spans are
# taken within an XCD (the fused launch: 16 boards per workgroup, workgroup
# w on XCD w % 8)
xcd = (np.arange(n) // 16) % 8
res["span_cycles_per_xcd"] = [int(st[xcd == x, 13].max() - st[xcd == x, 0].min()) for x in range(8)]
q = (0, 0.25, 0.5, 0.75, 0.95, 1)
live = st[:, 7] >= st[:, 0]
res["per_xcd"] = []
for x in range(8):
    sx = st[(xcd == x) & live]
    t0x = sx[:, 0].min()
    res["per_xcd"].append({"start": [int(np.quantile(sx[:, 0] - t0x, v)) for v in q],
                           "end": [int(np.quantile(sx[:, 13] - t0x, v)) for v in q]})
starts = np.sort(st[:, 0] - t0)
res["start_quantiles"] = [float(np.quantile(starts, q)) for q in (0, 0.25, 0.5, 0.75, 1)]
print(json.dumps(res, indent=1))
