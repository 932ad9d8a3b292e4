"""A/B of the residual tower as one launch (hz_tower_x6_blocks, every
workgroup through all 8 blocks) against one launch per block
(hz_resblock_x6_bias_act), in ONE process (interleaved rounds): the whole
leaf-eval forward (FoldedNet.predict) at `batch` rows, alternating blocks of
20 forwards for `rounds` rounds; outputs compared bit for bit, also at a
live-row count below the batch.
Usage (GPU box): python tools/tower_ab.py [rounds] [batch]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd.infer import FoldedNet  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
torch.manual_seed(0)
fnet = FoldedNet(HarmoniesNet().eval().cuda())
g = torch.Generator(device="cuda").manual_seed(0)
board = (torch.rand(B, 38, 5, 7, device="cuda", generator=g) > 0.8).float()
board[:, 37] = torch.randint(1, 3, (B, 1, 1), device="cuda", generator=g).float() / 3.0
glob = torch.rand(B, 42, device="cuda", generator=g)
live = torch.tensor([B - 77], dtype=torch.int32, device="cuda")
outs, outs_live, ts = {}, {}, {0: [], 1: []}
for t in (0, 1):
    fnet.tower_loop = t
    outs[t] = fnet.predict(board, glob)
    outs_live[t] = fnet.predict(board, glob, live)
for _ in range(40):
    fnet.predict(board, glob)
for r in range(rounds):
    for t in ((0, 1) if r % 2 == 0 else (1, 0)):
        fnet.tower_loop = t
        fnet.predict(board, glob)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fnet.predict(board, glob)
        e1.record()
        torch.cuda.synchronize()
        ts[t].append(e0.elapsed_time(e1) / 20)
same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
n = B - 77
same_live = all(torch.equal(a[:n], b[:n]) for a, b in zip(outs_live[0], outs_live[1]))
med = {t: sorted(v)[len(v) // 2] for t, v in ts.items()}
print(json.dumps({"batch": B, "bit_identical": same, "bit_identical_live_rows": same_live,
                  "ms_median": {"per_block": med[0], "tower": med[1]},
                  "ms_min": {"per_block": min(ts[0]), "tower": min(ts[1])},
                  "ms_all": {t: [round(x, 4) for x in v] for t, v in ts.items()}}))
