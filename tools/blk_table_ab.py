"""A/B of the fused residual block's row table in ONE process (interleaved
rounds, cdna_hip_programming.md rule 24): the whole leaf-eval forward
(FoldedNet.predict at 4096 rows) with hz_resblock_x6_set_table(0) (round 3's
placement) and (1) (the LDS-bank-conflict-free one), alternating blocks of
20 forwards for `rounds` rounds; outputs compared bit for bit.
Usage (GPU box): python tools/blk_table_ab.py [rounds]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

import hzamd._native as nat  # noqa: E402
from hzamd.infer import FoldedNet  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
B = 4096
torch.manual_seed(0)
fnet = FoldedNet(HarmoniesNet().eval().cuda())
g = torch.Generator(device="cuda").manual_seed(0)
board = (torch.rand(B, 38, 5, 7, device="cuda", generator=g) > 0.8).float()
board[:, 37] = torch.randint(1, 3, (B, 1, 1), device="cuda", generator=g).float() / 3.0
glob = torch.rand(B, 42, device="cuda", generator=g)
L = nat.lib()
outs, ts = {}, {0: [], 1: []}
for t in (0, 1):
    assert L.hz_resblock_x6_set_table(t) == 0
    outs[t] = fnet.predict(board, glob)
for _ in range(40):
    fnet.predict(board, glob)
for r in range(rounds):
    for t in ((0, 1) if r % 2 == 0 else (1, 0)):
        assert L.hz_resblock_x6_set_table(t) == 0
        fnet.predict(board, glob)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fnet.predict(board, glob)
        e1.record()
        torch.cuda.synchronize()
        ts[t].append(e0.elapsed_time(e1) / 20)
L.hz_resblock_x6_set_table(1)  # (the default)
same = all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
med = {t: sorted(v)[len(v) // 2] for t, v in ts.items()}
print(json.dumps({"batch": B, "bit_identical": same, "ms_median": med, "ms_min": {t: min(v) for t, v in ts.items()},
                  "ms_all": {t: [round(x, 4) for x in v] for t, v in ts.items()}}))
