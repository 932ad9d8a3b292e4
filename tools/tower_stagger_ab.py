"""A/B of the residual tower launch's start stagger (hz_tower_x6_set_stagger:
first-round workgroups on every other CU of each XCD start late, so that the
blocks' epilogue bursts stop coinciding), in ONE process: the whole leaf-eval
forward (FoldedNet.predict) at `batch` rows, the stagger values taking turns
in blocks of 20 forwards for `rounds` rounds; outputs compared bit for bit.
Usage (GPU box): python tools/tower_stagger_ab.py [rounds] [batch] [values...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd import _native as nat  # noqa: E402
from hzamd.infer import FoldedNet  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
vals = [int(v) for v in sys.argv[3:]] or [0, 2, 4, 8, 16]
torch.manual_seed(0)
fnet = FoldedNet(HarmoniesNet().eval().cuda())
g = torch.Generator(device="cuda").manual_seed(0)
board = (torch.rand(B, 38, 5, 7, device="cuda", generator=g) > 0.8).float()
board[:, 37] = torch.randint(1, 3, (B, 1, 1), device="cuda", generator=g).float() / 3.0
glob = torch.rand(B, 42, device="cuda", generator=g)
L = nat.lib()
outs, ts = {}, {v: [] for v in vals}
for v in vals:
    assert L.hz_tower_x6_set_stagger(v) == 0
    outs[v] = fnet.predict(board, glob)
for _ in range(40):
    fnet.predict(board, glob)
for r in range(rounds):
    order = vals if r % 2 == 0 else vals[::-1]
    for v in order:
        L.hz_tower_x6_set_stagger(v)
        fnet.predict(board, glob)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fnet.predict(board, glob)
        e1.record()
        torch.cuda.synchronize()
        ts[v].append(e0.elapsed_time(e1) / 20)
L.hz_tower_x6_set_stagger(0)
same = all(torch.equal(a, b) for v in vals for a, b in zip(outs[vals[0]], outs[v]))
med = {v: sorted(t)[len(t) // 2] for v, t in ts.items()}
print(json.dumps({"batch": B, "bit_identical": same, "ms_median": med, "ms_min": {v: min(t) for v, t in ts.items()}}))
