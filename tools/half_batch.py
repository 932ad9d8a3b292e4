"""Leaf-eval forward of the default 128x8 network at 4096 rows, timed as one
call against the same rows in 2 or 4 consecutive slices (each slice's
activations are a half or a quarter of the 73 MB a full-batch conv streams,
so more of a conv's working set stays in the MALL).  Prints ms per 4096 rows
for each split, HIP events around `reps` back-to-back forwards.
Usage (GPU box): python tools/half_batch.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]
import torch  # noqa: E402

from hzamd.infer import FoldedNet  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
torch.manual_seed(0)
net = HarmoniesNet().cuda().eval()
f = FoldedNet(net)
n = 4096
board = (torch.rand(n, 38, 5, 7, device="cuda") < 0.3).float()
glob = torch.rand(n, 42, device="cuda")
out = {}
ref = f.predict(board, glob)
for parts in (1, 2, 4, 1, 2):
    k = n // parts
    for _ in range(3):
        for p in range(parts):
            f.predict(board[p * k:(p + 1) * k], glob[p * k:(p + 1) * k])
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        for p in range(parts):
            pr, v = f.predict(board[p * k:(p + 1) * k], glob[p * k:(p + 1) * k])
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    same = bool(torch.equal(pr, ref[0][(parts - 1) * k:]) and torch.equal(v, ref[1][(parts - 1) * k:]))
    out.setdefault(str(parts), []).append({"ms_per_4096_rows": ms, "last_slice_bit_identical": same})
print(json.dumps(out, indent=1))
