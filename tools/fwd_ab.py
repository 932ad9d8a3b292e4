"""The whole leaf-eval forward (FoldedNet.predict) at the leaf-eval batch, one
library per process (HZ_LIB selects it): HIP events around back-to-back
forwards on encoder-like boards; outputs saved for a bitwise comparison.
Usage (GPU box): python tools/fwd_ab.py out.pt; python tools/fwd_ab.py --compare a.pt b.pt"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = (torch.load(p, weights_only=True) for p in sys.argv[2:4])
    print(json.dumps({k: bool(torch.equal(a[k], b[k])) for k in a}))
    sys.exit(0 if all(torch.equal(a[k], b[k]) for k in a) else 1)

from hzamd.infer import FoldedNet  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

B = int(os.environ.get("HZ_AB_BATCH", "4096"))
torch.manual_seed(0)
fnet = FoldedNet(HarmoniesNet().eval().cuda())
g = torch.Generator(device="cuda").manual_seed(0)
board = (torch.rand(B, 38, 5, 7, device="cuda", generator=g) > 0.8).float()
board[:, 37] = torch.randint(1, 3, (B, 1, 1), device="cuda", generator=g).float() / 3.0
glob = torch.rand(B, 42, device="cuda", generator=g)
p, v = fnet.predict(board, glob)
for _ in range(30):
    fnet.predict(board, glob)
ts = []
for blk in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fnet.predict(board, glob)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 20)
ts.sort()
torch.save({"probs": p.cpu(), "value": v.cpu()}, sys.argv[1])
print(json.dumps({"batch": B, "ms_median": ts[len(ts) // 2], "ms_all": [round(t, 4) for t in ts]}), flush=True)
