"""The fused head (hz_heads_fc) at the leaf-eval batch, one library per process
(HZ_LIB selects it): HIP events around back-to-back launches on a random
tower output; outputs saved for a bitwise comparison between libraries.
Usage (GPU box): python tools/head_ab.py out.pt; python tools/head_ab.py --compare a.pt b.pt"""
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

from hzamd.infer import FoldedNet, _heads_fc  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

B = int(os.environ.get("HZ_AB_BATCH", "4096"))
torch.manual_seed(0)
fnet = FoldedNet(HarmoniesNet().eval().cuda())
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=torch.channels_last)
gl = torch.rand(B, 42, device="cuda", generator=g)


def run():
    return _heads_fc(x, gl, *fnet.heads, fnet.fc, logits=True, probs=True)


lo, pr, v = run()
for _ in range(200):
    run()
ts = []
for blk in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 50 * 1e3)
ts.sort()
torch.save({"logits": lo.cpu(), "probs": pr.cpu(), "value": v.cpu()}, sys.argv[1])
print(json.dumps({"batch": B, "us_median": ts[len(ts) // 2], "us_all": [round(t, 2) for t in ts]}), flush=True)
