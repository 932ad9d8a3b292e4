"""Stem timing at the leaf-eval batch (one library per process, HZ_LIB selects
it): hz_stem3x3_x6_bias_act on encoder-like boards (0/1 planes and the phase
channel at 1/3, 2/3: the h-plane-only path) and on generic fp32 boards (all
six products), HIP events around back-to-back launches; the outputs are
saved for a bitwise comparison between libraries.
Usage (GPU box): python tools/stem_ab.py out.pt; python tools/stem_ab.py --compare a.pt b.pt"""
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

from hzamd.infer import _stem_x6_act, pack_stem_x6  # noqa: E402

B = int(os.environ.get("HZ_AB_BATCH", "4096"))
g = torch.Generator(device="cuda").manual_seed(0)
enc = (torch.rand(B, 38, 5, 7, device="cuda", generator=g) > 0.8).float()
enc[:, 37] = torch.randint(1, 3, (B, 1, 1), device="cuda", generator=g).float() / 3.0
gen = torch.rand(B, 38, 5, 7, device="cuda", generator=g)
w = pack_stem_x6(torch.randn(128, 38, 3, 3, device="cuda", generator=g) * 0.1)
b = torch.randn(128, device="cuda", generator=g) * 0.1
res = {"batch": B}
outs = {"encoder": _stem_x6_act(enc, w, b), "generic": _stem_x6_act(gen, w, b)}
for _ in range(200):
    _stem_x6_act(enc, w, b)
for name, x in (("encoder", enc), ("generic", gen)):
    ts = []
    for blk in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            _stem_x6_act(x, w, b)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 50 * 1e3)
    ts.sort()
    res[name + "_us_median"] = ts[len(ts) // 2]
    res[name + "_us_all"] = [round(t, 2) for t in ts]
torch.save({k: t.cpu() for k, t in outs.items()}, sys.argv[1])
print(json.dumps(res), flush=True)
