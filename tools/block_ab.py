"""A/B of one residual block at the leaf-eval batch, in one process:
hz_resblock_x6_bias_act as one launch (k_conv3x3_x6w4<true>) against the two
layered 4-wave convs, interleaved in blocks so both see the same clock
history; outputs compared bit for bit.  Prints one JSON line.
Usage (GPU box): python tools/block_ab.py [batch]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd._native import lib  # noqa: E402
from hzamd.infer import _conv3x3_x6_act, _resblock_x6, pack_conv3x3_x6  # noqa: E402

assert lib().hz_resblock_x6_set_fused(1) == 0  # _resblock_x6 = the one-launch form (the default)

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cl = torch.channels_last
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=cl)
p1 = pack_conv3x3_x6(torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.03)
p2 = pack_conv3x3_x6(torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.03)
b1 = torch.randn(128, device="cuda", generator=g) * 0.1
b2 = torch.randn(128, device="cuda", generator=g) * 0.1


def fused():
    return _resblock_x6(x, p1, b1, p2, b2)


def layered():
    return _conv3x3_x6_act(_conv3x3_x6_act(x, p1, b1), p2, b2, x)


res = {"batch": B, "bit_identical": bool(torch.equal(fused(), layered()))}
for _ in range(100):
    fused()
    layered()
times = {"fused": [], "layered": []}
for blk in range(8):
    for name, fn in (("fused", fused), ("layered", layered)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            fn()
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 30 * 1e3)
for name, v in times.items():
    v = sorted(v)
    res[name + "_us_median"] = v[len(v) // 2]
    res[name + "_us_all"] = [round(t, 2) for t in v]
flop = 2 * 2.0 * B * 35 * 128 * 1152
res["fused_tflops_fp32_equiv"] = flop / (res["fused_us_median"] * 1e-6) / 1e12
print(json.dumps(res), flush=True)
