"""A/B of the tower conv's 8-state forms at the leaf-eval batch, one form per
process (the form is chosen once per process: HZ_X6_W4=0 -> the 8-wave
k_conv3x3_x6<4,false,8,2>, otherwise the 4-wave k_conv3x3_x6w4).
Times back-to-back launches with HIP events (with and without the residual,
interleaved in blocks so both see the same clock history), saves the outputs
for a bitwise comparison and prints one JSON line.
Usage (GPU box): HZ_X6_W4=0 python tools/conv_ab.py out_a.pt; python tools/conv_ab.py out_b.pt
                 python tools/conv_ab.py --compare out_a.pt out_b.pt"""
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

from hzamd.infer import _conv3x3_x6_act, pack_conv3x3_x6  # noqa: E402

B = int(os.environ.get("HZ_AB_BATCH", "4096"))
cl = torch.channels_last
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=cl)
w = pack_conv3x3_x6(torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.03)
bias = torch.randn(128, device="cuda", generator=g)
r = torch.randn(B, 128, 5, 7, device="cuda", generator=g).contiguous(memory_format=cl)
flop = 2.0 * B * 35 * 128 * 1152
res = {"form": "w8" if os.environ.get("HZ_X6_W4", "1") == "0" else "w4", "batch": B}
outs = {"res": _conv3x3_x6_act(x, w, bias, r), "nores": _conv3x3_x6_act(x, w, bias, None)}
for _ in range(200):  # ~30 ms of warm-up: the clock settles under load
    _conv3x3_x6_act(x, w, bias, r)
times = {"res": [], "nores": []}
for blk in range(6):
    for name, rr in (("res", r), ("nores", None)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            _conv3x3_x6_act(x, w, bias, rr)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 50 * 1e3)
for name, v in times.items():
    v = sorted(v)
    res[name + "_us_median"] = v[len(v) // 2]
    res[name + "_us_all"] = [round(t, 2) for t in v]
res["tflops_fp32_equiv_res"] = flop / (res["res_us_median"] * 1e-6) / 1e12
torch.save({k: t.cpu() for k, t in outs.items()}, sys.argv[1])
print(json.dumps(res), flush=True)
