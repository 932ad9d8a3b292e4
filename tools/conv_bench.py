"""Tower conv kernels at the leaf-eval batch: hz_conv3x3_bias_act (f32 MFMA)
vs hz_conv3x3_x6_bias_act (bf16 MFMA, fp32-exact split products), HIP-event
timed over back-to-back launches; prints one JSON line.
Usage (GPU box): python tools/conv_bench.py [batch]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd.infer import (_conv3x3_act, _conv3x3_x6_act, _stem_act, _stem_x6_act, pack_conv3x3,  # noqa: E402
                         pack_conv3x3_x6, pack_stem, pack_stem_x6)

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cl = torch.channels_last
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=cl)
w = torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.03
b = torch.randn(128, device="cuda", generator=g)
r = torch.randn(B, 128, 5, 7, device="cuda", generator=g).contiguous(memory_format=cl)
flop = 2.0 * B * 35 * 128 * 1152
out = {"batch": B, "gflop_per_conv": flop / 1e9}
for name, fn, wp in (("f32", _conv3x3_act, pack_conv3x3(w)), ("x6", _conv3x3_x6_act, pack_conv3x3_x6(w))):
    for _ in range(20):
        fn(x, wp, b, r)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 100
    e0.record()
    for _ in range(reps):
        fn(x, wp, b, r)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    out[name] = {"us": us, "tflops": flop / (us * 1e-6) / 1e12}
k = 256  # float64 reference on the CPU for the first k states
want = (torch.nn.functional.conv2d(x[:k].double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
        + r[:k].double().cpu()).relu()
for name, fn, wp in (("f32", _conv3x3_act, pack_conv3x3(w)), ("x6", _conv3x3_x6_act, pack_conv3x3_x6(w))):
    out[name]["max_abs_err_vs_fp64"] = (fn(x, wp, b, r)[:k].double().cpu() - want).abs().max().item()
# x6 without the residual (the first conv of a block): the epilogue's share
for _ in range(20):
    _conv3x3_x6_act(x, pack_conv3x3_x6(w), b, None)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
wp6n = pack_conv3x3_x6(w)
e0.record()
for _ in range(100):
    _conv3x3_x6_act(x, wp6n, b, None)
e1.record()
torch.cuda.synchronize()
out["x6_nores_us"] = e0.elapsed_time(e1) / 100 * 1e3
# x6 with a device live-row count (gathered leaf batches): us per call
wp6 = pack_conv3x3_x6(w)
out["x6_live_us"] = {}
for lv in (4096, 3500, 3000, 2049, 2048, 1000, 256):
    lt = torch.tensor([lv], dtype=torch.int32, device="cuda")
    for _ in range(5):
        _conv3x3_x6_act(x, wp6, b, r, lt)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        _conv3x3_x6_act(x, wp6, b, r, lt)
    e1.record()
    torch.cuda.synchronize()
    out["x6_live_us"][lv] = e0.elapsed_time(e1) / 50 * 1e3
# the stem (38 -> 128 channels, NCHW board in)
board = (torch.rand(B, 38, 5, 7, device="cuda", generator=g) > 0.7).float()
ws = torch.randn(128, 38, 3, 3, device="cuda", generator=g) * 0.1
sflop = 2.0 * B * 35 * 128 * 342
for name, fn, wp in (("stem_f32", _stem_act, pack_stem(ws)), ("stem_x6", _stem_x6_act, pack_stem_x6(ws))):
    for _ in range(20):
        fn(board, wp, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        fn(board, wp, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 100 * 1e3
    out[name] = {"us": us, "tflops_algorithmic": sflop / (us * 1e-6) / 1e12}


def timed(fn, reps=100):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


# the stem on a board with non-bf16 values everywhere (the six-product path
# an encoder board, all of whose staged values are bf16 values, avoids)
board_g = board * 0.3
wps = pack_stem_x6(ws)
out["stem_x6_general_us"] = timed(lambda: _stem_x6_act(board_g, wps, b))
# the head: hz_heads_fc against hz_heads + three linear layers + softmax + tanh
from hzamd.infer import FoldedNet, _heads, _heads_fc  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402
fn = FoldedNet(HarmoniesNet().eval().cuda())
glob = torch.rand(B, 42, device="cuda", generator=g)
F = torch.nn.functional


def split_head():
    pcat, vcat = _heads(x, glob, *fn.heads)
    lo = F.linear(pcat, *fn.pfc)
    v = torch.tanh(F.linear(F.linear(vcat, *fn.vfc1).relu_(), *fn.vfc2))
    return torch.softmax(lo, 1), v


out["head_split_us"] = timed(split_head)
out["head_fused_us"] = timed(lambda: _heads_fc(x, glob, *fn.heads, fn.fc, logits=False, probs=True))
# the x6 conv at small batches (<= HZ_X6_SMALL_MAX rows: one state per workgroup)
out["x6_small_max"] = int(os.environ.get("HZ_X6_SMALL_MAX", "768"))
out["x6_batch_us"] = {}
for bs in (8, 32, 64, 128, 256, 512, 768, 1024, 2048):
    xs, rs = x[:bs].contiguous(memory_format=cl), r[:bs].contiguous(memory_format=cl)
    out["x6_batch_us"][bs] = timed(lambda: _conv3x3_x6_act(xs, wp6, b, rs), reps=50)
print(json.dumps(out))
