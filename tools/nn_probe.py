"""Time the reference-architecture network's leaf-eval forward at batch 4096."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import torch
from hzamd.net import HarmoniesNet, flops_per_eval
torch.backends.cudnn.benchmark = True
dev = "cuda:0"
torch.manual_seed(0)
net = HarmoniesNet().to(dev).eval()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
board = (torch.rand(B, 38, 5, 7, device=dev) > 0.8).float()
glob = torch.rand(B, 42, device=dev)
res = {}
for name, dtype, cl in [("fp32", None, False), ("fp32_cl", None, True), ("bf16", torch.bfloat16, False),
                        ("bf16_cl", torch.bfloat16, True)]:
    m = net.to(memory_format=torch.channels_last) if cl else net.to(memory_format=torch.contiguous_format)
    x = board.to(memory_format=torch.channels_last) if cl else board
    with torch.no_grad():
        for _ in range(3):
            if dtype:
                with torch.autocast("cuda", dtype=dtype):
                    m(x, glob)
            else:
                m(x, glob)
        torch.cuda.synchronize()
        t = time.perf_counter()
        R = 10
        for _ in range(R):
            if dtype:
                with torch.autocast("cuda", dtype=dtype):
                    m(x, glob)
            else:
                m(x, glob)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / R
    res[name] = {"ms": dt * 1e3, "tflops": flops_per_eval() * B / dt / 1e12}
from hzamd.infer import FoldedNet
fn = FoldedNet(net.to(memory_format=torch.contiguous_format))
with torch.no_grad():
    for _ in range(3):
        fn(board, glob)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        fn(board, glob)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 10
res["fp32_folded"] = {"ms": dt * 1e3, "tflops": flops_per_eval() * B / dt / 1e12}
print(json.dumps(res))
