"""Leaf-eval conv formulations at batch 4096 (fp32): MIOpen conv2d vs GEMM
formulations of the 3x3 / 128-channel conv on the 5x7 board."""
import json, sys, time
import torch
import torch.nn.functional as F
torch.backends.cudnn.benchmark = True
dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
C = 128
torch.manual_seed(0)
x = torch.randn(B, C, 5, 7, device=dev)
w = torch.randn(C, C, 3, 3, device=dev) * 0.05
bias = torch.randn(C, device=dev)
flop = 2 * B * 35 * C * C * 9


def timeit(fn, R=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(R):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / R
    return {"ms": ms, "tflops": flop / ms / 1e9}


res = {}
res["conv2d_nchw"] = timeit(lambda: F.conv2d(x, w, bias, padding=1))
xcl = x.to(memory_format=torch.channels_last)
wcl = w.to(memory_format=torch.channels_last)
res["conv2d_nhwc"] = timeit(lambda: F.conv2d(xcl, wcl, bias, padding=1))
# im2col in NHWC + one GEMM [B*35, 1152] @ [1152, 128]
xh = x.permute(0, 2, 3, 1).contiguous()                  # [B,5,7,C]
wk = w.permute(2, 3, 1, 0).reshape(9 * C, C).contiguous()  # [(ky,kx,ci), co]


def im2col_gemm():
    xp = F.pad(xh, (0, 0, 1, 1, 1, 1))                    # [B,7,9,C]
    cols = torch.cat([xp[:, ky:ky + 5, kx:kx + 7, :] for ky in range(3) for kx in range(3)], dim=3)
    return torch.addmm(bias, cols.view(B * 35, 9 * C), wk)


res["im2col_gemm"] = timeit(im2col_gemm)
# GEMM first: Y = x @ W_all [C, 9C], then shifted sum
wall = w.permute(1, 2, 3, 0).reshape(C, 9 * C).contiguous()  # [ci, (ky,kx,co)]


def gemm_shift():
    y = torch.mm(xh.view(B * 35, C), wall).view(B, 5, 7, 3, 3, C)
    yp = F.pad(y, (0, 0, 0, 0, 0, 0, 1, 1, 1, 1))          # pad H,W by 1: [B,7,9,3,3,C]
    out = bias.expand(B, 5, 7, C).clone()
    for ky in range(3):
        for kx in range(3):
            out += yp[:, 2 - ky:7 - ky, 2 - kx:9 - kx, ky, kx, :]
    return out


res["gemm_shift"] = timeit(gemm_shift)
res["gemm_only_1152x128"] = timeit(lambda: torch.mm(torch.empty(B * 35, 9 * C, device=dev), wk))
res["gemm_only_128x1152"] = timeit(lambda: torch.mm(xh.view(B * 35, C), wall))
# check formulations agree
ref = F.conv2d(x, w, bias, padding=1).permute(0, 2, 3, 1)
res["err_im2col"] = float((im2col_gemm().view(B, 5, 7, C) - ref).abs().max())
res["err_shift"] = float((gemm_shift() - ref).abs().max())
print(json.dumps(res))
