"""Seeding a 64-board wave's CPython MT streams with every word in global
memory (tools/alu_chain.hip mt_seed_global: no LDS operation in the chain
wave) against mt_seed in LDS: the words must be equal; cycles per seeding
(s_memtime around the chain) at 64, 256 and 1024 waves (1024 = one per
SIMD).  Usage (GPU box): python tools/seed_glob.py"""
import ctypes
import json
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libalu.so"))
lib.seed_glob.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int]
res = {}
for blocks in (64, 256, 1024):
    n = blocks * 64
    ref = torch.zeros(624, n, dtype=torch.int32, device="cuda")
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    cyc = torch.zeros(blocks, dtype=torch.int64, device="cuda")
    assert lib.seed_glob(0, out.data_ptr(), cyc.data_ptr(), ref.data_ptr(), n, blocks) == 0
    for pf in (8, 16, 24):
        ws = torch.zeros(624, n, dtype=torch.int32, device="cuda")
        for _ in range(3):
            assert lib.seed_glob(pf, out.data_ptr(), cyc.data_ptr(), ws.data_ptr(), n, blocks) == 0
        torch.cuda.synchronize()
        c = cyc.double()
        res[f"b{blocks}_pf{pf}"] = {"equal": bool(torch.equal(ws, ref)), "cycles_median": c.median().item(),
                                    "cycles_max": c.max().item(), "per_step": c.median().item() / 1246}
print(json.dumps(res))
