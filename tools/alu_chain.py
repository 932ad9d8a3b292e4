"""Cycles per dependent step of the candidate seeding-recurrence forms
(tools/alu_chain.hip), one wave per SIMD, and a check that the 24-bit
multiply forms equal the plain ones."""
import ctypes, json, os
import numpy as np
import torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libalu.so"))
names = ["mul_lo", "mul_u24", "xorshift", "seed1", "seed1_u24", "seed2", "seed2_u24"]
res, outs = {}, {}
for k, nm in enumerate(names):
    out = torch.zeros(64 * 64, dtype=torch.int32, device="cuda")
    cyc = torch.zeros(64, dtype=torch.int64, device="cuda")
    for _ in range(3):
        assert lib.alu_chain(k, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), 64) == 0
    torch.cuda.synchronize()
    res[nm] = float(cyc.double().median().item()) / 1024
    outs[nm] = out.cpu().numpy()
res["seed1_u24_equal"] = bool((outs["seed1"] == outs["seed1_u24"]).all())
res["seed2_u24_equal"] = bool((outs["seed2"] == outs["seed2_u24"]).all())
print(json.dumps(res))
sv = {}
outs = {}
for v, nm in [(0, "mt_seed_lds"), (1, "pass1_lds"), (2, "pass1_nostore"), (3, "pass1_ldstab"), (4, "mt_seed_tab64"),
              (6, "mt_seed_lds_256blk"), (7, "mt_seed_tab64_256blk"), (8, "pass2_as_is"), (9, "pass2_nostore"),
              (10, "pass2_noload")]:
    out = torch.zeros(256 * 64, dtype=torch.int32, device="cuda")
    cyc = torch.zeros(256, dtype=torch.int64, device="cuda")
    for _ in range(3):
        assert lib.seed_var(v, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()), 64) == 0
    torch.cuda.synchronize()
    nb = 256 if v in (6, 7) else 64
    sv[nm] = float(cyc[:nb].double().median().item())
    outs[nm] = out[:64 * 64].cpu().numpy()
sv["tab_equal"] = bool((outs["mt_seed_lds"] == outs["mt_seed_tab64"]).all())
print(json.dumps(sv))
# pass-2 chain forms (alu_chain.hip k_p2chain): cycles per step over 616 steps
L = lib
L.p2chain.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
gout = torch.zeros(64 * 64 * 624, dtype=torch.int32, device="cuda")
pc = {}
for v, s, nm in [(0, 0, "lds_col_read+b32_store (P2a)"), (1, 0, "lds_col_read"), (2, 0, "b32_store"), (3, 0, "bare"),
                 (4, 628, "lds_bm_b128_read s628"), (4, 632, "lds_bm_b128_read s632"),
                 (5, 628, "lds_bm_b128_read+b128_store/4 s628"), (5, 632, "lds_bm_b128_read+b128_store/4 s632"),
                 (6, 628, "lds_bm_b128_read+b32_store"), (7, 0, "b128_store/4")]:
    out = torch.zeros(64 * 64, dtype=torch.int32, device="cuda")
    cyc = torch.zeros(64, dtype=torch.int64, device="cuda")
    for _ in range(3):
        assert L.p2chain(v, s, ctypes.c_void_p(gout.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                         ctypes.c_void_p(cyc.data_ptr()), 64) == 0
    torch.cuda.synchronize()
    pc[nm] = float(cyc.double().median().item()) / 616
print(json.dumps({"p2chain_cycles_per_step": pc}))
