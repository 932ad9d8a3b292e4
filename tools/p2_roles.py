"""k_play2's stage durations (roles-only diag build, tools/libhz_roles.so):
steady state with every block type, then each block type alone (play, draw,
seed): [max, median] over boards in s_memtime cycles (as tools/diag.py),
and the launch's HIP-event time in us.  Pipeline 1's roles for comparison."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("HZ_LIB", os.path.join(ROOT, "tools", "libhz_roles.so"))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import torch
import hzamd._native as nat
from hzamd.env import BatchedEnv
n = 4096
L = nat.lib()
L.hz_diag_set_stamps.argtypes = [ctypes.c_void_p]
stamps = torch.zeros(n, 48, dtype=torch.int64, device="cuda")  # (k_play2 uses 48 slots per board)
L.hz_diag_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
out = {}
for pipe in (1, 2):
    env = BatchedEnv(n, device="cuda")
    env.set_pipeline(pipe)
    names = ({0: "play4", 1: "play3", 2: "play2", 3: "play1", 4: "D1", 5: "D2", 6: "D3", 7: "hashes", 8: "D4",
              9: "D5", 10: "play0", 12: "P2x", 13: "P2y", 14: "twist", 15: "P1",
              16: "play0_loaded", 17: "play0_plies", 18: "play1_loaded", 19: "play1_plies",
              20: "play2_loaded", 21: "play2_plies", 22: "play3_loaded", 23: "play3_plies",
              24: "play4_loaded", 25: "play4_plies", 26: "play4_scored",
              27: "D1_staged", 28: "D2_staged", 29: "D3_staged", 30: "D4_staged", 31: "D5_staged",
              32: "P2x_staged", 33: "P2y_staged",
              35: "twist_go", 36: "twist_it1", 37: "twist_looped"} if pipe == 2 else
             {5: "play", 6: "draw2", 15: "draw1", 7: "seed"})
    for only in (-1, 0, 1, 2, 3) if pipe == 2 else (-1,):
        L.hz_diag_set_role_only(-1)
        for _ in range(16):
            env.rollout(200, reset=True)
        L.hz_diag_set_role_only(only)
        stamps.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); env.rollout(200, reset=True); e1.record()
        torch.cuda.synchronize()
        s = stamps.cpu().double()
        if pipe == 1:  # (k_rollout's stamps: 16 slots per board)
            s = s.reshape(-1, 16)[:n]
        items = names.items()
        key = f"p{pipe}_" + ("all" if only < 0 else ("play", "drawX", "drawY", "seed")[only] + "_alone")
        out[key] = {"us": e0.elapsed_time(e1) * 1e3,
                    **{nm: [s[:, k].max().item(), s[:, k].median().item()] for k, nm in items}}
        if pipe == 2 and only < 0:  # every stage's worst board vs the kernel (the longest chain sets the time)
            out[key]["longest"] = max((v[0], k) for k, v in out[key].items() if k != "us" and isinstance(v, list))
    env.close()
L.hz_diag_set_role_only(-1)
print(json.dumps(out))
