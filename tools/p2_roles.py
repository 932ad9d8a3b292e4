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
    names = ({0: "playD", 1: "playC", 2: "playB", 3: "playA", 4: "D1", 5: "D2", 6: "P1b", 7: "hashes", 8: "D3",
              9: "D4", 10: "P1a", 12: "P2a", 13: "P2b", 14: "P2c", 15: "twist",
              16: "playA_loaded", 17: "playA_plies", 19: "playB_loaded", 20: "playB_plies",
              22: "playC_loaded", 23: "playC_plies", 25: "playD_loaded", 26: "playD_plies", 27: "playD_scored",
              28: "D1_staged", 29: "D2_staged", 30: "D3_staged", 31: "D4_staged",
              32: "P2a_staged", 33: "P2b_staged", 34: "P2c_staged",
              35: "twist_go", 36: "twist_it1", 37: "twist_looped", 38: "twist_done_seen"} if pipe == 2 else
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
