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
stamps = torch.zeros(n, 16, dtype=torch.int64, device="cuda")
L.hz_diag_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
out = {}
for pipe in (1, 2):
    env = BatchedEnv(n, device="cuda")
    env.set_pipeline(pipe)
    names = (["play_block", "play_block_", "drawA", "drawB", "drawC", "hashes", "P1", "P2", "playB",
              "playA"] if pipe == 2 else
             {5: "play", 6: "draw2", 15: "draw1", 7: "seed"})
    for only in (-1, 0, 1, 2) if pipe == 2 else (-1,):
        L.hz_diag_set_role_only(-1)
        for _ in range(8):
            env.rollout(200, reset=True)
        L.hz_diag_set_role_only(only)
        stamps.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); env.rollout(200, reset=True); e1.record()
        torch.cuda.synchronize()
        s = stamps.cpu().double()
        items = enumerate(names) if pipe == 2 else names.items()
        key = f"p{pipe}_" + ("all" if only < 0 else ("play", "draw", "seed")[only] + "_alone")
        out[key] = {"us": e0.elapsed_time(e1) * 1e3,
                    **{nm: [s[:, k].max().item(), s[:, k].median().item()] for k, nm in items}}
    env.close()
L.hz_diag_set_role_only(-1)
print(json.dumps(out))
