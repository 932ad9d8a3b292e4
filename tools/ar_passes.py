"""Auto-reset rollouts (hz_rollout(max_plies, auto_reset=1), continued launch
after launch): per wave, the reseeding passes and loop iterations of the
last launch and its in-kernel time (roles diag build, tools/libhz_roles.so:
slots 11/12 and the play role's slot 5), plus the launch time by events.
Usage (GPU box): python tools/ar_passes.py [plies]"""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("HZ_LIB", os.path.join(ROOT, "tools", "libhz_roles.so"))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import numpy as np
import torch
import hzamd._native as nat
from hzamd.env import BatchedEnv
n, plies = 4096, int(sys.argv[1]) if len(sys.argv) > 1 else 96
L = nat.lib()
L.hz_diag_set_stamps.argtypes = [ctypes.c_void_p]
stamps = torch.zeros(n, 48, dtype=torch.int64, device="cuda")
L.hz_diag_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
env = BatchedEnv(n, seed_base=7, device="cuda")
env.set_pipeline(1)
env.reset()
g = torch.zeros(n, dtype=torch.int32, device="cuda")
st = torch.zeros(n, dtype=torch.int32, device="cuda")
for _ in range(8):
    env.rollout(plies, auto_reset=True, games_done=g, steps_done=st)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
stamps.zero_()
e0.record()
env.rollout(plies, auto_reset=True, games_done=g, steps_done=st)
e1.record()
torch.cuda.synchronize()
s = stamps.cpu().numpy().reshape(-1, 16)[:n]
w = s[::64]  # lane 0 of each wave
out = {"plies": plies, "launch_us": e0.elapsed_time(e1) * 1e3,
       "passes": {"median": float(np.median(w[:, 11])), "max": int(w[:, 11].max()), "min": int(w[:, 11].min())},
       "iterations": {"median": float(np.median(w[:, 12])), "max": int(w[:, 12].max())},
       "wave_cycles": {"median": float(np.median(s[::64, 5])), "max": float(s[::64, 5].max())},
       "games_per_board": float(g.double().mean())}
env.close()
print(json.dumps(out))
