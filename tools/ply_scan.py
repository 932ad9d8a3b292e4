"""Play-role cycles vs plies played (roles-only diag build): hz_play with
max_plies = P, steady state; a linear fit separates per-ply cost from the
fixed per-launch cost (reset from the script, stream copy, final scoring)."""
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
env = BatchedEnv(n, device="cuda")
out = {}
for P in (8, 16, 32, 48, 64, 96):
    for _ in range(3):
        env.rollout(P, reset=True)
    stamps.zero_()
    env.rollout(P, reset=True)
    torch.cuda.synchronize()
    s = stamps.cpu().double()
    out[P] = {"play_max": s[:, 5].max().item(), "draw2_max": s[:, 6].max().item(), "draw1_max": s[:, 15].max().item(),
              "seed_max": s[:, 7].max().item()}
print(json.dumps(out))
