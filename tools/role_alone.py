"""Each k_rollout role's duration with the other roles' blocks exiting at
once (roles-only diag build), against all roles together: the cost of
sharing the chip.  Steady state first (all roles), then one role per launch."""
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
slot = {0: 6, 1: 15, 2: 7, 3: 5}
name = {0: "draw2", 1: "draw1", 2: "seed", 3: "play"}
out = {}
for only in (-1, 0, 1, 2, 3):
    L.hz_diag_set_role_only(-1)
    for _ in range(4):
        env.rollout(200, reset=True)
    L.hz_diag_set_role_only(only)
    stamps.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); env.rollout(200, reset=True); e1.record()
    torch.cuda.synchronize()
    s = stamps.cpu().double()
    key = "all" if only < 0 else name[only] + "_alone"
    out[key] = {"us": e0.elapsed_time(e1) * 1e3, **{name[r]: s[:, slot[r]].max().item() for r in slot}}
L.hz_diag_set_role_only(-1)
print(json.dumps(out))
