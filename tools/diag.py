"""Phase attribution for k_reset / k_rollout from the HZ_DIAG build
(tools/libhz_diag.so): per-lane s_memtime stamps, reported in cycles."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# tools/diag.py [roles]: "roles" uses libhz_roles.so (role durations only, no
# stamps inside the ply loop)
os.environ.setdefault("HZ_LIB", os.path.join(ROOT, "tools", "libhz_roles.so" if "roles" in sys.argv[1:] else "libhz_diag.so"))
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
for rep in range(3):
    stamps.zero_()
    a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    a.record(); env.reset(); b.record(); env.rollout(96); c.record()
    f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f0.record(); env.rollout(96, reset=True); f1.record()
    torch.cuda.synchronize()
    s = stamps.cpu().double()
    out = {"reset_us": a.elapsed_time(b) * 1e3, "rollout_us": b.elapsed_time(c) * 1e3, "play_us": f0.elapsed_time(f1) * 1e3,
           "reset_seed_cyc": (s[:, 1] - s[:, 0]).mean().item(), "reset_draw_cyc": (s[:, 2] - s[:, 1]).mean().item(),
           "reset_store_cyc": (s[:, 3] - s[:, 2]).mean().item(), "reset_writeout_cyc": (s[:, 4] - s[:, 3]).mean().item(),
           "reset_total_cyc_max": (s[:, 4] - s[:, 0]).max().item(),
           "roll_top_cyc": s[:, 8].mean().item(), "roll_legal_cyc": s[:, 9].mean().item(),
           "roll_pick_cyc": s[:, 10].mean().item(), "roll_step_cyc": s[:, 11].mean().item(),
           "roll_turnend_cyc": s[:, 12].mean().item(), "roll_final_cyc": s[:, 13].mean().item()}
# steady-state hz_play (chance-ahead primed: boards replay prepared pile scripts)
for _ in range(3):
    env.rollout(96, reset=True)
stamps.zero_()
f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
f0.record(); env.rollout(96, reset=True); f1.record()
torch.cuda.synchronize()
s = stamps.cpu().double()
out.update({"play_primed_us": f0.elapsed_time(f1) * 1e3,
            "primed_top_cyc": s[:, 8].mean().item(), "primed_legal_cyc": s[:, 9].mean().item(),
            "primed_pick_cyc": s[:, 10].mean().item(), "primed_step_cyc": s[:, 11].mean().item(),
            "primed_turnend_cyc": s[:, 12].mean().item(), "primed_final_cyc": s[:, 13].mean().item(),
            "role_play_cyc_max": s[:, 5].max().item(), "role_draw2_cyc_max": s[:, 6].max().item(),
            "role_seed_cyc_max": s[:, 7].max().item(),
            # preparation phases, cycles since the role began (max over boards)
            "role_draw1_cyc_max": s[:, 15].max().item(),
            # play role (roles build): cycles since the role began, max over boards
            "play_after_barrier": s[:, 13].max().item(), "play_after_reset": s[:, 8].max().item(), "play_after_loop": s[:, 9].max().item(),
            "play_after_final_scoring": s[:, 10].max().item(),
            "seed_waves13_overlap_done": s[:, 11].max().item(), "seed_after_barrier": s[:, 12].max().item(),
            "seed_after_seed": s[:, 0].max().item(), "seed_after_twist": s[:, 1].max().item(),
            "draw1_after_stage_in": s[:, 2].max().item(), "draw1_after_draws": s[:, 3].max().item(),
            "draw2_after_stage_in": s[:, 4].max().item(), "draw2_after_draws": s[:, 14].max().item()})
print(json.dumps(out))
