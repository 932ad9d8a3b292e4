"""k_play2's launch span against its waves' (roles diag build,
tools/libhz_roles.so): per wave the s_memrealtime start/end (100 MHz) and
s_memtime cycles of the last of a run of back-to-back launches; prints the
launch period (HIP events over 100 launches), the span from the first wave
start to the last wave end, the longest wave, the dispatch spread (last wave
start) and the in-kernel clock.  Usage (GPU box): python tools/p2_span.py"""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("HZ_LIB", os.path.join(ROOT, "tools", "libhz_roles.so"))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import numpy as np
import torch
import hzamd._native as nat
from hzamd.env import BatchedEnv
n = int(os.environ.get("HZ_P2_BOARDS", "4096"))
L = nat.lib()
L.hz_diag_set_stamps.argtypes = [ctypes.c_void_p]
stamps = torch.zeros(n, 48, dtype=torch.int64, device="cuda")
L.hz_diag_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
L.hz_diag_set_role_only(-1)
env = BatchedEnv(n, device="cuda")
env.set_pipeline(2)
g = torch.zeros(n, dtype=torch.int32, device="cuda")
st = torch.zeros(n, dtype=torch.int32, device="cuda")
for _ in range(20):
    env.rollout(200, games_done=g, steps_done=st, reset=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(100):  # back to back, as bench.py launches them
    env.rollout(200, games_done=g, steps_done=st, reset=True)
e1.record()
torch.cuda.synchronize()
ROLE = int(os.environ.get("HZ_P2_ROLE", "-1"))  # >= 0: one more launch with only that block role (0 play .. 3 seed)
if ROLE >= 0:
    L.hz_diag_set_role_only(ROLE)
    stamps.zero_()
    env.rollout(200, games_done=g, steps_done=st, reset=True)
    torch.cuda.synchronize()
    L.hz_diag_set_role_only(-1)
s = stamps[:, 40].cpu().numpy().astype(np.int64).reshape(-1, 64)  # [block][16 role + 4 w + k]
names = {0: ["playD", "playC", "playB", "playA"], 1: ["D1", "D2", "P1b", "hashes"], 2: ["D3", "D4", "P1a", "idle"],
         3: ["P2a", "P2b", "P2c", "twist"]}
rs, re_, ts, te = (s[:, k::4] for k in range(4))  # [block][role * 4 + w]
valid = rs > 0
base = rs[valid].min()
start, end = (rs - base) / 100.0, (re_ - base) / 100.0
dur = end - start
clk = (te - ts) / np.maximum(re_ - rs, 1) * 100.0
start, end, dur = (np.where(valid, x, np.nan) for x in (start, end, dur))
out = {"role_only": ROLE, "period_us": e0.elapsed_time(e1) * 1e3 / 100,
       "span_us": float(np.nanmax(end)), "last_start_us": float(np.nanmax(start)),
       "first_end_us": float(np.nanmin(end)), "clock_mhz_median": float(np.median(clk[valid]))}
waves = {}
for role in range(4):
    for w in range(4):
        c = role * 4 + w
        nm = names[role][w]
        if not valid[:, c].any():
            continue
        waves[nm] = {"start_max": float(np.nanmax(start[:, c])), "end_max": float(np.nanmax(end[:, c])),
                     "dur_max": float(np.nanmax(dur[:, c])), "dur_med": float(np.nanmedian(dur[:, c])),
                     "cycles_max": float((te - ts)[:, c].max())}
out["waves"] = waves
# block rounds (n > 4096: more blocks than CUs): per CU, the gap between a
# block's last wave end and the next block's first wave start there (a block
# is (rb, role): columns 4 role .. 4 role + 3 of row rb)
hw = stamps[:, 41].cpu().numpy().astype(np.int64).reshape(-1, 64)[:, 0::4]  # [rb][4 role + w]
blocks = []
for role in range(4):
    cols = slice(4 * role, 4 * role + 4)
    v = valid[:, cols].any(axis=1)
    for rb in np.flatnonzero(v):
        h = hw[rb, 4 * role]
        blocks.append((((h >> 8) & 0x7F) | ((h >> 32) << 8), np.nanmin(start[rb, cols]), np.nanmax(end[rb, cols])))
gaps, per_cu = [], {}
for c, b_s, b_e in blocks:
    per_cu.setdefault(c, []).append((b_s, b_e))
for c, lst in per_cu.items():
    lst.sort()
    for (s1, e1), (s2, e2) in zip(lst[:-1], lst[1:]):
        gaps.append(s2 - e1)
if gaps:
    out["block_gap_us"] = {"n": len(gaps), "median": float(np.median(gaps)), "max": float(np.max(gaps)),
                           "min": float(np.min(gaps))}
out["blocks_per_cu_max"] = max(len(v) for v in per_cu.values())
out["cus_used"] = len(per_cu)
# the last episode column's in-stage phases (cycles since the stage began;
# tools/p2_roles.py's slot names)
ph = stamps.cpu().numpy().astype(np.int64)
pnames = {16: "playA_loaded", 17: "playA_plies", 25: "playD_loaded", 26: "playD_plies", 27: "playD_scored",
          28: "D1_staged", 30: "D3_staged", 32: "P2a_staged", 33: "P2b_staged", 34: "P2c_staged",
          35: "twist_go", 36: "twist_it1", 37: "twist_looped"}
out["phases_last_column"] = {nm: [float(ph[:, k].max()), float(np.median(ph[:, k]))] for k, nm in pnames.items()}
out["longest"] = max((v["dur_max"], k) for k, v in waves.items())
env.close()
print(json.dumps(out))
