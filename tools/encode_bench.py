"""Encoder throughput (hz_encode_states): M states -> f32 [M,38,5,7] + [M,42],
5,488 B written per state; reports GB/s of output vs the 8 TB/s HBM peak."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
import torch
from hzamd.env import BatchedEnv
from hzamd.selfplay import encode_states
dev = "cuda:0"
n = 4096
env = BatchedEnv(n, device=dev)
env.reset()
# one batch of full games recorded ply by ply: realistic states
_, steps, (ts, tm, ta) = env.rollout(96, record=True)
valid = (ta >= 0).reshape(-1)
states = ts.permute(0, 2, 1).reshape(-1, 6)[valid].contiguous()
M = states.shape[0]
res = {"states": M}
for _ in range(3):
    encode_states(states)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
R = 20
e0.record()
for _ in range(R):
    encode_states(states)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / R
res.update({"ms": ms, "GBps": M * 5488 / (ms * 1e-3) / 1e9, "frac_of_8TBps": M * 5488 / (ms * 1e-3) / 8e12})
print(json.dumps(res))
# the store ceiling for the same bytes: torch's fill kernel and a memset
buf = torch.empty(M * 5488 // 4, dtype=torch.float32, device=dev)
for name, fn in (("fill", lambda: buf.fill_(1.0)), ("zero", lambda: buf.zero_())):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(R):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms2 = e0.elapsed_time(e1) / R
    res[f"{name}_GBps"] = buf.numel() * 4 / (ms2 * 1e-3) / 1e9
print(json.dumps(res))
