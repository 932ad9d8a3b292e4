"""k_play2 throughput at 16,384 boards: one env of 16,384 boards against four
envs of 4,096 launched round-robin (the same boards' work per round, each
launch one round of all four roles; the four envs' stream-slot hand-offs
together as large as the single env's).  Separates the dispatch-order effect
from the working-set effect behind the large-batch slowdown.
Usage (GPU box): python tools/p2_scale.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd")]

import torch  # noqa: E402

from hzamd.env import BatchedEnv  # noqa: E402

dev = "cuda:0"


def run(envs, launches=64, warm=24):
    """hz_play through the C-ABI with prepared arguments (as bench.py's timed
    launches: env.rollout's per-call Python work would leave the GPU idle
    between 13-us launches); steps counted from per-launch output rows."""
    import ctypes
    from hzamd import _native as nat
    play = nat.lib().hz_play
    for e in envs:
        e._sync_stream()
    bufs = [(torch.zeros(launches, e.n, dtype=torch.int32, device=dev),
             torch.zeros(launches, e.n, dtype=torch.int32, device=dev)) for e in envs]
    args = [[(ctypes.c_void_p(g[i].data_ptr()), ctypes.c_void_p(s[i].data_ptr())) for i in range(launches)]
            for g, s in bufs]

    def go(i):
        for e, a in zip(envs, args):
            rc = play(e._h, 96, 0, None, None, None, a[i][0], a[i][1])
            if rc:
                raise nat.NativeError(f"hz_play failed with code {rc}")

    for i in range(warm):
        go(i % launches)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(launches):
        go(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e in envs:
        e.epoch += 1
        e.check_errors()
    return sum(int(s.sum(dtype=torch.int64)) for _, s in bufs) / dt


res = {}
for label, sizes in (("one_4096", [4096]), ("one_16384", [16384]), ("four_4096_round_robin", [4096] * 4),
                     ("one_65536", [65536]), ("sixteen_4096_round_robin", [4096] * 16)):
    envs = [BatchedEnv(n, seed_base=1_000_000 * k, device=dev) for k, n in enumerate(sizes)]
    for e in envs:
        e.set_pipeline(2)
    res[label] = run(envs, launches=128 if len(sizes) * sizes[0] <= 16384 else 32)
    print(label, round(res[label] / 1e9, 3), "G env-steps/s", flush=True)
    for e in envs:
        e.close()
    del envs
    torch.cuda.empty_cache()
print(json.dumps(res))
