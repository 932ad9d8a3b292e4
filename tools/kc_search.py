"""The reference-fixture searches (tests/test_mcts_gpu.py) on the HZ_KEYCHECK
build (tools/libhz_kc.so): every expansion child's key is compared with
canon_key of its state in-kernel.  Prints the counters and per-fixture tree
sizes against the reference's.
    make -C tools libhz_kc.so && python tools/kc_search.py
"""
import ctypes
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HZ_LIB"] = os.path.join(ROOT, "tools", "libhz_kc.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "harmonies-alphazero_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_mcts_gpu import load, make_env  # noqa: E402


def main():
    from hzamd.mcts import BatchedMCTS, stub_evaluator
    import hzamd._native as nat
    f = load("mcts.npz")
    groups = defaultdict(list)
    for k in range(len(f["sims"])):
        groups[(int(f["sims"][k]), float(f["cpuct"][k]), int(f["testing"][k]), float(f["eps"][k]))].append(k)
    diffs = []
    for (sims, cpuct, testing, eps), ks in groups.items():
        env = make_env(f["state"][ks], f["mt_seed"][ks])
        mcts = BatchedMCTS(env, sims)
        noise = torch.from_numpy(np.ascontiguousarray(f["noise"][ks][:, :69]))
        mcts.search(stub_evaluator, cpuct, noise=noise, eps=eps, testing=bool(testing))
        counts = mcts.stats().cpu().numpy()
        for j, k in enumerate(ks):
            if counts[j, 0] != f["n_nodes"][k] or counts[j, 1] != f["n_edges"][k]:
                diffs.append([int(k), int(counts[j, 0]), int(f["n_nodes"][k]), int(counts[j, 1]), int(f["n_edges"][k])])
        mcts.close()
        env.close()
    c = (ctypes.c_ulonglong * 3)()
    nat.lib().hz_keycheck_counts(c)
    print(json.dumps({"child_key_mismatch": c[0], "leaf_key_mismatch": c[1], "children": c[2],
                      "tree_size_diffs": diffs[:20], "n_diffs": len(diffs)}))


if __name__ == "__main__":
    main()
