"""canon_key_child == canon_key over whole games (tools/key_check.hip).

Plays 4096 boards from reset to the end with the build's action rule and,
at every ply, checks the child key of every legal action of every board in
both key forms.  Prints one JSON line: pairs checked, mismatches.
    make -C tools libkeycheck.so && python tools/key_check.py
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "harmonies-alphazero_amd"))
from hzamd.env import BatchedEnv  # noqa: E402


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libkeycheck.so"))
    n = int(os.environ.get("HZ_KC_BOARDS", "4096"))
    env = BatchedEnv(n, seed_base=12345)
    env.reset()
    out = torch.zeros(3, dtype=torch.int64, device="cuda")
    plies = 0
    while not bool(env.done().all()):
        st = env.export_state().contiguous()
        torch.cuda.synchronize()
        if lib.hz_key_check(ctypes.c_void_p(st.data_ptr()), n, ctypes.c_void_p(out.data_ptr())):
            raise SystemExit("hz_key_check failed")
        env.rule_ply()
        plies += 1
    torch.cuda.synchronize()
    r = {"boards": n, "plies": plies, "pairs": int(out[0]), "mismatch": int(out[1]), "step_fail": int(out[2])}
    print(json.dumps(r))
    if r["mismatch"] or r["step_fail"] or not r["pairs"]:
        raise SystemExit(1)


if __name__ == "__main__":
    main()
