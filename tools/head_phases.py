"""Phase timing of k_heads_fc from the stamped diagnostic build
(tools/libnet_diag.so, -DHZ_NET_DIAG): wave 0 of each workgroup stamps
s_memtime at kernel start, after the globals are in LDS, after the 1x1 convs,
after the policy logits, after the value sums and at the end (+ realtime at
start/end).  Prints medians in cycles and the start/end spread.
Usage (GPU box): python tools/head_phases.py [batch]"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "harmonies-alphazero_amd"))
from hzamd.infer import FoldedNet  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "libnet_diag.so"))
vp = ctypes.c_void_p
lib.hz_heads_fc.argtypes = [vp] * 13 + [ctypes.c_int32, vp, vp]
lib.hz_net_diag_stamps.argtypes = [vp]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
fn = FoldedNet(HarmoniesNet().eval().cuda())
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=torch.channels_last)
glob = torch.rand(B, 42, device="cuda", generator=g)
probs = torch.empty(B, 143, device="cuda")
value = torch.empty(B, device="cuda")
args = [x, glob, *fn.heads, *fn.fc]
for _ in range(300):
    assert lib.hz_heads_fc(*(t.data_ptr() for t in args), None, probs.data_ptr(), value.data_ptr(), B, None,
                           torch.cuda.current_stream().cuda_stream) == 0
st = np.zeros((1024, 2, 16), dtype=np.uint64)
assert lib.hz_net_diag_stamps(st.ctypes.data) == 0
nwg = min(1024, (B + 7) // 8)
s = st[:nwg, 0].astype(np.int64)
names = ["setup_glob", "conv1x1", "policy_fc", "value_fc", "softmax"]
d = np.diff(s[:, :6], axis=1)
res = {"batch": B, "workgroups": nwg, "median_cycles": {n: float(np.median(d[:, i])) for i, n in enumerate(names)},
       "total_median": float(np.median(s[:, 5] - s[:, 0]))}
res["clock_mhz_median"] = float(np.median((s[:, 5] - s[:, 0]) / np.maximum(s[:, 9] - s[:, 8], 1) * 100.0))
t0 = s[:, 0].min()
res["start_quantiles"] = [float(np.quantile(s[:, 0] - t0, q)) for q in (0, 0.5, 1)]
res["end_quantiles"] = [float(np.quantile(s[:, 5] - t0, q)) for q in (0, 0.5, 1)]
print(json.dumps(res))
