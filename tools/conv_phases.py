"""Phase timing of k_conv3x3_w8 (or, with argument 2 = x6, k_conv3x3_x6) from the stamped diagnostic build
(tools/libnet_diag.so, -DHZ_NET_DIAG): per workgroup, waves 0 and 4 stamp
s_memtime at kernel start, after the halo/map setup, after chunk 0 is in
LDS, at the end of each of the 4 chunks and after the epilogue (+ realtime
at start/end for the in-kernel clock).  Prints medians in cycles."""
import ctypes, json, os, sys
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "harmonies-alphazero_amd"))
from hzamd.infer import pack_conv3x3, pack_conv3x3_x6  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("HZ_NET_DIAG_LIB", "libnet_diag.so")))
vp = ctypes.c_void_p
lib.hz_conv3x3_bias_act.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int32, vp, vp]
lib.hz_conv3x3_x6_bias_act.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int32, vp, vp]
lib.hz_net_diag_stamps.argtypes = [vp]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
X6 = len(sys.argv) > 2 and sys.argv[2] == "x6"
NORES = len(sys.argv) > 3 and sys.argv[3] == "nores"  # the first conv of a block (no skip input)
fn = lib.hz_conv3x3_x6_bias_act if X6 else lib.hz_conv3x3_bias_act
pack = pack_conv3x3_x6 if X6 else pack_conv3x3
cl = torch.channels_last
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=cl)
w = pack(torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.05)
b = torch.randn(128, device="cuda", generator=g)
r = torch.randn(B, 128, 5, 7, device="cuda", generator=g).contiguous(memory_format=cl)
out = torch.empty_like(x)
for _ in range(200):  # ~70 ms of back-to-back launches so the clock settles
    assert fn(x.data_ptr(), w.data_ptr(), b.data_ptr(), None if NORES else r.data_ptr(), out.data_ptr(), B,
                                   None, torch.cuda.current_stream().cuda_stream) == 0
st = np.zeros((1024, 2, 16), dtype=np.uint64)
assert lib.hz_net_diag_stamps(st.ctypes.data) == 0
nwg = (B + 7) // 8
s = st[:nwg].astype(np.int64)
names = ["setup", "chunk0_stage", "chunk0", "chunk1", "chunk2", "chunk3", "epilogue"]
res = {"batch": B, "workgroups": nwg, "kernel": "k_conv3x3_x6" if X6 else "k_conv3x3_w8", "residual": not NORES}
for wv in range(2):
    d = np.diff(s[:, wv, :8], axis=1)
    res[f"wave{4 * wv}_median_cycles"] = {n: float(np.median(d[:, i])) for i, n in enumerate(names)}
    res[f"wave{4 * wv}_total_median"] = float(np.median(s[:, wv, 7] - s[:, wv, 0]))
clk = (s[:, 0, 7] - s[:, 0, 0]) / np.maximum(s[:, 0, 9] - s[:, 0, 8], 1) * 100.0  # MHz
res["clock_mhz_median"] = float(np.median(clk))
t0 = s[:, 0, 0].min()
starts = np.sort(s[:, 0, 0] - t0)
ends = np.sort(s[:, 0, 7] - t0)
res["span_cycles"] = float(ends[-1])
res["start_quantiles"] = [float(np.quantile(starts, q)) for q in (0, 0.25, 0.5, 0.75, 1)]
res["end_quantiles"] = [float(np.quantile(ends, q)) for q in (0, 0.25, 0.5, 0.75, 1)]
print(json.dumps(res))
