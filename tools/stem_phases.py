"""Phase timing of the eight-state x6 stem (k_conv3x3_x6<2, true, 8, 2>) from
the stamped diagnostic build (tools/libnet_diag.so): per workgroup, wave 0's
s_memtime at start, after the setup, after chunk 0's staging, after chunk 0
(with chunk 1 staged), after the tap-packed chunk 1 and after the epilogue.
Prints medians in cycles (encoder-like boards at the leaf-eval batch).
Usage (GPU box): python tools/stem_phases.py [batch]"""
import ctypes, json, os, sys
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "harmonies-alphazero_amd"))
from hzamd.infer import pack_stem_x6  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("HZ_NET_DIAG_LIB", "libnet_diag.so")))
vp = ctypes.c_void_p
lib.hz_stem3x3_x6_bias_act.argtypes = [vp, vp, vp, vp, ctypes.c_int32, vp, vp]
lib.hz_net_diag_stamps.argtypes = [vp]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
g = torch.Generator(device="cuda").manual_seed(0)
board = (torch.rand(B, 38, 5, 7, device="cuda", generator=g) > 0.8).float()
board[:, 37] = 2.0 / 3.0
w = pack_stem_x6(torch.randn(128, 38, 3, 3, device="cuda", generator=g) * 0.1)
b = torch.randn(128, device="cuda", generator=g) * 0.1
out = torch.empty(B, 128, 5, 7, device="cuda").contiguous(memory_format=torch.channels_last)
for _ in range(300):
    assert lib.hz_stem3x3_x6_bias_act(board.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), B, None,
                                      torch.cuda.current_stream().cuda_stream) == 0
st = np.zeros((1024, 2, 16), dtype=np.uint64)
assert lib.hz_net_diag_stamps(st.ctypes.data) == 0
s = st[:(B + 7) // 8, 0].astype(np.int64)
pairs = [("setup", 0, 1), ("chunk0_stage", 1, 2), ("chunk0", 2, 3), ("chunk1_packed", 3, 4), ("epilogue", 4, 7)]
res = {"batch": B, "median_cycles": {n: float(np.median(s[:, j] - s[:, i])) for n, i, j in pairs},
       "total_median": float(np.median(s[:, 7] - s[:, 0])),
       "clock_mhz_median": float(np.median((s[:, 7] - s[:, 0]) / np.maximum(s[:, 9] - s[:, 8], 1) * 100.0))}
print(json.dumps(res))
