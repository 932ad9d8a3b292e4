"""Phase timing of k_tower_x6_split (config 1's one-board tower) from the
stamped diagnostic build (tools/libnet_diag.so, -DHZ_NET_DIAG): thread 0 of
each of state 0's 8 workgroups stamps s_memtime per conv at: conv start,
K-loop done (MFMAs issued and retired up to the epilogue), payload stores
drained, hand-off counter seen complete, next input loaded + staged, barrier.
Prints per-phase medians (cycles) over convs 1..nconv-2 and workgroups.
Usage (GPU box): python tools/split_phases.py [batch]"""
import ctypes, json, os, sys
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "harmonies-alphazero_amd"))
from hzamd.infer import FoldedNet  # noqa: E402
from hzamd.net import HarmoniesNet  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("HZ_NET_DIAG_LIB", "libnet_diag.so")))
vp = ctypes.c_void_p
lib.hz_tower_x6_split.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp]
lib.hz_net_diag_split_stamps.argtypes = [vp]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
torch.manual_seed(0)
f = FoldedNet(HarmoniesNet().eval().cuda())
allw, allb = f.resident
nconv = allw.shape[0]
x = torch.randn(B, 128, 5, 7, device="cuda").relu().contiguous(memory_format=torch.channels_last)
out = torch.empty_like(x)
xch = torch.empty(2 * B * 35 * 128, device="cuda")
sync = torch.zeros(33 * 32, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for _ in range(300):
    assert lib.hz_tower_x6_split(x.data_ptr(), allw.data_ptr(), allb.data_ptr(), out.data_ptr(), xch.data_ptr(),
                                 sync.data_ptr(), nconv, B, None, st) == 0
torch.cuda.synchronize()
assert int(sync[32 * 32].item()) == 0 and not sync.any().item(), "hand-off timed out or counters left set"
s = np.zeros((8, 64, 6), dtype=np.uint64)
assert lib.hz_net_diag_split_stamps(s.ctypes.data) == 0
s = s[:, :nconv].astype(np.int64)
names = ["kloop", "store_drain", "handoff_wait", "load_stage", "barrier"]
mid = s[:, 1:nconv - 1]
res = {"batch": B, "nconv": nconv, "median_cycles": {}}
for k, nm in enumerate(names):
    res["median_cycles"][nm] = float(np.median(mid[:, :, k + 1] - mid[:, :, k]))
res["median_cycles"]["conv_total"] = float(np.median(mid[:, :, 5] - mid[:, :, 0]))
res["median_cycles"]["conv_start_to_next_start"] = float(np.median(s[:, 2:nconv - 1, 0] - s[:, 1:nconv - 2, 0]))
res["whole_tower_cycles_group0"] = int(s[0, nconv - 1, 1] - s[0, 0, 0])
print(json.dumps(res))
