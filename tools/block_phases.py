"""Phase timing of the fused residual block (k_conv3x3_x6w4<true>) from the
stamped diagnostic build (tools/libnet_diag.so, -DHZ_NET_DIAG): wave 0 of
every workgroup stamps s_memtime after the setup, chunk 0's staging, each of
conv1's chunks, the switch between the convs, each of conv2's chunks and the
epilogue (+ realtime at start/end for the in-kernel clock).  Prints medians
in cycles, and the layered conv's phases from the same build for comparison.
Usage (GPU box): python tools/block_phases.py [batch]"""
import ctypes, json, os, sys
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "harmonies-alphazero_amd"))
from hzamd.infer import pack_conv3x3_x6  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("HZ_NET_DIAG_LIB", "libnet_diag.so")))
vp = ctypes.c_void_p
lib.hz_conv3x3_x6_bias_act.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int32, vp, vp]
lib.hz_resblock_x6_bias_act.argtypes = [vp] * 7 + [ctypes.c_int32, vp, vp]
lib.hz_net_diag_stamps.argtypes = [vp]
assert lib.hz_resblock_x6_set_fused(1) == 0
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cl = torch.channels_last
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(B, 128, 5, 7, device="cuda", generator=g).relu().contiguous(memory_format=cl)
p1 = pack_conv3x3_x6(torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.03)
p2 = pack_conv3x3_x6(torch.randn(128, 128, 3, 3, device="cuda", generator=g) * 0.03)
b1 = torch.randn(128, device="cuda", generator=g) * 0.1
b2 = torch.randn(128, device="cuda", generator=g) * 0.1
out, tmp = torch.empty_like(x), torch.empty_like(x)
sp = torch.cuda.current_stream().cuda_stream
nwg = (B + 7) // 8


def stamps():
    st = np.zeros((1024, 2, 16), dtype=np.uint64)
    assert lib.hz_net_diag_stamps(st.ctypes.data) == 0
    return st[:nwg, 0].astype(np.int64)


def med(a):
    return float(np.median(a))


res = {"batch": B, "lib": os.environ.get("HZ_NET_DIAG_LIB", "libnet_diag.so")}
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for i in range(200):
    if i == 50:
        ev0.record()
    assert lib.hz_resblock_x6_bias_act(x.data_ptr(), p1.data_ptr(), b1.data_ptr(), p2.data_ptr(), b2.data_ptr(),
                                       out.data_ptr(), tmp.data_ptr(), B, None, sp) == 0
ev1.record()
torch.cuda.synchronize()
res["fused_us_per_launch"] = ev0.elapsed_time(ev1) * 1e3 / 150
s = stamps()
# workgroup timeline of the last launch in us (s_memrealtime: 100 MHz)
rt0, rt1 = s[:, 8].astype(np.float64), s[:, 9].astype(np.float64)
base = rt0.min()
st, en = (rt0 - base) / 100.0, (rt1 - base) / 100.0
o = np.argsort(st)
r1, r2 = o[:256], o[256:]
res["timeline_us"] = {"round1_start_max": float(st[r1].max()), "round1_end_med": float(np.median(en[r1])),
                      "round1_end_max": float(en[r1].max()),
                      "round2_start_min": float(st[r2].min()) if len(r2) else None,
                      "round2_start_med": float(np.median(st[r2])) if len(r2) else None,
                      "round2_end_med": float(np.median(en[r2])) if len(r2) else None,
                      "span": float(en.max())}
order = [0, 1, 2, 3, 4, 5, 6, 10, 11, 12, 13, 14, 7]
names = ["setup", "chunk0_stage", "conv1_chunk0", "conv1_chunk1", "conv1_chunk2", "conv1_chunk3", "switch",
         "conv2_chunk0", "conv2_chunk1", "conv2_chunk2", "conv2_chunk3", "epilogue"]
res["fused_cycles"] = {n: med(s[:, order[i + 1]] - s[:, order[i]]) for i, n in enumerate(names)}
res["fused_total"] = med(s[:, 7] - s[:, 0])
res["fused_clock_mhz"] = med((s[:, 7] - s[:, 0]) / np.maximum(s[:, 9] - s[:, 8], 1) * 100.0)
# MFMA issue cycles per wave of one fused block: 2 convs x (66 block-taps of
# the wave's row half x 4 column blocks x 4 chunks x 6 bf16 products) x 16
# cycles (v_mfma_f32_16x16x32_bf16, MI355X_MICROARCH.md constants) = the
# SQ_VALU_MFMA_BUSY_CYCLES count per wave; busy = that over the workgroup's
# in-kernel cycles (setup to epilogue end), at the clock measured alongside
res["mfma_cycles_per_wave"] = 2 * 66 * 4 * 4 * 6 * 16
res["fused_mfma_busy"] = res["mfma_cycles_per_wave"] / res["fused_total"]
res["row_table"] = os.environ.get("HZ_BLK_TABLE", "1 (default)")
for _ in range(200):
    assert lib.hz_conv3x3_x6_bias_act(x.data_ptr(), p1.data_ptr(), b1.data_ptr(), x.data_ptr(), out.data_ptr(), B,
                                      None, sp) == 0
s = stamps()
names = ["setup", "chunk0_stage", "chunk0", "chunk1", "chunk2", "chunk3", "epilogue"]
res["layered_res_cycles"] = {n: med(s[:, i + 1] - s[:, i]) for i, n in enumerate(names)}
res["layered_res_total"] = med(s[:, 7] - s[:, 0])
res["layered_clock_mhz"] = med((s[:, 7] - s[:, 0]) / np.maximum(s[:, 9] - s[:, 8], 1) * 100.0)
print(json.dumps(res))
