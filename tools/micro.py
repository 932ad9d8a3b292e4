"""Time device-rule microbenchmarks (tools/micro.hip) at 4096 lanes."""
import ctypes, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libmicro.so"))
vp = ctypes.c_void_p
L.micro_run.argtypes = [ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp]
n = 4096
dev = "cuda"
mt = torch.zeros(n, 624, dtype=torch.int32, device=dev)
cur = torch.full((n,), 624 | (624 << 16), dtype=torch.int32, device=dev)
sink = torch.zeros(n, dtype=torch.int32, device=dev)
pl = torch.randint(0, 2**62, (4, n), dtype=torch.int64, device=dev)
seeds = torch.arange(n, dtype=torch.int64, device=dev)
stream = vp(torch.cuda.current_stream().cuda_stream)
P = lambda t: vp(t.data_ptr())

def timeit(which, a, b, reps):
    L.micro_run(which, a, b, n, reps, P(sink), stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); L.micro_run(which, a, b, n, reps, P(sink), stream); e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3

res = {}
L.micro_run(3, P(mt), None, n, 0, P(sink), stream)  # seed streams
res["seed_global_us"] = timeit(3, P(mt), None, 0)
res["seed_lds_us"] = timeit(4, P(mt), None, 0)
for reps in (16, 64):
    res[f"next_x{reps}_us"] = timeit(1, P(mt), P(cur), reps)
    res[f"draws_x{reps}_us"] = timeit(0, P(mt), P(cur), reps)
    res[f"score_x{reps}_us"] = timeit(2, P(pl), None, reps)
    res[f"pick_x{reps}_us"] = timeit(5, P(seeds), None, reps)
print(json.dumps(res))

L.micro_draws_lds.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, ctypes.c_int]
cyc = torch.zeros(n // 64, dtype=torch.int64, device=dev)
names = {0: "draw_fresh", 1: "draw_pretwisted", 2: "scan_only", 3: "draw_pile_only", 4: "prefetch_only"}
for mode, name in names.items():
    for reps in (1, 33):  # 33 draws stay inside the 224 pre-twisted words
        L.micro_draws_lds(P(mt), n, reps, P(sink), P(cyc), stream, mode)
        torch.cuda.synchronize()
        res[f"lds_{name}_x{reps}_cyc"] = float(cyc.double().mean())
    res[f"lds_{name}_per_draw_cyc"] = (res[f"lds_{name}_x33_cyc"] - res[f"lds_{name}_x1_cyc"]) / 32
print(json.dumps(res))

# turn-structured play (k_rollout's fast path), cycles per pair of turns
L.micro_turns.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, vp]
for mode, name in {0: "turns", 1: "turns_nohash"}.items():
    for pairs in (1, 17):
        L.micro_turns(mode, n, pairs, P(sink), P(cyc), stream)
        torch.cuda.synchronize()
        res[f"{name}_x{pairs}_cyc"] = float(cyc.double().mean())
    res[f"{name}_per_pair_cyc"] = (res[f"{name}_x17_cyc"] - res[f"{name}_x1_cyc"]) / 16
print(json.dumps(res))
