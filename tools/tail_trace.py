"""The tower kernels' per-dispatch durations in a complete-game self-play leg,
by live-row count (where does rocprof's tail come from?).

usage: tail_trace.py <run_kernel_trace.csv> <calls.json> <run_kernel_stats.csv> <out.json> [<out.json.gz>]

calls.json is bench.py's per-call dump (HZ_BENCH_CALL_DUMP): the live rows
and HIP-event milliseconds of every leaf-evaluation call of the game leg, in
order.  The trace's dispatches are cut into forwards at each head kernel
(k_heads_fc / k_heads_fc1 end every forward), and the last len(calls)
forwards are the game leg's calls, in the same order.  For every tower
kernel the summary gives the dispatch count, mean, standard deviation (numpy,
over the trace) next to the StdDev column of rocprofv3's own stats file, and
percentiles; per live-row bucket it gives the fused residual block's
durations and the call times."""
import csv
import gzip
import json
import sys

import numpy as np

TOWER = ("k_conv3x3_x6w4", "k_conv3x3_x6<", "k_tower_x6_resident", "k_tower_x6_split", "k_heads_fc")
BUCKETS = [0, 32, 256, 768, 1024, 2048, 3072, 4096]


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("hz::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].strip()


def stats(x):
    x = np.asarray(x, dtype=np.float64)
    if not x.size:
        return None
    q = np.percentile(x, [50, 90, 99, 99.9])
    return {"n": int(x.size), "mean_us": float(x.mean()), "sd_us": float(x.std()), "p50_us": float(q[0]),
            "p90_us": float(q[1]), "p99_us": float(q[2]), "p999_us": float(q[3]), "max_us": float(x.max()),
            "min_us": float(x.min())}


def main():
    trace, calls_p, kstats, out_p = sys.argv[1:5]
    gz_p = sys.argv[5] if len(sys.argv) > 5 else None
    disp = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            disp.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    disp.sort()
    calls = json.load(open(calls_p))
    rows, call_ms = calls["rows"], calls["ms"]
    per_kernel = {}
    for s, e, n in disp:
        if any(n.startswith(t) for t in TOWER):
            per_kernel.setdefault(n, []).append((e - s) / 1e3)
    rp = {}
    with open(kstats) as f:
        for r in csv.DictReader(f):
            rp[short(r["Name"])] = {"avg_us": float(r["AverageNs"]) / 1e3, "stddev_col_us": float(r["StdDev"]) / 1e3,
                                    "max_us": float(r["MaxNs"]) / 1e3, "calls": int(r["Calls"])}
    kernels = {n: {"trace": stats(v), "rocprof_stats": rp.get(n)} for n, v in per_kernel.items()}
    # forwards: dispatches up to and including each head kernel
    fwds, cur = [], []
    for s, e, n in disp:
        if any(n.startswith(t) for t in TOWER):
            cur.append((n, (e - s) / 1e3))
        if n.startswith("k_heads_fc"):
            fwds.append(cur)
            cur = []
    game = fwds[-len(rows):] if len(fwds) >= len(rows) else None
    by_rows = []
    if game is not None:
        for lo, hi in zip(BUCKETS[:-1], BUCKETS[1:]):
            idx = [i for i, r in enumerate(rows) if lo < r <= hi]
            if not idx:
                continue
            blk = [d for i in idx for n, d in game[i] if n.startswith("k_conv3x3_x6w4")]
            tower = [sum(d for n, d in game[i] if not n.startswith("k_heads_fc")) for i in idx]
            by_rows.append({"rows": [lo + 1, hi], "calls": len(idx), "call_ms": stats([call_ms[i] * 1e3 for i in idx]),
                            "fused_block_us": stats(blk), "tower_kernels_sum_us": stats(tower)})
    out = {"dispatches": len(disp), "forwards_in_trace": len(fwds), "game_calls": len(rows),
           "matched": game is not None, "kernels": kernels, "by_live_rows": by_rows,
           "call_ms_all": stats(np.array(call_ms) * 1e3),
           "note": "durations in us; sd_us is numpy's over the trace's dispatches, stddev_col_us the StdDev "
                   "column of rocprofv3's kernel_stats for the same kernel"}
    json.dump(out, open(out_p, "w"), indent=1)
    if gz_p and game is not None:
        with gzip.open(gz_p, "wt") as f:
            json.dump({"rows": rows, "call_ms": call_ms,
                       "dispatches_us": [[round(d, 2) for _, d in g] for g in game],
                       "names": sorted({n for g in game for n, _ in g})}, f)
    for n, k in kernels.items():
        t, r = k["trace"], k["rocprof_stats"] or {}
        print(f"{n[:48]:48s} n={t['n']:7d} mean={t['mean_us']:8.1f} sd={t['sd_us']:7.1f} max={t['max_us']:8.1f}"
              f"  rocprof avg={r.get('avg_us', 0):8.1f} StdDev={r.get('stddev_col_us', 0):8.1f}")
    for b in by_rows:
        fb = b["fused_block_us"]
        print(b["rows"], b["calls"], "call p50 %.0f us" % b["call_ms"]["p50_us"],
              "block mean %.1f sd %.1f max %.1f" % (fb["mean_us"], fb["sd_us"], fb["max_us"]) if fb else "")


if __name__ == "__main__":
    main()
