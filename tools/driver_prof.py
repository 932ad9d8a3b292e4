"""Per-dispatch summary of a rocprofv3 kernel trace of the driver's own bench
command (the roofline must be reproducible from
profiles/).

usage: driver_prof.py <run_kernel_trace.csv> <run_kernel_stats.csv> <bench.json> <out.json> [untraced_bench.json]

(bench.json: the line the traced run printed; untraced_bench.json: the same
command's line without the profiler, whose event-timed kernel_ms carries no
tracer overhead: the profile's median is checked against both)

For every kernel of interest: dispatch count, mean, median, 10 % trimmed mean
(the middle 80 % of dispatches), p90, p99 and max in us, next to rocprofv3's
own AverageNs.  For the headline kernel (`roofline.kernel` of the line) it
checks that 256 x median fits the same run's ms_per_step, and recomputes the
line's `frac` from the profile's median and trimmed mean (algorithmic bytes
per launch / duration / peak)."""
import csv
import json
import sys

import numpy as np

KEEP = ("k_play2", "k_rollout", "k_conv3x3_x6w4", "k_conv3x3_x6<", "k_stem", "k_heads_fc", "k_expand_backup",
        "k_select", "k_gather_encode", "k_ply", "k_legal", "k_step", "k_rule", "k_score", "k_tower_x6", "k_x6w4_tower")
# the full-batch leaf-eval forward: the residual tower in one launch, the stem, the fused head
# (the stem: 4-state workgroups since round 6, 8 before; whichever ran)
NN_KERNELS = ("k_x6w4_tower<true>", ("k_conv3x3_x6<2, true, 4, 2>", "k_conv3x3_x6<2, true, 8, 2>"), "k_heads_fc")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("hz::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].strip()


def summ(x):
    x = np.sort(np.asarray(x, dtype=np.float64))
    k = len(x) // 10
    t = x[k:len(x) - k] if len(x) > 2 * k else x
    q = np.percentile(x, [50, 90, 99])
    return {"n": int(x.size), "mean_us": float(x.mean()), "median_us": float(q[0]), "trimmed_mean_us": float(t.mean()),
            "p90_us": float(q[1]), "p99_us": float(q[2]), "max_us": float(x.max()), "min_us": float(x.min())}


def main():
    trace, kstats, bench_p, out_p = sys.argv[1:5]
    per = {}
    with open(trace) as f:
        for r in csv.DictReader(f):
            n = short(r["Kernel_Name"])
            if any(n.startswith(k) for k in KEEP):
                per.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rp = {}
    with open(kstats) as f:
        for r in csv.DictReader(f):
            rp[short(r["Name"])] = {"avg_us": float(r["AverageNs"]) / 1e3, "calls": int(r["Calls"])}
    kernels = {n: dict(summ(v), rocprof_avg_us=rp.get(n, {}).get("avg_us")) for n, v in per.items()}
    out = {"kernels": kernels}
    try:
        line = json.loads(open(bench_p).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        line = None
    if line:
        rf = line["roofline"]
        kn = rf.get("kernel", "k_play2")
        k = kernels.get(kn)
        lpstep = line["config"].get("launches_per_step", 256)
        chk = {"kernel": kn, "ms_per_step": line["ms_per_step"], "launches_per_step": lpstep,
               "line_kernel_ms": rf.get("kernel_ms"), "line_frac": rf["frac"]}
        if k:
            alg = rf["alg_bytes_per_launch"]
            for key in ("median_us", "trimmed_mean_us", "mean_us"):
                chk["launches_x_" + key + "_ms"] = lpstep * k[key] / 1e3
                chk["frac_from_" + key] = alg / (k[key] * 1e-6) / (rf["peak"] * 1e9)
            chk["fits_ms_per_step_median"] = lpstep * k["median_us"] / 1e3 <= line["ms_per_step"]
            chk["frac_rel_diff_median"] = abs(chk["frac_from_median_us"] / rf["frac"] - 1)
        out["driver_line_check"] = chk
        sp = line.get("selfplay") or {}
        if sp:
            out["selfplay_line"] = {k2: sp.get(k2) for k2 in ("games_per_s", "ms_per_move", "nn_ms_per_move",
                                                              "tree_ms_per_move")}
            nr = sp.get("nn_roofline") or {}
            out["selfplay_line"]["nn_roofline_frac"] = nr.get("frac")
            # the same roofline from the profile: the forward's kernels'
            # median dispatches (most dispatches are full 4,096-row batches)
            found = [next((a for a in (kn2 if isinstance(kn2, tuple) else (kn2,)) if a in kernels), None)
                     for kn2 in NN_KERNELS]
            if nr.get("flop_per_eval") and all(found):
                fwd_us = sum(kernels[kn2]["median_us"] for kn2 in found)
                rows = sp.get("boards") or 4096
                out["selfplay_line"]["nn_forward_us_from_median"] = fwd_us
                out["selfplay_line"]["nn_roofline_frac_from_median"] = (
                    nr["flop_per_eval"] * rows / (fwd_us * 1e-6) / (nr["peak"] * 1e12))
    if len(sys.argv) > 5 and "driver_line_check" in out:
        try:
            ul = json.loads(open(sys.argv[5]).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            ul = None
        k = kernels.get(out["driver_line_check"]["kernel"])
        if ul and k:
            rf = ul["roofline"]
            lpstep = ul["config"].get("launches_per_step", 256)
            fm = rf["alg_bytes_per_launch"] / (k["median_us"] * 1e-6) / (rf["peak"] * 1e9)
            out["untraced_line_check"] = {
                "ms_per_step": ul["ms_per_step"], "line_kernel_ms": rf.get("kernel_ms"), "line_frac": rf["frac"],
                "launches_x_median_us_ms": lpstep * k["median_us"] / 1e3,
                "fits_ms_per_step_median": lpstep * k["median_us"] / 1e3 <= ul["ms_per_step"],
                "frac_from_median_us": fm, "frac_rel_diff_median": abs(fm / rf["frac"] - 1)}
            nr = (ul.get("selfplay") or {}).get("nn_roofline") or {}
            if "nn_roofline_frac_from_median" in out.get("selfplay_line", {}) and nr.get("frac"):
                out["untraced_line_check"]["nn_roofline_frac"] = nr["frac"]
                out["untraced_line_check"]["nn_frac_rel_diff"] = abs(
                    out["selfplay_line"]["nn_roofline_frac_from_median"] / nr["frac"] - 1)
    json.dump(out, open(out_p, "w"), indent=1)
    for n, k in sorted(kernels.items(), key=lambda t: -t[1]["n"] * t[1]["mean_us"]):
        print(f"{n[:44]:44s} n={k['n']:7d} mean={k['mean_us']:8.2f} med={k['median_us']:8.2f} "
              f"trim={k['trimmed_mean_us']:8.2f} p99={k['p99_us']:8.2f} max={k['max_us']:9.2f}")
    if "driver_line_check" in out:
        print(json.dumps(out["driver_line_check"]))


if __name__ == "__main__":
    main()
