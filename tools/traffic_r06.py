"""profiles/r06/traffic.json: HBM bytes per launch from two rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE: each its own run of the same command) and
each kernel's mean duration from a kernel-trace pass of that command, for
the kernels bench.py prices: k_play2 (config 2), k_rollout<true, false>
(the auto-reset leg), k_x6w4_tower<true> (the leaf-eval tower) and
k_expand_backup<4, true, true, 16, false> (the tree).  Bytes = (2 x FETCH_SIZE +
WRITE_SIZE) x 1024: on gfx950 FETCH_SIZE counts half the bytes of wide
streaming reads (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact.

usage: python tools/traffic_r06.py <pass dir with p0 (trace) p1 p2 (pmc)> <out.json>
"""
import collections
import csv
import glob
import json
import os
import re
import sys

KERNELS = ("k_play2", "k_rollout<true, false>", "k_x6w4_tower<true>", "k_expand_backup<4, true, true, 16, false>")


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"([A-Za-z0-9_]+(<[^()]*>)?)", name.strip())
    return m.group(1) if m else name


def main(root, out_path):
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, counter) -> dispatch -> sum
    for f in sorted(glob.glob(os.path.join(root, "p[12]", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            cnt[(short(r["Kernel_Name"]), r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(os.path.join(root, "p0", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Name"])] = (float(r["AverageNs"]), int(r["Calls"]))
    out = {"source": root, "correction": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950: FETCH_SIZE counts "
                                          "half of wide streaming reads)", "kernels": {}}
    for k in KERNELS:
        f, w = cnt.get((k, "FETCH_SIZE")), cnt.get((k, "WRITE_SIZE"))
        if not f or not w:
            continue
        fk = sum(f.values()) / len(f)
        wk = sum(w.values()) / len(w)
        b = (2 * fk + wk) * 1024
        e = {"FETCH_SIZE_kB": fk, "WRITE_SIZE_kB": wk, "bytes_per_launch": b, "dispatches_counted": len(f)}
        if k in dur:
            ns, calls = dur[k]
            e.update({"mean_ns": ns, "trace_calls": calls, "GBps": b / ns, "frac_of_8TBps": b / ns / 8000.0})
        out["kernels"][k] = e
    # bench.py's older key for the config-2 kernel
    if "k_play2" in out["kernels"]:
        out["k_play2_bytes_per_launch"] = out["kernels"]["k_play2"]["bytes_per_launch"]
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
