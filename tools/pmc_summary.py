"""Summarise rocprofv3 --pmc CSVs: per kernel, mean per dispatch of each counter."""
import csv, sys, collections, json, glob, os, re
root = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        name = re.sub(r"<.*>", "", name).replace("void ", "").strip()  # k_rollout<false, false> -> k_rollout
        res[name][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
out = {}
for k, d in res.items():
    per = collections.defaultdict(list)
    for (c, disp), vals in d.items():
        per[c].append(sum(vals))   # sum over dimensions (XCD/SE instances) per dispatch
    out[k] = {c: sum(v) / len(v) for c, v in per.items()}
print(json.dumps(out, indent=1))
