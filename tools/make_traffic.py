"""profiles/<round>_traffic.json from a PMC summary: HBM bytes per launch of
the hz_play kernel (k_rollout, or k_play2 for pipeline 2) = (2 x FETCH_SIZE
+ WRITE_SIZE) x 1024 (gfx950: FETCH_SIZE reads half the bytes of wide
streaming reads, MI355X_MICROARCH.md §HBM).  bench.py reads the key
'<kernel>_bytes_per_launch'."""
import json, sys
summ = json.load(open(sys.argv[1]))
out = {"source": sys.argv[1], "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount)"}
for name in ("k_rollout", "k_play2"):
    k = summ.get(name)
    if k and "FETCH_SIZE" in k and "WRITE_SIZE" in k:
        out[f"{name}_bytes_per_launch"] = (2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024
        out[f"{name}_FETCH_SIZE_kB"] = k["FETCH_SIZE"]
        out[f"{name}_WRITE_SIZE_kB"] = k["WRITE_SIZE"]
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(out)
