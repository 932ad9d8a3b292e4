"""Per-kernel dispatch statistics from a rocprofv3 SQLite output (the
rocpd_*.db this image's rocprofv3 writes by default): n, mean, median, p90
in microseconds, name-filtered.  Usage: python tools/db_stats.py file.db [substr]"""
import json
import sqlite3
import sys


def stats(path, sub=""):
    c = sqlite3.connect(path)
    rows = c.execute("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    by = {}
    for name, dur in rows:
        if sub in name:
            by.setdefault(name, []).append(dur / 1e3)
    out = {}
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        out[name] = {"n": len(v), "mean_us": sum(v) / len(v), "median_us": v[len(v) // 2],
                     "p90_us": v[int(0.9 * (len(v) - 1))], "total_ms": sum(v) / 1e3}
    return out


if __name__ == "__main__":
    print(json.dumps(stats(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""), indent=1))
