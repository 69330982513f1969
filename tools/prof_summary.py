#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace database (rocpd SQLite):
python tools/prof_summary.py <dir or .db> [--json out.json]"""
import glob
import json
import os
import sqlite3
import sys


def summary(path):
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = {}
    for d in dbs:
        c = sqlite3.connect(d)
        for name, n, tot, mn, mx in c.execute(
                "select name, count(*), sum(end-start), min(end-start), max(end-start) from kernels group by name"):
            r = rows.setdefault(name, [0, 0, float("inf"), 0])
            r[0] += n
            r[1] += tot
            r[2] = min(r[2], mn)
            r[3] = max(r[3], mx)
    out = [{"kernel": k, "calls": v[0], "total_us": round(v[1] / 1e3, 1), "avg_us": round(v[1] / v[0] / 1e3, 2),
            "min_us": round(v[2] / 1e3, 2), "max_us": round(v[3] / 1e3, 2)} for k, v in rows.items()]
    return sorted(out, key=lambda r: -r["total_us"])


if __name__ == "__main__":
    s = summary(sys.argv[1])
    for r in s:
        print(f"{r['calls']:6d} {r['avg_us']:10.2f} {r['min_us']:10.2f} {r['max_us']:10.2f}  {r['kernel'][:90]}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(s, f, indent=1)
