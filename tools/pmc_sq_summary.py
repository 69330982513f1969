#!/usr/bin/env python3
"""Per-kernel sums of every PMC counter found under a directory of rocprofv3
--pmc CSV passes (tools/pmc_snappy_sorted.sh): one JSON object per kernel,
counters summed over its dispatches, dispatch count, and -- where present --
HBM bytes (2 x FETCH_SIZE: gfx950 reports half of a streaming read,
MI355X_MICROARCH.md) and WRITE_SIZE, in bytes.
    python tools/pmc_sq_summary.py DIR [--json out.json]"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if "psf::" not in k:
                continue
            name = k.replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add((path, r.get("Dispatch_Id")))
    out = {}
    for name, c in tot.items():
        d = dict(c)
        if "FETCH_SIZE" in d:
            d["read_bytes"] = 2 * 1024 * d.pop("FETCH_SIZE")
        if "WRITE_SIZE" in d:
            d["write_bytes"] = 1024 * d.pop("WRITE_SIZE")
        d["dispatch_records"] = len(disp[name])
        out[name] = d
    s = json.dumps(out, indent=1, sort_keys=True)
    print(s)
    if a.json:
        open(a.json, "w").write(s)


if __name__ == "__main__":
    main()
