#!/usr/bin/env python3
"""Per-kernel HBM traffic from two rocprofv3 PMC passes (CSV output).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d D/fetch -o run -- <cmd>
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d D/write -o run -- <cmd>
    python tools/pmc_summary.py D/fetch D/write [--alg 'snappy_compress_frags=268435456' ...]
        [--only psf::] [--json out.json]

Correction (MI355X_MICROARCH.md, HBM / rocprofv3): on gfx950 FETCH_SIZE
reports half the bytes of a coalesced streaming read, so read bytes =
2 x FETCH_SIZE (KiB); WRITE_SIZE is taken as reported.  `--alg name=bytes`
gives a kernel's algorithmic bytes per launch (substring of its name), and the
summary then carries traffic / algorithmic.
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = collections.defaultdict(list)
    for path in files:
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != counter:
                continue
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--alg", action="append", default=[])
    ap.add_argument("--only", default="psf::")
    ap.add_argument("--json")
    a = ap.parse_args()
    alg = dict(kv.split("=", 1) for kv in a.alg)
    fv, wv = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    out = []
    for name in sorted(set(fv) | set(wv)):
        if a.only and a.only not in name:
            continue
        f, w = fv.get(name, []), wv.get(name, [])
        fetch = sum(f) / len(f) if f else None
        write = sum(w) / len(w) if w else None
        rec = {"kernel": name[:160], "launches": max(len(f), len(w)),
               "read_bytes_per_launch": round(2 * fetch) if fetch is not None else None,
               "write_bytes_per_launch": round(write) if write is not None else None}
        if fetch is not None and write is not None:
            rec["hbm_bytes_per_launch"] = round(2 * fetch + write)
            for key, b in alg.items():
                if key in name:
                    rec["alg_bytes_per_launch"] = float(b)
                    rec["traffic_over_alg"] = round((2 * fetch + write) / float(b), 4)
        out.append(rec)
    for r in out:
        print(json.dumps(r))
    if a.json:
        json.dump({"correction": "read = 2 x FETCH_SIZE (gfx950 streaming-read calibration), write = WRITE_SIZE",
                   "kernels": out}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
