"""Turn rocprofv3 PMC passes into per-launch HBM traffic for profiles/.

    python tools/pmc_traffic.py --fetch gpurun_out/pmc/r01_fetch_counter_collection.csv \
        --write gpurun_out/pmc/r01_write_counter_collection.csv --n 134217728 --nb 1 \
        --out profiles/pmc_traffic.json --trim profiles/r01

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports exactly half
the bytes of a coalesced streaming read, so read bytes = 2 * FETCH_SIZE KiB;
WRITE_SIZE is taken as reported.  The counters were collected in their own
rocprofv3 passes (one counter per pass, no tracing domains besides the
implicit dispatch records).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os

KERNELS = {"ff_minmax_partials": "psf::ff_minmax_partials<float, true>",
           "ff_encode": "psf::ff_encode<float, 1, true>",
           "ff_decode": "psf::ff_decode<float, 1, true>"}
ALG = {"ff_minmax_partials": lambda n, nb: 4 * n,
       "ff_encode": lambda n, nb: (4 + nb) * n,
       "ff_decode": lambda n, nb: (4 + nb) * n}


def load(path, counter):
    vals = collections.defaultdict(list)
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for short, full in KERNELS.items():
            if full in r["Kernel_Name"]:
                vals[short].append(float(r["Counter_Value"]))
                rows.append({"kernel": short, "counter": counter, "value_kib": float(r["Counter_Value"]),
                             "start": r["Start_Timestamp"], "end": r["End_Timestamp"]})
    return vals, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--nb", type=int, default=1)
    ap.add_argument("--out", required=True)
    ap.add_argument("--trim", help="prefix for trimmed per-dispatch CSVs of the psf kernels")
    a = ap.parse_args()
    fv, frows = load(a.fetch, "FETCH_SIZE")
    wv, wrows = load(a.write, "WRITE_SIZE")
    out = {}
    for k in KERNELS:
        if not fv.get(k) or not wv.get(k):
            continue
        fetch = sum(fv[k]) / len(fv[k]) * 1024.0
        write = sum(wv[k]) / len(wv[k]) * 1024.0
        hbm = 2.0 * fetch + write
        alg = ALG[k](a.n, a.nb)
        out[k] = {"n": a.n, "nb": a.nb, "launches": len(fv[k]),
                  "fetch_size_bytes_raw": round(fetch), "write_size_bytes": round(write),
                  "hbm_bytes_per_launch": round(hbm), "alg_bytes_per_launch": alg,
                  "traffic_over_alg": round(hbm / alg, 4),
                  "correction": "read = 2 x FETCH_SIZE (gfx950 streaming-read calibration)"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))
    if a.trim:
        with open(a.trim + "_pmc_dispatches.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=["kernel", "counter", "value_kib", "start", "end"])
            w.writeheader()
            for r in frows + wrows:
                w.writerow(r)


if __name__ == "__main__":
    main()
