#!/usr/bin/env python3
"""Per-launch HBM traffic of every bench line's kernels, from one measurement
session's rocprofv3 PMC passes, into profiles/pmc_traffic.json (read by
bench.py for roofline.traffic).

    python tools/pmc_traffic.py gpurun_out/<tag> --out profiles/pmc_traffic.json

The session (tools/round_measure6.sh) holds, per bench line L,
pmc_L_fetch/ and pmc_L_write/: `rocprofv3 --pmc FETCH_SIZE` and
`--pmc WRITE_SIZE`, each its own run of `bench.py <L's args> --no-profile
--no-host-floor --steps 5 --warmup 1` (one counter per pass, no tracing
domain), so every launch of a kernel in a run has the line's shape.

Correction (MI355X_MICROARCH.md, HBM / rocprofv3): on gfx950 FETCH_SIZE
reports half the bytes of a coalesced streaming read, so read bytes =
2 x FETCH_SIZE (KiB x 1024); WRITE_SIZE is taken as reported.

The file maps line -> {"args": the bench arguments, "kernels": {profiler name
(libpsf's psf_profile_kernel_name, what bench.py's roofline.kernel says) ->
{launches, read / write / hbm bytes per launch}}}; several device kernels that
one profiler name covers (single-array and batched variants) are listed by
their own names under it.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os

# the bench lines of the session and their bench.py arguments (bench.py's
# line_key() names them the same way)
LINES = {
    "c2": "--no-128m --no-c4",
    "c1": "--config c1",
    "c3": "--config c3",
    "c4": "--config c4",
    "c4pull": "--config c4pull",
    "c5": "--config c5",
    "c5z": "--config c5 --compress",
}
# profiler name -> substrings of the device kernels it times
PROFILER = {
    "ff_minmax_partials": ["ff_minmax_partials<", "ff_minmax_batch<"],
    "ff_encode": ["ff_encode<", "ff_encode_batch<"],
    "ff_decode": ["ff_decode<", "ff_decode_batch<"],
    "ff_minmax_encode": ["ff_fused_batch<"],
    "ff_decode_minmax": ["ff_dec_mm_batch<"],
    "kvmap_get": ["kvmap_get_kernel", "kvmap_get_batch_kernel"],
    "crc32c_chunks": ["crc32c"],
}


def load(d, counter):
    per = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") == counter:
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
    return per


def line_traffic(session, line):
    fv = load(os.path.join(session, f"pmc_{line}_fetch"), "FETCH_SIZE")
    wv = load(os.path.join(session, f"pmc_{line}_write"), "WRITE_SIZE")
    out = {}
    for prof, subs in PROFILER.items():
        names = [n for n in set(fv) | set(wv) if any(s in n for s in subs)]
        if not names:
            continue
        per, rb, wb, launches = {}, 0.0, 0.0, 0
        for n in sorted(names):
            f, w = fv.get(n, []), wv.get(n, [])
            if not f or not w:
                continue
            r_ = 2.0 * sum(f) / len(f)
            w_ = sum(w) / len(w)
            per[n[:120]] = {"launches": len(f), "read_bytes_per_launch": round(r_),
                            "write_bytes_per_launch": round(w_)}
            rb, wb, launches = rb + r_ * len(f), wb + w_ * len(f), launches + len(f)
        if not launches:
            continue
        out[prof] = {"launches": launches, "read_bytes_per_launch": round(rb / launches),
                     "write_bytes_per_launch": round(wb / launches),
                     "hbm_bytes_per_launch": round((rb + wb) / launches), "device_kernels": per}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("session")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    res = {"correction": "read = 2 x FETCH_SIZE (gfx950 streaming-read calibration), write = WRITE_SIZE",
           "session": os.path.basename(os.path.normpath(a.session)), "lines": {}}
    for line, args in LINES.items():
        if not os.path.isdir(os.path.join(a.session, f"pmc_{line}_fetch")):
            continue
        k = line_traffic(a.session, line)
        if k:
            res["lines"][line] = {"args": args, "kernels": k}
    json.dump(res, open(a.out, "w"), indent=1)
    for line, v in res["lines"].items():
        print(line, {k: e["hbm_bytes_per_launch"] for k, e in v["kernels"].items()})


if __name__ == "__main__":
    main()
