"""Summarise a rocprofv3 --hip-trace CSV: per-API durations over the last
`--tail` calls of the busiest host thread, and the host time spent between API
calls (own bookkeeping).  Used to split C1's per-step host cost into HIP
runtime time and libpsf host logic.

    python tools/trace_gaps.py gpurun_out/c1host/c1_hip_api_trace.csv --tail 4000
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=int, default=4000)
    ap.add_argument("--seq", type=int, default=0, help="print this many calls from the middle of the tail")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    by_tid = collections.Counter(r["Thread_Id"] for r in rows)
    tid = by_tid.most_common(1)[0][0]
    rows = [r for r in rows if r["Thread_Id"] == tid]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.tail:]
    if a.seq:
        mid = len(rows) // 2
        t0 = int(rows[mid]["Start_Timestamp"])
        for r in rows[mid:mid + a.seq]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"{(s - t0) / 1e3:9.2f} +{(e - s) / 1e3:6.2f} {r['Function']}")
    dur = collections.defaultdict(list)
    gap_after = collections.defaultdict(list)
    for i, r in enumerate(rows):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[r["Function"]].append(e - s)
        if i + 1 < len(rows):
            gap_after[r["Function"]].append(int(rows[i + 1]["Start_Timestamp"]) - e)
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    tot_api = sum(sum(v) for v in dur.values())
    print(f"thread {tid}: {len(rows)} calls over {span / 1e3:.1f} us; in API {tot_api / 1e3:.1f} us, "
          f"between calls {(span - tot_api) / 1e3:.1f} us")
    for f, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        v = sorted(v)
        g = sorted(gap_after[f]) or [0]
        print(f"{f[:40]:40s} n={len(v):6d} tot={sum(v) / 1e3:9.1f}us med={v[len(v) // 2] / 1e3:6.2f} "
              f"p90={v[int(len(v) * .9)] / 1e3:6.2f}  gap-after med={g[len(g) // 2] / 1e3:6.2f} "
              f"tot={sum(g) / 1e3:9.1f}us")


if __name__ == "__main__":
    main()
