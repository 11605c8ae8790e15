#!/usr/bin/env python3
"""tools/trace_summary.py -- summarise a GROM_TRACE host timeline (pdecode.h).

Prints, per activity (piece decode, piece upload, chromosome scan), its first
start, last end and busy time, and how long each pair ran at the same time:
the evidence that decode, host->device staging and the scans overlap.

    python tools/trace_summary.py gpurun_out/cli_trace/trace.csv
"""
import csv
import sys


def intervals(rows, event):
    open_, out = {}, []
    for t, thread, ev, a, b in rows:
        if ev != event:
            continue
        key = (thread, a)
        if b == 0:
            open_[key] = t
        elif b == 1 and key in open_:
            out.append((open_.pop(key), t))
    return out


def union(iv):
    merged = []
    for s, e in sorted(iv):
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    return merged


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((float(r["t"]), r["thread"], r["event"], int(r["a"]), int(r["b"])))
    acts = {name: intervals(rows, name) for name in ("decode", "upload", "scan")}
    spans = {name: union(iv) for name, iv in acts.items()}
    for name, iv in acts.items():
        if not iv:
            continue
        print(f"{name:7s} n={len(iv):4d} first start {min(s for s, _ in iv):.3f} s, last end "
              f"{max(e for _, e in iv):.3f} s, summed {sum(e - s for s, e in iv):.3f} s, "
              f"wall covered {length(spans[name]):.3f} s")
    names = [n for n in spans if spans[n]]
    for i, a in enumerate(names):
        for b in names[i + 1:]:
            print(f"{a} and {b} at the same time: {length(intersect(spans[a], spans[b])):.3f} s")
    for t, _, ev, a, b in rows:
        if ev == "stats":
            print(f"insert statistics complete at {t:.3f} s")
    fin = [t for t, _, ev, _, _ in rows if ev == "final"]
    if fin:
        print(f"chromosomes finalised: {len(fin)}, first {min(fin):.3f} s, last {max(fin):.3f} s")


if __name__ == "__main__":
    main(sys.argv[1])
