#!/usr/bin/env python3
"""tools/timeline.py -- the decoder's GROM_TRACE timeline (pdecode.c pd_trace)
as intervals: each start/end pair per (thread, event, a) with its start, end
and length, in start order; phase codes named.  The start of a whole run (the
insert statistics, the first chromosome's decode) reads off the first lines.

    python tools/timeline.py trace.csv [--until SECONDS]
"""
import argparse
import csv

PHASES = {100: "decode context", 101: "run read (pread + block table)", 102: "run load (inflate + walk)",
          103: "insert statistics", 104: "decode buffers reserved", 105: "stages reserved"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--until", type=float, default=1e9)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((float(r["t"]), int(r["thread"]), r["event"], int(r["a"]), int(r["b"])))
    rows.sort()
    t0 = rows[0][0] if rows else 0.0
    open_, out = {}, []
    for t, th, ev, a, b in rows:
        if ev == "phase" and a == 103:  # a point event: statistics of run b
            out.append((t - t0, t - t0, th, "insert statistics (run %d)" % b))
            continue
        key = (th, ev, a)
        name = PHASES.get(a, "phase %d" % a) if ev == "phase" else "%s %d" % (ev, a)
        if b == 0:
            open_[key] = t
        elif key in open_:
            s = open_.pop(key)
            out.append((s - t0, t - t0, th, name))
        else:
            out.append((t - t0, t - t0, th, "%s (b=%d)" % (name, b)))
    for s, e, th, name in sorted(out):
        if s > args.until:
            break
        print(f"{s:8.3f} {e:8.3f} {1e3 * (e - s):9.1f} ms  thread {th:3d}  {name}")


if __name__ == "__main__":
    main()
