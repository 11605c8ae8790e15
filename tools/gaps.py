"""tools/gaps.py LAUNCHES.csv -- the decode streams' GPU timeline of a
whole-run kernel trace (tools/session.sh trace): busy time, gaps and the
kernels around each gap, per stream kind (inflate slot streams, the decode
context stream, scan contexts)."""
import collections
import csv
import sys

rows = [x for x in csv.DictReader(open(sys.argv[1]))]
for x in rows:
    x["s"], x["e"] = float(x["start_ms"]), float(x["end_ms"])
rows.sort(key=lambda x: x["s"])
by_stream = collections.defaultdict(list)
for x in rows:
    by_stream[x["stream_id"]].append(x)
inf_streams = {x["stream_id"] for x in rows if x["kernel"] == "k_inflate"}
ctx_streams = {x["stream_id"] for x in rows if x["kernel"] == "k_rec_meta"}
scan_streams = {x["stream_id"] for x in rows if x["kernel"].startswith("k_scan_tile")}


def union(xs):
    ev = sorted([(x["s"], 1) for x in xs] + [(x["e"], -1) for x in xs])
    c, last, busy = 0, 0.0, 0.0
    for t, d in ev:
        if c > 0:
            busy += t - last
        c += d
        last = t
    return busy


dec = [x for x in rows if x["stream_id"] in inf_streams | ctx_streams]
t0, t1 = dec[0]["s"], dec[-1]["e"]
print(f"decode window {t0:.1f}-{t1:.1f} ms ({t1 - t0:.1f}); busy on decode streams {union(dec):.1f} ms; "
      f"inflate busy {union([x for x in rows if x['kernel'] == 'k_inflate']):.1f} ms")
allk = [x for x in rows if t0 <= x["s"] <= t1]
print(f"any kernel busy in window {union(allk):.1f} ms")
# gaps on the decode streams
ev = sorted(dec, key=lambda x: x["s"])
end = ev[0]["e"]
gaps = []
for i, x in enumerate(ev[1:], 1):
    if x["s"] - end > float(sys.argv[2] if len(sys.argv) > 2 else 3.0):
        prev = max((y for y in ev[:i] if y["e"] <= x["s"] + 1e-9), key=lambda y: y["e"])
        gaps.append((end, x["s"], prev["kernel"][:28], x["kernel"][:28]))
    end = max(end, x["e"])
print(f"{len(gaps)} gaps, {sum(b - a for a, b, _, _ in gaps):.1f} ms")
for a, b, p, n in gaps:
    print(f"  {a:8.1f} -> {b:8.1f} ({b - a:6.1f} ms) after {p} before {n}")
