"""Summarise a rocprofv3 kernel-trace database (rocpd sqlite) per kernel:
total ms, launches, mean ms.  usage: python tools/kstats.py <run_results.db> [csv_out]"""
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e6 from kernels "
                 "group by name order by sum(end-start) desc").fetchall()
lines = ["kernel,launches,total_ms,mean_ms"]
for name, n, tot, avg in rows:
    short = name.replace("(anonymous namespace)::", "").replace("void ", "")
    short = short.split("(")[0]
    lines.append(f"{short},{n},{tot:.4f},{avg:.4f}")
print("\n".join(lines))
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write("\n".join(lines) + "\n")

# optional: every launch (short name, start/end in ms from the first launch,
# stream and queue ids where the database has them), for timelines
if len(sys.argv) > 3:
    cols = [d[0] for d in c.execute("select * from kernels limit 1").description]
    extra = [k for k in ("stream_id", "queue_id") if k in cols]
    q = "select name, start, end" + "".join(", " + k for k in extra) + " from kernels order by start"
    launches = c.execute(q).fetchall()
    t0 = launches[0][1] if launches else 0
    with open(sys.argv[3], "w") as f:
        f.write("kernel,start_ms,end_ms" + "".join("," + k for k in extra) + "\n")
        for r in launches:
            short = r[0].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            short = short.split("<rocprim")[0].replace(",", ";")[:60]
            f.write(f"{short},{(r[1] - t0) / 1e6:.4f},{(r[2] - t0) / 1e6:.4f}" + "".join(f",{v}" for v in r[3:]) + "\n")
