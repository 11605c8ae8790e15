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
