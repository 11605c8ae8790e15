"""Per-kernel mean of one rocprofv3 --pmc counter from a rocpd database.
usage: python tools/pmc_summary.py <run_results.db> [csv_out]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select kernel_name, counter_name, count(*), avg(value), avg(vgpr_count), avg(scratch_size) "
                 "from counters_collection group by kernel_name, counter_name order by avg(value) desc").fetchall()
lines = ["kernel,counter,launches,mean_value,vgpr,scratch_bytes"]
for name, ctr, n, v, vg, sc in rows:
    short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    lines.append(f"{short},{ctr},{n},{v:.3f},{vg:.0f},{sc:.0f}")
print("\n".join(lines))
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write("\n".join(lines) + "\n")
