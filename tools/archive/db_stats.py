"""Per-kernel stats from a rocprofv3 .db: python tools/db_stats.py run_results.db"""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
q = f"select {name}, count(*), avg(end-start)/1000.0, sum(end-start)/1e6 from kernels group by {name} order by 4 desc limit 15"
for n, cnt, avg, tot in c.execute(q):
    print(f"{tot:10.2f} ms  {cnt:7d} x {avg:9.2f} us  {n[:90]}")
