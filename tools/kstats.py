"""Per-kernel summary of a rocprofv3 results database (rocpd sqlite): calls, mean and total duration.
usage: python tools/kstats.py <results.db> [top]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rows = c.execute("select name, count(*), avg(end - start), sum(end - start) from kernels group by name "
                 "order by sum(end - start) desc").fetchall()
tot = sum(r[3] for r in rows)
print(f"{'kernel':90s} {'calls':>7s} {'mean us':>9s} {'total ms':>9s} {'%':>6s}")
for name, n, avg, s in rows[:top]:
    print(f"{name[:90]:90s} {n:7d} {avg / 1e3:9.2f} {s / 1e6:9.2f} {100 * s / tot:6.1f}")
