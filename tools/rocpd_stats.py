"""Per-kernel stats (calls, avg us, total us) from a rocprofv3 rocpd database (run_results.db)."""
import sqlite3
import sys


def stats(db, top=30):
    c = sqlite3.connect(db)
    q = ("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1000.0 from kernels "
         "group by name order by 4 desc limit ?")
    return [(r[0], r[1], r[2], r[3]) for r in c.execute(q, (top,))]


if __name__ == "__main__":
    for name, n, avg, tot in stats(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30):
        print(f"{n:6d} {avg:10.2f} {tot:11.1f}  {name[:120]}")
