#!/usr/bin/env python3
"""Per-kernel duration summary (calls, avg/min/max us) from a rocprofv3
SQLite output (rocpd_*.db), for runs that did not write the csv stats."""
import sqlite3
import sys


def main(path, width=110):
    c = sqlite3.connect(path)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in c.execute(f"pragma table_info({sym})")]
    name = "display_name" if "display_name" in cols else "kernel_name"
    q = (f"select s.{name}, count(*), avg(d.end - d.start), min(d.end - d.start), max(d.end - d.start) "
         f"from {disp} d join {sym} s on d.kernel_id = s.id group by s.{name} order by sum(d.end - d.start) desc")
    print(f"{'kernel':{width}s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s}")
    for nm, n, avg, mn, mx in c.execute(q):
        print(f"{nm[:width]:{width}s} {n:6d} {avg / 1e3:9.2f} {mn / 1e3:9.2f} {mx / 1e3:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
