"""Kernel stats (calls, avg/min/max us) from a rocprofv3 rocpd SQLite database (the default
output format of rocprofv3 in ROCm 7.x): python tools/rocpd_stats.py <db> [name-substring]"""
import sqlite3
import sys


def main():
    db, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    rows = c.execute(f"select s.kernel_name, d.end - d.start from {kd} d join {ks} s on d.kernel_id = s.id").fetchall()
    agg = {}
    for n, dt in rows:
        if pat in n:
            agg.setdefault(n, []).append(dt)
    tot = sum(sum(v) for v in agg.values())
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(v):5d} avg {sum(v)/len(v)/1e3:9.2f} us  min {min(v)/1e3:9.2f}  max {max(v)/1e3:9.2f}  "
              f"{100*sum(v)/tot:5.1f}%  {n[:110]}")


if __name__ == "__main__":
    main()
