"""Per-kernel average durations from rocprofv3 SQLite output: python tools/kstats.py DIR [DIR...]"""
import glob
import sqlite3
import sys

for d in sys.argv[1:]:
    db = glob.glob(f"{d}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), avg(end-start) from kernels group by name "
                     "order by sum(end-start) desc limit 14").fetchall()
    print(d)
    for r in rows:
        print("  %-64s %4d %9.1f" % (r[0][:64], r[1], r[2]))
