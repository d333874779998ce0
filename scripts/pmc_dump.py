"""Print per-kernel averages of every PMC counter in a rocpd db: python scripts/pmc_dump.py <db>..."""
import sqlite3
import sys

for db in sys.argv[1:]:
    con = sqlite3.connect(db)
    rows = con.execute("select name, counter_name, avg(counter_value), count(*) from pmc_events group by name, counter_name order by name").fetchall()
    last = None
    for name, c, v, k in rows:
        n = name.split("(")[0].replace("void ", "")
        if n != last:
            print(f"-- {n}")
            last = n
        print(f"   {c:28s} {v:16.1f}  (x{k})")
