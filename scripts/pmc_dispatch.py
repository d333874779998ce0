"""Per-dispatch PMC values of kernels matching a filter, in dispatch order, across passes:
python scripts/pmc_dispatch.py FILTER db1 db2 ...  (one column per counter)"""
import sqlite3
import sys

flt = sys.argv[1]
table = {}
names = {}
for db in sys.argv[2:]:
    con = sqlite3.connect(db)
    for did, name, c, v, dur in con.execute(
            "select dispatch_id, name, counter_name, counter_value, duration from pmc_events order by dispatch_id"):
        if flt not in name:
            continue
        key = (db, did)
        table.setdefault(key, {})[c] = v
        table[key]["dur_us"] = dur / 1e3
        names[key] = name.split("(")[0].replace("void ", "")[:40]
# dispatch order within each db; print grouped by db
for db in sys.argv[2:]:
    rows = [(k, v) for k, v in table.items() if k[0] == db]
    if not rows:
        continue
    print("==", db)
    for (_, did), v in sorted(rows, key=lambda kv: kv[0][1]):
        print(f"  {did:5d} {names[(db, did)]:40s} " + "  ".join(f"{c}={x:.4g}" for c, x in sorted(v.items())))
