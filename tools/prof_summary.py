"""Per-kernel summary (calls, total, average, share) from a rocprofv3 output:
either the kernel_stats.csv of `--stats --output-format csv` or a rocpd .db."""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    rows = cur.execute(
        "select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end-d.start), "
        "max(d.end-d.start) from %s d join %s s on d.kernel_id = s.id group by s.kernel_name" % (kd, ks)).fetchall()
    return [(r[0], r[1], r[2], r[3], r[4], r[5]) for r in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                        float(r["MinNs"]), float(r["MaxNs"])))
    return out


def main(path):
    if os.path.isdir(path):
        c = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
        d = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = c[0] if c else d[0]
    rows = from_csv(path) if path.endswith(".csv") else from_db(path)
    tot = sum(r[2] for r in rows)
    rows.sort(key=lambda r: -r[2])
    print("%-70s %7s %12s %12s %7s" % ("kernel", "calls", "total_ms", "avg_us", "share"))
    for name, n, t, a, mn, mx in rows:
        nm = name if len(name) < 70 else name[:67] + "..."
        print("%-70s %7d %12.3f %12.2f %6.1f%%" % (nm, n, t / 1e6, a / 1e3, 100 * t / tot))


if __name__ == "__main__":
    main(sys.argv[1])
