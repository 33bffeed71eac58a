"""Per-kernel summary (calls, total, average, share) from a rocprofv3 output:
either the kernel_stats.csv of `--stats --output-format csv` or a rocpd .db; with
the run's kernel_trace.csv beside it also the median and maximum launch (one
stalled launch, e.g. a 19.8 ms FVP among 80 of ~0.85 ms in profiles/r05q, moves
the average but not the median)."""
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


def medians(d):
    """name -> (median, max) launch duration in ns from a kernel_trace.csv under d."""
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not tr:
        return {}
    by = {}
    with open(tr[0]) as f:
        for r in csv.DictReader(f):
            by.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for k, v in by.items():
        v.sort()
        out[k] = (v[len(v) // 2] if len(v) % 2 else 0.5 * (v[len(v) // 2 - 1] + v[len(v) // 2]), v[-1])
    return out


def main(path):
    med = {}
    if os.path.isdir(path):
        med = medians(path)
        c = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
        d = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = c[0] if c else d[0]
    rows = from_csv(path) if path.endswith(".csv") else from_db(path)
    tot = sum(r[2] for r in rows)
    rows.sort(key=lambda r: -r[2])
    print("%-70s %7s %12s %12s %7s %10s %10s" % ("kernel", "calls", "total_ms", "avg_us", "share", "med_us",
                                                 "max_us"))
    for name, n, t, a, mn, mx in rows:
        nm = name if len(name) < 70 else name[:67] + "..."
        m = med.get(name)
        print("%-70s %7d %12.3f %12.2f %6.1f%% %10s %10s" % (
            nm, n, t / 1e6, a / 1e3, 100 * t / tot, "%.2f" % (m[0] / 1e3) if m else "-",
            "%.1f" % (m[1] / 1e3) if m else "-"))


if __name__ == "__main__":
    main(sys.argv[1])
