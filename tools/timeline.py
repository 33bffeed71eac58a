"""Per-update timeline from a rocprofv3 --kernel-trace CSV: for each update
(delimited by its k_pack_split / k_pack_batch launch) the span, the summed
kernel time, the idle gaps, and per-kernel-name time.
    python tools/timeline.py <kernel_trace.csv> [updates to skip]"""
import csv
import sys
from collections import defaultdict


def short(n):
    for p in ("void ", "(anonymous namespace)::"):
        n = n.replace(p, "")
    n = n.split("(")[0]
    return n[:60]


def main(path, skip=1):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_pack_split" in r["Kernel_Name"] or "k_pack_batch" in r["Kernel_Name"]]
    ups = [(starts[k], starts[k + 1] if k + 1 < len(starts) else len(rows)) for k in range(len(starts))]
    ups = ups[skip:-1] if len(ups) > skip + 1 else ups[skip:]
    agg = defaultdict(float)
    spans, busy = [], []
    for a, b in ups:
        seg = rows[a:b]
        t0 = int(seg[0]["Start_Timestamp"])
        t1 = max(int(r["End_Timestamp"]) for r in seg)
        spans.append((t1 - t0) / 1e3)
        # union of busy intervals (two streams overlap)
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
        tot, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        tot += ce - cs
        busy.append(tot / 1e3)
        for r in seg:
            agg[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = len(ups)
    print("updates %d  span %.1f us  GPU busy %.1f us  idle %.1f us" % (
        n, sum(spans) / n, sum(busy) / n, (sum(spans) - sum(busy)) / n))
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
        print("  %8.1f us  %s" % (v / n, k))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
