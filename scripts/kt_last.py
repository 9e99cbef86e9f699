"""Per-kernel mean duration over each kernel's last N launches from a rocprofv3 kernel trace
(--kernel-trace --output-format csv): the steady state of a run whose early launches work on
smaller trees.  python scripts/kt_last.py <kernel_trace.csv> [N] [name-filter ...]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    filt = sys.argv[3:]
    calls = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            m = re.search(r"(k_[a-z0-9_]+)(<[^>(]*>)?", name)
            key = m.group(1) + (m.group(2) or "") if m else name[:60]
            if filt and not any(x in key for x in filt):
                continue
            calls[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows = []
    for k, v in calls.items():
        v.sort()
        last = [d for _, d in v[-n_last:]]
        rows.append((sum(last) / len(last) / 1e3, len(v), k))
    rows.sort(reverse=True)
    tot = 0.0
    for us, n, k in rows:
        tot += us
        print(f"{us:10.1f} us  {n:6d} calls  {k}")
    print(f"{tot:10.1f} us  sum of the per-kernel means")


if __name__ == "__main__":
    main()
