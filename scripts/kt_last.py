"""Per-kernel steady-state times from a rocprofv3 kernel trace (--kernel-trace --output-format
csv), for runs whose early launches work on smaller trees.

  python scripts/kt_last.py <kernel_trace.csv> [N] [name-filter ...]
      mean duration of each kernel's last N launches (default 3)
  python scripts/kt_last.py <kernel_trace.csv> --rounds MARKER A B [name-filter ...]
      per-round sums: the trace cut into rounds at each launch of MARKER (e.g. k_sample_jobs,
      a joint round's first kernel), rounds A..B-1 averaged: every kernel's time a round
"""
import csv
import re
import sys
from collections import defaultdict


def key_of(name):
    m = re.search(r"(k_[a-z0-9_]+)(<[^>(]*>)?", name)
    return m.group(1) + (m.group(2) or "") if m else name[:60]


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.append((s, e - s, key_of(r["Kernel_Name"])))
    rows.sort()
    return rows


def last_n(rows, n_last, filt):
    calls = defaultdict(list)
    for s, d, k in rows:
        if not filt or any(x in k for x in filt):
            calls[k].append(d)
    out = [(sum(v[-n_last:]) / len(v[-n_last:]) / 1e3, len(v), k) for k, v in calls.items()]
    return sorted(out, reverse=True)


def per_round(rows, marker, a, b, filt):
    starts = [s for s, _, k in rows if marker in k]
    if len(starts) < b:
        raise SystemExit(f"only {len(starts)} launches of {marker}")
    sums, counts = defaultdict(float), defaultdict(int)
    for s, d, k in rows:
        if starts[a] <= s < (starts[b] if b < len(starts) else float("inf")):
            if not filt or any(x in k for x in filt):
                sums[k] += d
                counts[k] += 1
    n = b - a
    return sorted(((v / n / 1e3, counts[k] // n, k) for k, v in sums.items()), reverse=True)


def main():
    path = sys.argv[1]
    args = sys.argv[2:]
    rows = load(path)
    if args and args[0] == "--rounds":
        marker, a, b, filt = args[1], int(args[2]), int(args[3]), args[4:]
        res = per_round(rows, marker, a, b, filt)
        label = "a round"
    else:
        n_last = int(args[0]) if args else 3
        res = last_n(rows, n_last, args[1:])
        label = "calls"
    tot = 0.0
    for us, n, k in res:
        tot += us
        print(f"{us:10.1f} us  {n:6d} {label}  {k}")
    print(f"{tot:10.1f} us  sum")


if __name__ == "__main__":
    main()
