"""Summarise rocprofv3 PMC passes (scripts/profile.sh) into profiles/<tag>/pmc_summary.json.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, the correction
/opt/skills/guides/MI355X_MICROARCH.md (§HBM) prescribes for gfx950: FETCH_SIZE reports
half the bytes of a wide coalesced read.  The doubling is calibrated for 16-B-per-lane
vector loads only; kernels whose reads are scalar (s_load) loads are marked as such in
DESIGN.md.  Usage: python scripts/pmc_summary.py gpurun_out/prof_r01 profiles/r01 [window-start window-end]
"""
import collections
import csv
import json
import os
import shutil
import sys


def steady_durations(kt_csv, start=None, end=None):
    """Per kernel, the kernel-trace duration (us) of its steady-state launches: the mean over
    the same dispatch window as the counters when one is given (config 5: the last joint round),
    else the median of its launches after the first -- the first launch of a kernel in a process
    is cold (code object load, first touch of its buffers), and a bench's untimed work-counter
    round (same-address atomics: config 2's grid NN 405 us against 34) is one outlier."""
    rows = list(csv.DictReader(open(kt_csv)))
    for r in rows:
        r.setdefault("Dispatch_Id", r.get("Correlation_Id", "0"))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for i, r in enumerate(rows):
        r["Dispatch_Id"] = str(i)  # trace order (window() sorts by it)
    if start:
        rows = window(rows, start, end)
    per = collections.defaultdict(list)
    for r in rows:
        per[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for k, v in per.items():
        if start:
            out[k] = (round(sum(v) / len(v), 3), len(v))
        else:
            use = sorted(v[1:] if len(v) > 1 else v)
            out[k] = (round(use[len(use) // 2], 3), len(use))
    return out


def window(rows, start, end):
    """Dispatches from the first whose kernel name contains `start` ("last:<name>": the last
    such) up to (not including) the first after it whose name contains `end` (or the end) --
    e.g. config 5's last joint round only ("last:k_sample_jobs"): the round whose hipEvent stage
    times bench.py reports, at the same tree sizes as its compulsory bytes (an average over the
    run's growing trees does not match either)."""
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    if start.startswith("last:"):  # from the last dispatch matching the marker
        start = start[5:]
        hits = [i for i, r in enumerate(rows) if start in r["Kernel_Name"]]
        i0 = hits[-1] if hits else None
    else:
        i0 = next((i for i, r in enumerate(rows) if start in r["Kernel_Name"]), None)
    if i0 is None:
        return rows
    i1 = next((i for i in range(i0, len(rows)) if end and end in rows[i]["Kernel_Name"]), len(rows))
    return rows[i0:i1]


def main(src, dst, start=None, end=None):
    os.makedirs(dst, exist_ok=True)
    out = {}
    for tag, cn in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        path = os.path.join(src, tag, "run_counter_collection.csv")
        agg = collections.defaultdict(list)
        rows = list(csv.DictReader(open(path)))
        if start:
            rows = window(rows, start, end)
        for r in rows:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            out.setdefault(k, {})[cn] = sum(v) / len(v)
            out[k]["launches"] = len(v)
    summ = {}
    for k, v in out.items():
        f, w = v.get("FETCH_SIZE", 0.0), v.get("WRITE_SIZE", 0.0)
        summ[k] = {"FETCH_SIZE_KB": round(f, 3), "WRITE_SIZE_KB": round(w, 3),
                   "hbm_bytes_per_launch": round((2 * f + w) * 1024), "launches": v.get("launches", 1)}
    json.dump(summ, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    kt = os.path.join(src, "kt", "run_kernel_trace.csv")
    if os.path.exists(kt):
        steady = steady_durations(kt, start, end)
        for k, v in summ.items():
            if k in steady:
                v["steady_us"], v["steady_launches"] = steady[k]
        json.dump(summ, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    ks = os.path.join(src, "kt", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
    print(json.dumps({k[:60]: v["hbm_bytes_per_launch"] for k, v in summ.items()}, indent=1))


if __name__ == "__main__":
    # optional: a dispatch window (see window()), e.g. k_sample_jobs "k_sample("
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:5]))
