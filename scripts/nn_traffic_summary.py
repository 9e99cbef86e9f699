"""Summarise scripts/nn_traffic.sh: for each k_ct_nn1_jobs replay (and the last two rounds' own
launches) its kernel-trace duration, FETCH_SIZE, WRITE_SIZE and HBM bytes (2 FETCH + WRITE, the
guide's gfx950 reading) -> <dir>/summary.json.   python scripts/nn_traffic_summary.py <dir>"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_ct_nn1_jobs"


def csv_of(d, suffix):
    hits = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def nn_rows(path, key):
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
    return rows


def main(d):
    kt = nn_rows(csv_of(os.path.join(d, "kt"), "kernel_trace.csv"), "kt")
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in kt]
    counters = {}
    for tag, name in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        rows = nn_rows(csv_of(os.path.join(d, tag), "counter_collection.csv"), tag)
        counters[name] = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == name]
    n = len(dur)
    assert all(len(v) == n for v in counters.values()), (n, {k: len(v) for k, v in counters.items()})
    meta = json.load(open(os.path.join(d, "replay_kt.json")))
    LABELS = meta["replays_in_dispatch_order"]
    rounds = n - len(LABELS)
    names = [f"round_{rounds - 2}", f"round_{rounds - 1}"] + LABELS
    idx = [rounds - 2, rounds - 1] + list(range(rounds, n))
    out = {"kernel": "k_ct_nn1_jobs<7, 64, 8>", "seeds": meta["seeds"], "queries": meta["queries"],
           "nodes_indexed": meta["nodes_indexed"],
           "replay_ms_hipevent": meta["replay_ms"], "launches": {}}
    for name, i in zip(names, idx):
        f, w = counters["FETCH_SIZE"][i], counters["WRITE_SIZE"][i]
        out["launches"][name] = {"us": round(dur[i], 1), "FETCH_SIZE_KB": round(f), "WRITE_SIZE_KB": round(w),
                                 "hbm_bytes": round((2 * f + w) * 1024)}
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
