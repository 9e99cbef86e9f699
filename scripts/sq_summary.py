"""SQ counters of one kernel from a rocprofv3 --pmc run (counter_collection.csv).

  python scripts/sq_summary.py <counter_collection.csv> <out.json> <kernel substring> [last|all] [units] [note]

last: the kernel's last dispatch only (config 5: the last joint round, its largest trees);
all: summed over its dispatches (the per-dispatch mean is reported).  units: work items of one
dispatch (queries, units) for per-item instruction counts.  Derived (the guide's SQ table:
WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, disjoint, all in quad-cycles):
wait_any (parked on s_waitcnt / barrier: memory latency), wait_inst_any (issue stalls: the
pipe taken by other waves), active_inst_any (issuing) as fractions of SQ_WAVE_CYCLES."""
import collections
import csv
import json
import sys


def main(path, out, kernel, mode="last", units=None, note=None):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"no dispatch of {kernel}")
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    keep = {ids[-1]} if mode == "last" else set(ids)
    agg = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) in keep:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    n = len(keep)
    res = {"kernel": rows[-1]["Kernel_Name"][:160], "dispatches": n, "per_dispatch": {k: v / n for k, v in agg.items()}}
    if note:
        res["note"] = note
    wc = agg.get("SQ_WAVE_CYCLES")
    if wc:
        for c, k in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst_any"),
                     ("SQ_ACTIVE_INST_ANY", "active_inst_any"), ("SQ_ACTIVE_INST_VALU", "active_inst_valu")):
            if c in agg:
                res[f"{k}_over_wave_cycles"] = round(agg[c] / wc, 4)
    if agg.get("SQ_WAVES") and agg.get("SQ_INSTS_VALU"):
        res["valu_instructions_per_wave"] = round(agg["SQ_INSTS_VALU"] / agg["SQ_WAVES"], 1)
    if units and agg.get("SQ_INSTS_VALU"):
        res["units_per_dispatch"] = int(units)
        res["valu_instructions_per_unit"] = round(agg["SQ_INSTS_VALU"] / n / float(units), 1)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], a[2], a[3] if len(a) > 3 else "last", a[4] if len(a) > 4 else None, a[5] if len(a) > 5 else None)
