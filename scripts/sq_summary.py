"""Average per launch of every counter in scripts/sq_profile.sh's passes, per kernel.
Usage: python scripts/sq_summary.py gpurun_out/prof_TAG [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

src = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        per[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (name, _, cn), v in per.items():
        agg[name][cn].append(v)
out = {k: {cn: sum(v) / len(v) for cn, v in sorted(c.items())} for k, c in agg.items()}
for k, c in out.items():
    print(k)
    for cn, v in c.items():
        print(f"  {cn:28s} {v:16.1f}")
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
