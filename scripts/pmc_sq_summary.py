"""Per-kernel mean of every PMC counter found under a directory of rocprofv3 csv outputs."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

per = {}
for fn in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    with open(fn) as f:
        for row in csv.DictReader(f):
            per.setdefault(short(row["Kernel_Name"]), {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
json.dump(out, open(os.path.join(sys.argv[1], "sq_summary.json"), "w"), indent=1)
for k, cs in out.items():
    print(k, json.dumps({c: round(v) for c, v in cs.items()}))
