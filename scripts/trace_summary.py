"""Per-kernel averages from a rocprofv3 kernel trace, split into bench.py's phases.

rocprofv3 --stats averages every launch of a kernel, but bench.py also sends the 1M-event
host-path batches through the same kernels (same grid: the grid depends on the flow table, not the
batch).  Launches of each kernel are taken in time order and cut into the bench's phases.
Usage: python scripts/trace_summary.py run_kernel_trace.csv warmup:2,profile:3,timed:10,host:5
"""
import csv
import json
import sys
from collections import defaultdict


def main(path, phases):
    spec = [(p.split(":")[0], int(p.split(":")[1])) for p in phases.split(",")]
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "sentinel" not in name:
            continue
        short = name.split("(")[0].replace("void ", "").replace("sentinel::", "")
        acc[short].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    out = {}
    for k, rows in sorted(acc.items()):
        d = [x for _, x in sorted(rows)]
        if len(d) != sum(c for _, c in spec):
            out[k] = {"all": {"calls": len(d), "avg_us": round(sum(d) / len(d), 2)}}
            continue
        out[k], i = {}, 0
        for ph, c in spec:
            seg = d[i:i + c]
            i += c
            if seg:
                out[k][ph] = {"calls": c, "avg_us": round(sum(seg) / c, 2), "min_us": round(min(seg), 2),
                              "max_us": round(max(seg), 2)}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
