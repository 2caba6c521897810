"""Print a window of a rocprofv3 kernel trace: start / end relative to the first kernel named `anchor`
(its `skip`-th occurrence), duration, queue -- shows cross-stream overlap (pipelined submits, hot runs)."""
import csv
import re
import sys

path, anchor = sys.argv[1], sys.argv[2]
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 8
count = int(sys.argv[4]) if len(sys.argv) > 4 else 24
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
seq = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
        re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[-36:], r["Queue_Id"]) for r in rows]
idx = [i for i, s in enumerate(seq) if anchor in s[2]]
i0 = idx[min(skip, len(idx) - 1)]
t0 = seq[i0][0]
for a, b, name, q in seq[i0:i0 + count]:
    print(f"{(a - t0) / 1000:9.2f} {(b - t0) / 1000:9.2f} {(b - a) / 1000:8.2f}  q{q}  {name}")
