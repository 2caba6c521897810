"""Per-kernel durations and the idle gap before each kernel, over the last steps of a rocprofv3
kernel trace (usage: python scripts/trace_gaps.py run_kernel_trace.csv [N])."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
prev = None
for r in [r for r in rows if "sentinel::" in r["Kernel_Name"]][-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[-30:]
    print(f"{name:32s} dur {(e - s) / 1000:8.2f} us  gap {((s - prev) / 1000 if prev else 0):6.2f} us")
    prev = e
