"""Summarise the two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) per kernel.

Corrections exactly as /opt/skills/guides/MI355X_MICROARCH.md (HBM section) prescribes:
FETCH_SIZE / WRITE_SIZE are KiB per dispatch; on gfx950 FETCH_SIZE reports half of the bytes of a
wide coalesced read, so it is doubled.  Output: JSON with, per kernel symbol, the dispatch count and
the mean corrected read / write bytes per dispatch (the `traffic` of bench.py's roofline).

usage: python scripts/pmc_summary.py <dir holding pmc_fetch/ and pmc_write/> [bench.json]
With the bench JSON line of one of the passes, the summary records its workload `shape` (the keys
bench.py matches before it quotes the traffic of a kernel: config, flows, events, sample_count).
"""
import csv
import glob
import json
import os
import re
import sys


def short(name: str) -> str:
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^()]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0][-80:]


def load(d: str, counter: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row["Kernel_Name"])
                per.setdefault(k, []).append(float(row["Counter_Value"]))
    return per


def main():
    d = sys.argv[1]
    fetch = load(os.path.join(d, "pmc_fetch"), "FETCH_SIZE")
    write = load(os.path.join(d, "pmc_write"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        out[k] = {"dispatches": max(len(f), len(w)), "read_bytes_avg": fb, "write_bytes_avg": wb,
                  "traffic_bytes_avg": (fb or 0.0) + (wb or 0.0)}
    doc = {"correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate runs of bench.py --steps 3 --warmup 1",
           "kernels": out}
    if len(sys.argv) > 2:
        with open(sys.argv[2]) as f:
            cfg = json.loads(f.read().strip().splitlines()[-1])["config"]
        # the workload's own shape keys (bench.py W.shape(): flows or rules, events, sample count)
        doc["shape"] = {k: v for k, v in cfg.items() if k not in ("workload", "events_per_gpu_per_step", "parallelism")}
    json.dump(doc, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
