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


def req_summary(d: str, bench_json=None):
    """Round 5: bytes from the memory-side request counters by request size (scripts/gpu_pmc_req.sh),
    instead of FETCH_SIZE x2.  Reads = 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (with the
    remainder of RDREQ not in any of the three, if any, counted at 64 B and reported as `rdreq_other`);
    writes = 32 x (WRREQ - WRREQ_64B) + 64 x WRREQ_64B (rocprofv3's own WRITE_SIZE expression)."""
    names = {"rd": ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"],
             "wr": ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "TCC_BUBBLE_sum"]}
    vals = {}
    for sub, cs in names.items():
        for c in cs:
            for k, xs in load(os.path.join(d, sub), c).items():
                vals.setdefault(k, {})[c] = xs
    out = {}
    for k, m in sorted(vals.items()):
        def avg(c):
            xs = m.get(c, [])
            return sum(xs) / len(xs) if xs else 0.0
        rd, r32, r64, r128 = (avg(c) for c in names["rd"])
        wr, w64, bub = (avg(c) for c in names["wr"])
        other = max(0.0, rd - r32 - r64 - r128)
        rb = 32 * r32 + 64 * r64 + 128 * r128 + 64 * other
        wb = 32 * (wr - w64) + 64 * w64
        out[k] = {"dispatches": max(len(m.get(c, [])) for c in names["rd"] + names["wr"]),
                  "read_bytes_avg": rb, "write_bytes_avg": wb, "traffic_bytes_avg": rb + wb,
                  "rdreq_avg": rd, "rdreq_32b_avg": r32, "rdreq_64b_avg": r64, "rdreq_128b_avg": r128,
                  "rdreq_other_avg": other, "wrreq_avg": wr, "wrreq_64b_avg": w64, "bubble_avg": bub,
                  "fetch_size_x2_bytes_avg": 2 * (bub * 128 + (rd - bub - r32) * 64 + r32 * 32)}
    doc = {"correction": "bytes by request size: reads 32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B, writes "
                         "32 x (WRREQ - WRREQ_64B) + 64 x WRREQ_64B (no blanket x2); fetch_size_x2_bytes_avg = the "
                         "old FETCH_SIZE x2 figure from the same counters, for comparison",
           "source": "rocprofv3 --pmc, two separate passes (scripts/gpu_pmc_req.sh)", "kernels": out}
    if bench_json:
        try:
            with open(bench_json) as f:
                cfg = json.loads(f.read().strip().splitlines()[-1])["config"]
            doc["shape"] = {k: v for k, v in cfg.items() if k not in ("workload", "events_per_gpu_per_step", "parallelism")}
        except (OSError, ValueError, KeyError, IndexError):
            pass
    return doc


def main():
    if sys.argv[1] == "--req":
        json.dump(req_summary(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None), sys.stdout, indent=1)
        return
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
