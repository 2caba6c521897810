"""One-line summary of a bench.py JSON line (for GPU session logs)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
hp = d.get("host_path") or {}
print(json.dumps({
    "config": d["config"].get("config"), "value": d["value"], "ms_per_step": d["ms_per_step"],
    "p99_batch_ms": d["p99_batch_ms"], "p99_sync_ms": d.get("p99_sync_ms"),
    "dom": r.get("kernel"), "frac": r.get("frac"), "avg_us": r.get("avg_us"), "traffic": r.get("traffic"),
    "cpu": (d.get("cpu_baseline") or {}).get("value"), "cpu_cores": (d.get("cpu_baseline") or {}).get("cores"),
    "host_sync": (hp.get("sync") or {}).get("decisions_per_s"),
    "host_streamed": (hp.get("streamed") or {}).get("decisions_per_s"),
    "kernels": {k: v["avg_us"] for k, v in d.get("kernels", {}).items()},
    **({"count_min": d["count_min"]} if "count_min" in d else {}),
}))
