"""Time the flow pipelines on several event distributions (engine choice study, not the headline).

usage: SENTINEL_FLOW_PATH=partition|sorted python scripts/bench_variants.py
Prints one JSON line per workload: mean / p99 device ms per batch and decisions/s."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sentinel_amd as sa  # noqa: E402
from sentinel_amd import trace as T  # noqa: E402
from sentinel_amd.token_service import device_events  # noqa: E402


def run(name, n_flows, n_events, dist, sample_count=10, steps=8, warmup=2, zipf_s=1.1):
    rng = np.random.default_rng(7)
    rules = T.make_rules(n_flows, rng, sample_count=sample_count, window_interval_ms=1000)
    svc = sa.GpuTokenService(0)
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    dev = torch.device("cuda", 0)
    rate = 2.0 * float(rules.count.sum())
    evs = []
    for s in range(steps + warmup):
        if dist == "uniform":
            idx = rng.integers(0, n_flows, size=n_events).astype(np.int32)
        else:
            idx = T.zipf_indices(n_flows, zipf_s, n_events, rng)
        ts = T.timestamps(n_events, rate, T.T0_ALIGNED + int(s * n_events * 1000.0 / rate))
        evs.append(device_events(torch.from_numpy(idx).to(dev), torch.ones(n_events, dtype=torch.int32, device=dev),
                                 torch.from_numpy(ts).to(dev)))
    out = torch.empty(n_events, dtype=torch.int64, device=dev)
    ext = torch.cuda.ExternalStream(svc.stream, device=dev)
    for s in range(warmup):
        svc.submit_flow_batch(evs[s], verdicts=out)
    svc.synchronize()
    a = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    b = [torch.cuda.Event(enable_timing=True) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        a[k].record(ext)
        svc.submit_flow_batch(evs[warmup + k], verdicts=out)
        b[k].record(ext)
    svc.synchronize()
    wall = time.perf_counter() - t0
    lat = sorted(a[k].elapsed_time(b[k]) for k in range(steps))
    print(json.dumps({"workload": name, "path": os.environ.get("SENTINEL_FLOW_PATH", "auto"),
                      "decisions_per_s": round(n_events * steps / wall, 1), "mean_ms": round(sum(lat) / steps, 3),
                      "max_ms": round(lat[-1], 3)}), flush=True)
    svc.close()


if __name__ == "__main__":
    N = 8 * 1024 * 1024
    run("config3 uniform 1M flows n=10", 1_000_000, N, "uniform")
    run("zipf1.1 1M flows n=10", 1_000_000, N, "zipf")
    run("config2 zipf1.1 10k flows n=2", 10_000, 4 * 1024 * 1024, "zipf", sample_count=2)
    run("zipf1.1 100k flows n=2", 100_000, N, "zipf", sample_count=2)
    run("uniform 100k flows n=2", 100_000, N, "uniform", sample_count=2)
