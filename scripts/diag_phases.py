"""Cost diagnostic for k_part_fused (needs a -DSENTINEL_DIAG_PHASES build in SENTINEL_LIB):
per-workgroup wall-clock stamps of its phases on the bench workload (config 3, one batch)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sentinel_amd as sa  # noqa: E402
from sentinel_amd import trace as T  # noqa: E402
from sentinel_amd.token_service import device_events  # noqa: E402

F, N = int(os.environ.get("DIAG_FLOWS", "1000000")), 8 * 1024 * 1024   # 977 ranges for 125k..1M flows
rng = np.random.default_rng(3)
rules = T.make_rules(F, rng, sample_count=10, window_interval_ms=1000)
svc = sa.GpuTokenService(0)
svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                     rules.window_interval_ms, rules.namespace, rules.checker)
dev = torch.device("cuda", 0)
rate = 2.0 * float(rules.count.sum())
out = torch.empty(N, dtype=torch.int64, device=dev)
g = torch.Generator(device=dev).manual_seed(5)
for s in range(4):
    idx = torch.randint(0, F, (N,), dtype=torch.int32, device=dev, generator=g)
    base = torch.arange(s * N, (s + 1) * N, device=dev, dtype=torch.float64)
    ts = (T.T0_ALIGNED + torch.floor(base * (1000.0 / rate))).to(torch.int64)
    evb = device_events(idx, torch.ones(N, dtype=torch.int32, device=dev), ts)
    torch.cuda.synchronize()          # the events are made on torch's stream, decided on the engine's
    svc.submit_flow_batch(evb, verdicts=out)
    svc.synchronize()
nb = 16 * ((977 + 7) // 8)
buf = (C.c_ulonglong * (4096 * 12))()
assert svc._L.sentinel_diag_phases(buf, 4096) == 0
full = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 12)[:nb].astype(np.int64)
print("sequential segments per workgroup (all batches):", full[:, 6].mean(), " heterogeneous:", full[:, 7].mean(),
      " slow because prioritized:", full[:, 8].mean(), " occupy pending:", full[:, 9].mean(),
      " newer slot:", full[:, 10].mean())
a = full[:, :6]
a = a[(a[:, 0] > 0) & (a[:, 3] > 0)]
us = 0.01  # wall_clock64 = 100 MHz
t0 = a[:, 0].min()
print("span us", (a[:, 3].max() - t0) * us)
phases = [("hist+scan", 0, 1), ("sort", 1, 2), ("decide", 2, 3), ("total", 0, 3)]
if (a[:, 4] > 0).all() and (a[:, 5] > 0).all():     # cooperative halves: mark / walk / sweep
    phases += [("  mark", 2, 4), ("  walk", 4, 5), ("  sweep", 5, 3)]
for name, i, j in phases:
    d = (a[:, j] - a[:, i]) * us
    print(f"{name:10s} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  max {d.max():7.2f}")
st = (a[:, 0] - t0) * us
print("start times: quantiles", np.quantile(st, [0, .25, .5, .75, 1]).round(1))
en = (a[:, 3] - t0) * us
print("end times: quantiles", np.quantile(en, [0, .25, .5, .75, 1]).round(1))
