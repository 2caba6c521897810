"""Cost diagnostic for k_pp_decide (needs a -DSENTINEL_DIAG_PHASES build in SENTINEL_LIB): per-workgroup
wall-clock phase sums on the config-4 bench workload (a few batches, the last one's stamps)."""
import ctypes as C
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

args = types.SimpleNamespace(config="4", flows=None, events_per_gpu=None, sample_count=None, interval_ms=1000)
W = bench.ParamWorkload(args, 1, 0, torch.device("cuda", 0))
L = W.svc._L
nb = 1024
buf = (C.c_ulonglong * (4096 * 12))()
for s in range(6):
    b = W.batch(s)
    torch.cuda.synchronize()
    if s == 5:
        L.sentinel_diag_phases_clear()
    W.submit(b)
    W.svc.synchronize()
assert L.sentinel_diag_phases(buf, 4096) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 12)[:nb].astype(np.int64)
a = a[(a[:, 0] > 0) & (a[:, 3] > 0)]
us = 0.01  # wall_clock64 = 100 MHz
t0 = a[:, 0].min()
print("workgroups", len(a), "span us", (a[:, 3].max() - t0) * us)
for name, i in (("load+lds table", 4), ("rank+scan+place", 5), ("walk", 6)):
    d = a[:, i] * us
    print(f"{name:16s} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  max {d.max():7.2f}")
d = (a[:, 3] - a[:, 0]) * us
print(f"{'total':16s} mean {d.mean():7.2f} us  p50 {np.median(d):7.2f}  max {d.max():7.2f}")
print("rounds per wg", a[:, 7].mean(), " distinct keys per wg", a[:, 8].mean())
st = (a[:, 0] - t0) * us
print("start quantiles", np.quantile(st, [0, .25, .5, .75, 1]).round(1))
