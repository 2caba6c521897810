"""Host-fed path study: synchronous 1M batches vs the streamed (pipelined) path, warm.
Run under rocprofv3 --kernel-trace --memory-copy-trace to see copy/kernel overlap."""
import ctypes as C
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import sentinel_amd as sa
from sentinel_amd import trace as T
from sentinel_amd.token_service import device_events

F, N, m = 1_000_000, 8 << 20, 1 << 20
rng = np.random.default_rng(3)
rules = T.make_rules(F, rng, sample_count=10, window_interval_ms=1000)
svc = sa.GpuTokenService(0)
svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                     rules.window_interval_ms, rules.namespace, rules.checker)
dev = torch.device("cuda", 0)
idx = torch.randint(0, F, (N,), dtype=torch.int32, device=dev)
ms_per_event = 1000.0 / (2.0 * float(rules.count.sum()))
ts = (T.T0_ALIGNED + torch.floor(torch.arange(N, device=dev, dtype=torch.float64) * ms_per_event)).to(torch.int64)
ev = device_events(idx, torch.ones(N, dtype=torch.int32, device=dev), ts)
hev = torch.empty((N, 2), dtype=torch.int64, pin_memory=True)
hev.copy_(ev)
hout = torch.empty(N, dtype=torch.int64, pin_memory=True)
L, h = svc._L, svc.handle
bms = np.zeros(N // m, np.float32)
hts = hev[:, 1].numpy()
span = int(np.ceil(N * ms_per_event)) + 1


def advance():
    """every pass decides a later stretch of time (the clock never goes backwards)"""
    global hts
    hts += span


for rep in range(2):
    advance()
    t = time.perf_counter()
    for i in range(N // m):
        assert L.sentinel_submit_flow_batch_host(h, m, C.c_void_p(hev.data_ptr() + i * m * 16), None,
                                                 C.c_void_p(hout.data_ptr() + i * m * 8)) == 0
    print("sync  ", rep, round(N / (time.perf_counter() - t) / 1e9, 3), "e9/s", flush=True)
for bm in (None, bms):
    for b in (m, m // 2, 2 * m):
        for rep in range(2):
            advance()
            t = time.perf_counter()
            assert L.sentinel_submit_flow_stream_host(h, N, C.c_void_p(hev.data_ptr()), None, C.c_void_p(hout.data_ptr()),
                                                      b, None if bm is None else C.c_void_p(bms.ctypes.data)) == 0
            print("stream", b, bm is not None, rep, round(N / (time.perf_counter() - t) / 1e9, 3), "e9/s", flush=True)
# copy-only bandwidth for reference
d = torch.empty((N, 2), dtype=torch.int64, device=dev)
torch.cuda.synchronize(); t = time.perf_counter(); d.copy_(hev, non_blocking=True); torch.cuda.synchronize()
print("H2D GB/s", round(N * 16 / (time.perf_counter() - t) / 1e9, 1))
o = torch.empty(N, dtype=torch.int64, device=dev)
torch.cuda.synchronize(); t = time.perf_counter(); hout.copy_(o, non_blocking=True); torch.cuda.synchronize()
print("D2H GB/s", round(N * 8 / (time.perf_counter() - t) / 1e9, 1))
