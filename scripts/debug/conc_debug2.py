"""Debug: minimal release cases on the device and host concurrency paths."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import sentinel_amd as sa  # noqa: E402

dev = torch.device("cuda", 0)
for path in ("host", "device"):
    for nacq in (10, 200):
        svc = sa.GpuTokenService(0)
        svc.load_flow_rules([sa.FlowRule(count=1000, cluster_config=sa.ClusterFlowConfig(flow_id=7, threshold_type=1))])

        def run(fidx, acq, tok, kind):
            fidx, acq, tok, kind = (np.asarray(x) for x in (fidx, acq, tok, kind))
            flags = np.ones(len(kind), np.int32)
            if path == "host":
                return svc.submit_concurrent_batch_host(fidx, acq, tok, kind, flags)
            t = lambda a, d: torch.from_numpy(np.ascontiguousarray(a, dtype=d)).to(dev)   # noqa: E731
            ev = svc.concurrent_events(t(fidx, np.int32), t(acq, np.int32), t(tok, np.int64), t(kind, np.int32),
                                       t(flags, np.int32))
            res = torch.full((len(kind), 2), -99, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            svc.submit_concurrent_batch(ev, results=res)
            svc.synchronize()
            r = res.cpu().numpy()
            return r[:, 1], r[:, 0]
        st, tok = run(np.zeros(nacq, np.int32), np.ones(nacq, np.int32), np.zeros(nacq, np.int64), np.zeros(nacq, np.int32))
        print(path, nacq, "acquire statuses", np.unique(st, return_counts=True), "now", svc.concurrent_now_calls(0))
        # release each token twice, interleaved, plus an unknown token
        rel = np.concatenate([tok, tok, [12345]])
        st2, _ = run(np.zeros(len(rel), np.int32), np.zeros(len(rel), np.int32), rel, np.ones(len(rel), np.int32))
        print(path, nacq, "release statuses first half", np.unique(st2[:nacq], return_counts=True),
              "second half", np.unique(st2[nacq:2 * nacq], return_counts=True), "unknown", st2[-1],
              "now", svc.concurrent_now_calls(0), "count", svc.concurrent_token_count())
        svc.close()

# state dump of a 400-release batch on the device path
svc = sa.GpuTokenService(0)
svc.load_flow_rules([sa.FlowRule(count=1000, cluster_config=sa.ClusterFlowConfig(flow_id=7, threshold_type=1))])
st, tok = svc.submit_concurrent_batch_host(np.zeros(200, np.int32), np.ones(200, np.int32), np.zeros(200, np.int64),
                                           np.zeros(200, np.int32), np.ones(200, np.int32))
rel = np.concatenate([tok, tok])
n = len(rel)
t = lambda a, d: torch.from_numpy(np.ascontiguousarray(a, dtype=d)).to(dev)   # noqa: E731
ev = svc.concurrent_events(t(np.zeros(n), np.int32), t(np.zeros(n), np.int32), t(rel, np.int64), t(np.ones(n), np.int32),
                           t(np.ones(n), np.int32))
res = torch.full((n, 2), -99, dtype=torch.int64, device=dev)
torch.cuda.synchronize()
svc.submit_concurrent_batch(ev, results=res)
svc.synchronize()
r = res.cpu().numpy()
import ctypes as C  # noqa: E402
skey = np.zeros(n, np.uint32)
sval = np.zeros(n, np.uint64)
rs = np.zeros(n + 1, np.uint32)
ctl = np.zeros(4, np.uint32)
rsl = np.zeros(n, np.uint32)
svc._L.sentinel_debug_conc_state(svc.handle, C.c_int64(n), C.c_void_p(skey.ctypes.data), C.c_void_p(sval.ctypes.data),
                                 C.c_void_p(rs.ctypes.data), C.c_void_p(ctl.ctypes.data), C.c_void_p(rsl.ctypes.data))
seq = (sval & np.uint64((1 << 28) - 1)).astype(np.int64)
print("ctl", ctl, "runs", rs[:ctl[0] + 1], "keys", np.unique(skey, return_counts=True))
print("seq sorted?", bool((np.diff(seq) > 0).all()), "unique seq", len(np.unique(seq)), "first seqs", seq[:8], "last", seq[-8:])
print("statuses", np.unique(r[:, 1], return_counts=True))
print("unwritten positions", np.nonzero(r[:, 1] == -99)[0][:20])
print("relslot of 0..3 and 200..203", rsl[:4], rsl[200:204])
print("positions with 7:", np.nonzero(r[:, 1] == 7)[0], " with 6: range", np.nonzero(r[:, 1] == 6)[0][[0, -1]],
      " unwritten range", (np.nonzero(r[:, 1] == -99)[0][[0, -1]] if (r[:, 1] == -99).any() else None))
print("tokens of 7-positions", r[r[:, 1] == 7, 0][:4])
if os.environ.get("SENTINEL_LIB", "").endswith("lib_trace.so"):
    tr = sval
    kinds = (tr >> np.uint64(32)) & np.uint64(0xFF)
    seqs = tr & np.uint64(0xFFFFFFFF)
    thr_ = tr >> np.uint64(40)
    print("trace: kinds", np.unique(kinds, return_counts=True))
    print("items 196..204: kind", kinds[196:205], "seq", seqs[196:205], "thread", thr_[196:205])
    print("items written (not all-ones):", int((tr != np.uint64(0xFFFFFFFFFFFFFFFF)).sum()))
