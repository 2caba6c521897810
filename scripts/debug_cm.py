"""Debug: shared count-min violations -- which events pass on the sketch but fail on exact counters."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sentinel_amd as sa
from sentinel_amd import trace as T
from sentinel_amd.token_service import ServerNamespace

count, hot, rule_idx, vals, keys, ts = T.config4(200_000, seed=53, n_rules=5000, universe=200)
R = len(count)
svc = sa.GpuTokenService(0)
svc.set_namespaces([ServerNamespace()])
svc.load_param_rules([sa.ParamFlowRule(count=float(count[r]), cluster_config=sa.ClusterFlowConfig(
    flow_id=r + 1, threshold_type=1, sample_count=10, window_interval_ms=1000), hot_items=hot.get(r, {})) for r in range(R)])
svc.set_param_mode(sa._lib.PARAM_COUNT_MIN_SHARED, depth=4, width=1 << 10)
acq = np.ones(len(ts), np.int32)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000
st = np.concatenate([svc.submit_param_batch_host(rule_idx[i:i + B], acq[i:i + B], keys[i:i + B], ts[i:i + B])[0]
                     for i in range(0, len(ts), B)])
E = ts // 100
exact = {}
viol = []
for i in range(len(ts)):
    k = int(keys[i]); e = int(E[i]); r = int(rule_idx[i])
    ex = sum(c for (ee, c) in exact.get(k, []) if e - 10 < ee <= e)
    thr = float(hot.get(r, {}).get(k, count[r]))
    ex_pass = (thr - ex) - 1 >= 0
    if st[i] == 0:
        if not ex_pass:
            viol.append(i)
        exact.setdefault(k, []).append((e, 1))
print("statuses", {int(s): int((st == s).sum()) for s in np.unique(st)})
print("violations", len(viol))
for i in viol[:12]:
    k = int(keys[i]); r = int(rule_idx[i]); e = int(E[i])
    prev = [j for j in range(i) if keys[j] == keys[i]]
    print(f"i={i} batch={i // B} rule={r} key={k:#x} E={e} thr={float(hot.get(r, {}).get(k, count[r]))} "
          f"prev_events={[(j, int(E[j]), int(st[j])) for j in prev[-6:]]}")
