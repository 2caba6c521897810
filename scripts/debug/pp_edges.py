"""Debug: the param edge-case trace through every param path, mismatch details."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sentinel_amd import trace as T
from oracle import oracle as O
import sentinel_amd as sa
from sentinel_amd.token_service import ServerNamespace

path = sys.argv[1]
os.environ["SENTINEL_PARAM_PATH"] = path
R = 64
rng = np.random.default_rng(29)
prules = [dict(flow_id=500 + r, count=float(rng.integers(3, 400)), sample_count=(2, 4, 5, 10)[r % 4],
               window_interval_ms=1000) for r in range(R)]
fids = np.array([r["flow_id"] for r in prules], dtype=np.uint64)
hot_key = int((fids[3] << np.uint64(32)) | np.uint64(7))
prules[3]["hot"] = {hot_key: 50_000}
svc = sa.GpuTokenService(0)
svc.set_namespaces([ServerNamespace()])
svc.load_param_rules([sa.ParamFlowRule(count=r["count"], cluster_config=sa.ClusterFlowConfig(
    flow_id=r["flow_id"], threshold_type=1, sample_count=r["sample_count"],
    window_interval_ms=r["window_interval_ms"]), hot_items=r.get("hot", {})) for r in prules])
orc = O.TokenServiceOracle([], param_rules=prules, hot_items={3: [(hot_key, 50_000)]})
t0 = T.T0_ALIGNED + 13
for batch in range(2):
    m = 60_000
    ts = np.sort(t0 + rng.integers(0, 3000, size=m)).astype(np.int64)
    ts[m // 2:] += 20 * 3600 * 1000
    ridx = rng.integers(0, R, size=m).astype(np.int32)
    vals = T.zipf_indices(400, 1.1, m, rng, permute=False).astype(np.uint64)
    keys = (fids[ridx] << np.uint64(32)) | vals
    hot = rng.random(m) < 0.5
    ridx[hot] = 3
    keys[hot] = hot_key
    acq = np.where(rng.random(m) < 0.1, rng.integers(400, 3000, size=m), 1).astype(np.int32)
    bad = rng.random(m)
    acq[bad < 0.002] = 0
    ridx[(bad >= 0.002) & (bad < 0.004)] = R + 5
    ts[(bad >= 0.004) & (bad < 0.005)] = -1
    st_g, rem_g = svc.submit_param_batch_host(ridx, acq, keys, ts)
    st_o, rem_o = orc.param_replay(ridx, acq, keys, ts)
    mis = np.nonzero((st_g != st_o) | (rem_g != rem_o))[0]
    print(path, "batch", batch, "mismatches", len(mis), "table", svc.param_table_stats())
    for i in mis[:12]:
        print("  i", i, "ts", ts[i], "acq", acq[i], "rule", ridx[i], "hot", bool(hot[i]), "key", hex(int(keys[i])),
              "gpu", st_g[i], rem_g[i], "orc", st_o[i], rem_o[i])
    if len(mis):
        print("  mismatch hot frac", hot[mis].mean(), "acq>=511 frac", (acq[mis] >= 511).mean(),
              "second half frac", (mis >= m // 2).mean())
    t0 = int(ts.max()) + 1
