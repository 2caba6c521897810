"""N>1 path on CPU: world_size-2 gloo ranks, each owning the splitmix64(flowId) mod 2 shard.

Each rank decides its shard with the CPU oracle standing in for its GPU (test infrastructure only),
then the verdicts are merged and compared with one sequential replay of the whole trace; the
snapshot records are all-gathered and compared with the single-engine snapshot.  This exercises
the product's routing (sentinel_amd.shard) and its only collective (gather_snapshot).
"""
import os
import socket

import numpy as np
import pytest

from sentinel_amd import shard as SH
from sentinel_amd import trace as T


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rules, ev = T.config2(60_000, seed=42, n_flows=500)
        owner_rule = SH.owner_of(rules.flow_id, world)
        mine = np.nonzero(owner_rule == rank)[0]
        local = rules.subset(mine)
        remap = -np.ones(len(rules), np.int64)
        remap[mine] = np.arange(len(mine))
        owner_ev = owner_rule[ev.flow_idx]
        pos = SH.split_batch(owner_ev, world)[rank]
        orc = O.TokenServiceOracle(local.as_dicts())
        st, rem, _ = orc.replay(remap[ev.flow_idx[pos]].astype(np.int32), ev.acquire[pos], ev.ts[pos])
        t = int(ev.ts[-1]) + 1
        # snapshot rows from the oracle's window dumps (passQps/blockQps at t, no roll needed: t is
        # inside the last window for every flow that was touched last; others are read-only here)
        pq, bq = [], []
        for i in range(len(local)):
            d = orc.dump_flow(i)[: int(local.sample_count[i]) * 8].reshape(-1, 8)
            w = int(local.window_interval_ms[i]) // int(local.sample_count[i])
            E = t // w
            valid = (d[:, 0] >= 0) & (d[:, 0] // w > E - int(local.sample_count[i]))
            I_s = int(local.window_interval_ms[i]) / 1000.0
            pq.append(float(d[valid, 1].sum()) / I_s)
            bq.append(float(d[valid, 2].sum()) / I_s)
        snap = SH.gather_snapshot(SH.snapshot_records(local.flow_id, np.array(pq), np.array(bq)))
        q.put((rank, pos, st, rem, SH.unpack_snapshot(snap)))
    finally:
        dist.destroy_process_group()


def test_two_rank_shard_equals_single_engine():
    import torch.multiprocessing as mp
    from oracle import oracle as O
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x[0])
    rules, ev = T.config2(60_000, seed=42, n_flows=500)
    st = SH.merge_verdicts([r[2] for r in res], [r[1] for r in res], len(ev))
    rem = SH.merge_verdicts([r[3] for r in res], [r[1] for r in res], len(ev))
    st1, rem1, _ = O.TokenServiceOracle(rules.as_dicts()).replay(ev.flow_idx, ev.acquire, ev.ts)
    assert np.array_equal(st, st1) and np.array_equal(rem, rem1)
    # every rank received the same gathered snapshot covering all flows exactly once
    a, b = res[0][4], res[1][4]
    assert np.array_equal(a, b)
    assert sorted(a["flow_id"].tolist()) == sorted(rules.flow_id.tolist())


def test_split_merge_roundtrip():
    rng = np.random.default_rng(0)
    owner = rng.integers(0, 4, size=1000)
    parts = SH.split_batch(owner, 4)
    assert sum(len(p) for p in parts) == 1000
    for p in parts:
        assert np.all(np.diff(p) > 0)          # arrival order kept per rank
    vals = np.arange(1000) * 3
    back = SH.merge_verdicts([vals[p] for p in parts], parts, 1000)
    assert np.array_equal(back, vals)


def test_owner_is_deterministic_and_balanced():
    ids = np.arange(1, 1_000_001, dtype=np.int64)
    o = SH.owner_of(ids, 8)
    counts = np.bincount(o, minlength=8)
    assert counts.min() > 0.98 * counts.mean()
    assert np.array_equal(o, SH.owner_of(ids, 8))


def _param_trace():
    rng = np.random.default_rng(44)
    R = 240
    prules = [dict(flow_id=9000 + 7 * r, count=float(rng.integers(20, 200)), sample_count=4, window_interval_ms=1000)
              for r in range(R)]
    m = 40_000
    ts = T.timestamps(m, 30_000.0, T.T0_ALIGNED + 3)
    ridx = rng.integers(0, R, size=m).astype(np.int32)
    vals = T.zipf_indices(50, 1.3, m, rng, permute=False).astype(np.uint64)
    fids = np.array([p["flow_id"] for p in prules], dtype=np.uint64)
    keys = (fids[ridx] << np.uint64(20)) | vals
    acq = rng.integers(1, 3, size=m).astype(np.int32)
    return prules, ridx, acq, keys, ts


def _param_worker(rank, world, port, q):
    import torch.distributed as dist
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        prules, ridx, acq, keys, ts = _param_trace()
        fids = np.array([p["flow_id"] for p in prules], dtype=np.int64)
        mine = SH.local_rule_subset(fids, rank, world)
        remap = -np.ones(len(prules), np.int64)
        remap[mine] = np.arange(len(mine))
        pos = SH.split_batch(SH.owner_of(fids, world)[ridx], world)[rank]
        orc = O.TokenServiceOracle([], param_rules=[prules[i] for i in mine])
        orc.param_replay(remap[ridx[pos]].astype(np.int32), acq[pos], keys[pos], ts[pos])
        t = int(ts[-1]) + 1
        tops = [orc.param_top_values(i, t) for i in range(len(mine))]
        gathered = SH.gather_param_snapshot(SH.param_snapshot_records(fids[mine], tops))
        q.put((rank, SH.unpack_param_snapshot(gathered)))
    finally:
        dist.destroy_process_group()


def test_two_rank_param_snapshot_equals_single_engine():
    """The snapshot's param leg (ClusterMetricNodeGenerator.paramToMetricNode, top-5 values per param
    rule) all-gathered over two gloo ranks equals one engine's getTopValues for every rule."""
    import torch.multiprocessing as mp
    from oracle import oracle as O
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_param_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    prules, ridx, acq, keys, ts = _param_trace()
    orc = O.TokenServiceOracle([], param_rules=prules)
    orc.param_replay(ridx, acq, keys, ts)
    t = int(ts[-1]) + 1
    want = {p["flow_id"]: orc.param_top_values(i, t) for i, p in enumerate(prules)}
    assert res[0][1] == res[1][1]                  # every rank holds the same gathered snapshot
    assert res[0][1] == want
    assert any(len(v) == 5 for v in want.values())
