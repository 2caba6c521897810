"""Seeded synthetic workloads for BASELINE.json's configs.

A trace is a rule table plus events in arrival order: (flow_idx, acquire, flags, ts).  Timestamps
are non-decreasing milliseconds, i.e. the value TimeUtil.currentTimeMillis() would return when the
request reaches DefaultTokenService (sentinel-core/.../util/TimeUtil.java:49-51).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

T0_ALIGNED = 1_600_000_000_000


def splitmix64(x: np.ndarray) -> np.ndarray:
    """flowId -> shard hash (gpu = splitmix64(flowId) mod G)."""
    z = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15))
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def shard_of(flow_ids, world: int) -> np.ndarray:
    return (splitmix64(flow_ids) % np.uint64(world)).astype(np.int64)


@dataclass
class Rules:
    flow_id: np.ndarray
    count: np.ndarray
    threshold_type: np.ndarray
    sample_count: np.ndarray
    window_interval_ms: np.ndarray
    namespace: np.ndarray
    checker: np.ndarray

    def __len__(self):
        return len(self.flow_id)

    def as_dicts(self):
        return [dict(flow_id=int(self.flow_id[i]), count=float(self.count[i]),
                     threshold_type=int(self.threshold_type[i]), sample_count=int(self.sample_count[i]),
                     window_interval_ms=int(self.window_interval_ms[i]), namespace_idx=int(self.namespace[i]),
                     checker=int(self.checker[i])) for i in range(len(self))]

    def subset(self, idx):
        return Rules(*(getattr(self, f)[idx] for f in
                       ("flow_id", "count", "threshold_type", "sample_count", "window_interval_ms", "namespace",
                        "checker")))


@dataclass
class Events:
    flow_idx: np.ndarray    # int32
    acquire: np.ndarray     # int32
    ts: np.ndarray          # int64
    flags: Optional[np.ndarray] = None   # uint8

    def __len__(self):
        return len(self.ts)

    def slice(self, a, b):
        return Events(self.flow_idx[a:b], self.acquire[a:b], self.ts[a:b],
                      None if self.flags is None else self.flags[a:b])


def make_rules(n_flows: int, rng: np.random.Generator, count_lo=10, count_hi=1000, threshold_type=1,
               sample_count=2, window_interval_ms=1000, namespace=0, checker=0, flow_id_base=1,
               integral=True) -> Rules:
    if integral:
        count = rng.integers(count_lo, count_hi + 1, size=n_flows).astype(np.float64)
    else:
        count = rng.uniform(count_lo, count_hi, size=n_flows)
    full = lambda v, dt: np.full(n_flows, v, dtype=dt)
    return Rules(flow_id=np.arange(flow_id_base, flow_id_base + n_flows, dtype=np.int64), count=count,
                 threshold_type=full(threshold_type, np.int32), sample_count=full(sample_count, np.int32),
                 window_interval_ms=full(window_interval_ms, np.int32), namespace=full(namespace, np.int32),
                 checker=full(checker, np.int32))


def zipf_indices(n_items: int, s: float, size: int, rng: np.random.Generator, permute=True) -> np.ndarray:
    """Bounded Zipf(s) over n_items by inverse CDF; ranks randomly permuted over item indices."""
    w = 1.0 / np.power(np.arange(1, n_items + 1, dtype=np.float64), s)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    r = np.searchsorted(cdf, rng.random(size), side="right")
    r = np.minimum(r, n_items - 1)
    if permute:
        perm = rng.permutation(n_items)
        r = perm[r]
    return r.astype(np.int32)


def timestamps(n: int, rate_per_s: float, t0: int) -> np.ndarray:
    """Arrival i at t0 + floor(i * 1000 / rate): non-decreasing ms."""
    return (t0 + np.floor(np.arange(n, dtype=np.float64) * (1000.0 / rate_per_s))).astype(np.int64)


def config2(n_events: int, seed: int = 2, n_flows: int = 10_000, t0: int = T0_ALIGNED, zipf_s: float = 1.1,
            sample_count: int = 2, window_interval_ms: int = 1000, offered_ratio: float = 2.0):
    """Cluster token server, 10k flowIds, QPS grade, 1 s / 2-bucket window, Zipf(1.1) requests."""
    rng = np.random.default_rng(seed)
    rules = make_rules(n_flows, rng, sample_count=sample_count, window_interval_ms=window_interval_ms)
    rate = offered_ratio * float(rules.count.sum())
    ev = Events(flow_idx=zipf_indices(n_flows, zipf_s, n_events, rng), acquire=np.ones(n_events, np.int32),
                ts=timestamps(n_events, rate, t0))
    return rules, ev


def config3(n_events: int, seed: int = 3, n_flows: int = 1_000_000, t0: int = T0_ALIGNED, sample_count: int = 10,
            window_interval_ms: int = 1000, offered_ratio: float = 2.0):
    """1M flowIds, uniform, default cluster window n=10 / w=100 ms."""
    rng = np.random.default_rng(seed)
    rules = make_rules(n_flows, rng, sample_count=sample_count, window_interval_ms=window_interval_ms)
    rate = offered_ratio * float(rules.count.sum())
    ev = Events(flow_idx=rng.integers(0, n_flows, size=n_events, dtype=np.int32),
                acquire=np.ones(n_events, np.int32), ts=timestamps(n_events, rate, t0))
    return rules, ev


def config5(n_events: int, seed: int = 5, n_flows: int = 2_000, t0: int = T0_ALIGNED, p: float = 0.3,
            cap: int = 64, offered_ratio: float = 2.0):
    """Envoy RLS rules (SimpleClusterFlowChecker, n=1, w=1000, GLOBAL) with heterogeneous
    hitsAddend ~ geometric(0.3) capped at 64 (EnvoySentinelRuleConverter.java:57-64)."""
    rng = np.random.default_rng(seed)
    rules = make_rules(n_flows, rng, count_lo=50, count_hi=5000, sample_count=1, window_interval_ms=1000, checker=1)
    acq = np.minimum(rng.geometric(p, size=n_events), cap).astype(np.int32)
    rate = offered_ratio * float(rules.count.sum()) / float(acq.mean())
    ev = Events(flow_idx=zipf_indices(n_flows, 1.1, n_events, rng), acquire=acq, ts=timestamps(n_events, rate, t0))
    return rules, ev


def config4(n_events: int, seed: int = 4, n_rules: int = 100_000, universe: int = 1000, zipf_s: float = 1.2,
            t0: int = T0_ALIGNED, hot_frac: float = 0.01, offered_ratio: float = 2.0):
    """Hot-parameter cluster rules: 100k resources x Zipf(1.2) over 1000 values each.
    Param key = (rule index << 20) | value index: injective per (rule, value)."""
    rng = np.random.default_rng(seed)
    count = rng.integers(5, 101, size=n_rules).astype(np.float64)
    rule_idx = rng.integers(0, n_rules, size=n_events, dtype=np.int32)
    vals = zipf_indices(universe, zipf_s, n_events, rng, permute=False)
    keys = (rule_idx.astype(np.uint64) << np.uint64(20)) | vals.astype(np.uint64)
    hot = {}
    n_hot = max(1, int(hot_frac * universe))
    for r in range(min(n_rules, 64)):
        for v in range(n_hot):
            hot.setdefault(r, {})[int((np.uint64(r) << np.uint64(20)) | np.uint64(v))] = int(rng.integers(1, 20))
    rate = offered_ratio * float(count.sum()) * 0.05
    ts = timestamps(n_events, rate, t0)
    return count, hot, rule_idx, vals, keys, ts


def param_value_lists(rule_idx: np.ndarray, rng: np.random.Generator, universe: int = 300, zipf_s: float = 1.2,
                      max_values: int = 4):
    """Value lists for multi-value param requests (1..max_values values each, Zipf over a per-rule
    universe, repeats allowed).  Returns (value_begin, value_count, keys) with key = (rule << 20) | value."""
    n = len(rule_idx)
    counts = rng.integers(1, max_values + 1, size=n).astype(np.int32)
    begin = np.zeros(n, dtype=np.int32)
    if n:
        begin[1:] = np.cumsum(counts)[:-1]
    vals = zipf_indices(universe, zipf_s, int(counts.sum()), rng, permute=False)
    owner = np.repeat(np.asarray(rule_idx, dtype=np.int64), counts)
    keys = (owner.astype(np.uint64) << np.uint64(20)) | vals.astype(np.uint64)
    return begin, counts, keys


def config1(seed: int = 1, t0: int = T0_ALIGNED, duration_ms: int = 100_000, threads: int = 32):
    """FlowQpsDemo traffic (FlowQpsDemo.java:132-157): `threads` workers loop SphU.entry("abc")
    then sleep U[0, 50) ms, for `duration_ms`.  Returns the merged entry timestamps (arrival order:
    time, then worker) -- one resource, acquire 1."""
    rng = np.random.default_rng(seed)
    ts = []
    for w in range(threads):
        t = t0
        out = []
        while t < t0 + duration_ms:
            out.append(t)
            t += int(rng.integers(0, 50))
        ts.append(np.array(out, dtype=np.int64))
    allt = np.concatenate(ts)
    worker = np.concatenate([np.full(len(x), i) for i, x in enumerate(ts)])
    order = np.lexsort((worker, allt))
    return allt[order]
