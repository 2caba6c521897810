"""Envoy RLS front end (sentinel_amd/rls.py): key/flowId generation, Java HashSet/HashMap iteration
order, rule conversion (CPU), and batched shouldRateLimit parity against the oracle (GPU)."""
import json
import os

import numpy as np
import pytest

from sentinel_amd import rls
from sentinel_amd import trace as T

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_string_hash_matches_java_kat(oracle_mod):
    kat = json.load(open(os.path.join(GOLDEN, "kat_java_numerics.json")))
    for s, h in kat["string_hash"]:
        assert rls.java_string_hash(s) == h
        assert oracle_mod.java_string_hash(s) == h
    key = "testConvertToSentinelFlowRules|k1|v1"
    assert rls.generate_flow_id(key) == 2147483647 + rls.java_string_hash(key)
    assert rls.generate_flow_id("   ") == -1


def _java_hashmap_sim(hashes, initial):
    """Independent model of java.util.HashMap insertion + resize (JDK 8 split keeps relative order)."""
    cap = 1
    while cap < initial:
        cap <<= 1
    buckets = [[] for _ in range(cap)]
    size = 0
    for i, h in enumerate(hashes):
        sp = (h & 0xFFFFFFFF) ^ ((h & 0xFFFFFFFF) >> 16)
        buckets[sp & (cap - 1)].append((i, sp))
        size += 1
        if size > 0.75 * cap:
            old, cap = buckets, cap * 2
            buckets = [[] for _ in range(cap)]
            for b in old:
                for i2, sp2 in b:
                    buckets[sp2 & (cap - 1)].append((i2, sp2))
    return [i for b in buckets for i, _ in b]


def test_hash_iteration_order_model():
    rng = np.random.default_rng(3)
    for n in (1, 2, 5, 12, 13, 30, 100):
        hashes = [int(x) for x in rng.integers(-2**31, 2**31, size=n)]
        for init in (2, 16, n):
            assert rls.java_hash_iteration_order(hashes, init) == _java_hashmap_sim(hashes, init)


def test_rule_conversion_matches_reference_test():
    """EnvoySentinelRuleConverterTest.java:39-71: keys, counts, GLOBAL, sampleCount 1."""
    domain = "testConvertToSentinelFlowRules"
    d1 = rls.ResourceDescriptor([rls.KeyValueResource("k1", "v1")], 10.0)
    d2 = rls.ResourceDescriptor([rls.KeyValueResource("k2", "v2"), rls.KeyValueResource("k3", "v3")], 20.0)
    rules = [rls.to_sentinel_flow_rule(domain, d) for d in (d1, d2)]
    assert rules[0].resource == domain + "|k1|v1" and rules[0].count == 10.0
    assert rules[1].resource == domain + "|k2|v2|k3|v3" and rules[1].count == 20.0
    for r in rules:
        cc = r.cluster_config
        assert cc.threshold_type == 1 and cc.sample_count == 1 and cc.window_interval_ms == 1000
        assert cc.flow_id == rls.generate_flow_id(r.resource)


def test_rule_validity():
    good = rls.EnvoyRlsRule("d", [rls.ResourceDescriptor([rls.KeyValueResource("a", "b")], 1.0)])
    assert rls.is_valid_rule(good)
    assert not rls.is_valid_rule(rls.EnvoyRlsRule(" ", good.descriptors))
    assert not rls.is_valid_rule(rls.EnvoyRlsRule("d", []))
    assert not rls.is_valid_rule(rls.EnvoyRlsRule("d", [rls.ResourceDescriptor([rls.KeyValueResource("a", "b")], -1.0)]))
    assert not rls.is_valid_rule(rls.EnvoyRlsRule("d", [rls.ResourceDescriptor([rls.KeyValueResource("a", "")], 1.0)]))
    assert not rls.is_valid_rule(rls.EnvoyRlsRule("d", [rls.ResourceDescriptor([], 1.0)]))


def _rls_workload(rng, n_domains=6, per_domain=40, n_req=30_000):
    rules = []
    for d in range(n_domains):
        descs = []
        for j in range(per_domain):
            kvs = [rls.KeyValueResource(f"k{m}", f"v{d}_{j}_{m}") for m in range(1 + j % 3)]
            descs.append(rls.ResourceDescriptor(kvs, float(rng.integers(5, 200))))
        rules.append(rls.EnvoyRlsRule(f"domain{d}", descs))
    rules.append(rls.EnvoyRlsRule("domain0", rules[0].descriptors[:1]))     # duplicate domain: ignored
    rules.append(rls.EnvoyRlsRule("", rules[1].descriptors))                # invalid
    reqs = []
    for i in range(n_req):
        d = int(rng.integers(0, n_domains))
        descs = []
        for _ in range(int(rng.integers(1, 4))):
            j = int(rng.integers(0, per_domain + 5))                        # some descriptors have no rule
            if j < per_domain:
                rd = rules[d].descriptors[j]
                descs.append([(r.key, r.value) for r in rd.iteration_order()])
            else:
                descs.append([("unknown", str(j))])
        reqs.append(rls.RateLimitRequest(f"domain{d}", descs, int(min(rng.geometric(0.4), 8)) - 1))
    return rules, reqs


@pytest.mark.gpu
def test_rls_batch_parity(oracle_mod):
    import sentinel_amd as sa
    rng = np.random.default_rng(55)
    rules, reqs = _rls_workload(rng)
    svc = sa.GpuTokenService(0)
    service = rls.SentinelEnvoyRlsService(svc)
    flow_rules = service.load_rules(rules)
    reqs[17].hits_addend = -1                                               # onError
    ts = T.timestamps(len(reqs), 3000.0, T.T0_ALIGNED + 5)
    half = len(reqs) // 2
    got = service.should_rate_limit_batch(reqs[:half], ts[:half]) + service.should_rate_limit_batch(reqs[half:], ts[half:])
    # oracle: the same flattened per-descriptor events through SimpleClusterFlowChecker
    ids = {}
    orc_rules = []
    for fr in flow_rules:
        fid = fr.cluster_config.flow_id
        if fid not in ids:
            ids[fid] = len(orc_rules)
            orc_rules.append(None)
        orc_rules[ids[fid]] = dict(flow_id=fid, count=fr.count, threshold_type=1, sample_count=1,
                                   window_interval_ms=1000, namespace_idx=0, checker=1)
    orc = oracle_mod.TokenServiceOracle(orc_rules)
    idx, acq, tt = [], [], []
    for i, r in enumerate(reqs):
        if r.hits_addend < 0:
            continue
        for e in r.descriptors:
            idx.append(ids.get(rls.generate_flow_id(rls.generate_key(r.domain, e)), -1))
            acq.append(max(r.hits_addend, 1))
            tt.append(ts[i])
    st, rem, _ = orc.replay(np.array(idx), np.array(acq), np.array(tt))
    j = 0
    n_over = 0
    for i, r in enumerate(reqs):
        if r.hits_addend < 0:
            assert isinstance(got[i], ValueError)
            continue
        resp = got[i]
        blocked = False
        for k, e in enumerate(r.descriptors):
            s = 0 if st[j] == 3 else int(st[j])
            blocked |= s != 0
            ds = resp.statuses[k]
            assert ds.code == (rls.Code.OK if s == 0 else rls.Code.OVER_LIMIT)
            if st[j] != 3:
                assert ds.limit_remaining == rem[j]
                assert ds.requests_per_unit == int(orc_rules[idx[j]]["count"])
            else:
                assert ds.requests_per_unit is None
            j += 1
        assert resp.overall_code == (rls.Code.OVER_LIMIT if blocked else rls.Code.OK)
        n_over += blocked
    assert 0 < n_over < len(reqs)


@pytest.mark.gpu
def test_rls_reference_aggregation_cases():
    """SentinelEnvoyRlsServiceImplTest.java:40-118: all-OK -> OK; one blocked descriptor -> OVER_LIMIT overall."""
    import sentinel_amd as sa
    svc = sa.GpuTokenService(0)
    service = rls.SentinelEnvoyRlsService(svc)
    service.load_rules([rls.EnvoyRlsRule("testShouldRatePartialBlock", [
        rls.ResourceDescriptor([rls.KeyValueResource("a1", "b1")], 0.0),
        rls.ResourceDescriptor([rls.KeyValueResource("a2", "b2"), rls.KeyValueResource("a3", "b3")], 10.0)])])
    t = T.T0_ALIGNED
    ok = service.should_rate_limit(rls.RateLimitRequest("testShouldRateLimitPass", [[("a1", "b1")], [("a2", "b2"), ("a3", "b3")]], 1), t)
    assert ok.overall_code == rls.Code.OK and all(s.code == rls.Code.OK for s in ok.statuses)
    part = service.should_rate_limit(rls.RateLimitRequest("testShouldRatePartialBlock",
                                                          [[("a1", "b1")], [("a2", "b2"), ("a3", "b3")]], 1), t)
    assert part.overall_code == rls.Code.OVER_LIMIT and len(part.statuses) == 2
    assert [s.code for s in part.statuses] == [rls.Code.OVER_LIMIT, rls.Code.OK]
