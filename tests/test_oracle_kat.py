"""Pin the CPU oracle against the reference's own known-answer tests (tests/golden/kat_*.json).

Each fixture is a transcription of a reference JUnit test (file:line in its "source" field),
with the PowerMock'd clock (AbstractTimeBasedTest) replaced by explicit timestamps.
"""
import json
import math
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


EV = {"PASS": 0, "BLOCK": 1, "PASS_REQUEST": 2, "BLOCK_REQUEST": 3, "OCCUPIED_PASS": 4,
      "OCCUPIED_BLOCK": 5, "WAITING": 6}


def run_ops(o, ops, t0, keys=None):
    t = t0
    cm = pm = lim = None
    for op in ops:
        k = op["op"]
        if k == "sleep":
            t += op["ms"]
        elif k == "align":
            t -= t % op["w"]
        elif k == "cm_new":
            cm = o.ClusterMetric(op["n"], op["interval"])
        elif k == "cm_add":
            cm.add(t, EV[op["event"]], op["count"])
        elif k == "cm_touch":
            cm.window_start(t)
        elif k == "cm_sum":
            assert cm.get_sum(t, EV[op["event"]]) == op["expect"], op
        elif k == "cm_current":
            assert cm.get_current_count(t, EV[op["event"]]) == op["expect"], op
        elif k == "cm_avg":
            assert abs(cm.get_avg(t, EV[op["event"]]) - op["expect"]) <= op["tol"], op
        elif k == "cm_occupy":
            assert cm.try_occupy_next(t, EV[op["event"]], op["acquire"], op["threshold"]) == op["expect"], op
        elif k == "cm_list_count":
            assert cm.list_count(t) == op["expect"], op
        elif k == "cm_first_count":
            assert cm.first_count(t, EV[op["event"]]) == op["expect"], op
        elif k == "cm_window_start":
            w = op["w"]
            expect = {"t-t%w": t - t % w, "t": t, "t-500": t - 500}[op["expect"]]
            assert cm.window_start(t) == expect, op
        elif k == "pm_new":
            pm = o.ClusterParamMetric(op["n"], op["interval"], op["cap"])
        elif k == "pm_add":
            pm.add_value(t, keys[op["key"]], op["count"])
        elif k == "pm_sum":
            assert pm.get_sum(t, keys[op["key"]]) == op["expect"], op
        elif k == "pm_avg":
            assert abs(pm.get_avg(t, keys[op["key"]]) - op["expect"]) <= op["tol"], op
        elif k == "pm_top":
            got = pm.top_values(t, op["number"])
            assert got == {keys[kk]: v for kk, v in op["expect"].items()}, (op, got)
        elif k == "pm_top_illegal":
            with pytest.raises(ValueError):
                pm.top_values(t, op["number"])
        elif k == "lim_new":
            lim = o.RequestLimiter(op["qps"])
        elif k == "lim_add":
            lim.add(t, op["x"])
        elif k == "lim_can_pass":
            assert lim.can_pass(t) == op["expect"], op
        elif k == "lim_try_pass":
            assert lim.try_pass(t) == op["expect"], op
        elif k == "lim_sum":
            assert lim.get_sum(t) == op["expect"], op
        elif k == "lim_qps":
            assert abs(lim.get_qps(t) - op["expect"]) <= op["tol"], op
        else:
            raise KeyError(k)


def test_kat_cluster_metric(oracle_mod):
    kat = load("kat_cluster_metric.json")
    for t0 in kat["t0"]:
        run_ops(oracle_mod, kat["ops"], t0)


def test_kat_cluster_param_metric(oracle_mod):
    kat = load("kat_cluster_param_metric.json")
    for t0 in kat["t0"]:
        run_ops(oracle_mod, kat["ops"], t0, kat["keys"])


@pytest.mark.parametrize("fixture", ["kat_request_limiter.json", "kat_leap_array.json"])
def test_kat_cases(oracle_mod, fixture):
    kat = load(fixture)
    for case in kat["cases"]:
        for t0 in kat["t0"]:
            run_ops(oracle_mod, case["ops"], t0)


def _occ_ops(node, ops, t0):
    for op in ops:
        k, t = op["op"], t0 + op.get("dt", 0)
        if k == "add_pass":
            node.window_add_pass(t, op["n"])
        elif k == "window_pass":
            assert node.window_pass(t) == op["expect"], op
        elif k == "add_waiting":
            node.add_waiting(t, op["n"])
        elif k == "waiting":
            assert node.waiting(t0) == op["expect"], op          # currentWaiting() at the mocked clock
        elif k == "touch":
            node.window_pass(t)                                   # leapArray.currentWindow(t)
        elif k == "values":
            assert node.values(t) == (op["expect_size"], op["expect_sum"]), op
        elif k == "values_aligned":
            assert node.values(t0 - t0 % 200 + 2000) == (op["expect_size"], op["expect_sum"]), op
        else:
            raise KeyError(k)


def test_kat_occupiable_bucket_leap_array(oracle_mod):
    kat = load("kat_occupiable_bucket_leap_array.json")
    w = kat["window"]
    for case in kat["cases"]:
        for t0 in kat["t0"]:
            node = oracle_mod.StatisticNode(kat["n"], kat["interval"])
            for _ in range(case.get("repeat", 1)):
                _occ_ops(node, case["ops"], t0)
            for i in range(case.get("steps", 0)):                 # testWindowAfterOneInterval's loop
                node.window_add_pass(t0 + i * w, 1)
                node.add_waiting(t0 + (i + 1) * w, 1)
            _occ_ops(node, case.get("after", []), t0)


def test_kat_default_controller(oracle_mod):
    kat = load("kat_default_controller.json")
    for case in kat["mocked"]:
        got = [oracle_mod.default_controller_check(v, case["count"], case["grade"], case["acquire"])
               for v in case["values"]]
        assert got == case["expect"], case["name"]
    for case in kat["integration"]:
        for t0 in case["t0"]:
            node = oracle_mod.StatisticNode(2, 1000)
            got, t = [], t0
            for dt, acq in zip(case["dts"], case["acquire"]):
                t += dt
                ok = node.can_pass(case["count"], acq, t)
                (node.add_pass_request if ok else node.increase_block_qps)(t, acq)
                got.append(ok)
            assert got == case["expect"], case["name"]


def test_kat_param_default_checker(oracle_mod):
    kat = load("kat_param_default_checker.json")
    for case in kat["cases"]:
        for t0 in kat["t0"]:
            b = oracle_mod.ParamTokenBucket()
            t = t0
            for i, (dt, expect) in enumerate(case["steps"]):
                t += dt
                got = b.pass_default(7, case["token_count"], case["burst"], case["duration"], 1, t)
                assert got == int(expect), (case["name"], i)


def test_kat_cluster_flow_checker_nonauthoritative(oracle_mod):
    kat = load("kat_cluster_flow_checker.json")
    names = {"OK": 0, "BLOCKED": 1, "SHOULD_WAIT": 2}
    for t0 in kat["t0"]:
        svc = oracle_mod.TokenServiceOracle([kat["rule"]])
        t = t0
        for i, step in enumerate(kat["steps"]):
            t += step[0]
            st, rem, wait = svc.request_token(0, 1, step[1], t)
            assert st == names[step[2]], (i, st)
            if len(step) > 3:
                assert wait == step[3]


def test_kat_java_numerics(oracle_mod):
    kat = load("kat_java_numerics.json")
    for s, h in kat["string_hash"]:
        assert oracle_mod.java_string_hash(s) == h
    for d, i in kat["d2i"]:
        d = math.nan if d == "nan" else d
        assert oracle_mod.lib().orc_java_d2i(d) == i


def test_mt_replay_equals_sequential(oracle_mod):
    """The multi-threaded CPU baseline (flow-sharded) is the same replay as the sequential oracle."""
    from sentinel_amd import trace as T
    rules, ev = T.config2(200_000, seed=9, n_flows=2000)
    a = oracle_mod.TokenServiceOracle(rules.as_dicts()).replay(ev.flow_idx, ev.acquire, ev.ts)
    b = oracle_mod.TokenServiceOracle(rules.as_dicts()).replay_mt(ev.flow_idx, ev.acquire, ev.ts, 4)
    assert b[3] == 4
    for x, y in zip(a, b[:3]):
        assert (x == y).all()


def test_param_mt_replay_equals_sequential(oracle_mod):
    """Config 4's multi-threaded CPU baseline (rule-sharded) is the same replay as the sequential oracle."""
    from sentinel_amd import trace as T
    count, hot, rule_idx, vals, keys, ts = T.config4(200_000, seed=12, n_rules=3000, universe=200)
    prules = [dict(flow_id=r + 1, count=float(count[r]), threshold_type=1, sample_count=10, window_interval_ms=1000)
              for r in range(len(count))]
    acq = np.ones(len(ts), np.int32)

    def orc():
        return oracle_mod.TokenServiceOracle([], param_rules=prules, hot_items={r: list(h.items()) for r, h in hot.items()})
    a = orc().param_replay(rule_idx, acq, keys, ts)
    s, r, used = orc().param_replay_mt(rule_idx, acq, keys, ts, 4)
    assert used == 4 and (a[0] == s).all() and (a[1] == r).all()
    assert (s == 0).any() and (s == 1).any()


def test_concurrent_mt_replay_equals_sequential(oracle_mod):
    """Config 5conc's multi-threaded CPU baseline (flow-sharded, a token cache per thread, releases routed to
    the thread that issued their token) answers exactly as the sequential replay, over several batches."""
    from sentinel_amd import trace as T
    rng = np.random.default_rng(31)
    F, n, nb = 500, 20_000, 4
    rules = [dict(flow_id=f + 1, count=float(rng.integers(1, 40)), threshold_type=1, sample_count=10,
                  window_interval_ms=1000, namespace_idx=0, checker=0) for f in range(F)]
    ref = oracle_mod.TokenServiceOracle(rules)
    evs, ids = [], []
    outstanding = np.zeros(0, np.int64)
    next_id = 1
    for b in range(nb):
        ev = np.zeros(n, dtype=ref.CONC_EVENT)
        kind = (rng.random(n) < 0.45).astype(np.int32) if len(outstanding) else np.zeros(n, np.int32)
        ev["kind"] = kind
        ev["flow_idx"] = T.zipf_indices(F, 1.1, n, rng)
        ev["acquire"] = rng.integers(1, 3, size=n)
        ev["flags"] = 1
        rel = np.nonzero(kind == 1)[0]
        if len(rel):
            ev["token_id"][rel] = outstanding[rng.integers(0, len(outstanding), size=len(rel))]
        nid = np.arange(next_id, next_id + n, dtype=np.int64)
        next_id += n
        st, tok = ref.concurrent_replay(ev, nid)
        ids.append(np.where(st == 0, nid, 0))               # the engine's ids of the passing acquires
        evs.append((ev, st))
        released = set(ev["token_id"][(kind == 1) & (st == 6)].tolist())
        outstanding = np.array([t for t in outstanding.tolist() if t not in released] + tok[st == 0].tolist(), np.int64)
    all_ev = np.concatenate([e for e, _ in evs])
    st_mt, tok_mt, used = oracle_mod.TokenServiceOracle(rules).concurrent_replay_mt(all_ev, np.concatenate(ids), 4)
    assert used == 4
    assert (st_mt == np.concatenate([s for _, s in evs])).all()
    assert {0, 1, 6, 7} <= set(np.unique(st_mt).tolist())
