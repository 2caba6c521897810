"""sentinel_submit_flow_batches: several device batches in one call.  The verdicts and counters must
equal the same batches submitted one by one (and the oracle): hot flows (k_part_long), heterogeneous
acquires, prioritized requests, a skewed batch that may switch later batches to the radix path
mid-call."""
import numpy as np
import pytest

from sentinel_amd import trace as T

pytestmark = pytest.mark.gpu


def _engine(rules):
    import sentinel_amd as sa
    svc = sa.GpuTokenService(0)
    svc.load_rules_array(rules.flow_id, rules.count, rules.threshold_type, rules.sample_count,
                         rules.window_interval_ms, rules.namespace, rules.checker)
    return svc


def test_flow_batches_equal_one_by_one(oracle_mod):
    import torch
    from sentinel_amd.token_service import decode_verdicts, device_events
    rng = np.random.default_rng(71)
    F = 40_000
    rules = T.make_rules(F, rng, count_lo=5, count_hi=400, sample_count=4, window_interval_ms=400)
    dev = torch.device("cuda", 0)
    batches, flags = [], []
    t = T.T0_ALIGNED + 9
    for b in range(8):
        m = 300_000
        idx = rng.integers(0, F, size=m).astype(np.int32)
        if b in (2, 5):
            idx[rng.random(m) < 0.4] = 17                  # a hot flow: a long run
        if b == 6:
            idx[rng.random(m) < 0.9] = rng.integers(0, 50)  # skewed: may switch the next batches' path
        acq = np.where(rng.random(m) < 0.05, 3, 1).astype(np.int32)
        ts = T.timestamps(m, 2.0e6, t)
        fl = (rng.random(m) < 0.002).astype(np.uint8)
        batches.append((idx, acq, ts))
        flags.append(fl)
        t = int(ts[-1]) + 1
    A, B = _engine(rules), _engine(rules)
    orc = oracle_mod.TokenServiceOracle(rules.as_dicts())
    dev_ev = [device_events(torch.from_numpy(i).to(dev), torch.from_numpy(a).to(dev), torch.from_numpy(s).to(dev))
              for i, a, s in batches]
    dev_fl = [torch.from_numpy(f).to(dev) for f in flags]
    outs_a = [torch.empty(len(i), dtype=torch.int64, device=dev) for i, _, _ in batches]
    outs_b = [torch.empty(len(i), dtype=torch.int64, device=dev) for i, _, _ in batches]
    torch.cuda.synchronize()
    for k in range(len(batches)):
        A.submit_flow_batch(dev_ev[k], flags=dev_fl[k], verdicts=outs_a[k])
    A.synchronize()
    B.submit_flow_batches(dev_ev, outs_b, flags_list=dev_fl)
    B.synchronize()
    for k, (idx, acq, ts) in enumerate(batches):
        sa_, ra, wa = decode_verdicts(outs_a[k])
        sb, rb, wb = decode_verdicts(outs_b[k])
        so, ro, wo = orc.replay(idx, acq, ts, flags[k])
        assert np.array_equal(sa_, sb) and np.array_equal(ra, rb) and np.array_equal(wa, wb), k
        bad = np.nonzero((sb != so) | (rb != ro) | (wb != wo))[0]
        assert len(bad) == 0, (k, len(bad), bad[:5])
    for f in list(range(0, F, 997)) + [17]:
        assert np.array_equal(A.dump_flow(f, 4), B.dump_flow(f, 4)), f
