import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU-side test")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle


def use_ordered_param_host(monkeypatch):
    """Route GpuTokenService.submit_param_batch_host through the decide-order entry point
    (sentinel_submit_param_batch_ordered_host) and put the verdicts back at their arrival positions
    through the returned seq, which must be a permutation of [0, n)."""
    import numpy as np
    from sentinel_amd.token_service import GpuTokenService

    def host(self, rule_idx, acquire, param_key, ts):
        st, rem, seq = self.submit_param_batch_ordered_host(rule_idx, acquire, param_key, ts)
        n = len(seq)
        assert np.array_equal(np.sort(seq), np.arange(n, dtype=np.uint32)), "seq is not a permutation"
        idx = seq.astype(np.int64)
        o_st, o_rem = np.empty_like(st), np.empty_like(rem)
        o_st[idx] = st
        o_rem[idx] = rem
        return o_st, o_rem

    monkeypatch.setattr(GpuTokenService, "submit_param_batch_host", host)
