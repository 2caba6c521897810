"""Envoy RLS front end over the MI355X engine.

Mirrors (paths relative to sentinel-cluster/sentinel-cluster-server-envoy-rls/src/main/java/com/alibaba/csp/sentinel/cluster/server/envoy/rls/):
  SentinelEnvoyRlsServiceImpl.shouldRateLimit / checkToken / generateKey   SentinelEnvoyRlsServiceImpl.java:51-134
  EnvoySentinelRuleConverter.toSentinelFlowRule / generateFlowId / generateKey   rule/EnvoySentinelRuleConverter.java:44-85
  EnvoyRlsRuleManager.isValidRule / generateRuleMap                      rule/EnvoyRlsRuleManager.java (configUpdate, isValidRule)
  EnvoyRlsRule.KeyValueResource.hashCode (HashSet iteration order)        rule/EnvoyRlsRule.java:95-146
  SimpleClusterFlowChecker.acquireClusterToken (the checker, on the GPU)  flow/SimpleClusterFlowChecker.java:33-65

The gRPC server itself stays on the host; this module is what its `shouldRateLimit` calls.  Every
descriptor of every request in a batch becomes one event of ONE GPU batch, in request order and
descriptor order, so the verdicts equal the reference's sequential per-descriptor checks.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .token_service import ClusterFlowConfig, FlowRule, GpuTokenService, TokenResultStatus, _now_ms
from . import _lib

SEPARATOR = "|"                      # EnvoySentinelRuleConverter.SEPARATOR
INT_MAX = 2147483647


# Envoy ratelimit proto RateLimitResponse.Code
class Code:
    UNKNOWN = 0
    OK = 1
    OVER_LIMIT = 2


def _int32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x & 0x80000000 else x


def java_string_hash(s: str) -> int:
    """String.hashCode over UTF-16 code units, int overflow (JLS)."""
    h = 0
    units = np.frombuffer(s.encode("utf-16-le"), dtype="<u2")
    for u in units.tolist():
        h = (31 * h + u) & 0xFFFFFFFF
    return _int32(h)


def is_blank(s: Optional[str]) -> bool:
    """StringUtil.isBlank: null, empty or only Character.isWhitespace chars."""
    return s is None or all(c.isspace() for c in s)


def generate_flow_id(key: str) -> int:
    """EnvoySentinelRuleConverter.generateFlowId (java:67-73): Integer.MAX_VALUE + key.hashCode()."""
    if is_blank(key):
        return -1
    return INT_MAX + java_string_hash(key)


def _table_size_for(c: int) -> int:
    n = 1
    while n < c:
        n <<= 1
    return min(max(n, 1), 1 << 30)


def _spread(h: int) -> int:
    h &= 0xFFFFFFFF
    return h ^ (h >> 16)


def java_hash_iteration_order(hashes: Sequence[int], initial_capacity: int) -> List[int]:
    """Iteration order of a java.util.HashMap/HashSet filled with keys of these hashCodes in this
    order: final table capacity (doubling past 0.75 load), bucket order, insertion order inside a
    bucket (treeified bins -- 8+ keys in one bucket of a >= 64 table -- are not modelled)."""
    cap = _table_size_for(initial_capacity)
    for size in range(1, len(hashes) + 1):
        if size > 0.75 * cap:
            cap <<= 1
    return sorted(range(len(hashes)), key=lambda i: (_spread(hashes[i]) & (cap - 1), i))


@dataclass(frozen=True)
class KeyValueResource:
    key: str
    value: str

    def java_hash(self) -> int:   # Objects.hash(key, value)
        return _int32(31 * (31 * 1 + java_string_hash(self.key)) + java_string_hash(self.value))


@dataclass
class ResourceDescriptor:
    """`resources` in insertion order; the reference holds them in a HashSet."""
    resources: List[KeyValueResource] = field(default_factory=list)
    count: Optional[float] = None

    def iteration_order(self) -> List[KeyValueResource]:
        uniq: List[KeyValueResource] = []
        for r in self.resources:      # Set semantics: equals on (key, value)
            if r not in uniq:
                uniq.append(r)
        cap = max(int(len(uniq) / 0.75) + 1, 16)   # new HashSet<>(collection)
        return [uniq[i] for i in java_hash_iteration_order([r.java_hash() for r in uniq], cap)]


@dataclass
class EnvoyRlsRule:
    domain: str = ""
    descriptors: List[ResourceDescriptor] = field(default_factory=list)


def is_valid_rule(rule: Optional[EnvoyRlsRule]) -> bool:
    """EnvoyRlsRuleManager.isValidRule."""
    if rule is None or is_blank(rule.domain) or not rule.descriptors:
        return False
    for d in rule.descriptors:
        if d is None or d.count is None or d.count < 0 or not d.resources:
            return False
        for r in d.resources:
            if r is None or is_blank(r.key) or is_blank(r.value):
                return False
    return True


def generate_key(domain: str, entries: Sequence[Tuple[str, str]]) -> str:
    """domain|k1|v1|k2|v2... (EnvoySentinelRuleConverter.generateKey, SentinelEnvoyRlsServiceImpl.generateKey)."""
    parts = [domain]
    for k, v in entries:
        parts.append(k)
        parts.append(v)
    return SEPARATOR.join(parts)


def to_sentinel_flow_rule(domain: str, d: ResourceDescriptor) -> FlowRule:
    """EnvoySentinelRuleConverter.toSentinelFlowRule: GLOBAL threshold, sampleCount 1 (interval 1000)."""
    key = generate_key(domain, [(r.key, r.value) for r in d.iteration_order()])
    return FlowRule(resource=key, count=float(d.count), cluster_mode=True,
                    cluster_config=ClusterFlowConfig(flow_id=generate_flow_id(key), threshold_type=1, sample_count=1,
                                                     window_interval_ms=1000, fallback_to_local_when_fail=False),
                    namespace=0, checker=_lib.CHECKER_SIMPLE)


@dataclass
class RateLimitRequest:
    domain: str
    descriptors: List[List[Tuple[str, str]]]
    hits_addend: int = 0


@dataclass
class DescriptorStatus:
    code: int
    requests_per_unit: Optional[int] = None      # current_limit (unit SECOND) when a rule exists
    limit_remaining: Optional[int] = None


@dataclass
class RateLimitResponse:
    overall_code: int
    statuses: List[DescriptorStatus]


def _java_d2i(d: float) -> int:
    if d != d:
        return 0
    if d >= INT_MAX:
        return INT_MAX
    if d <= -INT_MAX - 1:
        return -INT_MAX - 1
    return int(d)


class SentinelEnvoyRlsService:
    """Batched SentinelEnvoyRlsServiceImpl over a GpuTokenService whose flow rules are the RLS rules."""

    def __init__(self, svc: GpuTokenService):
        self.svc = svc
        self.rule_count = {}        # flowId -> FlowRule.count of the rule that won the load

    def load_rules(self, rules: Sequence[EnvoyRlsRule]) -> List[FlowRule]:
        """EnvoyRlsRuleManager.loadRules: invalid rules dropped, first rule per domain kept, the rule
        map iterated in HashMap order, then ClusterFlowRuleManager.loadRules (last flowId wins)."""
        if not rules:
            kept: List[EnvoyRlsRule] = []
        else:
            kept = []
            seen = set()
            for r in rules:
                if not is_valid_rule(r) or r.domain in seen:
                    continue
                seen.add(r.domain)
                kept.append(r)
            order = java_hash_iteration_order([java_string_hash(r.domain) for r in kept], len(rules))
            kept = [kept[i] for i in order]
        flow_rules = [to_sentinel_flow_rule(r.domain, d) for r in kept for d in r.descriptors]
        self.svc.load_flow_rules(flow_rules)
        self.rule_count = {}
        for fr in flow_rules:
            fid = fr.cluster_config.flow_id
            if fid is not None and fid > 0:
                self.rule_count[fid] = fr.count
        return flow_rules

    def should_rate_limit(self, request: RateLimitRequest, ts: Optional[int] = None) -> RateLimitResponse:
        return self.should_rate_limit_batch([request], [ts])[0]

    def should_rate_limit_batch(self, requests: Sequence[RateLimitRequest], ts=None):
        """One GPU batch for every descriptor of every request.  A request with hitsAddend < 0 gets a
        ValueError in its slot (the reference calls responseObserver.onError)."""
        n = len(requests)
        if ts is None:
            ts = [None] * n
        flow_ids, acq, tss, owner = [], [], [], []
        out: List[object] = [None] * n
        for i, req in enumerate(requests):
            a = int(req.hits_addend)
            if a < 0:
                out[i] = ValueError(f"acquireCount should be positive, but actual: {a}")
                continue
            a = 1 if a == 0 else a
            t = _now_ms() if ts[i] is None else int(ts[i])
            for entries in req.descriptors:
                flow_ids.append(generate_flow_id(generate_key(req.domain, entries)))
                acq.append(a)
                tss.append(t)
                owner.append(i)
        if flow_ids:
            idx = self.svc.lookup_flow_idx(np.array(flow_ids, dtype=np.int64))
            idx[idx == _lib.IDX_BAD_ID] = _lib.IDX_NO_RULE   # checkToken: getFlowRuleById(id <= 0) -> null
            st, rem, _ = self.svc.submit_flow_batch_host(idx, np.array(acq, np.int32), np.array(tss, np.int64))
        else:
            st = rem = np.zeros(0, np.int32)
        j = 0
        for i, req in enumerate(requests):
            if out[i] is not None:
                continue
            blocked = False
            statuses = []
            for _entries in req.descriptors:
                s = int(st[j])
                if s == TokenResultStatus.NO_RULE_EXISTS:        # pass when the rule is absent
                    s = TokenResultStatus.OK
                if s != TokenResultStatus.OK:
                    blocked = True
                ds = DescriptorStatus(Code.OK if s == TokenResultStatus.OK else Code.OVER_LIMIT)
                cnt = self.rule_count.get(flow_ids[j])
                if cnt is not None and int(st[j]) != TokenResultStatus.NO_RULE_EXISTS:
                    ds.requests_per_unit = _java_d2i(cnt)
                    ds.limit_remaining = int(rem[j])
                statuses.append(ds)
                j += 1
            out[i] = RateLimitResponse(Code.OVER_LIMIT if blocked else Code.OK, statuses)
        return out
