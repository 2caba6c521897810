"""flowId-hash sharding across the GPUs of one node.

A flow's verdicts depend only on its own window (ClusterMetric per flowId,
srv/flow/statistic/ClusterMetricStatistics.java:56-58) plus host constants, so the flowId space is
partitioned with gpu = splitmix64(flowId) mod G and every GPU runs an independent engine: no
exchange on the decision path.  The namespace GlobalRequestLimiter couples flows of a namespace;
it is exact under sharding only when a namespace's flows live on one rank (shard_by_namespace) or
when the limiter is disabled.

The only collective is the periodic ClusterMetric snapshot (ClusterMetricNodeGenerator.java:36-106):
each rank's flow records {flowId, passQps, blockQps} (flowToMetricNode, :70-86) and param records
{flowId, top-5 (value, avg)} (paramToMetricNode, :88-105) are all-gathered (RCCL over xGMI on MI355X;
gloo in the CPU tests).  A param rule lives on its flowId's owner rank with all of its values, so a
rank's getTopValues is the rule's whole answer: the gathered records need no merge.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from .trace import shard_of


def owner_of(flow_ids, world: int) -> np.ndarray:
    """Rank owning each flowId."""
    return shard_of(np.asarray(flow_ids, dtype=np.int64), world)


def shard_by_namespace(namespace_of_flow: np.ndarray, world: int) -> np.ndarray:
    """Alternative placement that keeps every namespace on one rank (exact GlobalRequestLimiter)."""
    return (np.asarray(namespace_of_flow, dtype=np.int64) % world).astype(np.int64)


def split_batch(owner: np.ndarray, world: int) -> List[np.ndarray]:
    """Arrival positions routed to each rank, each list in arrival order (a stable split)."""
    order = np.argsort(owner, kind="stable")
    counts = np.bincount(owner, minlength=world)
    bounds = np.concatenate([[0], np.cumsum(counts)])
    return [order[bounds[r]:bounds[r + 1]] for r in range(world)]


def merge_verdicts(parts: Sequence[np.ndarray], positions: Sequence[np.ndarray], n: int) -> np.ndarray:
    """Inverse of split_batch for per-event results (any dtype)."""
    out = np.empty(n, dtype=parts[0].dtype) if parts else np.empty(0)
    for p, pos in zip(parts, positions):
        out[pos] = p
    return out


def local_rule_subset(flow_ids: np.ndarray, rank: int, world: int) -> np.ndarray:
    """Indices of the rule table this rank loads."""
    return np.nonzero(owner_of(flow_ids, world) == rank)[0]


def gather_records(local, group=None):
    """All-gather per-rank fixed-width records (torch tensor (F_rank, W) int64) into one
    (sum F_rank, W) tensor ordered by rank: one size exchange, then one all-gather of the rows padded
    to the largest rank (one collective call per snapshot leg)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo" and local.is_cuda:   # (gloo gathers host tensors)
        return gather_records(local.cpu(), group).to(local.device)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    mx = int(max(int(s.item()) for s in sizes))
    pad = torch.zeros((mx, local.shape[1]), dtype=torch.int64, device=local.device)
    pad[: local.shape[0]] = local
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad, group=group)
    return torch.cat([o[: int(s.item())] for o, s in zip(out, sizes)], dim=0)


def gather_snapshot(local, group=None):
    """All-gather per-rank flow snapshot records (torch tensor (F_rank, 3) int64 holding
    sentinel_flow_snapshot_t rows) into one (sum F_rank, 3) tensor ordered by rank."""
    return gather_records(local, group)


PARAM_RECORD_WORDS = 12          # sentinel_param_snapshot_t: 96 bytes


def gather_param_snapshot(local, group=None):
    """All-gather per-rank param snapshot records (sentinel_param_snapshot_t rows: a uint8 tensor of
    R_rank * 96 bytes as written by sentinel_param_snapshot_device, or an (R_rank, 12) int64 tensor)
    into one (sum R_rank, 12) int64 tensor ordered by rank."""
    import torch
    if local.dtype == torch.uint8:
        local = local.view(torch.int64).reshape(-1, PARAM_RECORD_WORDS)
    return gather_records(local, group)


def param_snapshot_records(flow_id, tops):
    """Pack (flowId, [(key, avg)] * <= 5) per param rule into the (R, 12) int64 layout of
    sentinel_param_snapshot_t."""
    import torch
    from . import _lib
    rec = np.zeros(len(flow_id), dtype=_lib.PARAM_SNAPSHOT_DTYPE)
    rec["flow_id"] = flow_id
    for r, top in enumerate(tops):
        rec["n_top"][r] = len(top)
        for k, (key, avg) in enumerate(top):
            rec["key"][r][k] = key
            rec["avg"][r][k] = avg
    return torch.from_numpy(rec.view(np.int64).reshape(-1, PARAM_RECORD_WORDS).copy())


def unpack_param_snapshot(t) -> dict:
    """flowId -> [(key, avg)] (getTopValues order) from gathered param records."""
    from . import _lib
    a = np.ascontiguousarray(t.cpu().numpy()).view(_lib.PARAM_SNAPSHOT_DTYPE).reshape(-1)
    return {int(a["flow_id"][r]): [(int(a["key"][r][k]), float(a["avg"][r][k])) for k in range(int(a["n_top"][r]))]
            for r in range(len(a))}


def snapshot_records(flow_id: np.ndarray, pass_qps: np.ndarray, block_qps: np.ndarray):
    """Pack snapshot fields into the (F, 3) int64 layout of sentinel_flow_snapshot_t."""
    import torch
    rec = np.zeros((len(flow_id), 3), dtype=np.int64)
    rec[:, 0] = flow_id
    rec[:, 1] = np.asarray(pass_qps, dtype=np.float64).view(np.int64)
    rec[:, 2] = np.asarray(block_qps, dtype=np.float64).view(np.int64)
    return torch.from_numpy(rec)


def unpack_snapshot(t) -> np.ndarray:
    a = t.cpu().numpy()
    out = np.zeros(len(a), dtype=[("flow_id", "<i8"), ("pass_qps", "<f8"), ("block_qps", "<f8")])
    out["flow_id"] = a[:, 0]
    out["pass_qps"] = a[:, 1].view(np.float64)
    out["block_qps"] = a[:, 2].view(np.float64)
    return out
