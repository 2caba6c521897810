"""bench.py -- token decisions/sec of the MI355X engine (BASELINE.json metric and configs).

Default workload (BASELINE.json configs[2], the config the headline metric is quoted on): a universe
of 1M flowIds (cluster FlowRules, GLOBAL threshold count ~ U{10..1000}, default cluster window
sampleCount=10 / windowIntervalMs=1000 -> 10 x 100 ms buckets), hash-sharded over the ranks by
splitmix64(flowId) mod N.  Every rank decides a fixed 8M-event batch per step over its own flows
(uniform, acquire 1, monotone timestamps at 2x the shard's summed thresholds): weak scaling, no
collective on the decision path.  A step = one batch through DefaultTokenService.requestToken
semantics (validation, window roll, ClusterFlowChecker admission, verdict write-back), inputs
already resident in HBM.

--config selects the other BASELINE configs (their JSON lines go under profiles/, never to the driver):
  2     10k flowIds, n=2 / 1000 ms, Zipf(1.1) requests, 4M-event batches (configs[1])
  4     hot-parameter cluster rules: 100k resources x Zipf(1.2) over 1000 Long values, exact counters
  4cm   the same on the shared count-min sketch (w=2^20, d=4) + the measured false-block rate vs e*N/w
  5     Envoy RLS rules (SimpleClusterFlowChecker, n=1 / 1000 ms), hitsAddend ~ geometric(0.3) capped at
        64: heterogeneous acquire -> the sequential per-segment path
  5conc the thread-grade half of config 5: concurrency-token acquire / release batches
        (ConcurrentClusterFlowChecker, sentinel_submit_concurrent_batch on device pointers): 20k
        thread-grade rules, Zipf(1.1) flows, every batch releases the tokens the previous batch acquired
  3lim  config 3 with the namespace GlobalRequestLimiter on (the reference creates one per namespace
        after any namespace-set change): the limiter pass, then the partition path

Prints ONE JSON line (rank 0).  Extra fields: p99 batch latency from >= 200 batches of an untimed
latency loop (device events, and host clock with a synchronize per batch), per-kernel profile, the
roofline of the dominant kernel, and the CPU oracle ("port") timed on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)

# Algorithmic bytes per processed event for each kernel of the pipelines (DESIGN.md "Kernels").
KERNEL_BYTES_PER_EVENT = {
    "flow_prep": 20.0,        # read the 16-B event, write the 4-B sort key (histograms stay in LDS)
    "radix_hist": 4.0,        # read key
    "radix_scatter": None,    # per pass: read key 4 + value 8, write 12; pass 0 reads the 16-B event instead of a value
    "scan_tiles": 8.0,
    "scan_add": 8.0,
    "seg_heads": 17.0,        # read key 4 + value 8, write head 4 + homogeneity flag 1
    "segments": 17.0,         # read key 4 + value 8, write segment id 4 + flag 1 (records are per segment)
    "seg_mark": 5.0,          # read segid 4 + flag 1 (segment records are per segment)
    "verdict": 20.0,          # read segid 4 + value 8, write the 8-B verdict
    "lim_prep": 32.0,         # one-limiter prep: read the 16-B event, write flow key 4 + limiter key 4 + value 8
    "part_prep": 16.0,        # read the 16-B event (range histogram in LDS; no key array without namespace routes)
    "part_scatter": 24.0,     # read the 16-B event (key re-derived), write the 8-B packed value (local key inside)
    "param_prep": 24.0,       # read the 24-B event (range histogram in LDS; rejected requests answered here)
    "param_scatter": 44.0,    # read the 24-B event, write key 8 + packed value 8 + rule 4
    "param_meta": 48.0,       # per slot after a rule / threshold / table change: key 8, rule fields ~16, write ~20 B
    "prule_prep": 36.0,       # read the 24-B event + value 8, write key 4
    "conc_prep": 38.0,        # read the 24-B event (+ a release's token probe 8), write flow key 4 + aux word 8
    "conc_apply": 52.5,       # read key 4 + value 8 + element 4 (+ pass 1 per acquire), write the 16-B result;
                              # per passing acquire (half the events) a token insert: probe 8 + record 32
}

# rocprofv3 kernel symbols behind each engine profile name (for the PMC traffic of the roofline).
KERNEL_SYMBOLS = {
    "flow_prep": ("k_flow_prep",), "radix_hist": ("k_radix_hist_pass",), "radix_scatter": ("k_radix_scatter_p",),
    "scan": ("k_scan_lookback",), "segments": ("k_segments",), "process": ("k_process",), "verdict": ("k_verdict",),
    "part_prep": ("k_part_prep",), "part_scatter": ("k_part_scatter",),
    "part_fused": ("k_part_half",), "part_big": ("k_part_big",), "part_long": ("k_part_long",),
    "param_prep": ("k_param_prep", "k_pp_prep"), "param_meta": ("k_param_meta",), "prule_prep": ("k_prule_prep",),
    "prule_process": ("k_prule_process",), "part_unsplit": ("k_part_unsplit",), "lim_prep": ("k_lim1_prep",),
    "param_scatter": ("k_pp_scatter",), "param_group": ("k_pp_group",), "param_cm_read": ("k_pp_cm_read",), "param_cm_walk": ("k_pp_cm_walk",),
    "param_cm_block": ("k_pp_cm_block",),
    "conc_prep": ("k_conc_prep",), "conc_scan": ("k_conc_scan",), "conc_apply": ("k_conc_apply",),
    "param_decide": ("k_pp_walk", "k_pp_decide"),
}
PMC_DIR = os.path.join(ROOT, "profiles", "pmc")


def pmc_traffic(kernel: str, shape: dict):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary of THIS workload shape
    (profiles/pmc/*.json written by scripts/pmc_summary.py; since round 5 from the memory-side request
    counters by request size -- scripts/gpu_pmc_req.sh, reads 128 / 64 / 32 B per request, writes 64 / 32 B,
    calibrated on known-byte patterns by tools/pmc_calib.cpp -- the newest file of the shape wins); None
    when no PMC run of this shape exists."""
    try:
        files = sorted(os.listdir(PMC_DIR))
    except OSError:
        return None, None
    for fn in reversed(files):
        try:
            with open(os.path.join(PMC_DIR, fn)) as f:
                summ = json.load(f)
        except (OSError, ValueError):
            continue
        if summ.get("shape") != shape:
            continue
        pats = KERNEL_SYMBOLS.get(kernel, ())
        tot = disp = 0.0
        for name, v in summ.get("kernels", {}).items():
            if any(name.startswith(p) for p in pats) and v.get("traffic_bytes_avg"):
                tot += v["traffic_bytes_avg"] * v["dispatches"]
                disp += v["dispatches"]
        if disp:
            return round(tot / disp, 1), f"profiles/pmc/{fn}: {summ.get('correction', '')}"
    return None, None


def cgroup_cpus():
    """CPUs the cgroup's CPU quota grants this process (cgroup v2 cpu.max / v1 cfs quota), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0:
            return max(1, q // per)
    except (OSError, ValueError):
        pass
    return None


def cpu_threads_default():
    """Threads for the sharded CPU baseline: every CPU this process may run on (sched_getaffinity, SURVEY
    section 8(d): T = nproc), capped by the cgroup's CPU quota when one is set (threads beyond the quota
    only time-slice on the same share)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    q = cgroup_cpus()
    return min(avail, q) if q else avail


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count()
    return model, os.cpu_count(), avail


def log(msg):
    """Progress on stderr (long GPU runs must keep writing)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="3", choices=["3", "2", "4", "4cm", "5", "5conc", "3lim"])
    ap.add_argument("--events-per-gpu", type=int, default=None)
    ap.add_argument("--flows", type=int, default=None)
    ap.add_argument("--sample-count", type=int, default=None)
    ap.add_argument("--interval-ms", type=int, default=1000)
    ap.add_argument("--cpu-steps-1core", type=int, default=2)
    ap.add_argument("--cpu-steps-mt", type=int, default=12)
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the sharded CPU baseline (default: every CPU this process may run on)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--kernel-every", type=int, default=2,
                    help="time the dominant kernel with HIP events on every k-th timed step")
    ap.add_argument("--latency-batches", type=int, default=200,
                    help="batches of the untimed latency loop (p99 from these, not from the timed steps)")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-fed legs")
    ap.add_argument("--output", choices=["arrival", "decide"], default="decide",
                    help="flow configs: verdicts in arrival order (sentinel_submit_flow_batch) or in decide order "
                         "with their arrival positions (sentinel_submit_flow_batch_ordered: what the batcher and the "
                         "wire server consume)")
    ap.add_argument("--host-reps", type=int, default=200)
    return ap.parse_args()


class FlowWorkload:
    """Flow events (sentinel_event_t) of configs 2, 3, 5 and 3lim, generated on the device."""

    def __init__(self, args, world, rank, dev):
        import torch
        from sentinel_amd import trace as T
        import sentinel_amd as sa
        from sentinel_amd.token_service import ServerNamespace
        self.T, self.torch, self.dev, self.args = T, torch, dev, args
        cfg = args.config
        rng = np.random.default_rng({"3": 3, "3lim": 3, "2": 2, "5": 5}[cfg])
        if cfg in ("3", "3lim"):
            flows = args.flows or 1_000_000
            n = args.sample_count or 10
            rules = T.make_rules(flows, rng, sample_count=n, window_interval_ms=args.interval_ms)
            self.N = args.events_per_gpu or 8 * 1024 * 1024
            self.dist, self.acq_kind, self.workload = "uniform", "ones", (
                f"config3: {flows} flowIds hash-sharded (splitmix64 mod N), cluster GLOBAL rules count~U{{10..1000}}, "
                f"n={n} w={args.interval_ms // n}ms, uniform flows, acquire=1, 2x offered load"
                + (", namespace GlobalRequestLimiter on (cap 1e15/s)" if cfg == "3lim" else ""))
        elif cfg == "2":
            flows = args.flows or 10_000
            n = args.sample_count or 2
            rules = T.make_rules(flows, rng, sample_count=n, window_interval_ms=args.interval_ms)
            self.N = args.events_per_gpu or 4 * 1024 * 1024
            self.dist, self.acq_kind, self.workload = "zipf1.1", "ones", (
                f"config2: {flows} flowIds, cluster GLOBAL rules count~U{{10..1000}}, n={n} w={args.interval_ms // n}ms, "
                f"Zipf(1.1) requests, acquire=1, 2x offered load, {self.N}-event batches")
        else:
            flows = args.flows or 20_000
            rules = T.make_rules(flows, rng, count_lo=50, count_hi=5000, sample_count=1, window_interval_ms=1000, checker=1)
            self.N = args.events_per_gpu or 4 * 1024 * 1024
            self.dist, self.acq_kind, self.workload = "zipf1.1", "geometric", (
                f"config5: {flows} Envoy RLS rules (SimpleClusterFlowChecker, n=1 w=1000ms, GLOBAL), Zipf(1.1) "
                f"descriptors, hitsAddend~geometric(0.3) capped at 64 (heterogeneous acquire: sequential path), "
                f"2x offered load")
        mine = np.nonzero(T.shard_of(rules.flow_id, world) == rank)[0] if world > 1 else np.arange(len(rules))
        self.rules = rules.subset(mine)
        self.F = len(self.rules)
        self.namespaces = [dict(connected_count=1, has_limiter=1, max_allowed_qps=1e15)] if cfg == "3lim" else None
        self.svc = sa.GpuTokenService(dev.index or 0)
        if self.namespaces:
            self.svc.set_namespaces([ServerNamespace(**x) for x in self.namespaces])
        r = self.rules
        self.svc.load_rules_array(r.flow_id, r.count, r.threshold_type, r.sample_count, r.window_interval_ms,
                                  r.namespace, r.checker)
        mean_acq = 1.0 if self.acq_kind == "ones" else 2.81
        self.rate = 2.0 * float(r.count.sum()) / mean_acq          # offered events per second
        self.ms_per_event = 1000.0 / self.rate
        self.gen = torch.Generator(device=dev).manual_seed(1000 + rank)
        if self.dist.startswith("zipf"):
            w = 1.0 / np.power(np.arange(1, self.F + 1, dtype=np.float64), 1.1)
            perm = np.random.default_rng(7 + rank).permutation(self.F)
            self.zipf_cdf = torch.from_numpy(np.cumsum(w) / w.sum()).to(dev)
            self.zipf_perm = torch.from_numpy(perm.astype(np.int32)).to(dev)
        self.verdicts = torch.empty(self.N, dtype=torch.int64, device=dev)
        self.seq = torch.empty(self.N, dtype=torch.int32, device=dev)
        self.ordered = args.output == "decide"
        if self.ordered:
            self.workload += ("; verdicts in decide order with their arrival positions (sentinel_submit_flow_batch_"
                              "ordered, the output the batcher / wire server consume: each response keyed by its "
                              "request)")
        self.kept = []
        self.parity_result = None

    def batch(self, s):
        """Step s's events (device tensor (N, 2) int64): consecutive in time across steps."""
        torch, N = self.torch, self.N
        if self.dist == "uniform":
            idx = torch.randint(0, self.F, (N,), dtype=torch.int32, device=self.dev, generator=self.gen)
        else:
            u = torch.rand(N, dtype=torch.float64, device=self.dev, generator=self.gen)
            idx = self.zipf_perm[torch.clamp(torch.searchsorted(self.zipf_cdf, u, right=True), max=self.F - 1)]
        if self.acq_kind == "ones":
            acq = torch.ones(N, dtype=torch.int32, device=self.dev)
        else:   # geometric(0.3) capped at 64: floor(log(U) / log(0.7)) + 1
            u = torch.rand(N, dtype=torch.float64, device=self.dev, generator=self.gen)
            acq = torch.clamp(torch.floor(torch.log1p(-u) / np.log(0.7)) + 1, max=64).to(torch.int32)
        base = torch.arange(s * N, (s + 1) * N, device=self.dev, dtype=torch.float64)
        ts = (self.T.T0_ALIGNED + torch.floor(base * self.ms_per_event)).to(torch.int64)
        from sentinel_amd.token_service import device_events
        return device_events(idx, acq, ts)

    def span_ms(self):
        return int(np.ceil(self.N * self.ms_per_event)) + 1

    def submit(self, b, keep=False):
        if keep:                          # a verdict buffer of its own: checked against the CPU baseline's replay
            v = self.torch.empty(self.N, dtype=self.torch.int64, device=self.dev)
            if self.ordered:
                sq = self.torch.empty(self.N, dtype=self.torch.int32, device=self.dev)
                self.svc.submit_flow_batch_ordered(b, verdicts=v, seq=sq)
                self.kept.append((v, sq))
            else:
                self.svc.submit_flow_batch(b, verdicts=v)
                self.kept.append(v)
        elif self.ordered:
            self.svc.submit_flow_batch_ordered(b, verdicts=self.verdicts, seq=self.seq)
        else:
            self.svc.submit_flow_batch(b, verdicts=self.verdicts)

    def parity(self, st, rem, wait):
        """The kept batches' GPU verdicts against the oracle replay of the same events (first batches)."""
        from sentinel_amd.token_service import decode_verdicts
        if not self.kept:
            return None
        g = [decode_verdicts(arrival_order(self.torch, v)) for v in self.kept]
        gs, gr, gw = (np.concatenate([x[i] for x in g]) for i in range(3))
        m = min(len(gs), len(st))
        bad = int(((gs[:m] != st[:m]) | (gr[:m] != rem[:m]) | (gw[:m] != wait[:m])).sum())
        return {"parity_checked_events": m, "parity_mismatches": bad,
                "parity_note": f"status, remaining and waitInMs of the first {len(self.kept)} batches (warmup + "
                               f"profile steps) against the CPU baseline's oracle replay of the same events"}

    def cpu_baseline(self, batches, k1, kmt, threads):
        from oracle import oracle as O
        r = self.rules

        def host_steps(k):
            e = self.torch.cat(batches[:k]).cpu().numpy()
            return (e[:, 0] & 0xFFFFFFFF).astype(np.int32), (e[:, 0] >> 32).astype(np.int32), e[:, 1].copy()

        def fresh():
            return O.TokenServiceOracle.from_arrays(r.flow_id, r.count, r.threshold_type, r.sample_count,
                                                    r.window_interval_ms, r.namespace, r.checker,
                                                    namespaces=self.namespaces)
        idx, acq, ts = host_steps(k1)
        orc = fresh()
        c0 = time.perf_counter()
        orc.replay(idx, acq, ts)
        cdt = time.perf_counter() - c0
        one = (len(ts), cdt, 1, "sequential oracle replay")
        if self.namespaces:          # a namespace limiter couples every flow: no sharded replay
            idx, acq, ts = host_steps(min(len(self.kept), len(batches)))
            st, rem, wt = fresh().replay(idx, acq, ts)
            self.parity_result = self.parity(st, rem, wt)
            return one, None
        idx, acq, ts = host_steps(kmt)
        orc = fresh()
        c0 = time.perf_counter()
        st, rem, wt, used = orc.replay_mt(idx, acq, ts, threads)
        cdt = time.perf_counter() - c0
        mt = (len(ts), cdt, int(used), f"oracle replay sharded by flow over {used} pthreads")
        self.parity_result = self.parity(st, rem, wt)
        return one, mt

    def bytes_of(self, dom, d, steps):
        """Algorithmic bytes per processed event of the dominant kernel."""
        n = int(self.rules.sample_count.max())
        e_f = self.N / max(1, self.F)
        if dom == "process":
            # per touched flow: read n epochs + n PASS, write epoch + 4 counters; per event: segment record
            return (n * 16 + 40 + 24) / max(1.0, e_f)
        if dom == "part_fused":
            # per event: read the 8-B packed value (local key inside), write the 8-B verdict; per
            # touched flow: read the window header (16 B per bucket) and the rule fields, write back
            # the rolled bucket's 16-B pair, read + write its BLOCK / PASS_REQUEST / BLOCK_REQUEST
            # counters (3 x 8 B each way, blocked counter rows); decide-order output also writes each
            # event's 4-B arrival position
            return (20.0 if self.ordered else 16.0) + (n * 16 + 42 + 16 + 48) / max(1.0, e_f)
        if dom == "radix_scatter":
            passes = max(1, round(d["calls"] / max(1, steps)))
            return (32.0 + 24.0 * (passes - 1)) / passes
        return KERNEL_BYTES_PER_EVENT.get(dom)

    def pipeline_bytes(self):
        n = int(self.rules.sample_count.max())
        return 21.0 + (n * 64 + 64 + 16) / max(1.0, self.N / max(1, self.F))

    def pipeline_bytes_engine(self):
        """The bytes this engine's own layout must move per decision: 16 B event + 8 B verdict, per
        touched flow the n {epoch, PASS} header pairs read (16 n) and the rolled one written (16), the
        rolled slot's BLOCK / PASS_REQUEST / BLOCK_REQUEST rows read and written (48) and ~42 B of rule
        fields (w, 1/w, I_s, threshold, kind, occupy flag)."""
        n = int(self.rules.sample_count.max())
        return (28.0 if self.ordered else 24.0) + (16 * n + 16 + 48 + 42) / max(1.0, self.N / max(1, self.F))

    def shape(self):
        return {"config": self.args.config, "flows": self.F, "events": self.N,
                "sample_count": int(self.rules.sample_count.max()),
                "output": "decide order + arrival positions" if self.ordered else "arrival order"}


class ParamWorkload:
    """Cluster hot-parameter requests (sentinel_param_event_t) of config 4, exact or count-min."""

    def __init__(self, args, world, rank, dev):
        import torch
        import sentinel_amd as sa
        from sentinel_amd import trace as T
        from sentinel_amd.token_service import ServerNamespace
        self.T, self.torch, self.dev, self.args = T, torch, dev, args
        self.R_total = args.flows or 100_000
        self.universe = 1000
        self.N = args.events_per_gpu or 4 * 1024 * 1024
        n = args.sample_count or 10
        rng = np.random.default_rng(4)
        count = rng.integers(5, 101, size=self.R_total).astype(np.float64)
        flow_id = np.arange(1, self.R_total + 1, dtype=np.int64)
        mine = np.nonzero(T.shard_of(flow_id, world) == rank)[0] if world > 1 else np.arange(self.R_total)
        self.flow_id, self.count = flow_id[mine], count[mine]
        self.R = len(mine)
        self.hot = {}
        for r in range(min(self.R, 1000)):                # ~1% of values are hot items on the first rules
            for v in range(10):
                self.hot.setdefault(r, {})[int((np.uint64(self.flow_id[r]) << np.uint64(20)) | np.uint64(v))] = \
                    int(rng.integers(1, 20))
        self.n, self.interval = n, args.interval_ms
        self.prules = [dict(flow_id=int(self.flow_id[r]), count=float(self.count[r]), threshold_type=1, sample_count=n,
                            window_interval_ms=self.interval) for r in range(self.R)]
        self.svc = sa.GpuTokenService(dev.index or 0)
        self.svc.set_namespaces([ServerNamespace()])
        self.svc.load_param_rules([sa.ParamFlowRule(count=p["count"], cluster_config=sa.ClusterFlowConfig(
            flow_id=p["flow_id"], threshold_type=1, sample_count=n, window_interval_ms=self.interval),
            hot_items=self.hot.get(r, {})) for r, p in enumerate(self.prules)])
        self.cm = args.config == "4cm"
        self.cm_width, self.cm_depth = 1 << 20, 4
        if self.cm:
            from sentinel_amd import _lib
            self.svc.set_param_mode(_lib.PARAM_COUNT_MIN_SHARED, self.cm_depth, self.cm_width)
        self.rate = 2.0 * float(self.count.sum()) * 0.05     # offered requests per second
        self.ms_per_event = 1000.0 / self.rate
        self.gen = torch.Generator(device=dev).manual_seed(2000 + rank)
        w = 1.0 / np.power(np.arange(1, self.universe + 1, dtype=np.float64), 1.2)
        self.zipf_cdf = torch.from_numpy(np.cumsum(w) / w.sum()).to(dev)
        self.fid_dev = torch.from_numpy(self.flow_id.astype(np.int64)).to(dev)
        self.verdicts = torch.empty(self.N, dtype=torch.int64, device=dev)
        self.seq = torch.empty(self.N, dtype=torch.int32, device=dev)
        self.ordered = args.output == "decide"
        self.kept = []
        self.parity_result = None
        self.workload = (f"config4: {self.R_total} hot-parameter cluster rules (count~U{{5..100}}, hot items), values "
                         f"Zipf(1.2) over 1000 Long keys per resource, n={n} w={self.interval // n}ms, acquire 1, "
                         f"{self.N}-event batches, " + (f"shared count-min sketch d={self.cm_depth} w=2^20"
                                                        if self.cm else "exact per-value counters")
                         + ("; verdicts in decide order with their arrival positions (sentinel_submit_param_batch_"
                            "ordered, what the wire server's PARAM path consumes)" if self.ordered else ""))

    def batch(self, s):
        torch, N = self.torch, self.N
        ridx = torch.randint(0, self.R, (N,), dtype=torch.int32, device=self.dev, generator=self.gen)
        u = torch.rand(N, dtype=torch.float64, device=self.dev, generator=self.gen)
        vals = torch.clamp(torch.searchsorted(self.zipf_cdf, u, right=True), max=self.universe - 1).to(torch.int64)
        keys = (self.fid_dev[ridx.long()] << 20) | vals       # injective per (rule flowId, value)
        base = torch.arange(s * N, (s + 1) * N, device=self.dev, dtype=torch.float64)
        ts = (self.T.T0_ALIGNED + torch.floor(base * self.ms_per_event)).to(torch.int64)
        w0 = (torch.ones(N, dtype=torch.int64, device=self.dev) << 32) | (ridx.to(torch.int64) & 0xFFFFFFFF)
        return torch.stack([w0, ts, keys], dim=1).contiguous()

    def span_ms(self):
        return int(np.ceil(self.N * self.ms_per_event)) + 1

    def submit(self, b, keep=False):
        if keep:
            v = self.torch.empty(self.N, dtype=self.torch.int64, device=self.dev)
            if self.ordered:
                sq = self.torch.empty(self.N, dtype=self.torch.int32, device=self.dev)
                self.svc.submit_param_batch_ordered(b, verdicts=v, seq=sq)
                self.kept.append((v, sq))
            else:
                self.svc.submit_param_batch(b, verdicts=v)
                self.kept.append(v)
        elif self.ordered:
            self.svc.submit_param_batch_ordered(b, verdicts=self.verdicts, seq=self.seq)
        else:
            self.svc.submit_param_batch(b, verdicts=self.verdicts)

    def _host(self, batches, k):
        e = self.torch.cat(batches[:k]).cpu().numpy()
        return (e[:, 0] & 0xFFFFFFFF).astype(np.int32), (e[:, 0] >> 32).astype(np.int32), e[:, 2].astype(np.uint64), e[:, 1].copy()

    def _oracle(self):
        from oracle import oracle as O
        return O.TokenServiceOracle([], param_rules=self.prules, hot_items={r: list(h.items()) for r, h in self.hot.items()})

    def cpu_baseline(self, batches, k1, kmt, threads):
        ridx, acq, keys, ts = self._host(batches, k1)
        orc = self._oracle()
        c0 = time.perf_counter()
        orc.param_replay(ridx, acq, keys, ts)
        cdt = time.perf_counter() - c0
        one = (len(ts), cdt, 1, "sequential oracle replay (ClusterParamFlowChecker, exact counters)")
        ridx, acq, keys, ts = self._host(batches, kmt)
        orc = self._oracle()
        c0 = time.perf_counter()
        st, rem, used = orc.param_replay_mt(ridx, acq, keys, ts, threads)
        cdt = time.perf_counter() - c0
        if self.kept and not self.cm:
            from sentinel_amd.token_service import decode_verdicts
            g = [decode_verdicts(arrival_order(self.torch, v)) for v in self.kept]
            gs, gr = np.concatenate([x[0] for x in g]), np.concatenate([x[1] for x in g])
            m = min(len(gs), len(st))
            self.parity_result = {
                "parity_checked_events": m, "parity_mismatches": int(((gs[:m] != st[:m]) | (gr[:m] != rem[:m])).sum()),
                "parity_note": f"status and remaining of the first {len(self.kept)} batches (warmup + profile steps) "
                               f"against the CPU baseline's oracle replay of the same requests"}
        elif self.cm:
            self.parity_result = {"parity_checked_events": 0, "parity_mismatches": None,
                                  "parity_note": "count-min mode is not exact by design: see count_min (one-sidedness "
                                                 "audit of the same batches on exact counters)"}
        return one, (len(ts), cdt, int(used), f"oracle replay sharded by rule over {used} pthreads (exact counters)")

    def false_blocks(self, batches, k, svc_verdicts):
        """Count-min audit: the sketch's verdicts replayed on exact counters (same admitted history):
        violations (sketch passed, exact would block) must be 0; false blocks are the price of the sketch."""
        ridx, acq, keys, ts = self._host(batches, k)
        from sentinel_amd.token_service import decode_verdicts
        st = np.concatenate([decode_verdicts(arrival_order(self.torch, v))[0] for v in svc_verdicts]).astype(np.int8)
        orc = self._oracle()
        ones = np.ones(len(ts), np.int32)
        viol, fb, dec = orc.param_cm_audit(ridx, acq, ts, np.arange(len(ts), dtype=np.int32), ones, keys, st)
        return viol, fb, dec

    def distinct_keys(self, b):
        """(rule, value) keys one batch touches (untimed; for the per-key share of the algorithmic bytes)."""
        if not hasattr(self, "_dk"):
            self._dk = int(self.torch.unique(b[:, 2]).numel())
        return self._dk

    def bytes_of(self, dom, d, steps):
        if dom == "radix_scatter":
            passes = max(1, round(d["calls"] / max(1, steps)))
            return (32.0 + 24.0 * (passes - 1)) / passes
        if dom == "param_group":
            # per request: the range's keys read once per sub-range workgroup (8 B x S, L2-shared), its
            # packed value 8 + rule 4 read, the grouped value written 8; per distinct key a 16-B record
            nsub = 1
            while 1024 * nsub * 1024 < self.N and nsub < 256:
                nsub *= 2
            e_k = self.N / max(1, self._dk) if hasattr(self, "_dk") else 1.0
            return 8.0 * nsub + 20.0 + 16.0 / e_k + (4.0 if self.ordered else 0.0)   # (+ seq in decide order)
        if dom == "param_decide":
            # per request: read the 8-B grouped value, write the 8-B verdict; per distinct (rule, value)
            # key: its 16-B record, the slot probe 8, its n {epoch, count} pairs read (16 n) and the
            # rolled pair written back (16), the rule's window fields + threshold (~24 B)
            e_k = self.N / max(1, self._dk) if hasattr(self, "_dk") else 1.0
            return 16.0 + (16 + 8 + 16 * self.n + 16 + 24) / e_k
        if dom == "process":
            # per touched (rule, value) slot: read n {epoch, count} pairs, write one; per event: segment record
            return 24.0 + (self.n * 16 + 16) / 4.0
        if dom == "param_cm_block":
            # per batch every sketch block with keys read once (all of them at 4cm: w x d x 2 n 8-B slots), the
            # slots added to written back; per request the grouped value read 8, the verdict written 8; per
            # distinct key its 16-B record and the rule record 32, and per live admitted epoch (within 2 n
            # epochs of the batch's end) one slot per row written (8)
            e_k = self.N / max(1, self._dk) if hasattr(self, "_dk") else 1.0
            live = min(1.0, 2.0 * self.interval / max(1.0, float(self.span_ms())))
            blocks = float(self.cm_width) * self.cm_depth * 2 * self.n * 8 / self.N
            return blocks + 16.0 + (16 + 32 + live * self.cm_depth * 8) / e_k
        if dom in ("param_cm_walk", "param_cm_read"):
            # walk, per request: the grouped value read 8, the verdict written 8 (+ M(E) 8 for the requests
            # within n epochs of the previous batch); per distinct key: its 16-B record, the rule record 32,
            # per sketch row one slot read-modify-written (8 + 8) per admitted epoch (>= 1).  read, per
            # request: the grouped value 8; per key in the first n epochs: d rings of 2 n 8-B slots
            e_k = self.N / max(1, self._dk) if hasattr(self, "_dk") else 1.0
            frac_early = min(1.0, self.interval / max(1.0, float(self.span_ms())))
            if dom == "param_cm_read":
                return 8.0 + 8.0 * frac_early + (16 + 32 + frac_early * self.cm_depth * 2 * self.n * 8) / e_k
            return 16.0 + 8.0 * frac_early + (16 + 32 + self.cm_depth * 16) / e_k
        if dom == "prule_process" and self.cm:
            # per request: its sorted value 8 + event 24 read, the verdict 8 written; per row of the sketch
            # the value's cell (a ring of 2 n 8-B slots) read and one slot read-modify-written (8 + 8)
            return 8 + 24 + 8 + self.cm_depth * (2 * self.n * 8 + 16)
        return KERNEL_BYTES_PER_EVENT.get(dom)

    def pipeline_bytes(self):
        return 24.0 + 8.0 + (self.n * 16 * 2 + 16) / 4.0

    def shape(self):
        return {"config": self.args.config, "rules": self.R, "events": self.N, "sample_count": self.n,
                "output": "decide order + arrival positions" if self.ordered else "arrival order"}


class ConcWorkload:
    """Concurrency-token batches of config 5's thread-grade half (sentinel_concurrent_event_t): a fixed
    pattern of acquire / release positions; batch s + 1 releases, at its release positions, the tokens
    batch s handed out at its acquire positions (a client holding a token releases it one batch later;
    blocked acquires hold no token, so their release answers ALREADY_RELEASE).  The release token ids
    are gathered on the engine stream from the previous batch's results before each submit (part of
    the timed step: it is the clients' traffic)."""

    def __init__(self, args, world, rank, dev):
        import torch
        import sentinel_amd as sa
        from sentinel_amd import trace as T
        self.T, self.torch, self.dev, self.args = T, torch, dev, args
        rng = np.random.default_rng(55)
        flows = args.flows or 20_000
        rules = T.make_rules(flows, rng, count_lo=50, count_hi=5000, sample_count=1, window_interval_ms=1000)
        mine = np.nonzero(T.shard_of(rules.flow_id, world) == rank)[0] if world > 1 else np.arange(len(rules))
        self.rules = rules.subset(mine)
        self.F = len(self.rules)
        self.N = args.events_per_gpu or 4 * 1024 * 1024
        self.svc = sa.GpuTokenService(dev.index or 0)
        r = self.rules
        self.svc.load_rules_array(r.flow_id, r.count, r.threshold_type, r.sample_count, r.window_interval_ms,
                                  r.namespace, r.checker)
        N = self.N
        # half of the positions acquire, the other half release the previous batch's acquires: a random
        # subset of the acquires, released in the order they were acquired (clients hand tokens back first
        # in, first out; the released tokens' flows are as random as before, and the glue's gather / scatter
        # runs over increasing positions -- 64 us per step as a random pairing, scripts/glue_study.py)
        perm = rng.permutation(N)
        self.acq_pos = np.sort(perm[: N // 2])
        self.rel_pos = np.sort(perm[N // 2:])
        src = np.sort(rng.permutation(len(self.acq_pos))[: len(self.rel_pos)])
        self.g = torch.Generator(device=dev).manual_seed(3000 + rank)
        self.acq_pos_d = torch.from_numpy(self.acq_pos.astype(np.int64)).to(dev)
        self.rel_pos_d = torch.from_numpy(self.rel_pos.astype(np.int64)).to(dev)
        self.rel_src_d = torch.from_numpy(self.acq_pos[src].astype(np.int64)).to(dev)
        # flat word indices of the same gather / scatter: token id = word 0 of a (N, 2) result row, word 1
        # of a (N, 3) event row (two 1-D kernels instead of strided index_select / index_copy_)
        self.rel_dst_w = self.rel_pos_d * 3 + 1
        self.rel_src_w = self.rel_src_d * 2
        # the same gather / scatter as one kernel with 32-bit positions (tools/bench_glue.hip, built by
        # __graft_entry__.build()); BENCH_GLUE=torch or a missing library keeps the two torch kernels
        self.glue = None
        glue_so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "libbench_glue.so")
        if os.environ.get("BENCH_GLUE", "kernel") != "torch" and os.path.exists(glue_so):
            import ctypes
            lib = ctypes.CDLL(glue_so)
            lib.bench_glue_forward_tokens.restype = ctypes.c_int
            lib.bench_glue_forward_tokens.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64, ctypes.c_void_p]
            self.glue = lib.bench_glue_forward_tokens
            self.rel_pos32 = self.rel_pos_d.to(torch.int32)
            self.rel_src32 = self.rel_src_d.to(torch.int32)
        self.glue_kind = "tools/bench_glue.hip kernel" if self.glue else "torch index_select + index_copy_"
        w = 1.0 / np.power(np.arange(1, self.F + 1, dtype=np.float64), 1.1)
        self.zipf_cdf = torch.from_numpy(np.cumsum(w) / w.sum()).to(dev)
        self.zipf_perm = torch.from_numpy(np.random.default_rng(9).permutation(self.F).astype(np.int32)).to(dev)
        self.results = [torch.zeros((N, 2), dtype=torch.int64, device=dev) for _ in range(2)]
        self.k = 0
        self.verdicts = self.results[0]
        self.workload = (f"config5conc: {self.F} thread-grade cluster rules (ConcurrentClusterFlowChecker, count~U{{50..5000}}), "
                         f"Zipf(1.1) flows, {N}-event batches of half acquires (1 token) and half releases of the "
                         f"previous batch's tokens, device-pointer path; release ids forwarded in the timed step "
                         f"by the {self.glue_kind}")
        self.kept = []
        self.parity_result = None

    def batch(self, s):
        torch, N = self.torch, self.N
        u = torch.rand(N, dtype=torch.float64, device=self.dev, generator=self.g)
        idx = self.zipf_perm[torch.clamp(torch.searchsorted(self.zipf_cdf, u, right=True), max=self.F - 1)]
        kind = torch.zeros(N, dtype=torch.int32, device=self.dev)
        kind[self.rel_pos_d] = 1
        return self.svc.concurrent_events(idx, torch.ones(N, dtype=torch.int32, device=self.dev),
                                          torch.zeros(N, dtype=torch.int64, device=self.dev), kind,
                                          torch.ones(N, dtype=torch.int32, device=self.dev))

    def span_ms(self):
        return 0

    def submit(self, b, keep=False):
        torch = self.torch
        prev, cur = self.results[self.k % 2], self.results[(self.k + 1) % 2]
        if self.glue:                                      # the releases name the previous batch's tokens
            assert b.is_contiguous() and b.shape == (self.N, 3) and prev.is_contiguous()
            rc = self.glue(b.data_ptr(), prev.data_ptr(), self.rel_pos32.data_ptr(), self.rel_src32.data_ptr(),
                           len(self.rel_pos), self.svc.stream)
            if rc != 0:
                raise RuntimeError(f"bench_glue_forward_tokens: {rc}")
        else:
            ext = torch.cuda.ExternalStream(self.svc.stream, device=self.dev)
            with torch.cuda.stream(ext):
                b.view(-1).index_copy_(0, self.rel_dst_w, prev.view(-1).index_select(0, self.rel_src_w))
        self.svc.submit_concurrent_batch(b, results=cur)
        self.verdicts = cur
        self.k += 1
        if keep:                                           # warmup / profile steps only
            self.svc.synchronize()
            self.kept.append((b.clone(), cur.clone()))

    def cpu_baseline(self, batches, k1, kmt, threads):
        from oracle import oracle as O
        r = self.rules
        orc = O.TokenServiceOracle.from_arrays(r.flow_id, r.count, r.threshold_type, r.sample_count,
                                               r.window_interval_ms, r.namespace, r.checker)
        evs = []
        for b, res in self.kept:
            e = b.cpu().numpy()
            ev = np.zeros(len(e), dtype=orc.CONC_EVENT)
            ev["flow_idx"] = (e[:, 0] & 0xFFFFFFFF).astype(np.int32)
            ev["acquire"] = (e[:, 0] >> 32).astype(np.int32)
            ev["token_id"] = e[:, 1]
            ev["kind"] = (e[:, 2] & 0xFFFFFFFF).astype(np.int32)
            ev["flags"] = (e[:, 2] >> 32).astype(np.int32)
            evs.append((ev, res[:, 0].cpu().numpy()))
        c0 = time.perf_counter()
        m = 0
        for ev, ids in evs[:k1]:
            orc.concurrent_replay(ev, ids)
            m += len(ev)
        cdt = time.perf_counter() - c0
        one = (m, cdt, 1, "sequential oracle replay (ConcurrentClusterFlowChecker, the engine's token ids)")
        orc = O.TokenServiceOracle.from_arrays(r.flow_id, r.count, r.threshold_type, r.sample_count,
                                               r.window_interval_ms, r.namespace, r.checker)
        all_ev = np.concatenate([ev for ev, _ in evs])
        all_ids = np.concatenate([ids for _, ids in evs])
        c0 = time.perf_counter()
        st, _, used = orc.concurrent_replay_mt(all_ev, all_ids, threads)
        cdt = time.perf_counter() - c0
        gst = np.concatenate([res[:, 1].cpu().numpy() for _, res in self.kept]).astype(np.int32).astype(np.int8)
        self.parity_result = {
            "parity_checked_events": int(len(st)), "parity_mismatches": int((gst != st).sum()),
            "parity_note": f"statuses of the first {len(self.kept)} batches (warmup + profile steps: half acquires, half "
                           f"releases of the previous batch's tokens) against the CPU baseline's oracle replay"}
        return one, (len(all_ev), cdt, int(used),
                     f"oracle replay sharded by flow over {used} pthreads (a token cache per thread, releases routed "
                     f"to their token's thread; the engine's token ids)")

    def bytes_of(self, dom, d, steps):
        if dom == "conc_scan":
            # per event: sorted key 4 + value 8 read (the value carries the amount / token slot), element
            # 4 written (+ pass byte per acquire); per release (half the events) its 32-B token record read
            # and written back
            return 4 + 8 + 4 + 0.5 * 1 + 0.5 * (32 + 32)
        if dom == "radix_scatter":
            passes = max(1, round(d["calls"] / max(1, steps)))
            return (32.0 + 24.0 * (passes - 1)) / passes
        return KERNEL_BYTES_PER_EVENT.get(dom)

    def pipeline_bytes(self):
        return 24.0 + 16.0 + 8.0 + 16.0

    def shape(self):
        return {"config": self.args.config, "flows": self.F, "events": self.N}


CM_AUDIT_BATCHES = 6    # consecutive 4cm batches audited on exact counters (each spans ~80 epochs of 100 ms)


def arrival_order(torch, k):
    """A kept batch's verdicts at their arrival positions: decide-order output (verdicts, seq) is put
    back through its seq after the fact (the parity check and the count-min audit only)."""
    if not isinstance(k, tuple):
        return k
    v, sq = k
    s = sq.to(torch.int64)
    assert torch.equal(torch.sort(s).values, torch.arange(len(s), device=s.device)), "decide-order seq is not a permutation"
    out = torch.empty_like(v)
    out[s] = v
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # SENTINEL_BENCH_ONE_DEVICE=1: every rank on cuda:0 over gloo -- a rehearsal of the N-rank path on a
    # one-GPU box (sharding, barriers, max-over-ranks timing, the snapshot all-gathers); never a result
    one_dev = os.environ.get("SENTINEL_BENCH_ONE_DEVICE") == "1"
    if one_dev:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if one_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    if args.config in ("4", "4cm"):
        W = ParamWorkload(args, world, rank, dev)
    elif args.config == "5conc":
        W = ConcWorkload(args, world, rank, dev)
    else:
        W = FlowWorkload(args, world, rank, dev)
    svc, N = W.svc, W.N
    # warmup | untimed per-kernel profile pass (every kernel timed: the breakdown) | timed steps
    # (only the dominant kernel timed, two events per step: its live duration for the roofline)
    pstep = 0 if args.no_profile else args.profile_steps
    steps_total = args.warmup + pstep + args.steps
    ev_b = [W.batch(s) for s in range(steps_total)]
    if hasattr(W, "distinct_keys"):
        W.distinct_keys(ev_b[0])
    torch.cuda.synchronize()
    log(f"config {args.config}: {steps_total} batches of {N} events generated")

    ext = torch.cuda.ExternalStream(svc.stream, device=dev)
    # the first batches (warmup + profile steps, never the timed ones) decide into verdict buffers of their
    # own, checked against the CPU baseline's oracle replay of the same events (parity_* fields)
    check = rank == 0 and world == 1 and not args.no_cpu_baseline
    keep_n = min(args.cpu_steps_mt, args.warmup + pstep) if check else 0
    if args.config == "4cm":                                    # the count-min audit's sample: the first six batches
        keep_n = max(keep_n, min(CM_AUDIT_BATCHES, args.warmup + pstep))   # (~480 epochs: a 140-240-epoch re-touch)
    for s in range(args.warmup):
        W.submit(ev_b[s], keep=s < keep_n)
    svc.synchronize()

    import ctypes as C

    def read_profile():
        mx = 64
        names = C.create_string_buffer(32 * mx)
        tot = (C.c_double * mx)()
        calls = (C.c_int64 * mx)()
        units = (C.c_int64 * mx)()
        k = svc._L.sentinel_profile_read(svc.handle, mx, names, tot, calls, units)
        out = {}
        for i in range(k):
            nm = names.raw[32 * i:32 * i + 32].split(b"\0")[0].decode()
            out[nm] = dict(total_ms=tot[i], calls=calls[i], avg_us=1000.0 * tot[i] / max(calls[i], 1),
                           units_per_call=units[i] / max(calls[i], 1))
        return out

    breakdown, dom = {}, None
    if not args.no_profile:
        svc._L.sentinel_profile_enable(svc.handle, 1)
        for s in range(args.warmup, args.warmup + pstep):
            W.submit(ev_b[s], keep=s < keep_n)
        svc.synchronize()
        breakdown = read_profile()
        svc._L.sentinel_profile_enable(svc.handle, 0)
        dom = max(breakdown, key=lambda k: breakdown[k]["total_ms"])
        svc._L.sentinel_profile_select(svc.handle, dom.encode())
        svc._L.sentinel_profile_enable(svc.handle, 1)
    # the timed steps: barrier + synchronize on both sides, max over ranks; the dominant kernel is
    # bracketed by the engine's HIP events on every `kernel_every`-th timed step
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        s = args.warmup + pstep + k
        if not args.no_profile:
            svc._L.sentinel_profile_gate(svc.handle, 1 if k % args.kernel_every == 0 else 0)
        W.submit(ev_b[s])
    svc.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    el = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if one_dev else dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    # ---- the dominant kernel's live duration over the timed region (HIP events on the engine stream)
    prof = {}
    if not args.no_profile:
        prof = read_profile()
        svc._L.sentinel_profile_enable(svc.handle, 0)
        svc._L.sentinel_profile_select(svc.handle, None)

    # ---- latency loop (untimed): >= 200 batches continuing the trace; K buffers reused with their
    # timestamps shifted forward in place (so time stays monotone), one torch event per batch boundary
    # on the engine stream (device batch latency, back to back), then the same batches each followed by
    # a host synchronize (submit -> verdicts visible to the host, host clock)
    log("timed steps done; latency loop")
    K = 8
    L = max(1, args.latency_batches)
    lat_b = [W.batch(steps_total + j) for j in range(K)]
    shift = K * W.span_ms()
    torch.cuda.synchronize()

    def advance():
        # the K buffers move one K-batch span forward in time, on the engine stream (ordered with the
        # batches that read them)
        with torch.cuda.stream(ext):
            for b in lat_b:
                b[:, 1] += shift

    for j in range(min(K, L)):
        W.submit(lat_b[j])                               # first use of these buffers (not timed)
    advance()
    # a start and an end event per batch: the timestamp shifts of `advance` (8 elementwise kernels,
    # ~0.4 ms, every K-th batch) run between one batch's end and the next one's start, outside both
    tev0 = [torch.cuda.Event(enable_timing=True) for _ in range(L)]
    tev1 = [torch.cuda.Event(enable_timing=True) for _ in range(L)]
    for i in range(L):
        if i and i % K == 0:
            advance()
        tev0[i].record(ext)
        W.submit(lat_b[i % K])
        tev1[i].record(ext)
    torch.cuda.synchronize()
    lat_seq = [tev0[i].elapsed_time(tev1[i]) for i in range(L)]
    lat = sorted(lat_seq)
    slow = sorted(range(L), key=lambda i: -lat_seq[i])[:8]
    log("slowest batches of the latency loop (index: ms): " + ", ".join(f"{i}: {lat_seq[i]:.3f}" for i in sorted(slow)))
    if os.environ.get("BENCH_LAT_ALL"):
        log("latency loop, every batch (ms): " + " ".join(f"{x:.3f}" for x in lat_seq))
    hl = []
    for i in range(L):
        if i % K == 0:
            advance()
            svc.synchronize()
        h0 = time.perf_counter()
        W.submit(lat_b[i % K])
        svc.synchronize()
        hl.append((time.perf_counter() - h0) * 1000.0)
    hl.sort()
    svc.synchronize()
    t_snap = int(lat_b[(L - 1) % K][-1, 1].item()) + 1    # right after the newest batch the engine decided
    advance()
    svc.synchronize()
    log("latency loop done")

    def pct(xs, q):
        return xs[min(len(xs) - 1, int(np.ceil(q * len(xs))) - 1)]

    # ---- snapshot + RCCL all-gather (the ClusterMetric snapshot, ClusterMetricNodeGenerator: flow records
    # for the flow configs, top-5 param records for config 4; off the decision path)
    from sentinel_amd import shard as SH
    snap_ms = snap_first_ms = None

    def snapshot_once():
        torch.cuda.synchronize()
        ts0 = time.perf_counter()
        if isinstance(W, FlowWorkload):
            snap = torch.empty((W.F, 3), dtype=torch.int64, device=dev)
            svc.snapshot_device(t_snap, snap)
            svc.synchronize()
            if world > 1:
                SH.gather_snapshot(snap)
        else:
            snap = torch.empty(W.R * SH.PARAM_RECORD_WORDS * 8, dtype=torch.uint8, device=dev)
            svc.param_snapshot_device(t_snap, snap)
            svc.synchronize()
            if world > 1:
                SH.gather_param_snapshot(snap)
        torch.cuda.synchronize()
        return (time.perf_counter() - ts0) * 1000.0

    if not isinstance(W, ConcWorkload):                  # (no windowed metrics: the snapshot is the flow configs')
        snap_first_ms = snapshot_once()                  # (first call: scratch allocation)
        snap_ms = float(np.median([snapshot_once() for _ in range(5)]))   # steady state: the periodic snapshot

    # PCIe-inclusive host paths (config 3 only; reported beside `value`, never as it)
    host_path = None
    if rank == 0 and not args.no_host_path and args.config == "3":
        m = min(N, 1 << 20)
        hev = torch.empty((N, 2), dtype=torch.int64, pin_memory=True)
        hev.copy_(lat_b[0])
        hout = torch.empty(N, dtype=torch.int64, pin_memory=True)
        reps = max(1, args.host_reps)
        nbs = (N + m - 1) // m
        bms = np.zeros(nbs, dtype=np.float32)
        assert svc._L.sentinel_submit_flow_batch_host(svc.handle, m, C.c_void_p(hev.data_ptr()), None,
                                                      C.c_void_p(hout.data_ptr())) == 0
        assert svc._L.sentinel_submit_flow_stream_host(svc.handle, N, C.c_void_p(hev.data_ptr()), None,
                                                       C.c_void_p(hout.data_ptr()), m, None) == 0
        hlp = []
        hts = hev[:, 1].numpy()          # every rep decides a batch later in time (its timestamps shifted)
        for _ in range(reps):
            hts += W.span_ms()
            h0 = time.perf_counter()
            rc = svc._L.sentinel_submit_flow_batch_host(svc.handle, m, C.c_void_p(hev.data_ptr()), None,
                                                        C.c_void_p(hout.data_ptr()))
            assert rc == 0
            hlp.append((time.perf_counter() - h0) * 1000.0)
        hlp.sort()
        sreps = 5
        sdts = []
        for _ in range(sreps):
            hts += W.span_ms()            # (the timestamp shift of the next pass stays outside its clock)
            s0 = time.perf_counter()
            rc = svc._L.sentinel_submit_flow_stream_host(svc.handle, N, C.c_void_p(hev.data_ptr()), None,
                                                         C.c_void_p(hout.data_ptr()), m,
                                                         C.c_void_p(bms.ctypes.data))
            sdts.append(time.perf_counter() - s0)
            assert rc == 0
        sdt = sum(sdts) / sreps
        bl = np.sort(bms)
        host_path = {
            "sync": {"decisions_per_s": round(m * reps / (sum(hlp) / 1000.0), 1), "batch": m, "reps": reps,
                     "median_ms": round(hlp[len(hlp) // 2], 3), "p99_ms": round(pct(hlp, 0.99), 3),
                     "note": "pinned host events -> H2D -> decide -> D2H, synchronous per batch, host clock"},
            "streamed": {"decisions_per_s": round(N / sdt, 1), "events": N, "batch": m,
                         "p99_batch_ms": round(float(pct(list(bl), 0.99)), 3), "batches_per_rep": nbs,
                         "note": "sentinel_submit_flow_stream_host: H2D / decide / D2H of consecutive batches "
                                 "overlapped on side streams; batch latency = HIP events H2D start -> D2H end "
                                 "(includes queueing behind the previous batch)"},
        }
        host_path["streamed_over_sync"] = round(host_path["streamed"]["decisions_per_s"] /
                                                max(1.0, host_path["sync"]["decisions_per_s"]), 3)
        if host_path["streamed_over_sync"] < 1.0:
            log(f"WARNING: the streamed host path is slower than the synchronous one "
                f"({host_path['streamed_over_sync']}x): the copy / decide overlap is not working")
        del hev, hout

    total_events = float(N) * args.steps * world
    value = total_events / elapsed

    # ---- roofline of the dominant kernel
    roof = None
    if prof and dom in prof:
        d = prof[dom]
        bpe = W.bytes_of(dom, d, args.steps)
        ach = (bpe or 0.0) * d["units_per_call"] / (d["avg_us"] * 1e-6) / 1e9
        traffic, traffic_src = pmc_traffic(dom, W.shape())
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_unit": "HBM bytes per launch (rocprofv3 memory-side requests of this workload shape: "
                                + (traffic_src or "no PMC run of this shape -> null") + ")",
                "algorithmic_bytes_per_launch": round((bpe or 0.0) * d["units_per_call"], 1),
                "bytes_per_event": bpe, "avg_us": round(d["avg_us"], 2)}

    # ---- rule reload at the workload's size (ClusterFlowRuleManager.loadRules: putMetricIfAbsent keeps
    # surviving flowIds' windows, the device remaps the blocked tables): 5% of the flowIds removed, 5% of
    # the survivors with a new window (they keep their old metric), 5% new flowIds; host clock around the
    # call, which returns with the new table in place (untimed region, after every other leg)
    reload_ms = None
    if isinstance(W, FlowWorkload) and args.config in ("3", "2"):
        r = W.rules
        F = len(r.flow_id)
        keep = np.arange(F) % 20 != 7
        fid = np.concatenate([r.flow_id[keep], r.flow_id.max() + 1 + np.arange(F // 20, dtype=np.int64)])
        cnt = np.concatenate([r.count[keep], r.count[: F // 20]])
        sc = np.concatenate([r.sample_count[keep], r.sample_count[: F // 20]]).astype(np.int32)
        sc[: len(sc) // 20] = np.where(sc[: len(sc) // 20] % 2 == 0, sc[: len(sc) // 20] // 2, sc[: len(sc) // 20])
        tt = np.full(len(fid), 1, np.int32)
        wi = np.full(len(fid), 1000, np.int32)
        ns = np.zeros(len(fid), np.int32)
        ck = np.zeros(len(fid), np.int32)
        svc.synchronize()
        r0 = time.perf_counter()
        svc.load_rules_array(fid, cnt, tt, sc, wi, ns, ck)
        svc.synchronize()
        reload_ms = (time.perf_counter() - r0) * 1000.0
        log(f"rule reload of {len(fid)} flows: {reload_ms:.1f} ms")

    # ---- CPU baseline: the oracle ("port") on bounded samples of the same workload, rank 0, N=1
    cpu = cpu1 = None
    extra_parity = {"parity_checked_events": 0, "parity_mismatches": None,
                    "parity_note": "not checked in this run (CPU baseline off, or rank > 0 / N > 1)"}
    model, ncpu, avail = cpu_info()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline")
        one, mt = W.cpu_baseline(ev_b, min(args.cpu_steps_1core, steps_total), min(args.cpu_steps_mt, steps_total),
                                 args.cpu_threads or cpu_threads_default())

        def leg(x):
            m, cdt, cores, how = x
            return {"value": round(m / cdt, 1), "unit": "decisions/s", "cores": cores, "kind": "port",
                    "cpu_model": model, "nproc": ncpu, "cpus_available": avail, "cgroup_cpu_quota": cgroup_cpus(),
                    "sample": f"the first {m} events of this workload (same rules and trace), {how}, {cdt:.1f} s"}
        cpu1 = leg(one)
        cpu = leg(mt) if mt else cpu1
        if W.parity_result is not None:
            extra_parity = W.parity_result
            log(f"parity: {extra_parity['parity_mismatches']} mismatches in {extra_parity['parity_checked_events']} events")

    extra = {}
    if args.config == "4cm" and rank == 0 and world == 1:
        keep_verdicts = W.kept[:CM_AUDIT_BATCHES]
        k = len(keep_verdicts)
        viol, fb, dec = W.false_blocks(ev_b, k, keep_verdicts)
        eps_n = float(np.e) / W.cm_width * float(N) * k      # e/w x (requests counted in the audited span)
        extra["count_min"] = {"depth": W.cm_depth, "width": W.cm_width, "audited_requests": int(dec),
                              "violations": int(viol), "false_blocks": int(fb),
                              "false_block_rate": round(fb / max(1, dec), 8),
                              "eps_N_bound_counts": round(eps_n, 2),
                              "note": f"the sketch's verdicts of the first {k} consecutive batches (warmup + profile) replayed on exact counters "
                                      "(oracle, same admitted history): violations = sketch passed what exact would "
                                      "block (must be 0); bound (blocked layout): P[overestimate > (e/64) N_B] <= exp(-d), N_B = the "
                                      "window count of the key's 64-column block, E[N_B] = 64 N / w, so (e/w) N on "
                                      "average, N = all requests counted in the window (upper bound used: every "
                                      "audited request)"}
        st = svc.param_table_stats()
        extra["param_table"] = st
    if args.config == "4" and rank == 0:
        extra["param_table"] = svc.param_table_stats()

    out = {
        "metric": "token decisions/sec (whole node) at 1M flowIds; p99 batch latency",
        "value": round(value, 1),
        "unit": "decisions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1000.0 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64+f64",
        "data": "synthetic (seeded events on the device; random-init rule table)",
        "config": {"workload": W.workload, "events_per_gpu_per_step": N,
                   "parallelism": f"flowid-shard x{world}", **W.shape()},
        "p99_batch_ms": round(pct(lat, 0.99), 4),
        "median_batch_ms": round(lat[len(lat) // 2], 4),
        "latency_note": (f"{L} batches of an untimed loop after the timed steps: device time per batch between "
                         f"a start and an end torch event around each submit on the engine stream (batches back "
                         f"to back); p99_sync_ms = host clock with a synchronize per batch"),
        "p99_sync_ms": round(pct(hl, 0.99), 4),
        "median_sync_ms": round(hl[len(hl) // 2], 4),
        "snapshot_allgather_ms": None if snap_ms is None else round(snap_ms, 3),
        "snapshot_first_call_ms": None if snap_first_ms is None else round(snap_first_ms, 3),
        "rule_reload_ms": None if reload_ms is None else round(reload_ms, 2),
        "host_path": host_path,
        "pipeline_bytes_per_decision": round(W.pipeline_bytes(), 2),
        "pipeline_hbm_frac": round(value / world * W.pipeline_bytes() / (HBM_PEAK_GBS * 1e9), 4),
        "pipeline_bytes_engine_layout": (round(W.pipeline_bytes_engine(), 2)
                                         if hasattr(W, "pipeline_bytes_engine") else None),
        "pipeline_hbm_frac_engine_layout": (round(value / world * W.pipeline_bytes_engine() / (HBM_PEAK_GBS * 1e9), 4)
                                            if hasattr(W, "pipeline_bytes_engine") else None),
        "roofline": roof,
        "cpu_baseline": cpu,
        "cpu_baseline_1core": cpu1,
        **extra_parity,
        **extra,
        "kernels": {k: {"avg_us": round(v["avg_us"], 2), "calls": v["calls"]} for k, v in breakdown.items()},
        "kernels_note": (f"per-kernel HIP-event averages from {pstep} untimed profiled steps after the warmup; the "
                         "timed steps time only the dominant kernel (roofline.avg_us)"),
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
