"""bench.py -- token decisions/sec of the MI355X engine on BASELINE config 3.

Workload (BASELINE.json configs[2], the config the headline metric is quoted on): a universe of
1M flowIds (cluster FlowRules, GLOBAL threshold count ~ U{10..1000}, default cluster window
sampleCount=10 / windowIntervalMs=1000 -> 10 x 100 ms buckets), hash-sharded over the ranks by
splitmix64(flowId) mod N.  Every rank decides a fixed 8M-event batch per step over its own flows
(uniform, acquire 1, monotone timestamps at 2x the shard's summed thresholds): weak scaling, no
collective on the decision path.  A step = one batch through DefaultTokenService.requestToken
semantics (validation, window roll, ClusterFlowChecker admission, verdict write-back), inputs
already resident in HBM.

Prints ONE JSON line (rank 0).  Extra fields: p99 device batch latency, per-kernel profile,
the roofline of the dominant kernel, and the CPU oracle ("port") timed on a bounded sample.
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

# Algorithmic bytes per processed event for each kernel of the pipeline (DESIGN.md "Kernels").
KERNEL_BYTES_PER_EVENT = {
    "flow_prep": 20.0,        # read the 16-B event, write the 4-B sort key (histograms stay in LDS)
    "radix_hist": 4.0,        # read key
    "radix_scatter": None,    # per pass: read key 4 + value 8, write 12; pass 0 reads the 16-B event instead of a value
    "scan_tiles": 8.0,
    "scan_add": 8.0,
    "seg_heads": 17.0,        # read key 4 + value 8, write head 4 + homogeneity flag 1
    "seg_mark": 5.0,          # read segid 4 + flag 1 (segment records are per segment)
    "verdict": 20.0,          # read segid 4 + value 8, write the 8-B verdict
    "part_prep": 16.0,        # read the 16-B event (range histogram in LDS; no key array without namespace routes)
    "part_scatter": 24.0,     # read the 16-B event (key re-derived), write the 8-B packed value (local key inside)
}


# rocprofv3 kernel symbols behind each engine profile name (for the PMC traffic of the roofline).
KERNEL_SYMBOLS = {
    "flow_prep": ("k_flow_prep",), "radix_hist": ("k_radix_hist_pass",), "radix_scatter": ("k_radix_scatter_p",),
    "scan": ("k_scan_lookback",), "segments": ("k_segments",), "process": ("k_process",), "verdict": ("k_verdict",),
    "part_prep": ("k_part_prep",), "part_scatter": ("k_part_scatter",),
    "part_fused": ("k_part_half",), "part_big": ("k_part_big",), "part_long": ("k_part_long",),
}
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_latest.json")


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this workload
    (scripts/gpu_round.sh: separate FETCH_SIZE / WRITE_SIZE passes, FETCH doubled on gfx950)."""
    try:
        with open(PMC_SUMMARY) as f:
            summ = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    pats = KERNEL_SYMBOLS.get(kernel, ())
    tot = disp = 0.0
    for name, v in summ.items():
        if any(name.startswith(p) for p in pats) and v.get("traffic_bytes_avg"):
            tot += v["traffic_bytes_avg"] * v["dispatches"]
            disp += v["dispatches"]
    return round(tot / disp, 1) if disp else None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--events-per-gpu", type=int, default=8 * 1024 * 1024)
    ap.add_argument("--flows", type=int, default=1_000_000)
    ap.add_argument("--sample-count", type=int, default=10)
    ap.add_argument("--interval-ms", type=int, default=1000)
    ap.add_argument("--cpu-steps-1core", type=int, default=2)
    ap.add_argument("--cpu-steps-mt", type=int, default=12)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--kernel-every", type=int, default=2,
                    help="time the dominant kernel with HIP events on every k-th timed step")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-fed legs")
    ap.add_argument("--host-reps", type=int, default=20)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import sentinel_amd as sa
    from sentinel_amd import trace as T

    # ---- rule universe (identical on every rank), then this rank's shard
    rng = np.random.default_rng(3)
    rules = T.make_rules(args.flows, rng, sample_count=args.sample_count, window_interval_ms=args.interval_ms)
    mine = np.nonzero(T.shard_of(rules.flow_id, world) == rank)[0] if world > 1 else np.arange(len(rules))
    shard = rules.subset(mine)
    F = len(shard)

    svc = sa.GpuTokenService(local)
    svc.load_rules_array(shard.flow_id, shard.count, shard.threshold_type, shard.sample_count,
                         shard.window_interval_ms, shard.namespace, shard.checker)

    N = args.events_per_gpu
    # warmup | untimed per-kernel profile pass (every kernel timed: the breakdown) | timed steps
    # (only the dominant kernel timed, two events per step: its live duration for the roofline)
    pstep = 0 if args.no_profile else args.profile_steps
    steps_total = args.warmup + pstep + args.steps
    rate = 2.0 * float(shard.count.sum())          # offered rate: 2x the shard's thresholds (per second)
    ms_per_event = 1000.0 / rate
    t0 = T.T0_ALIGNED
    from sentinel_amd.token_service import device_events
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    ev_b = []
    acq = torch.ones(N, dtype=torch.int32, device=dev)
    for s in range(steps_total):
        idx = torch.randint(0, F, (N,), dtype=torch.int32, device=dev, generator=gen)
        base = torch.arange(s * N, (s + 1) * N, device=dev, dtype=torch.float64)
        ts = (t0 + torch.floor(base * ms_per_event)).to(torch.int64)
        ev_b.append(device_events(idx, acq, ts))
        del idx, base, ts
    verdicts = torch.empty(N, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    ext = torch.cuda.ExternalStream(svc.stream, device=dev)
    for s in range(args.warmup):
        svc.submit_flow_batch(ev_b[s], verdicts=verdicts)
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
            svc.submit_flow_batch(ev_b[s], verdicts=verdicts)
        svc.synchronize()
        breakdown = read_profile()
        svc._L.sentinel_profile_enable(svc.handle, 0)
        dom = max(breakdown, key=lambda k: breakdown[k]["total_ms"])
        svc._L.sentinel_profile_select(svc.handle, dom.encode())
        svc._L.sentinel_profile_enable(svc.handle, 1)
    # batch boundaries: one event between consecutive batches (batch k = tev[k] -> tev[k + 1]);
    # the dominant kernel is bracketed by the engine's HIP events on every `kernel_every`-th timed
    # step (each event record idles the queue ~5 us)
    tev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for k in range(args.steps):
        s = args.warmup + pstep + k
        if not args.no_profile:
            svc._L.sentinel_profile_gate(svc.handle, 1 if k % args.kernel_every == 0 else 0)
        tev[k].record(ext)
        svc.submit_flow_batch(ev_b[s], verdicts=verdicts)
    tev[args.steps].record(ext)
    svc.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    lat = sorted(tev[k].elapsed_time(tev[k + 1]) for k in range(args.steps))
    p99 = lat[min(len(lat) - 1, int(np.ceil(0.99 * len(lat))) - 1)]

    # ---- the dominant kernel's live duration over the timed region (HIP events on the engine stream)
    prof = {}
    if not args.no_profile:
        prof = read_profile()
        svc._L.sentinel_profile_enable(svc.handle, 0)
        svc._L.sentinel_profile_select(svc.handle, None)

    # ---- snapshot + RCCL all-gather (config 3's ClusterMetric snapshot; off the decision path)
    t_snap = int(ev_b[-1][-1, 1].item()) + 1
    snap = torch.empty((F, 3), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ts0 = time.perf_counter()
    svc.snapshot_device(t_snap, snap)
    svc.synchronize()
    if world > 1:
        maxf = torch.tensor([F], device=dev)
        dist.all_reduce(maxf, op=dist.ReduceOp.MAX)
        pad = torch.zeros((int(maxf.item()), 3), dtype=torch.int64, device=dev)
        pad[:F] = snap
        gathered = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(gathered, pad)
        torch.cuda.synchronize()
    snap_ms = (time.perf_counter() - ts0) * 1000.0

    # PCIe-inclusive host paths (reported beside `value`, never as it): (i) synchronous 1M-event
    # batches from pinned host memory (H2D, decide, D2H) -> per-batch latency percentiles, the
    # north star's "host-fed 1M-event batches for the p99 number"; (ii) the streamed host path:
    # the step's N events in 1M-event batches pipelined over copy streams (double-buffered).
    host_path = None
    if rank == 0 and not args.no_host_path:
        import ctypes as C
        m = min(N, 1 << 20)
        hev = torch.empty((N, 2), dtype=torch.int64, pin_memory=True)
        hev.copy_(ev_b[-1])
        hout = torch.empty(N, dtype=torch.int64, pin_memory=True)
        reps = max(1, args.host_reps)
        nbs = (N + m - 1) // m
        bms = np.zeros(nbs, dtype=np.float32)
        # one untimed call of each leg: staging buffers and copy streams are created on first use
        assert svc._L.sentinel_submit_flow_batch_host(svc.handle, m, C.c_void_p(hev.data_ptr()), None,
                                                      C.c_void_p(hout.data_ptr())) == 0
        assert svc._L.sentinel_submit_flow_stream_host(svc.handle, N, C.c_void_p(hev.data_ptr()), None,
                                                       C.c_void_p(hout.data_ptr()), m, None) == 0
        hl = []
        for _ in range(reps):
            h0 = time.perf_counter()
            rc = svc._L.sentinel_submit_flow_batch_host(svc.handle, m, C.c_void_p(hev.data_ptr()), None,
                                                        C.c_void_p(hout.data_ptr()))
            assert rc == 0
            hl.append((time.perf_counter() - h0) * 1000.0)
        hl.sort()
        sreps = 3
        s0 = time.perf_counter()
        for _ in range(sreps):
            rc = svc._L.sentinel_submit_flow_stream_host(svc.handle, N, C.c_void_p(hev.data_ptr()), None,
                                                         C.c_void_p(hout.data_ptr()), m,
                                                         C.c_void_p(bms.ctypes.data))
            assert rc == 0
        sdt = (time.perf_counter() - s0) / sreps
        bl = np.sort(bms)
        host_path = {
            "sync": {"decisions_per_s": round(m * reps / (sum(hl) / 1000.0), 1), "batch": m, "reps": reps,
                     "median_ms": round(hl[len(hl) // 2], 3),
                     "p99_ms": round(hl[min(reps - 1, int(np.ceil(0.99 * reps)) - 1)], 3),
                     "note": "pinned host events -> H2D -> decide -> D2H, synchronous per batch, host clock"},
            "streamed": {"decisions_per_s": round(N / sdt, 1), "events": N, "batch": m,
                         "p99_batch_ms": round(float(bl[min(nbs - 1, int(np.ceil(0.99 * nbs)) - 1)]), 3),
                         "note": "sentinel_submit_flow_stream_host: H2D / decide / D2H of consecutive batches "
                                 "overlapped on side streams; batch latency = HIP events H2D start -> D2H end "
                                 "(includes queueing behind the previous batch)"},
        }
        del hev, hout

    total_events = float(N) * args.steps * world
    value = total_events / elapsed

    # ---- roofline of the dominant kernel
    roof = None
    if prof and dom in prof:
        d = prof[dom]
        bpe = KERNEL_BYTES_PER_EVENT.get(dom)
        if dom == "process":
            # per touched flow: read n epochs + n PASS, write epoch + 4 counters; per event: segment record
            e_f = N / max(1, F)
            bpe = (args.sample_count * 16 + 40 + 24) / max(1.0, min(e_f, 1e9)) if F else 0.0
        if dom == "part_fused":
            # per event: read the 8-B packed value (local key inside), write the 8-B verdict; per
            # touched flow: read the window header (16 B per bucket) and the 42 B of rule fields,
            # write back the rolled bucket's 16-B pair, read + write its BLOCK / PASS_REQUEST /
            # BLOCK_REQUEST counters (3 x 8 B each way, blocked counter rows)
            e_f = N / max(1, F)
            bpe = 16.0 + (args.sample_count * 16 + 42 + 16 + 48) / max(1.0, e_f)
        if dom == "radix_scatter":
            passes = max(1, round(d["calls"] / max(1, args.steps)))
            bpe = (32.0 + 24.0 * (passes - 1)) / passes
        ach = (bpe or 0.0) * d["units_per_call"] / (d["avg_us"] * 1e-6) / 1e9
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(dom),
                "traffic_unit": "bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_latest.json)",
                "algorithmic_bytes_per_launch": round((bpe or 0.0) * d["units_per_call"], 1),
                "bytes_per_event": bpe, "avg_us": round(d["avg_us"], 2)}

    # ---- CPU baseline: the oracle ("port") on bounded samples of the same workload, rank 0, N=1.
    # cpu_baseline = the flow-sharded multi-threaded replay on the box's CPU share (16 threads per
    # GPU); cpu_baseline_1core = the sequential replay (what one reference JVM thread does per call).
    cpu = cpu1 = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O

        def host_steps(k):
            e = torch.cat([ev_b[s] for s in range(min(k, steps_total))]).cpu().numpy()
            return (e[:, 0] & 0xFFFFFFFF).astype(np.int32), e[:, 1].copy()

        def fresh():
            return O.TokenServiceOracle.from_arrays(shard.flow_id, shard.count, shard.threshold_type,
                                                    shard.sample_count, shard.window_interval_ms,
                                                    shard.namespace, shard.checker)
        idx_c, ts_c = host_steps(args.cpu_steps_1core)
        m = len(ts_c)
        orc = fresh()
        c0 = time.perf_counter()
        orc.replay(idx_c, np.ones(m, np.int32), ts_c)
        cdt = time.perf_counter() - c0
        cpu1 = {"value": round(m / cdt, 1), "unit": "decisions/s", "cores": 1, "kind": "port",
                "sample": f"steps 0..{min(args.cpu_steps_1core, steps_total) - 1} of this workload ({m} events, same rules and trace), "
                          f"sequential oracle replay, {cdt:.1f} s"}
        del idx_c, ts_c
        idx_c, ts_c = host_steps(args.cpu_steps_mt)
        m = len(ts_c)
        orc = fresh()
        c0 = time.perf_counter()
        used = orc.replay_mt(idx_c, np.ones(m, np.int32), ts_c, args.cpu_threads)[3]
        cdt = time.perf_counter() - c0
        cpu = {"value": round(m / cdt, 1), "unit": "decisions/s", "cores": int(used), "kind": "port",
               "sample": f"steps 0..{min(args.cpu_steps_mt, steps_total) - 1} of this workload ({m} events, same rules and trace), "
                         f"oracle replay sharded by flow over {used} pthreads, {cdt:.1f} s wall"}
        del idx_c, ts_c

    pipeline_bytes = 21.0 + (args.sample_count * 64 + 64 + 16) / max(1.0, N / max(1, F))
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
        "data": "synthetic (seeded uniform events over the shard's flows; random-init rule table)",
        "config": {"workload": "config3: 1M flowIds hash-sharded (splitmix64 mod N), cluster GLOBAL rules "
                               "count~U{10..1000}, n=10 w=100ms, uniform flows, acquire=1, 2x offered load",
                   "flows_total": args.flows, "flows_this_rank": F, "events_per_gpu_per_step": N,
                   "parallelism": f"flowid-shard x{world}"},
        "p99_batch_ms": round(p99, 4),
        "median_batch_ms": round(lat[len(lat) // 2], 4),
        "snapshot_allgather_ms": round(snap_ms, 3),
        "host_path": host_path,
        "pipeline_bytes_per_decision": round(pipeline_bytes, 2),
        "pipeline_hbm_frac": round(value / world * pipeline_bytes / (HBM_PEAK_GBS * 1e9), 4),
        "roofline": roof,
        "cpu_baseline": cpu,
        "cpu_baseline_1core": cpu1,
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
