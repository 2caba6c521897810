// partition.hpp -- the partition-local flow path (gfx950): one scatter pass + one fused
// decide pass, instead of a full 3-pass radix sort followed by segment / process / verdict kernels.
//
// A flow's events only interact with each other (ClusterFlowChecker reads and writes one flow's
// ClusterMetric), so the batch only needs to be grouped by flow, in arrival order, not globally
// sorted.  The flow index space is cut into P <= 1024 contiguous ranges of 2^lb flows:
//
//   k_part_prep     validation + routing (as k_flow_prep) and per-tile histograms of the range
//                   digit d = flow >> lb (invalid events are decided here and leave the pipeline)
//   scan            exclusive scan of the digit-major histograms -> every tile's output offsets
//   k_part_scatter  stable multi-split of the events into their ranges (one pass, LDS-staged
//                   contiguous runs); writes the 16-bit local flow key and the 64-bit sorted value
//   k_part_half     one workgroup per half range (512 flows): the half's events counted and placed
//                   in LDS in (flow, arrival) order, then one lane per flow decides its run
//                   (window header in VGPRs, closed-form epoch segments, sequential fallback) and
//                   writes the verdicts straight to their arrival positions
//   k_part_big      the same for halves too large for LDS, sorted through HBM
//   k_part_long     runs longer than LONG_RUN: a workgroup per hot flow
//
// Order inside a half after placement = (local flow, arrival) = the order the 3-pass radix sort
// produces, in 1 scatter pass + 1 in-LDS pass.  A hot flow makes one lane long (it walks its
// events), which is why the engine uses this path for large flow tables (engine.hip, flow_path).
#pragma once

#include "admission.hpp"

namespace sentinel {

constexpr int PART_MAX_BITS = 10;                  // <= 1024 ranges, <= 1024 flows per range
constexpr int PART_BINS = 1 << PART_MAX_BITS;

// Partition tile (k_part_prep histogram rows and k_part_scatter blocks): PT_TILE events.
#ifndef SENTINEL_PT_THREADS
#define SENTINEL_PT_THREADS 512
#endif
#ifndef SENTINEL_PT_ITEMS
#define SENTINEL_PT_ITEMS 8
#endif
constexpr int PT_THREADS = SENTINEL_PT_THREADS;
constexpr int PT_WAVES = PT_THREADS / WAVE;
constexpr int PT_ITEMS = SENTINEL_PT_ITEMS;
constexpr int PT_TILE = PT_THREADS * PT_ITEMS;
static_assert(PT_THREADS >= 256 && PT_THREADS <= PART_BINS && PT_TILE <= 65535, "partition tile");
// the partition histograms (part_blocks(n) x PART_BINS words) live in the radix path's histogram buffer,
// sized for sort_blocks(n) x RADIX x MAX_PASSES words: a tile smaller than SORT_TILE would overrun it
// (a PT_ITEMS=4 build faulted)
static_assert(PT_TILE >= SORT_TILE && PART_BINS <= RADIX * MAX_PASSES, "partition histograms fit the radix buffer");
inline int64_t part_blocks(int64_t n) { return (n + PT_TILE - 1) / PT_TILE; }

// Validation + routing as k_flow_prep; histogram of the range digit of valid events only.
#ifndef SENTINEL_PREP_THREADS
#define SENTINEL_PREP_THREADS 1024    // 4 events per thread: measured 38 us vs 40 (512) and 47 (256)
#endif
constexpr int PP_THREADS = SENTINEL_PREP_THREADS;
constexpr int PP_ITEMS = PT_TILE / PP_THREADS;
__global__ __launch_bounds__(PP_THREADS) void k_part_prep(int64_t n, const Event *__restrict__ ev, int32_t nflows,
                                                            const int32_t *__restrict__ route,
                                                            uint64_t *__restrict__ out, uint32_t *__restrict__ fkey,
                                                            uint32_t finvalid, int lb, uint32_t *__restrict__ hist,
                                                            int64_t nblocks, int32_t nparts,
                                                            uint32_t *__restrict__ ctl_zero,
                                                            unsigned long long *__restrict__ stat_zero,
                                                            const uint32_t *__restrict__ keys_pre,
                                                            uint32_t *__restrict__ oseq = nullptr,
                                                            uint32_t *__restrict__ octr = nullptr, uint32_t opar = 0) {
    // oseq (decide-order output): a rejected event's verdict goes to position n - 1 - (its rank among the
    // batch's rejected events, counted in octr[opar]) -- the valid events fill [0, valid) in the ranges, so
    // the rejected ones fill [valid, n) -- with its arrival position in oseq; octr[opar ^ 1] is zeroed for
    // the next such batch (opar alternates per batch: no memset launch)
    if (blockIdx.x == 0 && threadIdx.x == 0) {        // the batch's work-list counters and skew statistic
        if (ctl_zero) { ctl_zero[0] = 0; ctl_zero[1] = 0; ctl_zero[2] = 0; }
        if (stat_zero) *stat_zero = 0;
        if (octr) octr[opar ^ 1u] = 0;
    }
    __shared__ uint32_t h[PART_BINS];
    const int64_t tile0 = (int64_t)blockIdx.x * PT_TILE;
    Event evs[PP_ITEMS];                            // every event load of the tile in flight at once
#pragma unroll
    for (int j = 0; j < PP_ITEMS; ++j) {
        const int64_t i = tile0 + j * PP_THREADS + threadIdx.x;
        if (i < n) evs[j] = ev[i];
    }
    for (int d = threadIdx.x; d < PART_BINS; d += PP_THREADS) h[d] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PP_ITEMS; ++j) {
        const int64_t i = tile0 + j * PP_THREADS + threadIdx.x;
        if (i >= n) break;
        const Event e = evs[j];
        int st = 127;
        uint32_t k = finvalid;
        if (keys_pre) {       // validated (and limited: GlobalRequestLimiter) upstream, verdicts written there
            k = keys_pre[i];
            if (k != finvalid) atomicAdd(&h[k >> lb], 1u);
            continue;
        }
        if (e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0) st = ST_BAD_REQUEST;      // DTS:38-40
        else if (e.idx < 0 || e.idx >= nflows) st = ST_NO_RULE_EXISTS;               // DTS:42-45
        else if (route && route[e.idx] == ROUTE_TOO_MANY) st = ST_TOO_MANY_REQUEST;  // namespace == null (CFC:50-53)
        else if (e.ts < 0) st = ST_FAIL;                                              // reference: NPE in LeapArray
        else k = (uint32_t)e.idx;
        if (fkey) fkey[i] = k;
        if (st == 127) atomicAdd(&h[k >> lb], 1u);
        else if (!oseq) put_verdict(out, (uint32_t)i, st, 0, 0);
        if (oseq) put_rejected_ordered(st != 127, out, oseq, &octr[opar], n, (uint32_t)i, st);
    }
    __syncthreads();
    // tile-major: this tile's 4 KB row is one contiguous store
    for (int d = threadIdx.x; d < nparts; d += PP_THREADS) hist[(int64_t)blockIdx.x * nparts + d] = h[d];
}

// Offsets of the multi-split from the tile-major histograms h[b][d] (b = tile, d = range):
// off[b][d] = start(d) + sum_{b' < b} h[b'][d], start(d) = sum_{d' < d} total(d').  Three small
// passes over groups of PS_GROUP tiles, every access a coalesced row: column sums per group,
// one workgroup scanning groups and ranges, then the running offsets written in place.
constexpr int PS_GROUP = 32;
constexpr int PS_THREADS = 256;

__global__ __launch_bounds__(PS_THREADS) void k_part_colsum(const uint32_t *__restrict__ hist, int64_t nb, int32_t P,
                                                            uint32_t *__restrict__ gsum) {
    const int64_t g = blockIdx.x;
    const int d = blockIdx.y * PS_THREADS + threadIdx.x;
    if (d >= P) return;
    const int64_t b0 = g * PS_GROUP, b1 = min(b0 + PS_GROUP, nb);
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < PS_GROUP; ++k) s += b0 + k < b1 ? hist[(b0 + k) * P + d] : 0u;
    gsum[g * P + d] = s;
}

// One wave per range: exclusive scan of the range's group sums (in place, 64 groups per step, one
// load per lane) and the range total -> tot[d].  Every CU takes a few ranges (the previous single
// 1024-thread workgroup left 255 CUs idle for 8 us).
constexpr int PC_THREADS = 256;
__global__ __launch_bounds__(PC_THREADS) void k_part_colscan(uint32_t *__restrict__ gsum, int64_t ng, int32_t P,
                                                             uint32_t *__restrict__ tot) {
    const int d = blockIdx.x * (PC_THREADS / WAVE) + threadIdx.x / WAVE;
    if (d >= P) return;                                   // wave-uniform
    const uint32_t lane = lane_id();
    uint32_t carry = 0;
    for (int64_t g0 = 0; g0 < ng; g0 += WAVE) {
        const int64_t g = g0 + lane;
        const uint32_t x = g < ng ? gsum[g * P + d] : 0u;
        const uint32_t inc = wave_inclusive_scan(x);
        if (g < ng) gsum[g * P + d] = carry + inc - x;
        carry += __shfl(inc, WAVE - 1, WAVE);
    }
    if (lane == 0) tot[d] = carry;
}

// Range starts: rstart[d] = sum of tot[d'] for d' < d, rstart[P] = valid events.  Computed by every
// k_part_offsets workgroup for its own 256 ranges (the totals are 4 KB, read from L2).
__device__ inline uint32_t part_range_start(const uint32_t *__restrict__ tot, int32_t P, int d0, int d,
                                            uint32_t *lds_waves, uint32_t *grand) {
    uint32_t before = 0;                                  // this lane's share of tot[0, d0)
    for (int k = threadIdx.x; k < d0; k += PS_THREADS) before += tot[k];
    uint32_t b_total;
    (void)block_exclusive_scan(before, lds_waves, &b_total);
    uint32_t chunk_total;
    const uint32_t ex = block_exclusive_scan(d < P ? tot[d] : 0u, lds_waves, &chunk_total);
    *grand = b_total + chunk_total;
    return b_total + ex;
}

__global__ __launch_bounds__(PS_THREADS) void k_part_offsets(uint32_t *__restrict__ hist, int64_t nb, int32_t P,
                                                             const uint32_t *__restrict__ gsum,
                                                             const uint32_t *__restrict__ tot,
                                                             uint32_t *__restrict__ rstart) {
    __shared__ uint32_t waves_tot[PS_THREADS / WAVE];
    const int64_t g = blockIdx.x;
    const int d0 = blockIdx.y * PS_THREADS;
    const int d = d0 + threadIdx.x;
    uint32_t grand;
    const uint32_t rs = part_range_start(tot, P, d0, d, waves_tot, &grand);
    if (d >= P) return;
    if (g == 0) {
        rstart[d] = rs;
        if (d == P - 1) rstart[P] = grand;
    }
    const int64_t b0 = g * PS_GROUP, b1 = min(b0 + PS_GROUP, nb);
    uint32_t run = rs + gsum[g * P + d];
    uint32_t x[PS_GROUP];                                 // the group's column in flight at once
#pragma unroll
    for (int k = 0; k < PS_GROUP; ++k) x[k] = b0 + k < b1 ? hist[(b0 + k) * P + d] : 0u;
#pragma unroll
    for (int k = 0; k < PS_GROUP; ++k) {
        if (b0 + k < b1) hist[(b0 + k) * P + d] = run;
        run += x[k];
    }
}

// Stable multi-split of the valid events by range digit (one pass).  Same tiling as k_part_prep;
// ranking with one 64-bit ballot per digit bit and wave-private LDS counters; the tile is staged
// in LDS in digit order and written out as contiguous per-range runs.  keys_in == null (no
// namespace routes, the common case): the flow key and validity are re-derived from the event the
// value is packed from anyway, so k_part_prep writes no key array and nothing reads one.
__global__ __launch_bounds__(PT_THREADS) void k_part_scatter(const uint32_t *__restrict__ keys_in, EventSrc src,
                                                               uint64_t *__restrict__ vals_out, int64_t n,
                                                               uint32_t finvalid, int lb, int pbits,
                                                               const uint32_t *__restrict__ offsets, int64_t nblocks,
                                                               int32_t nparts, int32_t nflows) {
    __shared__ uint16_t cnt[PT_WAVES][PART_BINS];
    __shared__ uint32_t goff[PART_BINS];
    __shared__ uint32_t loff[PART_BINS];
    __shared__ uint32_t waves_tot[PT_WAVES];
    __shared__ uint16_t sdig[PT_TILE];
    __shared__ uint64_t svals[PT_TILE];
    const int wave = threadIdx.x / WAVE;
    const uint32_t lane = lane_id();
    for (int d = threadIdx.x; d < PART_BINS; d += PT_THREADS) {
#pragma unroll
        for (int w = 0; w < PT_WAVES; ++w) cnt[w][d] = 0;
        goff[d] = d < nparts ? offsets[(int64_t)blockIdx.x * nparts + d] : 0u;   // tile-major row
    }
    __syncthreads();
    const int64_t tile0 = (int64_t)blockIdx.x * PT_TILE;
    const int64_t base = tile0 + (int64_t)wave * (PT_ITEMS * WAVE);
    const int64_t T0 = src.t0();
    uint32_t key[PT_ITEMS], rank[PT_ITEMS];
    uint64_t pk[PT_ITEMS];                       // packed values (keys_in == null: from the events loaded here)
    if (keys_in) {
#pragma unroll
        for (int j = 0; j < PT_ITEMS; ++j) {
            const int64_t i = base + j * WAVE + lane;
            key[j] = i < n ? keys_in[i] : finvalid;
        }
    } else {
        Event evs[PT_ITEMS];
        uint8_t fls[PT_ITEMS];
#pragma unroll
        for (int j = 0; j < PT_ITEMS; ++j) {
            const int64_t i = base + j * WAVE + lane;
            if (i < n) { evs[j] = src.ev[i]; fls[j] = src.flags ? src.flags[i] : 0; }
        }
#pragma unroll
        for (int j = 0; j < PT_ITEMS; ++j) {
            const int64_t i = base + j * WAVE + lane;
            const Event e = evs[j];
            // k_part_prep's validation without the route check (keys_in is only null without routes)
            const bool ok = i < n && e.idx != SENTINEL_IDX_BAD_ID && e.acquire > 0 && e.idx >= 0 && e.idx < nflows &&
                            e.ts >= 0;
            key[j] = ok ? (uint32_t)e.idx : finvalid;
            pk[j] = ok ? src.pack_event((uint32_t)i, e, fls[j], T0) : 0ull;
        }
    }
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j) {
        const bool valid = key[j] != finvalid;
        const uint32_t d = valid ? key[j] >> lb : 0u;
        const uint64_t peers = match_peers<PART_MAX_BITS>(d, valid, pbits);
        uint32_t r = 0;
        if (valid) r = cnt[wave][d] + mask_rank(peers);
        __builtin_amdgcn_wave_barrier();
        if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane) cnt[wave][d] += (uint16_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        rank[j] = valid ? r : 0xFFFFFFFFu;
    }
    __syncthreads();
    // per digit: exclusive over waves (in place), then an exclusive scan over digits -> loff
    constexpr int DPT = PART_BINS / PT_THREADS;   // digits per thread
    uint32_t dtot[DPT > 0 ? DPT : 1];
    uint32_t mine = 0;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
        const int d = threadIdx.x * DPT + q;
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < PT_WAVES; ++w) {
            const uint32_t c = cnt[w][d];
            cnt[w][d] = (uint16_t)run;
            run += c;
        }
        dtot[q] = run;
        mine += run;
    }
    uint32_t total;
    uint32_t pre = block_exclusive_scan(mine, waves_tot, &total);
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
        loff[threadIdx.x * DPT + q] = pre;
        pre += dtot[q];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j) {
        if (rank[j] == 0xFFFFFFFFu) continue;
        const uint32_t d = key[j] >> lb;
        const uint32_t p = loff[d] + cnt[wave][d] + rank[j];
        sdig[p] = (uint16_t)d;
        svals[p] = (keys_in ? src.pack((uint32_t)(base + j * WAVE + lane), T0) : pk[j]) |
                   ((uint64_t)(key[j] & ((1u << lb) - 1)) << VAL_KEY_SHIFT);
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < total; p += PT_THREADS) {
        const uint32_t d = sdig[p];
        const uint32_t dst = goff[d] + p - loff[d];
        if (dst >= (uint64_t)n) continue;          // guard: a corrupt offset must never write out of bounds
        vals_out[dst] = svals[p];
    }
}

// A flow's window header {epoch, PASS} x n held in VGPRs while its events are decided in arrival
// order (the k_process_reg scheme): closed-form homogeneous segments, the reference state machine
// (seq_event on global memory) for everything else, only dirty pairs written back.
// Verdict of the k-th event of a closed-form segment (ClusterFlowChecker.java:72-82): the first K
// pass with remaining = (int)((G - (S0 + k*a) / I_s) - a), the rest are BLOCKED.  `small`: every
// S0 + k*a of the segment fits in int32, so the int64 -> double conversion is one v_cvt_f64_i32.
__device__ inline uint64_t run_verdict(double thr, double I_s, int64_t s0, int32_t a, uint32_t K, uint32_t k, bool small) {
    if (k >= K) return pack_verdict(ST_BLOCKED, 0, 0);
    const double x = small ? (double)((int32_t)s0 + (int32_t)k * a) : (double)wrap_add(s0, wrap_mul((int64_t)k, a));
    return pack_verdict(ST_OK, java_d2i((thr - div_interval(x, I_s)) - (double)a), 0);
}

#ifdef SENTINEL_DIAG_PHASES     // cost diagnostic: wall-clock stamps per workgroup and phase
__device__ unsigned long long g_phase[4096][12];
#define PF_STAMP(i) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_phase[blockIdx.x][i] = wall_clock64(); } while (0)
#define PF_COUNT(i) do { if (blockIdx.x < 4096) atomicAdd(&g_phase[blockIdx.x][i], 1ull); } while (0)
#else
#define PF_STAMP(i) do { } while (0)
#define PF_COUNT(i) do { } while (0)
#endif

template <int NMAX>
struct FlowWindow {
    KeyState ks;
    int nsc;
    uint8_t kind;
    double thr, I_s, rcp;
    int32_t w;
    int64_t ep[NMAX], ps[NMAX];
    uint32_t dirty;
    bool occ_pending;
    uint8_t occ_raw;         // T.has_occ[key] as loaded (compared only where used: no early wait)
    // batch clock: epoch of T0 and T0 mod w, so an event's epoch is E0 + floor((r0 + dt) / w) in
    // 32-bit arithmetic (dt = ts - T0 from the packed value, |dt| < 2^23)
    int64_t E0;
    int32_t r0;
    float rcpf;

    // the rule part: independent loads only (may be issued long before the header is needed)
    __device__ inline void load_rule(const KeyTable &T, uint32_t key) {
        ks = key_state(T, key);
        nsc = ks.n;
        kind = T.kind[key];
        thr = T.thr[key];
        I_s = T.I_s[key];
        w = T.w[key];
        rcp = T.rcp_w[key];
        occ_raw = T.has_occ[key];
    }

    __device__ inline void load_header(int64_t T0) {
        occ_pending = occ_raw != 0 && ks.seven && kind == KIND_CLUSTER;
        dirty = 0;
        if (ks.hs != 2) {
            // blocked header region with NMAX slots per block: every pair load is in bounds, so
            // they are all issued without waiting for n
#pragma unroll
            for (int j = 0; j < NMAX; ++j) {
                const longlong2 v = *reinterpret_cast<const longlong2 *>(ks.pair(j));
                ep[j] = j < nsc ? v.x : EPOCH_ABSENT;
                ps[j] = j < nsc ? v.y : 0;
            }
        } else {
#pragma unroll
            for (int j = 0; j < NMAX; ++j) {
                if (j < nsc) {
                    const longlong2 v = *reinterpret_cast<const longlong2 *>(ks.pair(j));
                    ep[j] = v.x;
                    ps[j] = v.y;
                } else {
                    ep[j] = EPOCH_ABSENT;
                    ps[j] = 0;
                }
            }
        }
        E0 = epoch_of(T0, w, rcp);
        r0 = (int32_t)(T0 - E0 * (int64_t)w);
        rcpf = 1.0f / (float)w;
    }

    __device__ inline void load(const KeyTable &T, uint32_t key, int64_t T0) {
        load_rule(T, key);
        load_header(T0);
    }

    // Epoch, acquire and prioritized flag of a packed value.  Exact: q is within one of
    // floor(x / w) (x < 2^24 is exact in float, the product is off by at most one ulp) and the
    // remainder test fixes it; escaped values take the 64-bit path.
    __device__ inline int64_t event(uint64_t v, const EventSrc &src, int64_t T0, int32_t &a, bool &prio) const {
        const uint32_t dtf = (uint32_t)(v >> VAL_DT_SHIFT) & VAL_DT_ESC;
        const uint32_t af = (uint32_t)(v >> VAL_ACQ_SHIFT) & VAL_ACQ_ESC;
        prio = (v & VAL_PRIO) != 0;
        if (dtf == VAL_DT_ESC || af == VAL_ACQ_ESC || w >= (1 << 30)) {
            int64_t t;
            src.unpack(v, T0, t, a, prio);
            return epoch_of(t, w, rcp);
        }
        a = src.unit_acquire ? 1 : (int32_t)af;
        const int32_t x = r0 + val_dt(dtf);
        int32_t q = (int32_t)floorf((float)x * rcpf);
        const int32_t rem = x - q * w;
        if (rem < 0) --q;
        else if (rem >= w) ++q;
        return E0 + q;
    }

    __device__ inline void flush() {
#ifdef SENTINEL_DIAG_NOFLUSH    // cost diagnostic only (wrong state)
        return;
#endif
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (dirty & (1u << j)) *reinterpret_cast<longlong2 *>(ks.pair(j)) = longlong2{ep[j], ps[j]};
        dirty = 0;
    }

    // a segment at epoch E needs the sequential path (heterogeneous / prioritized, pending occupy
    // transfer, or a slot newer than E: the clock went backwards for this flow)
    __device__ inline bool slow(int64_t E, bool het) const {
        bool s = het || occ_pending;
#pragma unroll
        for (int j = 0; j < NMAX; ++j) s |= (ep[j] != EPOCH_ABSENT && ep[j] > E);
#ifdef SENTINEL_DIAG_PHASES
        if (het) PF_COUNT(8);
        if (occ_pending) PF_COUNT(9);
        if (s && !het && !occ_pending) {
            PF_COUNT(10);
            if (atomicAdd(&g_phase[4095][11], 1ull) < 6) {
                printf("newer: blk %u thr %u E %lld nsc %d w %d E0 %lld r0 %d ep:", blockIdx.x, threadIdx.x, (long long)E, nsc,
                       w, (long long)E0, r0);
                for (int j = 0; j < NMAX; ++j) printf(" %lld", (long long)ep[j]);
                printf("\n");
            }
        }
#endif
        return s;
    }

    // the sequential path over sorted positions [q, q2) of `vals`
    __device__ inline void sequential(const KeyTable &T, uint32_t key, int64_t E, const uint64_t *vals, uint32_t q,
                                      uint32_t q2, const EventSrc &src, const Verdicts &V) {
        PF_COUNT(6);
        flush();
        for (uint32_t i = q; i < q2; ++i) {
            const uint32_t seq = (uint32_t)vals[i] & SEQ_MASK;
            int64_t tt;
            int32_t aa;
            uint8_t fl;
            src.load(seq, tt, aa, fl);
            seq_event(T, key, ks, E, aa, fl, seq, V, V.at(i, vals[i]));
        }
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (j < nsc) { ep[j] = ks.ep(j); ps[j] = ks.cnt(EV_PASS, j); }
        occ_pending = ks.seven && kind == KIND_CLUSTER && T.has_occ[key];
    }

    // closed form for a homogeneous segment of `len` events with acquire a: roll, S0, K, counters
    __device__ inline void fast(int64_t E, int32_t a, uint32_t len, int64_t &s0, uint32_t &K) {
        const int slot = (int)(E % nsc);
        bool fresh = false;
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (j == slot && ep[j] != E) { fresh = true; ep[j] = E; ps[j] = 0; }
        s0 = 0;
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (ep[j] != EPOCH_ABSENT && ep[j] > E - nsc) s0 = wrap_add(s0, ps[j]);
        uint32_t lo = 0, hi = len;                      // K = first p with !admits(S0 + p*a)
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (admits(kind, thr, I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) lo = mid + 1;
            else hi = mid;
        }
        K = lo;
        const int64_t nb = (int64_t)(len - K);
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (j == slot) { ps[j] = wrap_add(ps[j], wrap_mul((int64_t)K, a)); dirty |= 1u << j; }
#ifdef SENTINEL_DIAG_NOREST     // cost diagnostic only (wrong counters)
        if (false) {
#else
        if (ks.seven) {
#endif
            int64_t blk = 0, preq = 0, breq = 0;
            if (!fresh) { blk = ks.rc(slot, 0); preq = ks.rc(slot, 1); breq = ks.rc(slot, 2); }
            ks.book_rest(slot, fresh, blk, preq, breq, nb, a, K);
        }
    }

    // heterogeneous-acquire segment at E (not prioritized, nothing pending, no newer slot): roll the
    // slot, return the window's PASS sum; het_book adds the segment's sums afterwards
    __device__ inline int64_t het_begin(int64_t E, bool &fresh) {
        const int slot = (int)(E % nsc);
        fresh = false;
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (j == slot && ep[j] != E) { fresh = true; ep[j] = E; ps[j] = 0; }
        int64_t s0 = 0;
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (ep[j] != EPOCH_ABSENT && ep[j] > E - nsc) s0 = wrap_add(s0, ps[j]);
        return s0;
    }

    __device__ inline void het_book(int64_t E, bool fresh, const HetSums &h) {
        const int slot = (int)(E % nsc);
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (j == slot) { ps[j] = wrap_add(ps[j], h.pass); dirty |= 1u << j; }
        if (ks.seven) {
            int64_t blk = 0, preq = 0, breq = 0;
            if (!fresh) { blk = ks.rc(slot, 0); preq = ks.rc(slot, 1); breq = ks.rc(slot, 2); }
            ks.book_rest_sums(slot, fresh, blk, preq, breq, h.block, h.npass, h.nblock);
        }
    }

    // after deciding events at epoch E: nothing more can pass at E (not even an acquire of 1) -- the
    // slot of E is rolled, no slot is newer, no occupy transfer is pending
    __device__ inline bool dead_at(int64_t E) const {
        if (occ_pending) return false;
        const int slot = (int)(E % nsc);
        bool rolled = false, newer = false;
        int64_t sum = 0;
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
            if (ep[j] == EPOCH_ABSENT) continue;
            newer |= ep[j] > E;
            if (ep[j] > E - nsc) sum = wrap_add(sum, ps[j]);
            if (j == slot) rolled = ep[j] == E;
        }
        return rolled && !newer && !admits(kind, thr, I_s, sum, 1);
    }

    // the whole heterogeneous segment [q, q2) by this lane (het_walk on the rolled window)
    __device__ inline void hetero(int64_t E, const uint64_t *vals, uint32_t q, uint32_t q2, const EventSrc &src,
                                  const Verdicts &V, int64_t T0) {
        PF_COUNT(7);
        bool fresh;
        const int64_t s0 = het_begin(E, fresh);
        const HetSums h = het_walk<2>(          // (few registers: this runs inside the lane walkers)
            kind, thr, I_s, s0, q2 - q, [&](uint32_t k) { return vals[q + k]; },
            [&](uint64_t v) {
                int32_t a;
                bool pr;
                (void)event(v, src, T0, a, pr);
                return a;
            },
            [&](uint32_t k, uint64_t v, uint64_t vd) { V.put(q + k, v, vd); });
        het_book(E, fresh, h);
    }

    // `small`: every S0 + k*a of the segment fits in int32, so the int64 -> double conversion is one
    // v_cvt_f64_i32 (same value)
    __device__ inline uint64_t verdict(int64_t s0, int32_t a, uint32_t K, uint32_t k, bool small) const {
        return run_verdict(thr, I_s, s0, a, K, k, small);
    }
};

// One flow's run of sorted events [q0, q1) (arrival order), decided by one lane; verdicts written
// to the arrival positions.
template <int NMAX>
__device__ inline void part_run_w(FlowWindow<NMAX> &fw, const KeyTable &T, uint32_t key, const uint64_t *s_val,
                                  uint32_t q0, uint32_t q1, const EventSrc &src, const Verdicts &V, int64_t T0) {
    uint32_t q = q0;
    while (q < q1) {
        int32_t a;
        bool prio;
        const int64_t E = fw.event(s_val[q], src, T0, a, prio);
        bool pr = prio && fw.kind == KIND_CLUSTER, ah = false;
        uint32_t q2 = q + 1;
        for (; q2 < q1; ++q2) {                       // the segment: same epoch
            int32_t a2;
            bool p2;
            if (fw.event(s_val[q2], src, T0, a2, p2) != E) break;
            ah |= a2 != a;
            pr |= p2 && fw.kind == KIND_CLUSTER;
        }
        if (fw.slow(E, pr)) {
            fw.sequential(T, key, E, s_val, q, q2, src, V);
        } else if (ah) {
            fw.hetero(E, s_val, q, q2, src, V, T0);
        } else {
            int64_t s0;
            uint32_t K;
            const uint32_t len = q2 - q;
            fw.fast(E, a, len, s0, K);
            const bool small = s0 >= 0 && s0 + (int64_t)len * a < (int64_t)INT32_MAX;
#ifdef SENTINEL_DIAG_VLINEAR   // cost diagnostic only (wrong output): one 64-byte line per flow
            for (uint32_t k = 0; k < len; ++k) V.out[key * 8 + (k & 7)] = fw.verdict(s0, a, K, k, small);
#else
#ifdef SENTINEL_DIAG_NOVERDICT  // cost diagnostic only (no output)
            {
                uint64_t acc = 0;
                for (uint32_t k = 0; k < len; ++k) acc ^= fw.verdict(s0, a, K, k, small) ^ s_val[q + k];
                if (acc == 0x123456789ull) V.out[0] = acc;
            }
#else
            for (uint32_t k = 0; k < len; ++k) V.put(q + k, s_val[q + k], fw.verdict(s0, a, K, k, small));
#endif
#endif
        }
        q = q2;
    }
    fw.flush();
}

// The common case of a run: every event of the flow in the batch falls in one epoch E with one
// acquire count and no prioritized cluster request (a flow sees ~8 events per batch over a few ms,
// windows are >= 100 ms).  Then the whole run is one closed-form segment (FlowWindow::fast), and the
// window header, folded as it arrives, is only needed as {PASS sum of the valid slots, the rolled
// slot's pair, "a slot is newer than E"}.  The rolled slot's rest line does not depend on the header,
// so its load is issued together with the header loads: one memory round trip instead of two.
// A run that crosses one window boundary -- epoch E, then E2 > E from position q0 + len1 on, each part
// with one acquire count: most flows of the ~1 batch in 10 whose time span holds a boundary at config 3
// -- is two closed-form segments from the same loads: after the first, every slot is at most E < E2, so
// the slot of E2 restarts (fresh, no rest line read) and its window sum is the header with the first
// segment's pair applied (part_run_w's fast(E) then fast(E2), same counters, same verdicts).
// Returns false, having written nothing, when the run needs the general walk (part_run_w).
// DEFER: the verdicts are not written here; the segments' {s0, K, a, small} come back to the caller in
// d_*[0] / d_*[1] with the first segment's length in *d_len1 (the run's length when it is one segment);
// k_part_half's cooperative verdict sweep writes them with every lane of the workgroup.
template <int NMAX, bool DEFER = false>
__device__ inline bool part_run_single(FlowWindow<NMAX> &fw, const uint64_t *s_val, uint32_t q0, uint32_t q1,
                                       const EventSrc &src, const Verdicts &V, int64_t T0, int64_t *d_s0 = nullptr,
                                       uint32_t *d_K = nullptr, int32_t *d_a = nullptr, bool *d_small = nullptr,
                                       uint32_t *d_len1 = nullptr) {
    if (fw.ks.hs == 2) return false;
    fw.E0 = epoch_of(T0, fw.w, fw.rcp);
    fw.r0 = (int32_t)(T0 - fw.E0 * (int64_t)fw.w);
    fw.rcpf = 1.0f / (float)fw.w;
    int32_t a;
    bool prio;
    const int64_t E = fw.event(s_val[q0], src, T0, a, prio);
    const bool cl = fw.kind == KIND_CLUSTER;
    bool ok = !(prio && cl) && !(fw.occ_raw != 0 && fw.ks.seven && cl);
    const uint32_t len = q1 - q0;
    uint32_t len1 = len;                                  // the first segment (epoch E)
    int64_t E2 = E;
    int32_t a2 = a;
    for (uint32_t q = q0 + 1; q < q1 && ok; ++q) {
        int32_t aq;
        bool pq;
        const int64_t Eq = fw.event(s_val[q], src, T0, aq, pq);
        ok = !(pq && cl);
        if (Eq == E2) {
            ok = ok && aq == a2;
        } else if (E2 == E && Eq > E) {                   // the boundary: the second segment starts
            E2 = Eq;
            a2 = aq;
            len1 = q - q0;
        } else {
            ok = false;                                   // a third epoch, or the clock went back
        }
    }
    if (!ok) return false;
    const bool two = len1 < len;
    const int nsc = fw.nsc;
    const int slot = (int)(E % nsc);
    // header pairs (every slot of the block: in bounds) and the rolled slot's rest line, in flight together
    longlong2 hp[NMAX];
#ifdef SENTINEL_DIAG_HDR1       // cost diagnostic only (wrong sums): the rolled slot's pair alone
#pragma unroll
    for (int j = 0; j < NMAX; ++j) hp[j] = longlong2{EPOCH_ABSENT, 0};
    hp[0] = *reinterpret_cast<const longlong2 *>(fw.ks.pair(slot));
#else
#pragma unroll
    for (int j = 0; j < NMAX; ++j) hp[j] = *reinterpret_cast<const longlong2 *>(fw.ks.pair(j));
#endif
#ifdef SENTINEL_DIAG_NOREST     // cost diagnostic only (wrong counters)
    const bool seven = false;
#else
    const bool seven = fw.ks.seven;
#endif
    int64_t blk = 0, preq = 0, breq = 0;
    if (seven) { blk = fw.ks.rc(slot, 0); preq = fw.ks.rc(slot, 1); breq = fw.ks.rc(slot, 2); }
    int64_t s_other = 0, ep_s = EPOCH_ABSENT, ps_s = 0;
    bool newer = false;
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
        if (j >= nsc) continue;
        const int64_t e = hp[j].x;
        if (j == slot) { ep_s = e; ps_s = hp[j].y; }
        else if (e != EPOCH_ABSENT && e > E - nsc) s_other = wrap_add(s_other, hp[j].y);
        newer |= e != EPOCH_ABSENT && e > E;
    }
    if (newer) return false;                              // clock went backwards: detached windows
    const bool fresh = ep_s != E;
    const int64_t base = fresh ? 0 : ps_s;
    const int64_t s0 = wrap_add(s_other, base);
    uint32_t lo = 0, hi = len1;                           // K = first p with !admits(S0 + p*a)
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (admits(fw.kind, fw.thr, fw.I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) lo = mid + 1;
        else hi = mid;
    }
    const uint32_t K = lo;
    const int64_t nb = (int64_t)(len1 - K);
    const int64_t p1 = wrap_add(base, wrap_mul((int64_t)K, a));   // the slot of E after the first segment
    const bool small = s0 >= 0 && s0 + (int64_t)len1 * a < (int64_t)INT32_MAX;
    int64_t s2 = 0;
    uint32_t K2 = 0;
    bool small2 = false;
    if (two) {
        const int slot2 = (int)(E2 % nsc);
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
            if (j >= nsc || j == slot2) continue;         // (the slot of E2 restarts at 0)
            const int64_t e = j == slot ? E : hp[j].x;
            if (e != EPOCH_ABSENT && e > E2 - nsc) s2 = wrap_add(s2, j == slot ? p1 : hp[j].y);
        }
        const uint32_t len2 = len - len1;
        lo = 0;
        hi = len2;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (admits(fw.kind, fw.thr, fw.I_s, wrap_add(s2, wrap_mul((int64_t)mid, a2)), a2)) lo = mid + 1;
            else hi = mid;
        }
        K2 = lo;
        small2 = s2 >= 0 && s2 + (int64_t)len2 * a2 < (int64_t)INT32_MAX;
        if (slot2 != slot) *reinterpret_cast<longlong2 *>(fw.ks.pair(slot)) = longlong2{E, p1};
        *reinterpret_cast<longlong2 *>(fw.ks.pair(slot2)) = longlong2{E2, wrap_mul((int64_t)K2, a2)};
        if (seven) {
            if (slot2 != slot) fw.ks.book_rest(slot, fresh, blk, preq, breq, nb, a, K);
            fw.ks.book_rest(slot2, true, 0, 0, 0, (int64_t)(len2 - K2), a2, K2);
        }
    } else {
        *reinterpret_cast<longlong2 *>(fw.ks.pair(slot)) = longlong2{E, p1};
        if (seven) fw.ks.book_rest(slot, fresh, blk, preq, breq, nb, a, K);
    }
    if (DEFER) {
        d_s0[0] = s0;
        d_K[0] = K;
        d_a[0] = a;
        d_small[0] = small;
        if (two) {
            d_s0[1] = s2;
            d_K[1] = K2;
            d_a[1] = a2;
            d_small[1] = small2;
        }
        *d_len1 = len1;
        return true;
    }
#if defined(SENTINEL_DIAG_NOVERDICT)     // cost diagnostic only (no output)
    uint64_t acc = 0;
    for (uint32_t k = 0; k < len; ++k) acc ^= fw.verdict(s0, a, K, k, small) ^ s_val[q0 + k];
    if (acc == 0x123456789ull) V.out[0] = acc;
#elif defined(SENTINEL_DIAG_VLINEAR)     // cost diagnostic only (wrong output): flow-contiguous stores
    for (uint32_t k = 0; k < len; ++k) V.out[(blockIdx.x * blockDim.x + threadIdx.x) * 8 + (k & 7)] = fw.verdict(s0, a, K, k, small);
#else
    for (uint32_t k = 0; k < len1; ++k) V.put(q0 + k, s_val[q0 + k], fw.verdict(s0, a, K, k, small));
    for (uint32_t k = len1; k < len; ++k) V.put(q0 + k, s_val[q0 + k], fw.verdict(s2, a2, K2, k - len1, small2));
#endif
    return true;
}

// cooperative verdict record flags (k_part_half<NMAX, true>): K in the low bits
constexpr uint32_t COOP_SKIP = 1u << 31, COOP_SMALL = 1u << 30;

// part_run_w for the cooperative sweep: the run's first two segments, when decided in closed form,
// are returned as records {s0, K | small, a} instead of written (the workgroup writes them from
// LDS); sequential segments and any third segment write their verdicts here.  len1 / len12 = end of
// the first / second segment relative to q0.
template <int NMAX>
__device__ inline void part_run_defer(FlowWindow<NMAX> &fw, const KeyTable &T, uint32_t key, const uint64_t *s_val,
                                      uint32_t q0, uint32_t q1, const EventSrc &src, const Verdicts &V, int64_t T0,
                                      int64_t *s0o, uint32_t *reco, int32_t *ao, uint32_t &len1, uint32_t &len12,
                                      const uint32_t *segb = nullptr, const uint32_t *hetb = nullptr,
                                      const uint32_t *prib = nullptr) {
    reco[0] = reco[1] = COOP_SKIP;
    len1 = len12 = 0;
    uint32_t q = q0;
    int si = 0;
    while (q < q1) {
        int32_t a;
        bool prio;
        const int64_t E = fw.event(s_val[q], src, T0, a, prio);
        bool pr = prio && fw.kind == KIND_CLUSTER, ah = false;
        uint32_t q2 = q + 1;
        if (segb) {
            // segment starts / acquire-differs / prioritized positions marked by the whole workgroup
            // (k_part_half)
            uint32_t wi = q2 >> 5;
            uint32_t m = q2 < q1 ? segb[wi] & (~0u << (q2 & 31)) : 0u;
            while (!m && (wi + 1) * 32 < q1) m = segb[++wi];
            q2 = m ? min(q1, wi * 32 + (uint32_t)__ffs(m) - 1) : q1;
            for (uint32_t hw = q >> 5; hw <= (q2 - 1) >> 5; ++hw) {
                uint32_t msk = ~0u;
                if (hw == q >> 5) msk &= ~0u << (q & 31);
                if (hw == (q2 - 1) >> 5 && ((q2 & 31) != 0)) msk &= (1u << (q2 & 31)) - 1u;
                ah |= (hetb[hw] & msk) != 0;
                pr |= (prib[hw] & msk) != 0;
            }
        } else {
            for (; q2 < q1; ++q2) {
                int32_t a2;
                bool p2;
                if (fw.event(s_val[q2], src, T0, a2, p2) != E) break;
                ah |= a2 != a;
                pr |= p2 && fw.kind == KIND_CLUSTER;
            }
        }
        if (fw.slow(E, pr)) {
            fw.sequential(T, key, E, s_val, q, q2, src, V);
        } else if (ah) {
            fw.hetero(E, s_val, q, q2, src, V, T0);
        } else {
            int64_t s0;
            uint32_t K;
            const uint32_t len = q2 - q;
            fw.fast(E, a, len, s0, K);
            const bool small = s0 >= 0 && s0 + (int64_t)len * a < (int64_t)INT32_MAX;
            if (si < 2) {
                s0o[si] = s0;
                reco[si] = K | (small ? COOP_SMALL : 0u);
                ao[si] = a;
            } else {
                for (uint32_t k = 0; k < len; ++k) V.put(q + k, s_val[q + k], fw.verdict(s0, a, K, k, small));
            }
        }
        if (si == 0) len1 = q2 - q0;
        if (si <= 1) len12 = q2 - q0;
        ++si;
        q = q2;
    }
    fw.flush();
}

template <int NMAX>
__device__ inline void part_run(const KeyTable &T, uint32_t key, const uint64_t *s_val, uint32_t q0, uint32_t q1,
                                const EventSrc &src, const Verdicts &V, int64_t T0) {
    FlowWindow<NMAX> fw;
    fw.load(T, key, T0);
    part_run_w<NMAX>(fw, T, key, s_val, q0, q1, src, V, T0);
}

// Runs longer than this are decided by a whole workgroup (k_part_long): one lane walking a hot
// flow's events would serialise the batch.
constexpr uint32_t LONG_RUN = 2048;
constexpr int PL_THREADS = 512;
constexpr int PL_ITEMS = 8;
constexpr int PL_CHUNK = PL_THREADS * PL_ITEMS;

// Block-wide exclusive scan of one int64 per thread (per-wave totals in lds_waves[THREADS / WAVE]).
__device__ inline int64_t block_exclusive_scan64(int64_t v, int64_t *lds_waves, int64_t *total) {
    const int lane = (int)lane_id();
    const int wave = threadIdx.x / WAVE;
    int64_t inc = v;
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
        const int64_t u = __shfl_up(inc, off, WAVE);
        if (lane >= off) inc += u;
    }
    if (lane == WAVE - 1) lds_waves[wave] = inc;
    __syncthreads();
    int64_t base = 0, tot = 0;
    const int nw = blockDim.x / WAVE;
    for (int w = 0; w < nw; ++w) {
        const int64_t x = lds_waves[w];
        if (w < wave) base += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// LDS scratch of the cooperative heterogeneous walk
struct HetLds {
    int64_t waves[16];
    uint32_t first[2];
    int64_t acq, np;
};

// A heterogeneous-acquire segment decided by the whole workgroup (k_part_long): chunk positions
// [st, en), thread t owning positions t*ITEMS + k with acquire a[k] (also staged in LDS, a_lds).  The
// greedy walk of het_walk: one workgroup round first -- every event passes while admits(x + the sum
// of the acquires before it): a block scan and a block min of the first failing position f settle
// [st, f) -- then, if the window saturated, wave 0 alone walks [f, en) with wave_walk (from there on
// passes are rare: at most the remaining capacity / min acquire of them, each a wave round, no
// workgroup barriers).  Returns the segment's sums (all lanes).
template <int ITEMS>
__device__ inline HetSums coop_het(uint32_t st, uint32_t en, const int32_t (&a)[ITEMS], const int32_t *a_lds,
                                   int64_t x, uint8_t kind, double thr, double I_s, const uint64_t *cval,
                                   const Verdicts &V, HetLds &L) {
    // (V.obase = the chunk's first position: cval[q]'s verdict goes to V.at(q, cval[q]))
    const uint32_t t0 = threadIdx.x * ITEMS;
    const int64_t x0 = x;
    int64_t mine = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k)
        if (t0 + k >= st && t0 + k < en) mine += a[k];
    if (threadIdx.x == 0) L.first[0] = en;
    int64_t total_acq;
    const int64_t pre = block_exclusive_scan64(mine, L.waves, &total_acq);   // (its barriers order the init)
    const bool live = admits(kind, thr, I_s, x, 1);
    uint32_t myf = en;
    int64_t pk = pre;
    if (live) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t q = t0 + k;
            if (q >= st && q < en) {
                if (myf == en && !admits(kind, thr, I_s, wrap_add(x, pk), a[k])) myf = q;
                pk += a[k];
            }
        }
    } else {
        myf = st;
    }
    if (myf < en) atomicMin(&L.first[0], myf);
    __syncthreads();
    const uint32_t f = L.first[0];
    pk = pre;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const uint32_t q = t0 + k;
        if (q >= st && q < f) {
            V.put(q, cval[q], pack_verdict(ST_OK, java_d2i(remaining_of(thr, I_s, wrap_add(x, pk), a[k])), 0));
            pk += a[k];
        }
        if (q == f && f < en) L.acq = pk;     // the passed sum before f (its prefix)
    }
    int64_t npass = (int64_t)(f - st);
    __syncthreads();
    if (f >= en) {
        x = wrap_add(x, total_acq);
    } else {
        x = wrap_add(x, L.acq);
        if (threadIdx.x < WAVE) {
            int64_t np = 0, acq = 0;
            const uint32_t d = wave_walk(
                kind, thr, I_s, en - f, x, np, acq, [&](uint32_t i) { return cval[f + i]; },
                [&](uint32_t i, uint64_t v, int32_t &ai, uint64_t *&dst) {
                    ai = a_lds[f + i];
                    dst = V.out + V.at(f + i, v);
                });
            if (threadIdx.x == 0) { L.acq = x; L.np = np; L.first[1] = f + d; }
        }
        __syncthreads();
        x = L.acq;
        npass += L.np;
        const uint32_t dead0 = L.first[1];      // from here on every event is blocked
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t q = t0 + k;
            if (q >= dead0 && q < en) V.put(q, cval[q], pack_verdict(ST_BLOCKED, 0, 0));
        }
        __syncthreads();
    }
    HetSums h;
    h.pass = wrap_add(x, -x0);
    h.npass = npass;
    h.block = wrap_add(total_acq, -h.pass);
    h.nblock = (int64_t)(en - st) - npass;
    return h;
}

// Hot runs, three kernels.  k_long_scan (every chunk of every run in parallel): the chunk's summary
// {first epoch, acquire sum, events, one epoch and no prioritized request?}.  k_part_long (one
// workgroup per run, chunks in order): a chunk that lies wholly in the epoch at which the window
// went dead -- not even an acquire of 1 admitted, no occupy transfer pending, no newer slot -- is
// only booked (BLOCK += its acquire sum, BLOCK_REQUEST += its events: a few scalar adds) and
// flagged; every other chunk is decided in full (below).  k_long_dead (every chunk in parallel)
// writes the flagged chunks' BLOCKED verdicts.  A saturated hot flow thus costs its live prefix plus
// a streaming pass, not a serial walk over its events.
static_assert(LR_CHUNK == (uint32_t)PL_CHUNK, "chunk records match the k_part_long chunk");
constexpr int LS_THREADS = 256;
constexpr int LS_ITEMS = LR_CHUNK / LS_THREADS;

__device__ inline void long_chunk(const LongRuns &L, uint32_t g, uint32_t &q0c, uint32_t &cn, uint32_t &key) {
    const uint32_t r = L.chunk_run[g];
    const uint32_t q0 = L.runs[4 * (uint64_t)r], q1 = L.runs[4 * (uint64_t)r + 1];
    key = L.runs[4 * (uint64_t)r + 2];
    q0c = q0 + (g - L.runs[4 * (uint64_t)r + 3]) * LR_CHUNK;
    cn = min(LR_CHUNK, q1 - q0c);
}

__global__ __launch_bounds__(LS_THREADS) void k_long_scan(KeyTable T, const uint64_t *__restrict__ sval, LongRuns L,
                                                          EventSrc src) {
    __shared__ int64_t w_min[LS_THREADS / WAVE], w_max[LS_THREADS / WAVE], w_sum[LS_THREADS / WAVE];
    __shared__ uint32_t w_pr[LS_THREADS / WAVE];
    const uint32_t total = *L.nchunk;
    const int64_t T0 = src.t0();
    for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
        uint32_t q0c, cn, key;
        long_chunk(L, g, q0c, cn, key);
        const int32_t w = T.w[key];
        const double rcp = T.rcp_w[key];
        const bool cluster = T.kind[key] == KIND_CLUSTER;
        int64_t mn = INT64_MAX, mx = INT64_MIN, sum = 0;
        uint32_t pr = 0;
        uint64_t v[LS_ITEMS];
#pragma unroll
        for (int k = 0; k < LS_ITEMS; ++k) {
            const uint32_t q = k * LS_THREADS + threadIdx.x;
            v[k] = q < cn ? sval[q0c + q] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < LS_ITEMS; ++k) {
            const uint32_t q = k * LS_THREADS + threadIdx.x;
            if (q >= cn) continue;
            int64_t t;
            int32_t a;
            bool prio;
            src.unpack(v[k], T0, t, a, prio);
            const int64_t E = epoch_of(t, w, rcp);
            mn = E < mn ? E : mn;
            mx = E > mx ? E : mx;
            sum += a;
            pr |= (prio && cluster) ? 1u : 0u;
        }
#pragma unroll
        for (int off = WAVE / 2; off > 0; off >>= 1) {
            const int64_t a1 = __shfl_xor(mn, off, WAVE), a2 = __shfl_xor(mx, off, WAVE), a3 = __shfl_xor(sum, off, WAVE);
            mn = a1 < mn ? a1 : mn;
            mx = a2 > mx ? a2 : mx;
            sum += a3;
            pr |= __shfl_xor(pr, off, WAVE);
        }
        const int wave = threadIdx.x / WAVE;
        if (lane_id() == 0) { w_min[wave] = mn; w_max[wave] = mx; w_sum[wave] = sum; w_pr[wave] = pr; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int i = 1; i < LS_THREADS / WAVE; ++i) {
                mn = w_min[i] < mn ? w_min[i] : mn;
                mx = w_max[i] > mx ? w_max[i] : mx;
                sum += w_sum[i];
                pr |= w_pr[i];
            }
            LongRec R;
            R.E = mn;
            R.acq = sum;
            R.cnt = cn;
            R.flags = (mn == mx && !pr) ? LR_UNIFORM : 0u;
            R.pad = 0;
            L.rec[g] = R;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(LS_THREADS) void k_long_dead(const uint64_t *__restrict__ sval, LongRuns L, Verdicts V) {
    const uint32_t total = *L.nchunk;
    for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
        if (!(L.rec[g].flags & LR_DEAD)) continue;
        uint32_t q0c, cn, key;
        long_chunk(L, g, q0c, cn, key);
#pragma unroll
        for (int k = 0; k < LS_ITEMS; ++k) {
            const uint32_t q = k * LS_THREADS + threadIdx.x;
            if (q < cn) V.put(q0c + q, sval[q0c + q], pack_verdict(ST_BLOCKED, 0, 0));
        }
    }
}

// k_part_long: one workgroup per run (grid-stride over the runs), its chunks in order.  A chunk
// decided in full: every lane computes the epochs of its 8 contiguous events, segment heads come
// from a block scan, lane 0 walks the chunk's segments with the window in its VGPRs (closed form or
// sequential) up to a heterogeneous-acquire one, which the workgroup decides (coop_het), then all
// lanes write the closed-form verdicts.  A chunk boundary only splits a segment in two consecutive
// segments of the same epoch, which the window algebra treats identically.
template <int NMAX>
__global__ __launch_bounds__(PL_THREADS) void k_part_long(KeyTable T, const uint64_t *__restrict__ sval, LongRuns L,
                                                          EventSrc src, Verdicts V,
                                                          const unsigned long long *__restrict__ stat,
                                                          unsigned long long *__restrict__ host_stat) {
    // the last kernel of a partition batch publishes the skew statistic to pinned host memory
    if (host_stat && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(host_stat, *stat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (L.host_chunks && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(L.host_chunks, *L.nchunk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __shared__ uint16_t seg_start[PL_CHUNK + 1];
    __shared__ int64_t seg_E[PL_CHUNK];
    __shared__ int32_t seg_a[PL_CHUNK];
    __shared__ int64_t seg_s0[PL_CHUNK];
    __shared__ uint32_t seg_K[PL_CHUNK];
    __shared__ uint32_t seg_flag[PL_CHUNK];      // bit0 prioritized, bit1 verdicts written, bit2 acquire differs
    __shared__ int64_t l_E[PL_THREADS];
    __shared__ int32_t l_a[PL_THREADS];
    __shared__ uint32_t waves_tot[PL_THREADS / WAVE];
    __shared__ uint32_t s_nseg;
    __shared__ HetLds hl;
    __shared__ uint32_t s_het;
    __shared__ int64_t s_hx;
    __shared__ uint32_t s_stop, s_dcnt;         // dead stretch: first chunk not in it, events in it
    __shared__ unsigned long long s_dacq;        // ... and their acquire sum
    __shared__ int32_t a_lds[PL_CHUNK];          // the chunk's acquire counts (coop_het's wave walk)
    __shared__ uint32_t s_dead;                  // the window is dead at epoch s_deadE
    __shared__ int64_t s_deadE;
    const uint32_t total = *L.nrun;
    const int64_t T0 = src.t0();
    for (uint32_t r = blockIdx.x; r < total; r += gridDim.x) {
        const uint32_t q0 = L.runs[4 * (uint64_t)r], q1 = L.runs[4 * (uint64_t)r + 1];
        const uint32_t key = L.runs[4 * (uint64_t)r + 2], cb = L.runs[4 * (uint64_t)r + 3];
        const uint32_t nch = (q1 - q0 + PL_CHUNK - 1) / PL_CHUNK;
        FlowWindow<NMAX> fw;                      // meaningful in lane 0 only
        if (threadIdx.x == 0) {
            fw.load(T, key, T0);
            s_dead = 0;
            if (L.rec) {                          // already dead at the first chunk's epoch (an earlier batch)?
                const LongRec R0 = L.rec[cb];
                if ((R0.flags & LR_UNIFORM) && fw.dead_at(R0.E)) {
                    s_dead = 1;
                    s_deadE = R0.E;
                }
            }
        }
        __syncthreads();                          // s_dead is read by every wave below
        const int32_t w = T.w[key];
        const double rcp = T.rcp_w[key];
        const uint8_t kind = T.kind[key];
        const bool cluster = kind == KIND_CLUSTER;
        const double thr = T.thr[key], I_s = T.I_s[key];
        bool h_fresh = false;                     // lane 0: the cooperative segment's rolled slot was fresh
        HetSums dsum{0, 0, 0, 0};                 // lane 0: dead chunks booked but not yet written back
#ifdef SENTINEL_DIAG_LONG
        uint32_t d_full = 0, d_dead = 0, d_deadflag = 0, d_unif = 0;
        uint64_t d_t0 = __builtin_amdgcn_s_memrealtime(), d_tfull = 0, d_tc = 0, d_tpro = 0, d_twalk = 0;
#endif
        for (uint32_t ci = 0; ci < nch; ++ci) {
            if (L.rec && s_dead) {
                // the dead stretch from ci: chunks wholly in the dead epoch (one epoch, no prioritized
                // request), PL_THREADS records at a time: booked and flagged in parallel
                const uint32_t j = ci + threadIdx.x;
                LongRec R{};
                bool elig = false;
                if (j < nch) {
                    R = L.rec[cb + j];
                    elig = (R.flags & LR_UNIFORM) && R.E == s_deadE;
                }
                if (threadIdx.x == 0) { s_stop = nch; s_dacq = 0; s_dcnt = 0; }
                __syncthreads();
                if (!elig && j < nch) atomicMin(&s_stop, j);
                __syncthreads();
                const uint32_t stop = min(s_stop, ci + (uint32_t)PL_THREADS);
                if (stop > ci) {
                    if (j < stop) {
                        L.rec[cb + j].flags = R.flags | LR_DEAD;
                        atomicAdd(&s_dacq, (unsigned long long)R.acq);
                        atomicAdd(&s_dcnt, R.cnt);
                    }
                    __syncthreads();
                    if (threadIdx.x == 0) {
#ifdef SENTINEL_DIAG_LONG
                        d_dead += stop - ci;
#endif
                        dsum.block = wrap_add(dsum.block, (int64_t)s_dacq);
                        dsum.nblock += s_dcnt;
                    }
                    __syncthreads();
                    ci = stop - 1;
                    continue;
                }
            }
            if (threadIdx.x == 0 && dsum.nblock) {
                fw.het_book(s_deadE, false, dsum);
                dsum = HetSums{0, 0, 0, 0};
            }
#ifdef SENTINEL_DIAG_LONG
            d_tc = __builtin_amdgcn_s_memrealtime();
#endif
            const uint32_t c0 = q0 + ci * PL_CHUNK;
            const uint32_t cn = min((uint32_t)PL_CHUNK, q1 - c0);
            int64_t E[PL_ITEMS];
            int32_t a[PL_ITEMS];
            uint32_t heads = 0, bad = 0, ahet = 0;
#pragma unroll
            for (int k = 0; k < PL_ITEMS; ++k) {
                const uint32_t qq = threadIdx.x * PL_ITEMS + k;
                E[k] = 0;
                a[k] = 0;
                if (qq < cn) {
                    int64_t t;
                    bool prio;
                    src.unpack(sval[c0 + qq], T0, t, a[k], prio);
                    E[k] = epoch_of(t, w, rcp);
                    if (prio && cluster) bad |= 1u << k;
                }
            }
            l_E[threadIdx.x] = E[PL_ITEMS - 1];
            l_a[threadIdx.x] = a[PL_ITEMS - 1];
#pragma unroll
            for (int k = 0; k < PL_ITEMS; ++k) a_lds[threadIdx.x * PL_ITEMS + k] = a[k];
            for (uint32_t g = threadIdx.x; g < PL_CHUNK; g += PL_THREADS) seg_flag[g] = 0;
            __syncthreads();
            int64_t pe = threadIdx.x ? l_E[threadIdx.x - 1] : 0;
            int32_t pa = threadIdx.x ? l_a[threadIdx.x - 1] : 0;
#pragma unroll
            for (int k = 0; k < PL_ITEMS; ++k) {
                const uint32_t qq = threadIdx.x * PL_ITEMS + k;
                if (qq < cn) {
                    if (qq == 0 || E[k] != pe) heads |= 1u << k;
                    else if (a[k] != pa) ahet |= 1u << k;
                }
                pe = E[k];
                pa = a[k];
            }
            uint32_t nseg;
            uint32_t g = block_exclusive_scan((uint32_t)__popc(heads), waves_tot, &nseg);
            uint32_t gid[PL_ITEMS];
#pragma unroll
            for (int k = 0; k < PL_ITEMS; ++k) {
                const uint32_t qq = threadIdx.x * PL_ITEMS + k;
                if (heads & (1u << k)) {
                    seg_start[g] = (uint16_t)qq;
                    seg_E[g] = E[k];
                    seg_a[g] = a[k];
                    ++g;
                }
                gid[k] = g - 1;
            }
            if (threadIdx.x == 0) s_nseg = nseg;
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PL_ITEMS; ++k)
                if (threadIdx.x * PL_ITEMS + k < cn && ((bad | ahet) & (1u << k)))
                    atomicOr(&seg_flag[gid[k]], ((bad >> k) & 1u) | (((ahet >> k) & 1u) << 2));
            __syncthreads();
            // lane 0 walks the segments (closed form / sequential) up to the next heterogeneous-acquire
            // one, which the whole workgroup decides (coop_het); then lane 0 goes on
            const uint32_t ns = s_nseg;
            uint32_t from = 0;
#ifdef SENTINEL_DIAG_LONG
            d_tpro += __builtin_amdgcn_s_memrealtime() - d_tc;
#endif
            for (;;) {
                if (threadIdx.x == 0) {
                    uint32_t sgi = from;
                    for (; sgi < ns; ++sgi) {
                        const uint32_t st = seg_start[sgi];
                        const uint32_t en = sgi + 1 < ns ? seg_start[sgi + 1] : cn;
                        const int64_t Es = seg_E[sgi];
                        if (fw.slow(Es, seg_flag[sgi] & 1u)) {
                            fw.sequential(T, key, Es, sval, c0 + st, c0 + en, src, V);
                            seg_flag[sgi] |= 2u;
                        } else if (seg_flag[sgi] & 4u) {
                            s_hx = fw.het_begin(Es, h_fresh);
                            seg_flag[sgi] |= 2u;
                            break;
                        } else {
                            int64_t s0;
                            uint32_t K;
                            fw.fast(Es, seg_a[sgi], en - st, s0, K);
                            seg_s0[sgi] = s0;
                            seg_K[sgi] = K;
                        }
                    }
                    s_het = sgi;
                    if (sgi >= ns) {               // the chunk is decided: is the window dead now?
                        const int64_t El = seg_E[ns - 1];
                        s_dead = fw.dead_at(El) ? 1u : 0u;
                        s_deadE = El;
#ifdef SENTINEL_DIAG_LONG
                        ++d_full;
                        d_deadflag += s_dead;
#endif
                    }
                }
                __syncthreads();
                const uint32_t hs = s_het;
                if (hs >= ns) break;
                const uint32_t st = seg_start[hs];
                const uint32_t en = hs + 1 < ns ? seg_start[hs + 1] : cn;
                const HetSums sums = coop_het<PL_ITEMS>(st, en, a, a_lds, s_hx, kind, thr, I_s, sval + c0, V.based(c0), hl);
                if (threadIdx.x == 0) fw.het_book(seg_E[hs], h_fresh, sums);
                from = hs + 1;
            }
#ifdef SENTINEL_DIAG_LONG
            d_twalk += __builtin_amdgcn_s_memrealtime() - d_tc;
#endif
#pragma unroll
            for (int k = 0; k < PL_ITEMS; ++k) {
                const uint32_t qq = threadIdx.x * PL_ITEMS + k;
                if (qq >= cn) continue;
                const uint32_t sg = gid[k];
                if (seg_flag[sg] & 2u) continue;
                uint64_t v;
                if (qq - seg_start[sg] < seg_K[sg])
                    v = pack_verdict(ST_OK, java_d2i(remaining_of(thr, I_s,
                                                                  wrap_add(seg_s0[sg], wrap_mul((int64_t)(qq - seg_start[sg]), seg_a[sg])),
                                                                  seg_a[sg])), 0);
                else
                    v = pack_verdict(ST_BLOCKED, 0, 0);
                V.put(c0 + qq, sval[c0 + qq], v);
            }
            __syncthreads();
#ifdef SENTINEL_DIAG_LONG
            d_tfull += __builtin_amdgcn_s_memrealtime() - d_tc;
#endif
        }
        if (threadIdx.x == 0) {
            if (dsum.nblock) fw.het_book(s_deadE, false, dsum);
            fw.flush();
#ifdef SENTINEL_DIAG_LONG
            if (nch >= 8)
                printf("long run key %u chunks %u full %u dead %u deadflag %u uniform %u recs %d thr %f kind %d occ %d "
                       "t_total_us %.1f t_full_us %.1f pro %.1f walk %.1f\n", key,
                       nch, d_full, d_dead, d_deadflag, d_unif, L.rec != nullptr, thr, (int)kind, (int)fw.occ_pending,
                       (__builtin_amdgcn_s_memrealtime() - d_t0) / 100.0, d_tfull / 100.0, d_tpro / 100.0,
                       d_twalk / 100.0);
#endif
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Fused per-range sort + decide (the default partition kernels).  A flow range of 2^lb flows is
// split in two halves of 2^hb flows (hb = lb - 1), one 512-thread workgroup per half, so that two
// workgroups fit per CU (LDS ~58 KB, <= 128 VGPRs) and one's HBM round trips overlap the other's
// work.  The two halves of a range run on the same XCD (blocks b and b + 8), so the range's keys
// and values come from HBM once and from that XCD's L2 the second time.  Per half:
//   1. all of the range's keys are loaded at once (24 per thread) and the half's events are
//      ranked with ballots (stable: arrival order kept) -> per-flow counts -> flow starts;
//   2. the half's values are gathered straight into their sorted slots in LDS;
//   3. thread t decides local flow t from LDS (closed-form epoch segments / sequential fallback)
//      and writes the verdicts to their arrival positions.
// A range of more than PH_KEYS events, or a half of more than PH_CAP, is appended to `big` and
// decided by k_part_big, which sorts into HBM; runs longer than LONG_RUN go to k_part_long.
constexpr int PH_THREADS = 512;
#ifndef SENTINEL_PH_MINB
// 4 waves per SIMD = the 2 workgroups per CU the LDS (~59 KB) admits: 128 VGPRs, a few spills.
// Measured: 2 waves per SIMD (no spills, 1 workgroup per CU) is 16% slower.
#define SENTINEL_PH_MINB 4
#endif
constexpr int PH_WAVES = PH_THREADS / WAVE;
// A half's workgroup scans up to PH_KEYS range events (20 per thread) and sorts up to PH_CAP of
// them in LDS; batches whose mean range exceeds 90% of PH_KEYS go to k_part_big whole (engine.hip).
// Measured on config 3 (mean range 8590): 10240 / 5120 is 2.5% faster than 12288 / 6144 (fewer
// value registers, fewer spills); 3 workgroups per CU (80 VGPRs) is 45% slower.
#ifndef SENTINEL_PH_KEYS
#define SENTINEL_PH_KEYS 10240
#endif
#ifndef SENTINEL_PH_CAP
#define SENTINEL_PH_CAP 5120
#endif
constexpr uint32_t PH_KEYS = SENTINEL_PH_KEYS;     // range events scanned by a half's workgroup
constexpr int PH_ITEMS = PH_KEYS / PH_THREADS;     // 20 keys per thread
constexpr uint32_t PH_CAP = SENTINEL_PH_CAP;       // events of one half sorted in LDS (40 KB)
constexpr int PH_BINS = PART_BINS / 2;             // flows per half
constexpr int PH_MAX_LONG = PH_CAP / (LONG_RUN + 1) + 1;
#ifndef SENTINEL_PH_SMALL_RUN
#define SENTINEL_PH_SMALL_RUN 64
#endif
constexpr uint32_t PH_SMALL_RUN = SENTINEL_PH_SMALL_RUN;   // longest run sorted by its own thread
#ifndef SENTINEL_PH_BALLOT_FIRST_HB
#define SENTINEL_PH_BALLOT_FIRST_HB 8
#endif
constexpr int PH_BALLOT_FIRST_HB = SENTINEL_PH_BALLOT_FIRST_HB;   // halves of <= 2^this flows rank by ballots only
// Cooperative verdicts: with at most 2^PH_COOP_HB flows per half (flow tables below 2^19 flows, e.g.
// a rank's shard of 1M flowIds at N >= 2), lanes own several events each; the owner lane of a
// single-segment run only computes {S0, K} and all 512 lanes then write the half's verdicts from LDS,
// instead of 2^hb lanes walking runs of 16..70 events while the other waves idle.
#ifndef SENTINEL_PH_COOP_HB
#define SENTINEL_PH_COOP_HB 8
#endif
#ifndef SENTINEL_PH_COOP_MINHB
#define SENTINEL_PH_COOP_MINHB 0
#endif
constexpr int PH_COOP_HB = SENTINEL_PH_COOP_HB;
#ifndef SENTINEL_PH_COOP_SINGLE_HB
#define SENTINEL_PH_COOP_SINGLE_HB 8
#endif
constexpr int PH_COOP_SINGLE_HB = SENTINEL_PH_COOP_SINGLE_HB;   // coop halves with >= 2^this flows try part_run_single first
constexpr int PH_COOP_FLOWS = 1 << (PH_COOP_HB > 0 ? PH_COOP_HB : 0);
inline bool part_coop(int lb) {
    const int hb = lb > 0 ? lb - 1 : 0;
    return PH_COOP_HB > 0 && hb <= PH_COOP_HB && hb >= SENTINEL_PH_COOP_MINHB;
}
static_assert(PH_BINS == PH_THREADS, "one flow per thread");

// block b -> (range, half): both halves of a range on the XCD b mod 8
__device__ inline void half_of_block(uint32_t b, uint32_t &p, uint32_t &h) {
    p = (b & 7u) | ((b >> 4) << 3);
    h = (b >> 3) & 1u;
}


template <int NMAX, bool COOP>
__global__ __launch_bounds__(PH_THREADS, SENTINEL_PH_MINB) void k_part_half(
    KeyTable T, const uint64_t *__restrict__ pval, uint64_t *__restrict__ gsval,
    const uint32_t *__restrict__ rstart, int lb, int32_t nranges, int32_t nflows, EventSrc src, Verdicts V,
    LongRuns LR, uint32_t *__restrict__ big,
    uint32_t *__restrict__ nbig, unsigned long long *__restrict__ max_range) {
    __shared__ uint64_t sv[PH_CAP];
    // the ballot ranking's per-wave counters and (after the sort) the cooperative verdict records,
    // one per flow of the half, share one LDS buffer
    constexpr int CF = COOP ? PH_COOP_FLOWS : 1;
    constexpr int CNT_BYTES = PH_WAVES * PH_BINS * 2;
    constexpr int COOP_BYTES = COOP ? CF * 56 : 0;
    __shared__ uint64_t ubuf[((CNT_BYTES > COOP_BYTES ? CNT_BYTES : COOP_BYTES) + 7) / 8];
    uint16_t(*cnt)[PH_BINS] = reinterpret_cast<uint16_t(*)[PH_BINS]>(ubuf);
    double *c_thr = reinterpret_cast<double *>(ubuf);                 // [CF]
    double *c_is = c_thr + CF;                                         // [CF]
    int64_t *c_s0 = reinterpret_cast<int64_t *>(c_is + CF);            // [2][CF]
    uint64_t *c_pos = reinterpret_cast<uint64_t *>(c_s0 + 2 * CF);     // [CF] start | len1 << 16 | len12 << 32
    uint32_t *c_K = reinterpret_cast<uint32_t *>(c_pos + CF);          // [2][CF]
    int32_t *c_a = reinterpret_cast<int32_t *>(c_K + 2 * CF);          // [2][CF]
    __shared__ uint32_t base[PH_BINS];
    __shared__ uint32_t waves_tot[PH_WAVES];
    __shared__ uint32_t s_nlong, s_cmax;
    __shared__ uint32_t s_long[PH_MAX_LONG][2];
#ifndef SENTINEL_NO_COOP_BITS
    // parallel segment marking for halves of <= 128 flows: per-flow epoch parameters, then one bit per
    // sorted event for "segment start" and "heterogeneous" (acquire differs from its predecessor's or
    // a prioritized cluster request)
    constexpr int CB = COOP ? (1 << (PH_COOP_HB < PH_COOP_SINGLE_HB - 1 ? PH_COOP_HB : PH_COOP_SINGLE_HB - 1)) : 1;
    static_assert(!COOP || CB <= PH_COOP_FLOWS, "bits-path records fit the coop flow count");
    constexpr int MW = COOP ? (int)(PH_CAP + 31) / 32 : 1;
    __shared__ int64_t p_E0[CB];
    __shared__ double p_rcp[CB];
    __shared__ int32_t p_r0[CB], p_w[CB];
    __shared__ float p_rcpf[CB];
    __shared__ uint32_t p_start[CB], p_cl[CB];
    __shared__ uint32_t segb[MW], hetb[MW], prib[MW];
#endif
    uint32_t p, h;
    half_of_block(blockIdx.x, p, h);
    const int hb = lb > 0 ? lb - 1 : 0;
    if ((int32_t)p >= nranges || (lb == 0 && h == 1)) return;
    const int wave = threadIdx.x / WAVE;
    const uint32_t lane = lane_id();
    const uint32_t t = threadIdx.x;
    const int64_t T0 = src.t0();
    const uint32_t pstart = rstart[p];
    const uint32_t pend = rstart[p + 1];
    const uint32_t size = pend - pstart;
    if (t == 0 && h == 0 && max_range) atomicMax(max_range, (unsigned long long)size);   // skew statistic
    if (size > PH_KEYS) {                                 // block-uniform
        if (t == 0) big[atomicAdd(nbig, 1u)] = (p << 1) | h;
        return;
    }
    PF_STAMP(0);
    // 1. keys (all at once) -> per-flow counts (LDS atomics) -> flow starts.  Item j of thread t is
    // range position j * PH_THREADS + t: the workgroup sweeps the range in arrival order, so the
    // slots handed out below come out nearly in arrival order and the per-run sort has little to do.
    const uint32_t b0 = (uint32_t)wave * (PH_ITEMS * WAVE);
    const uint32_t hmask = (1u << hb) - 1u;
    uint64_t val[PH_ITEMS];                               // every value load in flight at once
    // local flow of a value, or 0xFFFFFFFF: not this half's (recomputed where used: no registers)
    auto local = [&](uint64_t v) -> uint32_t {
        const uint32_t k = (uint32_t)(v >> VAL_KEY_SHIFT);
        return (v != ~0ull && (k >> hb) == h) ? (k & hmask) : 0xFFFFFFFFu;
    };
    // halves of <= 256 flows (runs of ~17+ events: the N >= 2 rank shards): the stable ballot ranking
    // from the start, over wave-contiguous positions -- its per-wave counts give the per-flow counts
    // too, so there is no counting pass and no second load of the range (measured: 500k / 250k / 125k
    // flows 21.9 / 18.9 / 19.9 -> 24.4 / 24.3 / 24.5e9 decisions/s)
    const bool ballot_first = hb <= PH_BALLOT_FIRST_HB;          // block-uniform
#pragma unroll
    for (int j = 0; j < PH_ITEMS; ++j) {
        const uint32_t q = ballot_first ? b0 + j * WAVE + lane : j * PH_THREADS + t;
        val[j] = q < size ? pval[pstart + q] : ~0ull;
    }
    base[t] = 0;
    if (t == 0) { s_nlong = 0; s_cmax = 0; }
    if (ballot_first) {
        uint32_t *z = reinterpret_cast<uint32_t *>(&cnt[0][0]);
        for (int d = t; d < PH_WAVES * PH_BINS / 2; d += PH_THREADS) z[d] = 0;
    }
    __syncthreads();
    const uint32_t key = (p << lb) | (h << hb) | t;
    // rule fields in flight during the sort: loaded unconditionally (a clamped key for lanes without a
    // flow, never used) so no branch join makes the compiler wait for them before the count phase
    FlowWindow<NMAX> fw;
    fw.load_rule(T, min(key, (uint32_t)nflows - 1u));
    uint32_t c, start, total;
    if (ballot_first) {
        uint32_t rank[PH_ITEMS];
#pragma unroll
        for (int j = 0; j < PH_ITEMS; ++j) {
            const uint32_t kj = local(val[j]);
            const bool valid = kj != 0xFFFFFFFFu;
            const uint32_t d = kj & hmask;
            const uint64_t peers = match_peers<PART_MAX_BITS>(d, valid, hb);
            uint32_t r = 0;
            if (valid) r = cnt[wave][d] + mask_rank(peers);
            __builtin_amdgcn_wave_barrier();
            if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane) cnt[wave][d] += (uint16_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
            rank[j] = r;
        }
        __syncthreads();
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < PH_WAVES; ++w) {
            const uint32_t x = cnt[w][t];
            cnt[w][t] = (uint16_t)run;
            run += x;
        }
        c = run;                                          // this thread's flow: events in the half
        start = block_exclusive_scan(c, waves_tot, &total);
        if (total > PH_CAP) {                             // block-uniform: the half does not fit in LDS
            if (t == 0) big[atomicAdd(nbig, 1u)] = (p << 1) | h;
            return;
        }
        base[t] = start;
        __syncthreads();
        PF_STAMP(1);
#pragma unroll
        for (int j = 0; j < PH_ITEMS; ++j) {
            const uint32_t kj = local(val[j]);
            if (kj == 0xFFFFFFFFu) continue;
            sv[base[kj] + cnt[wave][kj] + rank[j]] = val[j];
        }
    } else {
#pragma unroll
    for (int j = 0; j < PH_ITEMS; ++j) {
        const uint32_t kj = local(val[j]);
        if (kj != 0xFFFFFFFFu) atomicAdd(&base[kj], 1u);
    }
    __syncthreads();
    c = base[t];                                          // this thread's flow: events in the half
    start = block_exclusive_scan(c, waves_tot, &total);
    if (total > PH_CAP) {                                 // block-uniform: the half does not fit in LDS
        if (t == 0) big[atomicAdd(nbig, 1u)] = (p << 1) | h;
        return;
    }
    if (c) atomicMax(&s_cmax, c);
    base[t] = start;
    __syncthreads();
    PF_STAMP(1);
    // 2. values into their flow's slots, in arrival order
    if (s_cmax <= PH_SMALL_RUN) {
        // short runs (the common case): unordered slots by LDS atomics, then each thread
        // insertion-sorts its own run by arrival position (the low bits of the value)
#pragma unroll
        for (int j = 0; j < PH_ITEMS; ++j) {
            const uint32_t kj = local(val[j]);
            if (kj != 0xFFFFFFFFu) sv[atomicAdd(&base[kj], 1u)] = val[j];
        }
        __syncthreads();
        for (uint32_t i = start + 1; i < start + c; ++i) {
            const uint64_t v = sv[i];
            const uint32_t sq = (uint32_t)v & SEQ_MASK;
            uint32_t j = i;
            for (; j > start; --j) {
                const uint64_t u = sv[j - 1];
                if (((uint32_t)u & SEQ_MASK) < sq) break;
                sv[j] = u;
            }
            sv[j] = v;
        }
    } else {
        // a long run somewhere: stable ranking with ballots (arrival order kept by construction),
        // over wave-contiguous blocks of the range (item j of a lane = position b0 + j * 64 + lane)
#pragma unroll
        for (int j = 0; j < PH_ITEMS; ++j) {
            const uint32_t q = b0 + j * WAVE + lane;
            val[j] = q < size ? pval[pstart + q] : ~0ull;
        }
        {
            uint32_t *z = reinterpret_cast<uint32_t *>(&cnt[0][0]);
            for (int d = t; d < PH_WAVES * PH_BINS / 2; d += PH_THREADS) z[d] = 0;
        }
        __syncthreads();
        uint32_t rank[PH_ITEMS];
#pragma unroll
        for (int j = 0; j < PH_ITEMS; ++j) {
            const uint32_t kj = local(val[j]);
            const bool valid = kj != 0xFFFFFFFFu;
            const uint32_t d = kj & hmask;
            const uint64_t peers = match_peers<PART_MAX_BITS>(d, valid, hb);
            uint32_t r = 0;
            if (valid) r = cnt[wave][d] + mask_rank(peers);
            __builtin_amdgcn_wave_barrier();
            if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane) cnt[wave][d] += (uint16_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
            rank[j] = r;
        }
        __syncthreads();
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < PH_WAVES; ++w) {
            const uint32_t x = cnt[w][t];
            cnt[w][t] = (uint16_t)run;
            run += x;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PH_ITEMS; ++j) {
            const uint32_t kj = local(val[j]);
            if (kj == 0xFFFFFFFFu) continue;
            sv[base[kj] + cnt[wave][kj] + rank[j]] = val[j];
        }
    }
    }
    __syncthreads();
    PF_STAMP(2);
    // 3. decide.  Hot runs go to k_part_long from HBM: the half's region of gsval is its own
    // (half 0 at the range start, half 1 at its end).
    const uint32_t goff = pstart + (h ? size - total : 0u);
    // decide-order output: the half's sorted events own positions [goff, goff + total); their arrival
    // positions go out in one coalesced sweep, every verdict below to goff + its sorted index
    const Verdicts VV = V.based(goff);
    if (V.oseq)
        for (uint32_t i = t; i < total; i += PH_THREADS) V.oseq[goff + i] = (uint32_t)sv[i] & SEQ_MASK;
    if (c > LONG_RUN) {
        LR.push(goff + start, goff + start + c, key);
        const uint32_t l = atomicAdd(&s_nlong, 1u);
        s_long[l][0] = start;
        s_long[l][1] = c;
    }
    __syncthreads();
    for (uint32_t l = 0; l < s_nlong; ++l)
        for (uint32_t q = t; q < s_long[l][1]; q += PH_THREADS) gsval[goff + s_long[l][0] + q] = sv[s_long[l][0] + q];
    if (COOP) {                                           // launched only when 2^hb <= PH_COOP_FLOWS
#ifndef SENTINEL_NO_COOP_BITS
        const bool bits = hb < PH_COOP_SINGLE_HB;         // block-uniform
        if (bits) {
            for (uint32_t j = t; j < (uint32_t)MW; j += PH_THREADS) { segb[j] = 0; hetb[j] = 0; prib[j] = 0; }
            if (t < (1u << hb) && c > 0) {
                p_E0[t] = epoch_of(T0, fw.w, fw.rcp);
                p_r0[t] = (int32_t)(T0 - p_E0[t] * (int64_t)fw.w);
                p_rcpf[t] = 1.0f / (float)fw.w;
                p_w[t] = fw.w;
                p_rcp[t] = fw.rcp;
                p_start[t] = start;
                p_cl[t] = fw.kind == KIND_CLUSTER;
            }
            __syncthreads();
            for (uint32_t i = t; i < total; i += PH_THREADS) {
                const uint64_t v = sv[i];
                const uint32_t kj = (uint32_t)(v >> VAL_KEY_SHIFT) & hmask;
                FlowWindow<NMAX> lw;                      // epoch parameters only
                lw.w = p_w[kj];
                lw.rcp = p_rcp[kj];
                lw.E0 = p_E0[kj];
                lw.r0 = p_r0[kj];
                lw.rcpf = p_rcpf[kj];
                int32_t ai;
                bool pi;
                const int64_t Ei = lw.event(v, src, T0, ai, pi);
                bool st = i == p_start[kj];
                bool het = false;
                if (!st) {
                    int32_t ap;
                    bool pp;
                    const int64_t Ep = lw.event(sv[i - 1], src, T0, ap, pp);
                    st = Ep != Ei;
                    if (!st) het = ai != ap;
                }
                if (st) atomicOr(&segb[i >> 5], 1u << (i & 31));
                if (het) atomicOr(&hetb[i >> 5], 1u << (i & 31));
                if (pi && p_cl[kj]) atomicOr(&prib[i >> 5], 1u << (i & 31));
            }
            __syncthreads();
        }
        PF_STAMP(4);
#else
        const bool bits = false;
        const uint32_t *segb = nullptr, *hetb = nullptr, *prib = nullptr;
#endif
        if (t < (1u << hb)) {
            int64_t s0[2] = {0, 0};
            uint32_t rec[2] = {COOP_SKIP, COOP_SKIP};
            int32_t a[2] = {0, 0};
            uint32_t len1 = 0, len12 = 0;
            if (c > 0 && c <= LONG_RUN) {
                bool small[2];
                // the single-segment pre-pass pays off only for short runs: with >= ~34 events per flow
                // (hb <= 7) a run straddles an epoch boundary often and the walk alone is cheaper
                // (measured: 125k flows +4%, 250k +1%; 500k flows -1% without it)
                if (hb >= PH_COOP_SINGLE_HB &&
                    part_run_single<NMAX, true>(fw, sv, start, start + c, src, VV, T0, s0, rec, a, small, &len1)) {
                    rec[0] |= small[0] ? COOP_SMALL : 0u;
                    if (len1 < c) rec[1] |= small[1] ? COOP_SMALL : 0u;   // (a second segment: its K)
                    len12 = c;
                } else {
                    fw.load_header(T0);
                    part_run_defer<NMAX>(fw, T, key, sv, start, start + c, src, VV, T0, s0, rec, a, len1, len12,
                                         bits ? segb : nullptr, bits ? hetb : nullptr, bits ? prib : nullptr);
                }
                c_thr[t] = fw.thr;
                c_is[t] = fw.I_s;
            }
            c_s0[t] = s0[0];
            c_s0[CF + t] = s0[1];
            c_K[t] = rec[0];
            c_K[CF + t] = rec[1];
            c_a[t] = a[0];
            c_a[CF + t] = a[1];
            c_pos[t] = (uint64_t)start | ((uint64_t)len1 << 16) | ((uint64_t)len12 << 32);
        }
        __syncthreads();
        PF_STAMP(5);
        // every lane: positions t, t + 512, ... of the half's sorted events (flow key in the value)
        for (uint32_t i = t; i < total; i += PH_THREADS) {
            const uint64_t v = sv[i];
            const uint32_t kj = (uint32_t)(v >> VAL_KEY_SHIFT) & hmask;
            const uint64_t pos = c_pos[kj];
            const uint32_t k = i - (uint32_t)(pos & 0xFFFFu);
            const uint32_t l1 = (uint32_t)(pos >> 16) & 0xFFFFu, l12 = (uint32_t)(pos >> 32) & 0xFFFFu;
            if (k >= l12) continue;                               // third segment on: written by the walk
            const uint32_t sg = k < l1 ? 0u : 1u;
            const uint32_t rec = c_K[sg * CF + kj];
            if (rec & COOP_SKIP) continue;                        // sequential segment: written by the walk
            VV.put(i, v, run_verdict(c_thr[kj], c_is[kj], c_s0[sg * CF + kj], c_a[sg * CF + kj],
                                     rec & (COOP_SMALL - 1u), sg ? k - l1 : k, (rec & COOP_SMALL) != 0));
        }
    } else if (c > 0 && c <= LONG_RUN && !part_run_single<NMAX>(fw, sv, start, start + c, src, VV, T0)) {
        fw.load_header(T0);
        part_run_w<NMAX>(fw, T, key, sv, start, start + c, src, VV, T0);
    }
#ifdef SENTINEL_DIAG_PHASES
    __syncthreads();
    PF_STAMP(3);
#endif
}

// Oversized halves (or every half, `big == nullptr`): the same decision with the half sorted into
// HBM in chunks (any size).  Entry = (range << 1) | half.
constexpr int PB_ITEMS = 8;
constexpr int PB_CHUNK = PH_THREADS * PB_ITEMS;

template <int NMAX>
__global__ __launch_bounds__(PH_THREADS) void k_part_big(
    KeyTable T, const uint64_t *__restrict__ pval, uint64_t *__restrict__ gsval,
    const uint32_t *__restrict__ rstart, int lb, int32_t nranges, EventSrc src, Verdicts V,
    LongRuns LR, const uint32_t *__restrict__ big,
    const uint32_t *__restrict__ nbig, unsigned long long *__restrict__ max_range) {
    __shared__ uint16_t cnt[PH_WAVES][PH_BINS];
    __shared__ uint32_t base[PH_BINS];
    __shared__ uint32_t waves_tot[PH_WAVES];
    const int wave = threadIdx.x / WAVE;
    const uint32_t lane = lane_id();
    const uint32_t t = threadIdx.x;
    const int64_t T0 = src.t0();
    const int hb = lb > 0 ? lb - 1 : 0;
    const uint32_t hmask = (1u << hb) - 1u;
    const uint32_t nwork = big ? *nbig : 2u * (uint32_t)nranges;
    for (uint32_t wi = blockIdx.x; wi < nwork; wi += gridDim.x) {
        const uint32_t e = big ? big[wi] : wi;
        const uint32_t p = e >> 1, h = e & 1u;
        if (lb == 0 && h == 1) continue;                  // block-uniform
        const uint32_t pstart = rstart[p];
        const uint32_t pend = rstart[p + 1];
        const uint32_t size = pend - pstart;
        if (!big && h == 0 && t == 0 && max_range) atomicMax(max_range, (unsigned long long)size);
        base[t] = 0;
        __syncthreads();
        for (uint32_t q = pstart + t; q < pend; q += PH_THREADS) {
            const uint32_t k = (uint32_t)(pval[q] >> VAL_KEY_SHIFT);
            if ((k >> hb) == h) atomicAdd(&base[k & hmask], 1u);
        }
        __syncthreads();
        const uint32_t c = base[t];
        uint32_t total;
        const uint32_t start = block_exclusive_scan(c, waves_tot, &total);
        const uint32_t goff = pstart + (h ? size - total : 0u);
        base[t] = start;
        uint64_t *dst = gsval + goff;
        for (uint32_t c0 = pstart; c0 < pend; c0 += PB_CHUNK) {
            const uint32_t cn = min((uint32_t)PB_CHUNK, pend - c0);
            {
                uint32_t *z = reinterpret_cast<uint32_t *>(&cnt[0][0]);
                for (int d = t; d < PH_WAVES * PH_BINS / 2; d += PH_THREADS) z[d] = 0;
            }
            __syncthreads();
            uint32_t kk[PB_ITEMS], rank[PB_ITEMS];
            uint64_t val[PB_ITEMS];
            const uint32_t b0 = (uint32_t)wave * (PB_ITEMS * WAVE);
#pragma unroll
            for (int j = 0; j < PB_ITEMS; ++j) {
                const uint32_t qq = b0 + j * WAVE + lane;
                val[j] = qq < cn ? pval[c0 + qq] : 0ull;
                kk[j] = qq < cn ? (uint32_t)(val[j] >> VAL_KEY_SHIFT) : 0xFFFFFFFFu;
            }
#pragma unroll
            for (int j = 0; j < PB_ITEMS; ++j) {
                const bool valid = kk[j] != 0xFFFFFFFFu && (kk[j] >> hb) == h;
                const uint32_t d = kk[j] & hmask;
                const uint64_t peers = match_peers<PART_MAX_BITS>(d, valid, hb);
                uint32_t r = 0;
                if (valid) r = cnt[wave][d] + mask_rank(peers);
                __builtin_amdgcn_wave_barrier();
                if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane) cnt[wave][d] += (uint16_t)__popcll(peers);
                __builtin_amdgcn_wave_barrier();
                rank[j] = valid ? r : 0xFFFFFFFFu;
            }
            __syncthreads();
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < PH_WAVES; ++w) {
                const uint32_t x = cnt[w][t];
                cnt[w][t] = (uint16_t)run;
                run += x;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < PB_ITEMS; ++j) {
                if (rank[j] == 0xFFFFFFFFu) continue;
                const uint32_t d = kk[j] & hmask;
                dst[base[d] + cnt[wave][d] + rank[j]] = val[j];
            }
            __syncthreads();
            base[t] += run;
        }
        if (V.oseq)                                       // decide-order output: positions [goff, goff + total)
            for (uint32_t q = t; q < total; q += PH_THREADS) V.oseq[goff + q] = (uint32_t)dst[q] & SEQ_MASK;
        const uint32_t key = (p << lb) | (h << hb) | t;
        if (c > LONG_RUN) LR.push(goff + start, goff + start + c, key);
        if (c > 0 && c <= LONG_RUN) part_run<NMAX>(T, key, dst, start, start + c, src, V.based(goff), T0);
        __syncthreads();                                  // LDS reuse by the next entry
    }
}

}  // namespace sentinel
