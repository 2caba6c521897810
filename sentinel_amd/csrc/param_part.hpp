// param_part.hpp -- the partition-local exact hot-parameter path (gfx950).
//
// Single-value cluster param requests (DefaultTokenService.requestParamToken -> ClusterParamFlowChecker
// .acquireClusterToken, srv/flow/ClusterParamFlowChecker.java:42-87, DTS:51-62) on exact per-value
// counters: one open-addressing HBM slot per (rule, value) key holds the value's {epoch, count} x n
// window (ClusterParamMetric.java:46-82, the value's LongAdder in each bucket's CacheMap,
// ClusterParameterLeapArray.java:33-49; param_table.hpp keeps the table bounded).  A key's requests
// only read and write its own window, so the batch needs grouping by key in arrival order, not a
// global sort:
//
//   k_pp_prep     validation (DTS:51-62, CPFC:37-47) + per-tile histogram of the range digit
//                 d = top bits of mix64(param key); rejected requests are answered here
//   scan          the partition path's 2D scan of the tile-major histograms (partition.hpp)
//   k_pp_scatter  stable multi-split of the valid requests into their ranges: param key, packed
//                 {arrival position, acquire, ts - T0} and rule index, three coalesced arrays
//   k_pp_decide   one workgroup per range, in chunks of PD_CAP requests (arrival order): the chunk's
//                 distinct keys are staged in an LDS open-addressing table (the north star's
//                 "LDS-staged" table: a key's HBM slot is probed once per chunk, not once per
//                 request), its requests ranked stably by LDS entry with ballots and placed in
//                 (key, arrival) order, then one lane per distinct key probes / inserts the HBM
//                 slot, holds the window in VGPRs, decides the key's requests in arrival order and
//                 writes the verdicts to their arrival positions and the rolled pairs back.
//
// Replaces the per-slot radix-sort pipeline (k_param_prep -> 3 radix passes -> k_segments_v ->
// k_process_reg_o4 -> k_verdict): per request it reads the 24-B event twice, moves 20 B through
// the multi-split and writes the 8-B verdict; per distinct key and chunk one table probe, the
// slot's window header and the dirty pairs.
#pragma once

#include "param_rules.hpp"
#include "param_table.hpp"
#include "partition.hpp"

namespace sentinel {

// Packed param value: [0,28) arrival position, [28,37) acquire (escape 0x1FF), [37,64) ts - T0 as a
// signed 27-bit field (escape -2^26).  Escaped fields are read back from the event itself.
constexpr int PV_ACQ_SHIFT = 28;
constexpr uint32_t PV_ACQ_ESC = 0x1FFu;
constexpr int PV_DT_SHIFT = 37;
constexpr int PV_DT_BITS = 27;
constexpr uint32_t PV_DT_MASK = (1u << PV_DT_BITS) - 1u;
constexpr uint32_t PV_DT_ESC = 1u << (PV_DT_BITS - 1);       // -2^26

// The batch clock: ts of the first request (clamped: an invalid first request may carry ts < 0).
__device__ inline int64_t pp_t0(const ParamEvent *ev) {
    const int64_t t = ev[0].ts;
    return t < 0 ? 0 : t;
}

__device__ inline uint64_t pp_pack(uint32_t pos, int64_t ts, int32_t a, int64_t T0) {
    const int64_t dt = ts - T0;
    const uint32_t dtf = (dt > -(int64_t)PV_DT_ESC && dt < (int64_t)PV_DT_ESC) ? ((uint32_t)dt & PV_DT_MASK) : PV_DT_ESC;
    const uint32_t af = (a > 0 && a < (int32_t)PV_ACQ_ESC) ? (uint32_t)a : PV_ACQ_ESC;
    return (uint64_t)pos | ((uint64_t)af << PV_ACQ_SHIFT) | ((uint64_t)dtf << PV_DT_SHIFT);
}

__device__ inline void pp_unpack(uint64_t v, int64_t T0, const ParamEvent *ev, int64_t &ts, int32_t &a) {
    const uint32_t af = (uint32_t)(v >> PV_ACQ_SHIFT) & PV_ACQ_ESC;
    const uint32_t dtf = (uint32_t)(v >> PV_DT_SHIFT) & PV_DT_MASK;
    if (af == PV_ACQ_ESC || dtf == PV_DT_ESC) {
        const ParamEvent e = ev[(uint32_t)v & SEQ_MASK];
        ts = e.ts;
        a = e.acquire;
        return;
    }
    ts = T0 + (int64_t)((int32_t)(dtf << (32 - PV_DT_BITS)) >> (32 - PV_DT_BITS));
    a = (int32_t)af;
}

// Range digit of a param key: the top pbits of its hash (the HBM slot uses the low bits, the LDS
// table bits [32, 32 + PD_HBITS)).
__device__ inline uint32_t pp_digit(uint64_t h, int pbits) {
    return pbits ? (uint32_t)(h >> (64 - pbits)) : 0u;
}

// DefaultTokenService.requestParamToken validation (DTS:51-62: null id / acquire <= 0 -> BAD_REQUEST,
// unknown rule -> NO_RULE_EXISTS), ClusterParamFlowChecker.allowProceed (CPFC:37-47: namespace == null
// -> TOO_MANY_REQUEST); the reserved key 0xFFFFFFFFFFFFFFFF (include/sentinel_amd.h) is BAD_REQUEST;
// ts < 0 -> PP_NEG_TS (answered by param_negative_ts_status).  127 = valid.
constexpr int PP_NEG_TS = 126;
__device__ inline int pp_status(const ParamEvent &e, int32_t nrules, const int32_t *route) {
    if (e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0) return ST_BAD_REQUEST;
    if (e.idx < 0 || e.idx >= nrules) return ST_NO_RULE_EXISTS;
    if (route && route[e.idx] == ROUTE_TOO_MANY) return ST_TOO_MANY_REQUEST;
    if (e.key == PKEY_EMPTY) return ST_BAD_REQUEST;
    if (e.ts < 0) return PP_NEG_TS;
    return 127;
}

// ---------------------------------------------------------------- prep + multi-split
__global__ __launch_bounds__(PP_THREADS) void k_pp_prep(int64_t n, const ParamEvent *__restrict__ ev, int32_t nrules,
                                                         const int32_t *__restrict__ route, ParamRules PR,
                                                         uint64_t *__restrict__ out, int pbits,
                                                         uint32_t *__restrict__ hist, int32_t nparts) {
    __shared__ uint32_t h[PART_BINS];
    const int64_t tile0 = (int64_t)blockIdx.x * PT_TILE;
    ParamEvent evs[PP_ITEMS];                         // every event load of the tile in flight at once
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
        int st = pp_status(evs[j], nrules, route);
        if (st == PP_NEG_TS) st = param_negative_ts_status(PR, (uint32_t)evs[j].idx, evs[j].key, evs[j].acquire);
        if (st == 127) atomicAdd(&h[pp_digit(mix64(evs[j].key), pbits)], 1u);
        else put_verdict(out, (uint32_t)i, st, 0, 0);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nparts; d += PP_THREADS) hist[(int64_t)blockIdx.x * nparts + d] = h[d];
}

// Stable multi-split by range digit (the k_part_scatter scheme: one ballot per digit bit, wave-private
// LDS counters, the tile staged in digit order so every output run is contiguous).  The three output
// arrays are staged one after the other through one 32 KB LDS buffer.
__global__ __launch_bounds__(PT_THREADS) void k_pp_scatter(const ParamEvent *__restrict__ ev, int64_t n, int32_t nrules,
                                                            const int32_t *__restrict__ route, int pbits,
                                                            const uint32_t *__restrict__ offsets, int32_t nparts,
                                                            unsigned long long *__restrict__ okey,
                                                            uint64_t *__restrict__ oval, int32_t *__restrict__ orule) {
    __shared__ uint16_t cnt[PT_WAVES][PART_BINS];
    __shared__ uint32_t goff[PART_BINS];
    __shared__ uint32_t loff[PART_BINS];
    __shared__ uint32_t waves_tot[PT_WAVES];
    __shared__ uint16_t sdig[PT_TILE];
    __shared__ uint64_t stage[PT_TILE];
    const int wave = threadIdx.x / WAVE;
    const uint32_t lane = lane_id();
    for (int d = threadIdx.x; d < PART_BINS; d += PT_THREADS) {
#pragma unroll
        for (int w = 0; w < PT_WAVES; ++w) cnt[w][d] = 0;
        goff[d] = d < nparts ? offsets[(int64_t)blockIdx.x * nparts + d] : 0u;
    }
    const int64_t tile0 = (int64_t)blockIdx.x * PT_TILE;
    const int64_t base = tile0 + (int64_t)wave * (PT_ITEMS * WAVE);
    const int64_t T0 = pp_t0(ev);
    ParamEvent evs[PT_ITEMS];
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j) {
        const int64_t i = base + j * WAVE + lane;
        if (i < n) evs[j] = ev[i];
    }
    __syncthreads();
    uint32_t dig[PT_ITEMS], rank[PT_ITEMS];
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j) {
        const int64_t i = base + j * WAVE + lane;
        const bool valid = i < n && pp_status(evs[j], nrules, route) == 127;
        const uint32_t d = valid ? pp_digit(mix64(evs[j].key), pbits) : 0u;
        const uint64_t peers = match_peers<PART_MAX_BITS>(d, valid, pbits);
        uint32_t r = 0;
        if (valid) r = cnt[wave][d] + mask_rank(peers);
        __builtin_amdgcn_wave_barrier();
        if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane) cnt[wave][d] += (uint16_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        dig[j] = d;
        rank[j] = valid ? r : 0xFFFFFFFFu;
    }
    __syncthreads();
    constexpr int DPT = PART_BINS / PT_THREADS;
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
    uint32_t pos[PT_ITEMS];
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j) {
        pos[j] = 0xFFFFFFFFu;
        if (rank[j] == 0xFFFFFFFFu) continue;
        pos[j] = loff[dig[j]] + cnt[wave][dig[j]] + rank[j];
        sdig[pos[j]] = (uint16_t)dig[j];
        stage[pos[j]] = evs[j].key;
    }
    __syncthreads();
    auto write_out = [&](auto put) {
        for (uint32_t p = threadIdx.x; p < total; p += PT_THREADS) {
            const uint32_t d = sdig[p];
            const uint32_t dst = goff[d] + p - loff[d];
            if (dst >= (uint64_t)n) continue;          // guard: a corrupt offset must never write out of bounds
            put(dst, p);
        }
    };
    write_out([&](uint32_t dst, uint32_t p) { okey[dst] = stage[p]; });
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j)
        if (pos[j] != 0xFFFFFFFFu) stage[pos[j]] = pp_pack((uint32_t)(base + j * WAVE + lane), evs[j].ts, evs[j].acquire, T0);
    __syncthreads();
    write_out([&](uint32_t dst, uint32_t p) { oval[dst] = stage[p]; });
    __syncthreads();
    uint32_t *stage32 = reinterpret_cast<uint32_t *>(stage);
#pragma unroll
    for (int j = 0; j < PT_ITEMS; ++j)
        if (pos[j] != 0xFFFFFFFFu) stage32[pos[j]] = (uint32_t)evs[j].idx;
    __syncthreads();
    write_out([&](uint32_t dst, uint32_t p) { orule[dst] = (int32_t)stage32[p]; });
}

// ---------------------------------------------------------------- decide
#ifndef SENTINEL_PD_THREADS
#define SENTINEL_PD_THREADS 256
#endif
#ifndef SENTINEL_PD_ITEMS
#define SENTINEL_PD_ITEMS 8
#endif
#ifndef SENTINEL_PD_HBITS
#define SENTINEL_PD_HBITS 11
#endif
constexpr int PD_THREADS = SENTINEL_PD_THREADS;
constexpr int PD_WAVES = PD_THREADS / WAVE;
constexpr int PD_ITEMS = SENTINEL_PD_ITEMS;
constexpr uint32_t PD_CAP = PD_THREADS * PD_ITEMS;      // requests per chunk
constexpr int PD_HBITS = SENTINEL_PD_HBITS;
constexpr uint32_t PD_HT = 1u << PD_HBITS;              // LDS hash entries per round
constexpr int PD_PROBES = 32;                           // a key not placed within this many probes waits a round
constexpr int PD_EPT = PD_HT / PD_THREADS;               // entries per thread in the scans
static_assert(PD_HT % PD_THREADS == 0, "entries per thread");
static_assert(PD_CAP <= 65535, "16-bit wave counters");
// requests per range the host aims at (ranges <= PART_BINS)
constexpr int64_t PD_TARGET = 2048;

// Insert / find a key in the chunk's LDS table; -1: not within PD_PROBES probes (full neighbourhood).
// All requests of one key agree: entries never change once set, so every request of a key that fails
// saw the same PD_PROBES other keys.
__device__ inline int pd_insert(unsigned long long *hkey, int32_t *hrule, unsigned long long key, int32_t rule,
                                uint32_t h0) {
    uint32_t h = h0;
    for (int p = 0; p < PD_PROBES; ++p) {
        const unsigned long long cur = hkey[h];
        if (cur == key) return (int)h;
        if (cur == PKEY_EMPTY) {
            const unsigned long long prev = atomicCAS(&hkey[h], (unsigned long long)PKEY_EMPTY, key);
            if (prev == PKEY_EMPTY) {
                hrule[h] = rule;
                return (int)h;
            }
            if (prev == key) return (int)h;
        }
        h = (h + 1) & (PD_HT - 1);
    }
    return -1;
}

// One key's requests [q0, q1) of sv (arrival order) against its exact HBM slot: the ClusterParamFlowChecker
// state machine per request (CPFC:58-86 for one value: roll = LeapArray.currentWindow, sum over the valid
// buckets, R = (T_v - sum / I_s) - a, pass iff !(R < 0) -> addValue), the window {epoch, count} x NMAX in
// VGPRs, only the touched pairs written back.  A bucket newer than the request's epoch (the clock went
// backwards for this key) is the detached-bucket case (LeapArray.java:241-246): the sum reads the array,
// the add is lost.
template <int NMAX>
__device__ inline void pd_walk(const ParamRules &PR, const PSlots &S, unsigned long long key, int32_t rule,
                               const uint64_t *sv, uint32_t q0, uint32_t q1, const ParamEvent *ev, int64_t T0,
                               uint64_t *out, uint32_t &nfresh) {
    const int nsc = PR.n[rule];
    const int32_t w = PR.w[rule];
    const double rcp = PR.rcp_w[rule];
    const double I_s = PR.I_s[rule];
    const double thr = value_threshold(PR, (uint32_t)rule, key);        // CPFC:101-120
    const uint32_t before = nfresh;
    const int64_t h = slot_insert_counted(S.keys, S.mask, key, nfresh);
    if (h < 0) {                                                         // table full: param_reserve prevents it
        for (uint32_t q = q0; q < q1; ++q) put_verdict(out, (uint32_t)sv[q] & SEQ_MASK, ST_FAIL, 0, 0);
        return;
    }
    if (nfresh != before) S.rule[h] = rule;                              // read by the rebuild / top values
    int64_t *st = S.state + h * S.stride;
    int64_t ep[NMAX], ct[NMAX];
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {                                     // in bounds: stride >= 2 NMAX words
        const longlong2 v = *reinterpret_cast<const longlong2 *>(st + 2 * j);
        ep[j] = j < nsc ? v.x : EPOCH_ABSENT;
        ct[j] = j < nsc ? v.y : 0;
    }
    const double rcpn = 1.0 / (double)nsc;
    uint32_t dirty = 0;
    int64_t curE = -1, sum = 0;
    int slot = -1;
#pragma unroll 1
    for (uint32_t q = q0; q < q1; ++q) {
        const uint64_t v = sv[q];
        int64_t t;
        int32_t a;
        pp_unpack(v, T0, ev, t, a);
        const int64_t E = epoch_of(t, w, rcp);
        if (E != curE) {                                                 // LeapArray.currentWindow(t)
            curE = E;
            slot = (int)(E - epoch_of(E, nsc, rcpn) * nsc);
            bool detached = false;
#pragma unroll
            for (int j = 0; j < NMAX; ++j) {
                if (j != slot || ep[j] == E) continue;
                if (ep[j] != EPOCH_ABSENT && ep[j] > E) detached = true;
                else { ep[j] = E; ct[j] = 0; dirty |= 1u << j; }
            }
            if (detached) slot = -1;
            sum = 0;
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (ep[j] != EPOCH_ABSENT && ep[j] > E - nsc) sum = wrap_add(sum, ct[j]);
        }
        const double next = (thr - div_interval((double)sum, I_s)) - (double)a;
        uint64_t vd;
        if (!(next < 0.0)) {                                             // CPFC:64-66 (and addValue, CPFC:73-76)
            if (slot >= 0) {
#pragma unroll
                for (int j = 0; j < NMAX; ++j)
                    if (j == slot) { ct[j] = wrap_add(ct[j], a); dirty |= 1u << j; }
                sum = wrap_add(sum, a);
            }
            vd = pack_verdict(ST_OK, java_d2i(next), 0);
        } else {
            vd = pack_verdict(ST_BLOCKED, 0, 0);
        }
        store_verdict(out, (uint32_t)v & SEQ_MASK, vd);
    }
#pragma unroll
    for (int j = 0; j < NMAX; ++j)
        if (dirty & (1u << j)) *reinterpret_cast<longlong2 *>(st + 2 * j) = longlong2{ep[j], ct[j]};
}

template <int NMAX>
__global__ __launch_bounds__(PD_THREADS) void k_pp_decide(const unsigned long long *__restrict__ pkey,
                                                           const uint64_t *__restrict__ pval,
                                                           const int32_t *__restrict__ prule,
                                                           const uint32_t *__restrict__ rstart, int32_t nranges,
                                                           const ParamEvent *__restrict__ ev, ParamRules PR, PSlots S,
                                                           uint64_t *__restrict__ out, unsigned long long *fresh) {
    __shared__ unsigned long long hkey[PD_HT];
    __shared__ int32_t hrule[PD_HT];
    __shared__ uint16_t cnt[PD_WAVES][PD_HT];
    __shared__ uint32_t hstart[PD_HT + 1];
    __shared__ uint64_t sv[PD_CAP];
    __shared__ uint32_t waves_tot[PD_WAVES];
    __shared__ uint32_t s_fresh;
    const uint32_t p = blockIdx.x;
    if ((int32_t)p >= nranges) return;                                   // block-uniform
    const int wave = threadIdx.x / WAVE;
    const uint32_t lane = lane_id();
    const uint32_t t = threadIdx.x;
    if (t == 0) s_fresh = 0;
    const uint32_t r0 = rstart[p], r1 = rstart[p + 1];
    const int64_t T0 = pp_t0(ev);
    uint32_t nfresh = 0;
    for (uint32_t c0 = r0; c0 < r1; c0 += PD_CAP) {
        const uint32_t csz = min(PD_CAP, r1 - c0);
        // chunk item j of this lane: chunk position wave * PD_ITEMS * 64 + j * 64 + lane (wave-contiguous,
        // so the ballot ranking below keeps arrival order)
        uint32_t pend = 0;                                               // items still to decide (bit j)
#pragma unroll
        for (int j = 0; j < PD_ITEMS; ++j)
            if ((uint32_t)wave * (PD_ITEMS * WAVE) + j * WAVE + lane < csz) pend |= 1u << j;
        for (;;) {                                                       // rounds: keys past a full table wait
            // the pending items (re)loaded each round: nothing but `pend` stays live across the walk
            unsigned long long k[PD_ITEMS];
            uint64_t v[PD_ITEMS];
            int32_t ru[PD_ITEMS];
#pragma unroll
            for (int j = 0; j < PD_ITEMS; ++j) {
                const uint32_t q = c0 + (uint32_t)wave * (PD_ITEMS * WAVE) + j * WAVE + lane;
                if (pend & (1u << j)) {
                    k[j] = pkey[q];
                    v[j] = pval[q];
                    ru[j] = prule[q];
                }
            }
            for (uint32_t e = t; e < PD_HT; e += PD_THREADS) hkey[e] = PKEY_EMPTY;
            {
                uint32_t *z = reinterpret_cast<uint32_t *>(&cnt[0][0]);
                for (uint32_t d = t; d < PD_WAVES * PD_HT / 2; d += PD_THREADS) z[d] = 0;
            }
            __syncthreads();
            int eid[PD_ITEMS];
#pragma unroll
            for (int j = 0; j < PD_ITEMS; ++j) {
                eid[j] = -1;
                if (pend & (1u << j))
                    eid[j] = pd_insert(hkey, hrule, k[j], ru[j], (uint32_t)(mix64(k[j]) >> 32) & (PD_HT - 1));
            }
            __syncthreads();
            uint32_t rank[PD_ITEMS];
#pragma unroll
            for (int j = 0; j < PD_ITEMS; ++j) {
                const bool valid = eid[j] >= 0;
                const uint32_t d = valid ? (uint32_t)eid[j] : 0u;
                const uint64_t peers = match_peers<PD_HBITS>(d, valid, PD_HBITS);
                uint32_t r = 0;
                if (valid) r = cnt[wave][d] + mask_rank(peers);
                __builtin_amdgcn_wave_barrier();
                if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane) cnt[wave][d] += (uint16_t)__popcll(peers);
                __builtin_amdgcn_wave_barrier();
                rank[j] = r;
            }
            __syncthreads();
            // per entry: exclusive over waves in place, then an exclusive scan over entries -> run starts
            uint32_t tot[PD_EPT];
            uint32_t mine = 0;
#pragma unroll
            for (int q = 0; q < PD_EPT; ++q) {
                const uint32_t e = t * PD_EPT + q;
                uint32_t run = 0;
#pragma unroll
                for (int w = 0; w < PD_WAVES; ++w) {
                    const uint32_t x = cnt[w][e];
                    cnt[w][e] = (uint16_t)run;
                    run += x;
                }
                tot[q] = run;
                mine += run;
            }
            uint32_t total;
            uint32_t pre = block_exclusive_scan(mine, waves_tot, &total);
#pragma unroll
            for (int q = 0; q < PD_EPT; ++q) {
                hstart[t * PD_EPT + q] = pre;
                pre += tot[q];
            }
            if (t == 0) hstart[PD_HT] = total;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < PD_ITEMS; ++j) {
                if (eid[j] < 0) continue;
                const uint32_t e = (uint32_t)eid[j];
                sv[hstart[e] + cnt[wave][e] + rank[j]] = v[j];
                pend &= ~(1u << j);
            }
            __syncthreads();
#pragma unroll 1
            for (uint32_t e = t; e < PD_HT; e += PD_THREADS) {
                const uint32_t s0 = hstart[e], s1 = hstart[e + 1];
                if (s1 > s0) pd_walk<NMAX>(PR, S, hkey[e], hrule[e], sv, s0, s1, ev, T0, out, nfresh);
            }
            if (!__syncthreads_or(pend != 0)) break;                     // (also: the walk is done with the LDS)
        }
    }
    block_add_global(fresh, nfresh, &s_fresh);
}

}  // namespace sentinel
