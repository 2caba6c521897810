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
//   k_pp_group    one workgroup per (range, sub-range of 2^sbits): the sub-range's requests (arrival
//                 order) grouped by key in an LDS open-addressing table (the north star's "LDS-staged"
//                 table: a key's HBM slot is probed once per batch, not once per request), ranked
//                 stably with ballots and placed in (key, arrival) order; written out as grouped
//                 values + one record per distinct key
//   k_pp_walk     one lane per distinct key, no LDS: probes / inserts the key's HBM slot, holds the
//                 window in VGPRs, decides the key's requests in arrival order and writes the
//                 verdicts to their arrival positions and the rolled pairs back
//
// Replaces the per-slot radix-sort pipeline (k_param_prep -> 3 radix passes -> k_segments_v ->
// k_process_reg_o4 -> k_verdict): per request it reads the 24-B event twice, moves 20 B through
// the multi-split and writes the 8-B verdict; per distinct key and chunk one table probe, the
// slot's window header and the dirty pairs.
#pragma once

#include <type_traits>

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
// E mod m for an epoch E >= 0 and a small m, by the double reciprocal (epoch_of's method) instead of a
// 64-bit integer division (~120 instructions on gfx950)
__device__ inline uint32_t cm_ring_slot(int64_t E, int m, double rcp_m) {
    return (uint32_t)(E - epoch_of(E, m, rcp_m) * (int64_t)m);
}

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

// A key's run of grouped values read 4 ahead of its walk (a run is walked one request after the other;
// without the look-ahead every request waits for its own load: a hot key's run is a chain of round trips).
// Used by the count-min kernels (walk 1520 -> 1470 us); the exact walk measured no gain (551 vs 574 us).
struct RunQueue {
    const uint64_t *p;
    uint32_t q, end;
    uint64_t b[4];
    __device__ inline RunQueue(const uint64_t *src, uint32_t q0, uint32_t q1) : p(src), q(q0), end(q1) {
#pragma unroll
        for (int k = 0; k < 4; ++k) b[k] = q0 + k < q1 ? p[q0 + k] : 0ull;
    }
    __device__ inline uint64_t next() {                 // the value at q (caller checks q < end), then q + 1
        const uint64_t v = b[0];
        b[0] = b[1];
        b[1] = b[2];
        b[2] = b[3];
        b[3] = q + 4 < end ? p[q + 4] : 0ull;
        ++q;
        return v;
    }
};

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
                                                         uint32_t *__restrict__ hist, int32_t nparts,
                                                         uint32_t *__restrict__ zero_word,
                                                         unsigned long long *__restrict__ tspan,
                                                         uint32_t *__restrict__ oseq = nullptr,
                                                         uint32_t *__restrict__ octr = nullptr, uint32_t opar = 0) {
    // oseq: decide-order output -- rejected requests placed from the end (put_rejected_ordered)
    __shared__ uint32_t h[PART_BINS];
    __shared__ unsigned long long s_span[2];
    if (blockIdx.x == 0 && threadIdx.x == 0 && zero_word) *zero_word = 0;   // the batch's key-record count
    if (blockIdx.x == 0 && threadIdx.x == 0 && octr) octr[opar ^ 1u] = 0;
    if (threadIdx.x == 0) { s_span[0] = ~0ull; s_span[1] = ~0ull; }
    unsigned long long tmin = ~0ull, tnmax = ~0ull;    // this thread's valid requests: min ts, min ~ts
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
        if (st == 127) {
            atomicAdd(&h[pp_digit(mix64(evs[j].key), pbits)], 1u);
            tmin = min(tmin, (unsigned long long)evs[j].ts);                // ts >= 0 here
            tnmax = min(tnmax, ~(unsigned long long)evs[j].ts);
        } else if (!oseq) {
            put_verdict(out, (uint32_t)i, st, 0, 0);
        }
        if (oseq) put_rejected_ordered(st != 127, out, oseq, &octr[opar], n, (uint32_t)i, st);
    }
    if (tspan) {                                          // (block-uniform) the batch's ts range
#pragma unroll
        for (int o = WAVE / 2; o > 0; o >>= 1) {
            tmin = min(tmin, (unsigned long long)__shfl_xor(tmin, o, WAVE));
            tnmax = min(tnmax, (unsigned long long)__shfl_xor(tnmax, o, WAVE));
        }
        if (lane_id() == 0 && tmin != ~0ull) {
            atomicMin(&s_span[0], tmin);
            atomicMin(&s_span[1], tnmax);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < nparts; d += PP_THREADS) hist[(int64_t)blockIdx.x * nparts + d] = h[d];
    if (tspan && threadIdx.x == 0 && s_span[0] != ~0ull) {
        atomicMin(&tspan[0], s_span[0]);
        atomicMin(&tspan[1], s_span[1]);
    }
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
    // dst < n: p - loff[d] < this tile's count of digit d, which equals k_pp_prep's hist entry for (tile, d)
    // -- both kernels tile by PT_TILE (PP_ITEMS = PT_TILE / PP_THREADS) and count exactly the requests with
    // pp_status == 127 (prep's PP_NEG_TS conversion yields BLOCKED / FAIL, never 127) -- so dst lies in
    // [goff[d], goff[d] + hist[tile][d]) inside range d's [rstart[d], rstart[d + 1]) and rstart[P] <= n
    auto write_out = [&](auto put) {
        for (uint32_t p = threadIdx.x; p < total; p += PT_THREADS) {
            const uint32_t d = sdig[p];
            put(goff[d] + p - loff[d], p);
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
#ifndef SENTINEL_PD_HBITS
#define SENTINEL_PD_HBITS 11
#endif
constexpr int PD_THREADS = SENTINEL_PD_THREADS;
constexpr int PD_WAVES = PD_THREADS / WAVE;
#ifndef SENTINEL_PG_ITEMS
#define SENTINEL_PG_ITEMS 5
#endif
constexpr int PG_ITEMS = SENTINEL_PG_ITEMS;
constexpr uint32_t PG_CAP = PD_THREADS * PG_ITEMS;      // requests per chunk
constexpr int PD_HBITS = SENTINEL_PD_HBITS;
constexpr uint32_t PD_HT = 1u << PD_HBITS;              // LDS hash entries per round
constexpr int PD_PROBES = 32;                           // a key not placed within this many probes waits a round
constexpr int PD_EPT = PD_HT / PD_THREADS;               // entries per thread in the scans
static_assert(PD_HT % PD_THREADS == 0, "entries per thread");
static_assert(PG_CAP <= 65535 && PG_CAP < PD_HT, "16-bit wave counters, table larger than a chunk");
static_assert(PD_THREADS * 4 <= (int)PG_CAP, "a scan tile fits an empty chunk");
// requests per range the host aims at (ranges <= PART_BINS), and per sub-range (<= 0.8 PG_CAP)
constexpr int64_t PD_TARGET = 2048;
constexpr int64_t PG_TARGET = PG_CAP * 4 / 5;

// Insert / find a key in the chunk's LDS table; -1: not within PD_PROBES probes (full neighbourhood).
// All requests of one key agree: entries never change once set, so every request of a key that fails
// saw the same PD_PROBES other keys.
template <uint32_t HT = PD_HT>
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
        h = (h + 1) & (HT - 1);
    }
    return -1;
}

// A param rule's window fields and threshold in one 32-byte record (k_prule_pack): a key's walk reads
// one line for its rule instead of five arrays, and looks up the hot-item table only when the rule has
// hot items.
struct PRuleRec {
    double rcp_w;
    double I_s;
    double thr;          // rule count (x connectedCount for AVG_LOCAL)
    int32_t w;
    int32_t nf;          // n | has_hot_items << 16
};
static_assert(sizeof(PRuleRec) == 32, "one record per half line");

__global__ __launch_bounds__(256) void k_prule_pack(int32_t R, ParamRules PR, const uint8_t *__restrict__ hot,
                                                    PRuleRec *__restrict__ rec) {
    const int32_t r = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (r >= R) return;
    rec[r] = PRuleRec{PR.rcp_w[r], PR.I_s[r], PR.thr[r], PR.w[r], PR.n[r] | ((hot && hot[r]) ? 0x10000 : 0)};
}

// One key's requests [q0, q1) of sv (arrival order) against its exact HBM slot: the ClusterParamFlowChecker
// state machine per request (CPFC:58-86 for one value: roll = LeapArray.currentWindow, sum over the valid
// buckets, R = (T_v - sum / I_s) - a, pass iff !(R < 0) -> addValue), the window {epoch, count} x NMAX in
// VGPRs, only the touched pairs written back.  A bucket newer than the request's epoch (the clock went
// backwards for this key) is the detached-bucket case (LeapArray.java:241-246): the sum reads the array,
// the add is lost.
template <int NMAX>
__device__ inline void pd_walk(const ParamRules &PR, const PRuleRec *RR, const PSlots &S, unsigned long long key,
                               int32_t rule, const uint64_t *sv, uint32_t q0, uint32_t q1, const ParamEvent *ev,
                               int64_t T0, uint64_t *out, uint32_t &nfresh, bool ord = false, uint32_t pbase = 0) {
    // (ord: decide-order output, the verdict of sv[q] at out[pbase + q]; else at its arrival position)
    const PRuleRec rr = RR[rule];
    const int nsc = rr.nf & 0xFFFF;
    const int32_t w = rr.w;
    const double rcp = rr.rcp_w;
    const double I_s = rr.I_s;
    const double thr = (rr.nf >> 16) ? value_threshold(PR, (uint32_t)rule, key) : rr.thr;   // CPFC:101-120
    const uint32_t before = nfresh;
    const int64_t h = slot_insert_counted(S.keys, S.mask, key, nfresh);
    if (h < 0) {                                                         // table full: param_reserve prevents it
        for (uint32_t q = q0; q < q1; ++q) put_verdict(out, ord ? pbase + q : (uint32_t)sv[q] & SEQ_MASK, ST_FAIL, 0, 0);
        return;
    }
    const bool fresh = nfresh != before;
    if (fresh) S.rule[h] = rule;                                         // read by the rebuild / top values
    int64_t *st = S.state + h * S.stride;
    int64_t ep[NMAX], ct[NMAX];
    uint32_t dirty = 0;
    if (fresh) {                                                         // (the table's state is not pre-initialised)
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
            ep[j] = EPOCH_ABSENT;
            ct[j] = 0;
            if (j < nsc) dirty |= 1u << j;
        }
    } else {
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {                                 // in bounds: stride >= 2 NMAX words
            const longlong2 v = *reinterpret_cast<const longlong2 *>(st + 2 * j);
            ep[j] = j < nsc ? v.x : EPOCH_ABSENT;
            ct[j] = j < nsc ? v.y : 0;
        }
    }
    const double rcpn = 1.0 / (double)nsc;
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
        store_verdict(out, ord ? pbase + q : (uint32_t)v & SEQ_MASK, vd);
    }
#pragma unroll
    for (int j = 0; j < NMAX; ++j)
        if (dirty & (1u << j)) *reinterpret_cast<longlong2 *>(st + 2 * j) = longlong2{ep[j], ct[j]};
#ifdef SENTINEL_DIAG_NOEXPIRE   // cost diagnostic only (stale top-values hints): no hint store
    if (false) {
#else
    if (S.expire) {                                                      // getTopValues hint (param_table.hpp)
#endif
        int64_t nw = EPOCH_ABSENT;
#pragma unroll
        for (int j = 0; j < NMAX; ++j) nw = j < nsc && ep[j] > nw ? ep[j] : nw;
        S.expire[h] = slot_expire_c(nw, nsc, w);
    }
}

#ifdef SENTINEL_DIAG_PHASES     // per workgroup: [0] start, [3] end, [4..6] phase sums, [7] rounds, [8] keys
#define PD_ACC(i, v) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_phase[blockIdx.x][i] += (v); } while (0)
#define PD_NOW() wall_clock64()
#else
#define PD_ACC(i, v) do { } while (0)
#define PD_NOW() 0ull
#endif

// Sub-range of a param key inside its range: the sbits hash bits right below the range digit.
__device__ inline uint32_t pp_sub(uint64_t h, int pbits, int sbits) {
    return sbits ? (uint32_t)((h << pbits) >> (64 - sbits)) : 0u;
}

// Per-key records the grouping kernel hands to the walk kernel: the key, its rule, and its requests'
// run [start, start + count) in the grouped value array (arrival order inside the run).
struct PKeyRecs {
    unsigned long long *key;
    uint2 *run;              // {start, count}
    int32_t *rule;
    uint32_t *count;         // records written (zeroed by k_pp_prep)
    unsigned long long *overflow;   // shared count-min: set when a sub-range exceeds one chunk (else null)
    // shared count-min block walk (k_pp_cm_block): non-null = each sub-range's records are written at
    // their sub-range's first grouped-value position, sub[(range << sbits) | sub-range] = {first, count}
    uint2 *sub = nullptr;
    // decide-order output (sentinel_submit_param_batch_ordered): the verdict of the request at grouped
    // position q goes to out[q] and its arrival position to oseq[q] (written by k_pp_group with the
    // grouped values); null: out[arrival position]
    uint32_t *oseq = nullptr;
};

// k_pp_group: one workgroup per (range, sub-range): the S = 2^sbits workgroups of a range read the
// range's keys (one L2-resident pass each: they share blockIdx % 8, hence an XCD, and are dispatched
// together) and each keeps its sub-range's requests, compacted in arrival order (positions only, in
// LDS).  A sub-range that fits one chunk (PG_CAP requests: the common case, the host sizes S for it)
// is grouped by key in the LDS table -- distinct keys ranked stably with per-wave ballots, runs placed
// in (key, arrival) order -- and written out as one coalesced run of grouped values plus one record per
// distinct key; k_pp_walk decides the keys.  A larger sub-range (a skewed batch) is decided here, chunk
// after chunk in arrival order, one lane per distinct key of the chunk (a key spanning chunks is walked
// once per chunk, in order).
// HB: bits of the LDS key table (the count-min grouping, which only emits, uses a 1024-entry table: 40 KB of
// LDS, 2x the workgroups per CU; a chunk with more distinct keys than the table takes more rounds)
template <int NMAX, bool CM = false, int HB = PD_HBITS>
__global__ __launch_bounds__(PD_THREADS) void k_pp_group(const unsigned long long *__restrict__ pkey,
                                                          const uint64_t *__restrict__ pval,
                                                          const int32_t *__restrict__ prule,
                                                          const uint32_t *__restrict__ rstart, int32_t nranges,
                                                          int pbits, int sbits, const ParamEvent *__restrict__ ev,
                                                          ParamRules PR, const PRuleRec *__restrict__ RR, PSlots S,
                                                          uint64_t *__restrict__ out, unsigned long long *fresh,
                                                          uint64_t *__restrict__ gval, PKeyRecs RC) {
    constexpr uint32_t HT = 1u << HB;
    constexpr int EPT = HT / PD_THREADS;
    static_assert(HT % PD_THREADS == 0 && HT <= 65536, "entries per thread, 16-bit key list");
    __shared__ uint32_t cq[PG_CAP];                   // the chunk's requests: positions in pkey / pval / prule
    __shared__ uint64_t sv[PG_CAP];                   // grouped values
    __shared__ unsigned long long hkey[HT];
    __shared__ int32_t hrule[HT];
    __shared__ uint16_t cnt[PD_WAVES][HT];
    __shared__ uint32_t hstart[HT + 1];
    __shared__ uint32_t waves_tot[PD_WAVES];
    __shared__ uint32_t s_fresh, s_rbase;
    const uint32_t nsub = 1u << sbits;
    const uint32_t b = blockIdx.x;
    const uint32_t p = (b / (8u * nsub)) * 8u + b % 8u;
    const uint32_t sub = (b / 8u) % nsub;
    if ((int32_t)p >= nranges) return;                                   // block-uniform
    const int wave = threadIdx.x / WAVE;
    const uint32_t lane = lane_id();
    const uint32_t t = threadIdx.x;
    if (t == 0) s_fresh = 0;
    const uint32_t r0 = rstart[p], r1 = rstart[p + 1];
    const int64_t T0 = pp_t0(ev);
    uint32_t nfresh = 0;
    uint32_t below = 0;                                                  // this thread's requests of lower sub-ranges
    bool slow = false;                                                   // a chunk was decided before the scan ended
    uint32_t m = 0;                                                      // compacted requests (block-uniform)
    uint32_t kemit = 0;                                                  // records emitted (block-uniform)
    uint32_t kbase = 0;
    uint32_t sbase = 0, soff = 0;                                        // decide order, slow sub-range: its first
                                                                         // position, requests decided so far
    PF_STAMP(0);

    // decide / emit cq[0, m): rounds while the LDS table is full for some key
    auto chunk = [&](bool emit, uint32_t gbase) {
        uint32_t pend = 0;
#pragma unroll
        for (int j = 0; j < PG_ITEMS; ++j)
            if ((uint32_t)wave * (PG_ITEMS * WAVE) + j * WAVE + lane < m) pend |= 1u << j;
        uint32_t roff = 0;                                               // grouped values emitted by earlier rounds
        for (;;) {
            [[maybe_unused]] const unsigned long long pt0 = PD_NOW();
            unsigned long long k[PG_ITEMS];
            uint64_t v[PG_ITEMS];
            int32_t ru[PG_ITEMS];
#pragma unroll
            for (int j = 0; j < PG_ITEMS; ++j) {
                if (pend & (1u << j)) {
                    const uint32_t q = cq[(uint32_t)wave * (PG_ITEMS * WAVE) + j * WAVE + lane];
                    k[j] = pkey[q];
                    v[j] = pval[q];
                    ru[j] = prule[q];
                }
            }
            for (uint32_t e = t; e < HT; e += PD_THREADS) hkey[e] = PKEY_EMPTY;
            {
                uint32_t *z = reinterpret_cast<uint32_t *>(&cnt[0][0]);
                for (uint32_t d = t; d < PD_WAVES * HT / 2; d += PD_THREADS) z[d] = 0;
            }
            __syncthreads();
            int eid[PG_ITEMS];
#pragma unroll
            for (int j = 0; j < PG_ITEMS; ++j) {
                eid[j] = -1;
                if (pend & (1u << j))
                    eid[j] = pd_insert<HT>(hkey, hrule, k[j], ru[j], (uint32_t)(mix64(k[j]) >> 32) & (HT - 1));
            }
            __syncthreads();
            [[maybe_unused]] const unsigned long long pt1 = PD_NOW();
            uint32_t rank[PG_ITEMS];
#pragma unroll
            for (int j = 0; j < PG_ITEMS; ++j) {
                const bool valid = eid[j] >= 0;
                const uint32_t d = valid ? (uint32_t)eid[j] : 0u;
                const uint64_t peers = match_peers<HB>(d, valid, HB);
                uint32_t r = 0;
                if (valid) r = cnt[wave][d] + mask_rank(peers);
                __builtin_amdgcn_wave_barrier();
                if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane) cnt[wave][d] += (uint16_t)__popcll(peers);
                __builtin_amdgcn_wave_barrier();
                rank[j] = r;
            }
            __syncthreads();
            // per entry: exclusive over waves in place, then one exclusive scan over entries of
            // {requests : 16 | distinct keys : 16} -> run starts and each key's place in the key list
            uint32_t tot[EPT];
            uint32_t mine = 0;
#pragma unroll
            for (int q = 0; q < EPT; ++q) {
                const uint32_t e = t * EPT + q;
                uint32_t run = 0;
#pragma unroll
                for (int w = 0; w < PD_WAVES; ++w) {
                    const uint32_t x = cnt[w][e];
                    cnt[w][e] = (uint16_t)run;
                    run += x;
                }
                tot[q] = run;
                mine += run | (run ? 0x10000u : 0u);
            }
            uint32_t total;
            uint32_t pre = block_exclusive_scan(mine, waves_tot, &total);
            uint32_t kpos = pre >> 16;
            pre &= 0xFFFFu;
#pragma unroll
            for (int q = 0; q < EPT; ++q) {
                hstart[t * EPT + q] = pre;
                pre += tot[q];
            }
            const uint32_t nkeys = total >> 16;
            const uint32_t placed = total & 0xFFFFu;
            if (t == 0) hstart[HT] = placed;
            if (emit && t == 0 && !RC.sub) s_rbase = atomicAdd(RC.count, nkeys);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < PG_ITEMS; ++j) {
                if (eid[j] < 0) continue;
                const uint32_t e = (uint32_t)eid[j];
                sv[hstart[e] + cnt[wave][e] + rank[j]] = v[j];
                pend &= ~(1u << j);
            }
            __syncthreads();
            // the distinct keys listed densely (over the wave counters, free now)
            uint16_t *klist = &cnt[0][0];
#pragma unroll
            for (int q = 0; q < EPT; ++q)
                if (tot[q]) klist[kpos++] = (uint16_t)(t * EPT + q);
            __syncthreads();
            [[maybe_unused]] const unsigned long long pt2 = PD_NOW();
            if (emit) {
                for (uint32_t i = t; i < placed; i += PD_THREADS) {
                    gval[gbase + roff + i] = sv[i];
                    if (RC.oseq) RC.oseq[gbase + roff + i] = (uint32_t)sv[i] & SEQ_MASK;   // (decide order)
                }
                const uint32_t rb = RC.sub ? gbase + kemit : s_rbase;      // (records <= requests: inside the run)
                kbase = gbase;
                for (uint32_t q = t; q < nkeys; q += PD_THREADS) {
                    const uint32_t e = klist[q];
                    RC.key[rb + q] = hkey[e];
                    RC.run[rb + q] = make_uint2(gbase + roff + hstart[e], hstart[e + 1] - hstart[e]);
                    RC.rule[rb + q] = hrule[e];
                }
            } else if constexpr (!CM) {
                // (decide order: this round's requests own positions gbase + roff + [0, placed))
                if (RC.oseq)
                    for (uint32_t i = t; i < placed; i += PD_THREADS) RC.oseq[gbase + roff + i] = (uint32_t)sv[i] & SEQ_MASK;
#pragma unroll 1
                for (uint32_t q = t; q < nkeys; q += PD_THREADS) {
                    const uint32_t e = klist[q];
                    pd_walk<NMAX>(PR, RR, S, hkey[e], hrule[e], sv, hstart[e], hstart[e + 1], ev, T0, out, nfresh,
                                  RC.oseq != nullptr, gbase + roff);
                }
            }
            roff += placed;
            if (emit) kemit += nkeys;
            const int more = __syncthreads_or(pend != 0);                // (also: done with the LDS)
            [[maybe_unused]] const unsigned long long pt3 = PD_NOW();
            PD_ACC(4, pt1 - pt0);
            PD_ACC(5, pt2 - pt1);
            PD_ACC(6, pt3 - pt2);
            PD_ACC(7, 1ull);
            PD_ACC(8, (unsigned long long)nkeys);
            if (!more) break;
        }
    };

    // scan the range in tiles of PD_THREADS x 4 keys (4 consecutive keys per thread: the compaction
    // below keeps arrival order), keep this sub-range's positions
    for (uint32_t q0 = r0; q0 < r1; q0 += PD_THREADS * 4) {
        const uint32_t qa = q0 + t * 4;
        uint32_t mk = 0;                                                 // bit i: key qa + i is ours
        if (qa + 4 <= r1 && (qa & 1u) == 0) {
            const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(pkey + qa);
            const ulonglong2 c = *reinterpret_cast<const ulonglong2 *>(pkey + qa + 2);
            const unsigned long long kk[4] = {a.x, a.y, c.x, c.y};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t sd = pp_sub(mix64(kk[i]), pbits, sbits);
                mk |= (sd == sub ? 1u : 0u) << i;
                below += sd < sub;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (qa + i >= r1) break;
                const uint32_t sd = pp_sub(mix64(pkey[qa + i]), pbits, sbits);
                mk |= (sd == sub ? 1u : 0u) << i;
                below += sd < sub;
            }
        }
        uint32_t tile_n;
        const uint32_t off = block_exclusive_scan((uint32_t)__popc(mk), waves_tot, &tile_n);
        if (m + tile_n > PG_CAP) {                                       // the chunk is full: decide it now
            if (CM) {                          // (block-uniform) the key walk needs one run per key: the host
                if (t == 0) atomicOr(RC.overflow, 1ull);              // falls back to the per-rule lanes
                return;
            }
            if (RC.oseq && !slow) {
                // decide-order output: the sub-range owns grouped positions r0 + (the range's requests of
                // lower sub-ranges) + [0, its size) -- `below` covers the tiles up to this one, the rest of
                // the range is counted here (only a sub-range over one chunk pays this second read)
                uint32_t rest = 0;
                for (uint32_t qq = q0 + PD_THREADS * 4 + t; qq < r1; qq += PD_THREADS)
                    rest += pp_sub(mix64(pkey[qq]), pbits, sbits) < sub;
                uint32_t tot;
                (void)block_exclusive_scan(below + rest, waves_tot, &tot);
                sbase = r0 + tot;
            }
            slow = true;
            chunk(false, sbase + soff);
            soff += m;
            m = 0;
        }
        uint32_t w = m + off;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (mk & (1u << i)) cq[w++] = qa + i;
        m += tile_n;
        __syncthreads();
    }
    if (m) {
        if (slow) {
            chunk(false, sbase + soff);
        } else {
            uint32_t nb;
            const uint32_t base = block_exclusive_scan(below, waves_tot, &nb);   // (only the total is used)
            (void)base;
            chunk(true, r0 + nb);
        }
    }
    if (RC.sub && t == 0) RC.sub[(p << sbits) | sub] = make_uint2(kbase, kemit);
    PF_STAMP(3);
    block_add_global(fresh, nfresh, &s_fresh);
}

// The exact param table's fresh-insert count after batch `ord`, mirrored to pinned host memory (value
// first, then the ordinal: a host that reads the ordinal and then the value sees a count at least as
// new as that batch's -- the count only grows until the host resets it with the stream drained).
// One wave: lane l reads counter lane l (all loads in flight at once), a wave sum, lane 0 publishes.
__global__ __launch_bounds__(WAVE) void k_pfresh_publish(const unsigned long long *fresh, unsigned long long ord,
                                                         unsigned long long *host) {
    static_assert(CNT_LANES == WAVE, "one counter lane per lane of the wave");
    unsigned long long f = *(volatile const unsigned long long *)(fresh + threadIdx.x * CNT_STRIDE);
#pragma unroll
    for (int o = WAVE / 2; o >= 1; o >>= 1) f += __shfl_xor(f, o, WAVE);
    if (threadIdx.x != 0) return;
    __hip_atomic_store(&host[1], f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(&host[0], ord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// k_pp_walk: one lane per distinct key of the grouped sub-ranges (PKeyRecs), no LDS, register-lean
// so that several waves per SIMD hide the key's memory round trips (slot probe / insert, window, rule
// fields): the ClusterParamFlowChecker state machine over the key's run (pd_walk).
template <int NMAX>
__global__ __launch_bounds__(256) void k_pp_walk(PKeyRecs RC, const uint64_t *__restrict__ gval,
                                                  const ParamEvent *__restrict__ ev, ParamRules PR,
                                                  const PRuleRec *__restrict__ RR, PSlots S,
                                                  uint64_t *__restrict__ out, unsigned long long *fresh) {
    __shared__ uint32_t s_fresh;
    if (threadIdx.x == 0) s_fresh = 0;
    __syncthreads();
    const uint32_t nrec = *RC.count;
    const int64_t T0 = pp_t0(ev);
    uint32_t nfresh = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nrec; i += gridDim.x * blockDim.x) {
        const uint2 run = RC.run[i];
        pd_walk<NMAX>(PR, RR, S, RC.key[i], RC.rule[i], gval, run.x, run.x + run.y, ev, T0, out, nfresh,
                      RC.oseq != nullptr, 0);
    }
    block_add_global(fresh, nfresh, &s_fresh);
}

// ---------------------------------------------------------------- shared count-min, key-parallel
// Shared count-min sketch (SENTINEL_PARAM_COUNT_MIN_SHARED) on the grouped keys: one lane per distinct
// (rule, value) key instead of one lane per rule, in two phases per batch.
//
//   k_pp_cm_read  every key's requests whose window can still hold counts of earlier batches (epoch
//                 E < E_hi + n, E_hi = the newest epoch any earlier batch added) get
//                 M(E) = min over the d rows of the cell's window sum, from the cells as the earlier
//                 batches left them (nothing of this batch has been added yet: kernel boundary)
//   k_pp_cm_walk  one lane per key walks its requests in arrival order with the key's own admitted
//                 counts of this batch in a register window ({epoch, count} x n, as the exact walk):
//                 est = M(E) + own window sum, R = (T_v - est / I_s) - a, pass iff !(R < 0)
//                 (cm_check_sync for one value); each own epoch's count is added to the key's d cells
//                 when it leaves the register window or the walk ends
//
// est >= the key's exact window count (its earlier-batch counts are in every row's cell, its own
// counts of this batch are in the register window), so the sketch stays one-sided; other keys' counts
// of this batch are not seen (fewer false blocks than a sequential sketch).  Because every read of the
// batch precedes every add, a ring-slot reset by an add (epoch E' restarting the slot of E' - 2n) can
// no longer remove a count somebody still reads: no bands, no grid barriers, and a batch's verdicts
// depend only on the cells as the earlier batches left them (the adds' order only decides which epoch
// a colliding slot is tagged with when two keys' epochs 2n apart meet in it; the count is kept either
// way).  Precondition, as for the per-rule lanes: the requests' clock does not go back across batches
// (the server's one clock: TimeUtil.currentTimeMillis).
constexpr int64_t CM_EHI_NONE = INT64_MIN;       // no earlier batch added anything (cleared cells)
constexpr int64_t CM_EHI_ANY = INT64_MAX;        // unknown (the per-rule lanes ran): always read

// The reference epoch of a batch's tag arithmetic: its newest request's epoch, or E_hi when that is later.
// Every slot of the shared sketch holds an epoch <= E_hi (every writer advances E_hi past its adds:
// k_pp_cm_ehi after the key walks, the per-rule lanes before theirs), so every slot a batch loads lies at
// or before Eref, and its age Eref - epoch is exact modulo the tag width (2^24 in HBM, 2^8 in the block
// walk's 32-bit LDS cells, which the host takes only while every age the batch needs is < 256).
__device__ inline int64_t cm_eref(int64_t ebatch, int64_t ehi) {
    return (ehi != CM_EHI_NONE && ehi != CM_EHI_ANY && ehi > ebatch) ? ehi : ebatch;
}

// min over the d rows of the cell's window sum at E, reading only the ring slots of the epochs
// (E - n, E]: n / 2 + 1 aligned 16-byte pairs (contiguous modulo the ring: one or two lines per row
// instead of the whole 2 n ring; the one or two extra slots hold epochs outside the window and fail
// the tag test), every row's loads in flight at once.  Plain loads: nothing of this batch has been
// added yet.
template <int NMAX, int DMAX>
__device__ inline int64_t cm_window_min(const CountMin &CM, unsigned long long key, int nsc, int64_t E) {
    constexpr int DR = DMAX < 4 ? DMAX : 4;               // rows per round
    constexpr int NP = NMAX / 2 + 1;                      // pairs per row, at most
    const int np = nsc / 2 + 1 < nsc ? nsc / 2 + 1 : nsc; // (the ring holds nsc pairs)
    const int first = (int)cm_ring_slot(E + 1 + nsc, 2 * nsc, 0.5 / (double)nsc);   // slot of epoch E - n + 1
    const int p0 = first >> 1;
    int64_t m = INT64_MAX;
    for (int d0 = 0; d0 < CM.depth; d0 += DR) {
        ulonglong2 x[DR][NP];
#pragma unroll
        for (int r = 0; r < DR; ++r) {
            const bool on = d0 + r < CM.depth;
            const ulonglong2 *c = reinterpret_cast<const ulonglong2 *>(on ? cm_cell(CM, 0, d0 + r, key) : CM.cells);
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                int pk = p0 + k;
                pk = pk >= nsc ? pk - nsc : pk;
                x[r][k] = (on && k < np) ? c[pk] : make_ulonglong2(0ull, 0ull);
            }
        }
#pragma unroll
        for (int r = 0; r < DR; ++r) {
            if (d0 + r >= CM.depth) break;
            int64_t sum = 0;
#pragma unroll
            for (int k = 0; k < NP; ++k) {
                if (k >= np) break;
                const uint32_t ta = (uint32_t)(x[r][k].x >> CM_COUNT_BITS), tb = (uint32_t)(x[r][k].y >> CM_COUNT_BITS);
                if ((((uint32_t)E - ta) & CM_TAG_MASK) < (uint32_t)nsc) sum += (int64_t)(x[r][k].x & CM_COUNT_MAX);
                if ((((uint32_t)E - tb) & CM_TAG_MASK) < (uint32_t)nsc) sum += (int64_t)(x[r][k].y & CM_COUNT_MAX);
            }
            m = sum < m ? sum : m;
        }
    }
    return m;
}

__device__ inline bool cm_needs_read(int64_t E, int64_t ehi, int nsc) {
    if (ehi == CM_EHI_NONE) return false;
    if (ehi == CM_EHI_ANY) return true;
    return E < ehi + nsc;
}

// ctl: [0] E_hi (newest epoch added by earlier batches), [1] E_hi as this batch's read saw it,
// [2] this batch's newest request epoch (atomicMax by the walk)
template <int NMAX, int DMAX>
__global__ __launch_bounds__(256) void k_pp_cm_read(PKeyRecs RC, const uint64_t *__restrict__ gval,
                                                     const ParamEvent *__restrict__ ev,
                                                     const PRuleRec *__restrict__ RR, CountMin CM,
                                                     int64_t *__restrict__ mv, long long *__restrict__ ctl) {
    const int64_t T0 = pp_t0(ev);
    const int64_t ehi = ctl[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctl[1] = ehi;
        ctl[2] = CM_EHI_NONE;
    }
    if (ehi == CM_EHI_NONE) return;                       // (grid-uniform) nothing to read
    const uint32_t nrec = *RC.count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nrec; i += gridDim.x * blockDim.x) {
        const uint2 run = RC.run[i];
        const PRuleRec rr = RR[RC.rule[i]];
        const int nsc = rr.nf & 0xFFFF;
        const unsigned long long key = RC.key[i];
        int64_t lastE = 0, lastM = 0;
        bool have = false;
        RunQueue rq(gval, run.x, run.x + run.y);
#pragma unroll 1
        for (uint32_t q = run.x; q < run.x + run.y; ++q) {
            int64_t t;
            int32_t a;
            pp_unpack(rq.next(), T0, ev, t, a);
            const int64_t E = epoch_of(t, rr.w, rr.rcp_w);
#ifdef SENTINEL_DIAG_CM_BREAK                             // cost diagnostic only (assumes monotone runs)
            if (!cm_needs_read(E, ehi, nsc)) break;
#endif
            if (!cm_needs_read(E, ehi, nsc)) continue;
            if (!have || E != lastE) {
#ifdef SENTINEL_DIAG_CM_NOREAD                            // cost diagnostic only (wrong estimates)
                int64_t m = 0;
#else
                int64_t m = INT64_MAX;
#endif
#ifndef SENTINEL_DIAG_CM_NOREAD
                m = cm_window_min<NMAX, DMAX>(CM, key, nsc, E);
#endif
                lastE = E;
                lastM = m;
                have = true;
            }
            mv[q] = lastM;
        }
    }
}

template <int DMAX>
__device__ inline void cm_flush(const CountMin &CM, unsigned long long key, int nsc, int64_t E, int64_t Eref, int64_t a) {
#ifdef SENTINEL_DIAG_CM_NOADD                             // cost diagnostic only (wrong counters)
    return;
#endif
    const int js = (int)cm_ring_slot(E, 2 * nsc, 0.5 / (double)nsc);
    const CmTag te = cm_tag(E, Eref);
    unsigned long long *c[DMAX];
    unsigned long long x[DMAX], p[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {                      // every row's guess loaded at once
        if (d >= CM.depth) break;
        c[d] = reinterpret_cast<unsigned long long *>(cm_cell(CM, 0, d, key) + js);
        x[d] = *c[d];                                     // a plain load as the CAS's guess (atomics run at the
    }                                                     // memory side: one CAS instead of a failed one + retry)
#pragma unroll
    for (int d = 0; d < DMAX; ++d)                        // every row's first CAS in flight at once
        if (d < CM.depth) p[d] = atomicCAS(c[d], x[d], cm_slot_next(x[d], te, a));
#pragma unroll
    for (int d = 0; d < DMAX; ++d)                        // a lost CAS retries from the value it returned
        if (d < CM.depth && p[d] != x[d]) cm_slot_add(c[d], p[d], te, a);
}

template <int NMAX, int DMAX>
__global__ __launch_bounds__(256) void k_pp_cm_walk(PKeyRecs RC, const uint64_t *__restrict__ gval,
                                                     const ParamEvent *__restrict__ ev, ParamRules PR,
                                                     const PRuleRec *__restrict__ RR, CountMin CM,
                                                     const int64_t *__restrict__ mv, long long *__restrict__ ctl,
                                                     const unsigned long long *__restrict__ tspan,
                                                     uint64_t *__restrict__ out) {
    const int64_t T0 = pp_t0(ev);
    const int64_t ehi = ctl[1];
    const int64_t tmax = (int64_t)~tspan[1];              // the batch's newest request (k_pp_prep)
    int64_t emax = CM_EHI_NONE;
    const uint32_t nrec = *RC.count;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nrec; i += gridDim.x * blockDim.x) {
        const uint2 run = RC.run[i];
        const int32_t rule = RC.rule[i];
        const PRuleRec rr = RR[rule];
        const int nsc = rr.nf & 0xFFFF;
        const unsigned long long key = RC.key[i];
        const double thr = (rr.nf >> 16) ? value_threshold(PR, (uint32_t)rule, key) : rr.thr;   // CPFC:101-120
        const double rcpn = 1.0 / (double)nsc;
        // an epoch 2n older than the batch's newest request is in no window of a request within n epochs
        // of the batch's end (the ring drops it for the next such epoch anyway): its adds are skipped
        const int64_t Enew = epoch_of(tmax, rr.w, rr.rcp_w);
        const int64_t Edead = Enew - 2 * (int64_t)nsc;
        const int64_t Eref = cm_eref(Enew, ehi);         // (cm_slot_next's "newer" test)
        int64_t ep[NMAX], ct[NMAX];                       // this batch's own admitted counts per epoch
#pragma unroll
        for (int j = 0; j < NMAX; ++j) { ep[j] = EPOCH_ABSENT; ct[j] = 0; }
        int64_t curE = EPOCH_ABSENT, own = 0;
        int slot = 0;
        RunQueue rq(gval, run.x, run.x + run.y);
#pragma unroll 1
        for (uint32_t q = run.x; q < run.x + run.y; ++q) {
            const uint64_t v = rq.next();
            int64_t t;
            int32_t a;
            pp_unpack(v, T0, ev, t, a);
            const int64_t E = epoch_of(t, rr.w, rr.rcp_w);
            emax = E > emax ? E : emax;
            const bool late = curE != EPOCH_ABSENT && E < curE;   // (outside the precondition)
            int64_t mine = own;
            if (late) {                                   // every own count that may be in its window (and newer:
                mine = 0;                                 // over-counts, never under); its add goes to curE's slot
#pragma unroll
                for (int j = 0; j < NMAX; ++j)
                    if (ep[j] != EPOCH_ABSENT && ep[j] > E - nsc) mine += ct[j];
            } else if (E != curE) {
                curE = E;
                slot = (int)(E - epoch_of(E, nsc, rcpn) * nsc);
#pragma unroll
                for (int j = 0; j < NMAX; ++j) {
                    if (j != slot || ep[j] == E) continue;
                    if (ct[j] > 0 && ep[j] > Edead) cm_flush<DMAX>(CM, key, nsc, ep[j], Eref, ct[j]);   // leaves the register window
                    ep[j] = E;
                    ct[j] = 0;
                }
                own = 0;                                  // own counts inside the window (E - n, E]
#pragma unroll
                for (int j = 0; j < NMAX; ++j)
                    if (ep[j] != EPOCH_ABSENT && ep[j] > E - nsc) own += ct[j];
                mine = own;
            }
            const int64_t m = cm_needs_read(E, ehi, nsc) ? mv[q] : 0;
            const double next = remaining_of(thr, rr.I_s, m + mine, a);
            uint64_t vd;
            if (!(next < 0.0)) {                                          // CPFC:64-66, then addValue
#pragma unroll
                for (int j = 0; j < NMAX; ++j)
                    if (j == slot) ct[j] += a;
                own += a;
                vd = pack_verdict(ST_OK, java_d2i(next), 0);
            } else {
                vd = pack_verdict(ST_BLOCKED, 0, 0);
            }
            store_verdict(out, RC.oseq ? q : (uint32_t)v & SEQ_MASK, vd);
        }
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (ct[j] > 0 && ep[j] > Edead) cm_flush<DMAX>(CM, key, nsc, ep[j], Eref, ct[j]);
    }
    // the batch's newest epoch -> E_hi for the next batch's reads (ctl[0] is read by k_pp_cm_read only)
    for (int o = WAVE / 2; o > 0; o >>= 1) {
        const int64_t y = __shfl_xor(emax, o, WAVE);
        emax = y > emax ? y : emax;
    }
    if (lane_id() == 0 && emax != CM_EHI_NONE) atomicMax(reinterpret_cast<long long *>(&ctl[2]), (long long)emax);
}

// ---------------------------------------------------------------- shared count-min, block-owned
// k_pp_cm_block (round 5): the two phases above in one launch, one 256-thread workgroup per sketch
// block.  Every cell of a key lies in its block (cm_cell: block = top cbits bits of mix64(key), the bits
// the partition groups requests by), so a block's cells -- depth x cols x 2n slots, 40 KB at d = 4,
// n = 10 -- are read from HBM once (one coalesced stream), staged in LDS, and the slots the batch added
// to are written back: no memory-side atomic (a 128-B line read + a 64-B write) per row, key and
// admitted epoch.  Inside the workgroup the phases are those of k_pp_cm_read / k_pp_cm_walk:
//   A  every key's requests within n epochs of E_hi get M(E) = min over rows of the window sum, from
//      the block as the earlier batches left it;
//   B  (barrier: every read precedes every add) each key walks its requests with its own admitted
//      counts in registers, and adds each epoch's count to its d cells with LDS CAS (cm_slot_add's ring
//      semantics); keys of one block only meet in LDS.
// The block's keys: the sub-range(s) whose top (pbits + sbits) hash bits it covers (records written at
// deterministic positions by k_pp_group, RC.sub); when a sub-range is wider than a block, the block's
// workgroup filters the sub-range's keys by block.  One-sidedness is unchanged.
constexpr int CMB_DMAX = 4;                // rows of a block walk (the host checks depth <= 4)

// a key's d cells in the LDS block: word offsets of slot 0 (computed once per key)
__device__ inline void cm_lds_cells(uint32_t *co, int depth, int nmax, uint32_t cols, unsigned long long key) {
#pragma unroll
    for (int d = 0; d < CMB_DMAX; ++d) {
        if (d >= depth) break;
        const uint32_t col = (uint32_t)mix64(key + 0x9E3779B97F4A7C15ull * (uint64_t)(d + 1)) & (cols - 1);
        co[d] = ((uint32_t)d * cols + col) * (uint32_t)nmax;
    }
}

__device__ inline int64_t cm_lds_window_min(const unsigned long long *cl, const uint32_t *co, int depth, int nmax,
                                            double rcp_nmax, int nsc, int64_t E) {
    int64_t m = INT64_MAX;
    const int js0 = (int)cm_ring_slot(E, nmax, rcp_nmax);
#pragma unroll
    for (int d = 0; d < CMB_DMAX; ++d) {
        if (d >= depth) break;
        const unsigned long long *c = cl + co[d];
        int64_t sum = 0;
        int js = js0;
        for (int k = 0; k < nsc; ++k) {                   // the window's slots: epochs E .. E - n + 1
            const uint64_t x = c[js];
            if ((((uint32_t)E - (uint32_t)(x >> CM_COUNT_BITS)) & CM_TAG_MASK) < (uint32_t)nsc) sum += (int64_t)(x & CM_COUNT_MAX);
            js = js == 0 ? nmax - 1 : js - 1;
        }
        m = sum < m ? sum : m;
    }
    return m;
}

// Add a to the slot of E in the key's d cells: every row's slot read at once; a slot already on E (or on
// a newer epoch: cm_slot_add adds there too) takes a plain LDS add -- no return, no wait -- and only a
// slot that restarts at E (an older tag) needs the compare-and-swap.  An add racing with a restart to a
// newer epoch lands in the newer epoch's count (over, never under); a count within 2^39 of saturation
// takes the CAS (saturating) path.
__device__ inline void cm_lds_flush(unsigned long long *cl, unsigned long long *dirty, const uint32_t *co, int depth,
                                    int nmax, double rcp_nmax, int64_t E, int64_t Eref, int64_t a) {
    const uint32_t js = cm_ring_slot(E, nmax, rcp_nmax);
    const CmTag te = cm_tag(E, Eref);
    unsigned long long x[CMB_DMAX];
#pragma unroll
    for (int d = 0; d < CMB_DMAX; ++d)
        if (d < depth) x[d] = cl[co[d] + js];
#pragma unroll
    for (int d = 0; d < CMB_DMAX; ++d) {
        if (d >= depth) break;
        const uint32_t w = co[d] + js;
        atomicOr(&dirty[w >> 6], 1ull << (w & 63));       // (written back at the end)
        unsigned long long *c = cl + w;
        const uint32_t tag = (uint32_t)(x[d] >> CM_COUNT_BITS);
        const uint64_t cnt = x[d] & CM_COUNT_MAX;
        const bool newer = cnt != 0 && ((te.eref - tag) & CM_TAG_MASK) < te.dE;   // (cm_slot_next)
        if ((tag == te.te || newer) && cnt < (CM_COUNT_MAX >> 1) && (uint64_t)a < (CM_COUNT_MAX >> 1))
            atomicAdd(c, (unsigned long long)a);          // (ds_add_u64)
        else
            cm_slot_add(c, x[d], te, a);                  // (ds_cmpst_rtn_b64)
    }
}

// 32-bit LDS cells (k_pp_cm_block<true>): {tag : 8 = epoch mod 256, count : 24, saturating}, relative to
// the reference epoch Eref = max(the batch's newest epoch, E_hi) (cm_eref: no slot holds a later epoch).
// Loaded from the 64-bit HBM slots: a slot more than 255 epochs older than Eref is no window's (the host
// takes this path only while the batch's oldest epoch, less 2n, is within 200 epochs of Eref) and loads
// empty; a count at or past 2^24 - 1 loads saturated, and a saturated count reads as "at least 2^40"
// (over, never under).  Every other slot's age Eref - epoch is exact in 8 bits, so "the slot holds an
// epoch newer than E" is age(slot) < Eref - E (cm32_next), never a half-range guess.  Written back only
// where the batch added, the full tag rebuilt from Eref, a saturated count as CM_COUNT_MAX.  Half the LDS
// of the 64-bit cells: 5 workgroups per CU instead of 3 (the walk is latency-bound: 2 / 1 workgroups per
// CU measured 1.4x / 2.6x).
constexpr uint32_t CM32_SAT = 0xFFFFFFu;

__device__ inline uint32_t cm32_load(unsigned long long x, int64_t Eref) {
    const uint64_t cnt = x & CM_COUNT_MAX;
    if (cnt == 0) return 0u;
    const uint32_t tag = (uint32_t)(x >> CM_COUNT_BITS);
    const uint32_t d = ((uint32_t)Eref - tag) & CM_TAG_MASK;       // epochs the slot lies before Eref
    if (d > 255) return 0u;                                         // in no window of this batch
    return (tag & 0xFFu) << 24 | (uint32_t)(cnt < CM32_SAT ? cnt : CM32_SAT);
}

// (a written slot's epoch lies in [Eref - 255, Eref] whether it kept its loaded epoch -- loaded slots
// outside that range are empty -- or restarted at an epoch of this batch)
__device__ inline unsigned long long cm32_store(uint32_t v, int64_t Eref) {
    const uint32_t tag8 = v >> 24, cnt = v & CM32_SAT;
    const uint64_t c64 = cnt == CM32_SAT ? CM_COUNT_MAX : (uint64_t)cnt;
    const uint32_t tag = ((uint32_t)Eref - (((uint32_t)Eref - tag8) & 0xFFu)) & CM_TAG_MASK;
    return (unsigned long long)tag << CM_COUNT_BITS | c64;
}

// Add a to a slot for epoch E, dE = Eref - E < 256: same epoch -> add; an epoch newer than E (age < dE:
// another key of the block reached a later epoch congruent mod 2n first) -> add to it (over, never under);
// older or empty -> restart at E.  (A half-range test on tag - (E mod 256) took a slot 129..255 epochs
// old for a newer one, kept its stale tag and lost the add: VERDICT r05 weak #1.)
__device__ inline uint32_t cm32_next(uint32_t x, uint32_t eref8, uint32_t dE, int64_t a) {
    const uint32_t tag = x >> 24, cnt = x & CM32_SAT;
    const uint32_t age = (eref8 - tag) & 0xFFu;
    const bool keep = cnt != 0 && age <= dE;                        // the same epoch (age == dE) or newer
    const uint64_t c = (keep ? (uint64_t)cnt : 0u) + (uint64_t)a;
    return (keep ? tag : (eref8 - dE) & 0xFFu) << 24 | (uint32_t)(c < CM32_SAT ? c : CM32_SAT);
}

__device__ inline int64_t cm_lds_window_min(const uint32_t *cl, const uint32_t *co, int depth, int nmax,
                                            double rcp_nmax, int nsc, int64_t E) {
    int64_t m = INT64_MAX;
    const int js0 = (int)cm_ring_slot(E, nmax, rcp_nmax);
#pragma unroll
    for (int d = 0; d < CMB_DMAX; ++d) {
        if (d >= depth) break;
        const uint32_t *c = cl + co[d];
        int64_t sum = 0;
        int js = js0;
        for (int k = 0; k < nsc; ++k) {                   // the window's slots: epochs E .. E - n + 1
            const uint32_t x = c[js];
            const uint32_t cnt = x & CM32_SAT;
            if ((((uint32_t)E - (x >> 24)) & 0xFFu) < (uint32_t)nsc)
                sum += cnt == CM32_SAT ? ((int64_t)1 << 40) : (int64_t)cnt;
            js = js == 0 ? nmax - 1 : js - 1;
        }
        m = sum < m ? sum : m;
    }
    return m;
}

__device__ inline void cm_lds_flush(uint32_t *cl, unsigned long long *dirty, const uint32_t *co, int depth,
                                    int nmax, double rcp_nmax, int64_t E, int64_t Eref, int64_t a) {
    const uint32_t js = cm_ring_slot(E, nmax, rcp_nmax);
    const uint32_t eref8 = (uint32_t)Eref & 0xFFu, dE = (uint32_t)(Eref - E);   // (0 <= dE < 256: the host)
    uint32_t x[CMB_DMAX];
#pragma unroll
    for (int d = 0; d < CMB_DMAX; ++d)
        if (d < depth) x[d] = cl[co[d] + js];
#pragma unroll
    for (int d = 0; d < CMB_DMAX; ++d) {
        if (d >= depth) break;
        const uint32_t w = co[d] + js;
        atomicOr(&dirty[w >> 6], 1ull << (w & 63));       // (written back at the end)
        uint32_t cur = x[d];
        for (;;) {                                        // (ds_cmpst_rtn_b32)
            const uint32_t prev = atomicCAS(cl + w, cur, cm32_next(cur, eref8, dE, a));
            if (prev == cur) break;
            cur = prev;
        }
    }
}

constexpr uint32_t CMB_VCAP = 480;        // grouped values (and their M) of one block staged in LDS; listed keys
constexpr uint32_t CMB_WORDS = 6144;      // slots of one block (the host checks)

// one key of a block walk: its record and everything the walk reads about it (loaded once, kept in
// registers from phase A to phase B for the thread's first key)
struct CmbKey {
    unsigned long long key;
    uint2 run;
    PRuleRec rr;
    double thr;
    uint32_t co[CMB_DMAX];
};

// full = false (phase A): the shared sketch's rules all have one window (the host checks it when the
// rules load), so the rule record is not read -- `u` carries the window; phase B reads it for the threshold
__device__ inline CmbKey cmb_key(const PKeyRecs &RC, const PRuleRec *__restrict__ RR, const ParamRules &PR,
                                 const CountMin &CM, uint32_t r, unsigned long long key, bool full,
                                 const PRuleRec &u) {
    CmbKey k;
    k.key = key;
    k.run = RC.run[r];
    if (full) {
        const int32_t rule = RC.rule[r];
        k.rr = RR[rule];
        k.thr = (k.rr.nf >> 16) ? value_threshold(PR, (uint32_t)rule, key) : k.rr.thr;   // CPFC:101-120
    } else {
        k.rr = u;
        k.thr = 0.0;
    }
    cm_lds_cells(k.co, CM.depth, CM.nmax, CM.cols, key);
    return k;
}

template <bool C32>
__global__ __launch_bounds__(256) void k_pp_cm_block(PKeyRecs RC, int sb, uint64_t *gval,
                                                      const ParamEvent *__restrict__ ev, ParamRules PR,
                                                      const PRuleRec *__restrict__ RR, CountMin CM,
                                                      int64_t *__restrict__ mv, long long *__restrict__ ctl,
                                                      const unsigned long long *__restrict__ tspan,
                                                      uint64_t *__restrict__ out, int32_t wsk, double rcp_wsk,
                                                      int diag) {
    // diag (SENTINEL_CM_DIAG, cost diagnostics only -- wrong verdicts / counters): bit 0 no window reads,
    // bit 1 no walk, bit 2 no block load / store, bit 3 no key list, bit 4 no adds, bit 5 no verdict stores
    using Cell = typename std::conditional<C32, uint32_t, unsigned long long>::type;
    extern __shared__ __attribute__((aligned(16))) unsigned long long cl_raw[];
    Cell *cl = reinterpret_cast<Cell *>(cl_raw);          // depth x cols x nmax
    __shared__ uint64_t sv[CMB_VCAP];                     // the block's keys' runs, compacted in key order
    __shared__ int64_t sm[CMB_VCAP];                      // M(E) of each staged request (phase A)
    __shared__ uint32_t klist[CMB_VCAP];                  // the block's key records, longest run first
    __shared__ uint32_t khist[33];
    __shared__ uint32_t s_waves[256 / WAVE];
    __shared__ unsigned long long dirty[CMB_WORDS / 64];  // slots this batch added to
    const uint32_t b = blockIdx.x;
    const uint32_t t = threadIdx.x;
    const int64_t T0 = pp_t0(ev);
    const int64_t ehi = ctl[0];
    const int64_t tmax = (int64_t)~tspan[1];              // the batch's newest request (k_pp_prep)
    const int depth = CM.depth, nmax = CM.nmax;
    const double rcp_nmax = 1.0 / (double)nmax;
    const uint32_t cols = CM.cols;
    const uint32_t words = (uint32_t)depth * cols * (uint32_t)nmax;
    unsigned long long *gcl = reinterpret_cast<unsigned long long *>(CM.cells) + (uint64_t)b * words;
    // this block's sub-ranges: [s0, s0 + ns); filter by block when a sub-range spans several blocks
    const int cb = CM.cbits;
    const uint32_t s0 = sb >= cb ? b << (sb - cb) : b >> (cb - sb);
    const uint32_t ns = sb >= cb ? 1u << (sb - cb) : 1u;
    const bool filter = sb < cb;
    uint32_t nkeys = 0;
    for (uint32_t s = s0; s < s0 + ns; ++s) nkeys += RC.sub[s].y;
    if (nkeys == 0) return;                               // (block-uniform) no key: the block stays in HBM
    const int64_t Eref = cm_eref(epoch_of(tmax, wsk, rcp_wsk), ehi);   // (no slot holds a later epoch)
    for (uint32_t i = t; i < CMB_WORDS / 64; i += blockDim.x) dirty[i] = 0;
    if (!(diag & 4)) {
        // every 16-B load of the thread's share of the block in flight before the first LDS store (one
        // HBM round trip per block instead of one per loop iteration); words / 2 <= CMB_WORDS / 2 = 12 x 256
        constexpr int LK = CMB_WORDS / 2 / 256;
        const ulonglong2 *g2 = reinterpret_cast<const ulonglong2 *>(gcl);
        ulonglong2 xs[LK];
#pragma unroll
        for (int k = 0; k < LK; ++k) {
            const uint32_t i = t + (uint32_t)k * 256u;
            xs[k] = i < words / 2 ? g2[i] : make_ulonglong2(0ull, 0ull);
        }
#pragma unroll
        for (int k = 0; k < LK; ++k) {
            const uint32_t i = t + (uint32_t)k * 256u;
            if (i >= words / 2) break;
            if constexpr (C32) {
                reinterpret_cast<uint2 *>(cl)[i] = make_uint2(cm32_load(xs[k].x, Eref), cm32_load(xs[k].y, Eref));
            } else {
                reinterpret_cast<ulonglong2 *>(cl)[i] = xs[k];
            }
        }
    }
    auto for_span = [&](auto &&f) __attribute__((always_inline)) {                       // every record of the block's keys
        for (uint32_t s = s0; s < s0 + ns; ++s) {
            const uint2 sr = RC.sub[s];
            for (uint32_t i = t; i < sr.y; i += blockDim.x) {
                const uint32_t r = sr.x + i;
                const unsigned long long key = RC.key[r];
                if (filter && cm_block_of(CM, key) != b) continue;
                f(r, key);
            }
        }
    };
    // the keys listed by run length, longest first (a wave walks for as long as its longest run: this
    // packs the long runs into the first waves); a block with more records than the list holds walks
    // them in record order
    const bool listed = nkeys <= CMB_VCAP && !(diag & 8);   // (block-uniform)
    uint32_t nlisted = 0;
    if (listed) {
        if (t < 33) khist[t] = 0;
        __syncthreads();
        uint32_t m0 = 0, m1 = 0, b0 = 0, b1 = 0, nm = 0;  // (this thread's first two records of the span)
        for (uint32_t s = s0; s < s0 + ns; ++s) {         // (a plain loop and selects: kept in registers)
            const uint2 sr = RC.sub[s];
            for (uint32_t i = t; i < sr.y; i += blockDim.x) {
                const uint32_t r = sr.x + i;
                if (filter && cm_block_of(CM, RC.key[r]) != b) continue;
                const uint32_t y = RC.run[r].y;
                const uint32_t bk = 31 - (y < 31 ? y : 31);
                atomicAdd(&khist[bk], 1u);
                m0 = nm == 0 ? r : m0;
                b0 = nm == 0 ? bk : b0;
                m1 = nm == 1 ? r : m1;
                b1 = nm == 1 ? bk : b1;
                ++nm;
            }
        }
        __syncthreads();
        if (t == 0) {
            uint32_t acc = 0;
            for (int i = 0; i < 32; ++i) { const uint32_t x = khist[i]; khist[i] = acc; acc += x; }
            khist[32] = acc;
        }
        __syncthreads();
        if (nm <= 2) {
            if (nm > 0) klist[atomicAdd(&khist[b0], 1u)] = m0;
            if (nm > 1) klist[atomicAdd(&khist[b1], 1u)] = m1;
        } else {
            for_span([&](uint32_t r, unsigned long long) {
                const uint32_t y = RC.run[r].y;
                klist[atomicAdd(&khist[31 - (y < 31 ? y : 31)], 1u)] = r;
            });
        }
        __syncthreads();
        nlisted = khist[32];
    }
    const PRuleRec uwin{rcp_wsk, 0.0, 0.0, wsk, CM.nmax / 2};    // the sketch's one window (phase A)
    auto for_keys = [&](bool full, auto &&f) __attribute__((always_inline)) {   // (same keys, same order per thread)
        if (listed) {
            for (uint32_t i = t; i < nlisted; i += blockDim.x) {
                const uint32_t r = klist[i];
                f(cmb_key(RC, RR, PR, CM, r, RC.key[r], full, uwin));
            }
        } else {
            for_span([&](uint32_t r, unsigned long long key) __attribute__((always_inline)) {
                f(cmb_key(RC, RR, PR, CM, r, key, full, uwin));
            });
        }
    };
    // the staging offsets: this thread's keys' runs at [voff0, voff0 + myv) of sv / sm; a run that does
    // not fit CMB_VCAP stays in HBM (gval, and its M in mv)
    uint32_t myv = 0;
    if (listed) {
        for (uint32_t i = t; i < nlisted; i += blockDim.x) myv += RC.run[klist[i]].y;
    } else {
        for_span([&](uint32_t r, unsigned long long) { myv += RC.run[r].y; });
    }
    uint32_t vtot;
    const uint32_t voff0 = block_exclusive_scan(myv, s_waves, &vtot);   // (its barriers: the block is in LDS)
    // A. stage the runs; reads (the block as the earlier batches left it)
    uint32_t vo = voff0;
    for_keys(false, [&](const CmbKey &K) __attribute__((always_inline)) {
        const uint2 run = K.run;
        const bool lds = vo + run.y <= CMB_VCAP;
        const int nsc = K.rr.nf & 0xFFFF;
        int64_t lastE = 0, lastM = 0;
        bool have = false;
        RunQueue rq(gval, run.x, run.x + run.y);
        for (uint32_t k = 0; k < run.y; ++k) {
            const uint64_t v = rq.next();
            if (lds) sv[vo + k] = v;
            if (ehi == CM_EHI_NONE || (diag & 1)) continue;
            int64_t tt;
            int32_t a;
            pp_unpack(v, T0, ev, tt, a);
            const int64_t E = epoch_of(tt, K.rr.w, K.rr.rcp_w);
            if (!cm_needs_read(E, ehi, nsc)) continue;
            if (!have || E != lastE) {
                lastM = cm_lds_window_min(cl, K.co, depth, nmax, rcp_nmax, nsc, E);
                lastE = E;
                have = true;
            }
            if (lds) sm[vo + k] = lastM;
            else mv[run.x + k] = lastM;
        }
        vo += run.y;
    });
    __syncthreads();
    // B. walks and adds.  A key's own admitted count inside the window (E - n, E] comes from prefix sums
    // over its run: each request's slot of the staged run is overwritten with the epoch its admitted
    // count is charged to (monotone along the run), its M slot with Q = the run's admitted sum before it;
    // own(E) = Q - Q[lo], lo = the run's first request charged to an epoch > E - n.  Each (key, epoch)
    // count is added to the block's d cells once, when the walk moves past the epoch (reads never see
    // this batch's adds: they were all done in A) -- unless the epoch is at least 2n older than the
    // batch's newest request: no window of a request within n epochs of the batch's end reaches it (the
    // ring would drop it for the next such epoch anyway).  A late request (E below the run's newest
    // epoch: outside the precondition) counts every admitted request of the run before it (over, never
    // under) and is charged to the newest epoch, as k_pp_cm_walk does.
    int64_t emax = CM_EHI_NONE;
    vo = voff0;
    auto walk = [&](uint32_t n_, int64_t *eb, int64_t *qb, const uint64_t *vb, const CmbKey &K) __attribute__((always_inline)) {
        const int nsc = K.rr.nf & 0xFFFF;
        const int64_t Edead = epoch_of(tmax, K.rr.w, K.rr.rcp_w) - 2 * (int64_t)nsc;
        int64_t curE = EPOCH_ABSENT, cnt = 0, Q = 0;
        uint32_t lo = 0;                                  // the window's first request; eb / qb[lo] cached:
        int64_t elo = 0, qlo = 0;                         // (valid while lo < k)
        for (uint32_t k = 0; k < n_; ++k) {
            const uint64_t v = vb[k];
            int64_t tt;
            int32_t a;
            pp_unpack(v, T0, ev, tt, a);
            const int64_t E = epoch_of(tt, K.rr.w, K.rr.rcp_w);
            emax = E > emax ? E : emax;
            const bool late = curE != EPOCH_ABSENT && E < curE;
            if (!late && E != curE) {
                if (cnt > 0 && curE > Edead && !(diag & 16)) cm_lds_flush(cl, dirty, K.co, depth, nmax, rcp_nmax, curE, Eref, cnt);
                curE = E;
                cnt = 0;
                while (lo < k && elo <= E - nsc) {
                    ++lo;
                    if (lo < k) { elo = eb[lo]; qlo = qb[lo]; }
                }
            }
            const int64_t own = late ? Q : (lo < k ? Q - qlo : 0);
            const int64_t m = cm_needs_read(E, ehi, nsc) ? qb[k] : 0;
            qb[k] = Q;
            eb[k] = curE;
            if (lo == k) { elo = curE; qlo = Q; }
            const double next = remaining_of(K.thr, K.rr.I_s, m + own, a);
            uint64_t vd;
            if (!(next < 0.0)) {                                          // CPFC:64-66, then addValue
                Q += a;
                cnt += a;
                vd = pack_verdict(ST_OK, java_d2i(next), 0);
            } else {
                vd = pack_verdict(ST_BLOCKED, 0, 0);
            }
            if (!(diag & 32)) store_verdict(out, RC.oseq ? K.run.x + k : (uint32_t)v & SEQ_MASK, vd);
        }
        if (cnt > 0 && curE > Edead && !(diag & 16)) cm_lds_flush(cl, dirty, K.co, depth, nmax, rcp_nmax, curE, Eref, cnt);
    };
    if (!(diag & 2)) for_keys(true, [&](const CmbKey &K) __attribute__((always_inline)) {
        const uint2 run = K.run;
        const bool lds = vo + run.y <= CMB_VCAP;
        if (lds)
            walk(run.y, reinterpret_cast<int64_t *>(sv + vo), sm + vo, sv + vo, K);
        else                                              // (the grouped values are dead after this walk)
            walk(run.y, reinterpret_cast<int64_t *>(gval + run.x), mv + run.x, gval + run.x, K);
        vo += run.y;
    });
    for (int o = WAVE / 2; o > 0; o >>= 1) {
        const int64_t y = __shfl_xor(emax, o, WAVE);
        emax = y > emax ? y : emax;
    }
    if (lane_id() == 0 && emax != CM_EHI_NONE) atomicMax(reinterpret_cast<long long *>(&ctl[2]), (long long)emax);
    __syncthreads();
    // write back the slots the batch added to (the rest of the block is unchanged in HBM)
    if (!(diag & 4))
        for (uint32_t i = t; i < (words + 63) / 64; i += blockDim.x) {
            unsigned long long m = dirty[i];
            while (m) {
                const uint32_t w = i * 64 + (uint32_t)(__ffsll(m) - 1);
                m &= m - 1;
                if constexpr (C32) gcl[w] = cm32_store(cl[w], Eref);
                else gcl[w] = cl[w];
            }
        }
}

// E_hi <- max(E_hi, this batch's newest epoch) (after k_pp_cm_walk); CM_EHI_ANY stays.
__global__ void k_pp_cm_ehi(long long *ctl) {
    if (threadIdx.x != 0) return;
    const long long e = ctl[2], h = ctl[0];
    if (h != CM_EHI_ANY && e != CM_EHI_NONE && (h == CM_EHI_NONE || e > h)) ctl[0] = e;
}

// Per shared count-min key-walk batch: flag = 0, ts range = {~0, ~0} (atomicMin targets), ctl[2] = none.
__global__ void k_cm_batch_init(unsigned long long *flag, unsigned long long *tspan, long long *ctl) {
    if (threadIdx.x == 0) {
        *flag = 0;
        tspan[0] = ~0ull;
        tspan[1] = ~0ull;
        ctl[2] = CM_EHI_NONE;
    }
}

__global__ void k_set_i64(long long *p, long long v) {
    if (threadIdx.x == 0) *p = v;
}

}  // namespace sentinel
