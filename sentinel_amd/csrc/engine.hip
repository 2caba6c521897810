// engine.hip -- MI355X token-decision engine: rule tables in HBM, batch pipeline, C ABI.
//
// Implements include/sentinel_amd.h.  One engine = one GPU = one shard of the flowId space.
// The batched path replaces DefaultTokenService.requestToken / requestParamToken
// (srv/flow/DefaultTokenService.java:37-62) for a whole batch of events at once:
//
//   k_flow_prep     validation + rule lookup + namespace routing (DTS:37-48, CFC:50-60), and the
//                   digit histograms of every radix pass (one read of the batch)
//   [limiter run]   GlobalRequestLimiter.tryPass per namespace (GlobalRequestLimiter.java:46-55)
//   K2 radix sort   group by flow, keep arrival order (scan_sort.hpp)
//   K1+K3           segment heads, window roll + segmented admission (admission.hpp)
//   verdict         scatter packed {remaining, status, waitInMs} back to arrival order
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <memory>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <string>
#include <unordered_map>
#include <deque>
#include <vector>

#include "../../include/sentinel_amd.h"
#include "admission.hpp"
#include "common.hpp"
#include "concurrent.hpp"
#include "param_rules.hpp"
#include "param_table.hpp"
#include "partition.hpp"
#include "param_part.hpp"
#include "small.hpp"
#include "local_entry.hpp"
#include <random>
#include "scan_sort.hpp"

using namespace sentinel;

static_assert(sizeof(Event) == sizeof(sentinel_event_t), "event layout");
static_assert(sizeof(ParamEvent) == sizeof(sentinel_param_event_t), "param event layout");
static_assert(sizeof(sentinel_verdict_t) == 8, "verdict layout");

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_OK(expr)                                                                          \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) return fail(SENTINEL_E_DEVICE, std::string(#expr ": ") + hipGetErrorString(_e)); \
    } while (0)

int bits_for(int64_t nkeys) {     // smallest b with 2^b - 1 >= nkeys (room for the invalid key)
    int b = 1;
    while (((int64_t)1 << b) - 1 < nkeys) ++b;
    return b;
}

constexpr int64_t MAX_BATCH = (int64_t)1 << 28;

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    int ensure(size_t want) {
        if (want <= bytes) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t b = std::max<size_t>(want, 256);
        if (hipMalloc(&p, b) != hipSuccess) return fail(SENTINEL_E_NOMEM, "hipMalloc failed");
        bytes = b;
        return 0;
    }
    template <class T> T *as() const { return (T *)p; }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

template <class T>
int upload(DevBuf &b, const std::vector<T> &v) {
    int rc = b.ensure(std::max<size_t>(v.size() * sizeof(T), sizeof(T)));
    if (rc) return rc;
    if (!v.empty()) HIP_OK(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return 0;
}

// The flow routes as bytes (ROUTE_* or a limiter key < 128); released when a key does not fit, so the
// kernels gather the 32-bit routes.
int upload_route8(DevBuf &b, const std::vector<int32_t> &route) {
    std::vector<int8_t> r8(route.size());
    for (size_t i = 0; i < route.size(); ++i) {
        if (route[i] < -128 || route[i] > 127) { b.release(); return 0; }
        r8[i] = (int8_t)route[i];
    }
    return upload(b, r8);
}

// Device-side key tables (SoA).
struct TableBufs {
    DevBuf off, n, w, rcp, Is, thr, kind, state, occ, has_occ;
    void release() {
        for (DevBuf *b : {&off, &n, &w, &rcp, &Is, &thr, &kind, &state, &occ, &has_occ}) b->release();
    }
};



// ------------------------------------------------------------------ prep kernels

// DefaultTokenService.requestToken validation (DTS:37-48) + namespace / limiter routing
// (ClusterFlowChecker.allowProceed, CFC:50-53).  Decided events get their final verdict here.
// Also builds the per-tile digit histograms of every radix pass of the flow keys (and of the
// limiter keys) from this single read of the batch.
__global__ __launch_bounds__(SORT_THREADS) void k_flow_prep(
    int64_t n, const Event *__restrict__ ev, int32_t nflows, const int32_t *__restrict__ route,
    uint64_t *__restrict__ out, uint32_t *__restrict__ fkey, uint32_t finvalid, int fpasses,
    uint32_t *__restrict__ fhist, uint32_t *__restrict__ lkey, uint32_t linvalid, int lpasses,
    uint32_t *__restrict__ lhist, int64_t nblocks, const int8_t *__restrict__ route8 = nullptr,
    uint32_t *__restrict__ oseq = nullptr, uint32_t *__restrict__ octr = nullptr, uint32_t opar = 0) {
    // oseq (decide-order output, no limiters): a decided event goes to position n - 1 - its rank among the
    // batch's decided events (they sort last, key finvalid: positions [valid, n)), as in k_part_prep
    if (octr && blockIdx.x == 0 && threadIdx.x == 0) octr[opar ^ 1u] = 0;
    __shared__ uint32_t hf[MAX_PASSES][RADIX];
    __shared__ uint32_t hl[MAX_PASSES][RADIX];
    for (int d = threadIdx.x; d < MAX_PASSES * RADIX; d += SORT_THREADS) {
        (&hf[0][0])[d] = 0;
        (&hl[0][0])[d] = 0;
    }
    __syncthreads();
    const int64_t tile0 = (int64_t)blockIdx.x * SORT_TILE;
    // every event load of the tile in flight at once, then every route load (a load per item inside
    // the loop made each thread wait SORT_ITEMS memory round trips in a row)
    Event evs[SORT_ITEMS];
    int32_t rts[SORT_ITEMS];
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        evs[j] = i < n ? ev[i] : Event{SENTINEL_IDX_BAD_ID, 0, 0};
    }
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const bool in = evs[j].idx >= 0 && evs[j].idx < nflows;
        rts[j] = (route8 && in) ? (int32_t)route8[evs[j].idx] : (route && in) ? route[evs[j].idx] : ROUTE_PLAIN;
    }
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        if (i >= n) break;
        const Event e = evs[j];
        int st = 127;   // undecided
        uint32_t k = finvalid, l = linvalid;
        if (e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0) st = ST_BAD_REQUEST;
        else if (e.idx < 0 || e.idx >= nflows) st = ST_NO_RULE_EXISTS;
        else {
            const int32_t r = rts[j];
            if (r == ROUTE_TOO_MANY) st = ST_TOO_MANY_REQUEST;      // namespace == null
            else if (e.ts < 0) st = ST_FAIL;                          // reference: NPE in LeapArray
            else {
                k = (uint32_t)e.idx;
                if (r >= 0) l = (uint32_t)r;
            }
        }
        fkey[i] = k;
        tile_hist_accumulate(hf, k, fpasses);
        if (lkey) {
            lkey[i] = l;
            tile_hist_accumulate(hl, l, lpasses);
        }
        if (st != 127 && !oseq) put_verdict(out, (uint32_t)i, st, 0, 0);
        if (oseq) put_rejected_ordered(st != 127, out, oseq, &octr[opar], n, (uint32_t)i, st);
    }
    __syncthreads();
    tile_hist_store(hf, fhist, fpasses, nblocks);
    if (lkey) tile_hist_store(hl, lhist, lpasses, nblocks);
}

// One namespace limiter (what the reference holds after any namespace-set change with the default
// namespace only, ClusterServerConfigManager.java:228-257): k_flow_prep's validation and routing, and
// the limiter pipeline's stable partition, in one pass over the batch.  Requests that reach
// GlobalRequestLimiter.tryPass (route 0) are packed in arrival order at the front of (skey, sval) --
// exactly what the radix pass over their limiter key leaves there -- and every other position gets
// the invalid key (from the back; their order is never read: the pipeline stops at nvalid).  Loads
// stay coalesced (item j of thread t is event j * L1_THREADS + t of the tile); the arrival-order rank
// comes from one ballot per item and a scan of the (item, wave) counts; tiles take a ticket and find
// how many limiter requests precede them by decoupled look-back (generation-tagged words, LBState).
constexpr int L1_THREADS = 512, L1_ITEMS = 8, L1_TILE = L1_THREADS * L1_ITEMS, L1_WAVES = L1_THREADS / WAVE;
static_assert(L1_ITEMS * L1_WAVES == WAVE, "one (item, wave) count per lane of the scanning wave");
__global__ __launch_bounds__(L1_THREADS) void k_lim1_prep(
    int64_t n, const Event *__restrict__ ev, int32_t nflows, const int32_t *__restrict__ route,
    const int8_t *__restrict__ route8, uint64_t *__restrict__ out, uint32_t *__restrict__ fkey, uint32_t finvalid,
    uint32_t linvalid, uint32_t *__restrict__ skey, uint64_t *__restrict__ sval, EventSrc src, LBState L) {
    __shared__ uint32_t s_cnt[L1_ITEMS * L1_WAVES];   // [item][wave] limiter requests, then their offsets
    __shared__ uint32_t s_prefix;
    const int64_t bid = lookback_ticket(L);
    const int64_t tile0 = bid * L1_TILE;
    const int wave = threadIdx.x / WAVE;
    Event evs[L1_ITEMS];
#pragma unroll
    for (int j = 0; j < L1_ITEMS; ++j) {
        const int64_t i = tile0 + j * L1_THREADS + threadIdx.x;
        evs[j] = i < n ? ev[i] : Event{SENTINEL_IDX_BAD_ID, 0, 0};
    }
    int32_t rts[L1_ITEMS];
#pragma unroll
    for (int j = 0; j < L1_ITEMS; ++j) {
        const bool in = evs[j].idx >= 0 && evs[j].idx < nflows;
        rts[j] = !in ? ROUTE_PLAIN : route8 ? (int32_t)route8[evs[j].idx] : route[evs[j].idx];
    }
    uint64_t bal[L1_ITEMS];
#pragma unroll
    for (int j = 0; j < L1_ITEMS; ++j) {
        const int64_t i = tile0 + j * L1_THREADS + threadIdx.x;
        const Event e = evs[j];
        int st = 127;   // undecided
        uint32_t k = finvalid;
        bool lim = false;
        if (e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0) st = ST_BAD_REQUEST;
        else if (e.idx < 0 || e.idx >= nflows) st = ST_NO_RULE_EXISTS;
        else {
            const int32_t r = rts[j];
            if (r == ROUTE_TOO_MANY) st = ST_TOO_MANY_REQUEST;      // namespace == null
            else if (e.ts < 0) st = ST_FAIL;                          // reference: NPE in LeapArray
            else {
                k = (uint32_t)e.idx;
                lim = r >= 0;
            }
        }
        if (i < n) {
            fkey[i] = k;
            if (st != 127) put_verdict(out, (uint32_t)i, st, 0, 0);
        }
        bal[j] = __ballot(lim && i < n);
        if (lane_id() == 0) s_cnt[j * L1_WAVES + wave] = (uint32_t)__popcll(bal[j]);
    }
    __syncthreads();
    if (threadIdx.x < WAVE) {
        const uint32_t c = s_cnt[threadIdx.x];
        const uint32_t inc = wave_inclusive_scan(c);
        s_cnt[threadIdx.x] = inc - c;
        const uint32_t total = __shfl(inc, WAVE - 1);
        tile_lookback(bid, total, L, &s_prefix);
    }
    __syncthreads();
    const int64_t T0 = src.t0();
#pragma unroll
    for (int j = 0; j < L1_ITEMS; ++j) {
        const int64_t i = tile0 + j * L1_THREADS + threadIdx.x;
        if (i >= n) continue;
        // limiter requests before event i (global)
        const int64_t v = (int64_t)s_prefix + s_cnt[j * L1_WAVES + wave] + mask_rank(bal[j]);
        if ((bal[j] >> lane_id()) & 1) {
            skey[v] = 0;
            sval[v] = src.pack_event((uint32_t)i, evs[j], 0, T0);
        } else {
            skey[n - 1 - (i - v)] = linvalid;       // i - v other events before i
        }
    }
}

// requestParamToken validation (DTS:51-62) + param slot lookup/insert in the open-addressing
// table (exact per-value counters: ClusterParamMetric.java:46-82).  Param keys are unique per
// (rule, value): the host's injective encoding of the Java typed value.
__global__ __launch_bounds__(SORT_THREADS) void k_param_prep(
    int64_t n, const ParamEvent *__restrict__ ev, int32_t nrules, const int32_t *__restrict__ route,
    unsigned long long *table, uint64_t cap_mask, int32_t *slot_rule, ParamRules PR, SlotMeta M,
    unsigned long long *fresh,
    uint64_t *__restrict__ out, uint32_t *__restrict__ fkey, uint32_t finvalid, int fpasses, uint32_t *__restrict__ fhist,
    uint32_t *__restrict__ lkey, uint32_t linvalid, int lpasses, uint32_t *__restrict__ lhist, int64_t nblocks) {
    __shared__ uint32_t hf[MAX_PASSES][RADIX];
    __shared__ uint32_t hl[MAX_PASSES][RADIX];
    __shared__ uint32_t s_fresh;
    for (int d = threadIdx.x; d < MAX_PASSES * RADIX; d += SORT_THREADS) {
        (&hf[0][0])[d] = 0;
        (&hl[0][0])[d] = 0;
    }
    if (threadIdx.x == 0) s_fresh = 0;
    __syncthreads();
    uint32_t nfresh = 0;
    const int64_t tile0 = (int64_t)blockIdx.x * SORT_TILE;
    ParamEvent pevs[SORT_ITEMS];                           // every event load of the tile in flight at once
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        pevs[j] = i < n ? ev[i] : ParamEvent{SENTINEL_IDX_BAD_ID, 0, 0, 0};
    }
    // then every route load and every first probe of the slot table (a key already in the table is
    // found there at the table's load factor): one memory round trip for the tile instead of one per
    // item; the unrolled loop keeps the events in registers (a dynamically indexed array spills)
    int32_t rts[SORT_ITEMS];
    unsigned long long first[SORT_ITEMS];
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const bool in = pevs[j].idx >= 0 && pevs[j].idx < nrules;
        rts[j] = (route && in) ? route[pevs[j].idx] : ROUTE_PLAIN;
        first[j] = in ? table[mix64(pevs[j].key) & cap_mask] : PKEY_EMPTY;
    }
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        if (i >= n) continue;
        const ParamEvent e = pevs[j];
        int st = 127;
        uint32_t k = finvalid, l = linvalid;
        if (e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0) st = ST_BAD_REQUEST;
        else if (e.idx < 0 || e.idx >= nrules) st = ST_NO_RULE_EXISTS;
        else {
            const int32_t r = rts[j];
            if (r == ROUTE_TOO_MANY) st = ST_TOO_MANY_REQUEST;
            else if (e.ts < 0) st = r >= 0 ? ST_FAIL : param_negative_ts_status(PR, (uint32_t)e.idx, e.key, e.acquire);
            else {
                const uint32_t before = nfresh;
                // a slot goes EMPTY -> key once per kernel, so a first probe that saw the key is final
                const int64_t h = first[j] == e.key ? (int64_t)(mix64(e.key) & cap_mask)
                                                    : slot_insert_counted(table, cap_mask, e.key, nfresh);
                if (h < 0) st = ST_FAIL;          // table full: the host's param_reserve prevents it
                else {
                    k = (uint32_t)h;
                    // the inserting event writes the slot's rule and window fields once; they only change
                    // with the rules / thresholds / table, when k_param_meta_all rewrites every slot
                    if (nfresh != before) {
                        slot_rule[h] = e.idx;
                        M.n[h] = PR.n[e.idx];
                        M.w[h] = PR.w[e.idx];
                        M.rcp[h] = PR.rcp_w[e.idx];
                        M.Is[h] = PR.I_s[e.idx];
                        M.thr[h] = value_threshold(PR, (uint32_t)e.idx, e.key);   // CPFC:113-120
                        M.kind[h] = KIND_PARAM;
                        slot_state_init(M.state, M.stride, (uint64_t)h, PR.n[e.idx]);
                    }
                    if (r >= 0) l = (uint32_t)r;
                }
            }
        }
        fkey[i] = k;
        tile_hist_accumulate(hf, k, fpasses);
        if (lkey) {
            lkey[i] = l;
            tile_hist_accumulate(hl, l, lpasses);
        }
        if (st != 127) put_verdict(out, (uint32_t)i, st, 0, 0);
    }
    block_add_global(fresh, nfresh, &s_fresh);              // (synchronises the block)
    tile_hist_store(hf, fhist, fpasses, nblocks);
    if (lkey) tile_hist_store(hl, lhist, lpasses, nblocks);
}

// Every live slot's window fields and threshold from its rule (after a rule load, a threshold change
// or a table rebuild; fresh inserts write their own in k_param_prep).
__global__ __launch_bounds__(256) void k_param_meta_all(uint64_t cap, const unsigned long long *__restrict__ keys,
                                                        const int32_t *__restrict__ slot_rule, int32_t nrules,
                                                        ParamRules PR, SlotMeta M) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap) return;
    const unsigned long long key = keys[s];
    if (key == PKEY_EMPTY) return;
    const int32_t r = slot_rule[s];
    if ((uint32_t)r >= (uint32_t)nrules) return;
    M.n[s] = PR.n[r];
    M.w[s] = PR.w[r];
    M.rcp[s] = PR.rcp_w[r];
    M.Is[s] = PR.I_s[r];
    M.thr[s] = value_threshold(PR, (uint32_t)r, key);
    M.kind[s] = KIND_PARAM;
}

// One key's slot (or -1) for the host's read-only queries.
__global__ void k_slot_find_one(const unsigned long long *table, uint64_t mask, uint64_t key, int64_t *out) {
    *out = slot_find(table, mask, key);
}

// Snapshot of one flow: getAvg(BLOCK) then getAvg(PASS) at ts (ClusterMetricNodeGenerator.java:79-84).
__global__ __launch_bounds__(256) void k_snapshot(KeyTable T, int32_t nflows, int64_t ts,
                                                  const int64_t *__restrict__ flow_ids,
                                                  sentinel_flow_snapshot_t *out) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nflows) return;
    const KeyState ks = key_state(T, (uint32_t)f);
    const int64_t E = epoch_of(ts, T.w[f], T.rcp_w[f]);
    roll(T, (uint32_t)f, ks, E);
    const double block = (double)window_sum(ks, E, EV_BLOCK) / T.I_s[f];
    roll(T, (uint32_t)f, ks, E);
    const double pass = (double)window_sum(ks, E, EV_PASS) / T.I_s[f];
    out[f].flow_id = flow_ids[f];
    out[f].pass_qps = pass;
    out[f].block_qps = block;
}

// Initialise state records: epochs absent, counters zero.
__global__ void k_init_state(int64_t *state, const int64_t *__restrict__ off, int64_t stride,
                             const int32_t *__restrict__ nn, int32_t fixed_n, int64_t words_per_key_fixed,
                             int64_t nkeys) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nkeys) return;
    const int64_t o = off ? off[k] : k * stride;
    const int n = nn ? nn[k] : fixed_n;
    const int64_t words = nn ? flow_record_words(n) : words_per_key_fixed;
    for (int64_t j = 0; j < words; ++j) state[o + j] = (j < 2 * n && (j & 1) == 0) ? EPOCH_ABSENT : 0;
}

// Flow-table remap of a rule reload (ClusterMetricStatistics.putMetricIfAbsent, CFRM:361-362):
// new flow i takes the window state of old flow src[i] >= 0 (with the old window, which the host
// kept in nn[i]), of the staged record stg[stg_off[i]] when src[i] == -2 (an orphaned metric coming
// back), or starts empty (-1).  Blocked header / rest layouts of the old and new tables may differ
// (slots per block = header_block_slots of each table's largest n).  Staged record: 2n pair words,
// 6n rest words (slot-major, counters BLOCK .. WAITING), occupy PASS, occupy PASS_REQUEST, has_occ.
// The new state must be zeroed beforehand.  nowCalls (CurrentConcurrencyManager) moves with src >= 0.
__global__ __launch_bounds__(256) void k_flow_remap(
    int64_t *__restrict__ nst, int32_t nhb, int64_t nrb, const int32_t *__restrict__ nn,
    const int64_t *__restrict__ ost, int32_t ohb, int64_t orb, const int32_t *__restrict__ src,
    const int64_t *__restrict__ stg, const int64_t *__restrict__ stg_off, int64_t *__restrict__ nocc,
    uint8_t *__restrict__ nhocc, int32_t *__restrict__ nnow, const int64_t *__restrict__ oocc,
    const uint8_t *__restrict__ ohocc, const int32_t *__restrict__ onow, int32_t F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= F) return;
    const int n = nn[i];
    const int32_t s = src[i];
    const int64_t *r = s == -2 ? stg + stg_off[i] : nullptr;
    for (int j = 0; j < n; ++j) {
        const int64_t d = blocked_pair_word(i, nhb, j);
        int64_t ep = EPOCH_ABSENT, ps = 0;
        if (s >= 0) {
            const int64_t o = blocked_pair_word(s, ohb, j);
            ep = ost[o];
            ps = ost[o + 1];
        } else if (r) {
            ep = r[2 * j];
            ps = r[2 * j + 1];
        }
        nst[d] = ep;
        nst[d + 1] = ps;
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            int64_t v = 0;
            if (s >= 0) v = ost[orb + blocked_rest_word(s, ohb, j, c)];
            else if (r) v = r[2 * n + 6 * j + c];
            nst[nrb + blocked_rest_word(i, nhb, j, c)] = v;
        }
    }
    int64_t o0 = 0, o1 = 0;
    uint8_t h = 0;
    int32_t now = 0;
    if (s >= 0) { o0 = oocc[2 * s]; o1 = oocc[2 * s + 1]; h = ohocc[s]; now = onow ? onow[s] : 0; }
    else if (r) { o0 = r[8 * n]; o1 = r[8 * n + 1]; h = (uint8_t)r[8 * n + 2]; }
    nocc[2 * i] = o0;
    nocc[2 * i + 1] = o1;
    nhocc[i] = h;
    nnow[i] = now;
}

// Staged records (k_flow_remap's format) of the old flows idx[k] whose metric outlives their rule
// (an emptied namespace list: clearAndResetRulesFor keeps METRIC_MAP, CFRM:268-283).
__global__ __launch_bounds__(256) void k_flow_gather(const int64_t *__restrict__ ost, int32_t ohb, int64_t orb,
                                                     const int32_t *__restrict__ idx, const int32_t *__restrict__ nn,
                                                     const int64_t *__restrict__ off, int32_t K,
                                                     const int64_t *__restrict__ oocc,
                                                     const uint8_t *__restrict__ ohocc, int64_t *__restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const int32_t o = idx[k];
    const int n = nn[k];
    int64_t *r = out + off[k];
    for (int j = 0; j < n; ++j) {
        const int64_t p = blocked_pair_word(o, ohb, j);
        r[2 * j] = ost[p];
        r[2 * j + 1] = ost[p + 1];
        for (int c = 0; c < 6; ++c) r[2 * n + 6 * j + c] = ost[orb + blocked_rest_word(o, ohb, j, c)];
    }
    r[8 * n] = oocc[2 * o];
    r[8 * n + 1] = oocc[2 * o + 1];
    r[8 * n + 2] = ohocc[o];
}

inline unsigned grid_for(int64_t n, int threads = 256) { return (unsigned)std::max<int64_t>(1, (n + threads - 1) / threads); }

}  // namespace

// flowId -> dense index on the host: open addressing over a power-of-two table (the per-call and
// batcher front doors look up every request; a node-based map costs several cache misses each).
struct FlatIndex {
    std::vector<int64_t> keys;       // 0 = empty (flowIds are > 0)
    std::vector<int32_t> vals;
    uint64_t mask = 0;
    void build(const std::unordered_map<int64_t, int32_t> &m) {
        uint64_t cap = 16;
        while (cap < 2 * m.size() + 2) cap <<= 1;
        keys.assign(cap, 0);
        vals.assign(cap, -1);
        mask = cap - 1;
        for (auto &kv : m) {
            uint64_t h = mix64((uint64_t)kv.first) & mask;
            while (keys[h]) h = (h + 1) & mask;
            keys[h] = kv.first;
            vals[h] = kv.second;
        }
    }
    int32_t find(int64_t id) const {
        if (id <= 0) return SENTINEL_IDX_BAD_ID;                // ClusterRuleUtil.validId
        if (keys.empty()) return SENTINEL_IDX_NO_RULE;
        for (uint64_t h = mix64((uint64_t)id) & mask;; h = (h + 1) & mask) {
            if (keys[h] == id) return vals[h];
            if (!keys[h]) return SENTINEL_IDX_NO_RULE;
        }
    }
};

// ==================================================================== engine
// Hot-run work list laid out after `head` words of a control buffer: runs (4 words each), the
// chunk -> run map, then the 32-byte chunk records.
static size_t long_runs_bytes(int64_t n, uint32_t min_run, size_t head) {
    const size_t words = head + 4 * long_runs_cap(n, min_run) + long_chunks_cap(n, min_run);
    return ((words * 4 + 31) & ~(size_t)31) + long_chunks_cap(n, min_run) * sizeof(LongRec);
}
static LongRuns long_runs_at(uint32_t *ctl, int64_t n, uint32_t min_run, size_t head) {
    LongRuns L;
    L.nrun = ctl;
    L.nchunk = ctl + 2;
    L.runs = ctl + head;
    L.chunk_run = L.runs + 4 * long_runs_cap(n, min_run);
    const size_t words = head + 4 * long_runs_cap(n, min_run) + long_chunks_cap(n, min_run);
    L.rec = reinterpret_cast<LongRec *>(reinterpret_cast<char *>(ctl) + ((words * 4 + 31) & ~(size_t)31));
    return L;
}

// Buffers of one partition-path batch: the front (prep, scan, scatter) writes them, the back
// (k_part_half / big / long) reads them.
struct PartBufs {
    DevBuf *fkey, *hist, *pscan, *sval, *vtmp, *runs, *stat;
};

struct sentinel_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    sentinel_server_config_t cfg{1.0, 1.0};
    std::vector<sentinel_namespace_t> ns;

    // flows
    std::vector<sentinel_flow_rule_t> rules;
    std::unordered_map<int64_t, int32_t> flow_index;
    FlatIndex flat_flow;
    std::vector<int32_t> h_flow_n, h_flow_w, h_flow_interval;   // the window of each flow's METRIC
    std::vector<int64_t> h_flow_off;
    // metrics that outlived their rule (a namespace whose rule list became empty keeps METRIC_MAP
    // entries: ClusterFlowRuleManager.clearAndResetRulesFor, CFRM:268-283), by flowId: window +
    // staged record (k_flow_remap format); revived if the flowId is loaded again
    struct Orphan { int32_t n, interval; std::vector<int64_t> rec; };
    std::unordered_map<int64_t, Orphan> orphans;
    TableBufs ft;
    DevBuf d_flow_route, d_flow_ids;
    DevBuf d_flow_route8;            // the same routes as bytes when every limiter key fits (a 4x smaller gather)
    bool use_route8 = true;          // SENTINEL_ROUTE8=0: gather the 32-bit routes
    bool lim1 = true;                // one namespace limiter: k_lim1_prep (SENTINEL_LIM1=0: prep + radix pass)
    const int8_t *route8() { return use_route8 ? d_flow_route8.as<int8_t>() : nullptr; }
    bool flow_plain = true;          // no flow needs a limiter or namespace check
    int32_t flow_max_n = 1;
    int32_t flow_hblock = 2;        // slots per block of the flow header region (>= every flow's n)
    int64_t flow_rest_base = 0;     // word offset of the flow table's blocked rest region
    int process_impl = 0;
    bool process_occ = true;         // param pipeline: k_process_reg held to 4 waves per SIMD (SENTINEL_PROC_OCC=0: off)
    bool verdict_nt = false;   // SENTINEL_VERDICT_NT=1: non-temporal verdict stores
    bool use_lookback = true;  // SENTINEL_SCAN=3pass selects the three-kernel scan
    bool fused_segments = true; // SENTINEL_SEGMENTS=split selects heads -> scan -> mark
    int seg_impl = 2;            // fused segments: 0 LDS-staged tile, 1 / 2 per-thread vector runs (256x16 / 512x8)
    int flow_path = 0;         // SENTINEL_FLOW_PATH: 0 auto, 1 sorted (global radix sort), 2 partition-local,
                               // 3 small (every batch in one-launch chunks of SM_MAX events)
    // small-batch host path (k_small_flow reads / writes pinned host memory directly)
    Event *h_sm_ev = nullptr;
    uint8_t *h_sm_fl = nullptr;
    uint64_t *h_sm_out = nullptr;
    uint32_t *h_sm_done = nullptr;
    // auto policy: the partition path unless the last partition batch was skewed (its largest flow
    // range > 8x the mean): then the sorted path for the next 1024 batches, then one probe again
    DevBuf d_part_stat;
    unsigned long long *h_part_stat = nullptr;   // pinned mirror, written asynchronously after each batch
    // batches per flow path: small, sorted, partition, [3] of the partition batches those with decide-order
    // output (sentinel_submit_flow_batch_ordered; until round 5 [3] counted the one-sweep partition front,
    // removed in round 6 after losing its A/B: 134 vs 130 us at config 3)
    int64_t flow_path_count[4] = {0, 0, 0, 0};
    DevBuf d_octr;                               // decide-order batches: rejected-event counters [2]
    uint32_t opar = 0;                           // ... the current batch's counter
    int num_cu = 0;
    // pinned words a kernel sets when a bounded spin gave up (the batch's results are invalid): [0] unused
    // (was the one-sweep partition's grid barrier), [1] the concurrency scan's look-back, [2] the radix
    // path's look-back (LBState.err: 1 a spin gave up, 2 a tile ticket outside the grid) (dev_err_synced)
    uint32_t *h_dev_err = nullptr;
    uint32_t *h_long_chunks = nullptr;           // pinned: hot-run chunks of a recent batch (launch hint)
    uint32_t *h_het_hint = nullptr;              // pinned: the sorted path's heterogeneous-key deferral is on
    uint32_t hot_het_run = HOT_HET_RUN;          // sorted path: heterogeneous keys above this go to k_part_long
    int64_t flow_batches = 0, sorted_until = -1;
    bool diag_linear = false;  // SENTINEL_DIAG_LINEAR=1 (-DSENTINEL_DIAG_LINEAR_ENV builds): verdicts in sorted order (cost diagnostic, wrong output)
    int64_t flow_state_words = 0;

    // namespace limiters (RequestLimiter = UnaryLeapArray(10, 1000))
    std::vector<int32_t> h_ns_limiter;   // namespace -> limiter key or -1
    int32_t nlimiters = 0;
    TableBufs lt;
    int64_t lim_stride = header_words(10);

    // param rules + slots
    std::vector<sentinel_param_rule_t> prules;
    std::unordered_map<int64_t, int32_t> param_index;
    // read-only copy published at every param rule load: sentinel_lookup_param_idx reads it without the
    // engine mutex (a wire front end's I/O thread never waits behind a GPU batch)
    std::shared_ptr<const std::unordered_map<int64_t, int32_t>> param_index_pub;
    DevBuf d_prule_route, d_prule_n, d_prule_w, d_prule_rcp, d_prule_Is, d_prule_thr;
    DevBuf d_prule_rec, d_prule_hot;   // packed per-rule records (k_prule_pack) + has-hot-items flags
    bool prec_dirty = true;
    DevBuf d_ptable, d_slot_rule, d_hot_table, d_hot_thr;
    bool param_plain = true;
    TableBufs pt;
    uint64_t pcap = (uint64_t)1 << 20;     // initial param slots; grows on demand (param_reserve)
    int32_t pmax_n = 1;
    uint64_t hot_mask = 0;
    bool has_hot = false;
    DevBuf d_prule_kind;               // KIND_PARAM per rule (segment kernel of the per-rule path)
    std::vector<int32_t> h_prule_n, h_prule_interval;   // the window of each param rule's METRIC
    // param metrics that outlived their rule (emptied namespace list), by flowId: window + exported
    // slots ((2 + 2n) words each: key, -, n {epoch, count} pairs)
    struct POrphan { int32_t n, interval; std::vector<int64_t> recs; };
    std::unordered_map<int64_t, POrphan> porphans;
    uint64_t p_live = 0;               // live slots after the last rebuild
    uint64_t p_ub = 0;                 // values submitted since (an upper bound of the fresh inserts)
    DevBuf d_pfresh;                   // device: fresh inserts since the last rebuild
    // pinned mirror {batch ordinal, d_pfresh after it} written by the device after every partition-path
    // param batch: the reserve check knows the exact fresh count up to a recent batch without a sync
    unsigned long long *h_pfresh = nullptr;
    unsigned long long *h_cmband = nullptr;     // shared count-min key walk: the sub-range overflow flag read back
    DevBuf d_cmband;                   // [0] overflow flag, [1..3] E_hi, E_hi seen by the read, the batch's newest epoch
    bool cm_keys = true;               // shared sketch: the two-phase key walk (k_pp_cm_read / _walk) when allowed
    uint64_t cm_key_batches = 0;       // shared-sketch batches decided by the key walk
    uint64_t cm_block_batches = 0;     // ... of which by the block-owned walk (k_pp_cm_block)
    bool cm_block = true;              // SENTINEL_CM_BLOCK=0: the two-phase HBM walk instead of the block-owned
                                       // walk (k_pp_cm_block; config 4cm: 799 vs 946 us)
    bool cm_debug = false;             // SENTINEL_CM_DEBUG=1: the key walk's geometry on stderr
    bool cm_c32 = true;                // SENTINEL_CM_C32=0: the block walk keeps 64-bit cells in LDS
    int cm_diag = 0;                   // SENTINEL_CM_DIAG (read only by a -DSENTINEL_DIAG_CM_ENV build): k_pp_cm_block /
                                       // k_conc_prep cost diagnostics (wrong results)
    DevBuf w_cmsub;                    // block walk: per sub-range {first record, records}
    DevBuf d_pexpire;                  // exact param table: per slot the getTopValues expire hint (PSlots)
    bool pexp_valid = false;           // ... every live slot's hint is current (only the key walk wrote since)
    uint64_t cm_overflows = 0;         // ... sent to the per-rule lanes (a sub-range over PG_CAP requests)
    uint64_t p_ord = 0;                // param batches reserved so far
    uint64_t p_reset_ord = 0;          // first batch ordinal after d_pfresh was last zeroed
    std::deque<std::pair<uint64_t, uint64_t>> p_pending;   // (ordinal, values) reserved since the reset
    // the previous table's buffers, kept as the next rebuild's target (no hipMalloc / hipFree per rebuild)
    DevBuf sp_keys, sp_rule, sp_state, sp_n, sp_w, sp_rcp, sp_Is, sp_thr, sp_kind;
    uint64_t p_rebuilds = 0;
    int32_t pmode = SENTINEL_PARAM_EXACT;
    int32_t cm_depth = 4;
    uint32_t cm_width = 1024;
    DevBuf d_cm;                       // count-min cells (SENTINEL_PARAM_COUNT_MIN)
    DevBuf w_cm;                       // shared sketch: rule heads, cursors, grid barrier, level words
    int cm_sync_blocks = 0;            // co-resident workgroups of k_prule_cm_sync
    int param_path = 0;                // single-value exact requests: 0 partition-local (param_part.hpp),
                                       // 1 per-rule walk, 2 per-slot radix-sort segments
    bool pmeta_dirty = true;           // the slots' window fields / thresholds need k_param_meta_all
    bool cm_force_coop = false;        // shared sketch: always the cooperative kernel (tests)

    // local param rules (ParamFlowChecker.passLocalCheck); rule index = load position
    int32_t nlrules = 0;
    DevBuf d_lrule_valid, d_lrule_tok, d_lrule_burst, d_lrule_dur, d_lrule_w, d_lrule_rcp, d_lrule_kind;
    DevBuf d_lhot_keys, d_lhot_tok, d_ltable, d_lstate;
    uint64_t lhot_mask = 0;
    bool lhas_hot = false;
    uint64_t lcap = (uint64_t)1 << 22;

    // local resources (SphU.entry: DefaultController over the ClusterNode's StatisticNode)
    int32_t nlres = 0, lres_n = 2, lres_w = 500, lres_g = 500;
    double lres_Is = 1.0;
    int32_t lres_interval = 1000;      // IntervalProperty.INTERVAL of the local nodes
    int32_t occupy_timeout = 500;      // OccupyTimeoutProperty.occupyTimeout (OccupyTimeoutProperty.java:40)
    DevBuf d_lres_state, d_lres_count, d_lres_w, d_lres_rcp, d_lres_kind, d_lres_tcount, d_lres_flags;
    DevBuf w_lslow, io_lrt;
    // local rule graph (sentinel_load_local_rules): origin / default nodes, rules, components
    bool lgraph = false;
    int32_t lg_on = 0, lg_dn = 0;
    DevBuf d_lg_on, d_lg_dn, d_lg_created, d_lg_roff, d_lg_rules, d_lg_comp, io_lctx;
    DevBuf d_lrule_grade;              // local param rules: 1 QPS, 0 THREAD (sentinel_set_local_param_grades)
    bool lhas_grade = false;            // local batch: sequential-path marks; host-fed exit response times
    int64_t lres_max_rt = 5000;        // SentinelConfig.statisticMaxRt (DEFAULT_STATISTIC_MAX_RT)

    // concurrency tokens (ConcurrentClusterFlowChecker): nowCalls per flow, token cache in HBM
    DevBuf d_now, d_conc_thr, d_seg1_w, d_seg1_rcp, d_seg1_kind;
    DevBuf d_tok_rec, d_tok_counts, d_tok_ticket;   // token cache: one TokRec per slot (concurrent.hpp)
    DevBuf w_cbig;                     // concurrency scan: tile descriptors, fallback list, nowCalls after the batch
    int64_t cbig_n = 0;                // its bytes
    uint64_t tok_ub = 0;               // upper bound of live + tombstoned token slots (no device read per batch)
    // the cache's counts after a recent batch (k_tok_snapshot into pinned memory, read once its event has
    // completed): tok_ub = that count + the events of every batch submitted after it, never a synchronisation
    unsigned long long *h_tok_snap = nullptr;
    hipEvent_t tok_snap_ev = nullptr;
    bool tok_snap_out = false;
    uint64_t tok_n_total = 0, tok_snap_n = 0;   // events submitted so far / when the snapshot was enqueued
    uint32_t tok_gen = 0, tok_snap_gen = 0;      // tok_gen: bumped when the cache is replaced or recounted
    uint64_t tok_grow = 16;                      // SENTINEL_TOKEN_GROW: batches of headroom a compaction sizes for
    uint64_t tcap = (uint64_t)1 << 22;
    uint64_t tok_salt = 0, tok_counter = 1;

    // per-kernel profiling (HIP events on the launch stream)
    struct ProfRec { const char *name; hipEvent_t a, b; int64_t units; };
    struct ProfAcc { double ms = 0; int64_t calls = 0; int64_t units = 0; };
    bool prof = false;
    std::string prof_only;                 // non-empty: only this kernel is timed
    std::vector<ProfRec> prof_pending;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<std::string, ProfAcc>> prof_acc;

    hipEvent_t get_ev() {
        if (!ev_pool.empty()) { hipEvent_t e = ev_pool.back(); ev_pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        // timing only: no system-scope fence when the event completes (it costs ~6 us of queue
        // idle per record on MI355X)
        (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
        return e;
    }

    int prof_every = 1;                // time every k-th launch of the selected kernel only
    int64_t prof_count = 0;
    template <class F>
    void launch(const char *name, int64_t units, hipStream_t s, F &&f) {
        if (!prof || (!prof_only.empty() && prof_only != name)) { f(); return; }
        if (prof_every > 1 && (prof_count++ % prof_every) != 0) { f(); return; }
        hipEvent_t a = get_ev(), b = get_ev();
        (void)hipEventRecord(a, s);
        f();
        (void)hipEventRecord(b, s);
        prof_pending.push_back({name, a, b, units});
    }

    // the hot-run kernels: chunk summaries, the per-run walk, the dead chunks' verdicts
    template <int NM>
    void launch_long(const KeyTable &T, const uint64_t *sval, const LongRuns &L, const EventSrc &src, const Verdicts &V,
                     int64_t n, uint32_t min_run, hipStream_t s, const unsigned long long *stat,
                     unsigned long long *host_stat) {
        // the chunk summaries pay off only for batches with hot runs: launched when an earlier batch had
        // some (the count comes back through pinned memory; without them every chunk is decided in full)
        if (!h_long_chunks) {
            if (hipHostMalloc((void **)&h_long_chunks, 4, 0) != hipSuccess) h_long_chunks = nullptr;
            else *h_long_chunks = 1;
        }
        LongRuns LL = L;
        LL.host_chunks = h_long_chunks;
        const bool recs = !h_long_chunks || *(volatile uint32_t *)h_long_chunks > 0;
        if (!recs) LL.rec = nullptr;
        const unsigned gc = (unsigned)std::min<size_t>(long_chunks_cap(n, min_run), 2048);
        if (recs) k_long_scan<<<gc, LS_THREADS, 0, s>>>(T, sval, LL, src);
        k_part_long<NM><<<256, PL_THREADS, 0, s>>>(T, sval, LL, src, V, stat, host_stat);
        if (recs) k_long_dead<<<gc, LS_THREADS, 0, s>>>(sval, LL, V);
    }

    void prof_collect() {
        for (auto &r : prof_pending) {
            (void)hipEventSynchronize(r.b);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, r.a, r.b);
            auto it = std::find_if(prof_acc.begin(), prof_acc.end(), [&](auto &x) { return x.first == r.name; });
            if (it == prof_acc.end()) { prof_acc.emplace_back(r.name, ProfAcc{}); it = prof_acc.end() - 1; }
            it->second.ms += ms;
            it->second.calls += 1;
            it->second.units += r.units;
            ev_pool.push_back(r.a);
            ev_pool.push_back(r.b);
        }
        prof_pending.clear();
    }

    // batch workspace
    DevBuf w_fkey, w_lkey, w_skey, w_sval, w_ktmp, w_vtmp, w_fhist, w_lhist, w_parts, w_segid, w_bad, w_hep,
        w_hacq, w_segstart, w_segkey, w_segep, w_segacq, w_het, w_prio, w_done, w_s0, w_k, w_counters;
    DevBuf w_vslot;                    // slot of every value of a param batch
    DevBuf w_runs;                     // partition path: long-run / oversized-half work lists
    DevBuf w_pscan;                    // partition path: per-group range sums + range starts
    DevBuf w_lb;                       // look-back words (LBState): generation-tagged, zeroed when allocated
    uint32_t *seg_zero = nullptr;      // four counters the next segment kernel zeroes (BatchWork.zero4)
    DevBuf io_ev, io_fl, io_out, io_vals;
    // streamed host path (sentinel_submit_flow_stream_host): copy streams + two staging slots
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    hipEvent_t x_h2d[2] = {}, x_comp[2] = {};
    DevBuf st_ev[2], st_fl[2], st_out[2];
    int64_t ws_cap = 0;

    int ensure_ws(int64_t n) {
        if (n <= ws_cap) return 0;
        int64_t c = std::max<int64_t>(n, 4096);
        int rc = 0;
        for (DevBuf *b : {&w_fkey, &w_lkey, &w_skey, &w_ktmp, &w_segid, &w_segkey, &w_k, &w_hacq, &w_segacq})
            rc |= b->ensure(c * 4);
        for (DevBuf *b : {&w_hep, &w_segep, &w_s0, &w_sval, &w_vtmp}) rc |= b->ensure(c * 8);
        for (DevBuf *b : {&w_bad, &w_het, &w_prio, &w_done}) rc |= b->ensure(c);
        rc |= w_fhist.ensure((size_t)(hist_words(c, MAX_PASSES) + 64) * 4);
        rc |= w_lhist.ensure((size_t)hist_words(c, MAX_PASSES) * 4);
        rc |= w_parts.ensure((size_t)(scan_parts(std::max<int64_t>(c, hist_words(c, MAX_PASSES))) + 16) * 8);
        rc |= w_segstart.ensure((c + 1) * 4);
        rc |= w_counters.ensure(64);
        {
            // every look-back user's tiles: the scan of the radix histograms, the segments, the limiter prep
            const size_t lbw = 256 + (size_t)(scan_parts(std::max<int64_t>(c, hist_words(c, MAX_PASSES))) + 16) * 8;
            if (lbw > w_lb.bytes) {
                rc |= w_lb.ensure(lbw);
                if (!rc && hipMemset(w_lb.p, 0, w_lb.bytes) != hipSuccess) rc = SENTINEL_E_DEVICE;
                if (!rc && lb_tickets0 && hipMemcpy(w_lb.p, &lb_tickets0, 4, hipMemcpyHostToDevice) != hipSuccess)
                    rc = SENTINEL_E_DEVICE;                  // (the device ticket starts where the host count does)
                lb_gen = lb_gen0;
                lb_tickets = lb_tickets0;
            }
        }
        if (rc) return SENTINEL_E_NOMEM;
        ws_cap = c;
        return 0;
    }

    // The look-back words of the next launch of `ntiles` workgroups (each takes one ticket).  ensure_ws
    // sizes the buffer for every batch; a larger user grows it here (zeroed on the stream first).
    uint32_t lb_gen = 0, lb_tickets = 0;
    // (tests: SENTINEL_LB_START=<generation>,<tickets> starts a fresh buffer near the generation wrap and
    // the 32-bit ticket wrap)
    uint32_t lb_gen0 = 0, lb_tickets0 = 0;
    LBState lb_state(int64_t ntiles, hipStream_t s) {
        const size_t want = 256 + (size_t)ntiles * 8;
        if (want > w_lb.bytes && w_lb.ensure(want) == 0) lb_zero(s);
        if (++lb_gen > LB_GEN_MASK) lb_zero(s);
        const LBState L{reinterpret_cast<unsigned long long *>(w_lb.as<char>() + 256), w_lb.as<uint32_t>(), lb_gen,
                        lb_tickets, h_dev_err + 2};
        lb_tickets += (uint32_t)ntiles;
        return L;
    }
    void lb_zero(hipStream_t s) {
        (void)hipMemsetAsync(w_lb.p, 0, w_lb.bytes, s);
        lb_gen = 1;
        lb_tickets = 0;
    }

    PartBufs part_bufs() {
        return PartBufs{&w_fkey, &w_fhist, &w_pscan, &w_sval, &w_vtmp, &w_runs, &d_part_stat};
    }

    BatchWork work() {
        BatchWork W;
        W.skey = w_skey.as<uint32_t>();
        W.sval = w_sval.as<uint64_t>();
        W.segid = w_segid.as<uint32_t>();
        W.bad = w_bad.as<uint8_t>();
        W.h_epoch = w_hep.as<int64_t>();
        W.h_acq = w_hacq.as<int32_t>();
        W.seg_start = w_segstart.as<uint32_t>();
        W.seg_key = w_segkey.as<uint32_t>();
        W.seg_epoch = w_segep.as<int64_t>();
        W.seg_acq = w_segacq.as<int32_t>();
        W.seg_het = w_het.as<uint8_t>();
        W.seg_prio = w_prio.as<uint8_t>();
        W.seg_done = w_done.as<uint8_t>();
        W.seg_s0 = w_s0.as<int64_t>();
        W.seg_k = w_k.as<uint32_t>();
        W.zero4 = seg_zero;
        W.nvalid = w_counters.as<uint32_t>();
        W.nseg = w_counters.as<uint32_t>() + 1;
        return W;
    }

    KeyTable table(TableBufs &b, int ncounters, int64_t stride) {
        KeyTable T;
        T.state_off = stride ? nullptr : b.off.as<int64_t>();
        T.state_stride = stride;
        T.n = b.n.as<int32_t>();
        T.w = b.w.as<int32_t>();
        T.rcp_w = b.rcp.as<double>();
        T.I_s = b.Is.as<double>();
        T.thr = b.thr.as<double>();
        T.kind = b.kind.as<uint8_t>();
        T.state = b.state.as<int64_t>();
        T.occ = b.occ.as<int64_t>();
        T.has_occ = b.has_occ.as<uint8_t>();
        T.hblock = &b == &ft ? flow_hblock : 0;
        T.rest_base = &b == &ft ? flow_rest_base : 0;
        T.ncounters = ncounters;
        T.max_occupy_ratio = cfg.max_occupy_ratio;
        return T;
    }

    // Rule tables read by the segment kernel of the per-rule param path.
    KeyTable param_rule_table() {
        KeyTable T{};
        T.n = d_prule_n.as<int32_t>();
        T.w = d_prule_w.as<int32_t>();
        T.rcp_w = d_prule_rcp.as<double>();
        T.I_s = d_prule_Is.as<double>();
        T.thr = d_prule_thr.as<double>();
        T.kind = d_prule_kind.as<uint8_t>();
        T.ncounters = 1;
        return T;
    }
    KeyTable local_rule_table() {
        KeyTable T{};
        T.w = d_lrule_w.as<int32_t>();
        T.rcp_w = d_lrule_rcp.as<double>();
        T.kind = d_lrule_kind.as<uint8_t>();
        T.ncounters = 1;
        return T;
    }
    ParamCtx param_ctx() {
        ParamCtx C{};
        C.R = ParamRules{d_prule_n.as<int32_t>(), d_prule_w.as<int32_t>(), d_prule_rcp.as<double>(),
                         d_prule_Is.as<double>(), d_prule_thr.as<double>(),
                         has_hot ? d_hot_table.as<unsigned long long>() : nullptr, hot_mask, d_hot_thr.as<double>()};
        C.PT = table(pt, 1, param_stride(pmax_n));
        {
            const uint32_t cols = std::min<uint32_t>(cm_width, CM_BLOCK_COLS);
            int cb = 0;
            while (((uint32_t)cols << cb) < cm_width) ++cb;
            C.CM = CountMin{d_cm.as<uint64_t>(), cm_depth, cm_width, cm_slots(), pmode == SENTINEL_PARAM_COUNT_MIN_SHARED,
                            cb, cols};
        }
        C.L = LocalRules{d_lrule_valid.as<uint8_t>(), d_lrule_tok.as<int64_t>(), d_lrule_burst.as<int64_t>(),
                         d_lrule_dur.as<int64_t>(), lhas_hot ? d_lhot_keys.as<unsigned long long>() : nullptr,
                         lhot_mask, d_lhot_tok.as<int64_t>(), d_lstate.as<int64_t>(),
                         lhas_grade ? d_lrule_grade.as<uint8_t>() : nullptr, nullptr};
        C.vslot = w_vslot.as<uint32_t>();
        return C;
    }
    SlotMeta slot_meta() {
        return SlotMeta{pt.n.as<int32_t>(), pt.w.as<int32_t>(), pt.rcp.as<double>(), pt.Is.as<double>(),
                        pt.thr.as<double>(), pt.kind.as<uint8_t>(), d_slot_rule.as<int32_t>(), pt.state.as<int64_t>(),
                        param_stride(pmax_n)};
    }

    void scan(uint32_t *buf, int64_t n, bool exclusive, hipStream_t s) {
        if (n <= 0) return;
        const int64_t nb = scan_parts(n);
        if (use_lookback) {
            const LBState L = lb_state(nb, s);   // (self-cleaning: no memset in front of the launch)
            launch("scan", n, s, [&] {
                if (exclusive) k_scan_lookback<true><<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, s>>>(buf, buf, n, L);
                else k_scan_lookback<false><<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, s>>>(buf, buf, n, L);
            });
            return;
        }
        uint32_t *parts = w_parts.as<uint32_t>();
        launch("scan_tiles", n, s, [&] {
            if (exclusive) k_scan_tiles<true><<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, s>>>(buf, buf, n, parts);
            else k_scan_tiles<false><<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, s>>>(buf, buf, n, parts);
        });
        launch("scan_partials", nb, s, [&] { k_scan_partials<<<1, SCAN_THREADS, 0, s>>>(parts, nb); });
        launch("scan_add", n, s, [&] { k_scan_add<<<dim3((unsigned)nb), dim3(SCAN_THREADS), 0, s>>>(buf, n, parts); });
    }

    // K2: stable LSD radix sort of (key, seq|prio, payload) by the low `bits` key bits into
    // (skey, sval).  `hist` holds pass 0's per-tile digit histograms (built by the prep
    // kernel from the same tiles); later passes histogram their own input.
    void sort(const uint32_t *keys_in, int64_t n, int bits, uint32_t *hist, const EventSrc &src, hipStream_t s,
              uint8_t *z0 = nullptr, uint8_t *z1 = nullptr) {
        const int64_t nb = sort_blocks(n);
        const int passes = passes_for(bits);
        uint32_t *kb[2];
        uint64_t *vb[2];
        if (passes % 2 == 1) {
            kb[0] = w_skey.as<uint32_t>(); vb[0] = w_sval.as<uint64_t>();
            kb[1] = w_ktmp.as<uint32_t>(); vb[1] = w_vtmp.as<uint64_t>();
        } else {
            kb[0] = w_ktmp.as<uint32_t>(); vb[0] = w_vtmp.as<uint64_t>();
            kb[1] = w_skey.as<uint32_t>(); vb[1] = w_sval.as<uint64_t>();
        }
        const uint32_t *kin = keys_in;
        const uint64_t *vin = nullptr;
        for (int p = 0; p < passes; ++p) {
            const int shift = p * RADIX_BITS;
            if (p > 0)
                launch("radix_hist", n, s, [&] {
                    k_radix_hist_pass<<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(kin, n, shift, hist, nb);
                });
            scan(hist, nb * RADIX, true, s);
            uint32_t *ko = kb[p % 2];
            uint64_t *vo = vb[p % 2];
            if (p == 0)
                launch("radix_scatter", n, s, [&] {
                    k_radix_scatter_p<true><<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(kin, vin, src, ko, vo, n,
                                                                                               shift, hist, nb, z0, z1);
                });
            else
                launch("radix_scatter", n, s, [&] {
                    k_radix_scatter_p<false><<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(kin, vin, src, ko, vo, n,
                                                                                                shift, hist, nb);
                });
            kin = ko;
            vin = vo;
        }
    }

    void hist_pass0(const uint32_t *keys, int64_t n, uint32_t *hist, hipStream_t s) {
        const int64_t nb = sort_blocks(n);
        launch("radix_hist", n, s, [&] {
            k_radix_hist_pass<<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(keys, n, 0, hist, nb);
        });
    }

    // K2 sort by key + (key, epoch) segment records (W.seg_*).
    void sort_segments(const KeyTable &T, const uint32_t *keys, uint32_t *hist, int64_t n, int bits,
                       const EventSrc &src, hipStream_t s, bool presorted = false) {
        BatchWork W = work();
        const uint32_t invalid = ((uint32_t)1 << bits) - 1;
        if (!presorted) {
            sort(keys, n, bits, hist, src, s, W.seg_het, W.seg_prio);   // (the first pass clears the flags)
        } else {
            (void)hipMemsetAsync(W.seg_het, 0, (size_t)n, s);
            (void)hipMemsetAsync(W.seg_prio, 0, (size_t)n, s);
        }
        const unsigned g = grid_for(n);
        if (fused_segments) {
            const int64_t nt = (n + SEG_TILE - 1) / SEG_TILE;
            const LBState L = lb_state(nt, s);
            launch("segments", n, s, [&] {
                if (seg_impl == 1)
                    k_segments_v<256, 16><<<dim3((unsigned)nt), dim3(256), 0, s>>>(T, W, src, n, invalid, L);
                else if (seg_impl == 2)
                    k_segments_v<512, 8><<<dim3((unsigned)nt), dim3(512), 0, s>>>(T, W, src, n, invalid, L);
                else
                    k_segments<<<dim3((unsigned)nt), dim3(SEG_THREADS), 0, s>>>(T, W, src, n, invalid, L);
            });
        } else {
            launch("seg_heads", n, s, [&] { k_seg_heads<<<g, 256, 0, s>>>(T, W, src, n, invalid); });
            scan(W.segid, n, false, s);
            launch("seg_mark", n, s, [&] { k_seg_mark<<<g, 256, 0, s>>>(W, n); });
        }
    }

    // The limiter pass of a flow batch: validation + routing into fkey (decided verdicts written), then
    // GlobalRequestLimiter.tryPass for every routed request (failures answer TOO_MANY_REQUEST and
    // their flow key becomes invalid).  fpasses: pass-0 flow-key histograms wanted from the prep.
    void limiter_pass(int64_t n, const Event *ev, int32_t F, uint32_t *fkey, uint32_t finvalid, int fpasses,
                      uint64_t *out, hipStream_t s) {
        const int lbits = bits_for(nlimiters);
        const uint32_t linvalid = ((uint32_t)1 << lbits) - 1;
        const KeyTable LT = table(lt, 1, lim_stride);
        const EventSrc lsrc{ev, nullptr, nullptr, true};
        const Verdicts LV{out, fkey, finvalid};
        (void)hipMemsetAsync(w_counters.p, 0, 16, s);
        if (nlimiters == 1 && lim1 && fpasses == 0) {
            const int64_t nt = (n + L1_TILE - 1) / L1_TILE;
            const LBState L = lb_state(nt, s);
            launch("lim_prep", n, s, [&] {
                k_lim1_prep<<<dim3((unsigned)nt), dim3(L1_THREADS), 0, s>>>(
                    n, ev, F, d_flow_route.as<int32_t>(), route8(), out, fkey, finvalid, linvalid,
                    w_skey.as<uint32_t>(), w_sval.as<uint64_t>(), lsrc, L);
            });
            run_pipeline(LT, nullptr, nullptr, n, lbits, lsrc, LV, s, 10, true, false, true);
            return;
        }
        uint32_t *lkey = w_lkey.as<uint32_t>();
        const int64_t nbs = sort_blocks(n);
        launch("flow_prep", n, s, [&] {
            k_flow_prep<<<dim3((unsigned)nbs), dim3(SORT_THREADS), 0, s>>>(
                n, ev, F, d_flow_route.as<int32_t>(), out, fkey, finvalid, fpasses, w_fhist.as<uint32_t>(), lkey,
                linvalid, 1, w_lhist.as<uint32_t>(), nbs, route8());
        });
        run_pipeline(LT, lkey, w_lhist.as<uint32_t>(), n, lbits, lsrc, LV, s, 10, true);
    }

    // The generic pipeline: sort by key, segment, decide, scatter.
    void run_pipeline(const KeyTable &T, const uint32_t *keys, uint32_t *hist, int64_t n, int bits,
                      const EventSrc &src, const Verdicts &V, hipStream_t s, int max_n, bool limiter,
                      bool hot_het = false, bool presorted = false, bool occ4 = false) {
        const unsigned g = grid_for(n);
        // flow tables: keys hotter than HOT_HET_RUN with heterogeneous acquires go to the hot-run kernels
        // (and keys of WAVE_HET_RUN..HOT_HET_RUN events to k_process_wave)
        LongRuns LR{};
        WaveRuns WR{};
        uint32_t *hint = nullptr;
        if (hot_het && max_n <= 16 && process_impl == 0) {
            if (!h_het_hint && hipHostMalloc((void **)&h_het_hint, 4, 0) == hipSuccess) *h_het_hint = 1;
            hint = h_het_hint;
        }
        // deferral on while recent batches had heterogeneous keys worth it (else k_process_reg only
        // raises the pinned hint): batches without them skip two launches
        if (hint && *(volatile uint32_t *)hint != 0) {
            const size_t lb = long_runs_bytes(n, hot_het_run, 4);
            if (w_runs.ensure(lb + 4 * ((size_t)n / WAVE_HET_RUN + 2)) == 0) {
                LR = long_runs_at(w_runs.as<uint32_t>(), n, hot_het_run, 4);
                WR.n = w_runs.as<uint32_t>() + 3;
                WR.g0 = reinterpret_cast<uint32_t *>(w_runs.as<char>() + lb);
                if (fused_segments) seg_zero = w_runs.as<uint32_t>();    // (k_segments zeroes the four counters)
                else (void)hipMemsetAsync(w_runs.p, 0, 16, s);
            }
        }
        sort_segments(T, keys, hist, n, bits, src, s, presorted);
        seg_zero = nullptr;
        BatchWork W = work();
        // the hot runs (a few keys, a workgroup each: the launches leave most of the chip idle) go on the aux
        // stream, concurrently with the wave runs and the verdict kernel: their keys, events and verdict
        // positions are disjoint, and k_process_reg already marked their segments done (k_verdict skips
        // them); the batch's stream waits for them before anything after this pipeline
        hipEvent_t join = nullptr;
        auto hot = [&](auto nmax) {
            constexpr int NM = decltype(nmax)::value;
            if (LR.nrun) {
                hipStream_t hs = s;
                if (hot_fork && aux_stream()) {
                    hipEvent_t fork = get_ev();
                    join = get_ev();
                    if (fork && join && hipEventRecord(fork, s) == hipSuccess &&
                        hipStreamWaitEvent(s_aux, fork, 0) == hipSuccess)
                        hs = s_aux;
                    if (fork) ev_pool.push_back(fork);
                }
                launch("part_long", n, hs, [&] { launch_long<NM>(T, W.sval, LR, src, V, n, hot_het_run, hs, nullptr, nullptr); });
                if (hs != s) {
                    (void)hipEventRecord(join, hs);
                } else if (join) {
                    ev_pool.push_back(join);
                    join = nullptr;
                }
            }
            if (WR.n)
                launch("process_wave", n, s, [&] {
                    const unsigned gw = (unsigned)std::min<int64_t>(n / WAVE_HET_RUN / 4 + 1, 2048);
                    k_process_wave<NM><<<gw, 256, 0, s>>>(T, W, src, V, WR, LR.nrun, hint);
                });
        };
        if (max_n <= PROC_G * PROC_SLOTS_PER_LANE && process_impl == 1)
            launch("process", n, s, [&] {
                k_process_grp<<<std::min<unsigned>(grid_for(n * PROC_G), 8192), 256, 0, s>>>(T, W, src, V, n);
            });
        else if (max_n <= 16 && process_impl == 0) {
            auto reg = [&](auto nmax) {
                constexpr int NM = decltype(nmax)::value;
                launch("process", n, s, [&] {
                    if (occ4 && process_occ) k_process_reg_o4<NM><<<g, 256, 0, s>>>(T, W, src, V, n, LR, WR, hot_het_run, hint);
                    else k_process_reg<NM><<<g, 256, 0, s>>>(T, W, src, V, n, LR, WR, hot_het_run, hint);
                });
                hot(nmax);
            };
            if (max_n <= 2) reg(std::integral_constant<int, 2>{});
            else if (max_n <= 4) reg(std::integral_constant<int, 4>{});
            else if (max_n <= 10) reg(std::integral_constant<int, 10>{});
            else reg(std::integral_constant<int, 16>{});
        }
        else
            launch("process", n, s, [&] { k_process<<<g, 256, 0, s>>>(T, W, src, V, n); });
        if (limiter) launch("verdict", n, s, [&] { k_verdict<true, false><<<g, 256, 0, s>>>(T, W, V, n); });
        else if (verdict_nt) launch("verdict", n, s, [&] { k_verdict<false, true><<<g, 256, 0, s>>>(T, W, V, n); });
        else if (diag_linear) launch("verdict", n, s, [&] { k_verdict<false, false, true><<<g, 256, 0, s>>>(T, W, V, n); });
        else launch("verdict", n, s, [&] { k_verdict<false, false><<<g, 256, 0, s>>>(T, W, V, n); });
        if (join) {
            (void)hipStreamWaitEvent(s, join, 0);
            ev_pool.push_back(join);
        }
    }

    // The engine's second compute stream (created on first use): hot runs concurrent with the rest.
    hipStream_t s_aux = nullptr;
    bool hot_fork = true;              // SENTINEL_HOT_FORK=0: the hot runs on the batch's stream, in order
    bool aux_stream() {
        if (!s_aux && hipStreamCreateWithFlags(&s_aux, hipStreamNonBlocking) != hipSuccess) s_aux = nullptr;
        return s_aux != nullptr;
    }

    int rebuild_flow_thresholds();
    void flow_thresholds(const std::vector<sentinel_flow_rule_t> &rules, std::vector<double> &thr,
                         std::vector<double> &cthr) const;
    bool flow_routes(const std::vector<sentinel_flow_rule_t> &rules, std::vector<int32_t> &route) const;
    int rebuild_limiters();
    int rebuild_routes();
    int install_flows(std::vector<sentinel_flow_rule_t> &&nr, std::unordered_map<int64_t, int32_t> &&nidx,
                      std::vector<int32_t> &&gn, std::vector<int32_t> &&gint, std::vector<int32_t> &&src,
                      std::vector<int64_t> &&stg, std::vector<int64_t> &&stg_off, const std::vector<int32_t> &orphan_old);
    int clear_param_slots();
    int param_rebuild(uint64_t new_cap, const std::vector<int32_t> &rmap, int32_t new_maxn,
                      const std::vector<int32_t> &new_rn, const std::vector<int64_t> &imp, int64_t imp_stride,
                      const std::vector<int32_t> &imp_rule, std::vector<std::pair<int32_t, std::vector<int64_t>>> *exported);
    int param_reserve(int64_t nv);
    int param_thresholds();
    std::vector<uint64_t> h_phot_keys;          // the loaded param rules' hot items (hot_begin / hot_n index them)
    std::vector<int32_t> h_phot_counts;
    int reset_param_metrics(int32_t sample_count, int32_t interval_ms);
    bool uniform_param_window() const {
        for (size_t i = 1; i < h_prule_n.size(); ++i)
            if (h_prule_n[i] != h_prule_n[0] || h_prule_interval[i] != h_prule_interval[0]) return false;
        return true;
    }
    int rebuild_cm();
    int32_t cm_slots() const { return pmode == SENTINEL_PARAM_COUNT_MIN_SHARED ? 2 * pmax_n : pmax_n; }
    int ensure_tokens();
    int rewrite_tokens(bool compact, uint64_t new_cap = 0);
    int rebuild_tokens_device(uint64_t new_cap, hipStream_t s);
    DevBuf sp_tok_rec;                 // the next compaction's target
    // getTopValues scratch (param_top), kept between calls: candidate list {key, rule, sum} + its count,
    // per-rule selection state, the results and the rules' flowIds (grow-only: no allocation per snapshot)
    struct TopScratch {
        DevBuf ckey, crule, csum, cn, pr, pk, cr, ck, dc, dk, ds, ids, rank, fkey, frule, fsum, flist;
        std::vector<int64_t> h_ids;    // the flowIds in `ids` (uploaded again only when the rules change)
    } topw;
    TokenTable token_table() {
        return TokenTable{d_tok_rec.as<TokRec>(), tcap - 1, d_tok_counts.as<unsigned long long>()};
    }
    // {live, tombstones}: the striped counters summed (stream-ordered copy on s, synchronised)
    int token_counts(unsigned long long out[2], hipStream_t s) {
        unsigned long long h[TOK_CNT_LANES * TOK_CNT_STRIDE];
        HIP_OK(hipMemcpyAsync(h, d_tok_counts.p, TOK_CNT_BYTES, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        out[0] = out[1] = 0;
        for (int l = 0; l < TOK_CNT_LANES; ++l) {
            out[0] += h[l * TOK_CNT_STRIDE];
            out[1] += h[l * TOK_CNT_STRIDE + 1];
        }
        return 0;
    }
};

// Token cache: allocated on first use (SENTINEL_TOKEN_CAPACITY slots, default 4M).
int sentinel_engine::ensure_tokens() {
    if (d_tok_rec.p) return 0;
    if (const char *c = getenv("SENTINEL_TOKEN_CAPACITY")) {
        uint64_t v = strtoull(c, nullptr, 10), p = 1024;
        while (p < v) p <<= 1;
        tcap = p;
    }
    int rc = 0;
    rc |= d_tok_rec.ensure(tcap * sizeof(TokRec));
    rc |= d_tok_counts.ensure(TOK_CNT_BYTES);
    rc |= d_tok_ticket.ensure(8);
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemsetAsync(d_tok_rec.p, 0xFF, tcap * sizeof(TokRec), stream));   // empty keys, no claims
    tok_ub = 0;
    ++tok_gen;
    if (!h_tok_snap && hipHostMalloc((void **)&h_tok_snap, 16, 0) != hipSuccess) h_tok_snap = nullptr;
    if (!tok_snap_ev && hipEventCreateWithFlags(&tok_snap_ev, hipEventDisableTiming) != hipSuccess) tok_snap_ev = nullptr;
    HIP_OK(hipMemsetAsync(d_tok_counts.p, 0, TOK_CNT_BYTES, stream));
    HIP_OK(hipStreamSynchronize(stream));
    std::random_device rd;                 // token ids: {salt:23 | counter:40}, opaque to clients like UUID bits
    tok_salt = ((uint64_t)rd() ^ ((uint64_t)rd() << 11)) & ((1ull << 23) - 1);
    return 0;
}

// Host rewrite of the token cache: remap every live token's flow index from its flowId (after a
// rule load: tokens of removed flows answer NO_RULE_EXISTS until the flowId comes back), and
// optionally drop tombstones by re-inserting the live tokens into a fresh table.
int sentinel_engine::rewrite_tokens(bool compact, uint64_t new_cap) {
    if (!d_tok_rec.p) return 0;
    const uint64_t ocap = tcap;
    const uint64_t ncap = new_cap > ocap ? new_cap : ocap;   // growing re-places every token
    if (ncap != ocap) compact = true;
    std::vector<TokRec> old(ocap);
    HIP_OK(hipMemcpy(old.data(), d_tok_rec.p, ocap * sizeof(TokRec), hipMemcpyDeviceToHost));
    if (ncap != ocap) {
        d_tok_rec.release();
        if (d_tok_rec.ensure(ncap * sizeof(TokRec))) return SENTINEL_E_NOMEM;
        tcap = ncap;
    }
    TokRec empty;
    memset(&empty, 0xFF, sizeof(empty));
    std::vector<TokRec> nr(tcap, empty);
    uint64_t live = 0, dead = 0;
    for (uint64_t h = 0; h < ocap; ++h) {
        const TokRec &o = old[h];
        if (o.key == PKEY_EMPTY) continue;
        if (o.key == TOKEN_TOMB) {
            if (!compact) { nr[h].key = TOKEN_TOMB; ++dead; }
            continue;
        }
        uint64_t d = h;
        if (compact) {
            d = tok_home(o.key, tcap - 1);
            while (nr[d].key != PKEY_EMPTY) d = (d + 1) & (tcap - 1);
        }
        auto it = flow_index.find(o.flow_id);
        nr[d].key = o.key;
        nr[d].flow_id = o.flow_id;
        nr[d].flow_idx = it == flow_index.end() ? -1 : it->second;
        nr[d].acquire = o.acquire;
        ++live;
    }
    std::vector<unsigned long long> counts(TOK_CNT_LANES * TOK_CNT_STRIDE, 0ull);
    counts[0] = live;
    counts[1] = dead;
    tok_ub = live + dead;
    ++tok_gen;
    HIP_OK(hipMemcpy(d_tok_rec.p, nr.data(), tcap * sizeof(TokRec), hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(d_tok_counts.p, counts.data(), TOK_CNT_BYTES, hipMemcpyHostToDevice));
    return 0;
}

// Token cache compaction on the device (no host copy): the live tokens move into the spare buffers
// (re-sized to new_cap), which then become the cache; stream-ordered, no synchronisation.
int sentinel_engine::rebuild_tokens_device(uint64_t new_cap, hipStream_t s) {
    const uint64_t ocap = tcap, ncap = std::max(new_cap, ocap);
    int rc = 0;
    rc |= sp_tok_rec.ensure(ncap * sizeof(TokRec));
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemsetAsync(sp_tok_rec.p, 0xFF, ncap * sizeof(TokRec), s));
    HIP_OK(hipMemsetAsync(d_tok_counts.p, 0, TOK_CNT_BYTES, s));
    const TokenTable O = token_table();
    const TokenTable N{sp_tok_rec.as<TokRec>(), ncap - 1, d_tok_counts.as<unsigned long long>()};
    k_tok_rebuild<<<grid_for((int64_t)ocap), 256, 0, s>>>(O, ocap, N);
    HIP_OK(hipGetLastError());
    std::swap(d_tok_rec, sp_tok_rec);
    tcap = ncap;
    ++tok_gen;
    return 0;
}

// Exact param counters restart: every slot free, every window absent (stream synchronised).
int sentinel_engine::clear_param_slots() {
    if (!d_ptable.p) return 0;
    const uint64_t P = pcap;
    const int64_t stride = param_stride(pmax_n);
    HIP_OK(hipMemsetAsync(d_ptable.p, 0xFF, P * 8, stream));
    HIP_OK(hipMemsetAsync(d_pfresh.p, 0, CNT_BYTES, stream));
    k_init_state<<<grid_for((int64_t)P), 256, 0, stream>>>(pt.state.as<int64_t>(), nullptr, stride, nullptr, pmax_n,
                                                           stride, (int64_t)P);
    pexp_valid = false;
    HIP_OK(hipStreamSynchronize(stream));
    p_live = p_ub = 0;
    return 0;
}

// Rebuild of the exact param table into a fresh one of new_cap slots (param_table.hpp): live slots of
// rules with rmap[old rule] >= 0 move under the new index unless dead, rmap == -2 exports the rule's
// slots to `exported` (old rule, records), -1 drops them; `imp` (imp_stride words per record, rule
// imp_rule[k]) is inserted afterwards.  new_rn: the new rules' windows (n).  On failure the old table
// stays in place.
int sentinel_engine::param_rebuild(uint64_t new_cap, const std::vector<int32_t> &rmap, int32_t new_maxn,
                                   const std::vector<int32_t> &new_rn, const std::vector<int64_t> &imp,
                                   int64_t imp_stride, const std::vector<int32_t> &imp_rule,
                                   std::vector<std::pair<int32_t, std::vector<int64_t>>> *exported) {
    const int64_t nstride = param_stride(new_maxn);
    const int64_t ostride = param_stride(pmax_n);
    DevBuf &nkeys = sp_keys, &nrule = sp_rule, &nstate = sp_state, &nn = sp_n, &nw = sp_w, &nrcp = sp_rcp,
           &nIs = sp_Is, &nthr = sp_thr, &nkind = sp_kind;
    DevBuf dmap, dnewest, dcount, dxout, dimp, dimprule, dnrn;
    auto cleanup = [&] {
        for (DevBuf *b : {&dmap, &dnewest, &dcount, &dxout, &dimp, &dimprule, &dnrn}) b->release();
    };
    int rc = 0;
    rc |= nkeys.ensure(new_cap * 8);
    rc |= nrule.ensure(new_cap * 4);
    rc |= nstate.ensure(new_cap * (uint64_t)nstride * 8);
    rc |= nn.ensure(new_cap * 4);
    rc |= nw.ensure(new_cap * 4);
    rc |= nrcp.ensure(new_cap * 8);
    rc |= nIs.ensure(new_cap * 8);
    rc |= nthr.ensure(new_cap * 8);
    rc |= nkind.ensure(new_cap);
    rc |= dcount.ensure(16);
    if (rc) { cleanup(); return SENTINEL_E_NOMEM; }
    const int32_t OR = (int32_t)rmap.size();
    bool any_export = false;
    for (int32_t m : rmap) any_export |= m == -2;
    const bool have_old = d_ptable.p != nullptr && OR > 0;
    if (hipMemsetAsync(nkeys.p, 0xFF, new_cap * 8, stream) != hipSuccess || hipMemsetAsync(dcount.p, 0, 16, stream) != hipSuccess) {
        cleanup();
        return fail(SENTINEL_E_DEVICE, "memset failed");
    }
    // (no state initialisation: every slot is written by the rebuild / import below or by its fresh insert)
    const PSlots N{nkeys.as<unsigned long long>(), nrule.as<int32_t>(), nstate.as<int64_t>(), nstride, new_cap - 1};
    const PSlots O{d_ptable.as<unsigned long long>(), d_slot_rule.as<int32_t>(), pt.state.as<int64_t>(), ostride, pcap - 1};
    unsigned long long *live = dcount.as<unsigned long long>();
    unsigned long long *xcount = live + 1;
    uint64_t xcap = 0;
    const int64_t xstride = 2 + 2 * (int64_t)pmax_n;
    if (have_old) {
        rc |= upload(dmap, rmap);
        rc |= dnewest.ensure((size_t)OR * 8);
        if (any_export) {
            xcap = pcap;   // every slot could belong to an exported rule
            rc |= dxout.ensure(xcap * (uint64_t)xstride * 8);
        }
        if (rc) { cleanup(); return SENTINEL_E_NOMEM; }
        (void)hipMemsetAsync(dnewest.p, 0, (size_t)OR * 8, stream);
        k_ptable_rule_newest<<<grid_for((int64_t)pcap), 256, 0, stream>>>(O, pcap, OR, d_prule_n.as<int32_t>(),
                                                                         dnewest.as<unsigned long long>());
        k_ptable_rebuild<<<grid_for((int64_t)pcap), 256, 0, stream>>>(O, pcap, OR, dmap.as<int32_t>(), d_prule_n.as<int32_t>(),
                                                                     dnewest.as<unsigned long long>(), N, live,
                                                                     dxout.as<int64_t>(), xstride, xcount, xcap);
    }
    const int64_t K = imp_stride > 0 ? (int64_t)imp.size() / imp_stride : 0;
    if (K > 0) {
        rc |= upload(dimp, imp);
        rc |= upload(dimprule, imp_rule);
        rc |= upload(dnrn, new_rn);
        if (rc) { cleanup(); return SENTINEL_E_NOMEM; }
        k_ptable_import<<<grid_for(K), 256, 0, stream>>>(dimp.as<int64_t>(), imp_stride, K, dimprule.as<int32_t>(),
                                                        dnrn.as<int32_t>(), N, live);
    }
    unsigned long long cnt[2] = {0, 0};
    hipError_t he = hipGetLastError();
    if (he == hipSuccess) he = hipMemcpyAsync(cnt, dcount.p, 16, hipMemcpyDeviceToHost, stream);
    if (he == hipSuccess) he = hipStreamSynchronize(stream);
    if (he != hipSuccess) {
        cleanup();
        return fail(SENTINEL_E_DEVICE, std::string("param table rebuild failed: ") + hipGetErrorString(he));
    }
    if (exported && any_export && cnt[1] > 0) {
        const uint64_t nx = std::min<uint64_t>(cnt[1], xcap);
        std::vector<int64_t> x(nx * xstride);
        if (hipMemcpy(x.data(), dxout.p, x.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) {
            cleanup();
            return fail(SENTINEL_E_DEVICE, "param export failed");
        }
        for (uint64_t k = 0; k < nx; ++k) {
            const int64_t *r = x.data() + k * xstride;
            const int32_t orule = (int32_t)r[1];
            const int n = h_prule_n[orule];
            auto it = std::find_if(exported->begin(), exported->end(), [&](auto &p) { return p.first == orule; });
            if (it == exported->end()) { exported->emplace_back(orule, std::vector<int64_t>()); it = exported->end() - 1; }
            it->second.insert(it->second.end(), r, r + 2 + 2 * n);
        }
    }
    std::swap(d_ptable, nkeys);
    pexp_valid = false;                                  // (slots moved: the next snapshot recomputes the hints)
    std::swap(d_slot_rule, nrule);
    std::swap(pt.state, nstate);
    std::swap(pt.n, nn);
    std::swap(pt.w, nw);
    std::swap(pt.rcp, nrcp);
    std::swap(pt.Is, nIs);
    std::swap(pt.thr, nthr);
    std::swap(pt.kind, nkind);
    cleanup();
    if (!d_pfresh.p && d_pfresh.ensure(CNT_BYTES)) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemsetAsync(d_pfresh.p, 0, CNT_BYTES, stream));
    HIP_OK(hipStreamSynchronize(stream));
    pcap = new_cap;
    pmax_n = new_maxn;
    p_live = cnt[0];
    p_ub = 0;
    p_reset_ord = p_ord;
    p_pending.clear();
    ++p_rebuilds;
    pmeta_dirty = true;
    return 0;
}

// Room for nv more values before a batch: the table never holds more than 3/4 of its slots, so a
// slot insert cannot fail.  The bound is tracked without a device read (values submitted since the
// last rebuild); only when it could be crossed the exact count is read, dead slots are reclaimed, and
// the table grows if the live slots still leave too little room.
int sentinel_engine::param_reserve(int64_t nv) {
    if (!d_ptable.p) return 0;
    const uint64_t lim = pcap / 4 * 3;
    const uint64_t ord = p_ord++;
    if (p_live + p_ub + (uint64_t)nv <= lim) {
        p_ub += (uint64_t)nv;
        p_pending.emplace_back(ord, (uint64_t)nv);
        return 0;
    }
    if (h_pfresh) {                 // the device's last published count: exact up to that batch
        const uint64_t seq = ((volatile unsigned long long *)h_pfresh)[0];
        const uint64_t pub = ((volatile unsigned long long *)h_pfresh)[1];
        if (seq != ~0ull && seq >= p_reset_ord && seq < ord) {
            while (!p_pending.empty() && p_pending.front().first <= seq) p_pending.pop_front();
            uint64_t after = 0;
            for (auto &x : p_pending) after += x.second;
            if (p_live + pub + after + (uint64_t)nv <= lim) {
                p_ub = pub + after + (uint64_t)nv;
                p_pending.emplace_back(ord, (uint64_t)nv);
                return 0;
            }
        }
    }
    unsigned long long lanes[CNT_LANES * CNT_STRIDE], fresh = 0;
    HIP_OK(hipMemcpyAsync(lanes, d_pfresh.p, CNT_BYTES, hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    for (int l = 0; l < CNT_LANES; ++l) fresh += lanes[l * CNT_STRIDE];
    p_pending.clear();
    if (p_live + fresh + (uint64_t)nv <= lim) {
        p_live += fresh;
        p_ub = (uint64_t)nv;
        HIP_OK(hipMemsetAsync(d_pfresh.p, 0, CNT_BYTES, stream));
        // finished before returning: this batch's kernels may run on a caller's stream that waited on the
        // engine stream before the reset was queued, and their fresh-insert adds must land after it
        HIP_OK(hipStreamSynchronize(stream));
        p_reset_ord = ord;
        p_pending.emplace_back(ord, (uint64_t)nv);
        return 0;
    }
    std::vector<int32_t> ident(prules.size());
    for (size_t i = 0; i < ident.size(); ++i) ident[i] = (int32_t)i;
    int rc = param_rebuild(pcap, ident, pmax_n, h_prule_n, {}, 0, {}, nullptr);        // reclaim dead slots
    if (rc) return rc;
    // grow until the live slots plus this batch fit, and -- within a memory budget -- until a few more
    // batches of new values fit too, so that the reclaiming rebuild (a device-wide pass and a host sync)
    // comes back every few batches, not every batch, under a steady churn of values
    const uint64_t slot_bytes = 8 + 4 + (uint64_t)param_stride(pmax_n) * 8 + 4 + 4 + 8 + 8 + 8 + 1;
    const uint64_t budget = (uint64_t)24 << 30;           // per table (the rebuild holds two): 288 GB of HBM
    uint64_t cap = pcap;
    while (p_live + (uint64_t)nv > cap / 4 * 3) cap <<= 1;
    while (p_live + 8 * (uint64_t)nv > cap / 4 * 3 && 2 * cap * slot_bytes <= budget) cap <<= 1;
    if (cap != pcap) {
        rc = param_rebuild(cap, ident, pmax_n, h_prule_n, {}, 0, {}, nullptr);         // grow
        if (rc) return rc;
    }
    p_ub = (uint64_t)nv;
    p_reset_ord = ord;              // (param_rebuild zeroed d_pfresh)
    p_pending.clear();
    p_pending.emplace_back(ord, (uint64_t)nv);
    return 0;
}

// Param thresholds: ClusterParamFlowChecker.calcGlobalThreshold(rule, value) (CPFC:101-111) -- the
// hot-item count of the value if any, else rule.count (getRawThreshold, CPFC:113-120), times the
// namespace's connectedCount for AVG_LOCAL rules.  The reference evaluates it on every request, so
// it is recomputed whenever a connected count changes (not only at rule load).  Hot items live in a
// table keyed by param key (param keys are unique per (rule, value)).
int sentinel_engine::param_thresholds() {
    const size_t R = prules.size();
    std::vector<double> thr(std::max<size_t>(R, 1), 0.0);
    std::vector<std::pair<uint64_t, double>> hot;
    for (size_t i = 0; i < R; ++i) {
        const sentinel_param_rule_t &r = prules[i];
        const int32_t cc = (r.namespace_idx >= 0 && r.namespace_idx < (int32_t)ns.size()) ? ns[r.namespace_idx].connected_count : 0;
        double c = r.count;
        if (r.threshold_type != SENTINEL_THRESHOLD_GLOBAL) c = c * (double)cc;
        thr[i] = c;
        for (int32_t h = 0; h < r.hot_n; ++h) {
            const int32_t j = r.hot_begin + h;
            if (j < 0 || (size_t)j >= h_phot_counts.size()) continue;
            double hc = (double)h_phot_counts[j];
            if (r.threshold_type != SENTINEL_THRESHOLD_GLOBAL) hc = hc * (double)cc;
            hot.emplace_back(h_phot_keys[j], hc);
        }
    }
    uint64_t hcap = 16;
    while (hcap < 2 * hot.size() + 2) hcap <<= 1;
    std::vector<uint64_t> hk(hcap, PKEY_EMPTY);
    std::vector<double> hv(hcap, 0.0);
    for (auto &kv : hot) {
        uint64_t h = mix64(kv.first) & (hcap - 1);
        while (hk[h] != PKEY_EMPTY && hk[h] != kv.first) h = (h + 1) & (hcap - 1);
        hk[h] = kv.first;
        hv[h] = kv.second;
    }
    int rc = 0;
    rc |= upload(d_prule_thr, thr);
    rc |= upload(d_hot_table, hk);
    rc |= upload(d_hot_thr, hv);
    if (rc) return rc;
    hot_mask = hcap - 1;
    has_hot = !hot.empty();
    {
        std::vector<uint8_t> hf(std::max<size_t>(R, 1), 0);
        for (size_t i = 0; i < R; ++i) hf[i] = prules[i].hot_n > 0;
        if (upload(d_prule_hot, hf)) return SENTINEL_E_NOMEM;
    }
    pmeta_dirty = true;
    prec_dirty = true;
    return 0;
}

// Server window change: every param metric (orphans included) restarts with the server window
// (ClusterParamMetricStatistics.resetFlowMetrics, ClusterParamMetricStatistics.java:60-66).
int sentinel_engine::reset_param_metrics(int32_t sample_count, int32_t interval_ms) {
    for (auto &kv : porphans) {
        kv.second.n = sample_count;
        kv.second.interval = interval_ms;
        kv.second.recs.clear();
    }
    const size_t R = prules.size();
    if (R == 0) return 0;
    h_prule_n.assign(R, sample_count);
    h_prule_interval.assign(R, interval_ms);
    std::vector<int32_t> ww(R, interval_ms / sample_count);
    std::vector<double> rcp(R, 1.0 / (double)(interval_ms / sample_count)), Is(R, interval_ms / 1000.0);
    int rc = 0;
    rc |= upload(d_prule_n, h_prule_n);
    rc |= upload(d_prule_w, ww);
    rc |= upload(d_prule_rcp, rcp);
    rc |= upload(d_prule_Is, Is);
    if (rc) return rc;
    prec_dirty = true;
    pmax_n = sample_count;
    if (d_ptable.p) {
        rc = param_rebuild(pcap, std::vector<int32_t>(R, -1), pmax_n, h_prule_n, {}, 0, {}, nullptr);
        if (rc) return rc;
    }
    return rebuild_cm();
}

// Count-min cells for every param rule, zeroed (count 0 = nothing counted).
int sentinel_engine::rebuild_cm() {
    if (pmode == SENTINEL_PARAM_EXACT) return 0;
    // one sketch per rule, or one for every rule (SHARED: a single window for all param rules)
    const size_t R = pmode == SENTINEL_PARAM_COUNT_MIN_SHARED ? 1 : std::max<size_t>(prules.size(), 1);
    const size_t bytes = R * (size_t)cm_depth * (size_t)cm_width * (size_t)cm_slots() * 8;
    if (bytes > ((size_t)96 << 30)) return fail(SENTINEL_E_NOMEM, "count-min sketch would exceed 96 GiB");
    int rc = d_cm.ensure(bytes);
    if (rc) return rc;
    HIP_OK(hipMemsetAsync(d_cm.p, 0, bytes, stream));
    if (pmode == SENTINEL_PARAM_COUNT_MIN_SHARED) {       // the key walk's control words: cleared cells
        if (d_cmband.ensure(64)) return SENTINEL_E_NOMEM;
        k_set_i64<<<1, 64, 0, stream>>>(d_cmband.as<long long>() + 1, (long long)CM_EHI_NONE);
    }
    HIP_OK(hipStreamSynchronize(stream));
    return 0;
}

// Host mirror of ClusterFlowChecker.calcGlobalThreshold * exceedCount (CFC:38-48, 68) and
// SimpleClusterFlowChecker (SCFC:42), evaluated in double exactly as Java does.
int sentinel_engine::rebuild_flow_thresholds() {
    std::vector<double> thr, cthr;
    flow_thresholds(rules, thr, cthr);
    int rc = upload(ft.thr, thr);
    if (rc) return rc;
    return upload(d_conc_thr, cthr);
}

void sentinel_engine::flow_thresholds(const std::vector<sentinel_flow_rule_t> &rules, std::vector<double> &thr,
                                      std::vector<double> &cthr) const {
    thr.assign(rules.size(), 0.0);
    for (size_t i = 0; i < rules.size(); ++i) {
        const sentinel_flow_rule_t &r = rules[i];
        if (r.checker == SENTINEL_CHECKER_SIMPLE) {
            thr[i] = r.count * cfg.exceed_count;
        } else {
            double g;
            if (r.threshold_type == SENTINEL_THRESHOLD_GLOBAL) g = r.count;
            else {
                const int32_t c = (r.namespace_idx >= 0 && r.namespace_idx < (int32_t)ns.size()) ? ns[r.namespace_idx].connected_count : 0;
                g = r.count * (double)c;
            }
            thr[i] = g * cfg.exceed_count;
        }
    }
    // ConcurrentClusterFlowChecker.calcGlobalThreshold (CCFC:35-46): no exceedCount
    cthr.assign(std::max<size_t>(rules.size(), 1), 0.0);
    for (size_t i = 0; i < rules.size(); ++i) {
        const sentinel_flow_rule_t &r = rules[i];
        const int32_t c = (r.namespace_idx >= 0 && r.namespace_idx < (int32_t)ns.size()) ? ns[r.namespace_idx].connected_count : 0;
        cthr[i] = r.threshold_type == SENTINEL_THRESHOLD_GLOBAL ? r.count : r.count * (double)c;
    }
}

// Per-rule routing: TOO_MANY_REQUEST for a null namespace, limiter id, or plain.
// Per-rule routing of a flow table (namespace null -> TOO_MANY_REQUEST, limiter key, or plain);
// returns whether every flow is plain.
bool sentinel_engine::flow_routes(const std::vector<sentinel_flow_rule_t> &rules, std::vector<int32_t> &route) const {
    route.assign(rules.size(), ROUTE_PLAIN);
    bool plain = true;
    for (size_t i = 0; i < rules.size(); ++i) {
        const sentinel_flow_rule_t &r = rules[i];
        int32_t v = ROUTE_PLAIN;
        if (r.checker == SENTINEL_CHECKER_CLUSTER) {
            if (r.namespace_idx < 0 || r.namespace_idx >= (int32_t)ns.size()) v = ROUTE_TOO_MANY;
            else if (h_ns_limiter[r.namespace_idx] >= 0) v = h_ns_limiter[r.namespace_idx];
        }
        route[i] = v;
        if (v != ROUTE_PLAIN) plain = false;
    }
    return plain;
}

int sentinel_engine::rebuild_routes() {
    std::vector<int32_t> route;
    flow_plain = flow_routes(rules, route);
    int rc = upload(d_flow_route, route);
    if (rc) return rc;
    rc = upload_route8(d_flow_route8, route);
    if (rc) return rc;
    std::vector<int32_t> proute(prules.size());
    param_plain = true;
    for (size_t i = 0; i < prules.size(); ++i) {
        const sentinel_param_rule_t &r = prules[i];
        int32_t v = ROUTE_PLAIN;
        if (r.namespace_idx < 0 || r.namespace_idx >= (int32_t)ns.size()) v = ROUTE_TOO_MANY;
        else if (h_ns_limiter[r.namespace_idx] >= 0) v = h_ns_limiter[r.namespace_idx];
        proute[i] = v;
        if (v != ROUTE_PLAIN) param_plain = false;
    }
    return upload(d_prule_route, proute);
}

// One RequestLimiter per namespace with has_limiter (GlobalRequestLimiter.java:32-37):
// UnaryLeapArray(10, 1000) -> n = 10, w = 100, intervalInSecond = 1.0.
int sentinel_engine::rebuild_limiters() {
    h_ns_limiter.assign(ns.size(), -1);
    std::vector<int32_t> n, w;
    std::vector<double> rcp, Is, thr;
    std::vector<uint8_t> kind;
    for (size_t i = 0; i < ns.size(); ++i) {
        if (!ns[i].has_limiter) continue;
        h_ns_limiter[i] = (int32_t)n.size();
        n.push_back(10);
        w.push_back(100);
        rcp.push_back(1.0 / 100.0);
        Is.push_back(1000 / 1000.0);
        thr.push_back(ns[i].max_allowed_qps);
        kind.push_back(KIND_LIMITER);
    }
    nlimiters = (int32_t)n.size();
    int rc = 0;
    rc |= upload(lt.n, n);
    rc |= upload(lt.w, w);
    rc |= upload(lt.rcp, rcp);
    rc |= upload(lt.Is, Is);
    rc |= upload(lt.thr, thr);
    rc |= upload(lt.kind, kind);
    if (rc) return rc;
    rc = lt.state.ensure(std::max<int64_t>(1, nlimiters) * lim_stride * 8);
    if (rc) return rc;
    if (nlimiters > 0) {
        k_init_state<<<grid_for(nlimiters), 256, 0, stream>>>(lt.state.as<int64_t>(), nullptr, lim_stride, nullptr, 10,
                                                              lim_stride, nlimiters);
        HIP_OK(hipStreamSynchronize(stream));
    }
    return rebuild_routes();
}

// Partition-local flow path (partition.hpp): prep + range histogram, scan, one multi-split pass,
// one fused sort + decide pass per flow range (LDS), oversized ranges redone from HBM, hot flows.
template <int NMAX>
static void launch_part_decide(sentinel_engine_t *e, int32_t nparts, const KeyTable &FT, const uint32_t *rstart,
                               int lb, const EventSrc &src, const Verdicts &V, int64_t n, hipStream_t s,
                               uint32_t *ctl, unsigned long long *stat, const uint64_t *pval, uint64_t *gsval) {
    // ctl: [0] runs, [1] oversized halves, [2] chunks, [3] -, [4, 4 + 2 nparts) oversized halves, then the runs
    uint32_t *nbig = ctl + 1, *big = ctl + 4;
    const LongRuns LR = long_runs_at(ctl, n, LONG_RUN, 4 + 2 * (size_t)nparts);
    // a batch whose mean range does not fit goes straight to the HBM-sorting kernel
#ifndef SENTINEL_ALLBIG_PCT
#define SENTINEL_ALLBIG_PCT 90
#endif
    const bool all_big = n > (int64_t)nparts * (int64_t)(PH_KEYS * SENTINEL_ALLBIG_PCT / 100);
    if (!all_big) {
        e->launch("part_fused", n, s, [&] {
            const dim3 g(16u * (unsigned)((nparts + 7) / 8));
            if (part_coop(lb))      // <= 256 flows per half: cooperative verdict sweep
                k_part_half<NMAX, true><<<g, PH_THREADS, 0, s>>>(FT, pval, gsval, rstart, lb, nparts,
                                                                 (int32_t)e->rules.size(), src, V, LR,
                                                                 big, nbig, stat);
            else
                k_part_half<NMAX, false><<<g, PH_THREADS, 0, s>>>(FT, pval, gsval, rstart, lb, nparts,
                                                                  (int32_t)e->rules.size(), src, V, LR,
                                                                  big, nbig, stat);
        });
    }
    e->launch("part_big", n, s, [&] {
        k_part_big<NMAX><<<all_big ? 2u * (unsigned)nparts : (unsigned)std::min<int32_t>(2 * nparts, 256), PH_THREADS, 0, s>>>(
            FT, pval, gsval, rstart, lb, nparts, src, V, LR, all_big ? nullptr : big, nbig,
            stat);
    });
    e->launch("part_long", n, s, [&] {   // hot flows (runs > LONG_RUN events): a workgroup each
        e->launch_long<NMAX>(FT, gsval, LR, src, V, n, LONG_RUN, s, stat, e->h_part_stat);
    });
}

// Geometry of a partition-path batch.
struct PartGeo {
    int32_t F;
    uint32_t finvalid;
    int lb, pbits;
    int32_t nparts;
    int64_t nb, ng;
};
static PartGeo part_geo(const sentinel_engine_t *e, int64_t n) {
    PartGeo g;
    g.F = (int32_t)e->rules.size();
    const int fbits = bits_for(g.F);
    g.finvalid = ((uint32_t)1 << fbits) - 1;
    g.lb = std::max(0, fbits - PART_MAX_BITS);
    g.nparts = (int32_t)(((int64_t)g.F + (1 << g.lb) - 1) >> g.lb);
    g.pbits = bits_for(g.nparts - 1 > 0 ? g.nparts - 1 : 1);
    g.nb = part_blocks(n);
    g.ng = (g.nb + PS_GROUP - 1) / PS_GROUP;
    return g;
}

// The front of a partition batch (prep + range histogram, scan, multi-split) into buffer set B.
static int ensure_part_bufs(sentinel_engine_t *e, const PartBufs &B, int64_t n) {
    const PartGeo g = part_geo(e, n);
    int rc = B.pscan->ensure(((size_t)g.ng * g.nparts + 2 * (size_t)g.nparts + 1) * 4);
    rc |= B.runs->ensure(long_runs_bytes(n, LONG_RUN, 4 + 2 * (size_t)g.nparts));
    rc |= B.stat->ensure(8);
    return rc;
}

static int part_front(sentinel_engine_t *e, const PartBufs &B, int64_t n, const Event *ev, const uint8_t *fl,
                      uint64_t *out, hipStream_t s, uint32_t *oseq = nullptr) {
    const PartGeo g = part_geo(e, n);
    int rc = ensure_part_bufs(e, B, n);
    if (rc) return rc;
    if (!e->h_part_stat) {
        HIP_OK(hipHostMalloc((void **)&e->h_part_stat, 8, 0));
        *e->h_part_stat = 0;
    }
    uint32_t *fkey = B.fkey->as<uint32_t>();
    uint32_t *hist = B.hist->as<uint32_t>();                // tile-major range histograms -> offsets
    uint32_t *gsum = B.pscan->as<uint32_t>();
    uint32_t *rstart = gsum + (size_t)g.ng * g.nparts;
    uint32_t *rtot = rstart + g.nparts + 1;
    unsigned long long *stat = B.stat->as<unsigned long long>();
    uint32_t *ctl = B.runs->as<uint32_t>();
    // namespace limiters (GlobalRequestLimiter.tryPass before every flow check, CFC:50-57) couple the
    // flows of a namespace: validation and the limiter pass run first (the sorted path's k_flow_prep and
    // limiter pipeline, which mark failing events invalid); the multi-split then takes their keys
    const bool lim = e->nlimiters > 0 && !e->flow_plain;
    if (lim) e->limiter_pass(n, ev, g.F, fkey, g.finvalid, 0, out, s);
    e->flow_path_count[2] += 1;
    e->launch("part_prep", n, s, [&] {
        k_part_prep<<<dim3((unsigned)g.nb), dim3(PP_THREADS), 0, s>>>(
            n, ev, g.F, e->flow_plain ? nullptr : e->d_flow_route.as<int32_t>(), out,
            (e->flow_plain || lim) ? nullptr : fkey, g.finvalid, g.lb, hist, g.nb, g.nparts, ctl, stat,
            lim ? fkey : nullptr, oseq, oseq ? e->d_octr.as<uint32_t>() : nullptr, e->opar);
    });
    e->launch("scan", n, s, [&] {
        const dim3 g2((unsigned)g.ng, (unsigned)((g.nparts + PS_THREADS - 1) / PS_THREADS));
        k_part_colsum<<<g2, PS_THREADS, 0, s>>>(hist, g.nb, g.nparts, gsum);
        k_part_colscan<<<(unsigned)((g.nparts + PC_THREADS / WAVE - 1) / (PC_THREADS / WAVE)), PC_THREADS, 0, s>>>(
            gsum, g.ng, g.nparts, rtot);
        k_part_offsets<<<g2, PS_THREADS, 0, s>>>(hist, g.nb, g.nparts, gsum, rtot, rstart);
    });
    const EventSrc src{ev, nullptr, fl, false};
    e->launch("part_scatter", n, s, [&] {
        k_part_scatter<<<dim3((unsigned)g.nb), dim3(PT_THREADS), 0, s>>>(e->flow_plain ? nullptr : fkey, src,
                                                                           B.sval->as<uint64_t>(), n, g.finvalid, g.lb,
                                                                           g.pbits, hist, g.nb, g.nparts, g.F);
    });
    HIP_OK(hipGetLastError());
    return 0;
}

// The back of a partition batch: sort + decide per half range, oversized halves, hot flows.
static int part_back(sentinel_engine_t *e, const PartBufs &B, int64_t n, const Event *ev, const uint8_t *fl,
                     uint64_t *out, hipStream_t s, uint32_t *oseq = nullptr) {
    const PartGeo g = part_geo(e, n);
    uint32_t *rstart = B.pscan->as<uint32_t>() + (size_t)g.ng * g.nparts;
    const EventSrc src{ev, nullptr, fl, false};
    const KeyTable FT = e->table(e->ft, NEV, 0);
    Verdicts V{out, B.fkey->as<uint32_t>(), g.finvalid};
    V.oseq = oseq;
    uint32_t *ctl = B.runs->as<uint32_t>();
    unsigned long long *stat = B.stat->as<unsigned long long>();
    const uint64_t *pval = B.sval->as<uint64_t>();
    uint64_t *gsval = B.vtmp->as<uint64_t>();
    const int mx = e->flow_max_n;
    if (mx <= 2) launch_part_decide<2>(e, g.nparts, FT, rstart, g.lb, src, V, n, s, ctl, stat, pval, gsval);
    else if (mx <= 4) launch_part_decide<4>(e, g.nparts, FT, rstart, g.lb, src, V, n, s, ctl, stat, pval, gsval);
    else if (mx <= 10) launch_part_decide<10>(e, g.nparts, FT, rstart, g.lb, src, V, n, s, ctl, stat, pval, gsval);
    else launch_part_decide<16>(e, g.nparts, FT, rstart, g.lb, src, V, n, s, ctl, stat, pval, gsval);
    HIP_OK(hipGetLastError());
    return 0;
}

// the rejected-event counters of decide-order batches (two, alternating per batch: each batch's prep
// clears the other one)
static int ensure_octr(sentinel_engine_t *e, hipStream_t s) {
    if (e->d_octr.p) return 0;
    if (e->d_octr.ensure(64)) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemsetAsync(e->d_octr.p, 0, 64, s));
    e->opar = 0;
    return 0;
}

static int submit_flow_part(sentinel_engine_t *e, int64_t n, const Event *ev, const uint8_t *fl, uint64_t *out,
                            hipStream_t s, uint32_t *oseq = nullptr) {
    const PartBufs B = e->part_bufs();
    if (oseq && ensure_octr(e, s)) return SENTINEL_E_NOMEM;
    int rc = part_front(e, B, n, ev, fl, out, s, oseq);
    if (rc) return rc;
    rc = part_back(e, B, n, ev, fl, out, s, oseq);
    if (oseq) e->opar ^= 1u;
    return rc;
}

// Partition-local path for this batch?  (Windows of <= 16 buckets, <= 2^20 flows; auto picks it for
// large flow tables and falls back to the radix sort for 1024 batches after a skewed one: a hot flow
// serialises its range's workgroup.  Namespace limiters run their pass first, in part_front.)
static bool choose_part(sentinel_engine_t *e, int64_t n) {
    const int32_t F = (int32_t)e->rules.size();
    const bool lim = e->nlimiters > 0 && !e->flow_plain;
    (void)lim;                          // (namespace limiters: the limiter pass runs first, part_front)
    bool part = F > 0 && e->flow_max_n <= 16 && bits_for(F) <= 2 * PART_MAX_BITS &&
                (e->flow_path == 2 || (e->flow_path == 0 && F >= 32768));
    const int64_t batch = e->flow_batches++;
    if (part && e->flow_path == 0) {
        if (batch < e->sorted_until) {
            part = false;
        } else if (e->h_part_stat) {
            const int lb = std::max(0, bits_for(F) - PART_MAX_BITS);
            const int64_t nparts = ((int64_t)F + (1 << lb) - 1) >> lb;
            const uint64_t seen = *(volatile unsigned long long *)e->h_part_stat;
            if ((double)seen > 8.0 * (double)n / (double)nparts + 4096.0) {
                e->sorted_until = batch + 1024;
                *(volatile unsigned long long *)e->h_part_stat = 0;
                part = false;
            }
        }
    }
    return part;
}

static int submit_flow_sorted(sentinel_engine_t *e, int64_t n, const Event *ev, const uint8_t *fl, uint64_t *out,
                              hipStream_t s, uint32_t *oseq = nullptr) {
    const int32_t F = (int32_t)e->rules.size();
    const int fbits = bits_for(F);
    const uint32_t finvalid = ((uint32_t)1 << fbits) - 1;
    const bool lim = e->nlimiters > 0 && !e->flow_plain;
    uint32_t *fkey = e->w_fkey.as<uint32_t>();
    if (lim) oseq = nullptr;                              // (decide order only without namespace limiters)
    if (oseq && ensure_octr(e, s)) return SENTINEL_E_NOMEM;
    if (lim) {
        e->limiter_pass(n, ev, F, fkey, finvalid, 0, out, s);
        e->hist_pass0(fkey, n, e->w_fhist.as<uint32_t>(), s);   // the limiter invalidated some keys
    } else {
        const int64_t nb = sort_blocks(n);
        // (nvalid / nseg: the fused segment kernel always writes both)
        if (!e->fused_segments) HIP_OK(hipMemsetAsync(e->w_counters.p, 0, 16, s));
        e->launch("flow_prep", n, s, [&] {
            k_flow_prep<<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(
                n, ev, F, e->flow_plain ? nullptr : e->d_flow_route.as<int32_t>(), out, fkey, finvalid, 1,
                e->w_fhist.as<uint32_t>(), nullptr, 0, 1, nullptr, nb, e->flow_plain ? nullptr : e->route8(),
                oseq, oseq ? e->d_octr.as<uint32_t>() : nullptr, e->opar);
        });
    }
    Verdicts V{out, fkey, finvalid};
    V.oseq = oseq;                                        // (sorted positions: obase 0)
    EventSrc src{ev, nullptr, fl, false};
    if (F > 0) {
        KeyTable FT = e->table(e->ft, NEV, 0);
        e->run_pipeline(FT, fkey, e->w_fhist.as<uint32_t>(), n, fbits, src, V, s, e->flow_max_n, false, true);
    }
    if (oseq) e->opar ^= 1u;
    HIP_OK(hipGetLastError());
    return 0;
}

// The one-launch small-batch kernel applies: flow rules, no namespace limiter (a limiter couples
// flows: the sorted path's limiter pass), windows of <= 16 buckets; auto picks it up to SM_MAX events.
static bool small_ok(const sentinel_engine_t *e) {
    const bool lim = e->nlimiters > 0 && !e->flow_plain;
    return !lim && !e->rules.empty() && e->flow_max_n <= 16 && (e->flow_path == 0 || e->flow_path == 3);
}

// n <= SM_MAX events (device or pinned host pointers) in one launch on s; `done` (pinned, optional)
// is set to 1 by the kernel once the verdicts are visible to the host.
static int launch_small(sentinel_engine_t *e, int64_t n, const Event *ev, const uint8_t *fl, uint64_t *out,
                        hipStream_t s, uint32_t *done = nullptr) {
    const KeyTable FT = e->table(e->ft, NEV, 0);
    const int32_t F = (int32_t)e->rules.size();
    const int32_t *route = e->flow_plain ? nullptr : e->d_flow_route.as<int32_t>();
    const int mx = e->flow_max_n;
    const EventSrc src{ev, nullptr, fl, false};
    e->launch("small", n, s, [&] {
        if (mx <= 2) k_small_flow<2><<<1, SM_THREADS, 0, s>>>(FT, (uint32_t)n, src, out, F, route, done);
        else if (mx <= 4) k_small_flow<4><<<1, SM_THREADS, 0, s>>>(FT, (uint32_t)n, src, out, F, route, done);
        else if (mx <= 10) k_small_flow<10><<<1, SM_THREADS, 0, s>>>(FT, (uint32_t)n, src, out, F, route, done);
        else k_small_flow<16><<<1, SM_THREADS, 0, s>>>(FT, (uint32_t)n, src, out, F, route, done);
    });
    HIP_OK(hipGetLastError());
    return 0;
}

// Wait for a completion flag set by k_small_flow: poll the pinned word (a few us after the kernel's
// last store, where a stream synchronisation costs tens of us of wake-up), checking the stream for a
// device error now and then.
static int wait_done(sentinel_engine_t *e, const uint32_t *flag) {
    for (uint64_t it = 1;; ++it) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE)) return 0;
        __builtin_ia32_pause();
        if ((it & 0xFFFF) == 0) {
            const hipError_t q = hipStreamQuery(e->stream);
            if (q == hipSuccess) {                   // the stream drained: the flag must be set now
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE)) return 0;
                return fail(SENTINEL_E_DEVICE, "small batch finished without its completion flag");
            }
            if (q != hipErrorNotReady) return fail(SENTINEL_E_DEVICE, hipGetErrorString(q));
        }
    }
}

// A device submit on a caller's stream is ordered after everything already queued on the engine
// stream (a batcher's or the wire server's small-batch kernels: the engine lock does not wait for
// them) and before whatever the engine stream runs next -- one event each way.
struct ForeignStream {
    sentinel_engine_t *e;
    hipStream_t s;
    ForeignStream(sentinel_engine_t *e_, hipStream_t s_) : e(e_), s(s_) {
        if (s != e->stream) join(e->stream, s);
    }
    ~ForeignStream() {
        if (s != e->stream) join(s, e->stream);
    }
    void join(hipStream_t from, hipStream_t to) {
        hipEvent_t ev = e->get_ev();
        if (ev && hipEventRecord(ev, from) == hipSuccess) (void)hipStreamWaitEvent(to, ev, 0);
        if (ev) e->ev_pool.push_back(ev);
    }
};

// A kernel gave up a bounded spin (MI355X_MICROARCH.md: every spin bounded): the batch it belonged to has
// invalid results.  [1]: the concurrency scan's look-back waited past its bound (cannot happen with
// ticket-ordered tiles; a guard, not a path).  Reported where the batch's results are
// handed back -- every synchronous (host) entry point after its synchronisation, and
// sentinel_synchronize for batches submitted on device pointers -- so the caller never uses them; a
// flag still set at the next submit (an asynchronous caller that did not synchronise) fails that submit.
static int dev_err_synced(sentinel_engine_t *e) {
    if (!e->h_dev_err) return 0;
    const uint32_t conc = __atomic_load_n(&e->h_dev_err[1], __ATOMIC_ACQUIRE);
    const uint32_t lb = __atomic_load_n(&e->h_dev_err[2], __ATOMIC_ACQUIRE);
    if (!conc && !lb) return 0;
    e->h_dev_err[1] = 0;
    e->h_dev_err[2] = 0;
    if (conc) return fail(SENTINEL_E_DEVICE, "concurrency scan: look-back timed out (the batch's results are invalid)");
    return fail(SENTINEL_E_DEVICE, lb == 2 ? "look-back: tile ticket outside the grid (the batch's results are invalid)"
                                           : "look-back timed out (the batch's results are invalid)");
}

static int check_dev_err(sentinel_engine_t *e, hipStream_t s) {
    if (!e->h_dev_err) return 0;
    if (!__atomic_load_n(&e->h_dev_err[1], __ATOMIC_ACQUIRE) && !__atomic_load_n(&e->h_dev_err[2], __ATOMIC_ACQUIRE))
        return 0;
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipStreamSynchronize(e->stream));
    return dev_err_synced(e);
}

static int submit_flow(sentinel_engine_t *e, int64_t n, const Event *ev, const uint8_t *fl, uint64_t *out,
                       hipStream_t s) {
    if (n <= 0) return 0;
    if (n > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch too large (max 2^28 events)");
    if (int rc0 = check_dev_err(e, s)) return rc0;
    if (small_ok(e) && (n <= SM_MAX || e->flow_path == 3)) {
        // consecutive chunks decided in order = the whole batch decided in arrival order
        for (int64_t off = 0; off < n; off += SM_MAX) {
            const int rc = launch_small(e, std::min<int64_t>(SM_MAX, n - off), ev + off, fl ? fl + off : nullptr,
                                        out + off, s);
            if (rc) return rc;
        }
        e->flow_path_count[0] += 1;
        return 0;
    }
    int rc = e->ensure_ws(n);
    if (rc) return rc;
    if (choose_part(e, n)) return submit_flow_part(e, n, ev, fl, out, s);
    e->flow_path_count[1] += 1;
    return submit_flow_sorted(e, n, ev, fl, out, s);
}

__global__ void k_iota_u32(uint32_t *p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}

// Decide-order output (sentinel_submit_flow_batch_ordered): the same decisions and counters as
// submit_flow, with out[j] = the verdict of the event at arrival position oseq[j] (a permutation of
// [0, n)).  The partition path writes each half range's verdicts to its own positions -- whole lines
// instead of 8.4M random 8-byte sectors -- and the arrival positions from its sorted values; a batch the
// partition path does not take (small batches, the radix path after a skewed batch, namespace limiters)
// is decided in arrival order and oseq = identity.  The consumer (the batcher, the wire server) answers
// each request from (oseq[j], out[j]): no arrival-order permutation on the device.
static int submit_flow_ordered(sentinel_engine_t *e, int64_t n, const Event *ev, const uint8_t *fl, uint64_t *out,
                               uint32_t *oseq, hipStream_t s) {
    if (n <= 0) return 0;
    if (n > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch too large (max 2^28 events)");
    if (int rc0 = check_dev_err(e, s)) return rc0;
    const bool lim = e->nlimiters > 0 && !e->flow_plain;
    if (!(small_ok(e) && (n <= SM_MAX || e->flow_path == 3)) && !lim) {
        int rc = e->ensure_ws(n);
        if (rc) return rc;
        e->flow_path_count[3] += 1;
        if (choose_part(e, n)) return submit_flow_part(e, n, ev, fl, out, s, oseq);
        e->flow_path_count[1] += 1;
        return submit_flow_sorted(e, n, ev, fl, out, s, oseq);
    } else {
        int rc = submit_flow(e, n, ev, fl, out, s);
        if (rc) return rc;
    }
    k_iota_u32<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(oseq, n);
    HIP_OK(hipGetLastError());
    return 0;
}

static int submit_prules(sentinel_engine_t *e, int mode, int64_t n, const ParamEvent *pev, const MultiEvent *mev,
                         const uint64_t *values, int64_t n_values, uint64_t *out, hipStream_t s,
                         const uint8_t *kinds = nullptr);

// Single-value exact requests without namespace limiters: the partition-local path (param_part.hpp):
// prep + range histogram, the partition scan, the stable multi-split by key hash, then one workgroup
// per range deciding its distinct keys from an LDS-staged table.
static int submit_param_part(sentinel_engine_t *e, int64_t n, const ParamEvent *ev, uint64_t *out, hipStream_t s,
                             uint32_t *oseq = nullptr) {
    if (oseq && ensure_octr(e, s)) return SENTINEL_E_NOMEM;
    const int32_t R = (int32_t)e->prules.size();
    const bool have = R > 0 && e->d_ptable.p;
    int pbits = 0;                                        // ranges of ~PD_TARGET requests, <= PART_BINS
    while (pbits < PART_MAX_BITS && ((int64_t)2 << pbits) * PD_TARGET <= n) ++pbits;
    const int32_t P = 1 << pbits;
    const int64_t nb = part_blocks(n), ng = (nb + PS_GROUP - 1) / PS_GROUP;
    int rc = e->w_fhist.ensure((size_t)nb * P * 4);
    rc |= e->w_pscan.ensure(((size_t)ng * P + 2 * (size_t)P + 1) * 4);
    if (rc) return rc;
    uint32_t *hist = e->w_fhist.as<uint32_t>();
    uint32_t *gsum = e->w_pscan.as<uint32_t>();
    uint32_t *rstart = gsum + (size_t)ng * P;
    uint32_t *rtot = rstart + P + 1;
    const int32_t *route = e->param_plain ? nullptr : e->d_prule_route.as<int32_t>();
    e->launch("param_prep", n, s, [&] {
        k_pp_prep<<<dim3((unsigned)nb), dim3(PP_THREADS), 0, s>>>(n, ev, have ? R : 0, route, e->param_ctx().R, out,
                                                                  pbits, hist, P, e->w_counters.as<uint32_t>(), nullptr,
                                                                  oseq, oseq ? e->d_octr.as<uint32_t>() : nullptr, e->opar);
    });
    if (oseq) e->opar ^= 1u;                              // (the next decide-order batch's counter, zeroed by this prep)
    if (!have) {
        HIP_OK(hipGetLastError());
        return 0;
    }
    e->launch("scan", n, s, [&] {
        const dim3 g2((unsigned)ng, (unsigned)((P + PS_THREADS - 1) / PS_THREADS));
        k_part_colsum<<<g2, PS_THREADS, 0, s>>>(hist, nb, P, gsum);
        k_part_colscan<<<(unsigned)((P + PC_THREADS / WAVE - 1) / (PC_THREADS / WAVE)), PC_THREADS, 0, s>>>(gsum, ng, P,
                                                                                                          rtot);
        k_part_offsets<<<g2, PS_THREADS, 0, s>>>(hist, nb, P, gsum, rtot, rstart);
    });
    unsigned long long *pkey = e->w_vtmp.as<unsigned long long>();
    uint64_t *pval = e->w_sval.as<uint64_t>();
    int32_t *prule = e->w_fkey.as<int32_t>();
    e->launch("param_scatter", n, s, [&] {
        k_pp_scatter<<<dim3((unsigned)nb), dim3(PT_THREADS), 0, s>>>(ev, n, R, route, pbits, hist, P, pkey, pval, prule);
    });
    uint32_t *pexp = e->d_pexpire.bytes >= e->pcap * 4 ? e->d_pexpire.as<uint32_t>() : nullptr;
    const PSlots S{e->d_ptable.as<unsigned long long>(), e->d_slot_rule.as<int32_t>(), e->pt.state.as<int64_t>(),
                   param_stride(e->pmax_n), e->pcap - 1, pexp};
    const ParamRules PR = e->param_ctx().R;
    if (e->prec_dirty || e->d_prule_rec.bytes < (size_t)R * sizeof(PRuleRec)) {
        if (e->d_prule_rec.ensure((size_t)R * sizeof(PRuleRec))) return SENTINEL_E_NOMEM;
        k_prule_pack<<<(unsigned)((R + 255) / 256), 256, 0, s>>>(R, PR, e->d_prule_hot.p ? e->d_prule_hot.as<uint8_t>() : nullptr,
                                                                e->d_prule_rec.as<PRuleRec>());
        e->prec_dirty = false;
    }
    const PRuleRec *RR = e->d_prule_rec.as<PRuleRec>();
    unsigned long long *fresh = e->d_pfresh.as<unsigned long long>();
    // sub-ranges of <= PG_TARGET requests on average: one LDS chunk each (XCD-aware grid, k_pp_group)
    int sbits = 0;
    while (sbits < 8 && (int64_t)P * ((int64_t)1 << sbits) * PG_TARGET < n) ++sbits;
    const unsigned ggrid = (unsigned)(((P + 7) / 8) * 8 * (1 << sbits));
    uint64_t *gval = e->w_hep.as<uint64_t>();
    PKeyRecs RC{e->w_segep.as<unsigned long long>(), e->w_s0.as<uint2>(), e->w_k.as<int32_t>(),
                e->w_counters.as<uint32_t>(), nullptr};
    RC.oseq = oseq;
    const int hb = header_block_slots(e->pmax_n);
    e->launch("param_group", n, s, [&] {
        if (hb <= 2) k_pp_group<2><<<ggrid, PD_THREADS, 0, s>>>(pkey, pval, prule, rstart, P, pbits, sbits, ev, PR, RR, S, out, fresh, gval, RC);
        else if (hb <= 4) k_pp_group<4><<<ggrid, PD_THREADS, 0, s>>>(pkey, pval, prule, rstart, P, pbits, sbits, ev, PR, RR, S, out, fresh, gval, RC);
        else if (hb <= 10) k_pp_group<10><<<ggrid, PD_THREADS, 0, s>>>(pkey, pval, prule, rstart, P, pbits, sbits, ev, PR, RR, S, out, fresh, gval, RC);
        else k_pp_group<16><<<ggrid, PD_THREADS, 0, s>>>(pkey, pval, prule, rstart, P, pbits, sbits, ev, PR, RR, S, out, fresh, gval, RC);
    });
    e->launch("param_decide", n, s, [&] {
        const unsigned wg = (unsigned)std::min<int64_t>(2048, (n + 255) / 256);
        if (hb <= 2) k_pp_walk<2><<<wg, 256, 0, s>>>(RC, gval, ev, PR, RR, S, out, fresh);
        else if (hb <= 4) k_pp_walk<4><<<wg, 256, 0, s>>>(RC, gval, ev, PR, RR, S, out, fresh);
        else if (hb <= 10) k_pp_walk<10><<<wg, 256, 0, s>>>(RC, gval, ev, PR, RR, S, out, fresh);
        else k_pp_walk<16><<<wg, 256, 0, s>>>(RC, gval, ev, PR, RR, S, out, fresh);
    });
    if (!e->h_pfresh) {
        HIP_OK(hipHostMalloc((void **)&e->h_pfresh, 16, 0));
        e->h_pfresh[0] = ~0ull;
        e->h_pfresh[1] = 0;
    }
    k_pfresh_publish<<<1, WAVE, 0, s>>>(fresh, e->p_ord - 1, e->h_pfresh);
    HIP_OK(hipGetLastError());
    return 0;
}

// Single-value requests on the shared count-min sketch without namespace limiters: the partition-local
// grouping (k_pp_prep -> scan -> k_pp_scatter -> k_pp_group, emit only), then the two-phase key walk
// (k_pp_cm_read: every read of the batch; k_pp_cm_walk: decisions and adds; param_part.hpp).  One
// synchronisation reads whether every sub-range fit one chunk; a batch with a sub-range over PG_CAP
// requests (heavy skew: a key split over chunks) is decided by the per-rule lanes (submit_prules),
// which answer the invalid requests the same way.  Returns 1 = fall back.
static int submit_param_cm_part(sentinel_engine_t *e, int64_t n, const ParamEvent *ev, uint64_t *out, hipStream_t s,
                                uint32_t *oseq = nullptr) {
    const int32_t R = (int32_t)e->prules.size();
    if (R == 0 || !e->d_cmband.p) return 1;
    if (oseq && ensure_octr(e, s)) return SENTINEL_E_NOMEM;
    int pbits = 0;
    while (pbits < PART_MAX_BITS && ((int64_t)2 << pbits) * PD_TARGET <= n) ++pbits;
    const int32_t P = 1 << pbits;
    const int64_t nb = part_blocks(n), ng = (nb + PS_GROUP - 1) / PS_GROUP;
    int rc = e->w_fhist.ensure((size_t)nb * P * 4);
    rc |= e->w_pscan.ensure(((size_t)ng * P + 2 * (size_t)P + 1) * 4);
    if (rc) return rc;
    if (!e->h_cmband) HIP_OK(hipHostMalloc((void **)&e->h_cmband, 64, 0));
    uint32_t *hist = e->w_fhist.as<uint32_t>();
    uint32_t *gsum = e->w_pscan.as<uint32_t>();
    uint32_t *rstart = gsum + (size_t)ng * P;
    uint32_t *rtot = rstart + P + 1;
    unsigned long long *flag = e->d_cmband.as<unsigned long long>();          // [0] overflow
    long long *ctl = e->d_cmband.as<long long>() + 1;                          // [1..3] E_hi, E_hi seen, emax
    const int32_t *route = e->param_plain ? nullptr : e->d_prule_route.as<int32_t>();
    const ParamCtx C = e->param_ctx();
    unsigned long long *tspan = flag + 5;                                      // [5..6] the batch's ts range
    // the overflow flag (set by k_pp_group), the ts range (k_pp_prep) and the walk's newest epoch, reset
    // by one launch
    k_cm_batch_init<<<1, 64, 0, s>>>(flag, tspan, ctl);
    e->launch("param_prep", n, s, [&] {
        k_pp_prep<<<dim3((unsigned)nb), dim3(PP_THREADS), 0, s>>>(n, ev, R, route, C.R, out, pbits, hist, P,
                                                                  e->w_counters.as<uint32_t>(), tspan, oseq,
                                                                  oseq ? e->d_octr.as<uint32_t>() : nullptr, e->opar);
    });
    if (oseq) e->opar ^= 1u;                              // (the next decide-order batch's counter, zeroed by this prep)
    e->launch("scan", n, s, [&] {
        const dim3 g2((unsigned)ng, (unsigned)((P + PS_THREADS - 1) / PS_THREADS));
        k_part_colsum<<<g2, PS_THREADS, 0, s>>>(hist, nb, P, gsum);
        k_part_colscan<<<(unsigned)((P + PC_THREADS / WAVE - 1) / (PC_THREADS / WAVE)), PC_THREADS, 0, s>>>(gsum, ng, P,
                                                                                                          rtot);
        k_part_offsets<<<g2, PS_THREADS, 0, s>>>(hist, nb, P, gsum, rtot, rstart);
    });
    unsigned long long *pkey = e->w_vtmp.as<unsigned long long>();
    uint64_t *pval = e->w_sval.as<uint64_t>();
    int32_t *prule = e->w_fkey.as<int32_t>();
    e->launch("param_scatter", n, s, [&] {
        k_pp_scatter<<<dim3((unsigned)nb), dim3(PT_THREADS), 0, s>>>(ev, n, R, route, pbits, hist, P, pkey, pval, prule);
    });
    if (e->prec_dirty || e->d_prule_rec.bytes < (size_t)R * sizeof(PRuleRec)) {
        if (e->d_prule_rec.ensure((size_t)R * sizeof(PRuleRec))) return SENTINEL_E_NOMEM;
        k_prule_pack<<<(unsigned)((R + 255) / 256), 256, 0, s>>>(R, C.R, e->d_prule_hot.p ? e->d_prule_hot.as<uint8_t>() : nullptr,
                                                                e->d_prule_rec.as<PRuleRec>());
        e->prec_dirty = false;
    }
    const PRuleRec *RR = e->d_prule_rec.as<PRuleRec>();
    // sub-ranges of <= PG_CAP / 2 requests on average: a sub-range over PG_CAP (which sends the batch to
    // the per-rule lanes) is then a > 2x deviation (at PG_TARGET = 0.8 PG_CAP, Zipf-heavy keys made it
    // about one sub-range per 4M-request batch)
    int sbits = 0;
    while (sbits < 8 && (int64_t)P * ((int64_t)1 << sbits) * (PG_CAP / 2) < n) ++sbits;
    // block-owned walk (k_pp_cm_block) when a sketch block fits LDS; sub-ranges are made narrow enough
    // (up to 2^8 per range) that one spans at most 4 blocks
    const size_t blk_bytes = (size_t)C.CM.depth * C.CM.cols * (size_t)C.CM.nmax * 8;
    // (and at least 16 blocks: a narrower sketch would leave the batch to a handful of workgroups)
    bool use_block = e->cm_block && C.CM.shared && C.CM.depth <= 4 && blk_bytes <= 49152 && e->pmax_n <= 16 &&
                     C.CM.cbits >= 4;
    if (use_block)
        while (sbits < 8 && pbits + sbits + 2 < C.CM.cbits) ++sbits;
    const int sb = pbits + sbits;
    use_block = use_block && sb + 2 >= C.CM.cbits;
    if (e->cm_debug)
        fprintf(stderr, "[sentinel] cm key walk: n=%lld pbits=%d sbits=%d cbits=%d cols=%u depth=%d nmax=%d pmax_n=%d "
                        "shared=%d blk_bytes=%zu block=%d\n", (long long)n, pbits, sbits, C.CM.cbits, C.CM.cols,
                C.CM.depth, C.CM.nmax, e->pmax_n, (int)C.CM.shared, blk_bytes, (int)use_block);
    const unsigned ggrid = (unsigned)(((P + 7) / 8) * 8 * (1 << sbits));
    uint64_t *gval = e->w_hep.as<uint64_t>();
    if (use_block && e->w_cmsub.ensure(((size_t)P << sbits) * sizeof(uint2))) return SENTINEL_E_NOMEM;
    PKeyRecs RC{e->w_segep.as<unsigned long long>(), e->w_s0.as<uint2>(), e->w_k.as<int32_t>(),
                e->w_counters.as<uint32_t>(), flag};
    RC.oseq = oseq;
    if (use_block) RC.sub = e->w_cmsub.as<uint2>();
    const PSlots S{};
    e->launch("param_group", n, s, [&] {
        k_pp_group<2, true, 10><<<ggrid, PD_THREADS, 0, s>>>(pkey, pval, prule, rstart, P, pbits, sbits, ev, C.R, RR, S, out,
                                                         nullptr, gval, RC);
    });
    HIP_OK(hipMemcpyAsync(e->h_cmband, flag, 56, hipMemcpyDeviceToHost, s));   // the flag, ..., the ts range
    HIP_OK(hipStreamSynchronize(s));
    if (e->h_cmband[0] != 0ull) {
        ++e->cm_overflows;
        return 1;
    }
    // 32-bit LDS cells (tags mod 256 around Eref = max(the batch's newest epoch, E_hi), cm_eref) when every
    // age the batch needs -- from Eref back to its oldest epoch less 2n -- is < 200 epochs
    const int32_t wsk = e->h_prule_interval.empty() ? 1 : std::max(1, e->h_prule_interval[0] / std::max(1, e->h_prule_n[0]));
    const int64_t tlo = (int64_t)e->h_cmband[5], thi = (int64_t)~e->h_cmband[6];
    const int64_t ehi = (int64_t)e->h_cmband[1];          // E_hi (ctl[0]) as the grouping left it
    const int64_t eref = (ehi != CM_EHI_NONE && ehi != CM_EHI_ANY && ehi > thi / wsk) ? ehi : thi / wsk;
    const bool c32 = use_block && e->cm_c32 && tlo >= 0 && thi >= tlo &&
                     eref - tlo / wsk + 2 * (int64_t)e->pmax_n < 200;
    ++e->cm_key_batches;
    const int32_t nsc = e->pmax_n;
    int64_t *mv = e->w_sval.as<int64_t>();                // (the packed values are dead after the grouping)
    if (use_block) {
        ++e->cm_block_batches;                            // (ctl[2] reset by k_cm_batch_init)
        e->launch("param_cm_block", n, s, [&] {
            const dim3 g(1u << C.CM.cbits);
            // (SENTINEL_CM_DIAG bits 6 / 7: 24 / 56 KB of unused LDS per workgroup -- an occupancy diagnostic)
            const size_t pad = (e->cm_diag & 64) ? 24576 : (e->cm_diag & 128) ? 57344 : 0;
            if (c32)
                k_pp_cm_block<true><<<g, 256, blk_bytes / 2 + pad, s>>>(RC, sb, gval, ev, C.R, RR, C.CM, mv, ctl, tspan,
                                                                        out, wsk, 1.0 / (double)wsk, e->cm_diag & 63);
            else
                k_pp_cm_block<false><<<g, 256, blk_bytes + pad, s>>>(RC, sb, gval, ev, C.R, RR, C.CM, mv, ctl, tspan,
                                                                         out, wsk, 1.0 / (double)wsk, e->cm_diag & 63);
        });
        k_pp_cm_ehi<<<1, 64, 0, s>>>(ctl);
        HIP_OK(hipGetLastError());
        return 0;
    }
    const unsigned wg = (unsigned)std::min<int64_t>(2048, (n + 255) / 256);
    const bool d4 = C.CM.depth <= 4;
    e->launch("param_cm_read", n, s, [&] {
        if (d4 && nsc <= 2) k_pp_cm_read<2, 4><<<wg, 256, 0, s>>>(RC, gval, ev, RR, C.CM, mv, ctl);
        else if (d4 && nsc <= 4) k_pp_cm_read<4, 4><<<wg, 256, 0, s>>>(RC, gval, ev, RR, C.CM, mv, ctl);
        else if (d4 && nsc <= 10) k_pp_cm_read<10, 4><<<wg, 256, 0, s>>>(RC, gval, ev, RR, C.CM, mv, ctl);
        else if (d4) k_pp_cm_read<16, 4><<<wg, 256, 0, s>>>(RC, gval, ev, RR, C.CM, mv, ctl);
        else if (nsc <= 4) k_pp_cm_read<4, 16><<<wg, 256, 0, s>>>(RC, gval, ev, RR, C.CM, mv, ctl);
        else k_pp_cm_read<16, 16><<<wg, 256, 0, s>>>(RC, gval, ev, RR, C.CM, mv, ctl);
    });
    e->launch("param_cm_walk", n, s, [&] {
        if (d4 && nsc <= 2) k_pp_cm_walk<2, 4><<<wg, 256, 0, s>>>(RC, gval, ev, C.R, RR, C.CM, mv, ctl, tspan, out);
        else if (d4 && nsc <= 4) k_pp_cm_walk<4, 4><<<wg, 256, 0, s>>>(RC, gval, ev, C.R, RR, C.CM, mv, ctl, tspan, out);
        else if (d4 && nsc <= 10) k_pp_cm_walk<10, 4><<<wg, 256, 0, s>>>(RC, gval, ev, C.R, RR, C.CM, mv, ctl, tspan, out);
        else if (d4) k_pp_cm_walk<16, 4><<<wg, 256, 0, s>>>(RC, gval, ev, C.R, RR, C.CM, mv, ctl, tspan, out);
        else if (nsc <= 4) k_pp_cm_walk<4, 16><<<wg, 256, 0, s>>>(RC, gval, ev, C.R, RR, C.CM, mv, ctl, tspan, out);
        else k_pp_cm_walk<16, 16><<<wg, 256, 0, s>>>(RC, gval, ev, C.R, RR, C.CM, mv, ctl, tspan, out);
    });
    k_pp_cm_ehi<<<1, 64, 0, s>>>(ctl);
    HIP_OK(hipGetLastError());
    return 0;
}

// oseq (decide-order output): the key walks write grouped positions + arrival positions (ord_done =
// true); every other path writes arrival order and the caller makes oseq the identity.
static int submit_param_impl(sentinel_engine_t *e, int64_t n, const ParamEvent *ev, uint64_t *out, hipStream_t s,
                             uint32_t *oseq, bool &ord_done) {
    if (e->pmode == SENTINEL_PARAM_COUNT_MIN_SHARED && e->cm_keys && n > 0 && n <= MAX_BATCH && e->pmax_n <= 16 &&
        !(e->nlimiters > 0 && !e->param_plain)) {
        int rc = e->ensure_ws(n);
        if (rc) return rc;
        rc = submit_param_cm_part(e, n, ev, out, s, oseq);
        if (rc != 1) {
            ord_done = oseq != nullptr;
            return rc;
        }
    }
    if (e->pmode != SENTINEL_PARAM_EXACT) return submit_prules(e, PMODE_CM, n, ev, nullptr, nullptr, 0, out, s);
    // per-rule walk (sort by rule, one lane per rule, each request rolls and sums its value's slot): for
    // many (rule, value) keys with a few requests each spread over many epochs, where the per-slot
    // segment pipeline below builds one segment record per request
    if (e->param_path == 1) return submit_prules(e, PMODE_EXACT, n, ev, nullptr, nullptr, 0, out, s);
    if (n <= 0) return 0;
    if (n > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch too large (max 2^28 events)");
    int rc = e->ensure_ws(n);
    if (rc) return rc;
    const int32_t R = (int32_t)e->prules.size();
    if (R > 0 && e->d_ptable.p) {
        if (s != e->stream) HIP_OK(hipStreamSynchronize(s));
        rc = e->param_reserve(n);             // room for every value of the batch: never FAIL
        if (rc) return rc;
    }
    const bool plim = e->nlimiters > 0 && !e->param_plain && R > 0;
    if (e->param_path == 0 && !plim && e->pmax_n <= 16) {
        ord_done = oseq != nullptr;
        return submit_param_part(e, n, ev, out, s, oseq);
    }
    e->pexp_valid = false;                                // (the segment pipeline does not keep the hints)
    const uint64_t P = e->pcap;
    const int pbits = bits_for((int64_t)P);
    const uint32_t pinvalid = ((uint32_t)1 << pbits) - 1;
    const bool lim = e->nlimiters > 0 && !e->param_plain && R > 0;
    const int lbits = bits_for(e->nlimiters);
    const uint32_t linvalid = ((uint32_t)1 << lbits) - 1;
    uint32_t *fkey = e->w_fkey.as<uint32_t>();
    uint32_t *lkey = lim ? e->w_lkey.as<uint32_t>() : nullptr;
    const int64_t nb = sort_blocks(n);
    const bool have = R > 0 && e->d_ptable.p;
    HIP_OK(hipMemsetAsync(e->w_counters.p, 0, 16, s));
    e->launch("param_prep", n, s, [&] {
        k_param_prep<<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(
            n, ev, have ? R : 0, e->param_plain ? nullptr : e->d_prule_route.as<int32_t>(),
            e->d_ptable.as<unsigned long long>(), P - 1, e->d_slot_rule.as<int32_t>(), e->param_ctx().R,
            e->slot_meta(), e->d_pfresh.as<unsigned long long>(), out, fkey, pinvalid,
            1, e->w_fhist.as<uint32_t>(), lkey, linvalid, 1, e->w_lhist.as<uint32_t>(), nb);
    });
    if (!have) {
        HIP_OK(hipGetLastError());
        return 0;
    }
    if (e->pmeta_dirty) {                  // rules / thresholds / table changed since the last batch
        e->launch("param_meta", n, s, [&] {
            k_param_meta_all<<<grid_for((int64_t)P), 256, 0, s>>>(P, e->d_ptable.as<unsigned long long>(),
                                                                  e->d_slot_rule.as<int32_t>(), R, e->param_ctx().R,
                                                                  e->slot_meta());
        });
        e->pmeta_dirty = false;
    }
    Verdicts V{out, fkey, pinvalid};
    if (lim) {
        KeyTable LT = e->table(e->lt, 1, e->lim_stride);
        EventSrc lsrc{nullptr, ev, nullptr, true};
        e->run_pipeline(LT, lkey, e->w_lhist.as<uint32_t>(), n, lbits, lsrc, V, s, 10, true);
        e->hist_pass0(fkey, n, e->w_fhist.as<uint32_t>(), s);
    }
    KeyTable PT = e->table(e->pt, 1, param_stride(e->pmax_n));
    EventSrc src{nullptr, ev, nullptr, false};
    e->run_pipeline(PT, fkey, e->w_fhist.as<uint32_t>(), n, pbits, src, V, s, e->pmax_n, false, false, false, true);
    HIP_OK(hipGetLastError());
    return 0;
}

static int submit_param(sentinel_engine_t *e, int64_t n, const ParamEvent *ev, uint64_t *out, hipStream_t s,
                        uint32_t *oseq = nullptr) {
    if (int rc0 = check_dev_err(e, s)) return rc0;
    bool ord_done = false;
    const int rc = submit_param_impl(e, n, ev, out, s, oseq, ord_done);
    if (rc || !oseq || ord_done || n <= 0) return rc;
    k_iota_u32<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(oseq, n);
    HIP_OK(hipGetLastError());
    return 0;
}

// Hot-parameter requests decided per rule (param_rules.hpp): multi-value cluster requests (exact or
// count-min counters) and the local token bucket.  Events are single-value (pev) or multi-value
// (mev + values[0, n_values)).
static int submit_prules(sentinel_engine_t *e, int mode, int64_t n, const ParamEvent *pev, const MultiEvent *mev,
                         const uint64_t *values, int64_t n_values, uint64_t *out, hipStream_t s,
                         const uint8_t *kinds) {
    if (n <= 0) return 0;
    if (n > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch too large (max 2^28 events)");
    if (int rc0 = check_dev_err(e, s)) return rc0;
    int rc = e->ensure_ws(n);
    if (rc) return rc;
    const bool local = mode == PMODE_LOCAL;
    const int64_t nv = pev ? n : n_values;
    if (nv > ((int64_t)1 << 31) - 1) return fail(SENTINEL_E_INVALID, "too many values (max 2^31 - 1)");
    rc = e->w_vslot.ensure((size_t)std::max<int64_t>(nv, 1) * 4);
    if (rc) return rc;
    const int32_t R = local ? e->nlrules : (int32_t)e->prules.size();
    const int rbits = bits_for(R);
    const uint32_t rinvalid = ((uint32_t)1 << rbits) - 1;
    const bool lim = !local && e->nlimiters > 0 && !e->param_plain && R > 0;
    const int lbits = bits_for(e->nlimiters);
    const uint32_t linvalid = ((uint32_t)1 << lbits) - 1;
    uint32_t *fkey = e->w_fkey.as<uint32_t>();
    uint32_t *lkey = lim ? e->w_lkey.as<uint32_t>() : nullptr;
    const int64_t nb = sort_blocks(n);
    const ParamEvent *evp = pev ? pev : (const ParamEvent *)mev;
    const ValueSrc vs{pev, mev, values, nv};
    if (mode == PMODE_EXACT && R > 0) {
        if (s != e->stream) HIP_OK(hipStreamSynchronize(s));
        rc = e->param_reserve(nv);            // room for every value of the batch: never FAIL
        if (rc) return rc;
        e->pexp_valid = false;                // (the per-rule lanes do not keep the getTopValues hints)
    }
    ParamCtx C = e->param_ctx();
    C.L.kinds = local ? kinds : nullptr;
    unsigned long long *table = nullptr;
    uint64_t mask = 0;
    if (mode == PMODE_EXACT && R > 0) { table = e->d_ptable.as<unsigned long long>(); mask = e->pcap - 1; }
    if (local && R > 0) { table = e->d_ltable.as<unsigned long long>(); mask = e->lcap - 1; }
    HIP_OK(hipMemsetAsync(e->w_counters.p, 0, 16, s));
    e->launch("prule_prep", n, s, [&] {
        if (local)
            k_prule_prep<true><<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(
                n, evp, vs, R, e->d_lrule_valid.as<uint8_t>(), nullptr, C.R, table, mask, nullptr, SlotMeta{},
                e->w_vslot.as<uint32_t>(), out,
                fkey, rinvalid, e->w_fhist.as<uint32_t>(), nullptr, linvalid, e->w_lhist.as<uint32_t>(), nb);
        else
            k_prule_prep<false><<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(
                n, evp, vs, R, nullptr, e->param_plain ? nullptr : e->d_prule_route.as<int32_t>(), C.R, table, mask,
                e->d_pfresh.as<unsigned long long>(), e->slot_meta(), e->w_vslot.as<uint32_t>(), out, fkey, rinvalid, e->w_fhist.as<uint32_t>(), lkey, linvalid,
                e->w_lhist.as<uint32_t>(), nb);
    });
    if (R == 0) {
        HIP_OK(hipGetLastError());
        return 0;
    }
    if (lim) {   // ClusterParamFlowChecker.allowProceed: one limiter pass per request (CPFC:45-47)
        Verdicts V{out, fkey, rinvalid};
        KeyTable LT = e->table(e->lt, 1, e->lim_stride);
        EventSrc lsrc{nullptr, evp, nullptr, true};
        e->run_pipeline(LT, lkey, e->w_lhist.as<uint32_t>(), n, lbits, lsrc, V, s, 10, true);
        e->hist_pass0(fkey, n, e->w_fhist.as<uint32_t>(), s);
    }
    const KeyTable RT = local ? e->local_rule_table() : e->param_rule_table();
    const EventSrc src{nullptr, evp, nullptr, false};
    e->sort_segments(RT, fkey, e->w_fhist.as<uint32_t>(), n, rbits, src, s);
    const BatchWork W = e->work();
    const unsigned g = grid_for(n);
    if (mode == PMODE_CM && C.CM.shared) {
        // shared sketch: every rule's lane moves through the epochs together (k_prule_cm_sync)
        const int64_t H = std::min<int64_t>(n, R);
        const size_t cbase = ((size_t)2 * H * 4 + 255) & ~(size_t)255;   // control words after heads + cursors
        rc = e->w_cm.ensure(cbase + 256);
        if (rc) return rc;
        uint32_t *heads = e->w_cm.as<uint32_t>();
        uint32_t *cursor = heads + H;
        uint32_t *ctl = reinterpret_cast<uint32_t *>(e->w_cm.as<char>() + cbase);
        unsigned long long *lv = reinterpret_cast<unsigned long long *>(e->w_cm.as<char>() + cbase + 192);
        HIP_OK(hipMemsetAsync(ctl, 0, 192, s));            // head count, barrier arrivals and generation
        HIP_OK(hipMemsetAsync(lv, 0xFF, 8, s));            // span: min (all ones) ...
        HIP_OK(hipMemsetAsync(lv + 1, 0, 8, s));           // ... and max
        if (!e->cm_sync_blocks) {
            int per_cu = 0, cus = 0;
            HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(k_prule_cm_sync), 256, 0));
            HIP_OK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->device));
            // at most one workgroup per CU: the grid barrier's cost grows with the workgroups
            e->cm_sync_blocks = std::max(1, std::min(per_cu, 1)) * std::max(1, cus);
        }
        // the batch's epoch span: one launch per level when it is short (the kernel boundary is the
        // barrier), the cooperative kernel's grid barrier otherwise
        const unsigned hb = (unsigned)std::max<int64_t>(1, (H + 255) / 256);
        k_cm_heads<<<g, 256, 0, s>>>(W, heads, ctl);
        k_cm_span<<<hb, 256, 0, s>>>(W, heads, ctl, cursor, lv);
        unsigned long long span[2] = {~0ull, 0};
        HIP_OK(hipMemcpyAsync(span, lv, 16, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        if (e->d_cmband.p && span[0] != ~0ull) {         // the key walk's E_hi covers these adds too
            long long *ctl = e->d_cmband.as<long long>() + 1;
            k_set_i64<<<1, 64, 0, s>>>(ctl + 2, (long long)span[1]);
            k_pp_cm_ehi<<<1, 64, 0, s>>>(ctl);
        }
        if (span[0] != ~0ull && (int64_t)(span[1] - span[0]) < CM_LEVEL_LAUNCHES && !e->cm_force_coop) {
            const int band = e->pmax_n;                   // one launch per band of n epochs (ring of 2 n slots)
            e->launch("prule_process", n, s, [&] {
                for (int64_t E = (int64_t)span[0]; E <= (int64_t)span[1]; E += band)
                    k_prule_cm_level<<<hb, 256, 0, s>>>(C, W, evp, vs, out, heads, ctl, cursor, E, band,
                                                        (int64_t)span[1]);
            });
            HIP_OK(hipGetLastError());
            return 0;
        }
        HIP_OK(hipMemsetAsync(lv, 0xFF, 24, s));
        const unsigned nblk = (unsigned)std::max<int64_t>(1, std::min<int64_t>(e->cm_sync_blocks, (H + 255) / 256));
        hipError_t ce = hipSuccess;
        e->launch("prule_process", n, s, [&] {
            int band = e->pmax_n;
            int64_t eref = (int64_t)span[1];             // the batch's newest epoch (cm_slot_next's "newer" test)
            void *args[] = {(void *)&C, (void *)&W, (void *)&evp, (void *)&vs, (void *)&out, (void *)&heads, (void *)&ctl,
                            (void *)&cursor, (void *)&lv, (void *)&band, (void *)&eref};
            ce = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_prule_cm_sync), dim3(nblk), dim3(256), args, 0, s);
        });
        if (ce != hipSuccess) return fail(SENTINEL_E_DEVICE, std::string("cooperative launch failed: ") + hipGetErrorString(ce));
        HIP_OK(hipGetLastError());
        return 0;
    }
    e->launch("prule_process", n, s, [&] {
        if (mode == PMODE_LOCAL) k_prule_process<PMODE_LOCAL><<<g, 256, 0, s>>>(C, W, evp, vs, out, n);
        else if (mode == PMODE_CM) k_prule_process<PMODE_CM><<<g, 256, 0, s>>>(C, W, evp, vs, out, n);
        else k_prule_process<PMODE_EXACT><<<g, 256, 0, s>>>(C, W, evp, vs, out, n);
    });
    HIP_OK(hipGetLastError());
    return 0;
}

// Host-pointer variant of the per-rule param path: H2D, decide, D2H, synchronous.
static int submit_prules_host(sentinel_engine_t *e, int mode, int64_t n, const sentinel_param_multi_event_t *ev,
                              const uint64_t *values, int64_t n_values, sentinel_verdict_t *out,
                              const uint8_t *kinds = nullptr) {
    if (n == 0) return 0;
    hipStream_t s = e->stream;
    int rc = 0;
    rc |= e->io_ev.ensure(n * sizeof(MultiEvent));
    rc |= e->io_vals.ensure(std::max<int64_t>(n_values, 1) * 8);
    rc |= e->io_out.ensure(n * 8);
    if (kinds) rc |= e->io_fl.ensure(n);
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemcpyAsync(e->io_ev.p, ev, n * sizeof(MultiEvent), hipMemcpyHostToDevice, s));
    if (n_values > 0) HIP_OK(hipMemcpyAsync(e->io_vals.p, values, n_values * 8, hipMemcpyHostToDevice, s));
    if (kinds) HIP_OK(hipMemcpyAsync(e->io_fl.p, kinds, n, hipMemcpyHostToDevice, s));
    rc = submit_prules(e, mode, n, nullptr, e->io_ev.as<MultiEvent>(), e->io_vals.as<uint64_t>(), n_values,
                       e->io_out.as<uint64_t>(), s, kinds ? e->io_fl.as<uint8_t>() : nullptr);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, e->io_out.p, n * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return dev_err_synced(e);
}

// Local SphU.entry batches (local_entry.hpp): validation, sort by resource, (resource, epoch of
// gcd(second bucket, 1000 ms)) segments, one lane per resource, parallel verdicts.
static int submit_local_entry(sentinel_engine_t *e, int64_t n, const Event *ev, const uint8_t *fl, const int64_t *rt,
                              uint64_t *out, hipStream_t s) {
    if (n <= 0) return 0;
    if (e->lgraph) return fail(SENTINEL_E_STATE, "a local rule graph is loaded: use sentinel_submit_local_graph_batch");
    if (n > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch too large (max 2^28 events)");
    if (int rc0 = check_dev_err(e, s)) return rc0;
    int rc = e->ensure_ws(n);
    if (rc) return rc;
    const int32_t R = e->nlres;
    const int rbits = bits_for(R);
    const uint32_t rinvalid = ((uint32_t)1 << rbits) - 1;
    uint32_t *fkey = e->w_fkey.as<uint32_t>();
    const int64_t nb = sort_blocks(n);
    uint8_t *slow = nullptr;
    if (fl) {
        rc = e->w_lslow.ensure((size_t)n);
        if (rc) return rc;
        slow = e->w_lslow.as<uint8_t>();
    }
    HIP_OK(hipMemsetAsync(e->w_counters.p, 0, 16, s));
    e->launch("lentry_prep", n, s, [&] {
        k_lentry_prep<<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(n, ev, R, out, fkey, rinvalid,
                                                                        e->w_fhist.as<uint32_t>(), nb, fl, slow);
    });
    if (R == 0) {
        HIP_OK(hipGetLastError());
        return 0;
    }
    KeyTable RT{};
    RT.w = e->d_lres_w.as<int32_t>();
    RT.rcp_w = e->d_lres_rcp.as<double>();
    RT.kind = e->d_lres_kind.as<uint8_t>();
    RT.ncounters = 1;
    const EventSrc src{ev, nullptr, slow, false};
    e->sort_segments(RT, fkey, e->w_fhist.as<uint32_t>(), n, rbits, src, s);
    const BatchWork W = e->work();
    const LocalNodes L{e->d_lres_state.as<int64_t>(), e->d_lres_count.as<double>(), e->lres_n, e->lres_w, e->lres_Is,
                       e->lres_interval, e->occupy_timeout, e->d_lres_tcount.as<double>(),
                       e->d_lres_flags.as<uint8_t>(), e->lres_max_rt, fl, rt};
    e->launch("lentry_process", n, s, [&] { k_lentry_process<<<grid_for(n), 256, 0, s>>>(L, W, src, out); });
    e->launch("lentry_verdict", n, s, [&] { k_lentry_verdict<<<grid_for(n), 256, 0, s>>>(W, out, n); });
    HIP_OK(hipGetLastError());
    return 0;
}

// Local rule graph batches (local_entry.hpp, k_lgraph_*): validation, sort by the resource's RELATE
// component, one lane per component walking its events in arrival order.
static int submit_local_graph(sentinel_engine_t *e, int64_t n, const Event *ev, const LocalCtx *ctx,
                              const uint8_t *fl, const int64_t *rt, uint64_t *out, hipStream_t s) {
    if (n <= 0) return 0;
    if (n > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch too large (max 2^28 events)");
    if (!e->lgraph) return fail(SENTINEL_E_STATE, "no local rule graph loaded (sentinel_load_local_rules)");
    if (int rc0 = check_dev_err(e, s)) return rc0;
    int rc = e->ensure_ws(n);
    if (rc) return rc;
    const int32_t R = e->nlres;
    const int rbits = bits_for(R);
    const uint32_t rinvalid = ((uint32_t)1 << rbits) - 1;
    uint32_t *fkey = e->w_fkey.as<uint32_t>();
    const int64_t nb = sort_blocks(n);
    const LocalGraph G{e->d_lg_on.as<int64_t>(), e->d_lg_dn.as<int64_t>(), e->d_lg_created.as<uint8_t>(),
                       e->d_lg_roff.as<int32_t>(), e->d_lg_rules.as<LocalRule>(), ctx, e->d_lg_comp.as<uint32_t>(),
                       R, e->lg_on, e->lg_dn};
    HIP_OK(hipMemsetAsync(e->w_counters.p, 0, 16, s));
    e->launch("lgraph_prep", n, s, [&] {
        k_lgraph_prep<<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(n, ev, G, out, fkey, rinvalid,
                                                                        e->w_fhist.as<uint32_t>(), nb);
    });
    if (R == 0) {
        HIP_OK(hipGetLastError());
        return 0;
    }
    KeyTable RT{};
    RT.w = e->d_lres_w.as<int32_t>();
    RT.rcp_w = e->d_lres_rcp.as<double>();
    RT.kind = e->d_lres_kind.as<uint8_t>();
    RT.ncounters = 1;
    const EventSrc src{ev, nullptr, nullptr, false};
    e->sort_segments(RT, fkey, e->w_fhist.as<uint32_t>(), n, rbits, src, s);
    const BatchWork W = e->work();
    const LocalNodes L{e->d_lres_state.as<int64_t>(), e->d_lres_count.as<double>(), e->lres_n, e->lres_w, e->lres_Is,
                       e->lres_interval, e->occupy_timeout, e->d_lres_tcount.as<double>(),
                       e->d_lres_flags.as<uint8_t>(), e->lres_max_rt, fl, rt};
    e->launch("lgraph_process", n, s, [&] { k_lgraph_process<<<grid_for(n), 256, 0, s>>>(L, G, W, src, out); });
    HIP_OK(hipGetLastError());
    return 0;
}

static bool valid_window(int32_t n, int32_t interval) {  // FlowRuleUtil.isWindowConfigValid (FlowRuleUtil.java:229-231)
    return n > 0 && interval > 0 && interval % n == 0;
}

// ==================================================================== C ABI
extern "C" {

const char *sentinel_last_error(void) { return g_err.c_str(); }

int sentinel_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int sentinel_engine_create(int device, const sentinel_server_config_t *cfg, sentinel_engine_t **out) {
    if (!out) return fail(SENTINEL_E_INVALID, "out is null");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(SENTINEL_E_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(SENTINEL_E_INVALID, "bad device index");
    HIP_OK(hipSetDevice(device));
    sentinel_engine *e = new sentinel_engine();
    e->device = device;
    if (cfg) e->cfg = *cfg;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        delete e;
        return fail(SENTINEL_E_DEVICE, "hipStreamCreate failed");
    }
    if (const char *c = getenv("SENTINEL_PROCESS")) {
        const std::string v(c);
        e->process_impl = v == "group" ? 1 : v == "thread" ? 2 : 0;
    }
    if (const char *c = getenv("SENTINEL_VERDICT_NT")) e->verdict_nt = std::string(c) == "1";
    if (const char *c = getenv("SENTINEL_PARAM_PATH")) {
        const std::string v(c);
        e->param_path = v == "rule" ? 1 : v == "slot" ? 2 : 0;
    }
    if (const char *c = getenv("SENTINEL_CM_LEVELS")) {
        e->cm_force_coop = std::string(c) == "coop";
        e->cm_keys = std::string(c) == "keys";         // "launch" / "coop": always the per-rule lanes
    }
    if (const char *c = getenv("SENTINEL_SCAN")) e->use_lookback = std::string(c) != "3pass";
#ifdef SENTINEL_DIAG_LINEAR_ENV   // wrong output by design (a cost diagnostic): only in a -DSENTINEL_DIAG_LINEAR_ENV build
    if (const char *c = getenv("SENTINEL_DIAG_LINEAR")) e->diag_linear = std::string(c) == "1";
#endif
    if (const char *c = getenv("SENTINEL_HOT_HET_RUN")) e->hot_het_run = (uint32_t)std::max(WAVE_HET_RUN, (uint32_t)atoi(c));
    if (const char *c = getenv("SENTINEL_FLOW_PATH")) {
        const std::string v(c);
        e->flow_path = v == "sorted" ? 1 : v == "partition" ? 2 : v == "small" ? 3 : 0;
    }
    if (const char *c = getenv("SENTINEL_SEGMENTS")) e->fused_segments = std::string(c) != "split";
    if (const char *c = getenv("SENTINEL_LB_START")) {
        unsigned long g = 0, t = 0;
        if (sscanf(c, "%lu,%lu", &g, &t) == 2 && g < LB_GEN_MASK) {
            e->lb_gen0 = (uint32_t)g;
            e->lb_tickets0 = (uint32_t)t;
        }
    }
    if (const char *c = getenv("SENTINEL_HOT_FORK")) e->hot_fork = std::string(c) != "0";
    if (const char *c = getenv("SENTINEL_TOKEN_GROW")) e->tok_grow = std::max<uint64_t>(1, strtoull(c, nullptr, 10));
    if (const char *c = getenv("SENTINEL_SEG_IMPL")) e->seg_impl = atoi(c);
    if (const char *c = getenv("SENTINEL_ROUTE8")) e->use_route8 = std::string(c) != "0";
    if (const char *c = getenv("SENTINEL_LIM1")) e->lim1 = std::string(c) != "0";
    if (const char *c = getenv("SENTINEL_PROC_OCC")) e->process_occ = std::string(c) != "0";
    if (const char *c = getenv("SENTINEL_CM_BLOCK")) e->cm_block = std::string(c) != "0";
    if (const char *c = getenv("SENTINEL_CM_DEBUG")) e->cm_debug = std::string(c) == "1";
    if (const char *c = getenv("SENTINEL_CM_C32")) e->cm_c32 = std::string(c) != "0";
#ifdef SENTINEL_DIAG_CM_ENV   // cost diagnostics that change results: only in a -DSENTINEL_DIAG_CM_ENV build
    if (const char *c = getenv("SENTINEL_CM_DIAG")) e->cm_diag = atoi(c);
#endif
    if (hipDeviceGetAttribute(&e->num_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) e->num_cu = 0;
    if (const char *c = getenv("SENTINEL_PARAM_CAPACITY")) {
        uint64_t v = strtoull(c, nullptr, 10);
        uint64_t p = 1024;
        while (p < v) p <<= 1;
        e->pcap = p;
    }
    // default namespace set: one namespace ("default"), no limiter, connectedCount 0
    e->ns.push_back(sentinel_namespace_t{0, 0, 30000.0});
    int rc = e->rebuild_limiters();
    if (rc) {
        delete e;
        return rc;
    }
    if (hipHostMalloc((void **)&e->h_dev_err, 64, 0) != hipSuccess) {
        delete e;
        return fail(SENTINEL_E_DEVICE, "hipHostMalloc failed");
    }
    memset(e->h_dev_err, 0, 64);
    *out = e;
    return 0;
}

int sentinel_engine_destroy(sentinel_engine_t *e) {
    if (!e) return 0;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->stream);
    if (e->h_dev_err) (void)hipHostFree(e->h_dev_err);
    e->prof_collect();
    for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
    e->ft.release();
    for (DevBuf *b : {&e->topw.ckey, &e->topw.crule, &e->topw.csum, &e->topw.cn, &e->topw.pr, &e->topw.pk, &e->topw.cr,
                      &e->topw.ck, &e->topw.dc, &e->topw.dk, &e->topw.ds, &e->topw.ids, &e->topw.rank, &e->topw.fkey,
                      &e->topw.frule, &e->topw.fsum})
        b->release();
    e->lt.release();
    e->pt.release();
    for (DevBuf *b : {&e->d_flow_route, &e->d_flow_route8, &e->d_flow_ids, &e->d_prule_route, &e->d_prule_n, &e->d_prule_w,
                      &e->d_prule_rcp, &e->d_prule_Is, &e->d_prule_thr, &e->d_prule_rec, &e->d_prule_hot, &e->d_ptable, &e->d_slot_rule,
                      &e->d_hot_table, &e->d_hot_thr, &e->w_fkey, &e->w_lkey, &e->w_skey, &e->w_sval, &e->w_ktmp,
                      &e->w_vtmp, &e->w_fhist, &e->w_lhist, &e->w_parts, &e->w_segid, &e->w_bad, &e->w_hep,
                      &e->w_hacq, &e->w_segstart, &e->w_segkey, &e->w_segep, &e->w_segacq, &e->w_het, &e->w_prio, &e->w_done,
                      &e->w_s0, &e->w_k, &e->w_counters, &e->io_ev, &e->io_fl, &e->io_out, &e->io_vals, &e->w_vslot,
                      &e->d_prule_kind, &e->d_cm, &e->d_lrule_valid, &e->d_lrule_tok, &e->d_lrule_burst,
                      &e->d_lrule_dur, &e->d_lrule_w, &e->d_lrule_rcp, &e->d_lrule_kind, &e->d_lhot_keys,
                      &e->d_lhot_tok, &e->d_ltable, &e->d_lstate, &e->d_now, &e->d_conc_thr, &e->d_seg1_w,
                      &e->d_seg1_rcp, &e->d_seg1_kind, &e->d_tok_rec,
                      &e->d_tok_counts, &e->d_tok_ticket, &e->w_cbig, &e->sp_tok_rec, &e->w_runs, &e->w_pscan, &e->d_lres_state,
                      &e->d_lres_count, &e->w_lb, &e->d_lres_w, &e->d_lres_rcp, &e->d_lres_kind, &e->d_lres_tcount,
                      &e->d_lres_flags, &e->w_lslow, &e->io_lrt, &e->d_lrule_grade,
                      &e->d_lg_on, &e->d_lg_dn, &e->d_lg_created, &e->d_lg_roff, &e->d_lg_rules, &e->d_lg_comp,
                      &e->io_lctx, &e->sp_keys, &e->sp_rule, &e->sp_state, &e->sp_n, &e->sp_w, &e->sp_rcp,
                      &e->sp_Is, &e->sp_thr, &e->sp_kind, &e->w_cm})
        b->release();
    for (int k = 0; k < 2; ++k) {
        e->st_ev[k].release();
        e->st_fl[k].release();
        e->st_out[k].release();
        if (e->x_h2d[k]) (void)hipEventDestroy(e->x_h2d[k]);
        if (e->x_comp[k]) (void)hipEventDestroy(e->x_comp[k]);
    }
    if (e->s_h2d) (void)hipStreamDestroy(e->s_h2d);
    if (e->s_aux) (void)hipStreamDestroy(e->s_aux);
    if (e->tok_snap_ev) (void)hipEventDestroy(e->tok_snap_ev);
    if (e->h_tok_snap) (void)hipHostFree(e->h_tok_snap);
    if (e->s_d2h) (void)hipStreamDestroy(e->s_d2h);
    if (e->h_part_stat) (void)hipHostFree(e->h_part_stat);
    if (e->h_pfresh) (void)hipHostFree(e->h_pfresh);
    if (e->h_cmband) (void)hipHostFree(e->h_cmband);
    if (e->h_sm_ev) (void)hipHostFree(e->h_sm_ev);
    if (e->h_sm_fl) (void)hipHostFree(e->h_sm_fl);
    if (e->h_sm_out) (void)hipHostFree(e->h_sm_out);
    if (e->h_sm_done) (void)hipHostFree(e->h_sm_done);
    if (e->h_long_chunks) (void)hipHostFree(e->h_long_chunks);
    if (e->h_het_hint) (void)hipHostFree(e->h_het_hint);
    e->d_part_stat.release();
    e->d_octr.release();
    (void)hipStreamDestroy(e->stream);
    delete e;
    return 0;
}

void *sentinel_engine_stream(sentinel_engine_t *e) { return e ? (void *)e->stream : nullptr; }

int sentinel_profile_enable(sentinel_engine_t *e, int enable) {
    if (!e) return fail(SENTINEL_E_INVALID, "null engine");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    e->prof_collect();
    e->prof_acc.clear();
    e->prof = enable != 0;
    return 0;
}

int sentinel_set_flow_path(sentinel_engine_t *e, int path) {
    if (!e || path < 0 || path > 3) return fail(SENTINEL_E_INVALID, "bad flow path");
    std::lock_guard<std::mutex> g(e->mu);
    e->flow_path = path;
    return 0;
}

int sentinel_profile_gate(sentinel_engine_t *e, int on) {
    if (!e) return fail(SENTINEL_E_INVALID, "null engine");
    std::lock_guard<std::mutex> g(e->mu);
    e->prof = on != 0;
    return 0;
}

int sentinel_profile_every(sentinel_engine_t *e, int every) {
    if (!e || every < 1) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    e->prof_every = every;
    e->prof_count = 0;
    return 0;
}

int sentinel_profile_select(sentinel_engine_t *e, const char *kernel) {
    if (!e) return fail(SENTINEL_E_INVALID, "null engine");
    std::lock_guard<std::mutex> g(e->mu);
    e->prof_only = kernel ? kernel : "";
    return 0;
}

#ifdef SENTINEL_DIAG_PHASES
int sentinel_diag_phases(unsigned long long *out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), (size_t)n * 12 * 8) == hipSuccess ? 0 : -1;
}
int sentinel_diag_phases_clear() {
    static std::vector<unsigned long long> z(4096 * 12, 0ull);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z.data(), z.size() * 8) == hipSuccess ? 0 : -1;
}
#endif

int sentinel_profile_read(sentinel_engine_t *e, int max, char *names32, double *total_ms, int64_t *calls,
                          int64_t *units) {
    if (!e || max < 0 || (max > 0 && (!names32 || !total_ms || !calls || !units))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    e->prof_collect();
    int k = 0;
    for (auto &x : e->prof_acc) {
        if (k >= max) break;
        std::memset(names32 + 32 * k, 0, 32);
        std::strncpy(names32 + 32 * k, x.first.c_str(), 31);
        total_ms[k] = x.second.ms;
        calls[k] = x.second.calls;
        units[k] = x.second.units;
        ++k;
    }
    return k;
}

int sentinel_set_server_config(sentinel_engine_t *e, const sentinel_server_config_t *cfg) {
    if (!e || !cfg) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    e->cfg = *cfg;
    return e->rebuild_flow_thresholds();
}

int sentinel_set_namespaces(sentinel_engine_t *e, const sentinel_namespace_t *ns, int32_t n) {
    if (!e || (n > 0 && !ns) || n < 0) return fail(SENTINEL_E_INVALID, "bad namespaces");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    e->ns.assign(ns, ns + n);
    int rc = e->rebuild_limiters();
    if (rc) return rc;
    rc = e->rebuild_flow_thresholds();
    if (rc) return rc;
    return e->param_thresholds();
}

int sentinel_set_connected_count(sentinel_engine_t *e, int32_t nsi, int32_t connected) {
    if (!e || nsi < 0) return fail(SENTINEL_E_INVALID, "bad namespace");
    std::lock_guard<std::mutex> g(e->mu);
    if (nsi >= (int32_t)e->ns.size()) return fail(SENTINEL_E_INVALID, "bad namespace");
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    e->ns[nsi].connected_count = connected;
    const int rc = e->rebuild_flow_thresholds();
    if (rc) return rc;
    return e->param_thresholds();       // AVG_LOCAL param rules read connectedCount on every request too
}

int sentinel_load_flow_rules(sentinel_engine_t *e, const sentinel_flow_rule_t *rules, int32_t n) {
    if (!e || (n > 0 && !rules) || n < 0) return fail(SENTINEL_E_INVALID, "bad rules");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    // ClusterFlowRuleManager.applyClusterFlowRule (CFRM:325-372) over every namespace at once.
    // Raw list size per namespace group: an emptied list keeps its flows' metrics (CFRM:268-283).
    std::unordered_map<int32_t, int64_t> raw_ns;
    auto group = [&](int32_t nsi) { return (nsi >= 0 && nsi < (int32_t)e->ns.size()) ? nsi : -1; };
    for (int32_t i = 0; i < n; ++i) raw_ns[group(rules[i].namespace_idx)]++;
    // valid rules (FlowRuleUtil.isValidRule, FlowRuleUtil.java:184-231) deduplicated by flowId:
    // ruleMap.put keeps the last rule, the dense index is the first position; putMetricIfAbsent
    // (CFRM:361-362) runs in list order, so a new flowId gets its first occurrence's window
    std::vector<sentinel_flow_rule_t> nr;
    std::unordered_map<int64_t, int32_t> nidx;
    std::vector<int32_t> gn, gint;
    nr.reserve((size_t)n);                 // (1M-rule reloads: no rehashing / regrowth on the way)
    nidx.reserve((size_t)n);
    gn.reserve((size_t)n);
    gint.reserve((size_t)n);
    for (int32_t i = 0; i < n; ++i) {
        const sentinel_flow_rule_t &r = rules[i];
        if (r.flow_id <= 0 || !(r.count >= 0) || !valid_window(r.sample_count, r.window_interval_ms)) continue;
        auto it = nidx.find(r.flow_id);
        if (it != nidx.end()) { nr[it->second] = r; continue; }
        nidx.emplace(r.flow_id, (int32_t)nr.size());
        nr.push_back(r);
        gn.push_back(r.sample_count);
        gint.push_back(r.window_interval_ms);
    }
    const size_t F = nr.size();
    if (F > (size_t)INT32_MAX / 2) return fail(SENTINEL_E_INVALID, "too many flow rules");
    // where each flow's metric comes from: an existing flow (old window and counters), an orphaned
    // metric of the same flowId, or a fresh one
    std::vector<int32_t> src(F, -1);
    std::vector<int64_t> stg, stg_off(F, -1);
    for (size_t i = 0; i < F; ++i) {
        const int64_t fid = nr[i].flow_id;
        auto it = e->flow_index.find(fid);
        if (it != e->flow_index.end()) {
            src[i] = it->second;
            gn[i] = e->h_flow_n[it->second];
            gint[i] = e->h_flow_interval[it->second];
            continue;
        }
        auto o = e->orphans.find(fid);
        if (o != e->orphans.end()) {
            src[i] = -2;
            gn[i] = o->second.n;
            gint[i] = o->second.interval;
            stg_off[i] = (int64_t)stg.size();
            stg.insert(stg.end(), o->second.rec.begin(), o->second.rec.end());
        }
    }
    // flows that leave: their metric goes away (clearAndResetRulesConditional -> removeMetric,
    // CFRM:285-301) unless their namespace's list is empty
    std::vector<int32_t> orphan_old;
    for (size_t o = 0; o < e->rules.size(); ++o) {
        const sentinel_flow_rule_t &r = e->rules[o];
        if (nidx.count(r.flow_id)) continue;
        auto c = raw_ns.find(group(r.namespace_idx));
        if (c == raw_ns.end() || c->second == 0) orphan_old.push_back((int32_t)o);
    }
    return e->install_flows(std::move(nr), std::move(nidx), std::move(gn), std::move(gint), std::move(src),
                            std::move(stg), std::move(stg_off), orphan_old);
}

// Builds the new flow table on the device (every buffer fresh), remaps the window state of the old
// one, then swaps it in: on any failure the engine keeps its previous table untouched.
int sentinel_engine::install_flows(std::vector<sentinel_flow_rule_t> &&nr, std::unordered_map<int64_t, int32_t> &&nidx,
                                   std::vector<int32_t> &&gn, std::vector<int32_t> &&gint, std::vector<int32_t> &&src,
                                   std::vector<int64_t> &&stg, std::vector<int64_t> &&stg_off,
                                   const std::vector<int32_t> &orphan_old) {
    const size_t F = nr.size();
    const size_t F1 = std::max<size_t>(F, 1);
    std::vector<int64_t> off(F1, 0), ids(F1, 0);
    std::vector<int32_t> ww(F1, 1);
    std::vector<double> rcp(F1, 1.0), Is(F1, 1.0);
    std::vector<uint8_t> kind(F1, KIND_CLUSTER);
    int32_t maxn = 1;
    for (size_t i = 0; i < F; ++i) maxn = std::max(maxn, gn[i]);
    // layout: blocked slot-major header region (HB_KEYS flows x hblock slots per block), then the
    // blocked rest region (per block and slot, six counter rows of HB_KEYS flows)
    const int32_t hblock = header_block_slots(maxn);
    const int64_t nblk = ((int64_t)F + HB_KEYS - 1) / HB_KEYS;
    const int64_t hwords = nblk * hblock * HB_KEYS * 2;
    const int64_t words = std::max<int64_t>(hwords + nblk * hblock * 6 * HB_KEYS, 1);
    for (size_t i = 0; i < F; ++i) {
        off[i] = hwords + blocked_rest_word((int64_t)i, hblock, 0, 0);
        ww[i] = gint[i] / gn[i];
        rcp[i] = 1.0 / (double)ww[i];
        Is[i] = gint[i] / 1000.0;                       // LeapArray.intervalInSecond (LeapArray.java:74)
        kind[i] = nr[i].checker == SENTINEL_CHECKER_SIMPLE ? KIND_SIMPLE : KIND_CLUSTER;
        ids[i] = nr[i].flow_id;
    }
    std::vector<double> thr, cthr;
    flow_thresholds(nr, thr, cthr);
    thr.resize(F1, 0.0);
    std::vector<int32_t> route;
    const bool plain = flow_routes(nr, route);
    route.resize(F1, ROUTE_PLAIN);
    std::vector<int32_t> nnv(gn);
    nnv.resize(F1, 1);
    // new device buffers
    TableBufs nft;
    DevBuf nroute, nroute8, nids, nnow, ncthr, s1w, s1r, s1k, dsrc, dstg, dstgoff;
    auto cleanup = [&] {
        nft.release();
        for (DevBuf *b : {&nroute, &nroute8, &nids, &nnow, &ncthr, &s1w, &s1r, &s1k, &dsrc, &dstg, &dstgoff}) b->release();
    };
    int rc = 0;
    rc |= upload(nft.off, off);
    rc |= upload(nft.n, nnv);
    rc |= upload(nft.w, ww);
    rc |= upload(nft.rcp, rcp);
    rc |= upload(nft.Is, Is);
    rc |= upload(nft.kind, kind);
    rc |= upload(nft.thr, thr);
    rc |= upload(nroute, route);
    rc |= upload_route8(nroute8, route);
    rc |= upload(nids, ids);
    rc |= upload(ncthr, cthr);
    rc |= upload(s1w, std::vector<int32_t>(F1, 1 << 30));
    rc |= upload(s1r, std::vector<double>(F1, 1.0 / (double)(1 << 30)));
    rc |= upload(s1k, std::vector<uint8_t>(F1, KIND_LOCAL_PARAM));
    src.resize(F1, -1);
    stg_off.resize(F1, -1);
    if (stg.empty()) stg.push_back(0);
    rc |= upload(dsrc, src);
    rc |= upload(dstg, stg);
    rc |= upload(dstgoff, stg_off);
    rc |= nft.state.ensure((size_t)words * 8);
    rc |= nft.occ.ensure(F1 * 16);
    rc |= nft.has_occ.ensure(F1);
    rc |= nnow.ensure(F1 * 4);
    if (rc) { cleanup(); return rc < 0 ? rc : SENTINEL_E_NOMEM; }
    // orphans of this load: their old records, staged to the host before the old table goes
    std::vector<Orphan> new_orphans;
    if (!orphan_old.empty() && ft.state.p) {
        const int32_t K = (int32_t)orphan_old.size();
        std::vector<int32_t> on(K);
        std::vector<int64_t> ooff(K);
        int64_t tot = 0;
        for (int32_t k = 0; k < K; ++k) { on[k] = h_flow_n[orphan_old[k]]; ooff[k] = tot; tot += 8 * (int64_t)on[k] + 3; }
        DevBuf di, dn, doff, dout;
        rc |= upload(di, orphan_old);
        rc |= upload(dn, on);
        rc |= upload(doff, ooff);
        rc |= dout.ensure((size_t)tot * 8);
        std::vector<int64_t> recs(tot);
        if (!rc) {
            k_flow_gather<<<grid_for(K), 256, 0, stream>>>(ft.state.as<int64_t>(), flow_hblock, flow_rest_base,
                                                          di.as<int32_t>(), dn.as<int32_t>(), doff.as<int64_t>(), K,
                                                          ft.occ.as<int64_t>(), ft.has_occ.as<uint8_t>(), dout.as<int64_t>());
            if (hipGetLastError() != hipSuccess ||
                hipMemcpyAsync(recs.data(), dout.p, (size_t)tot * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
                hipStreamSynchronize(stream) != hipSuccess)
                rc = fail(SENTINEL_E_DEVICE, "orphan gather failed");
        }
        for (DevBuf *b : {&di, &dn, &doff, &dout}) b->release();
        if (rc) { cleanup(); return rc < 0 ? rc : SENTINEL_E_NOMEM; }
        for (int32_t k = 0; k < K; ++k)
            new_orphans.push_back(Orphan{on[k], h_flow_interval[orphan_old[k]],
                                         std::vector<int64_t>(recs.begin() + ooff[k], recs.begin() + ooff[k] + 8 * on[k] + 3)});
    }
    if (hipMemsetAsync(nft.state.p, 0, (size_t)words * 8, stream) != hipSuccess) { cleanup(); return fail(SENTINEL_E_DEVICE, "memset failed"); }
    if (F > 0) {
        const bool have_old = ft.state.p != nullptr && !rules.empty();
        k_flow_remap<<<grid_for((int64_t)F), 256, 0, stream>>>(
            nft.state.as<int64_t>(), hblock, hwords, nft.n.as<int32_t>(), have_old ? ft.state.as<int64_t>() : nullptr,
            flow_hblock, flow_rest_base, dsrc.as<int32_t>(), dstg.as<int64_t>(), dstgoff.as<int64_t>(),
            nft.occ.as<int64_t>(), nft.has_occ.as<uint8_t>(), nnow.as<int32_t>(), have_old ? ft.occ.as<int64_t>() : nullptr,
            have_old ? ft.has_occ.as<uint8_t>() : nullptr, have_old ? d_now.as<int32_t>() : nullptr, (int32_t)F);
    }
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(stream) != hipSuccess) {
        cleanup();
        return fail(SENTINEL_E_DEVICE, "flow remap failed");
    }
    // swap the new table in (nothing below can fail), then release the old buffers
    for (auto &kv : nidx) orphans.erase(kv.first);   // revived orphans left the registry
    for (size_t k = 0; k < orphan_old.size(); ++k) orphans[rules[orphan_old[k]].flow_id] = std::move(new_orphans[k]);
    std::swap(ft, nft);
    std::swap(d_flow_route, nroute);
    std::swap(d_flow_route8, nroute8);
    std::swap(d_flow_ids, nids);
    std::swap(d_now, nnow);
    std::swap(d_conc_thr, ncthr);
    std::swap(d_seg1_w, s1w);
    std::swap(d_seg1_rcp, s1r);
    std::swap(d_seg1_kind, s1k);
    cleanup();
    rules = std::move(nr);
    flow_index = std::move(nidx);
    flat_flow.build(flow_index);
    off.resize(F);
    h_flow_off = std::move(off);
    h_flow_n = std::move(gn);
    ww.resize(F);
    h_flow_w = std::move(ww);
    h_flow_interval = std::move(gint);
    flow_state_words = words;
    flow_hblock = hblock;
    flow_rest_base = hwords;
    flow_max_n = maxn;
    flow_plain = plain;
    return rewrite_tokens(false);
}

// ClusterServerConfigManager.applyGlobalFlowConfig with a new server window (ClusterServerConfigManager.java:
// 333-343): ClusterMetricStatistics.resetFlowMetrics / ClusterParamMetricStatistics.resetFlowMetrics
// replace every metric -- orphaned ones included -- with a fresh one of the server's window.
int sentinel_reset_metrics(sentinel_engine_t *e, int32_t sample_count, int32_t interval_ms) {
    if (!e) return fail(SENTINEL_E_INVALID, "null engine");
    if (!valid_window(sample_count, interval_ms)) return 0;   // invalid window: ignored (CSCM:335-336)
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    for (auto &kv : e->orphans) {
        sentinel_engine::Orphan &o = kv.second;
        o.n = sample_count;
        o.interval = interval_ms;
        o.rec.assign(8 * (size_t)sample_count + 3, 0);
        for (int j = 0; j < sample_count; ++j) o.rec[2 * j] = EPOCH_ABSENT;
    }
    const size_t F = e->rules.size();
    std::vector<sentinel_flow_rule_t> nr = e->rules;
    std::unordered_map<int64_t, int32_t> nidx = e->flow_index;
    int rc = e->install_flows(std::move(nr), std::move(nidx), std::vector<int32_t>(F, sample_count),
                              std::vector<int32_t>(F, interval_ms), std::vector<int32_t>(F, -1), {}, {}, {});
    if (rc) return rc;
    return e->reset_param_metrics(sample_count, interval_ms);
}

int sentinel_flow_window(sentinel_engine_t *e, int32_t idx, int32_t *sample_count, int32_t *interval_ms) {
    if (!e || !sample_count || !interval_ms) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    if (idx < 0 || idx >= (int32_t)e->rules.size()) return fail(SENTINEL_E_INVALID, "bad flow index");
    *sample_count = e->h_flow_n[idx];
    *interval_ms = e->h_flow_interval[idx];
    return 0;
}

int sentinel_param_table_stats(sentinel_engine_t *e, int64_t *out3) {
    if (!e || !out3) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    out3[0] = e->d_ptable.p ? (int64_t)e->pcap : 0;
    out3[1] = (int64_t)e->p_live;
    out3[2] = (int64_t)e->p_rebuilds;
    return 0;
}

int sentinel_flow_path_stats(sentinel_engine_t *e, int64_t *out4) {
    if (!e || !out4) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    for (int k = 0; k < 4; ++k) out4[k] = e->flow_path_count[k];
    return 0;
}

int sentinel_param_cm_stats(sentinel_engine_t *e, int64_t *out2) {
    if (!e || !out2) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    out2[0] = (int64_t)e->cm_key_batches;
    out2[1] = (int64_t)e->cm_overflows;
    return 0;
}

int sentinel_param_cm_block_batches(sentinel_engine_t *e, int64_t *out) {
    if (!e || !out) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    *out = (int64_t)e->cm_block_batches;
    return 0;
}

int64_t sentinel_metric_count(sentinel_engine_t *e) {
    if (!e) return fail(SENTINEL_E_INVALID, "null engine");
    std::lock_guard<std::mutex> g(e->mu);
    return (int64_t)e->rules.size() + (int64_t)e->orphans.size();
}

int32_t sentinel_flow_count(sentinel_engine_t *e) { return e ? (int32_t)e->rules.size() : 0; }
int32_t sentinel_param_count(sentinel_engine_t *e) { return e ? (int32_t)e->prules.size() : 0; }

int sentinel_lookup_flow_idx(sentinel_engine_t *e, int64_t n, const int64_t *ids, int32_t *out) {
    if (!e || n < 0 || (n > 0 && (!ids || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    for (int64_t i = 0; i < n; ++i) out[i] = e->flat_flow.find(ids[i]);
    return 0;
}

int sentinel_lookup_param_idx(sentinel_engine_t *e, int64_t n, const int64_t *ids, int32_t *out) {
    if (!e || n < 0 || (n > 0 && (!ids || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    const auto idx = std::atomic_load(&e->param_index_pub);     // (no engine mutex: see param_index_pub)
    for (int64_t i = 0; i < n; ++i) {
        if (ids[i] <= 0) { out[i] = SENTINEL_IDX_BAD_ID; continue; }
        if (!idx) { out[i] = SENTINEL_IDX_NO_RULE; continue; }
        auto it = idx->find(ids[i]);
        out[i] = it == idx->end() ? SENTINEL_IDX_NO_RULE : it->second;
    }
    return 0;
}

// ClusterParamFlowRuleManager.applyClusterParamRules (ClusterParamFlowRuleManager.java:318-360) over every
// namespace at once, with the flow table's reload semantics: valid rules deduplicated by flowId (the
// last rule wins, the first position keeps the dense index); putMetricIfAbsent (:355-356) keeps the
// metric -- window, per-value counters -- of a flowId present before and after; a flowId that left
// loses its metric unless its namespace's list is empty (the metric is kept aside and comes back with
// the flowId).
int sentinel_load_param_rules(sentinel_engine_t *e, const sentinel_param_rule_t *rules, int32_t n,
                              const uint64_t *hot_keys, const int32_t *hot_counts, int32_t n_hot) {
    if (!e || n < 0 || (n > 0 && !rules) || n_hot < 0 || (n_hot > 0 && (!hot_keys || !hot_counts)))
        return fail(SENTINEL_E_INVALID, "bad param rules");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    for (int32_t i = 0; i < n; ++i)
        if (rules[i].hot_n < 0 || (rules[i].hot_n > 0 && (rules[i].hot_begin < 0 || rules[i].hot_begin + rules[i].hot_n > n_hot)))
            return fail(SENTINEL_E_INVALID, "hot item range out of bounds");
    std::unordered_map<int32_t, int64_t> raw_ns;
    auto group = [&](int32_t nsi) { return (nsi >= 0 && nsi < (int32_t)e->ns.size()) ? nsi : -1; };
    for (int32_t i = 0; i < n; ++i) raw_ns[group(rules[i].namespace_idx)]++;
    std::vector<sentinel_param_rule_t> nr;
    std::unordered_map<int64_t, int32_t> nidx;
    std::vector<int32_t> gn, gint;
    for (int32_t i = 0; i < n; ++i) {
        const sentinel_param_rule_t &r = rules[i];
        // ParamFlowRuleUtil.isValidRule (ParamFlowRuleUtil.java:46-67): count >= 0, window, flowId > 0
        if (r.flow_id <= 0 || !(r.count >= 0) || !valid_window(r.sample_count, r.window_interval_ms)) continue;
        auto it = nidx.find(r.flow_id);
        if (it != nidx.end()) { nr[it->second] = r; continue; }
        nidx.emplace(r.flow_id, (int32_t)nr.size());
        nr.push_back(r);
        gn.push_back(r.sample_count);
        gint.push_back(r.window_interval_ms);
    }
    const size_t R = nr.size();
    // old rule -> new rule (>= 0), dropped (-1) or orphaned (-2); orphans coming back are imported
    std::vector<int32_t> rmap(e->prules.size(), -1);
    for (size_t o = 0; o < e->prules.size(); ++o) {
        const sentinel_param_rule_t &r = e->prules[o];
        auto it = nidx.find(r.flow_id);
        if (it != nidx.end()) {
            rmap[o] = it->second;
            gn[it->second] = e->h_prule_n[o];
            gint[it->second] = e->h_prule_interval[o];
            continue;
        }
        auto c = raw_ns.find(group(r.namespace_idx));
        if (c == raw_ns.end() || c->second == 0) rmap[o] = -2;
    }
    std::vector<int64_t> imp;
    std::vector<int32_t> imp_rule;
    std::vector<int64_t> revived;
    int32_t maxn = 1;
    for (size_t i = 0; i < R; ++i) {
        auto o = e->porphans.find(nr[i].flow_id);
        if (o != e->porphans.end() && !std::any_of(rmap.begin(), rmap.end(), [&](int32_t m) { return m == (int32_t)i; })) {
            gn[i] = o->second.n;
            gint[i] = o->second.interval;
            revived.push_back(nr[i].flow_id);
        }
        maxn = std::max(maxn, gn[i]);
    }
    if (e->pmode == SENTINEL_PARAM_COUNT_MIN_SHARED)
        for (size_t i = 1; i < R; ++i)
            if (gn[i] != gn[0] || gint[i] != gint[0])
                return fail(SENTINEL_E_INVALID, "a shared count-min sketch needs one window for every param rule");
    // imported records are re-strided to the new table: (2 + 2 maxn) words each
    const int64_t istride = 2 + 2 * (int64_t)maxn;
    for (int64_t fid : revived) {
        const sentinel_engine::POrphan &o = e->porphans[fid];
        const int64_t rs = 2 + 2 * (int64_t)o.n;
        for (size_t k = 0; k + rs <= o.recs.size(); k += rs) {
            imp.insert(imp.end(), o.recs.begin() + k, o.recs.begin() + k + rs);
            imp.resize(imp.size() + (istride - rs), 0);
            imp_rule.push_back(nidx[fid]);
        }
    }
    std::vector<int32_t> ww(std::max<size_t>(R, 1), 1);
    std::vector<double> rcp(std::max<size_t>(R, 1), 1.0), Is(std::max<size_t>(R, 1), 1.0);
    for (size_t i = 0; i < R; ++i) {
        ww[i] = gint[i] / gn[i];
        rcp[i] = 1.0 / (double)ww[i];
        Is[i] = gint[i] / 1000.0;
    }
    int rc = 0;
    if (!e->d_pfresh.p) rc |= e->d_pfresh.ensure(CNT_BYTES);
    if (rc) return SENTINEL_E_NOMEM;
    // the slot table: survivors move to their new index, orphans leave for the host, revived ones return
    std::vector<std::pair<int32_t, std::vector<int64_t>>> exported;
    std::vector<int32_t> nn_up(gn);
    nn_up.resize(std::max<size_t>(R, 1), 1);
    rc = e->param_rebuild(e->pcap, rmap, maxn, nn_up, imp, istride, imp_rule, &exported);
    if (rc) return rc;
    for (int64_t fid : revived) e->porphans.erase(fid);
    for (size_t o = 0; o < rmap.size(); ++o)
        if (rmap[o] == -2) e->porphans[e->prules[o].flow_id] = sentinel_engine::POrphan{e->h_prule_n[o], e->h_prule_interval[o], {}};
    for (auto &x : exported) e->porphans[e->prules[x.first].flow_id].recs = std::move(x.second);
    e->prules = std::move(nr);
    e->param_index = std::move(nidx);
    std::atomic_store(&e->param_index_pub, std::make_shared<const std::unordered_map<int64_t, int32_t>>(e->param_index));
    e->h_prule_n = gn;
    e->h_prule_interval = gint;
    rc |= upload(e->d_prule_n, nn_up);
    rc |= upload(e->d_prule_w, ww);
    rc |= upload(e->d_prule_rcp, rcp);
    rc |= upload(e->d_prule_Is, Is);
    e->prec_dirty = true;
    e->h_phot_keys.assign(hot_keys, hot_keys + n_hot);
    e->h_phot_counts.assign(hot_counts, hot_counts + n_hot);
    rc |= e->param_thresholds();
    rc |= upload(e->d_prule_kind, std::vector<uint8_t>(std::max<size_t>(R, 1), KIND_PARAM));
    if (rc) return rc;
    rc = e->rebuild_cm();
    if (rc) return rc;
    return e->rebuild_routes();
}

// Several device-resident batches decided in order on `stream` under one engine lock: the verdicts and
// counters equal those of the batches submitted one by one.  (A two-stream variant -- batch k + 1's
// validation, histogram and multi-split on a side stream under batch k's decisions -- was measured on
// MI355X at 1M flows: the side stream's kernels only got CUs as k_part_half's workgroups drained, so a
// batch took 0.325 ms of GPU time against 0.333 ms one by one, with more host time per batch; see
// DESIGN.md section 6.)
int sentinel_submit_flow_batches(sentinel_engine_t *e, int32_t nbatch, const int64_t *n,
                                 const sentinel_event_t *const *ev, const uint8_t *const *flags,
                                 sentinel_verdict_t *const *out, void *stream) {
    if (!e || nbatch < 0 || (nbatch > 0 && (!n || !ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    for (int32_t k = 0; k < nbatch; ++k) {
        if (n[k] < 0 || n[k] > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch size out of range (0 .. 2^28 events)");
        if (n[k] > 0 && (!ev[k] || !out[k])) return fail(SENTINEL_E_INVALID, "null batch pointer");
    }
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, s);
    for (int32_t k = 0; k < nbatch; ++k) {
        const int rc = submit_flow(e, n[k], (const Event *)ev[k], flags ? flags[k] : nullptr, (uint64_t *)out[k], s);
        if (rc) return rc;
    }
    return 0;
}

int sentinel_submit_flow_batch(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev, const uint8_t *flags,
                               sentinel_verdict_t *out, void *stream) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_flow(e, n, (const Event *)ev, flags, (uint64_t *)out, fs_s);
}

int sentinel_submit_flow_batch_ordered(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev, const uint8_t *flags,
                                       sentinel_verdict_t *out, uint32_t *out_seq, void *stream) {
    if (!e || n < 0 || (n > 0 && (!ev || !out || !out_seq))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_flow_ordered(e, n, (const Event *)ev, flags, (uint64_t *)out, out_seq, fs_s);
}

// H2D, decide (decide-order output), D2H of verdicts and arrival positions, synchronous, lock held.
static int submit_flow_ordered_host_locked(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                           const uint8_t *flags, sentinel_verdict_t *out, uint32_t *out_seq) {
    HIP_OK(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    int rc = e->io_ev.ensure(n * sizeof(Event));
    rc |= e->io_fl.ensure(n);
    rc |= e->io_out.ensure(n * 12 + 16);
    if (rc) return SENTINEL_E_NOMEM;
    uint64_t *dout = e->io_out.as<uint64_t>();
    uint32_t *dseq = reinterpret_cast<uint32_t *>(dout + n);
    HIP_OK(hipMemcpyAsync(e->io_ev.p, ev, n * sizeof(Event), hipMemcpyHostToDevice, s));
    if (flags) HIP_OK(hipMemcpyAsync(e->io_fl.p, flags, n, hipMemcpyHostToDevice, s));
    rc = submit_flow_ordered(e, n, e->io_ev.as<Event>(), flags ? e->io_fl.as<uint8_t>() : nullptr, dout, dseq, s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(out_seq, dseq, n * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return dev_err_synced(e);
}

int sentinel_submit_flow_batch_ordered_host(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                            const uint8_t *flags, sentinel_verdict_t *out, uint32_t *out_seq) {
    if (!e || n < 0 || (n > 0 && (!ev || !out || !out_seq))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    return submit_flow_ordered_host_locked(e, n, ev, flags, out, out_seq);
}

// H2D, decide, D2H of host events, synchronous, with the engine lock held.
static int submit_flow_host_locked(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev, const uint8_t *flags,
                                   sentinel_verdict_t *out);

int sentinel_submit_flow_batch_host(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                    const uint8_t *flags, sentinel_verdict_t *out) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    return submit_flow_host_locked(e, n, ev, flags, out);
}

// The per-call front doors: flowIds are mapped to dense indices and the batch decided under ONE
// engine lock, so a concurrent rule reload cannot slip between the lookup and the decision (the
// reference looks the rule up inside requestToken, DefaultTokenService.java:42).  ev[i].flow_idx is
// overwritten with the dense index.
static int submit_flow_ids_host(sentinel_engine_t *e, int64_t n, const int64_t *ids, sentinel_event_t *ev,
                                const uint8_t *flags, sentinel_verdict_t *out) {
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    for (int64_t i = 0; i < n; ++i) ev[i].flow_idx = e->flat_flow.find(ids[i]);
    return submit_flow_host_locked(e, n, ev, flags, out);
}

// The batcher's launch: flowIds looked up and the batch queued under one engine lock.  Small batches
// (k_small_flow applies) are launched on pinned ev / flags / out with the completion flag `done`
// (*async = true: the caller polls it); anything else is decided synchronously here.
static int submit_flow_ordered_host_locked(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                           const uint8_t *flags, sentinel_verdict_t *out, uint32_t *out_seq);

static int submit_flow_ids_pinned(sentinel_engine_t *e, int64_t n, const int64_t *ids, sentinel_event_t *ev,
                                  const uint8_t *flags, sentinel_verdict_t *out, uint32_t *done, bool *async,
                                  uint32_t *seq = nullptr, bool *ordered = nullptr) {
    *async = false;
    if (ordered) *ordered = false;
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    for (int64_t i = 0; i < n; ++i) ev[i].flow_idx = e->flat_flow.find(ids[i]);
    if (n <= SM_MAX && small_ok(e)) {
        HIP_OK(hipSetDevice(e->device));
        __atomic_store_n(done, 0u, __ATOMIC_RELAXED);
        const int rc = launch_small(e, n, (const Event *)ev, flags, (uint64_t *)out, e->stream, done);
        *async = rc == 0;
        return rc;
    }
    if (seq && ordered) {                                 // large batch: decide-order output (out[j] <-> seq[j])
        *ordered = true;
        return submit_flow_ordered_host_locked(e, n, ev, flags, out, seq);
    }
    return submit_flow_host_locked(e, n, ev, flags, out);
}

static int submit_flow_host_locked(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev, const uint8_t *flags,
                                   sentinel_verdict_t *out) {
    HIP_OK(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    int rc = 0;
    if (n <= SM_MAX && small_ok(e)) {
        // pinned staging read / written by the kernel itself: one launch, no copy commands
        if (!e->h_sm_ev) {
            HIP_OK(hipHostMalloc((void **)&e->h_sm_ev, SM_MAX * sizeof(Event), 0));
            HIP_OK(hipHostMalloc((void **)&e->h_sm_fl, SM_MAX, 0));
            HIP_OK(hipHostMalloc((void **)&e->h_sm_out, SM_MAX * 8, 0));
            HIP_OK(hipHostMalloc((void **)&e->h_sm_done, 64, 0));
        }
        memcpy(e->h_sm_ev, ev, n * sizeof(Event));
        if (flags) memcpy(e->h_sm_fl, flags, n);
        *e->h_sm_done = 0;
        rc = launch_small(e, n, e->h_sm_ev, flags ? e->h_sm_fl : nullptr, e->h_sm_out, s, e->h_sm_done);
        if (rc) return rc;
        rc = wait_done(e, e->h_sm_done);
        if (rc) return rc;
        memcpy(out, e->h_sm_out, n * 8);
        return 0;
    }
    rc |= e->io_ev.ensure(n * sizeof(Event));
    rc |= e->io_fl.ensure(n);
    rc |= e->io_out.ensure(n * 8);
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemcpyAsync(e->io_ev.p, ev, n * sizeof(Event), hipMemcpyHostToDevice, s));
    if (flags) HIP_OK(hipMemcpyAsync(e->io_fl.p, flags, n, hipMemcpyHostToDevice, s));
    rc = submit_flow(e, n, e->io_ev.as<Event>(), flags ? e->io_fl.as<uint8_t>() : nullptr, e->io_out.as<uint64_t>(), s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, e->io_out.p, n * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return dev_err_synced(e);
}

// Host-fed stream: consecutive batches pipelined over three HIP streams.  Batch i's H2D (s_h2d),
// decide (engine stream) and D2H (s_d2h) overlap batch i-1's D2H and batch i+1's H2D; device staging
// is double-buffered (slot i & 1), a slot is refilled only after the decide that read it finished and
// its verdicts left.  Batches are decided in order on one stream, so the verdicts equal one
// sequential replay of all n events (what sentinel_submit_flow_batch_host over all n returns).
int sentinel_submit_flow_stream_host(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                     const uint8_t *flags, sentinel_verdict_t *out, int64_t batch,
                                     float *batch_ms) {
    if (!e || n < 0 || batch <= 0 || batch > MAX_BATCH || (n > 0 && (!ev || !out)))
        return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    if (!e->s_h2d) {
        HIP_OK(hipStreamCreateWithFlags(&e->s_h2d, hipStreamNonBlocking));
        HIP_OK(hipStreamCreateWithFlags(&e->s_d2h, hipStreamNonBlocking));
        for (int k = 0; k < 2; ++k) {
            HIP_OK(hipEventCreateWithFlags(&e->x_h2d[k], hipEventDisableTiming));
            HIP_OK(hipEventCreateWithFlags(&e->x_comp[k], hipEventDisableTiming));
        }
    }
    const int64_t b = std::min(batch, n);
    int rc = 0;
    for (int k = 0; k < 2; ++k) {
        rc |= e->st_ev[k].ensure(b * sizeof(Event));
        rc |= e->st_out[k].ensure(b * 8);
        if (flags) rc |= e->st_fl[k].ensure(b);
    }
    if (rc) return SENTINEL_E_NOMEM;
    const int64_t nb = (n + b - 1) / b;
    std::vector<hipEvent_t> t0, t1;
    if (batch_ms) {
        t0.resize(nb);
        t1.resize(nb);
        for (int64_t i = 0; i < nb; ++i) {
            t0[i] = e->get_ev();
            t1[i] = e->get_ev();
        }
    }
    for (int64_t i = 0; i < nb; ++i) {
        const int k = (int)(i & 1);
        const int64_t off = i * b, m = std::min(b, n - off);
        // the slot's events were read by batch i-2's decide, its verdicts copied out by batch i-2's D2H
        if (i >= 2) HIP_OK(hipStreamWaitEvent(e->s_h2d, e->x_comp[k], 0));
        if (batch_ms) HIP_OK(hipEventRecord(t0[i], e->s_h2d));
        HIP_OK(hipMemcpyAsync(e->st_ev[k].p, ev + off, m * sizeof(Event), hipMemcpyHostToDevice, e->s_h2d));
        if (flags) HIP_OK(hipMemcpyAsync(e->st_fl[k].p, flags + off, m, hipMemcpyHostToDevice, e->s_h2d));
        HIP_OK(hipEventRecord(e->x_h2d[k], e->s_h2d));
        HIP_OK(hipStreamWaitEvent(e->stream, e->x_h2d[k], 0));
        if (i >= 2) HIP_OK(hipStreamWaitEvent(e->stream, t1.empty() ? e->x_comp[k] : t1[i - 2], 0));
        rc = submit_flow(e, m, e->st_ev[k].as<Event>(), flags ? e->st_fl[k].as<uint8_t>() : nullptr,
                         e->st_out[k].as<uint64_t>(), e->stream);
        if (rc) break;
        HIP_OK(hipEventRecord(e->x_comp[k], e->stream));
        HIP_OK(hipStreamWaitEvent(e->s_d2h, e->x_comp[k], 0));
        HIP_OK(hipMemcpyAsync(out + off, e->st_out[k].p, m * 8, hipMemcpyDeviceToHost, e->s_d2h));
        if (batch_ms) HIP_OK(hipEventRecord(t1[i], e->s_d2h));
        else HIP_OK(hipEventRecord(e->x_comp[k], e->s_d2h));   // D2H done: the slot is free again
    }
    HIP_OK(hipStreamSynchronize(e->s_d2h));
    HIP_OK(hipStreamSynchronize(e->stream));
    if (batch_ms) {
        for (int64_t i = 0; i < nb; ++i) {
            float ms = 0;
            if (rc == 0) HIP_OK(hipEventElapsedTime(&ms, t0[i], t1[i]));
            batch_ms[i] = ms;
            e->ev_pool.push_back(t0[i]);
            e->ev_pool.push_back(t1[i]);
        }
    }
    return rc ? rc : dev_err_synced(e);
}

int sentinel_submit_param_batch(sentinel_engine_t *e, int64_t n, const sentinel_param_event_t *ev,
                                sentinel_verdict_t *out, void *stream) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_param(e, n, (const ParamEvent *)ev, (uint64_t *)out, fs_s);
}

static int submit_param_host_locked(sentinel_engine_t *e, int64_t n, const sentinel_param_event_t *ev,
                                    sentinel_verdict_t *out, uint32_t *out_seq = nullptr);

int sentinel_submit_param_batch_host(sentinel_engine_t *e, int64_t n, const sentinel_param_event_t *ev,
                                     sentinel_verdict_t *out) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    return submit_param_host_locked(e, n, ev, out);
}

static int submit_param_host_locked(sentinel_engine_t *e, int64_t n, const sentinel_param_event_t *ev,
                                    sentinel_verdict_t *out, uint32_t *out_seq) {
    HIP_OK(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    int rc = 0;
    rc |= e->io_ev.ensure(n * sizeof(ParamEvent));
    rc |= e->io_out.ensure(n * 12 + 16);
    if (rc) return SENTINEL_E_NOMEM;
    uint64_t *dout = e->io_out.as<uint64_t>();
    uint32_t *dseq = out_seq ? reinterpret_cast<uint32_t *>(dout + n) : nullptr;
    HIP_OK(hipMemcpyAsync(e->io_ev.p, ev, n * sizeof(ParamEvent), hipMemcpyHostToDevice, s));
    rc = submit_param(e, n, e->io_ev.as<ParamEvent>(), dout, s, dseq);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, s));
    if (out_seq) HIP_OK(hipMemcpyAsync(out_seq, dseq, n * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return dev_err_synced(e);
}

// Decide-order output for single-value param requests (include/sentinel_amd.h): the key walks write each
// request's verdict at its grouped position (the requests of one (rule, value) key are contiguous) and
// its arrival position next to it; other paths answer in arrival order with seq = identity.
int sentinel_submit_param_batch_ordered(sentinel_engine_t *e, int64_t n, const sentinel_param_event_t *ev,
                                        sentinel_verdict_t *out, uint32_t *out_seq, void *stream) {
    if (!e || n < 0 || (n > 0 && (!ev || !out || !out_seq))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_param(e, n, (const ParamEvent *)ev, (uint64_t *)out, fs_s, out_seq);
}

int sentinel_submit_param_batch_ordered_host(sentinel_engine_t *e, int64_t n, const sentinel_param_event_t *ev,
                                             sentinel_verdict_t *out, uint32_t *out_seq) {
    if (!e || n < 0 || (n > 0 && (!ev || !out || !out_seq))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    return submit_param_host_locked(e, n, ev, out, out_seq);
}

int sentinel_submit_param_multi_batch(sentinel_engine_t *e, int64_t n, const sentinel_param_multi_event_t *ev,
                                      const uint64_t *values, int64_t n_values, sentinel_verdict_t *out, void *stream) {
    if (!e || n < 0 || n_values < 0 || (n > 0 && (!ev || !out)) || (n_values > 0 && !values))
        return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_prules(e, e->pmode != SENTINEL_PARAM_EXACT ? PMODE_CM : PMODE_EXACT, n, nullptr,
                         (const MultiEvent *)ev, values, n_values, (uint64_t *)out, fs_s);
}

int sentinel_submit_param_multi_batch_host(sentinel_engine_t *e, int64_t n, const sentinel_param_multi_event_t *ev,
                                           const uint64_t *values, int64_t n_values, sentinel_verdict_t *out) {
    if (!e || n < 0 || n_values < 0 || (n > 0 && (!ev || !out)) || (n_values > 0 && !values))
        return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    return submit_prules_host(e, e->pmode != SENTINEL_PARAM_EXACT ? PMODE_CM : PMODE_EXACT, n, ev, values,
                              n_values, out);
}

int sentinel_set_param_mode(sentinel_engine_t *e, int32_t mode, int32_t depth, int32_t width) {
    if (!e || (mode != SENTINEL_PARAM_EXACT && mode != SENTINEL_PARAM_COUNT_MIN && mode != SENTINEL_PARAM_COUNT_MIN_SHARED))
        return fail(SENTINEL_E_INVALID, "bad param mode");
    if (mode != SENTINEL_PARAM_EXACT && (depth < 1 || depth > 16 || width < 16 || (width & (width - 1)) != 0))
        return fail(SENTINEL_E_INVALID, "count-min needs 1 <= depth <= 16 and a power-of-two width >= 16");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    if (mode == SENTINEL_PARAM_COUNT_MIN_SHARED && !e->uniform_param_window())
        return fail(SENTINEL_E_INVALID, "a shared count-min sketch needs one window for every param rule");
    e->pmode = mode;
    if (mode != SENTINEL_PARAM_EXACT) {
        e->cm_depth = depth;
        e->cm_width = (uint32_t)width;
    }
    int rc = e->clear_param_slots();
    if (rc) return rc;
    return e->rebuild_cm();
}

int sentinel_load_local_param_rules(sentinel_engine_t *e, const sentinel_local_param_rule_t *rules, int32_t n,
                                    const uint64_t *hot_keys, const int32_t *hot_counts, int32_t n_hot) {
    if (!e || n < 0 || (n > 0 && !rules) || n_hot < 0 || (n_hot > 0 && (!hot_keys || !hot_counts)))
        return fail(SENTINEL_E_INVALID, "bad local param rules");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    const size_t N = (size_t)std::max(n, 1);
    std::vector<uint8_t> valid(N, 0), kind(N, KIND_LOCAL_PARAM);
    std::vector<int64_t> tok(N, 0), burst(N, 0), dur(N, 1);
    std::vector<int32_t> w(N, 1 << 30);
    std::vector<double> rcp(N, 1.0 / (double)(1 << 30));
    std::vector<std::pair<uint64_t, int64_t>> hot;
    for (int32_t i = 0; i < n; ++i) {
        const sentinel_local_param_rule_t &r = rules[i];
        // ParamFlowRuleUtil.isValidRule (ParamFlowRuleUtil.java:46-52): count >= 0, burstCount >= 0,
        // durationInSec > 0 (QPS grade, default control behaviour)
        if (!(r.count >= 0) || r.burst_count < 0 || r.duration_in_sec <= 0) continue;
        valid[i] = 1;
        tok[i] = java_d2l(r.count);                          // (long) rule.getCount()  (PFC:139)
        burst[i] = r.burst_count;
        dur[i] = wrap_mul(r.duration_in_sec, 1000);          // rule.getDurationInSec() * 1000
        for (int32_t h = 0; h < r.hot_n; ++h) {
            const int32_t j = r.hot_begin + h;
            if (j < 0 || j >= n_hot) return fail(SENTINEL_E_INVALID, "hot item range out of bounds");
            hot.emplace_back(hot_keys[j], (int64_t)hot_counts[j]);
        }
    }
    uint64_t hcap = 16;
    while (hcap < 2 * hot.size() + 2) hcap <<= 1;
    std::vector<uint64_t> hk(hcap, PKEY_EMPTY);
    std::vector<int64_t> hv(hcap, 0);
    for (auto &kv : hot) {
        uint64_t h = mix64(kv.first) & (hcap - 1);
        while (hk[h] != PKEY_EMPTY && hk[h] != kv.first) h = (h + 1) & (hcap - 1);
        hk[h] = kv.first;
        hv[h] = kv.second;
    }
    int rc = 0;
    rc |= upload(e->d_lrule_valid, valid);
    rc |= upload(e->d_lrule_tok, tok);
    rc |= upload(e->d_lrule_burst, burst);
    rc |= upload(e->d_lrule_dur, dur);
    rc |= upload(e->d_lrule_w, w);
    rc |= upload(e->d_lrule_rcp, rcp);
    rc |= upload(e->d_lrule_kind, kind);
    rc |= upload(e->d_lhot_keys, hk);
    rc |= upload(e->d_lhot_tok, hv);
    if (const char *c = getenv("SENTINEL_LOCAL_PARAM_CAPACITY")) {
        uint64_t v = strtoull(c, nullptr, 10), p = 1024;
        while (p < v) p <<= 1;
        e->lcap = p;
    }
    rc |= e->d_ltable.ensure(e->lcap * 8);
    rc |= e->d_lstate.ensure(e->lcap * 16);
    if (rc) return rc < 0 ? rc : SENTINEL_E_NOMEM;
    e->lhot_mask = hcap - 1;
    e->lhas_hot = !hot.empty();
    // ParameterMetric token/time counters restart with the rules (every slot free, every bucket absent)
    HIP_OK(hipMemsetAsync(e->d_ltable.p, 0xFF, e->lcap * 8, e->stream));
    k_fill_i64<<<grid_for((int64_t)(2 * e->lcap)), 256, 0, e->stream>>>(e->d_lstate.as<int64_t>(), (int64_t)(2 * e->lcap),
                                                                       LOCAL_ABSENT);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(e->stream));
    e->nlrules = n;
    e->lhas_grade = false;                 // every rule QPS grade until sentinel_set_local_param_grades
    return 0;
}

int sentinel_submit_local_param_batch(sentinel_engine_t *e, int64_t n, const sentinel_param_multi_event_t *ev,
                                      const uint64_t *values, int64_t n_values, sentinel_verdict_t *out, void *stream) {
    if (!e || n < 0 || n_values < 0 || (n > 0 && (!ev || !out)) || (n_values > 0 && !values))
        return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_prules(e, PMODE_LOCAL, n, nullptr, (const MultiEvent *)ev, values, n_values, (uint64_t *)out,
                         fs_s);
}

int sentinel_submit_local_param_batch_host(sentinel_engine_t *e, int64_t n, const sentinel_param_multi_event_t *ev,
                                           const uint64_t *values, int64_t n_values, sentinel_verdict_t *out) {
    if (!e || n < 0 || n_values < 0 || (n > 0 && (!ev || !out)) || (n_values > 0 && !values))
        return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    return submit_prules_host(e, PMODE_LOCAL, n, ev, values, n_values, out);
}

int sentinel_set_local_param_grades(sentinel_engine_t *e, const int32_t *grades, int32_t n) {
    if (!e || n < 0 || (n > 0 && !grades)) return fail(SENTINEL_E_INVALID, "bad grades");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    std::vector<uint8_t> gr((size_t)std::max(e->nlrules, 1), 1);
    for (int32_t i = 0; i < n && i < e->nlrules; ++i) gr[i] = grades[i] == 0 ? 0 : 1;   // FLOW_GRADE_THREAD = 0
    const int rc = upload(e->d_lrule_grade, gr);
    if (rc) return rc;
    e->lhas_grade = true;
    return 0;
}

int sentinel_submit_local_param_batch_ex(sentinel_engine_t *e, int64_t n, const sentinel_param_multi_event_t *ev,
                                         const uint8_t *kinds, const uint64_t *values, int64_t n_values,
                                         sentinel_verdict_t *out, void *stream) {
    if (!e || n < 0 || n_values < 0 || (n > 0 && (!ev || !out)) || (n_values > 0 && !values))
        return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_prules(e, PMODE_LOCAL, n, nullptr, (const MultiEvent *)ev, values, n_values, (uint64_t *)out,
                         fs_s, kinds);
}

int sentinel_submit_local_param_batch_ex_host(sentinel_engine_t *e, int64_t n, const sentinel_param_multi_event_t *ev,
                                              const uint8_t *kinds, const uint64_t *values, int64_t n_values,
                                              sentinel_verdict_t *out) {
    if (!e || n < 0 || n_values < 0 || (n > 0 && (!ev || !out)) || (n_values > 0 && !values))
        return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    return submit_prules_host(e, PMODE_LOCAL, n, ev, values, n_values, out, kinds);
}

int sentinel_local_param_state(sentinel_engine_t *e, uint64_t key, int64_t *last_add_ms, int64_t *tokens) {
    if (!e || !last_add_ms || !tokens) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    *last_add_ms = -1;
    *tokens = -1;
    if (!e->d_ltable.p) return 0;
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    std::vector<uint64_t> table(e->lcap);
    HIP_OK(hipMemcpy(table.data(), e->d_ltable.p, e->lcap * 8, hipMemcpyDeviceToHost));
    uint64_t h = mix64(key) & (e->lcap - 1);
    for (uint64_t p = 0; p < e->lcap; ++p) {
        if (table[h] == PKEY_EMPTY) return 0;
        if (table[h] == key) break;
        h = (h + 1) & (e->lcap - 1);
    }
    if (table[h] != key) return 0;
    int64_t st[2];
    HIP_OK(hipMemcpy(st, e->d_lstate.as<int64_t>() + 2 * h, 16, hipMemcpyDeviceToHost));
    *last_add_ms = st[0] == LOCAL_ABSENT ? -1 : st[0];
    *tokens = st[1] == LOCAL_ABSENT ? -1 : st[1];
    return 1;
}

int sentinel_load_local_resources_ex(sentinel_engine_t *e, const sentinel_local_resource_ex_t *res, int32_t n,
                                     int32_t sample_count, int32_t interval_ms) {
    if (!e || n < 0 || (n > 0 && !res)) return fail(SENTINEL_E_INVALID, "bad local resources");
    // SampleCountProperty / IntervalProperty validity: positive, INTERVAL % SAMPLE_COUNT == 0
    if (sample_count < 1 || sample_count > LOCAL_NMAX || interval_ms <= 0 || interval_ms % sample_count != 0)
        return fail(SENTINEL_E_INVALID, "sample_count must be 1..8 and divide interval_ms");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    const size_t N = (size_t)std::max(n, 1);
    int32_t w = interval_ms / sample_count, a = w, b = 1000;
    while (b) { const int32_t t = a % b; a = b; b = t; }            // segment length gcd(w, 1000)
    std::vector<double> count(N, HUGE_VAL), tcount(N, HUGE_VAL);
    std::vector<uint8_t> flags(N, 0);
    for (int32_t i = 0; i < n; ++i) {
        // FlowRuleUtil.isValidRule: count >= 0 (invalid rules are dropped)
        uint8_t f = res[i].flags & (LR_QPS | LR_THREAD | LR_THREAD_FIRST);
        if ((f & LR_QPS) && !(res[i].qps_count >= 0)) f &= (uint8_t)~LR_QPS;
        if ((f & LR_THREAD) && !(res[i].thread_count >= 0)) f &= (uint8_t)~LR_THREAD;
        if (f & LR_QPS) count[i] = res[i].qps_count;
        if (f & LR_THREAD) tcount[i] = res[i].thread_count;
        flags[i] = f;
    }
    std::vector<int64_t> st(N * LOCAL_WORDS, 0);
    for (size_t i = 0; i < N; ++i) {
        int64_t *r = st.data() + i * LOCAL_WORDS;
        for (int j = 0; j < LOCAL_NMAX; ++j) r[LOCAL_SEC_W * j] = r[LOCAL_BOR_OFF + LOCAL_BOR_W * j] = EPOCH_ABSENT;
        for (int j = 0; j < LOCAL_MIN_SLOTS; ++j) r[LOCAL_MIN_OFF + LOCAL_MIN_W * j] = EPOCH_ABSENT;
    }
    int rc = 0;
    rc |= upload(e->d_lres_state, st);
    rc |= upload(e->d_lres_count, count);
    rc |= upload(e->d_lres_tcount, tcount);
    rc |= upload(e->d_lres_flags, flags);
    rc |= upload(e->d_lres_w, std::vector<int32_t>(N, a));
    rc |= upload(e->d_lres_rcp, std::vector<double>(N, 1.0 / (double)a));
    // KIND_CLUSTER: a prioritized entry or an exit makes its segment heterogeneous (sequential path)
    rc |= upload(e->d_lres_kind, std::vector<uint8_t>(N, KIND_CLUSTER));
    if (rc) return rc;
    e->nlres = n;
    e->lgraph = false;
    e->lres_n = sample_count;
    e->lres_w = w;
    e->lres_g = a;
    e->lres_Is = interval_ms / 1000.0;                                 // LeapArray.intervalInSecond
    e->lres_interval = interval_ms;
    if (e->occupy_timeout > interval_ms) e->occupy_timeout = interval_ms;
    return 0;
}

int sentinel_load_local_resources(sentinel_engine_t *e, const sentinel_local_resource_t *res, int32_t n,
                                  int32_t sample_count, int32_t interval_ms) {
    if (!e || n < 0 || (n > 0 && !res)) return fail(SENTINEL_E_INVALID, "bad local resources");
    std::vector<sentinel_local_resource_ex_t> x((size_t)std::max(n, 1));
    for (int32_t i = 0; i < n; ++i) {
        x[i].qps_count = res[i].count;
        x[i].thread_count = 0;
        x[i].flags = res[i].has_rule ? LR_QPS : 0;
        x[i].reserved = 0;
    }
    return sentinel_load_local_resources_ex(e, x.data(), n, sample_count, interval_ms);
}

int sentinel_set_statistic_max_rt(sentinel_engine_t *e, int64_t max_rt_ms) {
    if (!e) return fail(SENTINEL_E_INVALID, "null engine");
    std::lock_guard<std::mutex> g(e->mu);
    e->lres_max_rt = max_rt_ms;
    return 0;
}

int sentinel_submit_local_batch(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev, const uint8_t *flags,
                                const int64_t *rt_ms, sentinel_verdict_t *out, void *stream) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_local_entry(e, n, (const Event *)ev, flags, flags ? rt_ms : nullptr, (uint64_t *)out,
                              fs_s);
}

int sentinel_submit_local_batch_host(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev, const uint8_t *flags,
                                     const int64_t *rt_ms, sentinel_verdict_t *out) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    int rc = 0;
    rc |= e->io_ev.ensure(n * sizeof(Event));
    rc |= e->io_out.ensure(n * 8);
    if (flags) rc |= e->io_fl.ensure(n);
    if (flags && rt_ms) rc |= e->io_lrt.ensure(n * 8);
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemcpyAsync(e->io_ev.p, ev, n * sizeof(Event), hipMemcpyHostToDevice, s));
    if (flags) HIP_OK(hipMemcpyAsync(e->io_fl.p, flags, n, hipMemcpyHostToDevice, s));
    if (flags && rt_ms) HIP_OK(hipMemcpyAsync(e->io_lrt.p, rt_ms, n * 8, hipMemcpyHostToDevice, s));
    rc = submit_local_entry(e, n, e->io_ev.as<Event>(), flags ? e->io_fl.as<uint8_t>() : nullptr,
                            flags && rt_ms ? e->io_lrt.as<int64_t>() : nullptr, e->io_out.as<uint64_t>(), s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, e->io_out.p, n * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return dev_err_synced(e);
}

int sentinel_submit_local_entry_batch(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                      const uint8_t *prioritized, sentinel_verdict_t *out, void *stream) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_local_entry(e, n, (const Event *)ev, prioritized, nullptr, (uint64_t *)out,
                              fs_s);
}

int sentinel_submit_local_entry_batch_host(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                           const uint8_t *prioritized, sentinel_verdict_t *out) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    int rc = 0;
    rc |= e->io_ev.ensure(n * sizeof(Event));
    rc |= e->io_out.ensure(n * 8);
    if (rc) return SENTINEL_E_NOMEM;
    if (prioritized) rc |= e->io_fl.ensure(n);
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemcpyAsync(e->io_ev.p, ev, n * sizeof(Event), hipMemcpyHostToDevice, s));
    if (prioritized) HIP_OK(hipMemcpyAsync(e->io_fl.p, prioritized, n, hipMemcpyHostToDevice, s));
    rc = submit_local_entry(e, n, e->io_ev.as<Event>(), prioritized ? e->io_fl.as<uint8_t>() : nullptr, nullptr,
                            e->io_out.as<uint64_t>(), s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, e->io_out.p, n * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return dev_err_synced(e);
}

int sentinel_local_node_stats(sentinel_engine_t *e, int32_t idx, int64_t ts, int64_t *out) {
    if (!e || !out || ts < 0) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    if (idx < 0 || idx >= e->nlres) return fail(SENTINEL_E_INVALID, "bad resource index");
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    std::vector<int64_t> st(LOCAL_WORDS);
    HIP_OK(hipMemcpy(st.data(), e->d_lres_state.as<int64_t>() + (int64_t)idx * LOCAL_WORDS, LOCAL_WORDS * 8,
                     hipMemcpyDeviceToHost));
    const int64_t E = ts / e->lres_w, E1 = ts / 1000;   // read-only view: valid epochs (E - n, E]
    for (int k = 0; k < 6; ++k) out[k] = 0;
    for (int j = 0; j < e->lres_n; ++j) {
        const int64_t *s = st.data() + LOCAL_SEC_W * j;
        if (s[0] != EPOCH_ABSENT && s[0] > E - e->lres_n && s[0] <= E) {
            out[0] += s[SC_PASS];
            out[1] += s[SC_BLOCK];
        }
        const int64_t *b = st.data() + LOCAL_BOR_OFF + LOCAL_BOR_W * j;
        if (b[0] != EPOCH_ABSENT && b[0] * e->lres_w > ts) out[5] += b[1];   // waiting(): future borrows
    }
    for (int j = 0; j < LOCAL_MIN_SLOTS; ++j) {
        const int64_t *m = st.data() + LOCAL_MIN_OFF + LOCAL_MIN_W * j;
        if (m[0] != EPOCH_ABSENT && m[0] > E1 - LOCAL_MIN_SLOTS && m[0] <= E1) {
            out[2] += m[MC_PASS];
            out[3] += m[MC_BLOCK];
            out[4] += m[MC_OCC];
        }
    }
    return 0;
}

// StatisticNode counters of one node record (device) at ts -> out14 (caller holds e->mu)
static int local_node_metrics_at(sentinel_engine_t *e, const int64_t *node, int64_t ts, int64_t *out) {
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    std::vector<int64_t> st(LOCAL_WORDS);
    HIP_OK(hipMemcpy(st.data(), node, LOCAL_WORDS * 8, hipMemcpyDeviceToHost));
    // read-only view of the rolled windows: epochs > E - n (LeapArray.values after currentWindow,
    // future buckets of a clock that went back included)
    const int64_t E = ts / e->lres_w, E1 = ts / 1000;
    for (int k = 0; k < 14; ++k) out[k] = 0;
    int64_t mrt_s = e->lres_max_rt, mrt_m = e->lres_max_rt;
    for (int j = 0; j < e->lres_n; ++j) {
        const int64_t *s = st.data() + LOCAL_SEC_W * j;
        if (s[0] == EPOCH_ABSENT || s[0] <= E - e->lres_n) continue;
        const int cols[5] = {SC_PASS, SC_BLOCK, SC_EXC, SC_SUCC, SC_RT};
        for (int k = 0; k < 5; ++k) out[k] = wrap_add(out[k], s[cols[k]]);
        mrt_s = std::min(mrt_s, s[SC_MINRT]);
    }
    for (int j = 0; j < LOCAL_MIN_SLOTS; ++j) {
        const int64_t *m = st.data() + LOCAL_MIN_OFF + LOCAL_MIN_W * j;
        if (m[0] == EPOCH_ABSENT || m[0] <= E1 - LOCAL_MIN_SLOTS) continue;
        const int cols[6] = {MC_PASS, MC_BLOCK, MC_OCC, MC_EXC, MC_SUCC, MC_RT};
        for (int k = 0; k < 6; ++k) out[6 + k] = wrap_add(out[6 + k], m[cols[k]]);
        mrt_m = std::min(mrt_m, m[MC_MINRT]);
    }
    out[5] = std::max<int64_t>(1, mrt_s);                 // ArrayMetric.minRt: Math.max(1, rt)
    out[12] = std::max<int64_t>(1, mrt_m);
    out[13] = st[LOCAL_THR_OFF];
    return 0;
}

int sentinel_local_node_metrics(sentinel_engine_t *e, int32_t idx, int64_t ts, int64_t *out) {
    if (!e || !out || ts < 0) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    if (idx < 0 || idx >= e->nlres) return fail(SENTINEL_E_INVALID, "bad resource index");
    return local_node_metrics_at(e, e->d_lres_state.as<int64_t>() + (int64_t)idx * LOCAL_WORDS, ts, out);
}

int sentinel_local_graph_node_metrics(sentinel_engine_t *e, int32_t kind, int32_t idx, int64_t ts, int64_t *out) {
    if (!e || !out || ts < 0) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    const int64_t *base = nullptr;
    int32_t cnt = 0;
    if (kind == SENTINEL_NODE_CLUSTER) { base = e->d_lres_state.as<int64_t>(); cnt = e->nlres; }
    else if (kind == SENTINEL_NODE_ORIGIN && e->lgraph) { base = e->d_lg_on.as<int64_t>(); cnt = e->lg_on; }
    else if (kind == SENTINEL_NODE_DEFAULT && e->lgraph) { base = e->d_lg_dn.as<int64_t>(); cnt = e->lg_dn; }
    if (!base || idx < 0 || idx >= cnt) return fail(SENTINEL_E_INVALID, "bad node kind or index");
    return local_node_metrics_at(e, base + (int64_t)idx * LOCAL_WORDS, ts, out);
}

int sentinel_load_local_rules(sentinel_engine_t *e, const sentinel_local_rule_t *rules, int32_t n, int32_t n_res,
                              int32_t n_origin_nodes, int32_t n_default_nodes, int32_t sample_count, int32_t interval_ms) {
    if (!e || n < 0 || (n > 0 && !rules) || n_res < 0 || n_origin_nodes < 0 || n_default_nodes < 0)
        return fail(SENTINEL_E_INVALID, "bad local rules");
    // every ClusterNode starts empty (and its resource's single-rule fields unused)
    std::vector<sentinel_local_resource_ex_t> none((size_t)std::max(n_res, 1));
    for (auto &x : none) { x.qps_count = 0; x.thread_count = 0; x.flags = 0; x.reserved = 0; }
    int rc = sentinel_load_local_resources_ex(e, none.data(), n_res, sample_count, interval_ms);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    // FlowRuleUtil.buildFlowRuleMap: invalid rules dropped (isValidRule, FRU:167-238), blank limitApp ->
    // "default", duplicates dropped (the HashSet), FlowRuleComparator's stable sort (non-"default"
    // limitApps first); the caller passes FlowRuleManager's order
    auto valid = [&](const sentinel_local_rule_t &r) {
        if (r.resource < 0 || r.resource >= n_res || !(r.count >= 0) || r.strategy < 0) return false;
        if (r.grade == SENTINEL_GRADE_QPS) return r.strategy > SENTINEL_STRATEGY_CHAIN || r.strategy == SENTINEL_STRATEGY_DIRECT || r.ref >= 0;
        return r.grade == SENTINEL_GRADE_THREAD;
    };
    std::vector<std::vector<LocalRule>> per((size_t)std::max(n_res, 1));
    for (int pass = 0; pass < 2; ++pass)
        for (int32_t i = 0; i < n; ++i) {
            const sentinel_local_rule_t &r = rules[i];
            if (!valid(r)) continue;
            const int32_t lim = r.limit_app < 0 ? SENTINEL_LIMIT_APP_DEFAULT : r.limit_app;
            if ((lim == SENTINEL_LIMIT_APP_DEFAULT) != (pass == 1)) continue;
            LocalRule x{r.count, r.grade, r.strategy, lim, r.ref};
            auto &v = per[r.resource];
            bool dup = false;
            for (const LocalRule &y : v)
                dup |= y.grade == x.grade && y.count == x.count && y.strategy == x.strategy && y.limit_app == x.limit_app &&
                       y.ref == x.ref;
            if (!dup) v.push_back(x);
        }
    std::vector<int32_t> roff((size_t)n_res + 1, 0);
    std::vector<LocalRule> flat;
    for (int32_t r = 0; r < n_res; ++r) {
        roff[r] = (int32_t)flat.size();
        flat.insert(flat.end(), per[r].begin(), per[r].end());
    }
    roff[n_res] = (int32_t)flat.size();
    if (flat.empty()) flat.push_back(LocalRule{0, 0, 0, 0, -1});
    // components: union-find over the RELATE edges (a rule reads its refResource's ClusterNode)
    std::vector<uint32_t> par((size_t)std::max(n_res, 1));
    for (int32_t r = 0; r < n_res; ++r) par[r] = (uint32_t)r;
    std::function<uint32_t(uint32_t)> find = [&](uint32_t x) { return par[x] == x ? x : (par[x] = find(par[x])); };
    for (int32_t r = 0; r < n_res; ++r)
        for (int32_t j = roff[r]; j < roff[r + 1]; ++j)
            if (flat[j].strategy == SENTINEL_STRATEGY_RELATE && flat[j].ref >= 0 && flat[j].ref < n_res) {
                const uint32_t a = find((uint32_t)r), b = find((uint32_t)flat[j].ref);
                if (a != b) par[std::max(a, b)] = std::min(a, b);
            }
    std::vector<uint32_t> comp((size_t)std::max(n_res, 1), 0);
    for (int32_t r = 0; r < n_res; ++r) comp[r] = find((uint32_t)r);
    auto empty_nodes = [](int32_t cnt) {
        std::vector<int64_t> st((size_t)std::max(cnt, 1) * LOCAL_WORDS, 0);
        for (int32_t i = 0; i < cnt; ++i) {
            int64_t *r = st.data() + (size_t)i * LOCAL_WORDS;
            for (int j = 0; j < LOCAL_NMAX; ++j) r[LOCAL_SEC_W * j] = r[LOCAL_BOR_OFF + LOCAL_BOR_W * j] = EPOCH_ABSENT;
            for (int j = 0; j < LOCAL_MIN_SLOTS; ++j) r[LOCAL_MIN_OFF + LOCAL_MIN_W * j] = EPOCH_ABSENT;
        }
        return st;
    };
    rc = 0;
    rc |= upload(e->d_lg_on, empty_nodes(n_origin_nodes));
    rc |= upload(e->d_lg_dn, empty_nodes(n_default_nodes));
    rc |= upload(e->d_lg_created, std::vector<uint8_t>((size_t)std::max(n_res, 1), 0));
    rc |= upload(e->d_lg_roff, roff);
    rc |= upload(e->d_lg_rules, flat);
    rc |= upload(e->d_lg_comp, comp);
    if (rc) return rc;
    e->lg_on = n_origin_nodes;
    e->lg_dn = n_default_nodes;
    e->lgraph = true;
    return 0;
}

int sentinel_submit_local_graph_batch(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                      const sentinel_local_ctx_t *ctx, const uint8_t *flags, const int64_t *rt_ms,
                                      sentinel_verdict_t *out, void *stream) {
    if (!e || n < 0 || (n > 0 && (!ev || !ctx || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_local_graph(e, n, (const Event *)ev, (const LocalCtx *)ctx, flags, flags ? rt_ms : nullptr,
                              (uint64_t *)out, fs_s);
}

int sentinel_submit_local_graph_batch_host(sentinel_engine_t *e, int64_t n, const sentinel_event_t *ev,
                                           const sentinel_local_ctx_t *ctx, const uint8_t *flags, const int64_t *rt_ms,
                                           sentinel_verdict_t *out) {
    if (!e || n < 0 || (n > 0 && (!ev || !ctx || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    int rc = 0;
    rc |= e->io_ev.ensure(n * sizeof(Event));
    rc |= e->io_out.ensure(n * 8);
    rc |= e->io_lctx.ensure(n * sizeof(LocalCtx));
    if (flags) rc |= e->io_fl.ensure(n);
    if (flags && rt_ms) rc |= e->io_lrt.ensure(n * 8);
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemcpyAsync(e->io_ev.p, ev, n * sizeof(Event), hipMemcpyHostToDevice, s));
    HIP_OK(hipMemcpyAsync(e->io_lctx.p, ctx, n * sizeof(LocalCtx), hipMemcpyHostToDevice, s));
    if (flags) HIP_OK(hipMemcpyAsync(e->io_fl.p, flags, n, hipMemcpyHostToDevice, s));
    if (flags && rt_ms) HIP_OK(hipMemcpyAsync(e->io_lrt.p, rt_ms, n * 8, hipMemcpyHostToDevice, s));
    rc = submit_local_graph(e, n, e->io_ev.as<Event>(), e->io_lctx.as<LocalCtx>(), flags ? e->io_fl.as<uint8_t>() : nullptr,
                            flags && rt_ms ? e->io_lrt.as<int64_t>() : nullptr, e->io_out.as<uint64_t>(), s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, e->io_out.p, n * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return dev_err_synced(e);
}

int sentinel_set_occupy_timeout(sentinel_engine_t *e, int32_t timeout_ms) {
    if (!e) return fail(SENTINEL_E_INVALID, "null engine");
    std::lock_guard<std::mutex> g(e->mu);
    // OccupyTimeoutProperty.updateTimeout (OccupyTimeoutProperty.java:64-78): < 0 or > INTERVAL ignored
    if (timeout_ms < 0 || timeout_ms > e->lres_interval) return 0;
    e->occupy_timeout = timeout_ms;
    return 0;
}

// A batch of concurrency-token acquires / releases (device pointers) on stream s, engine lock held.
// The token cache is kept below 3/4 of its slots (live + tombstones) from a host-side upper bound, so
// only a batch that could cross it reads the device counts and compacts the tombstones (a sync).
static int submit_concurrent(sentinel_engine_t *e, int64_t n, const ConcEvent *dev, uint64_t *dout, hipStream_t s) {
    if (n <= 0) return 0;
    if (int rc0 = check_dev_err(e, s)) return rc0;
    if (n > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch too large (max 2^28 events)");
    int rc = e->ensure_tokens();
    if (rc) return rc;
    if (e->tok_snap_out && hipEventQuery(e->tok_snap_ev) == hipSuccess) {
        e->tok_snap_out = false;                  // a completed snapshot: the bound from the device's counts
        if (e->tok_snap_gen == e->tok_gen) {
            const uint64_t ub = __atomic_load_n(&e->h_tok_snap[0], __ATOMIC_ACQUIRE) +
                                __atomic_load_n(&e->h_tok_snap[1], __ATOMIC_ACQUIRE) + (e->tok_n_total - e->tok_snap_n);
            if (ub < e->tok_ub) e->tok_ub = ub;
        }
    }
    if ((double)(e->tok_ub + (uint64_t)n) > 0.75 * (double)e->tcap) {
        ++e->tok_gen;                             // (recounted below: an older snapshot is dropped)
        if (s != e->stream) HIP_OK(hipStreamSynchronize(s));
        HIP_OK(hipStreamSynchronize(e->stream));
        unsigned long long counts[2];
        if (int rc2 = e->token_counts(counts, e->stream)) return rc2;
        e->tok_ub = counts[0] + counts[1];
        if ((double)(e->tok_ub + (uint64_t)n) > 0.75 * (double)e->tcap && counts[1] > e->tcap / 64) {
            // first the tombstone sweep (one pass over the keys), then the counts again
            k_tok_sweep<<<(unsigned)((e->tcap + 255) / 256), 256, 0, e->stream>>>(e->token_table());
            if (int rc2 = e->token_counts(counts, e->stream)) return rc2;
            e->tok_ub = counts[0] + counts[1];
        }
        if ((double)(e->tok_ub + (uint64_t)n) > 0.75 * (double)e->tcap) {
            // drop the tombstones, and grow until the live tokens plus tok_grow batches fit (a crossing of the
            // bound costs one host synchronisation).  Ids name their ring slot, so a released token's tombstone is
            // reused only when the ids come round again: the cache settles at a fixed fraction of live + tombstones,
            // and the headroom above it must cover the batches the host runs ahead of the device (the bound only
            // drops when a snapshot completes)
            uint64_t nc = e->tcap;
            while ((double)(counts[0] + e->tok_grow * (uint64_t)n) > 0.75 * (double)nc && nc < ((uint64_t)1 << 32)) nc <<= 1;
            rc = e->rebuild_tokens_device(nc, s);
            if (rc) return rc;
            e->tok_ub = counts[0];
        }
    }
    e->tok_ub += (uint64_t)n;                    // at most one new token per event
    e->tok_n_total += (uint64_t)n;
    rc = e->ensure_ws(n);
    if (rc) return SENTINEL_E_NOMEM;
    const int32_t F = (int32_t)e->rules.size();
    const int fbits = bits_for(F);
    const uint32_t finvalid = ((uint32_t)1 << fbits) - 1;
    uint32_t *fkey = e->w_fkey.as<uint32_t>();
    uint64_t *aux = e->w_hep.as<uint64_t>();                  // sorted values by arrival position (conc_value)
    const int64_t nb = sort_blocks(n);
    const TokenTable TT = e->token_table();
    // scan tiles' look-back descriptors (zeroed by k_conc_prep), fallback list, nowCalls after the batch
    const int64_t nt = (n + CS_TILE - 1) / CS_TILE, segs = std::min<int64_t>(n, std::max<int32_t>(F, 1));
    auto al = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
    const int64_t o_desc = 0, o_ser = o_desc + al(nt * 8), o_fin = o_ser + al(segs * 4), o_end = o_fin + al((int64_t)F * 4 + 4);
    if (o_end > e->cbig_n) {
        e->w_cbig.release();
        if (e->w_cbig.ensure((size_t)o_end)) return SENTINEL_E_NOMEM;
        e->cbig_n = o_end;
    }
    char *gb = e->w_cbig.as<char>();
    uint32_t *ctl = e->w_counters.as<uint32_t>();               // [0] tile ticket, [1] fallback segments
    const ConcScan S{(unsigned long long *)(gb + o_desc), ctl, (uint32_t *)(gb + o_ser), (int32_t *)(gb + o_fin),
                     e->h_dev_err + 1};
    e->launch("conc_prep", n, s, [&] {
        k_conc_prep<<<dim3((unsigned)nb), dim3(SORT_THREADS), 0, s>>>(n, dev, F, TT, dout, fkey, finvalid,
                                                                      e->w_fhist.as<uint32_t>(), nb, aux, S.desc, nt,
                                                                      e->cm_diag >> 8, ctl);
    });
    if (F > 0) {
        const EventSrc src{nullptr, (const ParamEvent *)dev, nullptr, false, aux};
        e->sort(fkey, n, fbits, e->w_fhist.as<uint32_t>(), src, s);
        const uint32_t *skey = e->w_skey.as<uint32_t>();
        const uint64_t *sval = e->w_sval.as<uint64_t>();
        const ConcElems X{e->w_hacq.as<int32_t>(), e->w_done.as<uint8_t>()};
        int32_t *now_calls = e->d_now.as<int32_t>();
        const double *thr = e->d_conc_thr.as<double>();
        e->launch("conc_scan", n, s, [&] {
            k_conc_scan<<<(unsigned)nt, CS_THREADS, 0, s>>>(sval, skey, finvalid, n, TT, thr, now_calls, X, S);
        });
        e->launch("conc_serial", n, s, [&] {
            k_conc_serial<<<grid_for(segs), 256, 0, s>>>(skey, n, now_calls, thr, X, S);
        });
        const uint64_t id_base = (e->tok_salt << 40) | e->tok_counter;
        e->launch("conc_apply", n, s, [&] {
            k_conc_apply<<<grid_for(n), 256, 0, s>>>(sval, skey, finvalid, n, X, TT, e->d_flow_ids.as<int64_t>(), id_base,
                                                     S.fin, now_calls, dout);
        });
        e->tok_counter += (uint64_t)n;
    }
    if (!e->tok_snap_out && e->tok_snap_ev && e->h_tok_snap) {
        k_tok_snapshot<<<1, WAVE, 0, s>>>(e->d_tok_counts.as<unsigned long long>(), e->h_tok_snap);
        if (hipEventRecord(e->tok_snap_ev, s) == hipSuccess) {
            e->tok_snap_out = true;
            e->tok_snap_n = e->tok_n_total;
            e->tok_snap_gen = e->tok_gen;
        }
    }
    HIP_OK(hipGetLastError());
    return 0;
}

int sentinel_submit_concurrent_batch_host(sentinel_engine_t *e, int64_t n, const sentinel_concurrent_event_t *ev,
                                          sentinel_concurrent_result_t *out) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    if (n > MAX_BATCH) return fail(SENTINEL_E_INVALID, "batch too large (max 2^28 events)");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t s = e->stream;
    int rc = e->io_ev.ensure(n * sizeof(ConcEvent));
    rc |= e->io_out.ensure(n * 16);
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemcpyAsync(e->io_ev.p, ev, n * sizeof(ConcEvent), hipMemcpyHostToDevice, s));
    rc = submit_concurrent(e, n, e->io_ev.as<ConcEvent>(), e->io_out.as<uint64_t>(), s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(out, e->io_out.p, n * 16, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    return dev_err_synced(e);
}

int sentinel_submit_concurrent_batch(sentinel_engine_t *e, int64_t n, const sentinel_concurrent_event_t *ev,
                                     sentinel_concurrent_result_t *out, void *stream) {
    if (!e || n < 0 || (n > 0 && (!ev || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    hipStream_t fs_s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, fs_s);
    return submit_concurrent(e, n, (const ConcEvent *)ev, (uint64_t *)out, fs_s);
}

int sentinel_concurrent_now_calls(sentinel_engine_t *e, int32_t flow_idx, int32_t *now_calls) {
    if (!e || !now_calls) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    if (flow_idx < 0 || flow_idx >= (int32_t)e->rules.size()) return fail(SENTINEL_E_INVALID, "bad flow index");
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    HIP_OK(hipMemcpy(now_calls, e->d_now.as<int32_t>() + flow_idx, 4, hipMemcpyDeviceToHost));
    return 0;
}

int sentinel_concurrent_token_count(sentinel_engine_t *e, int64_t *count) {
    if (!e || !count) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    *count = 0;
    if (!e->d_tok_counts.p) return 0;
    HIP_OK(hipSetDevice(e->device));
    unsigned long long c[2];
    if (int rc2 = e->token_counts(c, e->stream)) return rc2;
    *count = (int64_t)c[0];
    return 0;
}

int sentinel_concurrent_expire(sentinel_engine_t *e, int64_t max_tokens, int64_t *removed) {
    if (!e || !removed || max_tokens < 0) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    *removed = 0;
    if (!e->d_tok_rec.p || max_tokens == 0) return 0;
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipMemsetAsync(e->d_tok_ticket.p, 0, 8, e->stream));
    k_conc_expire<<<grid_for((int64_t)e->tcap), 256, 0, e->stream>>>(e->token_table(), e->d_now.as<int32_t>(),
                                                                    (unsigned long long)max_tokens,
                                                                    e->d_tok_ticket.as<unsigned long long>());
    HIP_OK(hipGetLastError());
    unsigned long long t = 0;
    HIP_OK(hipMemcpyAsync(&t, e->d_tok_ticket.p, 8, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    *removed = (int64_t)std::min<unsigned long long>(t, (unsigned long long)max_tokens);
    return 0;
}

int sentinel_request_token(sentinel_engine_t *e, int64_t flow_id, int32_t acquire, int32_t prio, int64_t ts,
                           sentinel_token_result_t *out) {
    if (!e || !out) return fail(SENTINEL_E_INVALID, "null argument");
    sentinel_event_t ev;
    ev.acquire = acquire;
    ev.ts = ts;
    uint8_t fl = prio ? SENTINEL_FLAG_PRIORITIZED : 0;
    sentinel_verdict_t v{0, SENTINEL_STATUS_FAIL, 0};
    int rc = submit_flow_ids_host(e, 1, &flow_id, &ev, &fl, &v);
    out->status = rc ? SENTINEL_STATUS_FAIL : v.status;
    out->remaining = rc ? 0 : v.remaining;
    out->wait_in_ms = rc ? 0 : v.wait_in_ms;
    out->reserved = 0;
    return rc;
}

int sentinel_request_param_token(sentinel_engine_t *e, int64_t flow_id, int32_t acquire, uint64_t param_key,
                                 int64_t ts, sentinel_token_result_t *out) {
    if (!e || !out) return fail(SENTINEL_E_INVALID, "null argument");
    sentinel_param_event_t ev;
    ev.acquire = acquire;
    ev.ts = ts;
    ev.param_key = param_key;
    sentinel_verdict_t v{0, SENTINEL_STATUS_FAIL, 0};
    int rc;
    {
        std::lock_guard<std::mutex> g(e->mu);   // lookup and decision under one lock (DTS:57)
        if (flow_id <= 0) ev.rule_idx = SENTINEL_IDX_BAD_ID;
        else {
            auto it = e->param_index.find(flow_id);
            ev.rule_idx = it == e->param_index.end() ? SENTINEL_IDX_NO_RULE : it->second;
        }
        rc = submit_param_host_locked(e, 1, &ev, &v);
    }
    out->status = rc ? SENTINEL_STATUS_FAIL : v.status;
    out->remaining = rc ? 0 : v.remaining;
    out->wait_in_ms = 0;
    out->reserved = 0;
    return rc;
}

int sentinel_synchronize(sentinel_engine_t *e) {
    if (!e) return fail(SENTINEL_E_INVALID, "null engine");
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    std::lock_guard<std::mutex> g(e->mu);
    return dev_err_synced(e);                            // a batch since the last check gave up a spin
}

int sentinel_dump_flow(sentinel_engine_t *e, int32_t idx, int64_t *out, int32_t out_len) {
    if (!e || !out) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    if (idx < 0 || idx >= (int32_t)e->rules.size()) return fail(SENTINEL_E_INVALID, "bad flow index");
    const int n = e->h_flow_n[idx];
    const int need = n * (1 + NEV) + NEV + 1;
    if (out_len < need) return fail(SENTINEL_E_INVALID, "output too small");
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    // the flow's words of the blocked rest region span (n - 1) slot rows + 6 counter rows
    const int64_t rspan = (int64_t)(n - 1) * 6 * HB_KEYS + 5 * HB_KEYS + 1;
    std::vector<int64_t> hdr(2 * (size_t)n), rspan_w((size_t)rspan), rest(8 * (size_t)n);
    for (int j = 0; j < n; ++j)
        HIP_OK(hipMemcpy(hdr.data() + 2 * j, e->ft.state.as<int64_t>() + blocked_pair_word(idx, e->flow_hblock, j), 16,
                         hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(rspan_w.data(), e->ft.state.as<int64_t>() + e->h_flow_off[idx], rspan * 8, hipMemcpyDeviceToHost));
    for (int j = 0; j < n; ++j)
        for (int c = 0; c < 6; ++c) rest[8 * j + c] = rspan_w[(size_t)j * 6 * HB_KEYS + c * HB_KEYS];
    int64_t occ[2];
    uint8_t hocc;
    HIP_OK(hipMemcpy(occ, e->ft.occ.as<int64_t>() + 2 * idx, 16, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(&hocc, e->ft.has_occ.as<uint8_t>() + idx, 1, hipMemcpyDeviceToHost));
    const int64_t w = e->h_flow_w[idx];
    for (int j = 0; j < n; ++j) {
        int64_t *o = out + j * (1 + NEV);
        const bool present = hdr[2 * j] != EPOCH_ABSENT;
        o[0] = present ? hdr[2 * j] * w : -1;
        o[1 + EV_PASS] = present ? hdr[2 * j + 1] : 0;
        for (int c = 1; c < NEV; ++c) o[1 + c] = present ? rest[8 * j + (c - 1)] : 0;
    }
    int64_t *o = out + n * (1 + NEV);
    for (int c = 0; c < NEV; ++c) o[c] = 0;
    o[EV_PASS] = occ[0];
    o[EV_PASS_REQUEST] = occ[1];
    o[NEV] = hocc;
    return need;
}

int sentinel_param_sum(sentinel_engine_t *e, int32_t ridx, uint64_t pkey, int64_t ts, int64_t *out) {
    if (!e || !out) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    if (ridx < 0 || ridx >= (int32_t)e->prules.size()) return fail(SENTINEL_E_INVALID, "bad rule index");
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    *out = 0;
    if (e->pmode != SENTINEL_PARAM_EXACT) {   // the sketch estimate (min over rows of the window sum)
        const int n = e->h_prule_n[ridx];
        const int64_t E = ts / (e->h_prule_interval[ridx] / n);
        const CountMin C = e->param_ctx().CM;
        int64_t est = INT64_MAX;
        std::vector<uint64_t> cell(e->cm_slots());
        for (int d = 0; d < e->cm_depth; ++d) {
            HIP_OK(hipMemcpy(cell.data(), cm_cell(C, (uint32_t)ridx, d, pkey), cell.size() * 8, hipMemcpyDeviceToHost));
            est = std::min(est, cm_cell_sum(cell.data(), n, E, (int)cell.size()));
        }
        *out = est;
        return 0;
    }
    if (!e->d_ptable.p) return 0;
    DevBuf d;
    if (d.ensure(8)) return SENTINEL_E_NOMEM;
    k_slot_find_one<<<1, 1, 0, e->stream>>>(e->d_ptable.as<unsigned long long>(), e->pcap - 1, pkey, d.as<int64_t>());
    int64_t h = -1;
    HIP_OK(hipMemcpyAsync(&h, d.p, 8, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    d.release();
    if (h < 0) return 0;
    const int n = e->h_prule_n[ridx];                                     // the metric's window
    const int64_t w = e->h_prule_interval[ridx] / n;
    const int64_t stride = param_stride(e->pmax_n);
    std::vector<int64_t> st(2 * n);
    HIP_OK(hipMemcpy(st.data(), e->pt.state.as<int64_t>() + h * stride, st.size() * 8, hipMemcpyDeviceToHost));
    const int64_t E = ts / w;   // read-only view (no roll): valid slots are epochs in (E - n, E]
    int64_t s = 0;
    for (int j = 0; j < n; ++j)
        if (st[2 * j] != EPOCH_ABSENT && st[2 * j] > E - n && st[2 * j] <= E) s += st[2 * j + 1];
    *out = s;
    return 0;
}

// getTopValues(number) of every param rule at ts into device arrays count[R], key[R][number], sum[R][number]
// (param_table.hpp, k_ptop_*): number rounds of a per-rule selection over the live slots.
static int param_top(sentinel_engine_t *e, int64_t ts, int32_t number, hipStream_t s) {
    const int32_t R = (int32_t)e->prules.size();
    auto &W = e->topw;
    int rc = 0;
    rc |= W.dc.ensure((size_t)std::max(R, 1) * 4);
    rc |= W.dk.ensure((size_t)std::max(R, 1) * number * 8);
    rc |= W.ds.ensure((size_t)std::max(R, 1) * number * 8);
    if (rc) return SENTINEL_E_NOMEM;
    HIP_OK(hipMemsetAsync(W.dc.p, 0, (size_t)std::max(R, 1) * 4, s));
    if (R == 0 || !e->d_ptable.p || e->pmode != SENTINEL_PARAM_EXACT) return 0;
    const uint64_t cap = e->pcap;
    // candidate list {key, rule, sum} (slots with a non-zero window sum at ts), sized for the live slots
    // (live after the last rebuild + the reserved upper bound of inserts since); a longer list than that
    // (never expected) reruns the selection with room for the whole table
    uint64_t mc = std::min<uint64_t>(cap, e->p_live + e->p_ub + 1);
    // finalists (candidates at or above their rule's number-th largest rank): a few per rule
    const uint64_t fc = std::min<uint64_t>(mc, (uint64_t)R * (uint64_t)(4 * number) + 4096);
    for (;;) {
        rc |= W.ckey.ensure(mc * 8);
        rc |= W.crule.ensure(mc * 4);
        rc |= W.csum.ensure(mc * 8);
        rc |= W.cn.ensure(16);
        rc |= W.fkey.ensure(fc * 8);
        rc |= W.frule.ensure(fc * 4);
        rc |= W.fsum.ensure(fc * 8);
        rc |= W.rank.ensure((size_t)R * number * 8);
        for (DevBuf *b : {&W.pr, &W.pk, &W.cr, &W.ck}) rc |= b->ensure((size_t)R * 8);
        if (rc) return SENTINEL_E_NOMEM;
        unsigned long long *pr = W.pr.as<unsigned long long>(), *pk = W.pk.as<unsigned long long>(),
                           *cr = W.cr.as<unsigned long long>(), *ck = W.ck.as<unsigned long long>();
        unsigned long long *cn = W.cn.as<unsigned long long>();
        PSlots T{e->d_ptable.as<unsigned long long>(), e->d_slot_rule.as<int32_t>(), e->pt.state.as<int64_t>(),
                 param_stride(e->pmax_n), cap - 1};
        if (e->d_pexpire.bytes < cap * 4) {
            if (e->d_pexpire.ensure(cap * 4)) return SENTINEL_E_NOMEM;
            e->pexp_valid = false;
        }
        T.expire = e->d_pexpire.as<uint32_t>();
        if (!e->pexp_valid) {                 // every slot's hint from its window, once; then the key walk keeps them
            k_ptable_expire<<<grid_for((int64_t)cap), 256, 0, s>>>(T, cap, R, e->d_prule_n.as<int32_t>(),
                                                                   e->d_prule_w.as<int32_t>());
            e->pexp_valid = true;
        }
        const TopCands C{W.ckey.as<unsigned long long>(), W.crule.as<int32_t>(), W.csum.as<int64_t>(), cn, mc};
        const TopCands F{W.fkey.as<unsigned long long>(), W.frule.as<int32_t>(), W.fsum.as<int64_t>(), cn + 1, fc};
        HIP_OK(hipMemsetAsync(cn, 0, 16, s));
        // the sums only (the expire hints leave few candidates: the rank cascade's contended atomics cost
        // more than selection rounds over all of them); the cascade and the finalists only for a long list
        // the slots whose window can be non-zero at ts (a coalesced pass over the 4-B hints), then their sums:
        // every slot of the list in flight at once instead of a dependent chain per 256 slots
        if (W.flist.ensure(mc * 4)) return SENTINEL_E_NOMEM;
        HIP_OK(hipMemsetAsync(cn + 1, 0, 8, s));          // (cn[1]: the list's count until the finalists)
        k_ptop_fresh<<<(unsigned)std::min<uint64_t>(2048, (cap + 255) / 256), 256, 0, s>>>(
            T.expire, cap, ts, W.flist.as<uint32_t>(), cn + 1, mc);
        k_ptop_sums<<<(unsigned)std::min<uint64_t>(2048, (mc + 255) / 256), 256, 0, s>>>(
            T, cap, R, e->d_prule_n.as<int32_t>(), e->d_prule_w.as<int32_t>(), e->d_prule_rcp.as<double>(), ts, C,
            W.flist.as<uint32_t>(), cn + 1, mc);
        unsigned long long found[2] = {0, 0};
        HIP_OK(hipMemcpyAsync(found, cn, 16, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        if ((found[0] > mc || found[1] > mc) && mc < cap) {   // (never expected) room for the whole table
            mc = cap;
            continue;
        }
        bool fin = false;
        if (found[0] > fc) {
            const unsigned gc = (unsigned)std::min<uint64_t>(2048, (mc + 255) / 256);
            HIP_OK(hipMemsetAsync(cn + 1, 0, 8, s));
            HIP_OK(hipMemsetAsync(W.rank.p, 0, (size_t)R * number * 8, s));
            k_ptop_cascade<<<gc, 256, 0, s>>>(C, W.rank.as<unsigned long long>(), number);
            k_ptop_final<<<gc, 256, 0, s>>>(C, W.rank.as<unsigned long long>(), number, F);
            HIP_OK(hipMemcpyAsync(found, cn, 16, hipMemcpyDeviceToHost, s));
            HIP_OK(hipStreamSynchronize(s));
            fin = found[1] <= fc;
        }
        const TopCands &L = fin ? F : C;             // rounds over the finalists, or over every candidate
        HIP_OK(hipMemsetAsync(pr, 0, (size_t)R * 8, s));
        HIP_OK(hipMemsetAsync(pk, 0, (size_t)R * 8, s));
        HIP_OK(hipMemsetAsync(cr, 0, (size_t)R * 8, s));
        HIP_OK(hipMemsetAsync(ck, 0xFF, (size_t)R * 8, s));
        const uint64_t ln = std::min<uint64_t>(fin ? found[1] : found[0], L.cap);
        const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(2048, (ln + 255) / 256));
        for (int k = 0; k < number; ++k) {
            k_ptop_best_sum<<<g, 256, 0, s>>>(L, pr, pk, cr);
            k_ptop_best_key<<<g, 256, 0, s>>>(L, pr, pk, cr, ck);
            k_ptop_take<<<g, 256, 0, s>>>(L, cr, ck, k, number, W.dk.as<uint64_t>(), W.ds.as<int64_t>());
            k_ptop_advance<<<grid_for(R), 256, 0, s>>>(R, pr, pk, cr, ck, W.dc.as<int32_t>());
        }
        HIP_OK(hipGetLastError());
        return 0;
    }
}

int sentinel_param_top_values(sentinel_engine_t *e, int64_t ts, int32_t number, int32_t *count, uint64_t *keys,
                              double *avgs) {
    if (!e || number <= 0 || !count || !keys || !avgs) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipStreamSynchronize(e->stream));
    const int32_t R = (int32_t)e->prules.size();
    int rc = param_top(e, ts, number, e->stream);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(e->stream));     // e->stream is non-blocking: the null-stream copies below do not wait for it
    std::vector<int64_t> sum((size_t)R * number);
    if (R > 0) {
        HIP_OK(hipMemcpy(count, e->topw.dc.p, (size_t)R * 4, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(keys, e->topw.dk.p, (size_t)R * number * 8, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(sum.data(), e->topw.ds.p, (size_t)R * number * 8, hipMemcpyDeviceToHost));
    }
    for (int32_t r = 0; r < R; ++r) {
        const double I_s = e->h_prule_interval[r] / 1000.0;
        for (int32_t k = 0; k < number; ++k) {
            const size_t i = (size_t)r * number + k;
            avgs[i] = k < count[r] ? (double)sum[i] / I_s : 0.0;     // (double) sum / intervalInSecond
            if (k >= count[r]) keys[i] = 0;
        }
    }
    return 0;
}

// ClusterMetricNodeGenerator.paramToMetricNode (ClusterMetricNodeGenerator.java:88-105) for every param rule:
// {flowId, topParams = getTopValues(5)} records in device memory (the param leg of the RCCL snapshot).
__global__ __launch_bounds__(256) void k_ptop_records(int32_t R, const int64_t *__restrict__ ids,
                                                      const int32_t *__restrict__ count, const uint64_t *__restrict__ key,
                                                      const int64_t *__restrict__ sum, const double *__restrict__ Is,
                                                      sentinel_param_snapshot_t *__restrict__ out) {
    const int32_t r = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (r >= R) return;
    sentinel_param_snapshot_t o;
    o.flow_id = ids[r];
    o.n_top = count[r];
    o.reserved = 0;
    for (int k = 0; k < SENTINEL_TOP_PARAMS; ++k) {
        const bool v = k < count[r];
        o.key[k] = v ? key[(int64_t)r * SENTINEL_TOP_PARAMS + k] : 0;
        o.avg[k] = v ? (double)sum[(int64_t)r * SENTINEL_TOP_PARAMS + k] / Is[r] : 0.0;
    }
    out[r] = o;
}

int sentinel_param_snapshot_device(sentinel_engine_t *e, int64_t ts, sentinel_param_snapshot_t *d_out, void *stream) {
    if (!e || !d_out) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    const int32_t R = (int32_t)e->prules.size();
    if (R == 0) return 0;
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, s);
    if (s != e->stream) HIP_OK(hipStreamSynchronize(e->stream));
    auto &W = e->topw;
    int rc = param_top(e, ts, SENTINEL_TOP_PARAMS, s);
    if (rc) return rc;
    std::vector<int64_t> fid(R);
    for (int32_t r = 0; r < R; ++r) fid[r] = e->prules[r].flow_id;
    if (fid != W.h_ids || !W.ids.p) {
        rc = upload(W.ids, fid);
        if (rc) return rc;
        W.h_ids.swap(fid);
    }
    k_ptop_records<<<grid_for(R), 256, 0, s>>>(R, W.ids.as<int64_t>(), W.dc.as<int32_t>(), W.dk.as<uint64_t>(),
                                              W.ds.as<int64_t>(), e->d_prule_Is.as<double>(), d_out);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(s));
    return 0;
}

int sentinel_snapshot_device(sentinel_engine_t *e, int64_t ts, sentinel_flow_snapshot_t *d_out, void *stream) {
    if (!e || !d_out) return fail(SENTINEL_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(e->mu);
    HIP_OK(hipSetDevice(e->device));
    const int32_t F = (int32_t)e->rules.size();
    if (F == 0) return 0;
    if (ts < 0) return fail(SENTINEL_E_INVALID, "negative timestamp");
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    const ForeignStream fs_(e, s);
    KeyTable FT = e->table(e->ft, NEV, 0);
    k_snapshot<<<grid_for(F), 256, 0, s>>>(FT, F, ts, e->d_flow_ids.as<int64_t>(), d_out);
    HIP_OK(hipGetLastError());
    return 0;
}

int sentinel_snapshot(sentinel_engine_t *e, int64_t ts, sentinel_flow_snapshot_t *out) {
    if (!e || !out) return fail(SENTINEL_E_INVALID, "null argument");
    const int32_t F = (int32_t)e->rules.size();
    if (F == 0) return 0;
    void *d = nullptr;
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipMalloc(&d, (size_t)F * sizeof(sentinel_flow_snapshot_t)));
    int rc = sentinel_snapshot_device(e, ts, (sentinel_flow_snapshot_t *)d, nullptr);
    if (!rc) {
        if (hipMemcpyAsync(out, d, (size_t)F * sizeof(sentinel_flow_snapshot_t), hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess)
            rc = fail(SENTINEL_E_DEVICE, "snapshot copy failed");
    }
    (void)hipFree(d);
    return rc;
}

}  // extern "C"

// ==================================================================== request batcher
// The reference TokenService is synchronous per call and called concurrently from Netty worker
// threads (NettyTransportServer.java:53-54, FlowRequestProcessor.java:36-45).  The batcher keeps
// that contract: callers block in sentinel_batcher_request_token while a dispatcher thread gathers
// concurrent requests into pinned host buffers and decides them as GPU batches in arrival order.
// Two batch slots: while batch k is on the GPU (k_small_flow reading and writing the slot's pinned
// buffers, then raising the slot's completion flag) the dispatcher gathers and launches batch k + 1
// on the same stream (so k + 1 is decided after k), then hands out k's verdicts.  When the GPU is
// idle a batch waits up to max_wait_us after its first request (or until max_batch requests).
struct BatchReq {
    sentinel_verdict_t out;
    int rc;
    std::atomic<int> done{0};
};

// One queued request: a blocked caller (waiter) or an asynchronous one (cb).
struct BatchItem {
    int64_t flow_id;
    sentinel_event_t ev;                 // flow_idx filled at launch (submit_flow_ids_pinned)
    uint8_t flag;
    BatchReq *waiter;
    sentinel_token_cb cb;
    void *ctx;
    uint64_t tag;
};

struct sentinel_batcher {
    static constexpr int NSLOT = 2;
    struct Slot {
        std::vector<BatchItem> items;
        std::vector<int64_t> ids;
        sentinel_event_t *h_ev = nullptr;  // pinned: read by the kernel
        uint8_t *h_fl = nullptr;
        sentinel_verdict_t *h_out = nullptr;
        uint32_t *h_seq = nullptr;         // pinned: decide-order output's arrival positions (large batches)
        uint32_t *h_done = nullptr;        // pinned completion flag
        bool ordered = false;              // h_out[j] answers items[h_seq[j]]
        bool async = false;
        int rc = 0;
    };
    sentinel_engine *e = nullptr;
    int32_t max_batch = 4096;
    int32_t max_wait_us = 50;
    std::mutex mu;
    std::condition_variable cv_in, cv_out;
    std::vector<BatchItem> queue;
    std::thread th;
    bool stop = false;
    Slot slot[NSLOT];
    std::atomic<int64_t> batches{0}, requests{0};
    int64_t callers = 0;               // requesters inside request_token (guarded by mu)
    std::condition_variable cv_idle;
    void (*hook)(void *) = nullptr;    // after each batch's callbacks (sentinel_batcher_set_batch_hook)
    void *hook_ctx = nullptr;

    void launch(Slot &S) {
        const int64_t n = (int64_t)S.items.size();
        S.ids.resize(n);
        for (int64_t i = 0; i < n; ++i) {
            S.ids[i] = S.items[i].flow_id;
            S.h_ev[i] = S.items[i].ev;
            S.h_fl[i] = S.items[i].flag;
        }
        S.rc = submit_flow_ids_pinned(e, n, S.ids.data(), S.h_ev, S.h_fl, S.h_out, S.h_done, &S.async, S.h_seq,
                                      &S.ordered);
    }

    void complete(Slot &S) {
        if (S.async && S.rc == 0) S.rc = wait_done(e, S.h_done);
        const int64_t n = (int64_t)S.items.size();
        const int rc = S.rc;
        bool any_sync = false;
        // a large batch comes back in decide order: verdict j answers request h_seq[j] (each request is
        // answered on its own -- by its caller or callback, the wire server by xid -- so no arrival-order
        // permutation is ever built)
        const bool ord = S.ordered && rc == 0;
        for (int64_t j = 0; j < n; ++j) {
            const int64_t i = ord ? (int64_t)S.h_seq[j] : j;
            const BatchItem &it = S.items[i];
            if (it.waiter) {
                it.waiter->out = S.h_out[j];
                it.waiter->rc = rc;
                it.waiter->done.store(1, std::memory_order_release);
                any_sync = true;
            } else {
                // engine down -> FAIL (the client falls back to its local check)
                sentinel_token_result_t r;
                r.status = rc ? SENTINEL_STATUS_FAIL : S.h_out[j].status;
                r.remaining = rc ? 0 : S.h_out[j].remaining;
                r.wait_in_ms = rc ? 0 : S.h_out[j].wait_in_ms;
                r.reserved = 0;
                it.cb(it.ctx, it.tag, &r);
            }
        }
        S.ordered = false;
        batches.fetch_add(1);
        requests.fetch_add(n);
        S.items.clear();
        S.async = false;
        void (*h)(void *);
        void *hc;
        {
            std::lock_guard<std::mutex> lk(mu);
            h = hook;
            hc = hook_ctx;
        }
        if (h) h(hc);
        if (any_sync) {
            { std::lock_guard<std::mutex> lk(mu); }
            cv_out.notify_all();
        }
    }

    void run() {
        int nin = 0, next = 0;             // batches in flight; the slot the next batch goes to
        for (;;) {
            bool took = false;
            if (nin < NSLOT) {
                Slot &S = slot[next];
                {
                    std::unique_lock<std::mutex> lk(mu);
                    if (nin == 0) {
                        cv_in.wait(lk, [&] { return stop || !queue.empty(); });
                        if (stop && queue.empty()) return;
                        if ((int32_t)queue.size() < max_batch && max_wait_us > 0)
                            cv_in.wait_for(lk, std::chrono::microseconds(max_wait_us),
                                           [&] { return stop || (int32_t)queue.size() >= max_batch; });
                    }
                    if ((int32_t)queue.size() <= max_batch) {
                        S.items.swap(queue);
                    } else {
                        S.items.assign(queue.begin(), queue.begin() + max_batch);
                        queue.erase(queue.begin(), queue.begin() + max_batch);
                    }
                }
                if (!S.items.empty()) {
                    launch(S);
                    ++nin;
                    next = (next + 1) % NSLOT;
                    took = true;
                }
            }
            if (nin > 0) {
                const int o = (next - nin + NSLOT) % NSLOT;             // the oldest batch in flight
                Slot &O = slot[o];
                // hand out the oldest batch once done; wait for it when nothing new was launched or
                // every slot is busy
                const bool ready = !O.async || O.rc != 0 || __atomic_load_n(O.h_done, __ATOMIC_ACQUIRE);
                if (ready || !took || nin == NSLOT) {
                    complete(O);
                    --nin;
                }
            }
        }
    }

    int enqueue(const BatchItem &it) {
        std::lock_guard<std::mutex> lk(mu);
        if (stop) return fail(SENTINEL_E_STATE, "batcher stopped");
        if (it.waiter) ++callers;
        queue.push_back(it);
        if ((int32_t)queue.size() == 1 || (int32_t)queue.size() >= max_batch) cv_in.notify_one();
        return 0;
    }
};

extern "C" {

int sentinel_batcher_create(sentinel_engine_t *e, int32_t max_batch, int32_t max_wait_us, sentinel_batcher_t **out) {
    if (!e || !out || max_batch <= 0 || max_wait_us < 0) return fail(SENTINEL_E_INVALID, "bad batcher arguments");
    sentinel_batcher *b = new sentinel_batcher();
    b->e = e;
    b->max_batch = max_batch;
    b->max_wait_us = max_wait_us;
    (void)hipSetDevice(e->device);
    for (auto &S : b->slot) {
        if (hipHostMalloc((void **)&S.h_ev, (size_t)max_batch * sizeof(sentinel_event_t), 0) != hipSuccess ||
            hipHostMalloc((void **)&S.h_fl, (size_t)max_batch, 0) != hipSuccess ||
            hipHostMalloc((void **)&S.h_out, (size_t)max_batch * sizeof(sentinel_verdict_t), 0) != hipSuccess ||
            hipHostMalloc((void **)&S.h_seq, (size_t)max_batch * sizeof(uint32_t), 0) != hipSuccess ||
            hipHostMalloc((void **)&S.h_done, 64, 0) != hipSuccess) {
            for (auto &T : b->slot)
                for (void *p : {(void *)T.h_ev, (void *)T.h_fl, (void *)T.h_out, (void *)T.h_seq, (void *)T.h_done})
                    if (p) (void)hipHostFree(p);
            delete b;
            return fail(SENTINEL_E_NOMEM, "hipHostMalloc failed");
        }
    }
    b->th = std::thread([b] { b->run(); });
    *out = b;
    return 0;
}

int sentinel_batcher_destroy(sentinel_batcher_t *b) {
    if (!b) return 0;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
    }
    b->cv_in.notify_all();
    if (b->th.joinable()) b->th.join();            // queued requests are decided before it exits
    {
        // requesters woken by the last batch still re-take mu before they return: wait for them
        std::unique_lock<std::mutex> lk(b->mu);
        b->cv_idle.wait(lk, [&] { return b->callers == 0; });
    }
    for (auto &S : b->slot)
        for (void *p : {(void *)S.h_ev, (void *)S.h_fl, (void *)S.h_out, (void *)S.h_seq, (void *)S.h_done})
            (void)hipHostFree(p);
    delete b;
    return 0;
}

int sentinel_batcher_request_token(sentinel_batcher_t *b, int64_t flow_id, int32_t acquire, int32_t prio, int64_t ts,
                                   sentinel_token_result_t *out) {
    if (!b || !out) return fail(SENTINEL_E_INVALID, "null argument");
    BatchReq r;
    BatchItem it{};
    it.flow_id = flow_id;
    it.ev.acquire = acquire;
    it.ev.ts = ts;
    it.flag = prio ? SENTINEL_FLAG_PRIORITIZED : 0;
    it.waiter = &r;
    if (int rc = b->enqueue(it)) return rc;
    {
        std::unique_lock<std::mutex> lk(b->mu);
        b->cv_out.wait(lk, [&] { return r.done.load(std::memory_order_acquire) != 0; });
        if (--b->callers == 0) b->cv_idle.notify_all();
    }
    out->status = r.rc ? SENTINEL_STATUS_FAIL : r.out.status;   // engine down -> FAIL (client falls back)
    out->remaining = r.rc ? 0 : r.out.remaining;
    out->wait_in_ms = r.rc ? 0 : r.out.wait_in_ms;
    out->reserved = 0;
    return r.rc;
}

int sentinel_batcher_request_token_async(sentinel_batcher_t *b, int64_t flow_id, int32_t acquire, int32_t prio,
                                         int64_t ts, sentinel_token_cb cb, void *ctx, uint64_t tag) {
    if (!b || !cb) return fail(SENTINEL_E_INVALID, "null argument");
    BatchItem it{};
    it.flow_id = flow_id;
    it.ev.acquire = acquire;
    it.ev.ts = ts;
    it.flag = prio ? SENTINEL_FLAG_PRIORITIZED : 0;
    it.cb = cb;
    it.ctx = ctx;
    it.tag = tag;
    return b->enqueue(it);
}

int sentinel_batcher_request_tokens_async(sentinel_batcher_t *b, int32_t n, const int64_t *flow_ids,
                                          const int32_t *acquire, const uint8_t *prio, const int64_t *ts,
                                          sentinel_token_cb cb, void *ctx, const uint64_t *tags) {
    if (!b || !cb || n < 0 || (n > 0 && (!flow_ids || !acquire || !ts || !tags)))
        return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> lk(b->mu);
    if (b->stop) return fail(SENTINEL_E_STATE, "batcher stopped");
    const bool wake = b->queue.empty();
    for (int32_t i = 0; i < n; ++i) {
        BatchItem it{};
        it.flow_id = flow_ids[i];
        it.ev.acquire = acquire[i];
        it.ev.ts = ts[i];
        it.flag = (prio && prio[i]) ? SENTINEL_FLAG_PRIORITIZED : 0;
        it.cb = cb;
        it.ctx = ctx;
        it.tag = tags[i];
        b->queue.push_back(it);
    }
    if (wake || (int32_t)b->queue.size() >= b->max_batch) b->cv_in.notify_one();
    return 0;
}

int sentinel_batcher_set_batch_hook(sentinel_batcher_t *b, void (*fn)(void *ctx), void *ctx) {
    if (!b) return fail(SENTINEL_E_INVALID, "null batcher");
    std::lock_guard<std::mutex> lk(b->mu);
    b->hook = fn;
    b->hook_ctx = ctx;
    return 0;
}

int sentinel_batcher_stats(sentinel_batcher_t *b, int64_t *batches, int64_t *requests) {
    if (!b) return fail(SENTINEL_E_INVALID, "null batcher");
    if (batches) *batches = b->batches.load();
    if (requests) *requests = b->requests.load();
    return 0;
}

}  // extern "C"

// ==================================================================== multi-device engine
// One engine per entry of device_ids (a device may repeat: several shards on one GPU).  The flowId
// space is partitioned shard = splitmix64(flowId) mod n: a flow's verdicts depend only
// on its own window, so the shards never exchange anything on the decision path.  Rule loads are
// split by shard; a shard whose subset of a namespace is empty while the namespace is not gets one
// invalid marker rule of that namespace (flowId 0: dropped, but the namespace's raw list stays
// non-empty), so the putMetricIfAbsent orphan rule sees the whole node's namespace lists.
struct sentinel_cluster {
    std::vector<sentinel_engine_t *> eng;
    std::vector<sentinel_batcher_t *> batchers;
    std::mutex mu;                                       // one host batch at a time
    std::vector<std::vector<int64_t>> pos, ids;
    std::vector<std::vector<sentinel_event_t>> ev;
    std::vector<std::vector<uint8_t>> fl;
    std::vector<std::vector<sentinel_verdict_t>> out;
};

static inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <class Rule>
static std::vector<std::vector<Rule>> split_rules(const Rule *rules, int32_t n, int32_t shards) {
    std::vector<std::vector<Rule>> part((size_t)shards);
    int32_t max_ns = -1;
    for (int32_t i = 0; i < n; ++i) {
        part[(size_t)(splitmix64((uint64_t)rules[i].flow_id) % (uint64_t)shards)].push_back(rules[i]);
        max_ns = std::max(max_ns, rules[i].namespace_idx);
    }
    std::vector<uint8_t> any((size_t)std::max(max_ns + 1, 1), 0);
    for (int32_t i = 0; i < n; ++i)
        if (rules[i].namespace_idx >= 0) any[(size_t)rules[i].namespace_idx] = 1;
    for (int32_t sh = 0; sh < shards; ++sh) {
        std::vector<uint8_t> mine(any.size(), 0);
        for (const Rule &r : part[(size_t)sh])
            if (r.namespace_idx >= 0) mine[(size_t)r.namespace_idx] = 1;
        for (size_t k = 0; k < any.size(); ++k)
            if (any[k] && !mine[k]) {
                Rule m{};
                m.flow_id = 0;                           // FlowRuleUtil.isValidRule: flowId > 0
                m.namespace_idx = (int32_t)k;
                part[(size_t)sh].push_back(m);
            }
    }
    return part;
}

// run f(shard) on every shard, one host thread each (the shards' devices work concurrently)
template <class F>
static int for_shards(sentinel_cluster_t *c, F f) {
    const size_t n = c->eng.size();
    if (n == 1) return f(0);
    std::vector<int> rc(n, 0);
    std::vector<std::string> err(n);
    std::vector<std::thread> th;
    for (size_t i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            rc[i] = f((int32_t)i);
            if (rc[i]) err[i] = g_err;
        });
    for (auto &t : th) t.join();
    for (size_t i = 0; i < n; ++i)
        if (rc[i]) {
            g_err = err[i];
            return rc[i];
        }
    return 0;
}

extern "C" {

int32_t sentinel_shard_of(int64_t flow_id, int32_t n) {
    return n <= 0 ? -1 : (int32_t)(splitmix64((uint64_t)flow_id) % (uint64_t)n);
}

int sentinel_cluster_create(const int32_t *device_ids, int32_t n, const sentinel_server_config_t *cfg,
                            sentinel_cluster_t **out) {
    if (!device_ids || n <= 0 || !out) return fail(SENTINEL_E_INVALID, "bad device list");
    auto *c = new sentinel_cluster_t();
    for (int32_t i = 0; i < n; ++i) {
        sentinel_engine_t *e = nullptr;
        const int rc = sentinel_engine_create(device_ids[i], cfg, &e);
        if (rc) {
            const std::string msg = g_err;
            for (auto *x : c->eng) sentinel_engine_destroy(x);
            delete c;
            g_err = msg;
            return rc;
        }
        c->eng.push_back(e);
    }
    const size_t k = (size_t)n;
    c->pos.resize(k);
    c->ids.resize(k);
    c->ev.resize(k);
    c->fl.resize(k);
    c->out.resize(k);
    *out = c;
    return 0;
}

int sentinel_cluster_destroy(sentinel_cluster_t *c) {
    if (!c) return fail(SENTINEL_E_INVALID, "null cluster");
    for (auto *b : c->batchers) sentinel_batcher_destroy(b);
    for (auto *e : c->eng) sentinel_engine_destroy(e);
    delete c;
    return 0;
}

int32_t sentinel_cluster_size(sentinel_cluster_t *c) { return c ? (int32_t)c->eng.size() : 0; }

int sentinel_cluster_engine(sentinel_cluster_t *c, int32_t shard, sentinel_engine_t **out) {
    if (!c || !out || shard < 0 || shard >= (int32_t)c->eng.size()) return fail(SENTINEL_E_INVALID, "bad shard");
    *out = c->eng[(size_t)shard];
    return 0;
}

int sentinel_cluster_set_server_config(sentinel_cluster_t *c, const sentinel_server_config_t *cfg) {
    if (!c) return fail(SENTINEL_E_INVALID, "null cluster");
    return for_shards(c, [&](int32_t i) { return sentinel_set_server_config(c->eng[(size_t)i], cfg); });
}

int sentinel_cluster_set_namespaces(sentinel_cluster_t *c, const sentinel_namespace_t *ns, int32_t n) {
    if (!c) return fail(SENTINEL_E_INVALID, "null cluster");
    // a namespace's GlobalRequestLimiter counts every request of the namespace (GlobalRequestLimiter
    // .java:46-55); with flows split by flowId hash each shard would run its own limiter at the full
    // maxAllowedQps and the node could admit up to n times the cap, so limiters need one shard
    if (c->eng.size() > 1 && ns)
        for (int32_t i = 0; i < n; ++i)
            if (ns[i].has_limiter)
                return fail(SENTINEL_E_INVALID, "namespace limiters (has_limiter) need a single-shard cluster: "
                                                "a flowId-hash split would apply the cap per shard");
    return for_shards(c, [&](int32_t i) { return sentinel_set_namespaces(c->eng[(size_t)i], ns, n); });
}

int sentinel_cluster_set_connected_count(sentinel_cluster_t *c, int32_t namespace_idx, int32_t connected) {
    if (!c) return fail(SENTINEL_E_INVALID, "null cluster");
    return for_shards(c, [&](int32_t i) { return sentinel_set_connected_count(c->eng[(size_t)i], namespace_idx, connected); });
}

int sentinel_cluster_load_flow_rules(sentinel_cluster_t *c, const sentinel_flow_rule_t *rules, int32_t n) {
    if (!c || n < 0 || (n > 0 && !rules)) return fail(SENTINEL_E_INVALID, "bad rules");
    std::lock_guard<std::mutex> g(c->mu);
    const auto part = split_rules(rules, n, (int32_t)c->eng.size());
    return for_shards(c, [&](int32_t i) {
        const auto &p = part[(size_t)i];
        return sentinel_load_flow_rules(c->eng[(size_t)i], p.data(), (int32_t)p.size());
    });
}

int sentinel_cluster_load_param_rules(sentinel_cluster_t *c, const sentinel_param_rule_t *rules, int32_t n,
                                      const uint64_t *hot_keys, const int32_t *hot_counts, int32_t n_hot) {
    if (!c || n < 0 || (n > 0 && !rules)) return fail(SENTINEL_E_INVALID, "bad rules");
    std::lock_guard<std::mutex> g(c->mu);
    const auto part = split_rules(rules, n, (int32_t)c->eng.size());
    return for_shards(c, [&](int32_t i) {
        const auto &p = part[(size_t)i];
        return sentinel_load_param_rules(c->eng[(size_t)i], p.data(), (int32_t)p.size(), hot_keys, hot_counts, n_hot);
    });
}

// requestToken for a host batch of flowIds: routed to the owning shards (arrival order kept within
// each shard: a flow lives on one shard, so its events stay in order), decided concurrently, the
// verdicts put back at the arrival positions.
int sentinel_cluster_submit_host(sentinel_cluster_t *c, int64_t n, const int64_t *flow_ids, const int32_t *acquire,
                                 const int64_t *ts, const uint8_t *flags, sentinel_verdict_t *out) {
    if (!c || n < 0 || (n > 0 && (!flow_ids || !acquire || !ts || !out))) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(c->mu);
    const size_t S = c->eng.size();
    for (size_t k = 0; k < S; ++k) {
        c->pos[k].clear();
        c->ids[k].clear();
        c->ev[k].clear();
        c->fl[k].clear();
    }
    for (int64_t i = 0; i < n; ++i) {
        const size_t k = (size_t)(splitmix64((uint64_t)flow_ids[i]) % (uint64_t)S);
        c->pos[k].push_back(i);
        c->ids[k].push_back(flow_ids[i]);
        c->ev[k].push_back(sentinel_event_t{0, acquire[i], ts[i]});
        c->fl[k].push_back(flags ? flags[i] : (uint8_t)0);
    }
    const int rc = for_shards(c, [&](int32_t sh) {
        const size_t k = (size_t)sh;
        const int64_t m = (int64_t)c->pos[k].size();
        c->out[k].resize((size_t)m);
        if (m == 0) return 0;
        return submit_flow_ids_host(c->eng[k], m, c->ids[k].data(), c->ev[k].data(), flags ? c->fl[k].data() : nullptr,
                                    c->out[k].data());
    });
    if (rc) return rc;
    for (size_t k = 0; k < S; ++k)
        for (size_t j = 0; j < c->pos[k].size(); ++j) out[c->pos[k][j]] = c->out[k][j];
    return 0;
}

// Snapshot of every shard's flows at ts, shard after shard (the node-wide ClusterMetricNode list);
// *n_out = the number of records (cap >= sentinel_cluster_flow_count).
int32_t sentinel_cluster_flow_count(sentinel_cluster_t *c) {
    if (!c) return 0;
    int32_t t = 0;
    for (auto *e : c->eng) t += sentinel_flow_count(e);
    return t;
}

int sentinel_cluster_snapshot(sentinel_cluster_t *c, int64_t ts, sentinel_flow_snapshot_t *out, int64_t cap,
                              int64_t *n_out) {
    if (!c || !out || !n_out) return fail(SENTINEL_E_INVALID, "bad arguments");
    std::lock_guard<std::mutex> g(c->mu);
    std::vector<int64_t> off(c->eng.size() + 1, 0);
    for (size_t k = 0; k < c->eng.size(); ++k) off[k + 1] = off[k] + sentinel_flow_count(c->eng[k]);
    if (off.back() > cap) return fail(SENTINEL_E_INVALID, "snapshot buffer too small");
    const int rc = for_shards(c, [&](int32_t sh) { return sentinel_snapshot(c->eng[(size_t)sh], ts, out + off[(size_t)sh]); });
    if (rc) return rc;
    *n_out = off.back();
    return 0;
}

// The concurrent front door over every shard: one batcher (dispatcher thread) per engine; a call is
// routed to its flow's shard.
int sentinel_cluster_batchers_create(sentinel_cluster_t *c, int32_t max_batch, int32_t max_wait_us) {
    if (!c) return fail(SENTINEL_E_INVALID, "null cluster");
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->batchers.empty()) return fail(SENTINEL_E_STATE, "batchers exist");
    for (auto *e : c->eng) {
        sentinel_batcher_t *b = nullptr;
        const int rc = sentinel_batcher_create(e, max_batch, max_wait_us, &b);
        if (rc) {
            for (auto *x : c->batchers) sentinel_batcher_destroy(x);
            c->batchers.clear();
            return rc;
        }
        c->batchers.push_back(b);
    }
    return 0;
}

int sentinel_cluster_request_token(sentinel_cluster_t *c, int64_t flow_id, int32_t acquire_count, int32_t prioritized,
                                   int64_t ts, sentinel_token_result_t *out) {
    if (!c || c->batchers.empty()) return fail(SENTINEL_E_STATE, "no batchers (sentinel_cluster_batchers_create)");
    const size_t k = (size_t)(splitmix64((uint64_t)flow_id) % (uint64_t)c->batchers.size());
    return sentinel_batcher_request_token(c->batchers[k], flow_id, acquire_count, prioritized, ts, out);
}

}  // extern "C"

#include "wire_server.hpp"
