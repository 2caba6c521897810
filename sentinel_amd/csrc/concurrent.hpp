// concurrent.hpp -- cluster concurrency tokens (thread grade) on gfx950.
//
// ConcurrentClusterFlowChecker (srv/flow/ConcurrentClusterFlowChecker.java:48-101) keeps, per flow,
// nowCalls (CurrentConcurrencyManager) and a token cache tokenId -> {flowId, acquireCount}
// (TokenCacheNodeManager).  acquire: nowCalls + acquireCount > threshold -> BLOCKED, else
// nowCalls += acquireCount and a new token; release: unknown token -> ALREADY_RELEASE, rule gone ->
// NO_RULE_EXISTS, else the token leaves the cache and nowCalls -= its acquireCount.
//
// A batch mixes acquires and releases of many flows.  Acquires and releases of one flow do not
// commute (nowCalls is not a monotone function of the event order), so events are grouped by flow
// (K2 radix sort, arrival order kept) and each flow's run is decided in arrival order (below: one
// segmented (min, +) scan over the sorted batch).  The token cache is one open-addressing table in
// HBM: inserts CAS an empty slot or a tombstone, a release empties its slot or leaves a tombstone.
#pragma once

#include "admission.hpp"

namespace sentinel {

// sentinel_concurrent_event_t: {flow_idx, acquire, token_id, kind, flags}.  The first 16 bytes are
// laid out like Event / ParamEvent, so the sort kernels read it through a ParamEvent pointer.
struct ConcEvent {
    int32_t idx;
    int32_t acquire;
    int64_t token;
    int32_t kind;     // 0 acquire, 1 release
    int32_t flags;    // bit0: clientAddress is non-empty
};
static_assert(sizeof(ConcEvent) == sizeof(ParamEvent), "concurrent events share the ParamEvent stride");

constexpr int CONC_ACQUIRE = 0;
constexpr int CONC_RELEASE = 1;
constexpr uint64_t TOKEN_TOMB = 0xFFFFFFFFFFFFFFFEull;    // released token (probe chains continue)
constexpr int ST_RELEASE_OK = 6;                          // TokenResultStatus.RELEASE_OK
constexpr int ST_ALREADY_RELEASE = 7;                     // TokenResultStatus.ALREADY_RELEASE

// One 32-byte record per cache slot (a probe, an insert with its fields, a release's claim, amount and
// tombstone all touch one line of the slot; memset 0xFF = empty slot, no claim).
struct TokRec {
    unsigned long long key;      // token id, PKEY_EMPTY or TOKEN_TOMB
    int64_t flow_id;
    int32_t flow_idx;            // -1: the flow's rule is gone (release -> NO_RULE_EXISTS)
    int32_t acquire;
    uint32_t claim;              // arrival position of the batch's first release of the token (~0 between batches)
    uint32_t pad;
};
static_assert(sizeof(TokRec) == 32, "one half line per slot");

struct TokenTable {
    TokRec *rec;
    uint64_t mask;
    unsigned long long *counts;  // {live tokens, tombstones} deltas, striped (tok_count_add; the host sums them)
};

// The cache counts are updated by one atomic pair per workgroup; many workgroups adding to one address
// queue at one memory channel (16K of them cost a batch ~60 us), so the pair is striped like the other
// batch counters (common.hpp, cnt_lane) and summed by the host when it needs them.
constexpr int TOK_CNT_LANES = CNT_LANES;
constexpr int TOK_CNT_STRIDE = CNT_STRIDE;
constexpr size_t TOK_CNT_BYTES = CNT_BYTES;
__device__ inline void tok_count_add(const TokenTable &T, int which, unsigned long long v) {
    atomicAdd(cnt_lane(T.counts) + which, v);
}

// A token's home slot is its id modulo the capacity (round 6): ids are dense -- id_base + the acquire's
// sorted position in its batch (k_conc_apply) -- so the cache is a ring indexed by id and the inserts of
// one batch land on consecutive records (coalesced CAS and stores, where a hashed home scattered them over
// the table); an id whose slot still holds a live older token continues along the probe chain as before.
// The host keeps live + tombstones below 3/4 of the slots and sizes the ring for several batches of ids,
// so a batch's ids meet slots its predecessors have mostly released.
__host__ __device__ inline uint64_t tok_home(uint64_t id, uint64_t mask) { return id & mask; }

__device__ inline int64_t token_find(const TokenTable &T, uint64_t id) {
    uint64_t h = tok_home(id, T.mask);
    for (uint64_t p = 0; p <= T.mask; ++p) {
        const unsigned long long k = T.rec[h].key;
        if (k == PKEY_EMPTY) return -1;
        if (k == id) return (int64_t)h;
        h = (h + 1) & T.mask;
    }
    return -1;
}

// Insert a fresh token id (never in the table): the first free slot on its probe path, a tombstone
// included -- released tokens' slots are reused, so the cache does not fill up with tombstones under a
// steady acquire / release churn (lookups skip tombstones and stop at an empty slot, which a reuse
// never creates or removes).  `tomb` tells whether a tombstone was taken.
// Many inserts run at once (k_conc_apply): a lost CAS re-examines the slot with the value the CAS
// returned -- a plain re-load could keep answering the stale free slot from this CU's cache and spin.
__device__ inline int64_t token_insert(const TokenTable &T, uint64_t id, bool &tomb) {
    uint64_t h = tok_home(id, T.mask);
    unsigned long long k = T.rec[h].key;
    for (uint64_t p = 0; p <= T.mask;) {
        if (k == PKEY_EMPTY || k == TOKEN_TOMB) {
            const unsigned long long prev = atomicCAS(&T.rec[h].key, k, (unsigned long long)id);
            if (prev == k) {
                tomb = k == TOKEN_TOMB;
                return (int64_t)h;
            }
            k = prev;                                     // taken (or changed) meanwhile: look again
            continue;
        }
        h = (h + 1) & T.mask;
        ++p;
        k = T.rec[h].key;
    }
    return -1;
}

// Device compaction of the token cache into a fresh table (tombstones dropped, capacity possibly
// larger): every live token re-placed with its record; counts = {live, 0}.
__global__ __launch_bounds__(256) void k_tok_rebuild(TokenTable O, uint64_t ocap, TokenTable N) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ocap) return;
    const TokRec r = O.rec[s];
    if (r.key == PKEY_EMPTY || r.key == TOKEN_TOMB) return;
    uint64_t h = tok_home(r.key, N.mask);
    while (atomicCAS(&N.rec[h].key, (unsigned long long)PKEY_EMPTY, r.key) != PKEY_EMPTY) h = (h + 1) & N.mask;
    N.rec[h].flow_id = r.flow_id;
    N.rec[h].flow_idx = r.flow_idx;
    N.rec[h].acquire = r.acquire;
    tok_count_add(N, 0, 1ull);
}

// Result record {token_id, status}: one 16-byte store (one write request per scattered record).
__device__ inline void put_conc(uint64_t *out, uint32_t i, int64_t token, int status) {
    *reinterpret_cast<ulonglong2 *>(out + 2 * (uint64_t)i) =
        make_ulonglong2((unsigned long long)token, (unsigned long long)(uint32_t)status);
}

// The sorted value of an event (written by k_conc_prep by arrival position, moved by the sort): the
// arrival position (SEQ_MASK bits), a release bit, and an acquire's amount or the released token's slot
// (35 bits: the token cache stays below 2^32 slots), so the scan reads everything from its sorted values.
constexpr int CV_REL_BIT = 28;
constexpr int CV_PAY_SHIFT = 29;
__device__ inline uint64_t conc_value(uint32_t seq, bool release, uint64_t payload) {
    return (uint64_t)seq | (uint64_t)(release ? 1 : 0) << CV_REL_BIT | payload << CV_PAY_SHIFT;
}

// DefaultTokenService.requestConcurrentToken validation (DTS:64-75, 89-91) and release lookup;
// sort key = flow index (acquire: the rule; release: the token's flow); pass-0 histograms.  A found
// release records its token slot (aux) and claims it with its arrival position (atomicMin): the
// first release of a token in the batch is the one that finds it cached (CCFC:82-86), later ones of
// the same token answer ALREADY_RELEASE.  Tokens issued in this batch are not yet known to any client.
__global__ __launch_bounds__(SORT_THREADS) void k_conc_prep(int64_t n, const ConcEvent *__restrict__ ev, int32_t nflows,
                                                            TokenTable TT, uint64_t *__restrict__ out,
                                                            uint32_t *__restrict__ fkey, uint32_t finvalid,
                                                            uint32_t *__restrict__ fhist, int64_t nblocks,
                                                            uint64_t *__restrict__ aux, unsigned long long *__restrict__ desc,
                                                            int64_t ndesc, int diag, uint32_t *__restrict__ sctl = nullptr) {
    for (int64_t j = (int64_t)blockIdx.x * SORT_THREADS + threadIdx.x; j < ndesc; j += (int64_t)gridDim.x * SORT_THREADS)
        desc[j] = 0;                                      // k_conc_scan's look-back descriptors: not yet
    if (sctl && blockIdx.x == 0 && threadIdx.x < 2) sctl[threadIdx.x] = 0u;   // its tile ticket and fallback count
    __shared__ uint32_t hf[MAX_PASSES][RADIX];
    for (int d = threadIdx.x; d < MAX_PASSES * RADIX; d += SORT_THREADS) (&hf[0][0])[d] = 0;
    __syncthreads();
    const int64_t tile0 = (int64_t)blockIdx.x * SORT_TILE;
    // every event of the tile loaded, then every release's home-slot probe (key + flow index) issued,
    // before any item is decided: the probes of one thread's items are in flight together
    ConcEvent evs[SORT_ITEMS];
    unsigned long long hk[SORT_ITEMS];
    int32_t hf_idx[SORT_ITEMS];
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        if (i < n) evs[j] = ev[i];
        else evs[j].kind = -1;
    }
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        hk[j] = PKEY_EMPTY;
        hf_idx[j] = -1;
        if (evs[j].kind == CONC_RELEASE) {
            const uint64_t h = tok_home((uint64_t)evs[j].token, TT.mask);
            hk[j] = TT.rec[h].key;
            hf_idx[j] = TT.rec[h].flow_idx;
        }
    }
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        if (i >= n) continue;
        const ConcEvent e = evs[j];
        int st = 127;
        uint32_t k = finvalid;
        uint64_t cv = conc_value((uint32_t)i, false, 0);
        if (e.kind == CONC_ACQUIRE) {
            if (!(e.flags & 1) || e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0) st = ST_BAD_REQUEST;
            else if (e.idx < 0 || e.idx >= nflows) st = ST_NO_RULE_EXISTS;
            else {
                k = (uint32_t)e.idx;
                cv = conc_value((uint32_t)i, false, (uint32_t)e.acquire);   // an acquire: its amount (> 0)
            }
        } else if (e.kind == CONC_RELEASE) {
            int64_t h = -1;                                                  // CCFC:82-86
            int32_t fidx = -1;
            const uint64_t h0 = tok_home((uint64_t)e.token, TT.mask);
            const bool issuable = (uint64_t)e.token != PKEY_EMPTY && (uint64_t)e.token != TOKEN_TOMB;  // (slot markers)
            if (!issuable) {
                // never issued (ids stay below 2^63): ALREADY_RELEASE
            } else if (hk[j] == (unsigned long long)e.token) {               // at its home slot (the common case)
                h = (int64_t)h0;
                fidx = hf_idx[j];
            } else if (hk[j] != PKEY_EMPTY) {                                // further along its probe chain
                h = token_find(TT, (uint64_t)e.token);
                if (h >= 0) fidx = TT.rec[h].flow_idx;
            }
            if (h < 0) st = ST_ALREADY_RELEASE;
            else if (fidx < 0) st = ST_NO_RULE_EXISTS;                       // CCFC:87-91
            else {
                k = (uint32_t)fidx;
                cv = conc_value((uint32_t)i, true, (uint64_t)h);             // a release: its token's slot
                if (diag & 1) TT.rec[h].claim = (uint32_t)i;          // cost diagnostic only (wrong with duplicates)
                else atomicMin(&TT.rec[h].claim, (uint32_t)i);
            }
        } else {
            st = ST_BAD_REQUEST;
        }
        fkey[i] = k;
        aux[i] = cv;
        tile_hist_accumulate(hf, k, 1);
        if (st != 127) put_conc(out, (uint32_t)i, 0, st);
    }
    __syncthreads();
    tile_hist_store(hf, fhist, 1, nblocks);
}

// ---------------------------------------------------------------- decisions
// After the sort a flow's events form a contiguous segment in arrival order, and the batch is decided
// by one segmented scan over the sorted positions (k_conc_scan), so that no lane walks a chain of
// dependent gathers and no per-run bookkeeping is needed:
//   element   one per sorted position, gathered once: x > 0 an acquire of x tokens, x < 0 a release of
//             -x tokens that found its token cached and claimed it (the batch's first release of it,
//             k_conc_prep; its slot is freed right there), 0 a release that answers ALREADY_RELEASE
//   scan      the greedy admission of unit acquires with releases interleaved is a (min, +)
//             recurrence: with T' = floor(threshold), an acquire passes iff the in-flight count y < T'
//             (CCFC:57-70: !((double)(y + 1) > threshold)), and while y <= T' it maps y to
//             min(y + 1, T'); a release of r tokens maps y to y - r (CCFC:92-98).  Both are
//             x -> min(x + P, C), closed under composition; a segment head resets the composition, so
//             the whole batch is one segmented scan with a decoupled look-back over tiles (a tile with
//             a head publishes its inclusive state at once, so look-backs are short)
//   fallback  a segment that the scan cannot decide exactly -- an amount other than 1, nowCalls above T'
//             at the start, or an int sum that could wrap -- is walked by one thread (k_conc_serial)
//   effects   one thread per sorted position (k_conc_apply): a passing acquire takes a token (insert
//             into the cache, id = id_base + sorted position), a failing one answers BLOCKED; the
//             segment's last position stores nowCalls
// A release's amount is read in k_conc_scan, a kernel before any insert of the batch, so a slot reused
// by an insert can never hand a release someone else's amount.
struct ConcElems {
    int32_t *elem;
    uint8_t *pass;
};

// CCFC:57-70 for one acquire of `a` tokens at nowCalls `now`: int + int (wraps) compared with the double
// threshold; passes -> now += a.
__device__ inline bool conc_acquire(int32_t &now, int32_t a, double threshold) {
    const int32_t sum = (int32_t)((uint32_t)now + (uint32_t)a);
    if ((double)sum > threshold) return false;
    now = sum;
    return true;
}

constexpr int64_t CONC_INF = (int64_t)1 << 60;
struct MinPlus { int64_t p, c; };
__device__ inline MinPlus mp_then(MinPlus a, MinPlus b) {
    const int64_t ac = a.c >= CONC_INF ? CONC_INF : a.c + b.p;
    return MinPlus{a.p + b.p, ac < b.c ? ac : b.c};
}
__device__ inline int64_t mp_apply(MinPlus f, int64_t y) { return f.c >= CONC_INF ? y + f.p : min(y + f.p, f.c); }

__device__ inline int64_t conc_tprime(double threshold) {
    if (threshold != threshold || threshold >= (double)(CONC_INF / 4)) return CONC_INF / 4;   // NaN: never >
    if (threshold <= -(double)(CONC_INF / 4)) return -(CONC_INF / 4);
    return (int64_t)floor(threshold);
}

// Segmented scan state: the composition since the last segment head in the range (or of the whole
// range when it holds none), whether the range holds a head, and whether an amount other than +-1
// occurred since the last head (such a segment is left to k_conc_serial).
struct ConcSeg {
    int64_t p, c;
    uint32_t hd;
    uint32_t nu;
};
__device__ inline ConcSeg cs_identity() { return ConcSeg{0, CONC_INF, 0u, 0u}; }
__device__ inline ConcSeg cs_then(const ConcSeg &a, const ConcSeg &b) {
    if (b.hd) return b;
    const MinPlus f = mp_then(MinPlus{a.p, a.c}, MinPlus{b.p, b.c});
    return ConcSeg{f.p, f.c, a.hd, a.nu | b.nu};
}
__device__ inline ConcSeg cs_shfl(const ConcSeg &v, int src) {
    return ConcSeg{__shfl(v.p, src, WAVE), __shfl(v.c, src, WAVE), (uint32_t)__shfl((int)v.hd, src, WAVE),
                   (uint32_t)__shfl((int)v.nu, src, WAVE)};
}
__device__ inline ConcSeg cs_shfl_up(const ConcSeg &v, int o) {
    return ConcSeg{__shfl_up(v.p, o, WAVE), __shfl_up(v.c, o, WAVE), (uint32_t)__shfl_up((int)v.hd, o, WAVE),
                   (uint32_t)__shfl_up((int)v.nu, o, WAVE)};
}

// A tile's look-back descriptor is one 64-bit word, published and read with relaxed agent-scope atomics
// (no fence: on gfx950 an agent-scope release writes back the XCD's L2 and an acquire invalidates it):
//   bits 0-1 status (0 not yet, 1 aggregate, 2 inclusive), 2 head, 3 not-unit, 4 c = infinity,
//   5-33 p, 34-62 d = c - T' of the state's flow (29-bit two's complement each).
// Within a unit segment |p| and |d| are at most its length (< 2^28, MAX_BATCH); a larger value only
// occurs in a segment that is not unit, and saturates with the not-unit bit set.  The state's composition
// belongs to the flow of the range's last element, which is the reader's first flow whenever the reader
// uses it (otherwise the reader's first element is a head), so d is rebased on the reader's T'.
constexpr int64_t CS_LIM = ((int64_t)1 << 28) - 1;
__device__ inline uint64_t cs_pack(const ConcSeg &v, int64_t tp, uint64_t status) {
    uint64_t nu = v.nu;
    int64_t p = v.p;
    if (p > CS_LIM || p < -CS_LIM) { p = p > 0 ? CS_LIM : -CS_LIM; nu = 1; }
    const bool inf = v.c >= CONC_INF;
    int64_t d = inf ? 0 : v.c - tp;
    if (d > CS_LIM || d < -CS_LIM) { d = d > 0 ? CS_LIM : -CS_LIM; nu = 1; }
    return status | (uint64_t)(v.hd ? 1 : 0) << 2 | nu << 3 | (uint64_t)(inf ? 1 : 0) << 4 |
           ((uint64_t)p & 0x1FFFFFFFull) << 5 | ((uint64_t)d & 0x1FFFFFFFull) << 34;
}
__device__ inline ConcSeg cs_unpack(uint64_t w, int64_t tp) {
    const int64_t p = (int64_t)(w << 30) >> 35;
    const int64_t d = (int64_t)(w << 1) >> 35;
    return ConcSeg{p, (w >> 4) & 1 ? CONC_INF : tp + d, (uint32_t)(w >> 2) & 1u, (uint32_t)(w >> 3) & 1u};
}

constexpr int CS_THREADS = 256;
constexpr int CS_WAVES = CS_THREADS / WAVE;
#ifndef SENTINEL_CONC_ITEMS
#define SENTINEL_CONC_ITEMS 4
#endif
constexpr int CS_ITEMS = SENTINEL_CONC_ITEMS;               // consecutive sorted positions per thread
constexpr int64_t CS_TILE = (int64_t)CS_THREADS * CS_ITEMS;

// Per tile the look-back descriptor (zeroed by k_conc_prep); the tile ticket and the fallback list; per
// flow nowCalls after the batch.
struct ConcScan {
    unsigned long long *desc;
    uint32_t *ctl;           // [0] tile ticket, [1] segments left to k_conc_serial
    uint32_t *serial;        // their last positions
    int32_t *fin;            // [flow] nowCalls after the batch (stored by k_conc_apply)
    uint32_t *err;           // pinned: set when a look-back spin gave up (engine.hip, check_dev_err)
};

// A claimed release frees its token's slot (CCFC:92-100), given its neighbours' keys as read earlier
// in the same kernel.  No insert runs in the same kernel, and
// concurrent releases only turn slots from occupied to tombstone / empty, so an empty successor seen
// here stays empty and a stale plain read can only show an older, occupied successor (the release then
// leaves a tombstone the next sweep may free).  A slot followed by an empty one ends no probe chain, so
// it becomes empty, and so do the tombstones right before it (as k_tok_sweep); otherwise it becomes a
// tombstone.  In a sparse cache almost every release empties its slot.
__device__ inline void token_free(const TokenTable &TT, uint32_t h, TokRec r, unsigned long long nxt,
                                  unsigned long long prv, int64_t &dtomb) {
    r.claim = ~0u;
    r.key = nxt == PKEY_EMPTY ? PKEY_EMPTY : TOKEN_TOMB;
    TT.rec[h] = r;                                        // the whole record: no partial-sector write
    if (nxt == PKEY_EMPTY) {
        if (prv == TOKEN_TOMB) {
            uint64_t g = (h - 1) & TT.mask;
            for (int k = 0; k < 256; ++k) {               // (bounded walk back over tombstones)
                if (atomicCAS(&TT.rec[g].key, (unsigned long long)TOKEN_TOMB, (unsigned long long)PKEY_EMPTY) != TOKEN_TOMB) break;
                --dtomb;
                g = (g - 1) & TT.mask;
            }
        }
    } else {
        ++dtomb;
    }
}

// The batch's decisions: each workgroup takes a tile of CS_TILE sorted positions in ticket order (a
// tile's predecessors were taken earlier, so its look-back always completes), gathers the elements
// (freeing the claimed releases' slots), scans them, looks back for the state before the tile and
// decides its acquires; a segment's last position stores nowCalls after the batch, or hands the segment
// to k_conc_serial.
__global__ __launch_bounds__(CS_THREADS) void k_conc_scan(const uint64_t *__restrict__ sval,
                                                          const uint32_t *__restrict__ skey, uint32_t invalid, int64_t n,
                                                          TokenTable TT, const double *__restrict__ thr,
                                                          const int32_t *__restrict__ now_calls, ConcElems X, ConcScan S) {
    __shared__ ConcSeg s_w[CS_WAVES];
    __shared__ ConcSeg s_prefix;
    __shared__ int64_t s_tpl, s_tpf;
    __shared__ uint32_t s_tile;
    __shared__ bool s_lb;
    __shared__ unsigned long long s_cnt[2];
    const uint32_t t = threadIdx.x;
    const uint32_t lane = lane_id();
    const int wave = (int)(t / WAVE);
    if (t == 0) {
        s_tile = atomicAdd(&S.ctl[0], 1u);
        s_prefix = cs_identity();
    }
    if (t < 2) s_cnt[t] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const int64_t b = (int64_t)tile * CS_TILE + (int64_t)t * CS_ITEMS;

    uint32_t k[CS_ITEMS];
    int32_t x[CS_ITEMS];
    int64_t tp[CS_ITEMS];
#pragma unroll
    for (int q = 0; q < CS_ITEMS; ++q) k[q] = b + q < n ? skey[b + q] : invalid;
    const uint32_t kprev = b > 0 && b - 1 < n ? skey[b - 1] : invalid;
    const uint32_t knext = b + CS_ITEMS < n ? skey[b + CS_ITEMS] : invalid;
    int64_t dtomb = 0;
    unsigned long long freed = 0;
    // the gathers in phases, each phase's loads of all items in flight together: sorted values, the
    // released tokens' records, the claimed slots' neighbours; then the slots are freed
    uint64_t w[CS_ITEMS];
    TokRec r[CS_ITEMS];
    bool win[CS_ITEMS];
    unsigned long long nxt[CS_ITEMS], prv[CS_ITEMS];
#pragma unroll
    for (int q = 0; q < CS_ITEMS; ++q) w[q] = k[q] != invalid ? sval[b + q] : 0;
#pragma unroll
    for (int q = 0; q < CS_ITEMS; ++q)
        if (k[q] != invalid && ((w[q] >> CV_REL_BIT) & 1)) r[q] = TT.rec[(uint32_t)(w[q] >> CV_PAY_SHIFT)];
#pragma unroll
    for (int q = 0; q < CS_ITEMS; ++q) {
        x[q] = 0;
        win[q] = false;
        if (k[q] == invalid) continue;
        if (!((w[q] >> CV_REL_BIT) & 1)) {
            x[q] = (int32_t)(w[q] >> CV_PAY_SHIFT);       // an acquire: > 0 (validated)
        } else if (r[q].claim == ((uint32_t)w[q] & SEQ_MASK)) {   // CCFC:82-86: this release finds its token
            x[q] = -r[q].acquire;
            win[q] = true;
            const uint32_t h = (uint32_t)(w[q] >> CV_PAY_SHIFT);
            nxt[q] = TT.rec[(h + 1) & TT.mask].key;
            prv[q] = TT.rec[(h - 1) & TT.mask].key;
        }
    }
#pragma unroll
    for (int q = 0; q < CS_ITEMS; ++q)
        if (win[q]) {
            token_free(TT, (uint32_t)(w[q] >> CV_PAY_SHIFT), r[q], nxt[q], prv[q], dtomb);
            ++freed;
        }
    uint32_t kc = invalid;
    int64_t tc = 0;
#pragma unroll
    for (int q = 0; q < CS_ITEMS; ++q) {
        tp[q] = 0;
        if (k[q] == invalid) continue;
        if (k[q] != kc) {
            kc = k[q];
            tc = conc_tprime(thr[kc]);
        }
        tp[q] = tc;
    }
    if (freed) atomicAdd(&s_cnt[0], 0ull - freed);        // (one live token less per release)
    if (dtomb) atomicAdd(&s_cnt[1], (unsigned long long)dtomb);

    // this thread's composition, the wave's and the block's inclusive scan; T' of the tile's first and
    // last valid elements (the descriptor's rebasing)
    ConcSeg mine = cs_identity();
#pragma unroll
    for (int q = 0; q < CS_ITEMS; ++q) {
        if (k[q] == invalid) continue;
        const bool head = k[q] != (q ? k[q - 1] : kprev);
        const int32_t v = x[q];
        const ConcSeg el{(int64_t)v, v > 0 ? tp[q] : CONC_INF, head ? 1u : 0u, (v > 1 || v < -1) ? 1u : 0u};
        mine = cs_then(mine, el);
        if ((q + 1 < CS_ITEMS ? k[q + 1] : knext) == invalid || (t == CS_THREADS - 1 && q == CS_ITEMS - 1))
            s_tpl = tp[q];                                // the tile's last valid element
    }
    if (t == 0) {
        s_tpf = tp[0];
        s_lb = tile > 0 && k[0] != invalid && k[0] == kprev;    // the tile continues a segment
    }
    ConcSeg inc = mine;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const ConcSeg u = cs_shfl_up(inc, o);
        if ((int)lane >= o) inc = cs_then(u, inc);
    }
    if (lane == WAVE - 1) s_w[wave] = inc;
    __syncthreads();
    ConcSeg wpre = cs_identity(), tagg = cs_identity();
#pragma unroll
    for (int w = 0; w < CS_WAVES; ++w) {
        if (w < wave) wpre = cs_then(wpre, s_w[w]);
        tagg = cs_then(tagg, s_w[w]);
    }
    ConcSeg excl = cs_shfl_up(inc, 1);
    if (lane == 0) excl = cs_identity();
    excl = cs_then(wpre, excl);                           // the tile's positions before this thread's

    // publish the tile's descriptor: inclusive at once unless the tile continues a segment with no head
    // of its own; such a tile looks back over earlier tiles (last wave, 64 tiles at a time, waiting only
    // for the tiles up to the nearest inclusive descriptor, composed earliest first)
    const bool lb = s_lb;
    const bool early = !lb || tagg.hd;
    const int64_t tpl = s_tpl, tpf = s_tpf;
    if (t == CS_THREADS - 1)
        __hip_atomic_store(&S.desc[tile], cs_pack(tagg, tpl, early ? 2u : 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lb && t >= CS_THREADS - WAVE) {
        ConcSeg pre = cs_identity();                      // tiles between the window and this one
        int64_t top = tile;                               // the window ends below top
        uint32_t spins = 0;
        for (;;) {
            const int64_t p = top - 1 - (int64_t)lane;    // lane 0: the nearest tile
            // (a position before tile 0 reads as an inclusive identity)
            const uint64_t f = p >= 0 ? __hip_atomic_load(&S.desc[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : (2ull | 1ull << 4);
            const uint64_t st = f & 3u;
            const uint64_t incl = __builtin_amdgcn_ballot_w64(st == 2u);
            const uint64_t waiting = __builtin_amdgcn_ballot_w64(st == 0u);
            const int first = incl ? __ffsll((unsigned long long)incl) - 1 : WAVE;   // the nearest inclusive one
            const uint64_t need = first >= WAVE - 1 ? ~0ull : ((2ull << first) - 1);
            if (waiting & need) {
                // tiles take tickets in order and publish without waiting, so a tile's predecessors always
                // publish: the bound only turns a broken invariant into a reported error instead of a hang
                if (++spins > (1u << 22)) {
                    if (lane == 0) __hip_atomic_store(S.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            const ConcSeg v = (int)lane <= first ? cs_unpack(f, tpf) : cs_identity();
            ConcSeg w = cs_identity();                    // lanes min(first, 63) .. 0, earliest first
            for (int l = min(first, WAVE - 1); l >= 0; --l) w = cs_then(w, cs_shfl(v, l));
            pre = cs_then(w, pre);
            if (first < WAVE) break;
            top -= WAVE;
        }
        if (t == CS_THREADS - 1) {
            s_prefix = pre;
            if (!early)
                __hip_atomic_store(&S.desc[tile], cs_pack(cs_then(pre, tagg), tpl, 2u), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (t == 0) {
        if (s_cnt[0]) tok_count_add(TT, 0, s_cnt[0]);
        if (s_cnt[1]) tok_count_add(TT, 1, s_cnt[1]);
    }
    const ConcSeg E = cs_then(s_prefix, excl);            // the sorted positions before this thread's

    // decide: y = nowCalls before each position (nowCalls before the batch at a segment head)
    int64_t y = 0, n0 = 0;
    uint32_t nu = E.nu;
    bool started = false;
#pragma unroll
    for (int q = 0; q < CS_ITEMS; ++q) {
        if (k[q] == invalid) continue;
        const int64_t i = b + q;
        const bool head = k[q] != (q ? k[q - 1] : kprev);
        if (head || !started) {
            n0 = now_calls[k[q]];
            if (head) {
                y = n0;
                nu = 0;
            } else {
                y = mp_apply(MinPlus{E.p, E.c}, n0);
            }
            started = true;
        }
        const int32_t v = x[q];
        if (v > 1 || v < -1) nu = 1;
        X.elem[i] = v;
        if (v > 0) {
            X.pass[i] = y < tp[q] ? 1 : 0;
            y = min(y + 1, tp[q]);
        } else {
            y += v;
        }
        if ((q + 1 < CS_ITEMS ? k[q + 1] : knext) != k[q]) {                 // the segment's last position
            // exact while every amount is +-1, nowCalls starts at or below T' and cannot wrap an int
            if (!nu && n0 <= tp[q] && (n0 < 0 ? -n0 : n0) + n < (int64_t)INT32_MAX) {
                S.fin[k[q]] = (int32_t)y;
            } else {
                S.serial[atomicAdd(&S.ctl[1], 1u)] = (uint32_t)i;
            }
        }
    }
}

// Segments the scan cannot decide: one thread walks each with the CCFC:57-98 recurrence (integer work
// on the elements only; amounts other than 1 and nowCalls above T' are rare).  The list holds the
// segments' last positions; the first is found by a binary search of the sorted keys.
__global__ __launch_bounds__(256) void k_conc_serial(const uint32_t *__restrict__ skey, int64_t n,
                                                     const int32_t *__restrict__ now_calls,
                                                     const double *__restrict__ thr, ConcElems X, ConcScan S) {
    const uint32_t cnt = S.ctl[1];
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < cnt; r += gridDim.x * blockDim.x) {
        const int64_t last = S.serial[r];
        const uint32_t flow = skey[last];
        int64_t lo = 0, hi = last;                        // the first position whose key is `flow`
        while (lo < hi) {
            const int64_t m = (lo + hi) >> 1;
            if (skey[m] < flow) lo = m + 1;
            else hi = m;
        }
        const int64_t b = lo;
        int32_t now = now_calls[flow];
        const double threshold = thr[flow];
        for (int64_t i0 = b;; i0 += 8) {
            uint32_t kk[8];
            int32_t xx[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                kk[q] = i0 + q < n ? skey[i0 + q] : ~flow;
                xx[q] = kk[q] == flow ? X.elem[i0 + q] : 0;
            }
            bool end = false;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (kk[q] != flow) { end = true; break; }
                if (xx[q] > 0) X.pass[i0 + q] = conc_acquire(now, xx[q], threshold) ? 1 : 0;
                else if (xx[q] < 0) now = (int32_t)((uint32_t)now + (uint32_t)xx[q]);     // CCFC:97-98
            }
            if (end) break;
        }
        S.fin[flow] = now;
    }
}

// The effects, one thread per sorted position (CCFC:57-100): a passing acquire takes a token
// (TokenCacheNode, id = id_base + sorted position), a failing one answers BLOCKED; a claimed release
// (freed by k_conc_scan) answers RELEASE_OK, any other release ALREADY_RELEASE; a segment's last position
// stores the flow's nowCalls.  Cache counts {live, tombstones} by one atomic pair per workgroup.
__global__ __launch_bounds__(256) void k_conc_apply(const uint64_t *__restrict__ sval, const uint32_t *__restrict__ skey,
                                                    uint32_t invalid, int64_t n, ConcElems X,
                                                    TokenTable TT, const int64_t *__restrict__ flow_ids, uint64_t id_base,
                                                    const int32_t *__restrict__ fin, int32_t *__restrict__ now_calls,
                                                    uint64_t *__restrict__ out) {
    __shared__ unsigned long long s_cnt[2];
    if (threadIdx.x < 2) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t dlive = 0, dtomb = 0;
    const uint32_t flow = i < n ? skey[i] : invalid;
    if (flow != invalid) {
        const uint32_t seq = (uint32_t)sval[i] & SEQ_MASK;
        const int32_t x = X.elem[i];
        if (x > 0) {
            if (!X.pass[i]) {
                put_conc(out, seq, 0, ST_BLOCKED);                            // CCFC:57-69
            } else {
                const uint64_t id = id_base + (uint64_t)i;                    // TokenCacheNode.java:59-70 (unique;
                                                                              // names its ring slot)
                bool tomb = false;
                const int64_t h = token_insert(TT, id, tomb);
                if (h < 0) {                                                  // token cache full
                    put_conc(out, seq, 0, ST_FAIL);
                } else {
                    if (tomb) --dtomb;
                    TT.rec[h] = TokRec{id, flow_ids[flow], (int32_t)flow, x, ~0u, 0u};   // (whole record)
                    ++dlive;
                    put_conc(out, seq, (int64_t)id, ST_OK);
                }
            }
        } else if (x < 0) {
            put_conc(out, seq, 0, ST_RELEASE_OK);
        } else {
            put_conc(out, seq, 0, ST_ALREADY_RELEASE);
        }
        if (i + 1 == n || skey[i + 1] != flow) now_calls[flow] = fin[flow];
    }
    if (dlive) atomicAdd(&s_cnt[0], (unsigned long long)dlive);
    if (dtomb) atomicAdd(&s_cnt[1], (unsigned long long)dtomb);    // (two's complement: wraps to a decrement)
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_cnt[0]) tok_count_add(TT, 0, s_cnt[0]);
        if (s_cnt[1]) tok_count_add(TT, 1, s_cnt[1]);
    }
}

// Tombstone sweep of the whole token cache (between batches): a tombstone whose successor slot is empty
// ends no probe chain (every cached token's chain from its home slot is unbroken, so it cannot pass
// through a slot followed by an empty one), so it may become empty itself, and so may the tombstones
// right before it.  Nothing is inserted during the sweep, so an empty successor stays empty.  Run when the
// host's bound on live + tombstones nears the compaction threshold: at a low load factor most released
// tokens sit alone in their cluster, so the sweep (one coalesced pass over the keys) usually makes the
// compaction (a rehash of every live token into a new table) unnecessary.
__global__ __launch_bounds__(256) void k_tok_sweep(TokenTable TT) {
    __shared__ unsigned long long s_freed;
    if (threadIdx.x == 0) s_freed = 0;
    __syncthreads();
    uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long freed = 0;
    if (h <= TT.mask && TT.rec[h].key == TOKEN_TOMB && TT.rec[(h + 1) & TT.mask].key == PKEY_EMPTY) {
        for (int k = 0; k < 256; ++k) {                   // (bounded walk back)
            if (atomicCAS(&TT.rec[h].key, (unsigned long long)TOKEN_TOMB, (unsigned long long)PKEY_EMPTY) != TOKEN_TOMB)
                break;
            ++freed;
            h = (h - 1) & TT.mask;
            if (TT.rec[h].key != TOKEN_TOMB) break;
        }
    }
    if (freed) atomicAdd(&s_freed, freed);
    __syncthreads();
    if (threadIdx.x == 0 && s_freed) tok_count_add(TT, 1, 0ull - s_freed);
}

// {live tokens, tombstones} of the cache into pinned host memory, stream-ordered after a batch (one
// wave sums the striped counters): the host reads it once the batch's event has completed, so its bound
// on live + tombstones tracks the cache without a synchronisation (engine.hip, submit_concurrent).
__global__ __launch_bounds__(WAVE) void k_tok_snapshot(const unsigned long long *__restrict__ counts,
                                                      unsigned long long *dst) {
    const int l = threadIdx.x;
    long long live = l < TOK_CNT_LANES ? (long long)counts[l * TOK_CNT_STRIDE] : 0;
    long long tomb = l < TOK_CNT_LANES ? (long long)counts[l * TOK_CNT_STRIDE + 1] : 0;
    for (int o = WAVE / 2; o > 0; o >>= 1) {
        live += __shfl_xor(live, o, WAVE);
        tomb += __shfl_xor(tomb, o, WAVE);
    }
    if (l == 0) {
        __hip_atomic_store(&dst[0], (unsigned long long)live, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&dst[1], (unsigned long long)tomb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// RegularExpireStrategy.clearToken (RegularExpireStrategy.java:94-124): with the reference's own
// conditions every cached token qualifies (clientTimeout / resourceTimeout are durations compared
// with the wall clock), so a sweep removes up to `max_tokens` tokens and returns their counts to
// nowCalls (a token whose rule is gone just leaves the cache).
__global__ __launch_bounds__(256) void k_conc_expire(TokenTable TT, int32_t *now_calls, unsigned long long max_tokens,
                                                     unsigned long long *ticket) {
    const uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h > TT.mask) return;
    const unsigned long long k = TT.rec[h].key;
    if (k == PKEY_EMPTY || k == TOKEN_TOMB) return;
    if (atomicAdd(ticket, 1ull) >= max_tokens) return;
    TT.rec[h].key = TOKEN_TOMB;
    tok_count_add(TT, 0, ~0ull);
    tok_count_add(TT, 1, 1ull);
    const int32_t f = TT.rec[h].flow_idx;
    if (f >= 0) atomicSub(&now_calls[f], TT.rec[h].acquire);
}

}  // namespace sentinel
