// param_rules.hpp -- hot-parameter requests decided one rule at a time (gfx950).
//
// Three checkers share one pipeline: events are grouped by rule (K2 radix sort, arrival order
// kept), and one lane walks each rule's events in order:
//
//   PMODE_EXACT  ClusterParamFlowChecker.acquireClusterToken over any number of values
//                (srv/flow/ClusterParamFlowChecker.java:42-87): every value is checked in order,
//                the first negative remaining blocks the request with no counter touched, else
//                every value's window counter is incremented (duplicates twice).  Per-value
//                state is the exact open-addressing slot of admission.hpp (KIND_PARAM keys).
//   PMODE_CM     the same checker over a count-min sketch of window counters (opt-in): every
//                rule owns depth x width cells of n slots {tag = epoch mod 2^24, count} (or every
//                rule shares one sketch keyed by the rule-unique param key, when all param rules
//                have one window: then a stale tag is always older by >= n epochs); the
//                estimate is the minimum over rows of the cell's window sum, so it never
//                undercounts the value's own passes (the sketch only adds) and a request can be
//                blocked that exact counters would pass, never the reverse.
//   PMODE_LOCAL  ParamFlowChecker.passLocalCheck / passDefaultLocalCheck
//                (pfc/slots/block/flow/param/ParamFlowChecker.java:78-202): a token bucket
//                {lastAddTokenTime, tokens} per (rule, value), every element of a collection
//                must pass, earlier elements keep their consumed tokens.
//
// A value list couples several counters of one rule, so a rule's events cannot be split into
// independent per-key segments: the per-rule lane is the "wave-per-segment fallback" of the
// north star applied at rule granularity.  Single-value cluster requests in exact mode keep the
// closed-form per-key path of admission.hpp.
#pragma once

#include "admission.hpp"

namespace sentinel {

// sentinel_param_multi_event_t.  Its first 16 bytes are those of Event / ParamEvent, so the sort,
// segment and limiter kernels read it through a ParamEvent pointer.
struct MultiEvent {
    int32_t idx;
    int32_t acquire;
    int64_t ts;
    int32_t begin;
    int32_t count;
};
static_assert(sizeof(MultiEvent) == sizeof(ParamEvent), "multi events share the ParamEvent stride");

// Value list of event s: single-value events carry their value (param key) in the event.
struct ValueSrc {
    const ParamEvent *pev;
    const MultiEvent *mev;
    const uint64_t *values;
    int64_t n_values;
    __device__ inline int32_t begin(uint32_t s) const { return pev ? (int32_t)s : mev[s].begin; }
    __device__ inline int32_t count(uint32_t s) const { return pev ? 1 : mev[s].count; }
    __device__ inline uint64_t value(int64_t j) const { return pev ? pev[j].key : values[j]; }
};

// Cluster param rule table (dense rule index) + hot items keyed by param key.
struct ParamRules {
    const int32_t *n;
    const int32_t *w;
    const double *rcp_w;
    const double *I_s;
    const double *thr;                    // count, x connectedCount for AVG_LOCAL (CPFC:101-111)
    const unsigned long long *hot_keys;   // null: no hot items
    uint64_t hot_mask;
    const double *hot_thr;
};

// Per-slot window parameters written by the prep kernel (exact mode).
struct SlotMeta {
    int32_t *n;
    int32_t *w;
    double *rcp;
    double *Is;
    double *thr;
    uint8_t *kind;
    int32_t *rule;        // the slot's rule (read by the slot-table rebuild and the top-values query)
    int64_t *state;       // the slots' windows (stride words each): a fresh insert writes its n absent pairs
    int64_t stride;
};

// A freshly inserted slot's window: n absent buckets (the table's state is not pre-initialised: a
// rebuild only clears the keys, the inserting thread writes the window before any kernel reads it).
__device__ inline void slot_state_init(int64_t *state, int64_t stride, uint64_t h, int n) {
    int64_t *st = state + (int64_t)h * stride;
    for (int j = 0; j < n; ++j) *reinterpret_cast<longlong2 *>(st + 2 * j) = longlong2{EPOCH_ABSENT, 0};
}

// Count-min sketch: rule-major [rule][depth][width][nmax] packed cells.
struct CountMin {
    uint64_t *cells;
    int32_t depth;
    uint32_t width;       // power of two
    int32_t nmax;         // slots per cell: n (per-rule sketch), 2 n (shared: a ring of two windows)
    bool shared;          // one sketch for every rule (param keys are unique per (rule, value))
    // shared sketch, round 5: each row's width is cut into 2^cbits blocks of `cols` columns; a key's d
    // cells all lie in block (top cbits bits of mix64(key)) -- the same bits the partition path groups
    // requests by -- so one workgroup owns a block and stages it in LDS (k_pp_cm_block)
    int32_t cbits;
    uint32_t cols;
};
constexpr uint32_t CM_BLOCK_COLS = 64;       // columns per row in one block of the shared sketch

constexpr int64_t LOCAL_ABSENT = INT64_MIN;   // CacheMap entry absent

// Local param rules (position = rule index) + hot items + token-bucket state per slot.
struct LocalRules {
    const uint8_t *valid;
    const int64_t *tokens;    // (long) rule.count  (PFC:139)
    const int64_t *burst;     // rule.burstCount    (PFC:148)
    const int64_t *dur_ms;    // rule.durationInSec * 1000 (PFC:166)
    const unsigned long long *hot_keys;
    uint64_t hot_mask;
    const int64_t *hot_tokens;
    int64_t *state;           // per slot {lastAddTokenTime, tokens}; THREAD grade: {-, thread count}
    const uint8_t *grade;     // per rule: 1 QPS (token bucket), 0 THREAD; null: all QPS
    const uint8_t *kinds;     // per event: 1 = Entry.exit (thread counts drop), else a check; null: checks
};

struct ParamCtx {
    ParamRules R;
    KeyTable PT;              // exact-mode slot state
    CountMin CM;
    LocalRules L;
    const uint32_t *vslot;    // slot of each value (exact / local)
};

constexpr int PMODE_EXACT = 0;
constexpr int PMODE_CM = 1;
constexpr int PMODE_LOCAL = 2;

// ClusterParamFlowChecker.getRawThreshold (CPFC:113-120): hot-item count, else rule count.
__device__ inline double value_threshold(const ParamRules &R, uint32_t rule, uint64_t key) {
    const int64_t h = slot_find(R.hot_keys, R.hot_mask, key);
    return h >= 0 ? R.hot_thr[h] : R.thr[rule];
}

// A cluster param request at ts < 0 (no namespace limiter): LeapArray.currentWindow(t < 0) == null
// (LeapArray.java:149-152) and values(t < 0) is empty (:375-378), so every value's getAvg is 0; a value
// with (T_v - 0) - a < 0 blocks the request with no counter touched (CPFC:66-70), and a request that
// would pass dies in addValue's currentWindow().value() (ClusterParamMetric.java:69,
// NullPointerException), which the engine answers FAIL.  With a namespace limiter the limiter's add dies
// first (FAIL).
__device__ inline int param_negative_ts_status(const ParamRules &R, uint32_t rule, uint64_t key, int32_t a) {
    return ((value_threshold(R, rule, key) - 0.0) - (double)a < 0.0) ? ST_BLOCKED : ST_FAIL;
}

// ------------------------------------------------------------------ prep

// Validation + routing of single- or multi-value events, slot of every value, sort keys (rule
// index) and the pass-0 digit histograms.  Cluster: DefaultTokenService.requestParamToken
// (DTS:51-62: null id, acquire <= 0, empty params -> BAD_REQUEST; unknown rule -> NO_RULE_EXISTS)
// and ClusterParamFlowChecker.allowProceed (CPFC:37-47).  Local: ParamFlowChecker.passCheck
// reaches passLocalCheck with no request validation; an empty collection passes (PFC:81-102).
template <bool LOCAL>
__global__ __launch_bounds__(SORT_THREADS) void k_prule_prep(
    int64_t n, const ParamEvent *__restrict__ ev, ValueSrc vs, int32_t nrules, const uint8_t *__restrict__ rule_valid,
    const int32_t *__restrict__ route, ParamRules R, unsigned long long *table, uint64_t cap_mask,
    unsigned long long *fresh, SlotMeta M,
    uint32_t *__restrict__ vslot, uint64_t *__restrict__ out, uint32_t *__restrict__ fkey, uint32_t finvalid,
    uint32_t *__restrict__ fhist, uint32_t *__restrict__ lkey, uint32_t linvalid, uint32_t *__restrict__ lhist,
    int64_t nblocks) {
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
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        if (i >= n) break;
        const ParamEvent e = ev[i];
        const int32_t cnt = vs.count((uint32_t)i);
        const int32_t b = vs.begin((uint32_t)i);
        const bool bad_range = cnt < 0 || b < 0 || (int64_t)b + cnt > vs.n_values;
        int st = 127;
        uint32_t l = linvalid;
        if (LOCAL) {
            if (bad_range) st = ST_BAD_REQUEST;
            else if (e.idx < 0 || e.idx >= nrules || (rule_valid && !rule_valid[e.idx])) st = ST_NO_RULE_EXISTS;
            else if (cnt == 0) st = ST_OK;
        } else {
            if (e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0 || cnt <= 0) st = ST_BAD_REQUEST;
            else if (bad_range) st = ST_BAD_REQUEST;
            else if (e.idx < 0 || e.idx >= nrules) st = ST_NO_RULE_EXISTS;
            else {
                const int32_t r = route ? route[e.idx] : ROUTE_PLAIN;
                if (r == ROUTE_TOO_MANY) st = ST_TOO_MANY_REQUEST;   // namespace == null
                else if (e.ts < 0) {                                   // param_negative_ts_status
                    st = ST_FAIL;
                    if (r < 0 && !bad_range)
                        for (int32_t q = 0; q < cnt; ++q)
                            if (param_negative_ts_status(R, (uint32_t)e.idx, vs.value((int64_t)b + q), e.acquire) == ST_BLOCKED) {
                                st = ST_BLOCKED;
                                break;
                            }
                }
                else if (r >= 0) l = (uint32_t)r;
            }
        }
        if (st == 127 && table) {
            for (int32_t q = 0; q < cnt; ++q) {
                const uint64_t key = vs.value((int64_t)b + q);
                const uint32_t before = nfresh;
                const int64_t h = slot_insert_counted(table, cap_mask, key, nfresh);
                if (h < 0) { st = ST_FAIL; break; }                    // table full
                vslot[b + q] = (uint32_t)h;
                if (!LOCAL) {   // identical values from every writer of this slot: stored only when they differ
                    const int32_t rn = R.n[e.idx], rw = R.w[e.idx];
                    if (nfresh != before) slot_state_init(M.state, M.stride, (uint64_t)h, rn);
                    const double rc = R.rcp_w[e.idx], is = R.I_s[e.idx];
                    const double th = value_threshold(R, (uint32_t)e.idx, key);
                    if (M.rule[h] != e.idx) M.rule[h] = e.idx;
                    if (M.n[h] != rn) M.n[h] = rn;
                    if (M.w[h] != rw) M.w[h] = rw;
                    if (__double_as_longlong(M.rcp[h]) != __double_as_longlong(rc)) M.rcp[h] = rc;
                    if (__double_as_longlong(M.Is[h]) != __double_as_longlong(is)) M.Is[h] = is;
                    if (__double_as_longlong(M.thr[h]) != __double_as_longlong(th)) M.thr[h] = th;
                    if (M.kind[h] != KIND_PARAM) M.kind[h] = KIND_PARAM;
                }
            }
        }
        const uint32_t k = st == 127 ? (uint32_t)e.idx : finvalid;
        if (st != 127) l = linvalid;
        fkey[i] = k;
        tile_hist_accumulate(hf, k, 1);
        if (lkey) {
            lkey[i] = l;
            tile_hist_accumulate(hl, l, 1);
        }
        if (st != 127) put_verdict(out, (uint32_t)i, st, 0, 0);
    }
    block_add_global(fresh, nfresh, &s_fresh);              // (synchronises the block)
    tile_hist_store(hf, fhist, 1, nblocks);
    if (lkey) tile_hist_store(hl, lhist, 1, nblocks);
}

// ------------------------------------------------------------------ checkers

// Exact counters: ClusterParamFlowChecker.acquireClusterToken (CPFC:58-86).  getAvg(value) rolls the
// value's window first (ClusterParamMetric.java:46-82 -> LeapArray.currentWindow).
__device__ inline uint64_t exact_check(const ParamCtx &C, int64_t E, int32_t a, int32_t b, int32_t cnt) {
    double remaining = -1.0;
    for (int32_t q = 0; q < cnt; ++q) {
        const uint32_t s = C.vslot[b + q];
        const KeyState ks = key_state(C.PT, s);
        roll(C.PT, s, ks, E);
        const int64_t sum = window_sum(ks, E, EV_PASS);
        const double next = remaining_of(C.PT.thr[s], C.PT.I_s[s], sum, a);
        remaining = next;
        if (next < 0.0) return pack_verdict(ST_BLOCKED, 0, 0);    // CPFC:66-70, no counter touched
    }
    for (int32_t q = 0; q < cnt; ++q) {                            // CPFC:73-76
        const uint32_t s = C.vslot[b + q];
        const KeyState ks = key_state(C.PT, s);
        add_counter(C.PT, s, ks, E, EV_PASS, a);
    }
    if (cnt > 1) remaining = -1.0;                                 // CPFC:81-84
    return pack_verdict(ST_OK, java_d2i(remaining), 0);
}

// Count-min cells: {tag = epoch mod 2^24 : 24 | count : 40}.
constexpr int CM_COUNT_BITS = 40;
constexpr uint64_t CM_COUNT_MAX = (1ull << CM_COUNT_BITS) - 1;
constexpr uint32_t CM_TAG_MASK = (1u << 24) - 1;

__host__ __device__ inline uint64_t cm_block_of(const CountMin &C, uint64_t key) {
    return C.cbits ? mix64(key) >> (64 - C.cbits) : 0ull;
}
// Row d's cell of a key.  Per-rule sketch: column = an independent hash per row over the full width.
// Shared sketch: block-major (block, row, column), the column an independent hash per row over the
// block's `cols` columns -- a row still has width = 2^cbits x cols cells and two keys meet in a row
// with probability 1 / width, but only keys of the same block can meet (the bound
// is stated against the block's total count).
__host__ __device__ inline uint64_t *cm_cell(const CountMin &C, uint32_t rule, int d, uint64_t key) {
    const uint64_t hd = mix64(key + 0x9E3779B97F4A7C15ull * (uint64_t)(d + 1));
    if (C.shared) {
        const uint64_t col = hd & (uint64_t)(C.cols - 1);
        return C.cells + ((cm_block_of(C, key) * (uint64_t)C.depth + (uint64_t)d) * C.cols + col) * (uint64_t)C.nmax;
    }
    const uint64_t col = hd & (uint64_t)(C.width - 1);
    return C.cells + (((uint64_t)rule * (uint64_t)C.depth + (uint64_t)d) * C.width + col) * (uint64_t)C.nmax;
}

// Window sum of one cell at epoch E: slots tagged with one of the epochs (E-n, E] (a tag 2^24
// epochs stale aliases into the window: it can only add, never remove, count).  `slots`: n, or 2 n
// in the shared sketch's ring.
__host__ __device__ inline int64_t cm_cell_sum(const uint64_t *c, int nsc, int64_t E, int slots = 0) {
    int64_t s = 0;
    if (slots <= 0) slots = nsc;
    for (int j = 0; j < slots; ++j) {
        const uint64_t x = c[j];
        const uint32_t tag = (uint32_t)(x >> CM_COUNT_BITS);
        if ((((uint32_t)E - tag) & CM_TAG_MASK) < (uint32_t)nsc) s += (int64_t)(x & CM_COUNT_MAX);
    }
    return s;
}

__device__ inline int64_t cm_estimate(const CountMin &C, uint32_t rule, uint64_t key, int nsc, int64_t E) {
    int64_t est = INT64_MAX;
    for (int d = 0; d < C.depth; ++d) {
        const int64_t s = cm_cell_sum(cm_cell(C, rule, d, key), nsc, E);
        est = s < est ? s : est;
    }
    return est;
}

// Add a to the value's slot E mod n in every row; a slot tagged with another epoch restarts at
// zero (the LeapArray reset); counts saturate instead of wrapping (never undercount).
__device__ inline void cm_add(const CountMin &C, uint32_t rule, uint64_t key, int nsc, int64_t E, int32_t a) {
    const int j = (int)(E % nsc);
    const uint64_t tag = (uint64_t)((uint32_t)E & CM_TAG_MASK) << CM_COUNT_BITS;
    for (int d = 0; d < C.depth; ++d) {
        uint64_t *c = cm_cell(C, rule, d, key) + j;
        const uint64_t x = *c;
        uint64_t cnt = ((x & ~CM_COUNT_MAX) == tag) ? (x & CM_COUNT_MAX) : 0;
        cnt += (uint64_t)(uint32_t)a;
        if (cnt > CM_COUNT_MAX) cnt = CM_COUNT_MAX;
        *c = tag | cnt;
    }
}

__device__ inline uint64_t cm_check(const ParamCtx &C, uint32_t rule, int64_t E, int32_t a, const ValueSrc &vs,
                                    int32_t b, int32_t cnt) {
    const int nsc = C.R.n[rule];
    const double I_s = C.R.I_s[rule];
    double remaining = -1.0;
    for (int32_t q = 0; q < cnt; ++q) {
        const uint64_t key = vs.value((int64_t)b + q);
        const int64_t est = cm_estimate(C.CM, rule, key, nsc, E);
        const double next = remaining_of(value_threshold(C.R, rule, key), I_s, est, a);
        remaining = next;
        if (next < 0.0) return pack_verdict(ST_BLOCKED, 0, 0);
    }
    for (int32_t q = 0; q < cnt; ++q) cm_add(C.CM, rule, vs.value((int64_t)b + q), nsc, E, a);
    if (cnt > 1) remaining = -1.0;
    return pack_verdict(ST_OK, java_d2i(remaining), 0);
}

// ---------------------------------------------------------------------------------------------
// Shared count-min sketch (one sketch for every rule): the cells are shared between rules, so the
// rules' lanes must move through the batch's epochs together.  If one rule's lane ran far ahead and
// reset a cell slot, a lagging lane would lose the count it had put there and could then admit what
// the exact checker blocks.  Each shared cell therefore keeps a ring of 2 n slots (epoch E in slot
// E mod 2n): a lane at epoch E' resets the slot of E' - 2n, and as long as every lane is within n
// epochs of the slowest one (at L: it needs epochs > L - n), no reset can remove a count anybody still
// reads.  k_prule_cm_sync decides band by band: band start L = the smallest epoch any rule still has
// pending; every lane decides its rules' segments at epochs < L + n (a rule's epochs only go up
// under the documented precondition of per-rule non-decreasing timestamps; a late segment is decided
// at once rather than waited for), then a grid barrier -- n times fewer barriers than one per
// epoch.  Within a band every cell update is atomic (a CAS loop): concurrent rules only add count to
// each other's cells (over-estimate, never under), so the sketch stays one-sided.  Cells are read with
// device-scope atomic loads (other CUs' updates, no stale L1).
__device__ inline uint64_t cm_load(const uint64_t *c) {
    return __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the n slots of one cell, every load in flight before the sum (device-scope loads: no stale L1)
constexpr int CM_NMAX = 32;                   // ring slots (2 n, n <= 16)
__device__ inline int64_t cm_cell_sum_sync(const uint64_t *c, int nsc, int64_t E) {
    uint64_t x[CM_NMAX];
    const int slots = 2 * nsc;
#pragma unroll
    for (int j = 0; j < CM_NMAX; ++j) x[j] = j < slots ? cm_load(c + j) : 0ull;
    int64_t s = 0;
#pragma unroll
    for (int j = 0; j < CM_NMAX; ++j) {
        const uint32_t tag = (uint32_t)(x[j] >> CM_COUNT_BITS);
        if (j < slots && (((uint32_t)E - tag) & CM_TAG_MASK) < (uint32_t)nsc) s += (int64_t)(x[j] & CM_COUNT_MAX);
    }
    return s;
}

// The epoch an add goes to, relative to the batch's newest epoch Eref: its tag te = E mod 2^24, Eref's tag
// and dE = Eref - E (every epoch a batch adds to lies in [Eref - dE, Eref]; saturated at 2^24 - 1).
struct CmTag {
    uint32_t te, eref, dE;
};
__host__ __device__ inline CmTag cm_tag(int64_t E, int64_t Eref) {
    const int64_t d = Eref - E;
    return CmTag{(uint32_t)E & CM_TAG_MASK, (uint32_t)Eref & CM_TAG_MASK,
                 d <= 0 ? 0u : d >= (int64_t)CM_TAG_MASK ? CM_TAG_MASK : (uint32_t)d};
}

// Add a to one cell slot of epoch E: same tag -> add (saturating); a newer epoch -> add to it (another key
// or lane reached a later epoch congruent mod 2n first: over-count, never under); any other tag -> restart
// at a.  "Newer" is decided by distance to Eref: every epoch written by this batch, or under the
// precondition by an earlier one, is <= Eref, so the slot's epoch lies in (E, Eref] iff Eref - tag < dE
// (mod 2^24).  A half-range test on tag - te would take a slot idle 2^23 .. 2^24 epochs (mod 2^24) for a
// newer one, keep its stale tag and lose the add (the 8-bit form of the same test).
// Residual aliasing: a slot idle exactly k 2^24 + j epochs, 0 < j < dE (19.4 days per 2^24 epochs at
// 100 ms), still counts as newer.  `x` = the caller's guess of the slot's current word (a failed CAS
// returns the real one).
__host__ __device__ inline unsigned long long cm_slot_next(unsigned long long x, const CmTag &g, int64_t a) {
    const uint32_t tag = (uint32_t)(x >> CM_COUNT_BITS);
    // (an empty cell, count 0, has no epoch: its tag bits mean nothing)
    const bool newer = (x & CM_COUNT_MAX) != 0 && ((g.eref - tag) & CM_TAG_MASK) < g.dE;
    uint64_t cnt = (tag == g.te || newer) ? (x & CM_COUNT_MAX) : 0;
    cnt = (uint64_t)a > CM_COUNT_MAX - cnt ? CM_COUNT_MAX : cnt + (uint64_t)a;   // (a >= 0)
    return ((unsigned long long)(newer ? tag : g.te) << CM_COUNT_BITS) | cnt;
}

__device__ inline void cm_slot_add(unsigned long long *c, unsigned long long x, const CmTag &g, int64_t a) {
    for (;;) {
        const unsigned long long prev = atomicCAS(c, x, cm_slot_next(x, g, a));
        if (prev == x) break;
        x = prev;
    }
}

// Add a to the slot of E in every row (Eref: the batch's newest epoch).
__device__ inline void cm_add_sync(const CountMin &C, uint32_t rule, uint64_t key, int nsc, int64_t E, int64_t Eref,
                                   int64_t a) {
    const int j = (int)(E % (2 * nsc));
    const CmTag g = cm_tag(E, Eref);
    for (int d = 0; d < C.depth; ++d) {
        unsigned long long *c = reinterpret_cast<unsigned long long *>(cm_cell(C, rule, d, key) + j);
        cm_slot_add(c, cm_load(reinterpret_cast<const uint64_t *>(c)), g, a);
    }
}

__device__ inline uint64_t cm_check_sync(const ParamCtx &C, uint32_t rule, int64_t E, int64_t Eref, int32_t a,
                                         const ValueSrc &vs, int32_t b, int32_t cnt) {
    const int nsc = C.R.n[rule];
    const double I_s = C.R.I_s[rule];
    double remaining = -1.0;
    for (int32_t q = 0; q < cnt; ++q) {
        const uint64_t key = vs.value((int64_t)b + q);
        int64_t est = INT64_MAX;
        for (int d = 0; d < C.CM.depth; ++d) {
            const int64_t x = cm_cell_sum_sync(cm_cell(C.CM, rule, d, key), nsc, E);
            est = x < est ? x : est;
        }
        const double next = remaining_of(value_threshold(C.R, rule, key), I_s, est, a);
        remaining = next;
        if (next < 0.0) return pack_verdict(ST_BLOCKED, 0, 0);
    }
    for (int32_t q = 0; q < cnt; ++q) cm_add_sync(C.CM, rule, vs.value((int64_t)b + q), nsc, E, Eref, a);
    if (cnt > 1) remaining = -1.0;
    return pack_verdict(ST_OK, java_d2i(remaining), 0);
}

// First segment of every rule present in the batch -> heads[] (cursor = that segment), count in *nh.
__global__ __launch_bounds__(256) void k_cm_heads(BatchWork W, uint32_t *__restrict__ heads, uint32_t *__restrict__ nh) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)*W.nseg;
    if (g >= S || (int64_t)*W.nvalid == 0) return;
    if (g > 0 && W.seg_key[g - 1] == W.seg_key[g]) return;
    heads[atomicAdd(nh, 1u)] = (uint32_t)g;
}

// Grid barrier for a cooperative launch (every workgroup resident): arrival count + generation.
__device__ inline void cm_grid_barrier(unsigned int *count, unsigned int *gen, unsigned int nblocks) {
    __threadfence();             // every thread's atomics (cells, next-level minimum) complete before arrival
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned int g = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (atomicAdd(count, 1u) == nblocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) __builtin_amdgcn_s_sleep(4);
        }
    }
    __syncthreads();
}

// Control words (each on its own 64-byte line): ctl[0] head count, ctl[16] barrier arrivals, ctl[32]
// barrier generation; level words lv[0..2] (64-bit) rotate: level k reads lv[k % 3], gathers the next
// level's epoch into lv[(k + 1) % 3] (atomicMin; CM_NO_LEVEL = nothing pending) and clears
// lv[(k + 2) % 3], which nobody touches during level k -- one grid barrier per level.
// cursor[h] = the next segment of head h's rule.
constexpr unsigned long long CM_NO_LEVEL = ~0ull;
__global__ __launch_bounds__(256) void k_prule_cm_sync(ParamCtx C, BatchWork W, const ParamEvent *__restrict__ ev,
                                                       ValueSrc vs, uint64_t *__restrict__ out,
                                                       const uint32_t *__restrict__ heads, uint32_t *__restrict__ ctl,
                                                       uint32_t *__restrict__ cursor, unsigned long long *lv, int band,
                                                       int64_t Eref) {
    const uint32_t H = ctl[0];
    const int64_t S = (int64_t)*W.nseg;
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t h = t0; h < H; h += stride) {           // level 0: the smallest first epoch
        cursor[h] = heads[h];
        atomicMin(&lv[0], (unsigned long long)W.seg_epoch[heads[h]]);
    }
    cm_grid_barrier(&ctl[16], &ctl[32], gridDim.x);
    for (uint32_t k = 0;; ++k) {
        const unsigned long long Eu = __hip_atomic_load(&lv[k % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (Eu == CM_NO_LEVEL) break;                                  // grid-uniform
        const int64_t E = (int64_t)Eu;
        unsigned long long *next = &lv[(k + 1) % 3];
        if (t0 == 0) __hip_atomic_store(&lv[(k + 2) % 3], CM_NO_LEVEL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t h = t0; h < H; h += stride) {
            uint32_t g = cursor[h];
            if (g == 0xFFFFFFFFu) continue;
            const uint32_t rule = W.seg_key[heads[h]];
            while ((int64_t)g < S && W.seg_key[g] == rule && W.seg_epoch[g] < E + band) {
                const int64_t Eg = W.seg_epoch[g];
                const uint32_t end = W.seg_start[g + 1];
                for (uint32_t i = W.seg_start[g]; i < end; ++i) {
                    const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
                    const ParamEvent e = ev[seq];
                    out[seq] = cm_check_sync(C, rule, Eg, Eref, e.acquire, vs, vs.begin(seq), vs.count(seq));
                }
                ++g;
            }
            if ((int64_t)g < S && W.seg_key[g] == rule) {
                cursor[h] = g;
                atomicMin(next, (unsigned long long)W.seg_epoch[g]);
            } else {
                cursor[h] = 0xFFFFFFFFu;
            }
        }
        cm_grid_barrier(&ctl[16], &ctl[32], gridDim.x);
    }
}

// The same level order with one launch per level (the kernel boundary is the barrier): for batches
// spanning up to CM_LEVEL_LAUNCHES epochs.  k_cm_span gives the host the batch's epoch range.
constexpr int64_t CM_LEVEL_LAUNCHES = 4096;
__global__ __launch_bounds__(256) void k_cm_span(BatchWork W, const uint32_t *__restrict__ heads,
                                                 const uint32_t *__restrict__ ctl, uint32_t *__restrict__ cursor,
                                                 unsigned long long *span) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= ctl[0]) return;
    const uint32_t g = heads[h];
    cursor[h] = g;
    const int64_t S = (int64_t)*W.nseg;
    const uint32_t rule = W.seg_key[g];
    uint32_t l = g;
    while ((int64_t)l + 1 < S && W.seg_key[l + 1] == rule) ++l;
    atomicMin(&span[0], (unsigned long long)W.seg_epoch[g]);
    atomicMax(&span[1], (unsigned long long)W.seg_epoch[l]);
}

__global__ __launch_bounds__(256) void k_prule_cm_level(ParamCtx C, BatchWork W, const ParamEvent *__restrict__ ev,
                                                        ValueSrc vs, uint64_t *__restrict__ out,
                                                        const uint32_t *__restrict__ heads,
                                                        const uint32_t *__restrict__ ctl, uint32_t *__restrict__ cursor,
                                                        int64_t E, int band, int64_t Eref) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= ctl[0]) return;
    uint32_t g = cursor[h];
    if (g == 0xFFFFFFFFu) return;
    const int64_t S = (int64_t)*W.nseg;
    const uint32_t rule = W.seg_key[heads[h]];
    if (W.seg_epoch[g] >= E + band) return;
    while ((int64_t)g < S && W.seg_key[g] == rule && W.seg_epoch[g] < E + band) {
        const int64_t Eg = W.seg_epoch[g];
        const uint32_t end = W.seg_start[g + 1];
        for (uint32_t i = W.seg_start[g]; i < end; ++i) {
            const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
            const ParamEvent e = ev[seq];
            out[seq] = cm_check_sync(C, rule, Eg, Eref, e.acquire, vs, vs.begin(seq), vs.count(seq));
        }
        ++g;
    }
    cursor[h] = ((int64_t)g < S && W.seg_key[g] == rule) ? g : 0xFFFFFFFFu;
}

// ParamFlowChecker.passDefaultLocalCheck (PFC:127-202) on one (rule, value) bucket, single-threaded
// (every CAS of the reference succeeds).  Returns 1 pass, 0 block, -1 when the time counter exists
// without a token counter (only after an LRU eviction; the reference spins there).
__device__ inline int bucket_pass(int64_t *st, int64_t token_count, int64_t burst, int64_t dur_ms, int32_t a, int64_t t) {
    if (token_count == 0) return 0;                                          // PFC:144-146
    const int64_t max_count = wrap_add(token_count, burst);                  // PFC:148
    if ((int64_t)a > max_count) return 0;                                    // PFC:149-151
    const int64_t last = st[0];
    if (last == LOCAL_ABSENT) {                                              // PFC:156-161
        st[0] = t;
        if (st[1] == LOCAL_ABSENT) st[1] = wrap_add(max_count, -(int64_t)a);
        return 1;
    }
    const int64_t pass_time = wrap_add(t, -last);                            // PFC:164
    const int64_t rest = st[1];
    if (pass_time > dur_ms) {                                                // PFC:166
        if (rest == LOCAL_ABSENT) {                                          // PFC:167-171
            st[1] = wrap_add(max_count, -(int64_t)a);
            st[0] = t;
            return 1;
        }
        const int64_t to_add = wrap_mul(pass_time, token_count) / dur_ms;    // PFC:174, long division
        const int64_t new_qps = wrap_add(to_add, rest) > max_count ? wrap_add(max_count, -(int64_t)a)
                                                                   : wrap_add(wrap_add(rest, to_add), -(int64_t)a);
        if (new_qps < 0) return 0;                                           // PFC:178-180
        st[1] = new_qps;                                                     // PFC:181-184
        st[0] = t;
        return 1;
    }
    if (rest == LOCAL_ABSENT) return -1;                                     // PFC:188-199
    if (wrap_add(rest, -(int64_t)a) >= 0) {
        st[1] = wrap_add(rest, -(int64_t)a);
        return 1;
    }
    return 0;
}

// ParamFlowChecker.passLocalCheck (PFC:78-103): every element must pass, in order; no rollback.
__device__ inline uint64_t local_check(const ParamCtx &C, uint32_t rule, int64_t t, int32_t a, const ValueSrc &vs,
                                       int32_t b, int32_t cnt) {
    for (int32_t q = 0; q < cnt; ++q) {
        const uint64_t key = vs.value((int64_t)b + q);
        const uint32_t s = C.vslot[b + q];
        const int64_t h = slot_find(C.L.hot_keys, C.L.hot_mask, key);       // PFC:138-142
        const int64_t tok = h >= 0 ? C.L.hot_tokens[h] : C.L.tokens[rule];
        const int r = bucket_pass(C.L.state + 2 * (int64_t)s, tok, C.L.burst[rule], C.L.dur_ms[rule], a, t);
        if (r == 0) return pack_verdict(ST_BLOCKED, 0, 0);
        if (r < 0) return pack_verdict(ST_FAIL, 0, 0);
    }
    return pack_verdict(ST_OK, 0, 0);
}

// THREAD grade (PFC:112-122): each value passes iff ++threadCount <= threshold (hot-item count,
// else (long) rule.count), threadCount = ParameterMetric.getThreadCount (ParameterMetric.java:241-249,
// absent 0).  The check only reads; a passing check then adds one per value, as the entry callback
// does (ParamFlowStatisticEntryCallback -> ParameterMetric.addThreadCount, ParameterMetric.java:184-239;
// AtomicInteger: 32-bit).
__device__ inline uint64_t thread_check(const ParamCtx &C, uint32_t rule, const ValueSrc &vs, int32_t b, int32_t cnt) {
    for (int32_t q = 0; q < cnt; ++q) {
        const uint64_t key = vs.value((int64_t)b + q);
        const int64_t h = slot_find(C.L.hot_keys, C.L.hot_mask, key);
        const int64_t thr = h >= 0 ? C.L.hot_tokens[h] : C.L.tokens[rule];
        const int64_t c = C.L.state[2 * (int64_t)C.vslot[b + q] + 1];
        const int64_t cur = c == LOCAL_ABSENT ? 0 : c;
        if (!(cur + 1 <= thr)) return pack_verdict(ST_BLOCKED, 0, 0);
    }
    for (int32_t q = 0; q < cnt; ++q) {
        int64_t *c = C.L.state + 2 * (int64_t)C.vslot[b + q] + 1;
        *c = *c == LOCAL_ABSENT ? 1 : (int64_t)(int32_t)((uint32_t)*c + 1u);
    }
    return pack_verdict(ST_OK, 0, 0);
}

// Entry.exit -> ParamFlowStatisticExitCallback -> ParameterMetric.decreaseThreadCount
// (ParameterMetric.java:125-181): an absent value gets a 0 entry (putIfAbsent), a present one is
// decremented and removed at <= 0.
__device__ inline void thread_exit(const ParamCtx &C, int32_t b, int32_t cnt) {
    for (int32_t q = 0; q < cnt; ++q) {
        int64_t *c = C.L.state + 2 * (int64_t)C.vslot[b + q] + 1;
        if (*c == LOCAL_ABSENT) { *c = 0; continue; }
        const int32_t v = (int32_t)((uint32_t)*c - 1u);
        *c = v <= 0 ? LOCAL_ABSENT : (int64_t)v;
    }
}

// One lane per rule: walks the rule's sorted (arrival-ordered) events through its segments.
template <int MODE>
__global__ __launch_bounds__(256) void k_prule_process(ParamCtx C, BatchWork W, const ParamEvent *__restrict__ ev,
                                                       ValueSrc vs, uint64_t *__restrict__ out, int64_t n) {
    const int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)*W.nseg;
    if (g0 >= S || (int64_t)*W.nvalid == 0) return;
    const uint32_t rule = W.seg_key[g0];
    if (g0 > 0 && W.seg_key[g0 - 1] == rule) return;    // not the first segment of its rule
    for (int64_t g = g0; g < S; ++g) {
        if (g > g0 && W.seg_key[g] != rule) break;
        const int64_t E = W.seg_epoch[g];
        const uint32_t end = W.seg_start[g + 1];
        for (uint32_t i = W.seg_start[g]; i < end; ++i) {
            const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
            const ParamEvent e = ev[seq];
            const int32_t b = vs.begin(seq);
            const int32_t cnt = vs.count(seq);
            uint64_t v;
            if (MODE == PMODE_LOCAL) {
                const bool thread_grade = C.L.grade && C.L.grade[rule] == 0;
                if (C.L.kinds && C.L.kinds[seq] == 1) {         // exit
                    if (thread_grade) thread_exit(C, b, cnt);
                    v = pack_verdict(ST_OK, 0, 0);
                } else if (thread_grade) {
                    v = thread_check(C, rule, vs, b, cnt);
                } else {
                    v = local_check(C, rule, e.ts, e.acquire, vs, b, cnt);
                }
            }
            else if (MODE == PMODE_CM) v = cm_check(C, rule, E, e.acquire, vs, b, cnt);
            else v = exact_check(C, E, e.acquire, b, cnt);
            out[seq] = v;
        }
    }
}

__global__ void k_fill_i64(int64_t *p, int64_t n, int64_t v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

}  // namespace sentinel
