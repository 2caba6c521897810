// local_entry.hpp -- local SphU.entry admission on gfx950: DefaultController over a resource's
// ClusterNode (StatisticNode) with StatisticSlot's booking, prioritized entries, THREAD grade rules
// and Entry.exit included.
//
//   FlowRuleChecker.checkFlow -> passLocalCheck -> DefaultController.canPass  (FlowRuleChecker.java:44-86,
//       DefaultController.java:49-76): cur = (int) passQps (QPS grade) or (int) curThreadNum (THREAD
//       grade, StatisticNode.java:241-243), block iff (double)(cur + acquire) > count (int add, wraps);
//       every rule of one grade must pass, so the smallest count of that grade decides; the rules are
//       checked in order, the first failure throws
//   prioritized and over a QPS limit: StatisticNode.tryOccupyNext (StatisticNode.java:288-320) borrows
//       from a future window; a wait below OccupyTimeoutProperty's timeout books addWaitingRequest
//       (the borrow array) + addOccupiedPass (the minute counter) and the entry passes after the
//       wait (PriorityWaitException, DefaultController.java:52-64; StatisticSlot.java:81-95)
//   StatisticNode.passQps = rollingCounterInSecond.pass() / intervalInSec    (StatisticNode.java:96-97, 200-202)
//       over an OccupiableBucketLeapArray: a new or reset second bucket starts with the PASS borrowed
//       into its window (OccupiableBucketLeapArray.java:40-64; FutureBucketLeapArray.java:28-53)
//   StatisticSlot.entry: pass -> increaseThreadNum + addPassRequest, occupied pass ->
//       increaseThreadNum, block -> increaseBlockQps: both the second window (SAMPLE_COUNT x
//       INTERVAL/SAMPLE_COUNT ms) and the minute window (60 x 1000 ms) (StatisticSlot.java:55-123,
//       StatisticNode.java:246-280)
//   StatisticSlot.exit of a passed entry at its completion time: addRtAndSuccess (SUCCESS and RT into
//       both windows, MetricBucket.addRT keeps the bucket's minRt), decreaseThreadNum, and
//       increaseExceptionQps when a business exception was traced (StatisticSlot.java:126-164,
//       MetricBucket.java:132-139)
//
// Per resource state (int64 words): second window {epoch, PASS, BLOCK, EXCEPTION, SUCCESS, RT,
// minRt} x 8, minute window {epoch, PASS, BLOCK, OCCUPIED_PASS, EXCEPTION, SUCCESS, RT, minRt} x
// 60, borrow array {epoch, PASS} x 8, curThreadNum.  Events are grouped by resource (K2 radix sort);
// segments are stretches of one epoch of g = gcd(second bucket, 1000) ms, inside which neither
// window rolls.  A homogeneous segment of plain entries (no prioritized entry, no exit) of a
// resource with nothing borrowed into the current or a future window is monotone in the number of
// passes (the PASS sum and the thread count both grow with it, until cur + acquire could overflow an
// int), so the passing events are the first K (binary search of the exact predicate); other
// segments run the reference state machine event by event.
#pragma once

#include "admission.hpp"

namespace sentinel {

constexpr int LOCAL_NMAX = 8;                       // SampleCountProperty.SAMPLE_COUNT <= 8
constexpr int LOCAL_MIN_SLOTS = 60;                 // rollingCounterInMinute = ArrayMetric(60, 60000)
constexpr int LOCAL_SEC_W = 7, LOCAL_MIN_W = 8, LOCAL_BOR_W = 2;   // words per slot
// second-window / minute-window columns after the epoch word
constexpr int SC_PASS = 1, SC_BLOCK = 2, SC_EXC = 3, SC_SUCC = 4, SC_RT = 5, SC_MINRT = 6;
constexpr int MC_PASS = 1, MC_BLOCK = 2, MC_OCC = 3, MC_EXC = 4, MC_SUCC = 5, MC_RT = 6, MC_MINRT = 7;
constexpr int LOCAL_MIN_OFF = LOCAL_SEC_W * LOCAL_NMAX;
constexpr int LOCAL_BOR_OFF = LOCAL_MIN_OFF + LOCAL_MIN_W * LOCAL_MIN_SLOTS;
constexpr int LOCAL_THR_OFF = LOCAL_BOR_OFF + LOCAL_BOR_W * LOCAL_NMAX;
constexpr int LOCAL_WORDS = LOCAL_THR_OFF + 8;      // 560 words per resource (curThreadNum + pad)

// rule flags of a resource (sentinel_local_resource_ex_t.flags)
constexpr uint8_t LR_QPS = 1, LR_THREAD = 2, LR_THREAD_FIRST = 4;
// event flags of a local batch (sentinel_submit_local_batch)
constexpr uint8_t LF_PRIO = 1, LF_EXIT = 2, LF_ERROR = 4;

struct LocalNodes {
    int64_t *state;            // LOCAL_WORDS per resource
    const double *count;       // min count of the resource's QPS rules
    int32_t n;                 // second-window buckets (SAMPLE_COUNT)
    int32_t w;                 // second-window bucket length (ms)
    double I_s;                // INTERVAL / 1000.0
    int32_t interval;          // IntervalProperty.INTERVAL (ms)
    int32_t occupy_timeout;    // OccupyTimeoutProperty.occupyTimeout (ms)
    const double *thread_count;  // min count of the resource's THREAD rules
    const uint8_t *rflags;     // LR_* per resource
    int64_t max_rt;            // SentinelConfig.statisticMaxRt: a fresh bucket's minRt (MetricBucket.java:58-60)
    const uint8_t *ofl;        // the batch's event flags (LF_*); null: plain entries
    const int64_t *rt;         // the batch's exit response times; null: none
};

// LeapArray.currentWindow on a ring of {epoch, counters...} slots (plain reset; minRt reset to
// statisticMaxRt when the slot has one): the slot, or -1 (clock went back: a detached bucket whose
// writes are lost).
template <int STRIDE>
__device__ inline int ring_roll(int64_t *ring, int n, int64_t E, int minrt_col = -1, int64_t max_rt = 0) {
    const int slot = (int)(E % n);
    int64_t *s = ring + STRIDE * slot;
    if (s[0] == E) return slot;
    if (s[0] != EPOCH_ABSENT && s[0] > E) return -1;
    s[0] = E;
#pragma unroll
    for (int c = 1; c < STRIDE; ++c) s[c] = 0;
    if (minrt_col > 0) s[minrt_col] = max_rt;
    return slot;
}

__device__ inline int min_roll(int64_t *st, const LocalNodes &L, int64_t E1) {
    return ring_roll<LOCAL_MIN_W>(st + LOCAL_MIN_OFF, LOCAL_MIN_SLOTS, E1, MC_MINRT, L.max_rt);
}

template <int STRIDE>
__device__ inline int64_t ring_sum(const int64_t *ring, int n, int64_t E, int col) {
    int64_t s = 0;
    for (int j = 0; j < n; ++j) {
        const int64_t e = ring[STRIDE * j];
        if (e != EPOCH_ABSENT && e > E - n) s = wrap_add(s, ring[STRIDE * j + col]);
    }
    return s;
}

// OccupiableBucketLeapArray.currentWindow: a new bucket copies the borrow bucket of its window
// (newEmptyBucket -> MetricBucket.reset(borrow)), a reset one gets addPass((int) borrow.pass())
// (OccupiableBucketLeapArray.java:40-64); the borrow bucket is the one whose window holds the time
// (LeapArray.getWindowValue, WindowWrap.isTimeInWindow), i.e. the borrow slot of the same epoch.
// Either way the bucket's minRt restarts at statisticMaxRt.
__device__ inline int sec_roll(int64_t *st, int n, int64_t E, int64_t max_rt) {
    int64_t *sec = st;
    const int64_t *bor = st + LOCAL_BOR_OFF;
    const int slot = (int)(E % n);
    int64_t *s = sec + LOCAL_SEC_W * slot;
    if (s[0] == E) return slot;
    if (s[0] != EPOCH_ABSENT && s[0] > E) return -1;
    const bool fresh = s[0] == EPOCH_ABSENT;
    const int64_t *b = bor + LOCAL_BOR_W * slot;
    const int64_t borrowed = b[0] == E ? b[1] : 0;
    s[0] = E;
    s[SC_PASS] = fresh ? borrowed : (int64_t)(int32_t)borrowed;
#pragma unroll
    for (int c = SC_BLOCK; c < SC_MINRT; ++c) s[c] = 0;
    s[SC_MINRT] = max_rt;
    return slot;
}

__device__ inline bool local_admits(double count, double I_s, int64_t pass_sum, int32_t a) {
    const int32_t cur = java_d2i((double)pass_sum / I_s);                              // (int) passQps
    return !((double)(int32_t)((uint32_t)cur + (uint32_t)a) > count);                // DC:50-51
}

// THREAD grade: cur = (int) curThreadNum.sum() (a long -> int cast: the low 32 bits)
__device__ inline bool thread_admits(double count, int64_t threads, int32_t a) {
    const int32_t cur = (int32_t)threads;
    return !((double)(int32_t)((uint32_t)cur + (uint32_t)a) > count);
}

// Anything borrowed into window E or later: the closed form (which rolls without borrowing) is
// only exact without.
__device__ inline bool borrow_pending(const int64_t *st, int n, int64_t E) {
    const int64_t *bor = st + LOCAL_BOR_OFF;
    bool p = false;
    for (int j = 0; j < n; ++j) p |= bor[LOCAL_BOR_W * j] != EPOCH_ABSENT && bor[LOCAL_BOR_W * j] >= E;
    return p;
}

// ArrayMetric.waiting -> OccupiableBucketLeapArray.currentWaiting: roll the borrow array at t,
// sum the PASS of its future buckets (FutureBucketLeapArray: deprecated iff t >= windowStart).
__device__ inline int64_t local_waiting(int64_t *st, const LocalNodes &L, int64_t t) {
    int64_t *bor = st + LOCAL_BOR_OFF;
    ring_roll<LOCAL_BOR_W>(bor, L.n, t / L.w);
    int64_t s = 0;
    for (int j = 0; j < L.n; ++j) {
        const int64_t e = bor[LOCAL_BOR_W * j];
        if (e != EPOCH_ABSENT && e * L.w > t) s = wrap_add(s, bor[LOCAL_BOR_W * j + 1]);
    }
    return s;
}

// StatisticNode.tryOccupyNext (StatisticNode.java:288-320), Java operation order.
__device__ inline int64_t local_try_occupy(int64_t *st, const LocalNodes &L, int64_t t, int32_t a, double threshold) {
    const double max_count = threshold * (double)L.interval / 1000;
    const int64_t borrow = local_waiting(st, L, t);
    if ((double)borrow >= max_count) return L.occupy_timeout;
    const int32_t wl = L.interval / L.n;
    int64_t earliest = t - t % wl + wl - L.interval;
    int64_t cur_pass = (sec_roll(st, L.n, t / L.w, L.max_rt), ring_sum<LOCAL_SEC_W>(st, L.n, t / L.w, SC_PASS));
    for (int idx = 0; earliest < t; ++idx) {
        const int64_t wait = (int64_t)idx * wl + wl - t % wl;
        if (wait >= L.occupy_timeout) break;
        int64_t wpass = 0;                                  // ArrayMetric.getWindowPass(earliest)
        if (earliest >= 0) {
            const int64_t e = earliest / L.w;
            const int64_t *s = st + LOCAL_SEC_W * (int)(e % L.n);
            if (s[0] == e) wpass = s[SC_PASS];
        }
        if ((double)wrap_add(wrap_add(wrap_add(cur_pass, borrow), a), -wpass) <= max_count) return wait;
        earliest += wl;
        cur_pass = wrap_add(cur_pass, -wpass);
    }
    return L.occupy_timeout;
}

// add x to column `col` of the second and minute buckets of t
__device__ inline void local_book(const LocalNodes &L, int64_t *st, int64_t t, int sc, int mc, int64_t x) {
    const int s1 = sec_roll(st, L.n, t / L.w, L.max_rt);
    if (s1 >= 0) st[LOCAL_SEC_W * s1 + sc] = wrap_add(st[LOCAL_SEC_W * s1 + sc], x);
    int64_t *mn = st + LOCAL_MIN_OFF;
    const int s2 = min_roll(st, L, t / 1000);
    if (s2 >= 0) mn[LOCAL_MIN_W * s2 + mc] = wrap_add(mn[LOCAL_MIN_W * s2 + mc], x);
}

// One SphU.entry through the reference state machine (the sequential path): 1 pass / 0 block,
// *wait = waitInMs of an occupied (prioritized) pass.
__device__ inline bool local_seq_entry(const LocalNodes &L, int64_t *st, uint32_t res, int64_t t, int32_t a,
                                       bool prio, int32_t *wait) {
    int64_t *mn = st + LOCAL_MIN_OFF;
    const int64_t E = t / L.w, E1 = t / 1000;
    const uint8_t rf = L.rflags[res];
    *wait = 0;
    bool blocked = false;
    for (int k = 0; k < 2 && !blocked; ++k) {                                         // FRC:44-60, rules in order
        const bool thread_rule = ((rf & LR_THREAD_FIRST) != 0) == (k == 0);
        if (thread_rule) {
            if ((rf & LR_THREAD) && !thread_admits(L.thread_count[res], st[LOCAL_THR_OFF], a)) blocked = true;
            continue;
        }
        if (!(rf & LR_QPS)) continue;
        sec_roll(st, L.n, E, L.max_rt);                                                // ArrayMetric.pass(): roll + sum
        if (local_admits(L.count[res], L.I_s, ring_sum<LOCAL_SEC_W>(st, L.n, E, SC_PASS), a)) continue;
        if (prio) {                                                                    // DC:52-64
            const int64_t w = local_try_occupy(st, L, t, a, L.count[res]);
            if (w < L.occupy_timeout) {
                const int64_t ft = t + w;                                              // addWaitingRequest
                const int sb = ring_roll<LOCAL_BOR_W>(st + LOCAL_BOR_OFF, L.n, ft / L.w);
                if (sb >= 0) st[LOCAL_BOR_OFF + LOCAL_BOR_W * sb + 1] = wrap_add(st[LOCAL_BOR_OFF + LOCAL_BOR_W * sb + 1], a);
                const int s2 = min_roll(st, L, E1);                                    // addOccupiedPass (minute)
                if (s2 >= 0) {
                    mn[LOCAL_MIN_W * s2 + MC_OCC] = wrap_add(mn[LOCAL_MIN_W * s2 + MC_OCC], a);
                    mn[LOCAL_MIN_W * s2 + MC_PASS] = wrap_add(mn[LOCAL_MIN_W * s2 + MC_PASS], a);
                }
                st[LOCAL_THR_OFF] = wrap_add(st[LOCAL_THR_OFF], 1);                     // SS:81-82
                *wait = (int32_t)w;
                return true;
            }
        }
        blocked = true;
    }
    if (blocked) {
        local_book(L, st, t, SC_BLOCK, MC_BLOCK, a);                                   // SS:96-104 increaseBlockQps
        return false;
    }
    st[LOCAL_THR_OFF] = wrap_add(st[LOCAL_THR_OFF], 1);                                 // SS:62-63
    local_book(L, st, t, SC_PASS, MC_PASS, a);
    return true;
}

// MetricBucket.addRT: RT += rt, minRt = min(minRt, rt) (MetricBucket.java:132-139)
__device__ inline void local_add_rt(const LocalNodes &L, int64_t *st, int64_t t, int64_t rt) {
    const int s1 = sec_roll(st, L.n, t / L.w, L.max_rt);
    if (s1 >= 0) {
        int64_t *b = st + LOCAL_SEC_W * s1;
        b[SC_RT] = wrap_add(b[SC_RT], rt);
        if (rt < b[SC_MINRT]) b[SC_MINRT] = rt;
    }
    const int s2 = min_roll(st, L, t / 1000);
    if (s2 >= 0) {
        int64_t *b = st + LOCAL_MIN_OFF + LOCAL_MIN_W * s2;
        b[MC_RT] = wrap_add(b[MC_RT], rt);
        if (rt < b[MC_MINRT]) b[MC_MINRT] = rt;
    }
}

// StatisticSlot.exit of a passed entry (SS:126-164): recordCompleteFor -> addRtAndSuccess(rt, count)
// (SN:252-258, second then minute window), decreaseThreadNum, increaseExceptionQps(count) on error.
__device__ inline void local_seq_exit(const LocalNodes &L, int64_t *st, int64_t t, int32_t count, int64_t rt,
                                      bool error) {
    const int s1 = sec_roll(st, L.n, t / L.w, L.max_rt);                               // second: SUCCESS, RT
    if (s1 >= 0) {
        int64_t *b = st + LOCAL_SEC_W * s1;
        b[SC_SUCC] = wrap_add(b[SC_SUCC], count);
        b[SC_RT] = wrap_add(b[SC_RT], rt);
        if (rt < b[SC_MINRT]) b[SC_MINRT] = rt;
    }
    const int s2 = min_roll(st, L, t / 1000);                                          // minute: SUCCESS, RT
    if (s2 >= 0) {
        int64_t *b = st + LOCAL_MIN_OFF + LOCAL_MIN_W * s2;
        b[MC_SUCC] = wrap_add(b[MC_SUCC], count);
        b[MC_RT] = wrap_add(b[MC_RT], rt);
        if (rt < b[MC_MINRT]) b[MC_MINRT] = rt;
    }
    st[LOCAL_THR_OFF] = wrap_add(st[LOCAL_THR_OFF], -1);                                // SN:278-280
    if (error) local_book(L, st, t, SC_EXC, MC_EXC, count);                            // SN:267-270
}

// Validation and sort keys: an unknown resource answers NO_RULE_EXISTS, t < 0 FAIL.  With event
// flags, `slow` gets bit 0 for a prioritized entry or an exit (either makes its segment take the
// sequential path: the segment builder marks bit-0 events of KIND_CLUSTER keys).
__global__ __launch_bounds__(SORT_THREADS) void k_lentry_prep(int64_t n, const Event *__restrict__ ev, int32_t nres,
                                                              uint64_t *__restrict__ out, uint32_t *__restrict__ fkey,
                                                              uint32_t finvalid, uint32_t *__restrict__ fhist,
                                                              int64_t nblocks, const uint8_t *__restrict__ ofl,
                                                              uint8_t *__restrict__ slow) {
    __shared__ uint32_t hf[MAX_PASSES][RADIX];
    for (int d = threadIdx.x; d < MAX_PASSES * RADIX; d += SORT_THREADS) (&hf[0][0])[d] = 0;
    __syncthreads();
    const int64_t tile0 = (int64_t)blockIdx.x * SORT_TILE;
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        if (i >= n) break;
        const Event e = ev[i];
        uint32_t k = finvalid;
        if (e.idx < 0 || e.idx >= nres) put_verdict(out, (uint32_t)i, ST_NO_RULE_EXISTS, 0, 0);
        else if (e.ts < 0) put_verdict(out, (uint32_t)i, ST_FAIL, 0, 0);
        else k = (uint32_t)e.idx;
        fkey[i] = k;
        if (slow) slow[i] = (ofl[i] & (LF_PRIO | LF_EXIT)) ? 1 : 0;
        tile_hist_accumulate(hf, k, 1);
    }
    __syncthreads();
    tile_hist_store(hf, fhist, 1, nblocks);
}

// One lane per resource: walks its segments; fast segments leave {S0, K} in the segment records
// for k_lentry_verdict, sequential ones write their verdicts and are marked done.
__global__ __launch_bounds__(256) void k_lentry_process(LocalNodes L, BatchWork W, EventSrc src, uint64_t *out) {
    const int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)*W.nseg;
    if (g0 >= S || (int64_t)*W.nvalid == 0) return;
    const uint32_t key = W.seg_key[g0];
    if (g0 > 0 && W.seg_key[g0 - 1] == key) return;
    int64_t *st = L.state + (int64_t)key * LOCAL_WORDS;
    int64_t *sec = st;
    int64_t *mn = st + LOCAL_MIN_OFF;
    const double count = L.count[key], tcount = L.thread_count[key];
    const uint8_t rf = L.rflags[key];
    const int64_t T0 = src.t0();
    for (int64_t g = g0; g < S; ++g) {
        if (g > g0 && W.seg_key[g] != key) break;
        const uint32_t q0 = W.seg_start[g], q1 = W.seg_start[g + 1];
        const uint32_t len = q1 - q0;
        int64_t t;
        int32_t a;
        bool prio;
        src.unpack(W.sval[q0], T0, t, a, prio);
        const int64_t E = t / L.w, E1 = t / 1000;
        // prioritized entries / exits / borrowed PASS / a window newer than E: sequential
        bool slow = W.seg_het[g] != 0 || borrow_pending(st, L.n, E);
        for (int j = 0; j < L.n; ++j) slow |= sec[LOCAL_SEC_W * j] != EPOCH_ABSENT && sec[LOCAL_SEC_W * j] > E;
        for (int j = 0; j < LOCAL_MIN_SLOTS; ++j) slow |= mn[LOCAL_MIN_W * j] != EPOCH_ABSENT && mn[LOCAL_MIN_W * j] > E1;
        const int64_t T = st[LOCAL_THR_OFF];
        // the predicates are monotone while cur + a stays an int
        slow |= (rf & LR_THREAD) && (T < 0 || T + (int64_t)len + a > 2147483000ll);
        int64_t s0 = 0;
        if (!slow) {
            const int s1 = sec_roll(st, L.n, E, L.max_rt);
            s0 = ring_sum<LOCAL_SEC_W>(sec, L.n, E, SC_PASS);
            slow = (rf & LR_QPS) && (double)s0 + (double)len * (double)a + (double)a > 2147483000.0 * L.I_s;
            if (!slow) {
                uint32_t lo = 0, hi = len;          // K = first k with a failing rule after k passes
                while (lo < hi) {
                    const uint32_t mid = lo + (hi - lo) / 2;
                    const bool ok = (!(rf & LR_QPS) || local_admits(count, L.I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) &&
                                    (!(rf & LR_THREAD) || thread_admits(tcount, T + mid, a));
                    if (ok) lo = mid + 1;
                    else hi = mid;
                }
                const uint32_t K = lo;
                const int64_t pass = wrap_mul((int64_t)K, a), block = wrap_mul((int64_t)(len - K), a);
                sec[LOCAL_SEC_W * s1 + SC_PASS] = wrap_add(sec[LOCAL_SEC_W * s1 + SC_PASS], pass);
                sec[LOCAL_SEC_W * s1 + SC_BLOCK] = wrap_add(sec[LOCAL_SEC_W * s1 + SC_BLOCK], block);
                const int s2 = min_roll(st, L, E1);
                mn[LOCAL_MIN_W * s2 + MC_PASS] = wrap_add(mn[LOCAL_MIN_W * s2 + MC_PASS], pass);
                mn[LOCAL_MIN_W * s2 + MC_BLOCK] = wrap_add(mn[LOCAL_MIN_W * s2 + MC_BLOCK], block);
                st[LOCAL_THR_OFF] = wrap_add(T, (int64_t)K);
                W.seg_s0[g] = s0;
                W.seg_k[g] = K;
                W.seg_done[g] = 0;
                continue;
            }
        }
        for (uint32_t i = q0; i < q1; ++i) {
            const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
            int64_t tt;
            int32_t aa;
            uint8_t fl;
            src.load(seq, tt, aa, fl);
            const uint8_t of = L.ofl ? L.ofl[seq] : 0;
            if (of & LF_EXIT) {
                local_seq_exit(L, st, tt, aa, L.rt ? L.rt[seq] : 0, (of & LF_ERROR) != 0);
                put_verdict(out, seq, ST_OK, 0, 0);
                continue;
            }
            int32_t wait;
            const bool ok = local_seq_entry(L, st, key, tt, aa, (of & LF_PRIO) != 0, &wait);
            put_verdict(out, seq, ok ? ST_OK : ST_BLOCKED, 0, ok ? wait : 0);
        }
        W.seg_done[g] = 1;
    }
}

// ---------------------------------------------------------------------------------------------
// Local rule graph: FlowRuleChecker with every limitApp / strategy (FlowRuleChecker.java:44-145)
// over the nodes the slot chain builds -- a ClusterNode per resource (created by the resource's
// first entry, ClusterBuilderSlot.java:74-92), an origin StatisticNode per (resource, origin)
// (ClusterNode.getOrCreateOriginNode, CBS:97-100) and a DefaultNode per (context, resource) whose
// booking also reaches the ClusterNode (DefaultNode.java:110-143).  A RELATE rule of resource A reads
// the ClusterNode of its refResource B, which B's entries write: A and B are one "component" (host
// union-find over the RELATE edges), and one lane walks a component's events in arrival order
// through the reference state machine.  Every node is a LOCAL_WORDS StatisticNode record.
struct LocalRule {
    double count;
    int32_t grade;        // 1 QPS, 0 THREAD
    int32_t strategy;     // 0 DIRECT, 1 RELATE, 2 CHAIN, other: no node
    int32_t limit_app;    // 0 "default", 1 "other", >= 2 an origin id
    int32_t ref;          // RELATE: resource index, CHAIN: context id, -1 blank
};
struct LocalCtx {
    int32_t origin;       // -1: "" (no origin node)
    int32_t origin_node;
    int32_t context;
    int32_t default_node;
};
struct LocalGraph {
    int64_t *on_state;            // origin nodes
    int64_t *dn_state;            // DefaultNodes
    uint8_t *created;             // ClusterNode exists (ClusterBuilderSlot.clusterNodeMap)
    const int32_t *roff;          // rules of resource r: [roff[r], roff[r + 1]) (comparator-sorted)
    const LocalRule *rules;
    const LocalCtx *ctx;          // per event
    const uint32_t *comp;         // component of each resource
    int32_t n_res, n_on, n_dn;
};

// FRC:87-103 selectReferenceNode
__device__ inline int64_t *lg_ref_node(const LocalNodes &L, const LocalGraph &G, const LocalRule &r, const LocalCtx &c) {
    if (r.ref < 0) return nullptr;
    if (r.strategy == 1) return r.ref < G.n_res && G.created[r.ref] ? L.state + (int64_t)r.ref * LOCAL_WORDS : nullptr;
    if (r.strategy == 2) return r.ref == c.context ? G.dn_state + (int64_t)c.default_node * LOCAL_WORDS : nullptr;
    return nullptr;
}

// FRC:110-145 selectNodeByRequesterAndStrategy (filterOrigin: the origin is not "default" / "other")
__device__ inline int64_t *lg_select(const LocalNodes &L, const LocalGraph &G, uint32_t res, const LocalRule &r,
                                     const LocalCtx &c) {
    int64_t *onode = c.origin >= 0 ? G.on_state + (int64_t)c.origin_node * LOCAL_WORDS : nullptr;
    if (r.limit_app == c.origin && c.origin >= 2) return r.strategy == 0 ? onode : lg_ref_node(L, G, r, c);
    if (r.limit_app == 0) return r.strategy == 0 ? L.state + (int64_t)res * LOCAL_WORDS : lg_ref_node(L, G, r, c);
    if (r.limit_app == 1 && c.origin >= 0) {                  // FlowRuleManager.isOtherOrigin (:113-129)
        bool other = true;
        for (int32_t j = G.roff[res]; j < G.roff[res + 1]; ++j) other &= G.rules[j].limit_app != c.origin;
        if (other) return r.strategy == 0 ? onode : lg_ref_node(L, G, r, c);
    }
    return nullptr;
}

// One SphU.entry(res) in context c: node creation, every rule in order (DefaultController.canPass on
// the selected node, DC:49-69), StatisticSlot.entry's booking (SS:55-116).
__device__ inline bool lg_entry(const LocalNodes &L, const LocalGraph &G, uint32_t res, int64_t t, int32_t a, bool prio,
                                const LocalCtx &c, int32_t *wait) {
    *wait = 0;
    G.created[res] = 1;
    int64_t *cn = L.state + (int64_t)res * LOCAL_WORDS;
    int64_t *dn = G.dn_state + (int64_t)c.default_node * LOCAL_WORDS;
    int64_t *on = c.origin >= 0 ? G.on_state + (int64_t)c.origin_node * LOCAL_WORDS : nullptr;
    bool blocked = false, occupied = false;
    for (int32_t j = G.roff[res]; j < G.roff[res + 1] && !blocked && !occupied; ++j) {
        const LocalRule r = G.rules[j];
        int64_t *nd = lg_select(L, G, res, r, c);
        if (!nd) continue;                                   // FRC:78-81: no node -> pass
        int32_t cur;
        if (r.grade == 0) {
            cur = (int32_t)nd[LOCAL_THR_OFF];                // (int) curThreadNum
        } else {
            const int64_t E = t / L.w;
            sec_roll(nd, L.n, E, L.max_rt);                  // (int) passQps
            cur = java_d2i((double)ring_sum<LOCAL_SEC_W>(nd, L.n, E, SC_PASS) / L.I_s);
        }
        if (!((double)(int32_t)((uint32_t)cur + (uint32_t)a) > r.count)) continue;
        if (prio && r.grade == 1) {                          // DC:52-64
            const int64_t w = local_try_occupy(nd, L, t, a, r.count);
            if (w < L.occupy_timeout) {
                const int64_t ft = t + w;                    // addWaitingRequest
                const int sb = ring_roll<LOCAL_BOR_W>(nd + LOCAL_BOR_OFF, L.n, ft / L.w);
                if (sb >= 0) nd[LOCAL_BOR_OFF + LOCAL_BOR_W * sb + 1] = wrap_add(nd[LOCAL_BOR_OFF + LOCAL_BOR_W * sb + 1], a);
                int64_t *mn = nd + LOCAL_MIN_OFF;            // addOccupiedPass (minute)
                const int s2 = min_roll(nd, L, t / 1000);
                if (s2 >= 0) {
                    mn[LOCAL_MIN_W * s2 + MC_OCC] = wrap_add(mn[LOCAL_MIN_W * s2 + MC_OCC], a);
                    mn[LOCAL_MIN_W * s2 + MC_PASS] = wrap_add(mn[LOCAL_MIN_W * s2 + MC_PASS], a);
                }
                *wait = (int32_t)w;
                occupied = true;                             // PriorityWaitException
                continue;
            }
        }
        blocked = true;
    }
    if (blocked) {                                           // SS:96-104
        local_book(L, dn, t, SC_BLOCK, MC_BLOCK, a);
        local_book(L, cn, t, SC_BLOCK, MC_BLOCK, a);
        if (on) local_book(L, on, t, SC_BLOCK, MC_BLOCK, a);
        return false;
    }
    dn[LOCAL_THR_OFF] = wrap_add(dn[LOCAL_THR_OFF], 1);      // SS:62-69 / 81-86
    cn[LOCAL_THR_OFF] = wrap_add(cn[LOCAL_THR_OFF], 1);
    if (!occupied) {
        local_book(L, dn, t, SC_PASS, MC_PASS, a);
        local_book(L, cn, t, SC_PASS, MC_PASS, a);
    }
    if (on) {
        on[LOCAL_THR_OFF] = wrap_add(on[LOCAL_THR_OFF], 1);
        if (!occupied) local_book(L, on, t, SC_PASS, MC_PASS, a);
    }
    return true;
}

// Validation (unknown resource / node index -> NO_RULE_EXISTS, t < 0 -> FAIL) and the sort key: the
// resource's component.
__global__ __launch_bounds__(SORT_THREADS) void k_lgraph_prep(int64_t n, const Event *__restrict__ ev, LocalGraph G,
                                                              uint64_t *__restrict__ out, uint32_t *__restrict__ fkey,
                                                              uint32_t finvalid, uint32_t *__restrict__ fhist,
                                                              int64_t nblocks) {
    __shared__ uint32_t hf[MAX_PASSES][RADIX];
    for (int d = threadIdx.x; d < MAX_PASSES * RADIX; d += SORT_THREADS) (&hf[0][0])[d] = 0;
    __syncthreads();
    const int64_t tile0 = (int64_t)blockIdx.x * SORT_TILE;
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        if (i >= n) break;
        const Event e = ev[i];
        const LocalCtx c = G.ctx[i];
        uint32_t k = finvalid;
        if (e.idx < 0 || e.idx >= G.n_res || c.default_node < 0 || c.default_node >= G.n_dn ||
            (c.origin >= 0 && (c.origin_node < 0 || c.origin_node >= G.n_on)))
            put_verdict(out, (uint32_t)i, ST_NO_RULE_EXISTS, 0, 0);
        else if (e.ts < 0) put_verdict(out, (uint32_t)i, ST_FAIL, 0, 0);
        else k = G.comp[e.idx];
        fkey[i] = k;
        tile_hist_accumulate(hf, k, 1);
    }
    __syncthreads();
    tile_hist_store(hf, fhist, 1, nblocks);
}

// One lane per component: every event of the component in arrival order (entries and exits).
__global__ __launch_bounds__(256) void k_lgraph_process(LocalNodes L, LocalGraph G, BatchWork W, EventSrc src,
                                                        uint64_t *out) {
    const int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)*W.nseg;
    if (g0 >= S || (int64_t)*W.nvalid == 0) return;
    const uint32_t key = W.seg_key[g0];
    if (g0 > 0 && W.seg_key[g0 - 1] == key) return;
    int64_t g1 = g0 + 1;
    while (g1 < S && W.seg_key[g1] == key) ++g1;
    for (uint32_t i = W.seg_start[g0]; i < W.seg_start[g1]; ++i) {
        const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
        const Event e = src.ev[seq];
        const LocalCtx c = G.ctx[seq];
        const uint8_t of = L.ofl ? L.ofl[seq] : 0;
        if (of & LF_EXIT) {                                  // SS:126-164: DefaultNode (+ ClusterNode), origin node
            const int64_t rt = L.rt ? L.rt[seq] : 0;
            const bool err = (of & LF_ERROR) != 0;
            local_seq_exit(L, G.dn_state + (int64_t)c.default_node * LOCAL_WORDS, e.ts, e.acquire, rt, err);
            local_seq_exit(L, L.state + (int64_t)e.idx * LOCAL_WORDS, e.ts, e.acquire, rt, err);
            if (c.origin >= 0) local_seq_exit(L, G.on_state + (int64_t)c.origin_node * LOCAL_WORDS, e.ts, e.acquire, rt, err);
            put_verdict(out, seq, ST_OK, 0, 0);
            continue;
        }
        int32_t wait;
        const bool ok = lg_entry(L, G, (uint32_t)e.idx, e.ts, e.acquire, (of & LF_PRIO) != 0, c, &wait);
        put_verdict(out, seq, ok ? ST_OK : ST_BLOCKED, 0, ok ? wait : 0);
    }
}

__global__ __launch_bounds__(256) void k_lentry_verdict(BatchWork W, uint64_t *out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || i >= (int64_t)*W.nvalid) return;
    const uint32_t g = W.segid[i] - 1;
    if (W.seg_done[g]) return;
    const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
    put_verdict(out, seq, (uint32_t)i - W.seg_start[g] < W.seg_k[g] ? ST_OK : ST_BLOCKED, 0, 0);
}

}  // namespace sentinel
