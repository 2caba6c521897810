// local_entry.hpp -- local SphU.entry admission on gfx950: DefaultController over a resource's
// ClusterNode (StatisticNode) with StatisticSlot's pass / block booking, prioritized entries
// included.
//
//   FlowRuleChecker.checkFlow -> passLocalCheck -> DefaultController.canPass  (FlowRuleChecker.java:44-86,
//       DefaultController.java:49-76): cur = (int) passQps, block iff (double)(cur + acquire) > count
//       (int add, wraps); every QPS rule of the resource must pass, so the smallest count decides
//   prioritized and over the limit: StatisticNode.tryOccupyNext (StatisticNode.java:288-320) borrows
//       from a future window; a wait below OccupyTimeoutProperty's timeout books addWaitingRequest
//       (the borrow array) + addOccupiedPass (the minute counter) and the entry passes after the
//       wait (PriorityWaitException, DefaultController.java:52-64; StatisticSlot.java:81-95)
//   StatisticNode.passQps = rollingCounterInSecond.pass() / intervalInSec    (StatisticNode.java:96-97, 200-202)
//       over an OccupiableBucketLeapArray: a new or reset second bucket starts with the PASS borrowed
//       into its window (OccupiableBucketLeapArray.java:40-64; FutureBucketLeapArray.java:28-53)
//   StatisticSlot.entry: pass -> addPassRequest, block -> increaseBlockQps: both the second window
//       (SAMPLE_COUNT x INTERVAL/SAMPLE_COUNT ms) and the minute window (60 x 1000 ms)
//       (StatisticSlot.java:55-116, StatisticNode.java:246-264)
//
// Per resource state (int64 words): second window {epoch, PASS, BLOCK} x 8, minute window {epoch,
// PASS, BLOCK, OCCUPIED_PASS} x 60, borrow array {epoch, PASS} x 8.  Events are grouped by resource
// (K2 radix sort); segments are stretches of one epoch of g = gcd(second bucket, 1000) ms, inside
// which neither window rolls.  A homogeneous, non-prioritized segment of a resource with nothing
// borrowed into the current or a future window is monotone in the PASS sum (until cur + acquire
// could overflow an int), so the passing events are the first K (binary search of the exact
// predicate); other segments run the reference state machine event by event.
#pragma once

#include "admission.hpp"

namespace sentinel {

constexpr int LOCAL_NMAX = 8;                       // SampleCountProperty.SAMPLE_COUNT <= 8
constexpr int LOCAL_MIN_SLOTS = 60;                 // rollingCounterInMinute = ArrayMetric(60, 60000)
constexpr int LOCAL_SEC_W = 3, LOCAL_MIN_W = 4, LOCAL_BOR_W = 2;   // words per slot
constexpr int LOCAL_MIN_OFF = LOCAL_SEC_W * LOCAL_NMAX;
constexpr int LOCAL_BOR_OFF = LOCAL_MIN_OFF + LOCAL_MIN_W * LOCAL_MIN_SLOTS;
constexpr int LOCAL_WORDS = LOCAL_BOR_OFF + LOCAL_BOR_W * LOCAL_NMAX;    // 280 words per resource

struct LocalNodes {
    int64_t *state;            // LOCAL_WORDS per resource
    const double *count;       // min count of the resource's QPS rules; +inf: no rule
    int32_t n;                 // second-window buckets (SAMPLE_COUNT)
    int32_t w;                 // second-window bucket length (ms)
    double I_s;                // INTERVAL / 1000.0
    int32_t interval;          // IntervalProperty.INTERVAL (ms)
    int32_t occupy_timeout;    // OccupyTimeoutProperty.occupyTimeout (ms)
};

// LeapArray.currentWindow on a ring of {epoch, counters...} slots (plain reset): the slot, or -1
// (clock went back: a detached bucket whose writes are lost).
template <int STRIDE>
__device__ inline int ring_roll(int64_t *ring, int n, int64_t E) {
    const int slot = (int)(E % n);
    int64_t *s = ring + STRIDE * slot;
    if (s[0] == E) return slot;
    if (s[0] != EPOCH_ABSENT && s[0] > E) return -1;
    s[0] = E;
#pragma unroll
    for (int c = 1; c < STRIDE; ++c) s[c] = 0;
    return slot;
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
__device__ inline int sec_roll(int64_t *st, int n, int64_t E) {
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
    s[1] = fresh ? borrowed : (int64_t)(int32_t)borrowed;
    s[2] = 0;
    return slot;
}

__device__ inline bool local_admits(double count, double I_s, int64_t pass_sum, int32_t a) {
    const int32_t cur = java_d2i((double)pass_sum / I_s);                              // (int) passQps
    return !((double)(int32_t)((uint32_t)cur + (uint32_t)a) > count);                // DC:50-51
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
    int64_t cur_pass = (sec_roll(st, L.n, t / L.w), ring_sum<LOCAL_SEC_W>(st, L.n, t / L.w, 1));
    for (int idx = 0; earliest < t; ++idx) {
        const int64_t wait = (int64_t)idx * wl + wl - t % wl;
        if (wait >= L.occupy_timeout) break;
        int64_t wpass = 0;                                  // ArrayMetric.getWindowPass(earliest)
        if (earliest >= 0) {
            const int64_t e = earliest / L.w;
            const int64_t *s = st + LOCAL_SEC_W * (int)(e % L.n);
            if (s[0] == e) wpass = s[1];
        }
        if ((double)wrap_add(wrap_add(wrap_add(cur_pass, borrow), a), -wpass) <= max_count) return wait;
        earliest += wl;
        cur_pass = wrap_add(cur_pass, -wpass);
    }
    return L.occupy_timeout;
}

// One SphU.entry through the reference state machine (the sequential path): 1 pass / 0 block,
// *wait = waitInMs of an occupied (prioritized) pass.
__device__ inline bool local_seq_entry(const LocalNodes &L, int64_t *st, double count, int64_t t, int32_t a,
                                       bool prio, int32_t *wait) {
    int64_t *mn = st + LOCAL_MIN_OFF;
    const int64_t E = t / L.w, E1 = t / 1000;
    *wait = 0;
    sec_roll(st, L.n, E);                                                              // ArrayMetric.pass(): roll + sum
    if (local_admits(count, L.I_s, ring_sum<LOCAL_SEC_W>(st, L.n, E, 1), a)) {
        const int s1 = sec_roll(st, L.n, E);                                          // SS:62-63 addPassRequest
        if (s1 >= 0) st[LOCAL_SEC_W * s1 + 1] = wrap_add(st[LOCAL_SEC_W * s1 + 1], a);
        const int s2 = ring_roll<LOCAL_MIN_W>(mn, LOCAL_MIN_SLOTS, E1);
        if (s2 >= 0) mn[LOCAL_MIN_W * s2 + 1] = wrap_add(mn[LOCAL_MIN_W * s2 + 1], a);
        return true;
    }
    if (prio) {                                                                        // DC:52-64
        const int64_t w = local_try_occupy(st, L, t, a, count);
        if (w < L.occupy_timeout) {
            const int64_t ft = t + w;                                                  // addWaitingRequest
            const int sb = ring_roll<LOCAL_BOR_W>(st + LOCAL_BOR_OFF, L.n, ft / L.w);
            if (sb >= 0) st[LOCAL_BOR_OFF + LOCAL_BOR_W * sb + 1] = wrap_add(st[LOCAL_BOR_OFF + LOCAL_BOR_W * sb + 1], a);
            const int s2 = ring_roll<LOCAL_MIN_W>(mn, LOCAL_MIN_SLOTS, E1);           // addOccupiedPass (minute)
            if (s2 >= 0) {
                mn[LOCAL_MIN_W * s2 + 3] = wrap_add(mn[LOCAL_MIN_W * s2 + 3], a);
                mn[LOCAL_MIN_W * s2 + 1] = wrap_add(mn[LOCAL_MIN_W * s2 + 1], a);
            }
            *wait = (int32_t)w;
            return true;
        }
    }
    const int s1 = sec_roll(st, L.n, E);                                              // SS:96-104 increaseBlockQps
    if (s1 >= 0) st[LOCAL_SEC_W * s1 + 2] = wrap_add(st[LOCAL_SEC_W * s1 + 2], a);
    const int s2 = ring_roll<LOCAL_MIN_W>(mn, LOCAL_MIN_SLOTS, E1);
    if (s2 >= 0) mn[LOCAL_MIN_W * s2 + 2] = wrap_add(mn[LOCAL_MIN_W * s2 + 2], a);
    return false;
}

// Validation and sort keys: an unknown resource answers NO_RULE_EXISTS, t < 0 FAIL.
__global__ __launch_bounds__(SORT_THREADS) void k_lentry_prep(int64_t n, const Event *__restrict__ ev, int32_t nres,
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
        uint32_t k = finvalid;
        if (e.idx < 0 || e.idx >= nres) put_verdict(out, (uint32_t)i, ST_NO_RULE_EXISTS, 0, 0);
        else if (e.ts < 0) put_verdict(out, (uint32_t)i, ST_FAIL, 0, 0);
        else k = (uint32_t)e.idx;
        fkey[i] = k;
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
    const double count = L.count[key];
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
        bool slow = W.seg_het[g] != 0 || borrow_pending(st, L.n, E);   // prioritized events / borrowed PASS
        for (int j = 0; j < L.n; ++j) slow |= sec[LOCAL_SEC_W * j] != EPOCH_ABSENT && sec[LOCAL_SEC_W * j] > E;
        for (int j = 0; j < LOCAL_MIN_SLOTS; ++j) slow |= mn[LOCAL_MIN_W * j] != EPOCH_ABSENT && mn[LOCAL_MIN_W * j] > E1;
        int64_t s0 = 0;
        if (!slow) {
            const int s1 = sec_roll(st, L.n, E);
            s0 = ring_sum<LOCAL_SEC_W>(sec, L.n, E, 1);
            // the predicate is monotone while cur + a stays an int
            slow = (double)s0 + (double)len * (double)a + (double)a > 2147483000.0 * L.I_s;
            if (!slow) {
                uint32_t lo = 0, hi = len;
                while (lo < hi) {
                    const uint32_t mid = lo + (hi - lo) / 2;
                    if (local_admits(count, L.I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) lo = mid + 1;
                    else hi = mid;
                }
                const uint32_t K = lo;
                const int64_t pass = wrap_mul((int64_t)K, a), block = wrap_mul((int64_t)(len - K), a);
                sec[LOCAL_SEC_W * s1 + 1] = wrap_add(sec[LOCAL_SEC_W * s1 + 1], pass);
                sec[LOCAL_SEC_W * s1 + 2] = wrap_add(sec[LOCAL_SEC_W * s1 + 2], block);
                const int s2 = ring_roll<LOCAL_MIN_W>(mn, LOCAL_MIN_SLOTS, E1);
                mn[LOCAL_MIN_W * s2 + 1] = wrap_add(mn[LOCAL_MIN_W * s2 + 1], pass);
                mn[LOCAL_MIN_W * s2 + 2] = wrap_add(mn[LOCAL_MIN_W * s2 + 2], block);
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
            int32_t wait;
            const bool ok = local_seq_entry(L, st, count, tt, aa, (fl & 1u) != 0, &wait);
            put_verdict(out, seq, ok ? ST_OK : ST_BLOCKED, 0, ok ? wait : 0);
        }
        W.seg_done[g] = 1;
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
