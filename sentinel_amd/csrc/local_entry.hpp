// local_entry.hpp -- local SphU.entry admission on gfx950: DefaultController over a resource's
// ClusterNode (StatisticNode) with StatisticSlot's pass / block booking.
//
//   FlowRuleChecker.checkFlow -> passLocalCheck -> DefaultController.canPass  (FlowRuleChecker.java:44-86,
//       DefaultController.java:49-76): cur = (int) passQps, block iff (double)(cur + acquire) > count
//       (int add, wraps); every QPS rule of the resource must pass, so the smallest count decides
//   StatisticNode.passQps = rollingCounterInSecond.pass() / intervalInSec    (StatisticNode.java:96-97, 200-202)
//   StatisticSlot.entry: pass -> addPassRequest, block -> increaseBlockQps: both the second window
//       (SAMPLE_COUNT x INTERVAL/SAMPLE_COUNT ms) and the minute window (60 x 1000 ms)
//       (StatisticSlot.java:55-116, StatisticNode.java:246-264)
//
// Per resource state (int64 words): second window {epoch, PASS, BLOCK} x n (n <= 8), then the minute
// window {epoch, PASS, BLOCK} x 60.  Events are grouped by resource (K2 radix sort); segments are
// stretches of one epoch of g = gcd(second bucket, 1000) ms, inside which neither window rolls.  A
// homogeneous segment is monotone in the PASS sum (until cur + acquire could overflow an int), so the
// passing events are the first K (binary search of the exact predicate); other segments run the
// reference state machine event by event.
#pragma once

#include "admission.hpp"

namespace sentinel {

constexpr int LOCAL_NMAX = 8;                       // SampleCountProperty.SAMPLE_COUNT <= 8
constexpr int LOCAL_MIN_SLOTS = 60;                 // rollingCounterInMinute = ArrayMetric(60, 60000)
constexpr int LOCAL_WORDS = 3 * (LOCAL_NMAX + LOCAL_MIN_SLOTS);   // 204 words per resource

struct LocalNodes {
    int64_t *state;            // LOCAL_WORDS per resource
    const double *count;       // min count of the resource's QPS rules; +inf: no rule
    int32_t n;                 // second-window buckets
    int32_t w;                 // second-window bucket length (ms)
    double I_s;                // INTERVAL / 1000.0
};

// LeapArray.currentWindow on a {epoch, PASS, BLOCK} ring: the slot, or -1 (clock went back: detached).
__device__ inline int local_roll(int64_t *ring, int n, int64_t E) {
    const int slot = (int)(E % n);
    int64_t *s = ring + 3 * slot;
    if (s[0] == E) return slot;
    if (s[0] != EPOCH_ABSENT && s[0] > E) return -1;
    s[0] = E;
    s[1] = 0;
    s[2] = 0;
    return slot;
}

__device__ inline int64_t local_sum(const int64_t *ring, int n, int64_t E, int ev) {
    int64_t s = 0;
    for (int j = 0; j < n; ++j) {
        const int64_t e = ring[3 * j];
        if (e != EPOCH_ABSENT && e > E - n) s = wrap_add(s, ring[3 * j + 1 + ev]);
    }
    return s;
}

__device__ inline bool local_admits(double count, double I_s, int64_t pass_sum, int32_t a) {
    const int32_t cur = java_d2i((double)pass_sum / I_s);                              // (int) passQps
    return !((double)(int32_t)((uint32_t)cur + (uint32_t)a) > count);                // DC:50-51
}

// One SphU.entry through the reference state machine (the sequential path).
__device__ inline bool local_seq_entry(const LocalNodes &L, int64_t *st, double count, int64_t t, int32_t a) {
    int64_t *sec = st;
    int64_t *mn = st + 3 * LOCAL_NMAX;
    const int64_t E = t / L.w, E1 = t / 1000;
    local_roll(sec, L.n, E);                                                           // ArrayMetric.pass(): roll + sum
    const bool ok = local_admits(count, L.I_s, local_sum(sec, L.n, E, 0), a);
    const int ev = ok ? 1 : 2;                                                         // PASS : BLOCK word
    const int s1 = local_roll(sec, L.n, E);
    if (s1 >= 0) sec[3 * s1 + ev] = wrap_add(sec[3 * s1 + ev], a);
    const int s2 = local_roll(mn, LOCAL_MIN_SLOTS, E1);
    if (s2 >= 0) mn[3 * s2 + ev] = wrap_add(mn[3 * s2 + ev], a);
    return ok;
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
    int64_t *mn = st + 3 * LOCAL_NMAX;
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
        bool slow = W.seg_het[g] != 0;
        for (int j = 0; j < L.n; ++j) slow |= sec[3 * j] != EPOCH_ABSENT && sec[3 * j] > E;
        for (int j = 0; j < LOCAL_MIN_SLOTS; ++j) slow |= mn[3 * j] != EPOCH_ABSENT && mn[3 * j] > E1;
        int64_t s0 = 0;
        if (!slow) {
            const int s1 = local_roll(sec, L.n, E);
            s0 = local_sum(sec, L.n, E, 0);
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
                sec[3 * s1 + 1] = wrap_add(sec[3 * s1 + 1], pass);
                sec[3 * s1 + 2] = wrap_add(sec[3 * s1 + 2], block);
                const int s2 = local_roll(mn, LOCAL_MIN_SLOTS, E1);
                mn[3 * s2 + 1] = wrap_add(mn[3 * s2 + 1], pass);
                mn[3 * s2 + 2] = wrap_add(mn[3 * s2 + 2], block);
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
            put_verdict(out, seq, local_seq_entry(L, st, count, tt, aa) ? ST_OK : ST_BLOCKED, 0, 0);
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
