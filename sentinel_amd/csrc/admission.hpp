// admission.hpp -- K1 window roll + K3 segmented greedy admission + verdict scatter (gfx950).
//
// After K2 has grouped a batch by key (flow, namespace limiter or param slot) in arrival order,
// each key's events split into segments of one window epoch.  Inside a segment every event sees
// the same rolled window, and the reference check (ClusterFlowChecker.java:67-71,
// SimpleClusterFlowChecker.java:41-45, RequestLimiter.java:72-74, ClusterParamFlowChecker.java:62-66)
// is a monotone predicate of the running PASS sum.  With a homogeneous acquire count a the k-th
// event passes iff k < K, K = first p with !cond(S0 + p*a): found by binary search over exact
// double evaluations in Java operation order, so verdicts and counters are bit-exact.  Segments
// with heterogeneous acquire, prioritized events or a clock that moved backwards take the
// sequential per-event path (the same state machine as the reference, one event at a time).
//
// Window semantics (LeapArray.java:149-248, 316-318, 375-390, 399-409) restated on epochs
// e = floor(start / w): after currentWindow(t) a slot is in values(t) iff e > E - n where
// E = epoch(t) (future slots included), the rolled slot is E mod n, and getValidHead(t) reads
// slot (E + 1) mod n under the same validity test.  The proof is in DESIGN.md ("Window algebra").
#pragma once

#include "common.hpp"

namespace sentinel {

// Per-key tables (device pointers).  State pool per key at state_off[k]:
//   epochs[n] then counters[ncounters][n]  (int64 each).
struct KeyTable {
    const int64_t *state_off;  // null => key * state_stride
    int64_t state_stride;
    const int32_t *n;
    const int32_t *w;
    const double *rcp_w;
    const double *I_s;       // LeapArray.intervalInSecond = intervalInMs / 1000.0
    const double *thr;       // CLUSTER/SIMPLE: global threshold*exceedCount; LIMITER: qpsAllowed; PARAM: per key
    const uint8_t *kind;
    int64_t *state;
    int64_t *occ;            // CLUSTER only: [2*k] occupy PASS, [2*k+1] occupy PASS_REQUEST (CMLA:129)
    uint8_t *has_occ;        // CMLA:130
    int32_t ncounters;       // 7 (flows) or 1 (limiter / param)
    double max_occupy_ratio; // ServerFlowConfig.maxOccupyRatio
};

// Batch working set, all device pointers, sized for n events.
struct BatchWork {
    uint32_t *skey, *sseq;       // sorted keys / arrival positions
    int64_t *s_epoch;            // epoch of each sorted event
    int32_t *s_acq;              // acquire of each sorted event
    uint8_t *s_fl;               // flags of each sorted event
    uint32_t *segid;             // inclusive scan of segment heads (1-based segment id)
    uint32_t *seg_start;         // S+1 entries
    uint8_t *seg_het;            // heterogeneous / prioritized segment
    uint8_t *seg_done;           // decided by the sequential path
    int64_t *seg_s0;             // PASS sum at segment start (after the roll)
    uint32_t *seg_k;             // number of passing events
    uint32_t *nvalid;            // device counter: events with a valid key
    uint32_t *nseg;              // device: number of segments
};

// Outputs of one pipeline run.
struct Verdicts {
    int8_t *status;
    int32_t *remaining;
    int32_t *wait_ms;            // may be null
    // LIMITER mode: events that fail get status TOO_MANY_REQUEST and flow_key[seq] = flow_key_invalid
    uint32_t *flow_key;
    uint32_t flow_key_invalid;
};

__device__ inline int64_t *cnt_ptr(const KeyTable &T, int64_t off, int n, int ev) {
    return T.state + off + (int64_t)(1 + ev) * n;
}

// LeapArray.currentWindow(t) on epochs: returns the slot, or -1 for the detached wrap (clock
// went backwards: LeapArray.java:241-246, writes to it are lost).
__device__ inline int roll(const KeyTable &T, int key, int64_t off, int n, int64_t E) {
    int64_t *ep = T.state + off;
    const int slot = (int)(E % n);
    const int64_t cur = ep[slot];
    if (cur == E) return slot;                                  // LA:195-209 same window
    if (cur != EPOCH_ABSENT && cur > E) return -1;              // LA:241-246 detached
    const bool reset = cur != EPOCH_ABSENT;                     // LA:210-240 vs LA:172-194
    ep[slot] = E;
    for (int c = 0; c < T.ncounters; ++c) cnt_ptr(T, off, n, c)[slot] = 0;
    if (reset && T.kind[key] == KIND_CLUSTER && T.has_occ[key]) {
        // ClusterMetricLeapArray.transferOccupyToBucket (ClusterMetricLeapArray.java:154-169)
        int64_t *o = T.occ + 2 * (int64_t)key;
        cnt_ptr(T, off, n, EV_OCCUPIED_PASS)[slot] = wrap_add(cnt_ptr(T, off, n, EV_OCCUPIED_PASS)[slot], o[0]);
        cnt_ptr(T, off, n, EV_PASS)[slot] = wrap_add(cnt_ptr(T, off, n, EV_PASS)[slot], o[0]);
        o[0] = 0;
        cnt_ptr(T, off, n, EV_PASS_REQUEST)[slot] = wrap_add(cnt_ptr(T, off, n, EV_PASS_REQUEST)[slot], o[1]);
        o[1] = 0;
        T.has_occ[key] = 0;
    }
    return slot;
}

__device__ inline int64_t window_sum(const KeyTable &T, int64_t off, int n, int64_t E, int ev) {
    const int64_t *ep = T.state + off;
    const int64_t *c = cnt_ptr(T, off, n, ev);
    int64_t s = 0;
    for (int j = 0; j < n; ++j) {
        const int64_t e = ep[j];
        if (e != EPOCH_ABSENT && e > E - n) s = wrap_add(s, c[j]);
    }
    return s;
}

__device__ inline void add_counter(const KeyTable &T, int key, int64_t off, int n, int64_t E, int ev, int64_t x) {
    const int slot = roll(T, key, off, n, E);
    if (slot >= 0) {
        int64_t *c = cnt_ptr(T, off, n, ev);
        c[slot] = wrap_add(c[slot], x);
    }
}

// The monotone admission predicate of each checker, evaluated in Java operation order.
__device__ inline bool admits(uint8_t kind, double thr, double I_s, int64_t x, int32_t a) {
    const double avg = (double)x / I_s;
    switch (kind) {
        case KIND_LIMITER: return avg + 1.0 <= thr;                      // RequestLimiter.java:72-74
        case KIND_PARAM: return !(((thr - avg) - (double)a) < 0.0);       // ClusterParamFlowChecker.java:64-66
        default: return ((thr - avg) - (double)a) >= 0.0;                 // ClusterFlowChecker.java:69-71
    }
}

__device__ inline double remaining_of(double thr, double I_s, int64_t x, int32_t a) {
    return (thr - (double)x / I_s) - (double)a;
}

__device__ inline void reject_limited(const Verdicts &V, uint32_t seq) {
    V.status[seq] = ST_TOO_MANY_REQUEST;
    V.remaining[seq] = 0;
    if (V.wait_ms) V.wait_ms[seq] = 0;
    V.flow_key[seq] = V.flow_key_invalid;
}

// One event through the reference state machine (the sequential path).
__device__ inline void seq_event(const KeyTable &T, int key, int64_t off, int n, int64_t E, int32_t a,
                                 uint8_t flags, uint32_t seq, const Verdicts &V) {
    const uint8_t kind = T.kind[key];
    const double thr = T.thr[key];
    const double I_s = T.I_s[key];
    if (kind == KIND_LIMITER) {
        roll(T, key, off, n, E);
        const int64_t sum = window_sum(T, off, n, E, 0);
        if (admits(kind, thr, I_s, sum, 1)) add_counter(T, key, off, n, E, 0, 1);
        else reject_limited(V, seq);
        return;
    }
    if (kind == KIND_PARAM) {
        roll(T, key, off, n, E);
        const int64_t sum = window_sum(T, off, n, E, 0);
        const double next = remaining_of(thr, I_s, sum, a);
        if (!(next < 0.0)) {
            add_counter(T, key, off, n, E, 0, a);
            V.status[seq] = ST_OK; V.remaining[seq] = java_d2i(next);
        } else {
            V.status[seq] = ST_BLOCKED; V.remaining[seq] = 0;
        }
        if (V.wait_ms) V.wait_ms[seq] = 0;
        return;
    }
    const bool prio = kind == KIND_CLUSTER && (flags & 1u);
    roll(T, key, off, n, E);
    const int64_t sum = window_sum(T, off, n, E, EV_PASS);
    const double next = remaining_of(thr, I_s, sum, a);
    if (next >= 0.0) {
        add_counter(T, key, off, n, E, EV_PASS, a);
        add_counter(T, key, off, n, E, EV_PASS_REQUEST, 1);
        if (prio) add_counter(T, key, off, n, E, EV_OCCUPIED_PASS, a);
        V.status[seq] = ST_OK; V.remaining[seq] = java_d2i(next);
        if (V.wait_ms) V.wait_ms[seq] = 0;
        return;
    }
    if (prio) {
        // ClusterFlowChecker.java:84-98 + ClusterMetric.tryOccupyNext (ClusterMetric.java:79-98)
        roll(T, key, off, n, E);
        const double occupy_avg = (double)window_sum(T, off, n, E, EV_WAITING) / I_s;
        if (occupy_avg <= T.max_occupy_ratio * thr) {
            roll(T, key, off, n, E);
            const double latest = (double)window_sum(T, off, n, E, EV_PASS) / I_s;
            const int64_t *ep = T.state + off;
            const int hs = (int)((E + 1) % n);
            const int64_t he = ep[hs];
            const int64_t head = (he != EPOCH_ABSENT && he > E - n) ? cnt_ptr(T, off, n, EV_PASS)[hs] : 0;
            int64_t *o = T.occ + 2 * (int64_t)key;
            const int64_t inner = wrap_add((int64_t)a, o[0]);
            const double lhs = (latest + (double)inner) - (double)head;
            if (lhs <= thr) {
                o[0] = wrap_add(o[0], a);
                o[1] = wrap_add(o[1], 1);
                T.has_occ[key] = 1;
                add_counter(T, key, off, n, E, EV_WAITING, a);
                const int wait = 1000 / n;
                if (wait > 0) {
                    V.status[seq] = ST_SHOULD_WAIT; V.remaining[seq] = 0;
                    if (V.wait_ms) V.wait_ms[seq] = wait;
                    return;
                }
            }
        }
    }
    add_counter(T, key, off, n, E, EV_BLOCK, a);
    add_counter(T, key, off, n, E, EV_BLOCK_REQUEST, 1);
    if (prio) add_counter(T, key, off, n, E, EV_OCCUPIED_BLOCK, a);
    V.status[seq] = ST_BLOCKED; V.remaining[seq] = 0;
    if (V.wait_ms) V.wait_ms[seq] = 0;
}

// ------------------------------------------------------------------------- kernels

// Gathers each sorted event's epoch / acquire / flags into sorted order.
__global__ __launch_bounds__(256) void k_gather_sorted(KeyTable T, BatchWork W, const int64_t *__restrict__ ts,
                                                       const int32_t *__restrict__ acquire,
                                                       const uint8_t *__restrict__ flags, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || i >= (int64_t)*W.nvalid) return;
    const uint32_t k = W.skey[i];
    const uint32_t s = W.sseq[i];
    W.s_epoch[i] = epoch_of(ts[s], T.w[k], T.rcp_w[k]);
    W.s_acq[i] = acquire ? acquire[s] : 1;
    W.s_fl[i] = flags ? flags[s] : 0;
}

// Segment heads: a new (key, epoch) run starts.  head array is scanned in place into segid.
__global__ __launch_bounds__(256) void k_heads(BatchWork W, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t nv = (int64_t)*W.nvalid;
    uint32_t h = 0;
    if (i < nv) h = (i == 0) || W.skey[i] != W.skey[i - 1] || W.s_epoch[i] != W.s_epoch[i - 1];
    W.segid[i] = h;
}

__global__ __launch_bounds__(256) void k_seg_start(BatchWork W, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nv = (int64_t)*W.nvalid;
    if (i >= n || i >= nv) return;
    const uint32_t g = W.segid[i];
    if (i == 0 || W.segid[i - 1] != g) {
        W.seg_start[g - 1] = (uint32_t)i;
        W.seg_het[g - 1] = 0;
        W.seg_done[g - 1] = 0;
    }
    if (i == nv - 1) {
        W.seg_start[g] = (uint32_t)nv;
        *W.nseg = g;
    }
}

__global__ __launch_bounds__(256) void k_seg_het(KeyTable T, BatchWork W, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nv = (int64_t)*W.nvalid;
    if (i >= n || i >= nv) return;
    const uint32_t g = W.segid[i] - 1;
    const uint32_t first = W.seg_start[g];
    const bool prio = (W.s_fl[i] & 1u) && T.kind[W.skey[i]] == KIND_CLUSTER;
    if (W.s_acq[i] != W.s_acq[first] || prio) W.seg_het[g] = 1;
}

// One thread per key run: walks its epoch segments in order (epochs of a key depend on the
// previous epochs' passes).  Fast segments: O(n + log L); others: sequential.
__global__ __launch_bounds__(256) void k_process(KeyTable T, BatchWork W, Verdicts V, int64_t n) {
    const int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)*W.nseg;
    if (g0 >= S || (int64_t)*W.nvalid == 0) return;
    const uint32_t key = W.skey[W.seg_start[g0]];
    if (g0 > 0 && W.skey[W.seg_start[g0 - 1]] == key) return;    // not the first segment of its key
    const int64_t off = T.state_off ? T.state_off[key] : (int64_t)key * T.state_stride;
    const int nsc = T.n[key];
    const uint8_t kind = T.kind[key];
    const double thr = T.thr[key];
    const double I_s = T.I_s[key];
    const int ev_pass = (kind == KIND_LIMITER || kind == KIND_PARAM) ? 0 : EV_PASS;
    for (int64_t g = g0; g < S; ++g) {
        const uint32_t st = W.seg_start[g];
        if (W.skey[st] != key) break;
        const uint32_t len = W.seg_start[g + 1] - st;
        const int64_t E = W.s_epoch[st];
        // fast path eligibility: homogeneous, and time did not move backwards for this key
        bool fast = !W.seg_het[g];
        if (fast) {
            const int64_t *ep = T.state + off;
            for (int j = 0; j < nsc; ++j)
                if (ep[j] != EPOCH_ABSENT && ep[j] > E) { fast = false; break; }
        }
        if (!fast) {
            for (uint32_t i = st; i < st + len; ++i)
                seq_event(T, key, off, nsc, E, W.s_acq[i], W.s_fl[i], W.sseq[i], V);
            W.seg_done[g] = 1;
            continue;
        }
        const int32_t a = kind == KIND_LIMITER ? 1 : W.s_acq[st];
        const int slot = roll(T, key, off, nsc, E);
        const int64_t s0 = window_sum(T, off, nsc, E, ev_pass);
        uint32_t lo = 0, hi = len;                      // K = first p with !admits(S0 + p*a)
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (admits(kind, thr, I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) lo = mid + 1;
            else hi = mid;
        }
        const uint32_t K = lo;
        const int64_t nb = (int64_t)(len - K);
        if (kind == KIND_LIMITER) {
            int64_t *c = cnt_ptr(T, off, nsc, 0);
            c[slot] = wrap_add(c[slot], (int64_t)K);
        } else if (kind == KIND_PARAM) {
            int64_t *c = cnt_ptr(T, off, nsc, 0);
            c[slot] = wrap_add(c[slot], wrap_mul((int64_t)K, a));
        } else {
            int64_t *c;
            c = cnt_ptr(T, off, nsc, EV_PASS);          c[slot] = wrap_add(c[slot], wrap_mul((int64_t)K, a));
            c = cnt_ptr(T, off, nsc, EV_PASS_REQUEST);  c[slot] = wrap_add(c[slot], (int64_t)K);
            c = cnt_ptr(T, off, nsc, EV_BLOCK);         c[slot] = wrap_add(c[slot], wrap_mul(nb, a));
            c = cnt_ptr(T, off, nsc, EV_BLOCK_REQUEST); c[slot] = wrap_add(c[slot], nb);
        }
        W.seg_s0[g] = s0;
        W.seg_k[g] = K;
    }
}

// Per sorted event: rank inside its segment decides; scatter the verdict to its arrival slot.
__global__ __launch_bounds__(256) void k_verdict(KeyTable T, BatchWork W, Verdicts V, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nv = (int64_t)*W.nvalid;
    if (i >= n || i >= nv) return;
    const uint32_t g = W.segid[i] - 1;
    if (W.seg_done[g]) return;
    const uint32_t rank = (uint32_t)i - W.seg_start[g];
    const uint32_t K = W.seg_k[g];
    const uint32_t seq = W.sseq[i];
    const uint32_t key = W.skey[i];
    const uint8_t kind = T.kind[key];
    if (kind == KIND_LIMITER) {
        if (rank >= K) reject_limited(V, seq);
        return;
    }
    if (rank < K) {
        const int32_t a = W.s_acq[i];
        const int64_t x = wrap_add(W.seg_s0[g], wrap_mul((int64_t)rank, a));
        V.status[seq] = ST_OK;
        V.remaining[seq] = java_d2i(remaining_of(T.thr[key], T.I_s[key], x, a));
    } else {
        V.status[seq] = ST_BLOCKED;
        V.remaining[seq] = 0;
    }
    if (V.wait_ms) V.wait_ms[seq] = 0;
}

}  // namespace sentinel
