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
//
// State layout per key (int64 words, 64-byte aligned records):
//   header  : epoch[n], pass[n]            (padded to a multiple of 8 words)
//   rest    : n slots x 8 words            (only for 7-counter flow keys)
//             {BLOCK, PASS_REQUEST, BLOCK_REQUEST, OCCUPIED_PASS, OCCUPIED_BLOCK, WAITING, -, -}
// The fast path reads only the header (16n bytes) and writes one header word pair + one rest line.
#pragma once

#include "common.hpp"

namespace sentinel {

// AoS event / verdict records of the C ABI (include/sentinel_amd.h).
struct Event {
    int32_t idx;
    int32_t acquire;
    int64_t ts;
};
struct ParamEvent {
    int32_t idx;
    int32_t acquire;
    int64_t ts;
    uint64_t key;
};

__host__ __device__ inline int64_t header_words(int n) { return ((2 * (int64_t)n) + 7) & ~(int64_t)7; }
__host__ __device__ inline int64_t flow_record_words(int n) { return header_words(n) + 8 * (int64_t)n; }

// Per-key tables (device pointers).
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

// Where the events of a pipeline run come from (one of the two is non-null).
struct EventSrc {
    const Event *ev;
    const ParamEvent *pev;
    const uint8_t *flags;    // may be null
    bool unit_acquire;       // limiter: acquire == 1 for every request

    __device__ inline void load(uint32_t s, int64_t &ts, int32_t &a, uint8_t &fl) const {
        if (ev) { const Event e = ev[s]; ts = e.ts; a = e.acquire; }
        else { const ParamEvent e = pev[s]; ts = e.ts; a = e.acquire; }
        if (unit_acquire) a = 1;
        fl = flags ? flags[s] : 0;
    }
};

// Batch working set, all device pointers, sized for n events.
struct BatchWork {
    uint32_t *skey, *sseq;       // sorted keys / arrival positions
    uint32_t *segid;             // head flags, scanned in place (1-based segment id)
    uint8_t *bad;                // element breaks segment homogeneity (acquire differs / prioritized)
    int64_t *h_epoch;            // epoch at head positions (sparse)
    int32_t *h_acq;              // acquire at head positions (sparse)
    uint32_t *seg_start;         // S+1 entries
    uint32_t *seg_key;
    int64_t *seg_epoch;
    int32_t *seg_acq;
    uint8_t *seg_het;            // heterogeneous / prioritized segment
    uint8_t *seg_done;           // decided by the sequential path
    int64_t *seg_s0;             // PASS sum at segment start (after the roll)
    uint32_t *seg_k;             // number of passing events
    uint32_t *nvalid;            // device: events with a valid key
    uint32_t *nseg;              // device: number of segments
};

// Packed TokenResult: {int32 remaining; int16 status; uint16 waitInMs} as one 8-byte store.
__device__ inline void put_verdict(uint64_t *out, uint32_t seq, int status, int32_t remaining, int wait) {
    out[seq] = (uint64_t)(uint32_t)remaining | ((uint64_t)(uint16_t)(int16_t)status << 32) |
               ((uint64_t)(uint16_t)wait << 48);
}

// Outputs of one pipeline run.
struct Verdicts {
    uint64_t *out;
    // LIMITER mode: events that fail get status TOO_MANY_REQUEST and flow_key[seq] = flow_key_invalid
    uint32_t *flow_key;
    uint32_t flow_key_invalid;
};

struct KeyState {
    int64_t *base;
    int n;
    bool seven;   // 7-counter flow layout
    __device__ inline int64_t *epoch() const { return base; }
    __device__ inline int64_t *pass() const { return base + n; }
    __device__ inline int64_t &cnt(int ev, int slot) const {
        if (ev == EV_PASS || !seven) return base[n + slot];
        return base[header_words(n) + 8 * (int64_t)slot + (ev - 1)];
    }
};

__device__ inline KeyState key_state(const KeyTable &T, uint32_t key) {
    KeyState k;
    const int64_t off = T.state_off ? T.state_off[key] : (int64_t)key * T.state_stride;
    k.base = T.state + off;
    k.n = T.n[key];
    k.seven = T.ncounters == NEV;
    return k;
}

// LeapArray.currentWindow(t) on epochs: returns the slot, or -1 for the detached wrap (clock
// went backwards: LeapArray.java:241-246, writes to it are lost).
__device__ inline int roll(const KeyTable &T, uint32_t key, const KeyState &S, int64_t E) {
    int64_t *ep = S.epoch();
    const int slot = (int)(E % S.n);
    const int64_t cur = ep[slot];
    if (cur == E) return slot;                                  // LA:195-209 same window
    if (cur != EPOCH_ABSENT && cur > E) return -1;              // LA:241-246 detached
    const bool reset = cur != EPOCH_ABSENT;                     // LA:210-240 vs LA:172-194
    ep[slot] = E;
    S.cnt(EV_PASS, slot) = 0;
    if (S.seven) {
        int64_t *r = &S.cnt(EV_BLOCK, slot);
#pragma unroll
        for (int c = 0; c < 6; ++c) r[c] = 0;
        if (reset && T.kind[key] == KIND_CLUSTER && T.has_occ[key]) {
            // ClusterMetricLeapArray.transferOccupyToBucket (ClusterMetricLeapArray.java:154-169)
            int64_t *o = T.occ + 2 * (int64_t)key;
            S.cnt(EV_OCCUPIED_PASS, slot) = wrap_add(S.cnt(EV_OCCUPIED_PASS, slot), o[0]);
            S.cnt(EV_PASS, slot) = wrap_add(S.cnt(EV_PASS, slot), o[0]);
            o[0] = 0;
            S.cnt(EV_PASS_REQUEST, slot) = wrap_add(S.cnt(EV_PASS_REQUEST, slot), o[1]);
            o[1] = 0;
            T.has_occ[key] = 0;
        }
    }
    return slot;
}

__device__ inline int64_t window_sum(const KeyState &S, int64_t E, int ev) {
    const int64_t *ep = S.epoch();
    int64_t s = 0;
    for (int j = 0; j < S.n; ++j) {
        const int64_t e = ep[j];
        if (e != EPOCH_ABSENT && e > E - S.n) s = wrap_add(s, S.cnt(ev, j));
    }
    return s;
}

__device__ inline void add_counter(const KeyTable &T, uint32_t key, const KeyState &S, int64_t E, int ev, int64_t x) {
    const int slot = roll(T, key, S, E);
    if (slot >= 0) S.cnt(ev, slot) = wrap_add(S.cnt(ev, slot), x);
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
    put_verdict(V.out, seq, ST_TOO_MANY_REQUEST, 0, 0);
    V.flow_key[seq] = V.flow_key_invalid;
}

// One event through the reference state machine (the sequential path).
__device__ inline void seq_event(const KeyTable &T, uint32_t key, const KeyState &S, int64_t E, int32_t a,
                                 uint8_t flags, uint32_t seq, const Verdicts &V) {
    const uint8_t kind = T.kind[key];
    const double thr = T.thr[key];
    const double I_s = T.I_s[key];
    if (kind == KIND_LIMITER) {
        roll(T, key, S, E);
        const int64_t sum = window_sum(S, E, EV_PASS);
        if (admits(kind, thr, I_s, sum, 1)) add_counter(T, key, S, E, EV_PASS, 1);
        else reject_limited(V, seq);
        return;
    }
    if (kind == KIND_PARAM) {
        roll(T, key, S, E);
        const int64_t sum = window_sum(S, E, EV_PASS);
        const double next = remaining_of(thr, I_s, sum, a);
        if (!(next < 0.0)) {
            add_counter(T, key, S, E, EV_PASS, a);
            put_verdict(V.out, seq, ST_OK, java_d2i(next), 0);
        } else {
            put_verdict(V.out, seq, ST_BLOCKED, 0, 0);
        }
        return;
    }
    const bool prio = kind == KIND_CLUSTER && (flags & 1u);
    roll(T, key, S, E);
    const int64_t sum = window_sum(S, E, EV_PASS);
    const double next = remaining_of(thr, I_s, sum, a);
    if (next >= 0.0) {
        add_counter(T, key, S, E, EV_PASS, a);
        add_counter(T, key, S, E, EV_PASS_REQUEST, 1);
        if (prio) add_counter(T, key, S, E, EV_OCCUPIED_PASS, a);
        put_verdict(V.out, seq, ST_OK, java_d2i(next), 0);
        return;
    }
    if (prio) {
        // ClusterFlowChecker.java:84-98 + ClusterMetric.tryOccupyNext (ClusterMetric.java:79-98)
        roll(T, key, S, E);
        const double occupy_avg = (double)window_sum(S, E, EV_WAITING) / I_s;
        if (occupy_avg <= T.max_occupy_ratio * thr) {
            roll(T, key, S, E);
            const double latest = (double)window_sum(S, E, EV_PASS) / I_s;
            const int hs = (int)((E + 1) % S.n);
            const int64_t he = S.epoch()[hs];
            const int64_t head = (he != EPOCH_ABSENT && he > E - S.n) ? S.cnt(EV_PASS, hs) : 0;
            int64_t *o = T.occ + 2 * (int64_t)key;
            const int64_t inner = wrap_add((int64_t)a, o[0]);
            const double lhs = (latest + (double)inner) - (double)head;
            if (lhs <= thr) {
                o[0] = wrap_add(o[0], a);
                o[1] = wrap_add(o[1], 1);
                T.has_occ[key] = 1;
                add_counter(T, key, S, E, EV_WAITING, a);
                const int wait = 1000 / S.n;
                if (wait > 0) {
                    put_verdict(V.out, seq, ST_SHOULD_WAIT, 0, wait);
                    return;
                }
            }
        }
    }
    add_counter(T, key, S, E, EV_BLOCK, a);
    add_counter(T, key, S, E, EV_BLOCK_REQUEST, 1);
    if (prio) add_counter(T, key, S, E, EV_OCCUPIED_BLOCK, a);
    put_verdict(V.out, seq, ST_BLOCKED, 0, 0);
}

// ------------------------------------------------------------------------- kernels

// Segment heads.  Each sorted event's epoch is computed once; neighbours are exchanged in LDS.
// head = new (key, epoch) run; bad = same run but different acquire, or prioritized (CLUSTER).
// Also records nvalid and the head's epoch / acquire (sparse) for k_seg_mark.
__global__ __launch_bounds__(256) void k_seg_heads(KeyTable T, BatchWork W, EventSrc src, int64_t n,
                                                   uint32_t invalid) {
    __shared__ uint32_t s_key[256];
    __shared__ int64_t s_ep[256];
    __shared__ int32_t s_acq[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t key = invalid;
    int64_t E = 0;
    int32_t a = 0;
    uint8_t fl = 0;
    if (i < n) {
        key = W.skey[i];
        if (key != invalid) {
            int64_t t;
            src.load(W.sseq[i], t, a, fl);
            E = epoch_of(t, T.w[key], T.rcp_w[key]);
        }
    }
    s_key[threadIdx.x] = key;
    s_ep[threadIdx.x] = E;
    s_acq[threadIdx.x] = a;
    __syncthreads();
    if (i >= n) return;
    if (key == invalid) {
        W.segid[i] = 0;
        if (i == 0) *W.nvalid = 0;
        return;
    }
    uint32_t pk;
    int64_t pE;
    int32_t pa;
    if (i == 0) { pk = invalid; pE = 0; pa = 0; }
    else if (threadIdx.x > 0) { pk = s_key[threadIdx.x - 1]; pE = s_ep[threadIdx.x - 1]; pa = s_acq[threadIdx.x - 1]; }
    else {
        pk = W.skey[i - 1];
        int64_t t;
        uint8_t f2;
        src.load(W.sseq[i - 1], t, pa, f2);
        pE = epoch_of(t, T.w[pk], T.rcp_w[pk]);
    }
    const bool head = pk != key || pE != E;
    W.segid[i] = head ? 1u : 0u;
    const bool prio = (fl & 1u) && T.kind[key] == KIND_CLUSTER;
    W.bad[i] = (!head && pa != a) || prio;
    if (head) { W.h_epoch[i] = E; W.h_acq[i] = a; }
    if (i == n - 1 || W.skey[i + 1] == invalid) *W.nvalid = (uint32_t)(i + 1);
}

// After the inclusive scan of heads: per-segment records.  seg_het must be zeroed beforehand.
__global__ __launch_bounds__(256) void k_seg_mark(BatchWork W, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t nv = (int64_t)*W.nvalid;
    if (i >= nv) return;
    const uint32_t g = W.segid[i];
    if (i == 0 || W.segid[i - 1] != g) {
        W.seg_start[g - 1] = (uint32_t)i;
        W.seg_key[g - 1] = W.skey[i];
        W.seg_epoch[g - 1] = W.h_epoch[i];
        W.seg_acq[g - 1] = W.h_acq[i];
    }
    if (W.bad[i]) W.seg_het[g - 1] = 1;
    if (i == nv - 1) {
        W.seg_start[g] = (uint32_t)nv;
        *W.nseg = g;
    }
}

// One thread per key run: walks its epoch segments in order (epochs of a key depend on the
// previous epochs' passes).  Fast segments: O(n + log L); others: sequential.
__global__ __launch_bounds__(256) void k_process(KeyTable T, BatchWork W, EventSrc src, Verdicts V, int64_t n) {
    const int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)*W.nseg;
    if (g0 >= S || (int64_t)*W.nvalid == 0) return;
    const uint32_t key = W.seg_key[g0];
    if (g0 > 0 && W.seg_key[g0 - 1] == key) return;    // not the first segment of its key
    const KeyState ks = key_state(T, key);
    const uint8_t kind = T.kind[key];
    const double thr = T.thr[key];
    const double I_s = T.I_s[key];
    for (int64_t g = g0; g < S; ++g) {
        if (g > g0 && W.seg_key[g] != key) break;
        const uint32_t st = W.seg_start[g];
        const uint32_t len = W.seg_start[g + 1] - st;
        const int64_t E = W.seg_epoch[g];
        // fast path eligibility: homogeneous, and time did not move backwards for this key
        bool fast = !W.seg_het[g];
        if (fast) {
            const int64_t *ep = ks.epoch();
            for (int j = 0; j < ks.n; ++j)
                if (ep[j] != EPOCH_ABSENT && ep[j] > E) { fast = false; break; }
        }
        if (!fast) {
            for (uint32_t i = st; i < st + len; ++i) {
                const uint32_t seq = W.sseq[i];
                int64_t t;
                int32_t a;
                uint8_t fl;
                src.load(seq, t, a, fl);
                seq_event(T, key, ks, E, a, fl, seq, V);
            }
            W.seg_done[g] = 1;
            continue;
        }
        const int32_t a = W.seg_acq[g];
        const int slot = roll(T, key, ks, E);
        const int64_t s0 = window_sum(ks, E, EV_PASS);
        uint32_t lo = 0, hi = len;                      // K = first p with !admits(S0 + p*a)
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (admits(kind, thr, I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) lo = mid + 1;
            else hi = mid;
        }
        const uint32_t K = lo;
        const int64_t nb = (int64_t)(len - K);
        ks.cnt(EV_PASS, slot) = wrap_add(ks.cnt(EV_PASS, slot), wrap_mul((int64_t)K, a));
        if (ks.seven) {
            ks.cnt(EV_PASS_REQUEST, slot) = wrap_add(ks.cnt(EV_PASS_REQUEST, slot), (int64_t)K);
            ks.cnt(EV_BLOCK, slot) = wrap_add(ks.cnt(EV_BLOCK, slot), wrap_mul(nb, a));
            ks.cnt(EV_BLOCK_REQUEST, slot) = wrap_add(ks.cnt(EV_BLOCK_REQUEST, slot), nb);
        }
        W.seg_s0[g] = s0;
        W.seg_k[g] = K;
        W.seg_done[g] = 0;
    }
}

// Per sorted event: rank inside its segment decides; scatter the verdict to its arrival slot.
__global__ __launch_bounds__(256) void k_verdict(KeyTable T, BatchWork W, Verdicts V, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t nv = (int64_t)*W.nvalid;
    if (i >= nv) return;
    const uint32_t g = W.segid[i] - 1;
    if (W.seg_done[g]) return;
    const uint32_t rank = (uint32_t)i - W.seg_start[g];
    const uint32_t K = W.seg_k[g];
    const uint32_t seq = W.sseq[i];
    const uint32_t key = W.seg_key[g];
    const uint8_t kind = T.kind[key];
    if (kind == KIND_LIMITER) {
        if (rank >= K) reject_limited(V, seq);
        return;
    }
    if (rank < K) {
        const int32_t a = W.seg_acq[g];
        const int64_t x = wrap_add(W.seg_s0[g], wrap_mul((int64_t)rank, a));
        put_verdict(V.out, seq, ST_OK, java_d2i(remaining_of(T.thr[key], T.I_s[key], x, a)), 0);
    } else {
        put_verdict(V.out, seq, ST_BLOCKED, 0, 0);
    }
}

}  // namespace sentinel
