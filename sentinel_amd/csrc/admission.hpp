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
//   header  : {epoch_j, pass_j} pairs      (16 B per slot, padded to a multiple of 64 B)
//   rest    : n slots x 8 words            (only for 7-counter flow keys)
//             {BLOCK, PASS_REQUEST, BLOCK_REQUEST, OCCUPIED_PASS, OCCUPIED_BLOCK, WAITING, -, -}
// The fast path reads only the header (16n bytes) and writes one header word pair + one rest line.
#pragma once

#include "common.hpp"
#include "scan_sort.hpp"

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
constexpr int HB_KEYS = 64;    // flows per block of the blocked header region (one wave)
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
    int32_t hblock;          // > 0: headers in the blocked slot-major region (slots per block),
                             // rest counters in the blocked rest region at word rest_base
    int64_t rest_base;
    double max_occupy_ratio; // ServerFlowConfig.maxOccupyRatio
};

// The sorted 64-bit value of an event: [0,28) arrival position, [28] prioritized flag,
// [29,45) ts - T0 (signed 16 bits), [45,54) acquire (9 bits), [54,64) the partition path's local
// flow key (10 bits; 0 elsewhere).  Out-of-range ts deltas or acquire counts use the all-ones
// escape and are read back from the event itself.
constexpr uint32_t SEQ_MASK = 0x0FFFFFFFu;
constexpr uint64_t VAL_PRIO = 1ull << 28;
constexpr int VAL_DT_SHIFT = 29;
constexpr int VAL_DT_BITS = 16;
constexpr uint32_t VAL_DT_ESC = 0xFFFFu;
constexpr int VAL_ACQ_SHIFT = 45;
constexpr uint32_t VAL_ACQ_ESC = 0x1FFu;        // 9 bits
constexpr int VAL_KEY_SHIFT = 54;

__host__ __device__ inline int32_t val_dt(uint32_t dtf) {
    return (int32_t)(dtf << (32 - VAL_DT_BITS)) >> (32 - VAL_DT_BITS);
}

// Where the events of a pipeline run come from (one of the two is non-null).
struct EventSrc {
    const Event *ev;
    const ParamEvent *pev;
    const uint8_t *flags;    // may be null
    bool unit_acquire;       // limiter: acquire == 1 for every request
    const uint64_t *vals = nullptr;   // precomputed sorted values by arrival position (concurrency tokens)

    __device__ inline void load(uint32_t s, int64_t &ts, int32_t &a, uint8_t &fl) const {
        if (ev) { const Event e = ev[s]; ts = e.ts; a = e.acquire; }
        else { const ParamEvent e = pev[s]; ts = e.ts; a = e.acquire; }
        if (unit_acquire) a = 1;
        fl = flags ? flags[s] : 0;
    }

    __device__ inline int64_t t0() const { return ev ? ev[0].ts : pev[0].ts; }

    // Sorted value of arrival position s (layout above).
    __device__ inline uint64_t pack(uint32_t s, int64_t T0) const {
        if (vals) return vals[s];
        int64_t t;
        int32_t a;
        uint8_t fl;
        load(s, t, a, fl);
        return pack_fields(s, t, a, fl, T0);
    }
    // ... of an event already loaded (flow events)
    __device__ inline uint64_t pack_event(uint32_t s, const Event &e, uint8_t fl, int64_t T0) const {
        return pack_fields(s, e.ts, unit_acquire ? 1 : e.acquire, fl, T0);
    }
    __device__ inline uint64_t pack_fields(uint32_t s, int64_t t, int32_t a, uint8_t fl, int64_t T0) const {
        const int64_t dt = t - T0;
        const uint32_t dtf = (dt > -(1 << (VAL_DT_BITS - 1)) && dt < (1 << (VAL_DT_BITS - 1)) - 1)
                                 ? ((uint32_t)dt & VAL_DT_ESC) : VAL_DT_ESC;
        const uint32_t af = (a > 0 && a < (int32_t)VAL_ACQ_ESC) ? (uint32_t)a : VAL_ACQ_ESC;
        return (uint64_t)s | ((fl & 1u) ? VAL_PRIO : 0ull) | ((uint64_t)dtf << VAL_DT_SHIFT) | ((uint64_t)af << VAL_ACQ_SHIFT);
    }

    // Timestamp, acquire and prioritized flag of a sorted value (exact: escapes read the event).
    __device__ inline void unpack(uint64_t v, int64_t T0, int64_t &t, int32_t &a, bool &prio) const {
        const uint32_t dtf = (uint32_t)(v >> VAL_DT_SHIFT) & VAL_DT_ESC;
        const uint32_t af = (uint32_t)(v >> VAL_ACQ_SHIFT) & VAL_ACQ_ESC;
        prio = (v & VAL_PRIO) != 0;
        if (dtf == VAL_DT_ESC || af == VAL_ACQ_ESC) {
            uint8_t fl;
            load((uint32_t)v & SEQ_MASK, t, a, fl);
            return;
        }
        t = T0 + (int64_t)val_dt(dtf);
        a = unit_acquire ? 1 : (int32_t)af;
    }
};

// Batch working set, all device pointers, sized for n events.
struct BatchWork {
    uint32_t *skey;              // sorted keys
    uint64_t *sval;              // sorted values (arrival position, prio, ts - T0, acquire)
    uint32_t *segid;             // head flags, scanned in place (1-based segment id)
    uint8_t *bad;                // element breaks segment homogeneity (acquire differs / prioritized)
    int64_t *h_epoch;            // epoch at head positions (sparse)
    int32_t *h_acq;              // acquire at head positions (sparse)
    uint32_t *seg_start;         // S+1 entries
    uint32_t *seg_key;
    int64_t *seg_epoch;
    int32_t *seg_acq;
    uint8_t *seg_het;            // heterogeneous / prioritized segment
    uint8_t *seg_prio;           // segment holds a prioritized cluster request (the sequential path)
    uint8_t *seg_done;           // decided by the sequential path
    int64_t *seg_s0;             // PASS sum at segment start (after the roll)
    uint32_t *seg_k;             // number of passing events
    uint32_t *nvalid;            // device: events with a valid key
    uint32_t *nseg;              // device: number of segments
    uint32_t *zero4 = nullptr;   // four words the segment kernel zeroes (the hot-run list counters: no memset)
};

// Packed TokenResult: {int32 remaining; int16 status; uint16 waitInMs} as one 8-byte store.
__device__ inline uint64_t pack_verdict(int status, int32_t remaining, int wait) {
    return (uint64_t)(uint32_t)remaining | ((uint64_t)(uint16_t)(int16_t)status << 32) | ((uint64_t)(uint16_t)wait << 48);
}
// A verdict store to its arrival position (random 8-byte writes over the whole output).
__device__ inline void store_verdict(uint64_t *out, uint32_t seq, uint64_t v) {
#ifdef SENTINEL_NT_VERDICT
    __builtin_nontemporal_store(v, out + seq);
#else
    out[seq] = v;
#endif
}
__device__ inline void put_verdict(uint64_t *out, uint32_t seq, int status, int32_t remaining, int wait) {
    out[seq] = pack_verdict(status, remaining, wait);
}

// Outputs of one pipeline run.
struct Verdicts {
    uint64_t *out;
    // LIMITER mode: events that fail get status TOO_MANY_REQUEST and flow_key[seq] = flow_key_invalid
    uint32_t *flow_key;
    uint32_t flow_key_invalid;
    // decide-order output (partition path, sentinel_submit_flow_batch_ordered): the verdict of the event
    // at sorted position q of a run goes to out[obase + q] -- whole lines, range-local -- and oseq[obase +
    // q] holds its arrival position (written from the sorted values, not per verdict); null: out[arrival]
    uint32_t *oseq = nullptr;
    uint32_t obase = 0;
    // where the verdict of the event at sorted position q (packed value v) goes
    __device__ inline uint32_t at(uint32_t q, uint64_t v) const { return oseq ? obase + q : (uint32_t)v & SEQ_MASK; }
    __device__ inline void put(uint32_t q, uint64_t v, uint64_t vd) const { store_verdict(out, at(q, v), vd); }
    __device__ inline Verdicts based(uint32_t b) const {
        Verdicts r = *this;
        r.obase = b;
        return r;
    }
};

// Decide-order output (Verdicts::oseq): a request decided by validation (rej) goes to position n - 1 - its
// rank among the batch's rejected requests, counted in *ctr with one atomic per wave -- the pipeline's
// sorted / grouped requests fill [0, valid), so the rejected ones fill [valid, n) -- with its arrival
// position in oseq.  Called by every lane of the wave that reached the item (divergent lanes are fine:
// the ballot sees the active ones).
__device__ inline void put_rejected_ordered(bool rej, uint64_t *out, uint32_t *oseq, uint32_t *ctr, int64_t n,
                                            uint32_t seq, int st) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(rej);
    if (!m) return;
    const uint32_t lane = lane_id();
    const int lead = __ffsll((unsigned long long)m) - 1;
    uint32_t b = 0;
    if ((int)lane == lead) b = atomicAdd(ctr, (uint32_t)__popcll(m));
    b = __shfl(b, lead, WAVE);
    if (rej) {
        const uint32_t pos = (uint32_t)(n - 1) - (b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull)));
        put_verdict(out, pos, st, 0, 0);
        oseq[pos] = seq;
    }
}

// A key's state: header pair j {epoch, PASS} at base + hs*j (hs = 2: contiguous record;
// hs = 2*HB_KEYS: the flow table's blocked slot-major header region); the other six counters of
// slot j (BLOCK .. WAITING) at rbase + rs*j + rcs*c (rs = 8, rcs = 1: a contiguous rest line;
// rs = 6*HB_KEYS, rcs = HB_KEYS: the flow table's blocked rest region, counter-major per slot, so
// the 64 lanes of a wave touching counter c of slot j of 64 consecutive flows touch 512 B).
struct KeyState {
    int64_t *base;
    int64_t *rbase;
    int hs;
    int n;
    int rs, rcs;
    bool seven;   // 7-counter flow layout
    __device__ inline int64_t *pair(int slot) const { return base + (int64_t)hs * slot; }
    __device__ inline int64_t &ep(int slot) const { return pair(slot)[0]; }
    __device__ inline int64_t &cnt(int ev, int slot) const {
        if (ev == EV_PASS || !seven) return pair(slot)[1];
        return rc(slot, ev - 1);
    }
    __device__ inline int64_t &rc(int slot, int c) const { return rbase[(int64_t)rs * slot + (int64_t)rcs * c]; }
    // ClusterMetric.add of a decided homogeneous segment on slot `slot` (CFC:76-77,100-101):
    // BLOCK += nb*a, PASS_REQUEST += K, BLOCK_REQUEST += nb, from the slot's previous values
    // (zero for a fresh bucket, whose other counters are cleared: LeapArray.resetWindowTo)
    // the same for a heterogeneous segment: BLOCK += sum of blocked acquires, PASS_REQUEST += passes,
    // BLOCK_REQUEST += blocks
    __device__ inline void book_rest_sums(int slot, bool fresh, int64_t blk, int64_t preq, int64_t breq,
                                          int64_t add_blk, int64_t add_preq, int64_t add_breq) const {
        if (fresh) { blk = 0; preq = 0; breq = 0; }
        rc(slot, EV_BLOCK - 1) = wrap_add(blk, add_blk);
        rc(slot, EV_PASS_REQUEST - 1) = wrap_add(preq, add_preq);
        rc(slot, EV_BLOCK_REQUEST - 1) = wrap_add(breq, add_breq);
        if (fresh)
#pragma unroll
            for (int c = 3; c < 6; ++c) rc(slot, c) = 0;
    }
    __device__ inline void book_rest(int slot, bool fresh, int64_t blk, int64_t preq, int64_t breq, int64_t nb,
                                     int32_t a, uint32_t K) const {
        if (fresh) { blk = 0; preq = 0; breq = 0; }
        rc(slot, EV_BLOCK - 1) = wrap_add(blk, wrap_mul(nb, a));
        rc(slot, EV_PASS_REQUEST - 1) = wrap_add(preq, (int64_t)K);
        rc(slot, EV_BLOCK_REQUEST - 1) = wrap_add(breq, nb);
        if (fresh)
#pragma unroll
            for (int c = 3; c < 6; ++c) rc(slot, c) = 0;
    }
};

// Slots per block of the flow header region: the kernel template bucket of the largest n, so a
// kernel instantiated for NMAX slots may load all NMAX pairs of any flow without bounds checks.
__host__ __device__ inline int32_t header_block_slots(int32_t maxn) {
    return maxn <= 2 ? 2 : maxn <= 4 ? 4 : maxn <= 10 ? 10 : maxn <= 16 ? 16 : maxn;
}

// Words per param-table slot: the header of the kernel template bucket of the largest n, so that
// k_process_reg<NMAX> may request all NMAX pairs of a slot before its n is known (one dependent
// memory round trip less per key).
__host__ __device__ inline int64_t param_stride(int32_t maxn) { return header_words(header_block_slots(maxn)); }

// Flow-table header region: blocks of HB_KEYS flows, slot-major inside a block, so the 64 lanes
// of a wave that read slot j of 64 consecutive flows read 1 KB of contiguous memory.
__host__ __device__ inline int64_t blocked_pair_word(int64_t key, int hblock, int slot) {
    return 2 * ((((key / HB_KEYS) * hblock + slot) * HB_KEYS) + key % HB_KEYS);
}

// Flow-table rest region (after the header region): blocks of HB_KEYS flows, per slot six
// counter rows of HB_KEYS words.  Word of counter c of slot j of flow `key`, from the region start.
__host__ __device__ inline int64_t blocked_rest_word(int64_t key, int hblock, int slot, int c) {
    return (((key / HB_KEYS) * hblock + slot) * 6 + c) * HB_KEYS + key % HB_KEYS;
}

__device__ inline KeyState key_state(const KeyTable &T, uint32_t key) {
    KeyState k;
    k.n = T.n[key];
    k.seven = T.ncounters == NEV;
    if (T.hblock) {                              // pure address arithmetic: no dependent load
        k.base = T.state + blocked_pair_word(key, T.hblock, 0);
        k.hs = 2 * HB_KEYS;
        k.rbase = T.state + T.rest_base + blocked_rest_word(key, T.hblock, 0, 0);
        k.rs = 6 * HB_KEYS;
        k.rcs = HB_KEYS;
    } else {
        const int64_t off = T.state_off ? T.state_off[key] : (int64_t)key * T.state_stride;
        k.base = T.state + off;
        k.hs = 2;
        k.rbase = k.base + header_words(k.n);
        k.rs = 8;
        k.rcs = 1;
    }
    return k;
}

// LeapArray.currentWindow(t) on epochs: returns the slot, or -1 for the detached wrap (clock
// went backwards: LeapArray.java:241-246, writes to it are lost).
__device__ inline int roll(const KeyTable &T, uint32_t key, const KeyState &S, int64_t E) {
    const int slot = (int)(E % S.n);
    const int64_t cur = S.ep(slot);
    if (cur == E) return slot;                                  // LA:195-209 same window
    if (cur != EPOCH_ABSENT && cur > E) return -1;              // LA:241-246 detached
    const bool reset = cur != EPOCH_ABSENT;                     // LA:210-240 vs LA:172-194
    S.ep(slot) = E;
    S.cnt(EV_PASS, slot) = 0;
    if (S.seven) {
#pragma unroll
        for (int c = 0; c < 6; ++c) S.rc(slot, c) = 0;
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
    int64_t s = 0;
    for (int j = 0; j < S.n; ++j) {
        const int64_t e = S.ep(j);
        if (e != EPOCH_ABSENT && e > E - S.n) s = wrap_add(s, S.cnt(ev, j));
    }
    return s;
}

__device__ inline void add_counter(const KeyTable &T, uint32_t key, const KeyState &S, int64_t E, int ev, int64_t x) {
    const int slot = roll(T, key, S, E);
    if (slot >= 0) S.cnt(ev, slot) = wrap_add(S.cnt(ev, slot), x);
}

// The monotone admission predicate of each checker, evaluated in Java operation order.
// x / I_s as Java evaluates it (one correctly rounded IEEE division).  When I_s is a normal power
// of two (1.0 for every 1000 ms interval) the quotient is x * 2^-k, which v_ldexp_f64 produces
// exactly with the same rounding -- one instruction instead of the div_scale/rcp/fma/fixup chain.
__device__ inline double div_interval(double x, double I_s) {
    const uint64_t b = (uint64_t)__double_as_longlong(I_s);
    const uint32_t ex = (uint32_t)(b >> 52) & 0x7FFu;
    if ((b & 0x000FFFFFFFFFFFFFull) == 0 && ex != 0 && ex != 0x7FFu && !(b >> 63))
        return ldexp(x, 1023 - (int)ex);
    return x / I_s;
}

__device__ inline bool admits(uint8_t kind, double thr, double I_s, int64_t x, int32_t a) {
    const double avg = div_interval((double)x, I_s);
    switch (kind) {
        case KIND_LIMITER: return avg + 1.0 <= thr;                      // RequestLimiter.java:72-74
        case KIND_PARAM: return !(((thr - avg) - (double)a) < 0.0);       // ClusterParamFlowChecker.java:64-66
        default: return ((thr - avg) - (double)a) >= 0.0;                 // ClusterFlowChecker.java:69-71
    }
}

__device__ inline double remaining_of(double thr, double I_s, int64_t x, int32_t a) {
    return (thr - div_interval((double)x, I_s)) - (double)a;
}

// A segment whose events share the epoch but not the acquire count, with no prioritized cluster
// request, no pending occupy transfer and no slot newer than its epoch: the reference state machine
// (seq_event) reduced to what such a segment can reach.  Every event reads the same rolled window, so
// the running PASS sum lives in a register -- x = S0 + passed, event k passes iff the checker's test
// holds for (x, a_k) in Java operation order (ClusterFlowChecker.java:67-82,
// SimpleClusterFlowChecker.java:41-64, ClusterParamFlowChecker.java:62-70) -- and the counters are
// booked once at the end instead of per event in global memory.
struct HetSums {
    int64_t pass, npass, block, nblock;
};

// Events are fetched HW at a time (independent loads in flight together, values kept in registers
// for the verdict stores); once not even an acquire of 1 is admitted (acquire >= 1 past validation,
// admits monotone in both arguments) the rest of the segment is blocked without evaluating the test.
// load(k) -> the k-th packed value, acq(v) -> its acquire count, put(k, v, verdict).
template <uint32_t HW, class Load, class Acq, class Put>
__device__ inline HetSums het_walk(uint8_t kind, double thr, double I_s, int64_t s0, uint32_t len, Load load, Acq acq,
                                   Put put) {
    HetSums h{0, 0, 0, 0};
    bool dead = false;
    for (uint32_t k0 = 0; k0 < len; k0 += HW) {
        uint64_t vv[HW];
#pragma unroll
        for (uint32_t j = 0; j < HW; ++j) vv[j] = k0 + j < len ? load(k0 + j) : 0ull;
        if (!dead) dead = !admits(kind, thr, I_s, wrap_add(s0, h.pass), 1);
#pragma unroll
        for (uint32_t j = 0; j < HW; ++j) {
            if (k0 + j >= len) continue;
            const int32_t a = acq(vv[j]);
            const double next = dead ? -1.0 : remaining_of(thr, I_s, wrap_add(s0, h.pass), a);
            const bool ok = kind == KIND_PARAM ? !(next < 0.0) : next >= 0.0;
            if (ok) {
                h.pass = wrap_add(h.pass, a);
                h.npass += 1;
                put(k0 + j, vv[j], pack_verdict(ST_OK, java_d2i(next), 0));
            } else {
                h.block = wrap_add(h.block, a);
                h.nblock += 1;
                put(k0 + j, vv[j], pack_verdict(ST_BLOCKED, 0, 0));
            }
        }
    }
    return h;
}

__device__ inline void reject_limited(const Verdicts &V, uint32_t seq, uint32_t at) {
    put_verdict(V.out, at, ST_TOO_MANY_REQUEST, 0, 0);
    V.flow_key[seq] = V.flow_key_invalid;
}

// One event through the reference state machine (the sequential path).
__device__ inline void seq_event(const KeyTable &T, uint32_t key, const KeyState &S, int64_t E, int32_t a,
                                 uint8_t flags, uint32_t seq, const Verdicts &V, uint32_t at) {
    // (at: where the verdict goes -- seq, or the sorted position in decide-order output; seq keys the
    // limiter's flow-key invalidation)
    const uint8_t kind = T.kind[key];
    const double thr = T.thr[key];
    const double I_s = T.I_s[key];
    if (kind == KIND_LIMITER) {
        roll(T, key, S, E);
        const int64_t sum = window_sum(S, E, EV_PASS);
        if (admits(kind, thr, I_s, sum, 1)) add_counter(T, key, S, E, EV_PASS, 1);
        else reject_limited(V, seq, at);
        return;
    }
    if (kind == KIND_PARAM) {
        roll(T, key, S, E);
        const int64_t sum = window_sum(S, E, EV_PASS);
        const double next = remaining_of(thr, I_s, sum, a);
        if (!(next < 0.0)) {
            add_counter(T, key, S, E, EV_PASS, a);
            put_verdict(V.out, at, ST_OK, java_d2i(next), 0);
        } else {
            put_verdict(V.out, at, ST_BLOCKED, 0, 0);
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
        put_verdict(V.out, at, ST_OK, java_d2i(next), 0);
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
            const int64_t he = S.ep(hs);
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
                    put_verdict(V.out, at, ST_SHOULD_WAIT, 0, wait);
                    return;
                }
            }
        }
    }
    add_counter(T, key, S, E, EV_BLOCK, a);
    add_counter(T, key, S, E, EV_BLOCK_REQUEST, 1);
    if (prio) add_counter(T, key, S, E, EV_OCCUPIED_BLOCK, a);
    put_verdict(V.out, at, ST_BLOCKED, 0, 0);
}

// K2 pass with payload: stable scatter of (key, seq|prio, payload) by one 8-bit digit.  The first
// pass (FIRST) reads the arrival-ordered events themselves, so the sorted events never have to
// be gathered back by position: later kernels read key, seq and {ts - T0, acquire} coalesced.
// Tile = 4096 (4 waves x 16 items, lane-striped to keep arrival order), ranked with 8 ballots
// per item, staged in LDS in digit order and written as contiguous per-digit runs.
template <bool FIRST>
__global__ __launch_bounds__(SORT_THREADS) void k_radix_scatter_p(
    const uint32_t *__restrict__ keys_in, const uint64_t *__restrict__ vals_in, EventSrc src,
    uint32_t *__restrict__ keys_out, uint64_t *__restrict__ vals_out, int64_t n, int shift,
    const uint32_t *__restrict__ offsets, int64_t nblocks, uint8_t *__restrict__ z0 = nullptr,
    uint8_t *__restrict__ z1 = nullptr) {
    // z0 / z1 (optional): byte arrays of n entries zeroed over this tile's positions -- the segment
    // flags k_segments sets, cleared here instead of by two fill launches in front of it
    __shared__ uint32_t cnt[SORT_WAVES][RADIX];
    __shared__ uint32_t goff[RADIX];
    __shared__ uint32_t loff[RADIX];
    __shared__ uint32_t waves_tot[SORT_WAVES];
    __shared__ uint32_t skeys[SORT_TILE];
    __shared__ uint64_t svals[SORT_TILE];
    const int wave = threadIdx.x / WAVE;
    const uint32_t lane = lane_id();
    for (int d = threadIdx.x; d < RADIX; d += SORT_THREADS) {
#pragma unroll
        for (int w = 0; w < SORT_WAVES; ++w) cnt[w][d] = 0;
        goff[d] = offsets[(int64_t)d * nblocks + blockIdx.x];
    }
    __syncthreads();
    const int64_t tile0 = (int64_t)blockIdx.x * SORT_TILE;
    const int64_t base = tile0 + (int64_t)wave * (SORT_ITEMS * WAVE);
    const int64_t T0 = FIRST ? src.t0() : 0;
    if (z0) {
        const int64_t end = n - tile0 < SORT_TILE ? n : tile0 + SORT_TILE;
        const int64_t wend = tile0 + ((end - tile0) & ~(int64_t)3);   // whole words inside [tile0, end)
        for (int64_t q = tile0 + 4 * (int64_t)threadIdx.x; q < wend; q += 4 * SORT_THREADS) {
            *reinterpret_cast<uint32_t *>(z0 + q) = 0u;
            *reinterpret_cast<uint32_t *>(z1 + q) = 0u;
        }
        if ((int64_t)threadIdx.x < end - wend) {
            z0[wend + threadIdx.x] = 0;
            z1[wend + threadIdx.x] = 0;
        }
    }
    uint32_t key[SORT_ITEMS], rank[SORT_ITEMS];
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = base + j * WAVE + lane;
        key[j] = i < n ? keys_in[i] : 0u;
    }
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = base + j * WAVE + lane;
        const bool valid = i < n;
        const uint32_t d = (key[j] >> shift) & (RADIX - 1);
        const uint64_t peers = match_peers<RADIX_BITS>(d, valid, RADIX_BITS);
        uint32_t r = 0;
        if (valid) r = cnt[wave][d] + mask_rank(peers);
        __builtin_amdgcn_wave_barrier();
        if (valid && (uint32_t)(__ffsll((unsigned long long)peers) - 1) == lane)
            cnt[wave][d] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        rank[j] = valid ? r : 0xFFFFFFFFu;
    }
    __syncthreads();
    uint32_t dtot = 0;
    const int d0 = threadIdx.x;   // one thread per digit (SORT_THREADS >= RADIX)
    if (d0 < RADIX) {
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < SORT_WAVES; ++w) {
            const uint32_t c = cnt[w][d0];
            cnt[w][d0] = run;
            run += c;
        }
        dtot = run;
    }
    uint32_t total;
    const uint32_t lst = block_exclusive_scan(dtot, waves_tot, &total);
    if (d0 < RADIX) loff[d0] = lst;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        if (rank[j] == 0xFFFFFFFFu) continue;
        const int64_t i = base + j * WAVE + lane;
        const uint32_t d = (key[j] >> shift) & (RADIX - 1);
        const uint32_t p = loff[d] + cnt[wave][d] + rank[j];
        skeys[p] = key[j];
        svals[p] = FIRST ? src.pack((uint32_t)i, T0) : vals_in[i];
    }
    __syncthreads();
    const int64_t valid_in_tile = (n - tile0) < SORT_TILE ? (n - tile0) : SORT_TILE;
    for (int p = threadIdx.x; p < valid_in_tile; p += SORT_THREADS) {
        const uint32_t k = skeys[p];
        const uint32_t d = (k >> shift) & (RADIX - 1);
        const uint32_t dst = goff[d] + (uint32_t)p - loff[d];
        if (dst >= (uint64_t)n) continue;          // guard: a corrupt offset must never write out of bounds
        keys_out[dst] = k;
        vals_out[dst] = svals[p];
    }
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
    const int64_t T0 = src.t0();
    uint32_t key = invalid;
    int64_t E = 0;
    int32_t a = 0;
    bool prio = false;
    if (i < n) {
        key = W.skey[i];
        if (key != invalid) {
            int64_t t;
            src.unpack(W.sval[i], T0, t, a, prio);
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
        bool pp;
        src.unpack(W.sval[i - 1], T0, t, pa, pp);
        pE = epoch_of(t, T.w[pk], T.rcp_w[pk]);
    }
    const bool head = pk != key || pE != E;
    W.segid[i] = head ? 1u : 0u;
    prio = prio && T.kind[key] == KIND_CLUSTER;
    W.bad[i] = (!head && pa != a) || prio;
    if (head) { W.h_epoch[i] = E; W.h_acq[i] = a; }
    if (i == n - 1 || W.skey[i + 1] == invalid) *W.nvalid = (uint32_t)(i + 1);
}

// Segment construction in one pass (replaces heads -> scan -> mark): per 4096-element tile of the
// sorted batch, compute each event's epoch, (key, epoch) run heads and homogeneity; a block scan
// plus decoupled look-back gives every event its global segment id; heads write the segment
// records {start, key, epoch, acquire}, non-homogeneous events flag their segment.  seg_het must
// be zeroed before the launch (the look-back words need no clearing: LBState).
constexpr int SEG_THREADS = 256;
constexpr int SEG_ITEMS = 16;
constexpr int SEG_TILE = SEG_THREADS * SEG_ITEMS;

__global__ __launch_bounds__(SEG_THREADS) void k_segments(KeyTable T, BatchWork W, EventSrc src, int64_t n,
                                                          uint32_t invalid, LBState L) {
    __shared__ uint32_t s_key[SEG_TILE];
    __shared__ uint64_t s_val[SEG_TILE];
    __shared__ uint32_t l_key[SEG_THREADS];
    __shared__ int64_t l_ep[SEG_THREADS];
    __shared__ int32_t l_acq[SEG_THREADS];
    __shared__ uint32_t waves[SEG_THREADS / WAVE];
    __shared__ uint32_t s_prefix;
    __shared__ uint32_t p_key;
    __shared__ int64_t p_ep;
    __shared__ int32_t p_acq;
    const int64_t bid = lookback_ticket(L);
    const int64_t base = bid * SEG_TILE;
    if (W.zero4 && bid == 0 && threadIdx.x < 4) W.zero4[threadIdx.x] = 0u;
    const int64_t T0 = src.t0();
#pragma unroll
    for (int j = 0; j < SEG_ITEMS; ++j) {
        const int64_t i = base + j * SEG_THREADS + threadIdx.x;
        const bool in = i < n;
        s_key[j * SEG_THREADS + threadIdx.x] = in ? W.skey[i] : invalid;
        s_val[j * SEG_THREADS + threadIdx.x] = in ? W.sval[i] : 0ull;
    }
    if (threadIdx.x == 0) {           // the element just before this tile
        p_key = invalid;
        p_ep = 0;
        p_acq = 0;
        if (base > 0 && base - 1 < n) {
            const uint32_t k = W.skey[base - 1];
            if (k != invalid) {
                int64_t t;
                int32_t a;
                bool pr;
                src.unpack(W.sval[base - 1], T0, t, a, pr);
                p_key = k;
                p_ep = epoch_of(t, T.w[k], T.rcp_w[k]);
                p_acq = a;
            }
        }
    }
    __syncthreads();
    // this thread's contiguous run of SEG_ITEMS sorted events
    uint32_t key[SEG_ITEMS];
    int64_t ep[SEG_ITEMS];
    int32_t acq[SEG_ITEMS];
    bool prio[SEG_ITEMS];
#pragma unroll
    for (int j = 0; j < SEG_ITEMS; ++j) {
        const int q = threadIdx.x * SEG_ITEMS + j;
        key[j] = s_key[q];
        ep[j] = 0;
        acq[j] = 0;
        prio[j] = false;
        if (key[j] != invalid) {
            int64_t t;
            src.unpack(s_val[q], T0, t, acq[j], prio[j]);
            ep[j] = epoch_of(t, T.w[key[j]], T.rcp_w[key[j]]);
            prio[j] = prio[j] && T.kind[key[j]] == KIND_CLUSTER;
        }
    }
    l_key[threadIdx.x] = key[SEG_ITEMS - 1];
    l_ep[threadIdx.x] = ep[SEG_ITEMS - 1];
    l_acq[threadIdx.x] = acq[SEG_ITEMS - 1];
    __syncthreads();
    uint32_t pk = threadIdx.x ? l_key[threadIdx.x - 1] : p_key;
    int64_t pe = threadIdx.x ? l_ep[threadIdx.x - 1] : p_ep;
    int32_t pa = threadIdx.x ? l_acq[threadIdx.x - 1] : p_acq;
    uint32_t headmask = 0, badmask = 0;
#pragma unroll
    for (int j = 0; j < SEG_ITEMS; ++j) {
        if (key[j] != invalid) {
            const bool head = pk != key[j] || pe != ep[j];
            if (head) headmask |= 1u << j;
            if ((!head && pa != acq[j]) || prio[j]) badmask |= 1u << j;
        }
        pk = key[j];
        pe = ep[j];
        pa = acq[j];
    }
    uint32_t total;
    uint32_t g = block_exclusive_scan((uint32_t)__popc(headmask), waves, &total);
    tile_lookback(bid, total, L, &s_prefix);
    __syncthreads();
    g += s_prefix;                   // segments started before this thread's run
#pragma unroll
    for (int j = 0; j < SEG_ITEMS; ++j) {
        const int q = threadIdx.x * SEG_ITEMS + j;
        const int64_t i = base + q;
        if (key[j] == invalid) { s_key[q] = 0; continue; }
        if (headmask & (1u << j)) {
            ++g;
            W.seg_start[g - 1] = (uint32_t)i;
            W.seg_key[g - 1] = key[j];
            W.seg_epoch[g - 1] = ep[j];
            W.seg_acq[g - 1] = acq[j];
        }
        if (badmask & (1u << j)) W.seg_het[g - 1] = 1;
        if (prio[j]) W.seg_prio[g - 1] = 1;
        s_key[q] = g;                // 1-based segment id
        const bool last = (i == n - 1) || (j + 1 < SEG_ITEMS ? key[j + 1] == invalid : W.skey[i + 1] == invalid);
        if (last) {
            *W.nvalid = (uint32_t)(i + 1);
            *W.nseg = g;
            W.seg_start[g] = (uint32_t)(i + 1);
        }
    }
    if (bid == 0 && threadIdx.x == 0 && key[0] == invalid) { *W.nvalid = 0; *W.nseg = 0; }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SEG_ITEMS; ++j) {
        const int64_t i = base + j * SEG_THREADS + threadIdx.x;
        if (i < n) W.segid[i] = s_key[j * SEG_THREADS + threadIdx.x];
    }
}

// k_segments without staging the tile in LDS: each thread reads its own ITEMS contiguous sorted
// keys and values with 16-byte vector loads (a wave still covers one contiguous stretch), issues
// every item's window-width gather before the first epoch is computed, and exchanges only its run's
// first / last element through LDS.  Same outputs and preconditions as k_segments.
template <int THREADS, int ITEMS>
__global__ __launch_bounds__(THREADS) void k_segments_v(KeyTable T, BatchWork W, EventSrc src, int64_t n,
                                                         uint32_t invalid, LBState L) {
    static_assert(ITEMS % 4 == 0, "4 keys / 2 values per vector load");
    constexpr int TILE = THREADS * ITEMS;
    __shared__ uint32_t f_key[THREADS + 1];     // first key of every thread's run (+ the next tile's)
    __shared__ uint32_t l_key[THREADS];
    __shared__ int64_t l_ep[THREADS];
    __shared__ int32_t l_acq[THREADS];
    __shared__ uint32_t waves[THREADS / WAVE];
    __shared__ uint32_t s_prefix;
    __shared__ uint32_t p_key;
    __shared__ int64_t p_ep;
    __shared__ int32_t p_acq;
    const int64_t bid = lookback_ticket(L);
    const int64_t base = bid * TILE;
    if (W.zero4 && bid == 0 && threadIdx.x < 4) W.zero4[threadIdx.x] = 0u;
    const int64_t i0 = base + (int64_t)threadIdx.x * ITEMS;
    const int64_t T0 = src.t0();
    uint32_t key[ITEMS];
    uint64_t val[ITEMS];
    const bool full = i0 + ITEMS <= n;
    if (full) {
        const uint4 *kp = reinterpret_cast<const uint4 *>(W.skey + i0);
        const uint4 *vp = reinterpret_cast<const uint4 *>(W.sval + i0);
#pragma unroll
        for (int m = 0; m < ITEMS / 4; ++m) {
            const uint4 k = kp[m];
            key[4 * m] = k.x; key[4 * m + 1] = k.y; key[4 * m + 2] = k.z; key[4 * m + 3] = k.w;
        }
#pragma unroll
        for (int m = 0; m < ITEMS / 2; ++m) {
            const uint4 v = vp[m];
            val[2 * m] = (uint64_t)v.x | ((uint64_t)v.y << 32);
            val[2 * m + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
        }
    } else {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const bool in = i0 + j < n;
            key[j] = in ? W.skey[i0 + j] : invalid;
            val[j] = in ? W.sval[i0 + j] : 0ull;
        }
    }
    if (threadIdx.x == 0) {           // the element just before this tile, and the one after it
        p_key = invalid;
        p_ep = 0;
        p_acq = 0;
        if (base > 0 && base - 1 < n) {
            const uint32_t k = W.skey[base - 1];
            if (k != invalid) {
                int64_t t;
                int32_t a;
                bool pr;
                src.unpack(W.sval[base - 1], T0, t, a, pr);
                p_key = k;
                p_ep = epoch_of(t, T.w[k], T.rcp_w[k]);
                p_acq = a;
            }
        }
        f_key[THREADS] = base + TILE < n ? W.skey[base + TILE] : invalid;
    }
    // only the window length is gathered (param tables: one random line per distinct slot); its
    // reciprocal is the host's 1.0 / w, recomputed (epoch_of is exact for any close reciprocal anyway)
    int32_t wv[ITEMS];
    double rc[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) wv[j] = key[j] != invalid ? T.w[key[j]] : 1;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) rc[j] = 1.0 / (double)wv[j];
    int64_t ep[ITEMS];
    int32_t acq[ITEMS];
    uint32_t priomask = 0;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        ep[j] = 0;
        acq[j] = 0;
        if (key[j] != invalid) {
            int64_t t;
            bool pr;
            src.unpack(val[j], T0, t, acq[j], pr);
            ep[j] = epoch_of(t, wv[j], rc[j]);
            if (pr && T.kind[key[j]] == KIND_CLUSTER) priomask |= 1u << j;
        }
    }
    f_key[threadIdx.x] = key[0];
    l_key[threadIdx.x] = key[ITEMS - 1];
    l_ep[threadIdx.x] = ep[ITEMS - 1];
    l_acq[threadIdx.x] = acq[ITEMS - 1];
    __syncthreads();
    uint32_t pk = threadIdx.x ? l_key[threadIdx.x - 1] : p_key;
    int64_t pe = threadIdx.x ? l_ep[threadIdx.x - 1] : p_ep;
    int32_t pa = threadIdx.x ? l_acq[threadIdx.x - 1] : p_acq;
    const uint32_t next_key = f_key[threadIdx.x + 1];
    uint32_t headmask = 0, badmask = 0;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        if (key[j] != invalid) {
            const bool head = pk != key[j] || pe != ep[j];
            if (head) headmask |= 1u << j;
            if ((!head && pa != acq[j]) || (priomask & (1u << j))) badmask |= 1u << j;
        }
        pk = key[j];
        pe = ep[j];
        pa = acq[j];
    }
    uint32_t total;
    uint32_t g = block_exclusive_scan((uint32_t)__popc(headmask), waves, &total);
    tile_lookback(bid, total, L, &s_prefix);
    __syncthreads();
    g += s_prefix;                   // segments started before this thread's run
    uint32_t sid[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
        const int64_t i = i0 + j;
        sid[j] = 0;
        if (key[j] == invalid) continue;
        if (headmask & (1u << j)) {
            ++g;
            W.seg_start[g - 1] = (uint32_t)i;
            W.seg_key[g - 1] = key[j];
            W.seg_epoch[g - 1] = ep[j];
            W.seg_acq[g - 1] = acq[j];
        }
        if (badmask & (1u << j)) W.seg_het[g - 1] = 1;
        if (priomask & (1u << j)) W.seg_prio[g - 1] = 1;
        sid[j] = g;                  // 1-based segment id
        const bool last = (i == n - 1) || (j + 1 < ITEMS ? key[j + 1] == invalid : next_key == invalid);
        if (last) {
            *W.nvalid = (uint32_t)(i + 1);
            *W.nseg = g;
            W.seg_start[g] = (uint32_t)(i + 1);
        }
    }
    if (bid == 0 && threadIdx.x == 0 && key[0] == invalid) { *W.nvalid = 0; *W.nseg = 0; }
    if (full) {
        uint4 *sp = reinterpret_cast<uint4 *>(W.segid + i0);
#pragma unroll
        for (int m = 0; m < ITEMS / 4; ++m) sp[m] = make_uint4(sid[4 * m], sid[4 * m + 1], sid[4 * m + 2], sid[4 * m + 3]);
    } else {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j)
            if (i0 + j < n) W.segid[i0 + j] = sid[j];
    }
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
    if (W.bad[i]) { W.seg_het[g - 1] = 1; W.seg_prio[g - 1] = 1; }   // (split path: prio not told apart)
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
        if (fast && ks.seven && kind == KIND_CLUSTER && T.has_occ[key]) fast = false;   // occupy transfer pending
        if (fast) {
            for (int j = 0; j < ks.n; ++j)
                if (ks.ep(j) != EPOCH_ABSENT && ks.ep(j) > E) { fast = false; break; }
        }
        if (!fast) {
            for (uint32_t i = st; i < st + len; ++i) {
                const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
                int64_t t;
                int32_t a;
                uint8_t fl;
                src.load(seq, t, a, fl);
                seq_event(T, key, ks, E, a, fl, seq, V, V.oseq ? V.obase + i : seq);
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

// K1+K3, one thread per key with the key's header {epoch, pass} pairs held in registers
// (NMAX >= n).  All header lines are requested at once with 16-byte loads, so each line of the
// state crosses the memory system once per batch; only the rolled slot's pair and its rest line
// are written back.  Slow segments fall back to the sequential path on global memory.
// A key with more events than this and a heterogeneous-acquire segment is handed to the workgroup
// kernels (k_part_long, cooperative walk) instead of one lane walking every event (the engine's
// default; SENTINEL_HOT_HET_RUN overrides it).
constexpr uint32_t HOT_HET_RUN = 4096;

// Hot runs handed to the workgroup kernels (k_long_scan -> k_part_long -> k_long_dead).  Run r =
// {q0, q1, key, first chunk} over the sorted values; its events are cut in LR_CHUNK-event chunks
// numbered consecutively over the batch (chunk_run[g] = run of chunk g), each with a summary record.
constexpr uint32_t LR_CHUNK = 4096;
constexpr uint32_t LR_UNIFORM = 1u;    // one epoch, no prioritized cluster request
constexpr uint32_t LR_DEAD = 2u;       // every event blocked: k_long_dead writes the verdicts
struct LongRec {
    int64_t E;            // epoch of the chunk's first event
    int64_t acq;          // sum of the chunk's acquire counts
    uint32_t cnt;         // events
    uint32_t flags;
    int64_t pad;
};
struct LongRuns {
    uint32_t *nrun;       // runs pushed
    uint32_t *nchunk;     // chunks pushed
    uint32_t *runs;       // 4 words per run
    uint32_t *chunk_run;
    LongRec *rec;         // null: no chunk summaries this batch (k_part_long decides every chunk)
    uint32_t *host_chunks;  // pinned: the batch's chunk count, a hint for the next batch's launch
    __device__ inline void push(uint32_t q0, uint32_t q1, uint32_t key) const {
        const uint32_t nch = (q1 - q0 + LR_CHUNK - 1) / LR_CHUNK;
        const uint32_t j = atomicAdd(nrun, 1u);
        const uint32_t cb = atomicAdd(nchunk, nch);
        runs[4 * (uint64_t)j] = q0;
        runs[4 * (uint64_t)j + 1] = q1;
        runs[4 * (uint64_t)j + 2] = key;
        runs[4 * (uint64_t)j + 3] = cb;
        for (uint32_t c = 0; c < nch; ++c) chunk_run[cb + c] = j;
    }
};
// capacities for a batch of n events whose runs are all longer than min_run
inline size_t long_runs_cap(int64_t n, uint32_t min_run) { return (size_t)n / min_run + 2; }
inline size_t long_chunks_cap(int64_t n, uint32_t min_run) {
    return (size_t)n / LR_CHUNK + long_runs_cap(n, min_run) + 1;
}

// Keys with more events than this and a heterogeneous-acquire segment (but not hot enough for the
// workgroup kernels) are walked by one wave each (k_process_wave): {count, first segment of each key}.
constexpr uint32_t WAVE_HET_RUN = 48;
struct WaveRuns {
    uint32_t *n;
    uint32_t *g0;
};

template <int NMAX>
__device__ __forceinline__ void process_reg_body(KeyTable T, BatchWork W, EventSrc src, Verdicts V, int64_t n,
                                                 LongRuns L, WaveRuns WR, uint32_t hot_run, uint32_t *het_hint) {
    const int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)*W.nseg;
    if (g0 >= S || (int64_t)*W.nvalid == 0) return;
    const uint32_t key = W.seg_key[g0];
    if (g0 > 0 && W.seg_key[g0 - 1] == key) return;    // not the first segment of its key
    if (L.nrun || het_hint) {
        int64_t ge = g0;
        bool het = false;
        for (; ge < S && W.seg_key[ge] == key; ++ge) het |= W.seg_het[ge] && !W.seg_prio[ge];
        const uint32_t q0 = W.seg_start[g0], q1 = W.seg_start[ge];
        if (!L.nrun) {           // deferral off this batch: ask for it (pinned host word) if it would pay
            if (het && q1 - q0 > WAVE_HET_RUN)
                __hip_atomic_store(het_hint, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else if (het && q1 - q0 > hot_run) {
            L.push(q0, q1, key);
            for (int64_t g = g0; g < ge; ++g) W.seg_done[g] = 1;
            return;
        }
        if (het && WR.n && q1 - q0 > WAVE_HET_RUN) {
            WR.g0[atomicAdd(WR.n, 1u)] = (uint32_t)g0;
            return;
        }
    }
    const KeyState ks = key_state(T, key);
    const int nsc = ks.n;
    const uint8_t kind = T.kind[key];
    const double thr = T.thr[key];
    const double I_s = T.I_s[key];
    int64_t ep[NMAX], ps[NMAX];
    uint32_t dirty = 0;
    if (T.hblock || T.state_stride >= 2 * NMAX) {
        // every slot has room for NMAX pairs (blocked flow headers, bucketed param / limiter strides):
        // the header loads go out with the key's n instead of waiting for it
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
            const longlong2 v = *reinterpret_cast<const longlong2 *>(ks.pair(j));
            ep[j] = v.x;
            ps[j] = v.y;
        }
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (j >= nsc) { ep[j] = EPOCH_ABSENT; ps[j] = 0; }
    } else {
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
            if (j < nsc) {
                const longlong2 v = *reinterpret_cast<const longlong2 *>(ks.pair(j));
                ep[j] = v.x;
                ps[j] = v.y;
            } else {
                ep[j] = EPOCH_ABSENT;
                ps[j] = 0;
            }
        }
    }
    bool occ_pending = ks.seven && kind == KIND_CLUSTER && T.has_occ[key];
    for (int64_t g = g0; g < S; ++g) {
        if (g > g0 && W.seg_key[g] != key) break;
        const uint32_t st = W.seg_start[g];
        const uint32_t len = W.seg_start[g + 1] - st;
        const int64_t E = W.seg_epoch[g];
        bool slow = W.seg_prio[g] || occ_pending;
#pragma unroll
        for (int j = 0; j < NMAX; ++j) slow |= (ep[j] != EPOCH_ABSENT && ep[j] > E);
        if (!slow && W.seg_het[g]) {          // heterogeneous acquire counts: the register walk
            const int slot = (int)(E % nsc);
            bool fresh = false;
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (j == slot && ep[j] != E) { fresh = true; ep[j] = E; ps[j] = 0; }
            int64_t s0 = 0;
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (ep[j] != EPOCH_ABSENT && ep[j] > E - nsc) s0 = wrap_add(s0, ps[j]);
            const int64_t T0 = src.t0();
            const HetSums hs = het_walk<16>(
                kind, thr, I_s, s0, len, [&](uint32_t k) { return W.sval[st + k]; },
                [&](uint64_t v) {
                    int64_t t;
                    int32_t a;
                    bool pr;
                    src.unpack(v, T0, t, a, pr);
                    return a;
                },
                [&](uint32_t k, uint64_t v, uint64_t vd) { V.put(st + k, v, vd); });
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (j == slot) { ps[j] = wrap_add(ps[j], hs.pass); dirty |= 1u << j; }
            if (ks.seven) {
                int64_t blk = 0, preq = 0, breq = 0;
                if (!fresh) { blk = ks.rc(slot, 0); preq = ks.rc(slot, 1); breq = ks.rc(slot, 2); }
                ks.book_rest_sums(slot, fresh, blk, preq, breq, hs.block, hs.npass, hs.nblock);
            }
            W.seg_done[g] = 1;
            continue;
        }
        if (slow || W.seg_het[g]) {
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (dirty & (1u << j)) *reinterpret_cast<longlong2 *>(ks.pair(j)) = longlong2{ep[j], ps[j]};
            dirty = 0;
            for (uint32_t i = st; i < st + len; ++i) {
                const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
                int64_t t;
                int32_t a;
                uint8_t fl;
                src.load(seq, t, a, fl);
                seq_event(T, key, ks, E, a, fl, seq, V, V.oseq ? V.obase + i : seq);
            }
            W.seg_done[g] = 1;
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (j < nsc) { ep[j] = ks.ep(j); ps[j] = ks.cnt(EV_PASS, j); }
            // the sequential path may have left an occupy transfer pending
            occ_pending = ks.seven && kind == KIND_CLUSTER && T.has_occ[key];
            continue;
        }
        const int32_t a = W.seg_acq[g];
        const int slot = (int)(E % nsc);
        bool fresh = false;
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (j == slot && ep[j] != E) { fresh = true; ep[j] = E; ps[j] = 0; }
        int64_t s0 = 0;
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (ep[j] != EPOCH_ABSENT && ep[j] > E - nsc) s0 = wrap_add(s0, ps[j]);
        uint32_t lo = 0, hi = len;                      // K = first p with !admits(S0 + p*a)
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (admits(kind, thr, I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) lo = mid + 1;
            else hi = mid;
        }
        const uint32_t K = lo;
        const int64_t nb = (int64_t)(len - K);
#pragma unroll
        for (int j = 0; j < NMAX; ++j)
            if (j == slot) { ps[j] = wrap_add(ps[j], wrap_mul((int64_t)K, a)); dirty |= 1u << j; }
        if (ks.seven) {
            int64_t blk = 0, preq = 0, breq = 0;
            if (!fresh) { blk = ks.rc(slot, 0); preq = ks.rc(slot, 1); breq = ks.rc(slot, 2); }
            ks.book_rest(slot, fresh, blk, preq, breq, nb, a, K);
        }
        W.seg_s0[g] = s0;
        W.seg_k[g] = K;
        W.seg_done[g] = 0;
    }
#pragma unroll
    for (int j = 0; j < NMAX; ++j)
        if (dirty & (1u << j)) *reinterpret_cast<longlong2 *>(ks.pair(j)) = longlong2{ep[j], ps[j]};
}

template <int NMAX>
__global__ __launch_bounds__(256) void k_process_reg(KeyTable T, BatchWork W, EventSrc src, Verdicts V, int64_t n,
                                                     LongRuns L = LongRuns{}, WaveRuns WR = WaveRuns{},
                                                     uint32_t hot_run = HOT_HET_RUN, uint32_t *het_hint = nullptr) {
    process_reg_body<NMAX>(T, W, src, V, n, L, WR, hot_run, het_hint);
}

// The same kernel held to <= 128 VGPRs (4 waves per SIMD, some spills): the param tables' millions of
// short keys are latency-bound on their window and segment-record loads, where occupancy beats
// spill-free code (config 4: 1032 -> 845 us; a separate low-register kernel for one-segment keys
// measured slower overall, `profiles/r02_param4`).
template <int NMAX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_process_reg_o4(
    KeyTable T, BatchWork W, EventSrc src, Verdicts V, int64_t n, LongRuns L = LongRuns{}, WaveRuns WR = WaveRuns{},
    uint32_t hot_run = HOT_HET_RUN, uint32_t *het_hint = nullptr) {
    process_reg_body<NMAX>(T, W, src, V, n, L, WR, hot_run, het_hint);
}


// Wave-wide greedy walk (k_process_wave, and coop_het past its first failure): events i in [0, len),
// 64 at a time, one per lane (load(i) -> the raw value, issued one window ahead; decode(i, raw, a,
// dst)), decided as het_walk would, in rounds that each settle at least one event (wave scans and
// ballots, no barriers):
//   P: lanes >= cur pass while admits(x + their exclusive acquire prefix): first failing lane f;
//   S: f blocked; the next pass is the first lane c > f with admits(x, a_c) (x does not grow until
//      then, admits is monotone in x); (f, c) blocked, c passes.
// Stops where not even an acquire of 1 is admitted any more and returns that index (len if never):
// every event from there on is blocked, which the caller writes with all its lanes.  x, npass and acq
// (the acquire sum of the events decided here) are updated in every lane.
template <class Load, class Decode>
__device__ inline uint32_t wave_walk(uint8_t kind, double thr, double I_s, uint32_t len, int64_t &x, int64_t &npass,
                                     int64_t &acq, Load load, Decode decode) {
    const uint32_t lane = lane_id();
    uint64_t raw = lane < len ? load(lane) : 0ull;
    for (uint32_t c0 = 0; c0 < len; c0 += WAVE) {
        const uint32_t cnt = min((uint32_t)WAVE, len - c0);
        const bool valid = lane < cnt;
        const uint64_t cur_raw = raw;
        raw = c0 + WAVE + lane < len ? load(c0 + WAVE + lane) : 0ull;     // next window in flight
        int32_t a = 0;
        uint64_t *dst = nullptr;
        if (valid) decode(c0 + lane, cur_raw, a, dst);
        uint32_t cur = 0;
        while (cur < cnt) {
            if (!admits(kind, thr, I_s, x, 1)) {
                int64_t sa = lane < cur ? (int64_t)a : 0;
#pragma unroll
                for (int off = 1; off < WAVE; off <<= 1) sa += __shfl_xor(sa, off, WAVE);
                acq = wrap_add(acq, sa);
                return c0 + cur;
            }
            // P round
            const int64_t m = (valid && lane >= cur) ? (int64_t)a : 0;
            int64_t inc = m;
#pragma unroll
            for (int off = 1; off < WAVE; off <<= 1) {
                const int64_t u = __shfl_up(inc, off, WAVE);
                if ((int)lane >= off) inc += u;
            }
            const int64_t pre = inc - m;
            const bool fail = valid && lane >= cur && !admits(kind, thr, I_s, wrap_add(x, pre), a);
            const unsigned long long fm = __ballot(fail);
            const uint32_t f = fm ? (uint32_t)__ffsll((long long)fm) - 1 : cnt;
            if (valid && lane >= cur && lane < f)
                *dst = pack_verdict(ST_OK, java_d2i(remaining_of(thr, I_s, wrap_add(x, pre), a)), 0);
            npass += (int64_t)(f - cur);
            if (f >= cnt) {
                x = wrap_add(x, __shfl(inc, (int)cnt - 1, WAVE));
                break;
            }
            x = wrap_add(x, __shfl(pre, (int)f, WAVE));
            // S round
            const bool cand = valid && lane > f && admits(kind, thr, I_s, x, a);
            const unsigned long long cm = __ballot(cand);
            const uint32_t c = cm ? (uint32_t)__ffsll((long long)cm) - 1 : cnt;
            if (valid && lane >= f && lane < c) *dst = pack_verdict(ST_BLOCKED, 0, 0);
            if (lane == c && c < cnt) *dst = pack_verdict(ST_OK, java_d2i(remaining_of(thr, I_s, x, a)), 0);
            if (c >= cnt) break;
            x = wrap_add(x, (int64_t)__shfl(a, (int)c, WAVE));
            npass += 1;
            cur = c + 1;
        }
        int64_t sa = a;
#pragma unroll
        for (int off = 1; off < WAVE; off <<= 1) sa += __shfl_xor(sa, off, WAVE);
        acq = wrap_add(acq, sa);
    }
    return len;
}

// A heterogeneous segment [st, st + len) of the sorted values, walked by one wave.
__device__ inline HetSums wave_het(uint8_t kind, double thr, double I_s, int64_t x, const uint64_t *sval, uint32_t st,
                                   uint32_t len, const EventSrc &src, int64_t T0, const Verdicts &V) {
    const uint32_t lane = lane_id();
    const int64_t x0 = x;
    int64_t npass = 0;
    auto decode = [&](uint32_t i, uint64_t v, int32_t &a, uint64_t *&dst) {
        int64_t t;
        bool pr;
        src.unpack(v, T0, t, a, pr);
        dst = V.out + V.at(st + i, v);
    };
    int64_t tot = 0;
    const uint32_t dpos = wave_walk(kind, thr, I_s, len, x, npass, tot, [&](uint32_t i) { return sval[st + i]; }, decode);
    // the blocked tail, 8 windows of loads in flight (its acquires complete the BLOCK sum)
    int64_t tail = 0;
    for (uint32_t i0 = dpos; i0 < len; i0 += 8 * WAVE) {
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = i0 + k * WAVE + lane < len ? sval[st + i0 + k * WAVE + lane] : 0ull;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (i0 + k * WAVE + lane < len) {
                int64_t t;
                int32_t a;
                bool pr;
                src.unpack(v[k], T0, t, a, pr);
                tail += a;
                V.put(st + i0 + k * WAVE + lane, v[k], pack_verdict(ST_BLOCKED, 0, 0));
            }
    }
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) tail += __shfl_xor(tail, off, WAVE);
    tot = wrap_add(tot, tail);
    HetSums h;
    h.pass = wrap_add(x, -x0);
    h.npass = npass;
    h.block = wrap_add(tot, -h.pass);
    h.nblock = (int64_t)len - npass;
    return h;
}

// One wave per key of the wave list (k_process_reg's keys of WAVE_HET_RUN..HOT_HET_RUN events with a
// heterogeneous segment): the key's segments in order, the window header in every lane's VGPRs (the
// same values: uniform), memory written by lane 0.  Closed-form segments leave {s0, K} for
// k_verdict; heterogeneous ones are decided by wave_het; prioritized / pending-occupy / clock-went-
// back ones take the sequential path in lane 0, after which every lane re-reads the header.
template <int NMAX>
__global__ __launch_bounds__(256) void k_process_wave(KeyTable T, BatchWork W, EventSrc src, Verdicts V, WaveRuns WR,
                                                      const uint32_t *nrun, uint32_t *het_hint) {
    const uint32_t total = *WR.n;
    // keep the deferral on for the next batch only while batches have heterogeneous keys to defer
    if (het_hint && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(het_hint, (total || *nrun) ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t lane = lane_id();
    const int64_t T0 = src.t0();
    for (uint32_t wi = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE; wi < total;
         wi += gridDim.x * blockDim.x / WAVE) {
        const int64_t S = (int64_t)*W.nseg;
        const int64_t g0 = WR.g0[wi];
        const uint32_t key = W.seg_key[g0];
        const KeyState ks = key_state(T, key);
        const int nsc = ks.n;
        const uint8_t kind = T.kind[key];
        const double thr = T.thr[key];
        const double I_s = T.I_s[key];
        int64_t ep[NMAX], ps[NMAX];
        uint32_t dirty = 0;
#pragma unroll
        for (int j = 0; j < NMAX; ++j) {
            if (j < nsc) {
                const longlong2 v = *reinterpret_cast<const longlong2 *>(ks.pair(j));
                ep[j] = v.x;
                ps[j] = v.y;
            } else {
                ep[j] = EPOCH_ABSENT;
                ps[j] = 0;
            }
        }
        bool occ_pending = ks.seven && kind == KIND_CLUSTER && T.has_occ[key];
        for (int64_t g = g0; g < S && W.seg_key[g] == key; ++g) {
            const uint32_t st = W.seg_start[g];
            const uint32_t len = W.seg_start[g + 1] - st;
            const int64_t E = W.seg_epoch[g];
            bool slow = W.seg_prio[g] || occ_pending;
#pragma unroll
            for (int j = 0; j < NMAX; ++j) slow |= (ep[j] != EPOCH_ABSENT && ep[j] > E);
            if (slow) {
                if (lane == 0) {
#pragma unroll
                    for (int j = 0; j < NMAX; ++j)
                        if (dirty & (1u << j)) *reinterpret_cast<longlong2 *>(ks.pair(j)) = longlong2{ep[j], ps[j]};
                    for (uint32_t i = st; i < st + len; ++i) {
                        const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
                        int64_t t;
                        int32_t a;
                        uint8_t fl;
                        src.load(seq, t, a, fl);
                        seq_event(T, key, ks, E, a, fl, seq, V, V.oseq ? V.obase + i : seq);
                    }
                    W.seg_done[g] = 1;
#pragma unroll
                    for (int j = 0; j < NMAX; ++j)
                        if (j < nsc) { ep[j] = ks.ep(j); ps[j] = ks.cnt(EV_PASS, j); }
                    occ_pending = ks.seven && kind == KIND_CLUSTER && T.has_occ[key];
                }
                dirty = 0;
#pragma unroll
                for (int j = 0; j < NMAX; ++j) {
                    ep[j] = __shfl(ep[j], 0, WAVE);
                    ps[j] = __shfl(ps[j], 0, WAVE);
                }
                occ_pending = __shfl((int)occ_pending, 0, WAVE) != 0;
                continue;
            }
            const int slot = (int)(E % nsc);
            bool fresh = false;
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (j == slot && ep[j] != E) { fresh = true; ep[j] = E; ps[j] = 0; }
            int64_t s0 = 0;
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (ep[j] != EPOCH_ABSENT && ep[j] > E - nsc) s0 = wrap_add(s0, ps[j]);
            int64_t blk = 0, preq = 0, breq = 0;
            if (ks.seven && !fresh) { blk = ks.rc(slot, 0); preq = ks.rc(slot, 1); breq = ks.rc(slot, 2); }
            if (W.seg_het[g]) {
                const HetSums hs = wave_het(kind, thr, I_s, s0, W.sval, st, len, src, T0, V);
#pragma unroll
                for (int j = 0; j < NMAX; ++j)
                    if (j == slot) { ps[j] = wrap_add(ps[j], hs.pass); dirty |= 1u << j; }
                if (lane == 0) {
                    if (ks.seven) ks.book_rest_sums(slot, fresh, blk, preq, breq, hs.block, hs.npass, hs.nblock);
                    W.seg_done[g] = 1;
                }
                continue;
            }
            const int32_t a = W.seg_acq[g];
            uint32_t lo = 0, hi = len;                      // K = first p with !admits(S0 + p*a)
            while (lo < hi) {
                const uint32_t mid = lo + (hi - lo) / 2;
                if (admits(kind, thr, I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) lo = mid + 1;
                else hi = mid;
            }
            const uint32_t K = lo;
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (j == slot) { ps[j] = wrap_add(ps[j], wrap_mul((int64_t)K, a)); dirty |= 1u << j; }
            if (lane == 0) {
                if (ks.seven) ks.book_rest(slot, fresh, blk, preq, breq, (int64_t)(len - K), a, K);
                W.seg_s0[g] = s0;
                W.seg_k[g] = K;
                W.seg_done[g] = 0;
            }
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < NMAX; ++j)
                if (dirty & (1u << j)) *reinterpret_cast<longlong2 *>(ks.pair(j)) = longlong2{ep[j], ps[j]};
        }
    }
}

// K1+K3 with a lane group per key (G lanes, up to PROC_SLOTS_PER_LANE slots per lane, so
// n <= G * PROC_SLOTS_PER_LANE): the header {epoch, pass} pairs of one key are read by the group
// with coalesced 16-byte loads, the window sum is a group reduction, and only the rolled slot is
// written back.  Segments that are heterogeneous, prioritized, behind the key's newest epoch or
// carry a pending occupy transfer run the sequential path on lane 0 of the group.
constexpr int PROC_G = 16;
constexpr int PROC_SLOTS_PER_LANE = 4;

__device__ inline int64_t group_sum(int64_t v) {
#pragma unroll
    for (int m = PROC_G / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, PROC_G);
    return v;
}

__device__ inline bool group_any(bool p) {
    int v = p ? 1 : 0;
#pragma unroll
    for (int m = PROC_G / 2; m >= 1; m >>= 1) v |= __shfl_xor(v, m, PROC_G);
    return v != 0;
}

__device__ inline void process_key_group(const KeyTable &T, const BatchWork &W, const EventSrc &src,
                                         const Verdicts &V, int64_t g0, int64_t S, int lg) {
    const uint32_t key = W.seg_key[g0];
    const KeyState ks = key_state(T, key);
    const int nsc = ks.n;
    const uint8_t kind = T.kind[key];
    const double thr = T.thr[key];
    const double I_s = T.I_s[key];
    int64_t ep[PROC_SLOTS_PER_LANE], ps[PROC_SLOTS_PER_LANE];
    bool dirty[PROC_SLOTS_PER_LANE];
#pragma unroll
    for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q) {
        const int j = lg + PROC_G * q;
        dirty[q] = false;
        if (j < nsc) {
            ep[q] = ks.ep(j);
            ps[q] = ks.cnt(EV_PASS, j);
        } else {
            ep[q] = EPOCH_ABSENT;
            ps[q] = 0;
        }
    }
    for (int64_t g = g0; g < S; ++g) {
        if (g > g0 && W.seg_key[g] != key) break;
        const uint32_t st = W.seg_start[g];
        const uint32_t len = W.seg_start[g + 1] - st;
        const int64_t E = W.seg_epoch[g];
        bool fut = false;
#pragma unroll
        for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q) fut |= (ep[q] != EPOCH_ABSENT && ep[q] > E);
        bool slow = W.seg_het[g] || group_any(fut);
        if (!slow && ks.seven && kind == KIND_CLUSTER && T.has_occ[key]) slow = true;
        if (slow) {
#pragma unroll
            for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q) {
                const int j = lg + PROC_G * q;
                if (dirty[q]) { ks.ep(j) = ep[q]; ks.cnt(EV_PASS, j) = ps[q]; dirty[q] = false; }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            if (lg == 0) {
                for (uint32_t i = st; i < st + len; ++i) {
                    const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
                    int64_t t;
                    int32_t a;
                    uint8_t fl;
                    src.load(seq, t, a, fl);
                    seq_event(T, key, ks, E, a, fl, seq, V, V.oseq ? V.obase + i : seq);
                }
                W.seg_done[g] = 1;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#pragma unroll
            for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q) {
                const int j = lg + PROC_G * q;
                if (j < nsc) { ep[q] = ks.ep(j); ps[q] = ks.cnt(EV_PASS, j); }
            }
            continue;
        }
        const int32_t a = W.seg_acq[g];
        const int slot = (int)(E % nsc);
        const int owner = slot % PROC_G;
        const int qs = slot / PROC_G;
        int64_t cur = EPOCH_ABSENT;
#pragma unroll
        for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q) if (q == qs) cur = ep[q];
        cur = __shfl(cur, owner, PROC_G);
        if (cur != E) {                                            // NEW or RESET: fresh bucket
            if (lg == owner) {
#pragma unroll
                for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q) if (q == qs) { ep[q] = E; ps[q] = 0; dirty[q] = true; }
            }
            if (ks.seven && lg < 6) ks.rc(slot, lg) = 0;
        }
        int64_t part = 0;
#pragma unroll
        for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q)
            if (ep[q] != EPOCH_ABSENT && ep[q] > E - nsc) part = wrap_add(part, ps[q]);
        const int64_t s0 = group_sum(part);
        uint32_t lo = 0, hi = len;                      // K = first p with !admits(S0 + p*a)
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (admits(kind, thr, I_s, wrap_add(s0, wrap_mul((int64_t)mid, a)), a)) lo = mid + 1;
            else hi = mid;
        }
        const uint32_t K = lo;
        const int64_t nb = (int64_t)(len - K);
        if (lg == owner) {
#pragma unroll
            for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q)
                if (q == qs) { ps[q] = wrap_add(ps[q], wrap_mul((int64_t)K, a)); dirty[q] = true; }
        }
        if (ks.seven) {
            if (lg == EV_PASS_REQUEST - 1) ks.rc(slot, lg) = wrap_add(ks.rc(slot, lg), (int64_t)K);
            else if (lg == EV_BLOCK - 1) ks.rc(slot, lg) = wrap_add(ks.rc(slot, lg), wrap_mul(nb, a));
            else if (lg == EV_BLOCK_REQUEST - 1) ks.rc(slot, lg) = wrap_add(ks.rc(slot, lg), nb);
        }
        if (lg == 0) {
            W.seg_s0[g] = s0;
            W.seg_k[g] = K;
            W.seg_done[g] = 0;
        }
    }
#pragma unroll
    for (int q = 0; q < PROC_SLOTS_PER_LANE; ++q) {
        const int j = lg + PROC_G * q;
        if (dirty[q]) { ks.ep(j) = ep[q]; ks.cnt(EV_PASS, j) = ps[q]; }
    }
}

// Grid-stride over segments: a group takes segment g0 when it starts its key's run.
__global__ __launch_bounds__(256) void k_process_grp(KeyTable T, BatchWork W, EventSrc src, Verdicts V, int64_t n) {
    const int lg = threadIdx.x % PROC_G;
    const int64_t S = (int64_t)*W.nseg;
    if (*W.nvalid == 0) return;
    const int64_t ngroups = (int64_t)gridDim.x * (blockDim.x / PROC_G);
    for (int64_t g0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / PROC_G; g0 < S; g0 += ngroups) {
        if (g0 > 0 && W.seg_key[g0 - 1] == W.seg_key[g0]) continue;   // group-uniform
        process_key_group(T, W, src, V, g0, S, lg);
    }
}

// Per sorted event: rank inside its segment decides; scatter the verdict to its arrival slot.
template <bool LIMITER, bool NT, bool LINEAR = false>
__global__ __launch_bounds__(256) void k_verdict(KeyTable T, BatchWork W, Verdicts V, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t nv = (int64_t)*W.nvalid;
    if (i >= nv) return;
    const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
    if (V.oseq) V.oseq[i] = seq;                   // decide-order output: every sorted position's arrival position
    const uint32_t g = W.segid[i] - 1;
    if (W.seg_done[g]) return;
    const uint32_t rank = (uint32_t)i - W.seg_start[g];
    const uint32_t K = W.seg_k[g];
    const uint32_t key = W.seg_key[g];
    if (LIMITER) {
        if (rank >= K) reject_limited(V, seq, seq);
        return;
    }
    uint64_t v;
    if (rank < K) {
        const int32_t a = W.seg_acq[g];
        const int64_t x = wrap_add(W.seg_s0[g], wrap_mul((int64_t)rank, a));
        v = pack_verdict(ST_OK, java_d2i(remaining_of(T.thr[key], T.I_s[key], x, a)), 0);
    } else {
        v = pack_verdict(ST_BLOCKED, 0, 0);
    }
    if (LINEAR || V.oseq) V.out[i] = v;  // decide-order output (LINEAR: the old diagnostic of the same stores)
    else if (NT) __builtin_nontemporal_store(v, V.out + seq);
    else V.out[seq] = v;
}

}  // namespace sentinel
