// param_table.hpp -- the exact hot-parameter slot table, kept bounded (gfx950).
//
// One open-addressing slot per (rule, value) key holds the value's window {epoch, count} x n: the
// value's entries in the buckets of ClusterParamMetric's leap array (ClusterParamMetric.java:46-82,
// ClusterParameterLeapArray.java:33-49; one CacheMap<value, LongAdder> per bucket).  The host never
// lets the table fill up: before a batch whose values could exceed 3/4 of the capacity it rebuilds
// the table (engine.hip, sentinel_engine::param_reserve), which
//   * drops dead slots: a slot none of whose buckets can be valid again -- every epoch <= E_r - n,
//     E_r = the newest epoch of any slot of its rule (every request of rule r rolls its values'
//     slots to the request's epoch, so E_r = epoch of the rule's latest timestamp) -- reads exactly
//     like a value with no CacheMap entry (the reference's bucket reset clears the whole map,
//     CPLA:40-49), given per-rule non-decreasing timestamps (the documented precondition of exact
//     param parity);
//   * grows the table when the live slots alone would still exceed the bound;
//   * carries a rule reload (ClusterParamMetricStatistics.putMetricIfAbsent, ClusterParamFlowRuleManager
//     .java:355-356): slots of surviving rules move to the rule's new index, slots of removed rules
//     go, slots of orphaned rules (emptied namespace list) are exported to the host and imported back
//     if the flowId returns.
// getTopValues (ClusterParamMetric.java:84-127) for the ClusterMetricNode snapshot is a selection
// over the live slots of each rule (k_ptop_*).
#pragma once

#include "admission.hpp"

namespace sentinel {

struct PSlots {
    unsigned long long *keys;   // PKEY_EMPTY = free
    int32_t *rule;              // dense param rule index of the slot
    int64_t *state;             // stride words per slot: {epoch, count} x n
    int64_t stride;
    uint64_t mask;              // capacity - 1
    // getTopValues hint (round 5): per slot the 1024-ms bucket from which its window sums to zero,
    // ceil((newest epoch + n) * w / 1024) (0: nothing counted), written by the key walk (pd_walk); null
    // when the engine does not keep it
    uint32_t *expire = nullptr;
};

// A window whose newest epoch is e sums to zero at every ts >= (e + n) w: every bucket's epoch is then
// <= E - n (E = ts / w).  Kept in 1024-ms units, rounded up (so a slot is only ever skipped late).
__host__ __device__ inline uint32_t slot_expire_c(int64_t newest, int n, int32_t w) {
    if (newest == EPOCH_ABSENT) return 0u;
    const int64_t t = (newest + (int64_t)n) * (int64_t)w;
    if (t <= 0) return 0u;
    const int64_t c = (t + 1023) >> 10;
    return c >= (int64_t)0xFFFFFFFF ? 0xFFFFFFFFu : (uint32_t)c;
}

// Insert a key known to be absent (a rebuild re-inserts unique keys): linear probing.
__device__ inline int64_t slot_place(unsigned long long *keys, uint64_t mask, uint64_t key) {
    uint64_t h = mix64(key) & mask;
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        if (atomicCAS(&keys[h], (unsigned long long)PKEY_EMPTY, (unsigned long long)key) == PKEY_EMPTY) return (int64_t)h;
        h = (h + 1) & mask;
    }
    return -1;
}

__device__ inline int64_t slot_newest(const int64_t *st, int n) {
    int64_t m = EPOCH_ABSENT;
    for (int j = 0; j < n; ++j) m = st[2 * j] > m ? st[2 * j] : m;
    return m;
}

// Every slot's expire hint from its window (the rebuild moved slots, or a path other than the key
// walk wrote windows since the last snapshot).
__global__ __launch_bounds__(256) void k_ptable_expire(PSlots T, uint64_t cap, int32_t R, const int32_t *__restrict__ rn,
                                                       const int32_t *__restrict__ rw) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= cap) return;
    uint32_t x = 0;
    if (T.keys[s] != PKEY_EMPTY && (uint32_t)T.rule[s] < (uint32_t)R) {
        const int32_t r = T.rule[s];
        x = slot_expire_c(slot_newest(T.state + (int64_t)s * T.stride, rn[r]), rn[r], rw[r]);
    }
    T.expire[s] = x;
}

// Per rule: the newest epoch over its live slots (wave-aggregated when a wave's slots share a rule).
__global__ __launch_bounds__(256) void k_ptable_rule_newest(PSlots T, uint64_t cap, int32_t R,
                                                            const int32_t *__restrict__ rn,
                                                            unsigned long long *__restrict__ newest) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool live = false;
    int32_t r = 0;
    int64_t e = EPOCH_ABSENT;
    if (s < cap && T.keys[s] != PKEY_EMPTY && (uint32_t)T.rule[s] < (uint32_t)R) {
        r = T.rule[s];
        e = slot_newest(T.state + (int64_t)s * T.stride, rn[r]);
        live = e != EPOCH_ABSENT;
    }
    const uint64_t act = __builtin_amdgcn_ballot_w64(live);
    if (!act) return;
    const int first = __ffsll((unsigned long long)act) - 1;
    const int32_t r0 = __shfl(r, first, WAVE);
    const uint64_t same = __builtin_amdgcn_ballot_w64(live && r == r0);
    if (same == act) {                                    // one rule in the wave: reduce, one atomic
        int64_t m = live ? e : EPOCH_ABSENT;
#pragma unroll
        for (int o = WAVE / 2; o >= 1; o >>= 1) {
            const int64_t x = __shfl_xor(m, o, WAVE);
            m = x > m ? x : m;
        }
        if ((int)lane_id() == first) atomicMax(&newest[r0], (unsigned long long)(m + 1));
    } else if (live) {
        atomicMax(&newest[r], (unsigned long long)(e + 1));
    }
}

// Rebuild: every live slot of the old table whose rule survives (rmap[r] >= 0) and which is not dead
// moves to the new table (pre-initialised: keys free, state absent) under rule rmap[r]; rmap[r] == -2
// exports the slot (key, old rule, 2n state words) to `xout` (xcount counts them); -1 drops it.
// newest[r] - 1 = the rule's newest epoch (0: never seen -> nothing is dead).
__global__ __launch_bounds__(256) void k_ptable_rebuild(PSlots O, uint64_t ocap, int32_t OR, const int32_t *__restrict__ rmap,
                                                        const int32_t *__restrict__ orn,
                                                        const unsigned long long *__restrict__ newest, PSlots N,
                                                        unsigned long long *__restrict__ live,
                                                        int64_t *__restrict__ xout, int64_t xstride,
                                                        unsigned long long *__restrict__ xcount, uint64_t xcap) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ocap) return;
    const unsigned long long key = O.keys[s];
    if (key == PKEY_EMPTY) return;
    const int32_t r = O.rule[s];
    if ((uint32_t)r >= (uint32_t)OR) return;                 // never: every live slot has its rule
    const int32_t m = rmap[r];
    if (m == -1) return;
    const int n = orn[r];
    const int64_t *st = O.state + (int64_t)s * O.stride;
    if (m == -2) {
        const unsigned long long k = atomicAdd(xcount, 1ull);
        if (k >= xcap) return;
        int64_t *x = xout + (int64_t)k * xstride;
        x[0] = (int64_t)key;
        x[1] = r;
        for (int j = 0; j < 2 * n; ++j) x[2 + j] = st[j];
        return;
    }
    const int64_t E = (int64_t)newest[r] - 1;
    if (newest[r] != 0) {
        bool valid = false;
        for (int j = 0; j < n; ++j) valid |= st[2 * j] != EPOCH_ABSENT && st[2 * j] > E - n;
        if (!valid) return;                               // dead: reads like an absent value
    }
    const int64_t h = slot_place(N.keys, N.mask, key);
    if (h < 0) return;                                    // cannot happen: the new table has room
    int64_t *d = N.state + h * N.stride;
    for (int j = 0; j < 2 * n; ++j) d[j] = st[j];
    N.rule[h] = m;
    atomicAdd(live, 1ull);
}

// Import exported slots (k_ptable_rebuild's record format) under rule rule_of[k].
__global__ __launch_bounds__(256) void k_ptable_import(const int64_t *__restrict__ x, int64_t xstride, int64_t K,
                                                       const int32_t *__restrict__ rule_of, const int32_t *__restrict__ nn,
                                                       PSlots N, unsigned long long *__restrict__ live) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const int64_t *r = x + k * xstride;
    const int32_t rule = rule_of[k];
    const int64_t h = slot_place(N.keys, N.mask, (uint64_t)r[0]);
    if (h < 0) return;
    const int n = nn[rule];
    int64_t *d = N.state + h * N.stride;
    for (int j = 0; j < 2 * n; ++j) d[j] = r[2 + j];
    N.rule[h] = rule;
    atomicAdd(live, 1ull);
}

// ---------------------------------------------------------------- getTopValues (snapshot)
// Per live slot at time ts: the value's window sum over its valid buckets (a read-only view equals
// the sum after currentWindow(): the roll only empties an invalid bucket), and (int) of it, the
// reference's sort key ((int) b - (int) a, ClusterParamMetric.java:107-113).  Values with no count
// have no CacheMap entry in the reference and are not candidates: only slots with a non-zero sum are
// appended (wave-aggregated) to a compact candidate list {key, rule, sum}, and the selection rounds run
// over that list instead of the whole table.
struct TopCands {
    unsigned long long *key;
    int32_t *rule;
    int64_t *sum;
    unsigned long long *n;      // candidates found (may exceed cap: the caller retries with a larger list)
    unsigned long long cap;
};

__device__ inline uint64_t top_rank(int64_t v) { return ((uint64_t)1 << 32) | ((uint32_t)(int32_t)v ^ 0x80000000u); }

// Per rule the `number` largest ranks with multiplicity (0 = none), by an atomicMax cascade: a slot
// keeps the larger of its value and the incoming one and passes the smaller on, so slot j ends with the
// (j+1)-th largest rank of everything inserted.  A rank at or below the rule's last slot cannot change
// the multiset (a stale read of that slot is lower, so the test never skips a rank that belongs).
__device__ inline void top_cascade(unsigned long long *top, int number, unsigned long long v) {
    if (v <= top[number - 1]) return;
    for (int j = 0; j < number && v; ++j) {
        const unsigned long long o = atomicMax(&top[j], v);
        v = o < v ? o : v;
    }
}

// One wave per 64 consecutive slots.  A slot's {epoch, count} pairs lie in one contiguous run of the
// state region, so its window sum is read by a 16-lane group (lane j loads pair j, one 16-B load, then a
// 16-lane reduction): the wave's live slots go through four at a time, each load instruction reading
// four contiguous runs instead of 64 scattered ones.
constexpr uint32_t TOP_LDS = 1024;        // candidates a k_ptop_sums workgroup gathers before one global append

// The slots whose window can still sum to non-zero at ts (expire hint > ts in 1024-ms units), listed:
// a coalesced pass over the 4-B hints, the indices gathered in LDS, one append per TOP_LDS of them.
__global__ __launch_bounds__(256) void k_ptop_fresh(const uint32_t *__restrict__ expire, uint64_t cap, int64_t ts,
                                                    uint32_t *__restrict__ list, unsigned long long *__restrict__ list_n,
                                                    uint64_t list_cap) {
    __shared__ uint32_t s_idx[TOP_LDS];
    __shared__ uint32_t s_n;
    __shared__ unsigned long long s_base;
    const uint32_t t = threadIdx.x;
    const uint32_t lane = lane_id();
    if (t == 0) s_n = 0;
    __syncthreads();
    auto flush = [&] {                                    // (block-uniform, after a barrier)
        const uint32_t m = s_n;
        if (m == 0) return;
        if (t == 0) s_base = atomicAdd(list_n, (unsigned long long)m);
        __syncthreads();
        const unsigned long long b0 = s_base;
        for (uint32_t i = t; i < m; i += blockDim.x)
            if (b0 + i < list_cap) list[b0 + i] = s_idx[i];
        __syncthreads();
        if (t == 0) s_n = 0;
        __syncthreads();
    };
    const uint32_t uts = (uint32_t)((uint64_t)(ts < 0 ? 0 : ts) >> 10);
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + t; s - t < cap; s += (uint64_t)gridDim.x * blockDim.x) {
        const bool fresh = s < cap && expire[s] > uts;
        const uint64_t act = __builtin_amdgcn_ballot_w64(fresh);
        if (act) {
            const int first = __ffsll((unsigned long long)act) - 1;
            uint32_t wb = 0;
            if ((int)lane == first) wb = atomicAdd(&s_n, (uint32_t)__popcll(act));
            wb = __shfl(wb, first, WAVE);
            if (fresh) s_idx[wb + (uint32_t)__popcll(act & ((1ull << lane) - 1ull))] = (uint32_t)s;
        }
        __syncthreads();
        // every wave reads the count before any wave of the next iteration can add to it (a wave that
        // skipped the flush on a later read would disagree with the others about the flush's barriers)
        const uint32_t cur = s_n;
        __syncthreads();
        if (cur > TOP_LDS - blockDim.x) flush();
    }
    flush();
}

__global__ __launch_bounds__(256) void k_ptop_sums(PSlots T, uint64_t cap, int32_t R, const int32_t *__restrict__ rn,
                                                   const int32_t *__restrict__ rw, const double *__restrict__ rrcp,
                                                   int64_t ts, TopCands C, const uint32_t *__restrict__ list,
                                                   const unsigned long long *__restrict__ list_n, uint64_t list_cap) {
    // list (k_ptop_fresh): walk only the listed slots; else every slot (with the expire hint test)
    // candidates gathered in LDS and appended with one atomic per TOP_LDS of them: one atomic per wave on
    // the list's single counter queued at one memory channel (4.2 ms for ~1M waves at config 4)
    __shared__ unsigned long long s_key[TOP_LDS];
    __shared__ int32_t s_rule[TOP_LDS];
    __shared__ int64_t s_sum[TOP_LDS];
    __shared__ uint32_t s_n;
    __shared__ unsigned long long s_base;
    const uint32_t t = threadIdx.x;
    const uint32_t lane = lane_id();
    if (t == 0) s_n = 0;
    __syncthreads();
    auto flush = [&] {                                    // (block-uniform, after a barrier)
        const uint32_t m = s_n;
        if (m == 0) return;
        if (t == 0) s_base = atomicAdd(C.n, (unsigned long long)m);
        __syncthreads();
        const unsigned long long b0 = s_base;
        for (uint32_t i = t; i < m; i += blockDim.x)
            if (b0 + i < C.cap) {
                C.key[b0 + i] = s_key[i];
                C.rule[b0 + i] = s_rule[i];
                C.sum[b0 + i] = s_sum[i];
            }
        __syncthreads();
        if (t == 0) s_n = 0;
        __syncthreads();
    };
    const uint64_t uts = (uint64_t)(ts < 0 ? 0 : ts) >> 10;
    uint64_t nitems = cap;
    if (list) {
        nitems = *list_n;
        nitems = nitems < list_cap ? nitems : list_cap;
    }
    for (uint64_t chunk = blockIdx.x; chunk * blockDim.x < nitems; chunk += gridDim.x) {
        const uint64_t li = chunk * blockDim.x + t;
        const uint64_t s = li < nitems ? (list ? (uint64_t)list[li] : li) : cap;
        unsigned long long key = PKEY_EMPTY;
        int32_t r = -1;
        // with the expire hints only the slots whose window can still sum to non-zero at ts are read
        // (4 B per slot instead of the key and the whole window)
        const bool fresh = list || !T.expire || (s < cap && T.expire[s] > (uint32_t)uts);
        if (s < cap && fresh) key = T.keys[s];
        if (key != PKEY_EMPTY) {
            r = T.rule[s];
            if ((uint32_t)r >= (uint32_t)R) r = -1;
        }
        uint64_t live = __builtin_amdgcn_ballot_w64(r >= 0);
        const int grp = (int)(lane >> 4), j = (int)(lane & 15);
        uint64_t v = 0;                                   // this lane's slot's sum (wrapping, like wrap_add)
        while (live) {
            int pos[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                pos[q] = live ? __ffsll((unsigned long long)live) - 1 : -1;
                live &= live ? live - 1 : 0;
            }
            const int p = pos[grp];
            const int32_t rg = __shfl(r, p < 0 ? 0 : p, WAVE);
            const uint64_t sg = __shfl(s, p < 0 ? 0 : p, WAVE);
            uint64_t part = 0;
            if (p >= 0) {
                const int n = rn[rg];
                if (j < n) {
                    const int64_t E = epoch_of(ts, rw[rg], rrcp[rg]);
                    const longlong2 *run = (const longlong2 *)(T.state + (int64_t)sg * T.stride);
                    for (int jj = j; jj < n; jj += 16) {          // n > 16: lane j also sums pairs j + 16, ...
                        const longlong2 b = run[jj];
                        if (b.x != EPOCH_ABSENT && b.x > E - n) part += (uint64_t)b.y;
                    }
                }
            }
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) part += __shfl_xor(part, o, WAVE);     // within the 16-lane group
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t g = __shfl(part, q * 16, WAVE);
                if ((int)lane == pos[q]) v = g;
            }
        }
        const uint64_t act = __builtin_amdgcn_ballot_w64(v != 0);
        if (act) {
            const int first = __ffsll((unsigned long long)act) - 1;
            uint32_t wb = 0;
            if ((int)lane == first) wb = atomicAdd(&s_n, (uint32_t)__popcll(act));
            wb = __shfl(wb, first, WAVE);
            if (v != 0) {
                const uint32_t k = wb + (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
                s_key[k] = key;
                s_rule[k] = r;
                s_sum[k] = (int64_t)v;
            }
        }
        __syncthreads();
        const uint32_t cur = s_n;                         // (read by every wave before the next iteration's adds)
        __syncthreads();
        if (cur > TOP_LDS - blockDim.x) flush();          // (room for the next chunk's candidates)
    }
    flush();
}

// The rank cascade over a candidate list (when k_ptop_sums ran without it and the candidates are too
// many to run the selection rounds over all of them).
__global__ __launch_bounds__(256) void k_ptop_cascade(TopCands C, unsigned long long *__restrict__ toprank, int number) {
    const unsigned long long m = *C.n < C.cap ? *C.n : C.cap;
    for (unsigned long long k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x)
        top_cascade(toprank + (int64_t)C.rule[k] * number, number, top_rank(C.sum[k]));
}

// Order (int) sum descending, key ascending; `prev` = the rule's previous pick (none in round 0).

__device__ inline bool top_after(uint64_t rk, uint64_t key, uint64_t prk, uint64_t pkey) {
    return prk == 0 || rk < prk || (rk == prk && key > pkey);
}

// The finalists: candidates ranked at or above their rule's number-th largest rank (every other
// candidate has `number` better ones), appended to a short list F the selection rounds then run over
// (ties at that rank are kept, so the key order among them is decided by the rounds as before).
__global__ __launch_bounds__(256) void k_ptop_final(TopCands C, const unsigned long long *__restrict__ toprank, int number,
                                                    TopCands F) {
    const unsigned long long m = *C.n < C.cap ? *C.n : C.cap;
    for (unsigned long long k0 = (uint64_t)blockIdx.x * blockDim.x; k0 < m; k0 += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long k = k0 + threadIdx.x;
        bool fin = false;
        int32_t r = 0;
        int64_t v = 0;
        if (k < m) {
            r = C.rule[k];
            v = C.sum[k];
            fin = top_rank(v) >= toprank[(int64_t)r * number + number - 1];
        }
        const uint64_t act = __builtin_amdgcn_ballot_w64(fin);
        if (!act) continue;
        const uint32_t lane = lane_id();
        const int first = __ffsll((unsigned long long)act) - 1;
        unsigned long long base = 0;
        if ((int)lane == first) base = atomicAdd(F.n, (unsigned long long)__popcll(act));
        base = __shfl(base, first, WAVE);
        const unsigned long long j = base + (unsigned long long)__popcll(act & ((1ull << lane) - 1ull));
        if (fin && j < F.cap) {
            F.key[j] = C.key[k];
            F.rule[j] = r;
            F.sum[j] = v;
        }
    }
}

// Round phase A: best (int) sum among the candidates after the previous pick.
__global__ __launch_bounds__(256) void k_ptop_best_sum(TopCands C, const unsigned long long *__restrict__ prev_rank,
                                                       const unsigned long long *__restrict__ prev_key,
                                                       unsigned long long *__restrict__ cand_rank) {
    const unsigned long long m = *C.n < C.cap ? *C.n : C.cap;
    for (unsigned long long k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t r = C.rule[k];
        const uint64_t rk = top_rank(C.sum[k]);
        if (top_after(rk, C.key[k], prev_rank[r], prev_key[r])) atomicMax(&cand_rank[r], (unsigned long long)rk);
    }
}

// Round phase B: smallest key with that (int) sum (after the previous pick).
__global__ __launch_bounds__(256) void k_ptop_best_key(TopCands C, const unsigned long long *__restrict__ prev_rank,
                                                       const unsigned long long *__restrict__ prev_key,
                                                       const unsigned long long *__restrict__ cand_rank,
                                                       unsigned long long *__restrict__ cand_key) {
    const unsigned long long m = *C.n < C.cap ? *C.n : C.cap;
    for (unsigned long long k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t r = C.rule[k];
        const uint64_t rk = top_rank(C.sum[k]);
        const unsigned long long key = C.key[k];
        if (rk == cand_rank[r] && top_after(rk, key, prev_rank[r], prev_key[r])) atomicMin(&cand_key[r], key);
    }
}

// Round phase C: the pick's long sum (keys are unique) -> the rule's k-th entry.
__global__ __launch_bounds__(256) void k_ptop_take(TopCands C, const unsigned long long *__restrict__ cand_rank,
                                                   const unsigned long long *__restrict__ cand_key, int kth, int number,
                                                   uint64_t *__restrict__ out_key, int64_t *__restrict__ out_sum) {
    const unsigned long long m = *C.n < C.cap ? *C.n : C.cap;
    for (unsigned long long k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t r = C.rule[k];
        const unsigned long long key = C.key[k];
        if (cand_rank[r] != 0 && key == cand_key[r]) {
            out_key[(int64_t)r * number + kth] = key;
            out_sum[(int64_t)r * number + kth] = C.sum[k];
        }
    }
}

// Per rule: advance prev <- cand, reset cand, count the entries found.
__global__ __launch_bounds__(256) void k_ptop_advance(int32_t R, unsigned long long *__restrict__ prev_rank,
                                                      unsigned long long *__restrict__ prev_key,
                                                      unsigned long long *__restrict__ cand_rank,
                                                      unsigned long long *__restrict__ cand_key,
                                                      int32_t *__restrict__ count) {
    const int32_t r = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (r >= R) return;
    if (cand_rank[r] != 0) {
        prev_rank[r] = cand_rank[r];
        prev_key[r] = cand_key[r];
        count[r] += 1;
    } else {
        prev_rank[r] = 1;                                 // exhausted: nothing ranks after this
        prev_key[r] = ~0ull;
    }
    cand_rank[r] = 0;
    cand_key[r] = ~0ull;
}

}  // namespace sentinel
