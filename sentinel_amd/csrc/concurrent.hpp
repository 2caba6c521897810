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
// (K2 radix sort, arrival order kept) and each flow's run is decided in arrival order (below: the
// elements gathered in parallel, short runs by one lane, long runs by a (min, +) scan).  The token
// cache is one open-addressing table in HBM: inserts CAS an empty slot or a tombstone, a release
// turns its slot into a tombstone.
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

struct TokenTable {
    unsigned long long *keys;    // token id, PKEY_EMPTY or TOKEN_TOMB
    int64_t *flow_id;
    int32_t *flow_idx;           // -1: the flow's rule is gone (release -> NO_RULE_EXISTS)
    int32_t *acquire;
    uint64_t mask;
    unsigned long long *counts;  // [0] live tokens, [1] tombstones
};

__device__ inline int64_t token_find(const TokenTable &T, uint64_t id) {
    uint64_t h = mix64(id) & T.mask;
    for (uint64_t p = 0; p <= T.mask; ++p) {
        const unsigned long long k = T.keys[h];
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
    uint64_t h = mix64(id) & T.mask;
    unsigned long long k = T.keys[h];
    for (uint64_t p = 0; p <= T.mask;) {
        if (k == PKEY_EMPTY || k == TOKEN_TOMB) {
            const unsigned long long prev = atomicCAS(&T.keys[h], k, (unsigned long long)id);
            if (prev == k) {
                tomb = k == TOKEN_TOMB;
                return (int64_t)h;
            }
            k = prev;                                     // taken (or changed) meanwhile: look again
#ifdef SENTINEL_CONC_GUARD
            if (++p > T.mask) { printf("token_insert: CAS spin id %llx h %llu\n", (unsigned long long)id, (unsigned long long)h); return -1; }
#endif
            continue;
        }
        h = (h + 1) & T.mask;
        ++p;
        k = T.keys[h];
    }
    return -1;
}

// Device compaction of the token cache into a fresh table (tombstones dropped, capacity possibly
// larger): every live token re-placed with its record; counts = {live, 0}.
__global__ __launch_bounds__(256) void k_tok_rebuild(TokenTable O, uint64_t ocap, TokenTable N) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ocap) return;
    const unsigned long long k = O.keys[s];
    if (k == PKEY_EMPTY || k == TOKEN_TOMB) return;
    uint64_t h = mix64(k) & N.mask;
    while (atomicCAS(&N.keys[h], (unsigned long long)PKEY_EMPTY, k) != PKEY_EMPTY) h = (h + 1) & N.mask;
    N.flow_id[h] = O.flow_id[s];
    N.flow_idx[h] = O.flow_idx[s];
    N.acquire[h] = O.acquire[s];
    atomicAdd(&N.counts[0], 1ull);
}

// Result record {token_id, status}: two 8-byte stores.
__device__ inline void put_conc(uint64_t *out, uint32_t i, int64_t token, int status) {
    out[2 * (uint64_t)i] = (uint64_t)token;
    out[2 * (uint64_t)i + 1] = (uint64_t)(uint32_t)status;
}

// DefaultTokenService.requestConcurrentToken validation (DTS:64-75, 89-91) and release lookup;
// sort key = flow index (acquire: the rule; release: the token's flow); pass-0 histograms.  A found
// release records its token slot (relslot) and claims it with its arrival position (atomicMin): the
// first release of a token in the batch is the one that finds it cached (CCFC:82-86), later ones of
// the same token answer ALREADY_RELEASE.  Tokens issued in this batch are not yet known to any client.
__global__ __launch_bounds__(SORT_THREADS) void k_conc_prep(int64_t n, const ConcEvent *__restrict__ ev, int32_t nflows,
                                                            TokenTable TT, uint64_t *__restrict__ out,
                                                            uint32_t *__restrict__ fkey, uint32_t finvalid,
                                                            uint32_t *__restrict__ fhist, int64_t nblocks,
                                                            uint32_t *__restrict__ relslot, uint32_t *__restrict__ claim) {
    __shared__ uint32_t hf[MAX_PASSES][RADIX];
    for (int d = threadIdx.x; d < MAX_PASSES * RADIX; d += SORT_THREADS) (&hf[0][0])[d] = 0;
    __syncthreads();
    const int64_t tile0 = (int64_t)blockIdx.x * SORT_TILE;
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = tile0 + j * SORT_THREADS + threadIdx.x;
        if (i >= n) break;
        const ConcEvent e = ev[i];
        int st = 127;
        uint32_t k = finvalid;
        if (e.kind == CONC_ACQUIRE) {
            if (!(e.flags & 1) || e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0) st = ST_BAD_REQUEST;
            else if (e.idx < 0 || e.idx >= nflows) st = ST_NO_RULE_EXISTS;
            else k = (uint32_t)e.idx;
        } else if (e.kind == CONC_RELEASE) {
            const int64_t h = token_find(TT, (uint64_t)e.token);             // CCFC:82-86
            if (h < 0) st = ST_ALREADY_RELEASE;
            else if (TT.flow_idx[h] < 0) st = ST_NO_RULE_EXISTS;             // CCFC:87-91
            else {
                k = (uint32_t)TT.flow_idx[h];
                relslot[i] = (uint32_t)h;
                atomicMin(&claim[h], (uint32_t)i);
            }
        } else {
            st = ST_BAD_REQUEST;
        }
        fkey[i] = k;
        tile_hist_accumulate(hf, k, 1);
        if (st != 127) put_conc(out, (uint32_t)i, 0, st);
    }
    __syncthreads();
    tile_hist_store(hf, fhist, 1, nblocks);
}

// Flow runs of the sorted batch: head flags (a valid key differing from its predecessor), scanned by
// the engine, then each head's run start; the last valid element publishes the valid count and the
// number of runs.
__global__ __launch_bounds__(256) void k_conc_heads(const uint32_t *__restrict__ skey, int64_t n, uint32_t invalid,
                                                    uint32_t *__restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = skey[i];
    flag[i] = (k != invalid && (i == 0 || skey[i - 1] != k)) ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_conc_runs(const uint32_t *__restrict__ skey, int64_t n, uint32_t invalid,
                                                   const uint32_t *__restrict__ pos, uint32_t *__restrict__ run_start,
                                                   uint32_t *__restrict__ ctl) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = skey[i];
    if (k == invalid) return;
    const bool head = i == 0 || skey[i - 1] != k;
    if (head) run_start[pos[i]] = (uint32_t)i;
    if (i + 1 == n || skey[i + 1] == invalid) {          // the last valid element
        const uint32_t nruns = pos[i] + (head ? 1u : 0u);
        run_start[nruns] = (uint32_t)(i + 1);
        ctl[0] = nruns;
    }
}

// ---------------------------------------------------------------- decisions
// After the sort a flow's events form a contiguous run in arrival order.  The batch is decided in four
// data-parallel steps, so that no lane walks a chain of dependent gathers:
//   k_conc_elems   one thread per sorted position gathers the event once and writes its element:
//                  elem > 0 an acquire of elem tokens, elem < 0 a release of -elem tokens that found its
//                  token cached and claimed it (the batch's first release of it, k_conc_prep), 0 a
//                  release that answers ALREADY_RELEASE; relh = the released token's slot
//   k_conc_lanes   one lane per run of <= CONC_LANE_RUN events: the CCFC:48-101 recurrence over the run's
//                  elements (nowCalls in a register, integer work only), one pass byte per acquire;
//                  longer runs are registered for the chunk kernels
//   k_conc_info / k_conc_chunks   long runs in 1024-event chunks: a (min, +) scan with a decoupled
//                  look-back for unit-acquire runs, a workgroup walk otherwise
//   k_conc_apply   one thread per sorted position: a passing acquire takes a token (insert into the
//                  cache, id = id_base + arrival position), a failing one answers BLOCKED, a claimed
//                  release tombstones its token, the rest answer ALREADY_RELEASE
// A release's amount is read in k_conc_elems, a kernel before any tombstone store, so a slot reused by an
// insert of this batch can never hand a release someone else's amount.
struct ConcElems {
    int32_t *elem;
    uint32_t *relh;
    uint8_t *pass;
};

__global__ __launch_bounds__(256) void k_conc_elems(const ConcEvent *__restrict__ ev, const uint64_t *__restrict__ sval,
                                                    const uint32_t *__restrict__ skey, uint32_t invalid, int64_t n,
                                                    const uint32_t *__restrict__ relslot,
                                                    const uint32_t *__restrict__ claim, TokenTable TT, ConcElems X) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || skey[i] == invalid) return;             // invalid events were answered by k_conc_prep
    const uint32_t seq = (uint32_t)sval[i] & SEQ_MASK;
    const ConcEvent e = ev[seq];
    int32_t x = 0;
    if (e.kind == CONC_ACQUIRE) {
        x = e.acquire;                                    // > 0 (validated)
    } else {
        const uint32_t h = relslot[seq];
        if (claim[h] == seq) {                            // CCFC:82-86: this release finds its token
            x = -TT.acquire[h];
            X.relh[i] = h;
        }
    }
    X.elem[i] = x;
}

// CCFC:57-70 for one acquire of `a` tokens at nowCalls `now`: int + int (wraps) compared with the double
// threshold; passes -> now += a.
__device__ inline bool conc_acquire(int32_t &now, int32_t a, double threshold) {
    const int32_t sum = (int32_t)((uint32_t)now + (uint32_t)a);
    if ((double)sum > threshold) return false;
    now = sum;
    return true;
}

#ifndef SENTINEL_CONC_LANE_RUN
#define SENTINEL_CONC_LANE_RUN 64
#endif
constexpr uint32_t CONC_LANE_RUN = SENTINEL_CONC_LANE_RUN;   // longer runs are decided in chunks by workgroups
constexpr uint32_t CONC_CHUNK = 1024;       // events of a long run per workgroup step (4 per thread)

// The greedy admission of unit acquires with releases interleaved is a (min, +) recurrence: while the
// in-flight count y is <= the largest admissible T' (the largest y with !((double)(y + 1) > threshold),
// minus one), an acquire maps y to min(y + 1, T') (it passes iff y < T') and a release of r tokens maps
// y to y - r.  Both are x -> min(x + P, C); composition (P1, C1) then (P2, C2) = (P1 + P2,
// min(C1 + P2, C2)) is associative, so the chunks of one long run are decided in parallel with a
// decoupled look-back over their compositions.
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

// the scan element of a unit-acquire run's element x
__device__ inline MinPlus conc_mp(int32_t x, int64_t Tp) {
    return x > 0 ? MinPlus{1, Tp} : x < 0 ? MinPlus{(int64_t)x, CONC_INF} : MinPlus{0, CONC_INF};
}

constexpr int CB_THREADS = 256;
constexpr int CB_WAVES = CB_THREADS / WAVE;

// Inclusive block scan of MinPlus over the 256 threads (wave shuffles, then the waves' totals, which
// stay in lds[] for the caller).
__device__ inline MinPlus mp_block_inclusive(MinPlus v, MinPlus *lds) {
    const uint32_t lane = lane_id();
    const int wave = threadIdx.x / WAVE;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const int64_t pp = __shfl_up(v.p, o, WAVE);
        const int64_t pc = __shfl_up(v.c, o, WAVE);
        if ((int)lane >= o) v = mp_then(MinPlus{pp, pc}, v);
    }
    if (lane == WAVE - 1) lds[wave] = v;
    __syncthreads();
    MinPlus pre{0, CONC_INF};
    for (int w = 0; w < wave; ++w) pre = mp_then(pre, lds[w]);
    __syncthreads();
    return mp_then(pre, v);
}
// ... and the exclusive value of this thread (the previous thread's inclusive one)
__device__ inline MinPlus mp_block_exclusive_of(MinPlus inc, const MinPlus *lds) {
    const uint32_t lane = lane_id();
    const int wave = threadIdx.x / WAVE;
    const int64_t pp = __shfl_up(inc.p, 1, WAVE), pc = __shfl_up(inc.c, 1, WAVE);
    MinPlus ex{pp, pc};
    if (lane == 0) {
        ex = MinPlus{0, CONC_INF};
        for (int w = 0; w < wave; ++w) ex = mp_then(ex, lds[w]);
    }
    return ex;
}

// Long runs of a batch: per run slot its run, nowCalls before the batch, T', whether every acquire
// asks for one token and the sum of |amounts| (the scan's eligibility); per chunk its slot, its index
// in the run and the look-back status {epoch << 2 | 1 aggregate / 2 inclusive, composition}.
struct ConcBig {
    uint32_t *run;
    int32_t *now0;
    int64_t *tp;
    uint32_t *unit;
    unsigned long long *mag;
    uint2 *chunks;           // [slot] {first chunk, chunk count}
    uint32_t *chunk_slot;
    uint32_t *chunk_j;
    uint32_t *flag;
    MinPlus *agg;
    MinPlus *inc;
    uint32_t *ctl;           // [0] runs, [1] long runs, [2] chunks, [3] chunk ticket
    uint32_t epoch;
};

// One lane per flow run of <= CONC_LANE_RUN events: the run's elements in arrival order (read 8 at a time);
// longer runs are cut into chunks for k_conc_chunks.
__global__ __launch_bounds__(256) void k_conc_lanes(const uint32_t *__restrict__ run_start,
                                                    const uint32_t *__restrict__ skey, int32_t *__restrict__ now_calls,
                                                    const double *__restrict__ thr, ConcElems X, ConcBig G) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= G.ctl[0]) return;
    const uint32_t b = run_start[r], e = run_start[r + 1];
    const uint32_t flow = skey[b];
    if (e - b > CONC_LANE_RUN) {
        const uint32_t slot = atomicAdd(&G.ctl[1], 1u);
        const uint32_t nch = (e - b + CONC_CHUNK - 1) / CONC_CHUNK;
        const uint32_t first = atomicAdd(&G.ctl[2], nch);
        G.run[slot] = r;
        G.now0[slot] = now_calls[flow];
        G.tp[slot] = conc_tprime(thr[flow]);
        G.unit[slot] = 1u;
        G.mag[slot] = 0ull;
        G.chunks[slot] = make_uint2(first, nch);
        for (uint32_t j = 0; j < nch; ++j) {
            G.chunk_slot[first + j] = slot;
            G.chunk_j[first + j] = j;
        }
        return;
    }
    int32_t now = now_calls[flow];
    const double threshold = thr[flow];
    for (uint32_t i0 = b; i0 < e; i0 += 8) {
        int32_t x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = i0 + k < e ? X.elem[i0 + k] : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (x[k] > 0) X.pass[i0 + k] = conc_acquire(now, x[k], threshold) ? 1 : 0;
            else if (x[k] < 0) now = (int32_t)((uint32_t)now + (uint32_t)x[k]);     // CCFC:97-98
        }
    }
    now_calls[flow] = now;
}

// Eligibility of the long runs for the scan: every acquire of 1 token, and the int sums cannot wrap.
__global__ __launch_bounds__(256) void k_conc_info(const uint32_t *__restrict__ run_start, ConcElems X, ConcBig G) {
    const uint32_t nch = G.ctl[2];
    for (uint32_t c = blockIdx.x; c < nch; c += gridDim.x) {
        const uint32_t slot = G.chunk_slot[c], j = G.chunk_j[c];
        const uint32_t r = G.run[slot];
        const uint32_t b = run_start[r] + j * CONC_CHUNK, e = min(run_start[r + 1], b + CONC_CHUNK);
        bool unit = true;
        unsigned long long mag = 0;
        for (uint32_t i = b + threadIdx.x; i < e; i += blockDim.x) {
            const int32_t x = X.elem[i];
            if (x > 1) unit = false;
            mag += (unsigned long long)(x < 0 ? -(int64_t)x : (int64_t)x);
        }
        if (__syncthreads_or(!unit) && threadIdx.x == 0) atomicAnd(&G.unit[slot], 0u);
#pragma unroll
        for (int o = WAVE / 2; o >= 1; o >>= 1) mag += __shfl_xor(mag, o, WAVE);
        if (lane_id() == 0 && mag) atomicAdd(&G.mag[slot], mag);
    }
}

// A long run that cannot take the whole-run scan (an acquire of several tokens, an int sum that could
// wrap, or nowCalls above T' when the batch starts): its elements walked by one thread with the
// CCFC:57-98 recurrence (integer work on the gathered elements only: rare runs, no barriers).
__device__ inline void conc_run_serial(const ConcElems &X, uint32_t b, uint32_t e, double threshold, int32_t &now) {
    for (uint32_t i0 = b; i0 < e; i0 += 8) {
        int32_t x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = i0 + k < e ? X.elem[i0 + k] : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (x[k] > 0) X.pass[i0 + k] = conc_acquire(now, x[k], threshold) ? 1 : 0;
            else if (x[k] < 0) now = (int32_t)((uint32_t)now + (uint32_t)x[k]);     // CCFC:97-98
        }
    }
}

// Chunks of long runs, one workgroup step each, taken in ticket order (a chunk's predecessors in its
// run were taken earlier, so the look-back always completes).  An eligible run's chunk composes its
// 1024 elements (4 consecutive per thread), publishes the composition, looks back over its run's
// earlier chunks for the prefix and decides its acquires from y = prefix(nowCalls); the run's last chunk
// writes nowCalls.  An ineligible run is walked whole by the workgroup that takes its first chunk.
__global__ __launch_bounds__(CB_THREADS) void k_conc_chunks(const uint32_t *__restrict__ run_start,
                                                            const uint32_t *__restrict__ skey, int32_t *__restrict__ now_calls,
                                                            const double *__restrict__ thr, ConcElems X, ConcBig G) {
    __shared__ MinPlus s_mp[CB_WAVES];
    __shared__ uint32_t s_ticket;
    __shared__ MinPlus s_prefix;
    const uint32_t t = threadIdx.x;
    const uint32_t nch = G.ctl[2];
#ifdef SENTINEL_CONC_GUARD
    if (blockIdx.x == 0 && t == 0) printf("k_conc_chunks: %u chunks, %u long runs, %u runs\n", nch, G.ctl[1], G.ctl[0]);
#endif
    for (;;) {
        if (t == 0) s_ticket = atomicAdd(&G.ctl[3], 1u);
        __syncthreads();
        const uint32_t c = s_ticket;
        __syncthreads();
        if (c >= nch) break;
        const uint32_t slot = G.chunk_slot[c], j = G.chunk_j[c];
        const uint32_t r = G.run[slot];
        const uint32_t rb = run_start[r], re = run_start[r + 1];
        const uint32_t flow = skey[rb];
        const int64_t now0 = G.now0[slot];
        const int64_t Tp = G.tp[slot];
        const bool ok = G.unit[slot] && (now0 < 0 ? -now0 : now0) + (int64_t)G.mag[slot] < (int64_t)INT32_MAX && now0 <= Tp;
        if (!ok) {                                        // block-uniform
            if (j == 0 && t == 0) {
                int32_t now = now_calls[flow];
                conc_run_serial(X, rb, re, thr[flow], now);
                now_calls[flow] = now;
            }
            continue;
        }
        const uint32_t b = rb + j * CONC_CHUNK;
        int32_t x[4];
        MinPlus mine{0, CONC_INF};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = b + t * 4 + q;
            x[q] = i < re ? X.elem[i] : 0;
            mine = mp_then(mine, conc_mp(x[q], Tp));
        }
        const MinPlus inc = mp_block_inclusive(mine, s_mp);
        const MinPlus exl = mp_block_exclusive_of(inc, s_mp);
        // the chunk's composition: published by thread 255, then the last wave looks back over the run's
        // earlier chunks 64 at a time (each lane waits for one chunk's flag; the window is composed
        // earliest first up to the nearest inclusive prefix)
        const uint32_t cf = G.chunks[slot].x;
        if (t == CB_THREADS - 1) {
            if (j == 0) {
                G.inc[c] = inc;
                __threadfence();
                __hip_atomic_store(&G.flag[c], (G.epoch << 2) | 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_prefix = MinPlus{0, CONC_INF};
            } else {
                G.agg[c] = inc;
                __threadfence();
                __hip_atomic_store(&G.flag[c], (G.epoch << 2) | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (j > 0 && t >= CB_THREADS - WAVE) {                               // last wave (block-uniform j)
            const uint32_t lane = t - (CB_THREADS - WAVE);
            MinPlus pre{0, CONC_INF};                                        // chunks between the window and c
            uint32_t top = c;                                                // the window ends below top
            for (;;) {
                const int64_t p = (int64_t)top - 1 - lane;                   // lane 0: the nearest chunk
                uint32_t f = 0;
                MinPlus v{0, CONC_INF};
                if (p >= (int64_t)cf) {
#ifdef SENTINEL_CONC_GUARD
                    uint64_t spins = 0;
#endif
                    do {
                        f = __hip_atomic_load(&G.flag[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef SENTINEL_CONC_GUARD
                        if (++spins == (1ull << 24)) { printf("look-back spin: chunk %u waits for %lld flag %x epoch %u\n", c, (long long)p, f, G.epoch); f = (G.epoch << 2) | 2u; }
#endif
                    } while ((f >> 2) != G.epoch || (f & 3u) == 0);
                    __threadfence();
                    v = (f & 3u) == 2u ? G.inc[p] : G.agg[p];
                }
                const uint64_t incl = __builtin_amdgcn_ballot_w64(p >= (int64_t)cf && (f & 3u) == 2u);
                const uint32_t valid = (uint32_t)min<int64_t>(WAVE, (int64_t)top - (int64_t)cf);
                const uint32_t last = incl ? (uint32_t)(__ffsll((unsigned long long)incl) - 1) : valid - 1;
                // compose lanes last .. 0 (earliest first): a shuffle chain in lane 0
                MinPlus w{0, CONC_INF};
                for (int l = (int)last; l >= 0; --l) {
                    const int64_t pp = __shfl(v.p, l, WAVE), pc = __shfl(v.c, l, WAVE);
                    w = mp_then(w, MinPlus{pp, pc});
                }
                pre = mp_then(w, pre);
                if (incl || top - cf <= (uint32_t)WAVE) break;               // reached an inclusive prefix / chunk cf
                top -= WAVE;
            }
            if (lane == WAVE - 1) {                                          // thread 255
                s_prefix = pre;
                const MinPlus acc = mp_then(pre, inc);
                G.inc[c] = acc;
                __threadfence();
                __hip_atomic_store(&G.flag[c], (G.epoch << 2) | 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (j + 1 == G.chunks[slot].y) now_calls[flow] = (int32_t)mp_apply(acc, now0);
            }
        } else if (j == 0 && t == CB_THREADS - 1 && j + 1 == G.chunks[slot].y) {
            now_calls[flow] = (int32_t)mp_apply(inc, now0);
        }
        __syncthreads();
        int64_t y = mp_apply(mp_then(s_prefix, exl), now0);   // before this thread's first event
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = b + t * 4 + q;
            if (i < re && x[q] > 0) {
                X.pass[i] = y < Tp ? 1 : 0;
                y = min(y + 1, Tp);
            } else if (i < re && x[q] < 0) {
                y += x[q];
            }
        }
        __syncthreads();
    }
}

// The effects, one thread per sorted position (CCFC:57-100): a passing acquire takes a token
// (TokenCacheNode, id = id_base + arrival position), a failing one answers BLOCKED; a claimed release
// frees its slot (a tombstone: probe chains continue through it) and answers RELEASE_OK; any other
// release ALREADY_RELEASE.  Cache counts {live, tombstones} by one atomic pair per workgroup.
__global__ __launch_bounds__(256) void k_conc_apply(const uint64_t *__restrict__ sval, const uint32_t *__restrict__ skey,
                                                    uint32_t invalid, int64_t n, ConcElems X, uint32_t *__restrict__ claim,
                                                    TokenTable TT, const int64_t *__restrict__ flow_ids, uint64_t id_base,
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
                const uint64_t id = id_base + seq;                            // TokenCacheNode.java:59-70
                bool tomb = false;
                const int64_t h = token_insert(TT, id, tomb);
                if (h < 0) {                                                  // token cache full
                    put_conc(out, seq, 0, ST_FAIL);
                } else {
                    if (tomb) --dtomb;
                    TT.flow_id[h] = flow_ids[flow];
                    TT.flow_idx[h] = (int32_t)flow;
                    TT.acquire[h] = x;
                    ++dlive;
                    put_conc(out, seq, (int64_t)id, ST_OK);
                }
            }
        } else if (x < 0) {
            const uint32_t h = X.relh[i];
            claim[h] = ~0u;
            __hip_atomic_store(&TT.keys[h], (unsigned long long)TOKEN_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            --dlive;                                                          // CCFC:92-100
            ++dtomb;
            put_conc(out, seq, 0, ST_RELEASE_OK);
        } else {
            put_conc(out, seq, 0, ST_ALREADY_RELEASE);
        }
    }
    if (dlive) atomicAdd(&s_cnt[0], (unsigned long long)dlive);    // (two's complement: wraps to a decrement)
    if (dtomb) atomicAdd(&s_cnt[1], (unsigned long long)dtomb);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_cnt[0]) atomicAdd(&TT.counts[0], s_cnt[0]);
        if (s_cnt[1]) atomicAdd(&TT.counts[1], s_cnt[1]);
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
    if (h <= TT.mask && TT.keys[h] == TOKEN_TOMB && TT.keys[(h + 1) & TT.mask] == PKEY_EMPTY) {
        for (int k = 0; k < 256; ++k) {                   // (bounded walk back)
            if (atomicCAS(&TT.keys[h], (unsigned long long)TOKEN_TOMB, (unsigned long long)PKEY_EMPTY) != TOKEN_TOMB)
                break;
            ++freed;
            h = (h - 1) & TT.mask;
            if (TT.keys[h] != TOKEN_TOMB) break;
        }
    }
    if (freed) atomicAdd(&s_freed, freed);
    __syncthreads();
    if (threadIdx.x == 0 && s_freed) atomicAdd(&TT.counts[1], 0ull - s_freed);
}

// RegularExpireStrategy.clearToken (RegularExpireStrategy.java:94-124): with the reference's own
// conditions every cached token qualifies (clientTimeout / resourceTimeout are durations compared
// with the wall clock), so a sweep removes up to `max_tokens` tokens and returns their counts to
// nowCalls (a token whose rule is gone just leaves the cache).
__global__ __launch_bounds__(256) void k_conc_expire(TokenTable TT, int32_t *now_calls, unsigned long long max_tokens,
                                                     unsigned long long *ticket) {
    const uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h > TT.mask) return;
    const unsigned long long k = TT.keys[h];
    if (k == PKEY_EMPTY || k == TOKEN_TOMB) return;
    if (atomicAdd(ticket, 1ull) >= max_tokens) return;
    TT.keys[h] = TOKEN_TOMB;
    atomicAdd(&TT.counts[0], ~0ull);
    atomicAdd(&TT.counts[1], 1ull);
    const int32_t f = TT.flow_idx[h];
    if (f >= 0) atomicSub(&now_calls[f], TT.acquire[h]);
}

}  // namespace sentinel
