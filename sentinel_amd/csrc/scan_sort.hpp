// scan_sort.hpp -- device-wide prefix scan and radix-sort building blocks for gfx950.
//
// K2 of the engine ("radix sort keys each batch by (flowId, seq)"): keys are dense flow (or
// namespace / param-slot) indices, values are arrival positions (seq).  LSD radix sort is stable,
// so events of one key stay in arrival order -- exactly the per-flow serialisation the reference
// gets from one ClusterMetric per flowId (srv/flow/statistic/ClusterMetricStatistics.java:56-58).
//
// Wave-64 design: a 256-thread workgroup = 4 waves owns a 4096-key tile; each wave ranks its
// 1024 keys (16 per lane, lane-striped so coalesced loads keep arrival order) with 8 ballots per
// item (64-bit match masks) and a wave-private LDS digit counter -- no LDS atomics.  The ranked
// tile is staged in LDS in digit order and written out as contiguous per-digit runs.
// Pass 0's per-tile digit histogram is fused into the producer of the keys (the prep kernel);
// each later pass histograms its own input tiles (per-tile offsets need the pass's tiling).
#pragma once

#include "common.hpp"

namespace sentinel {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;     // 4096

constexpr int RADIX_BITS = 8;
constexpr int RADIX = 1 << RADIX_BITS;
constexpr int MAX_PASSES = 4;
#ifndef SENTINEL_SORT_THREADS
#define SENTINEL_SORT_THREADS 512
#endif
#ifndef SENTINEL_SORT_ITEMS
#define SENTINEL_SORT_ITEMS 8
#endif
constexpr int SORT_THREADS = SENTINEL_SORT_THREADS;   // >= RADIX
constexpr int SORT_WAVES = SORT_THREADS / WAVE;
constexpr int SORT_ITEMS = SENTINEL_SORT_ITEMS;
constexpr int SORT_TILE = SORT_THREADS * SORT_ITEMS;     // 4096 by default
static_assert(SORT_THREADS >= 256 && SORT_THREADS % 64 == 0, "one thread per digit");

__device__ inline uint32_t wave_inclusive_scan(uint32_t v) {
    const int lane = (int)lane_id();
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
        uint32_t u = __shfl_up(v, off, WAVE);
        if (lane >= off) v += u;
    }
    return v;
}

// Block-wide exclusive scan of one value per thread; returns the exclusive prefix and the block
// total through *total.
__device__ inline uint32_t block_exclusive_scan(uint32_t v, uint32_t *lds_waves, uint32_t *total) {
    const int lane = (int)lane_id();
    const int wave = threadIdx.x / WAVE;
    uint32_t inc = wave_inclusive_scan(v);
    if (lane == WAVE - 1) lds_waves[wave] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    const int nw = blockDim.x / WAVE;
    for (int w = 0; w < nw; ++w) {
        uint32_t x = lds_waves[w];
        if (w < wave) base += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

// Pass A: per-tile scan into out, tile totals into partials.
template <bool EXCLUSIVE>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_tiles(const uint32_t *__restrict__ in,
                                                             uint32_t *__restrict__ out, int64_t n,
                                                             uint32_t *__restrict__ partials) {
    __shared__ uint32_t tile[SCAN_TILE];
    __shared__ uint32_t waves[SCAN_THREADS / WAVE];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        int64_t i = base + j * SCAN_THREADS + threadIdx.x;
        tile[j * SCAN_THREADS + threadIdx.x] = i < n ? in[i] : 0u;
    }
    __syncthreads();
    uint32_t loc[SCAN_ITEMS];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        loc[j] = tile[threadIdx.x * SCAN_ITEMS + j];
        sum += loc[j];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, waves, &total);
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        uint32_t x = loc[j];
        if (EXCLUSIVE) { tile[threadIdx.x * SCAN_ITEMS + j] = run; run += x; }
        else { run += x; tile[threadIdx.x * SCAN_ITEMS + j] = run; }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        int64_t i = base + j * SCAN_THREADS + threadIdx.x;
        if (i < n) out[i] = tile[j * SCAN_THREADS + threadIdx.x];
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

// Pass B: exclusive scan of the tile totals, one workgroup.
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_partials(uint32_t *partials, int64_t nparts) {
    __shared__ uint32_t waves[SCAN_THREADS / WAVE];
    uint32_t carry = 0;
    for (int64_t b = 0; b < nparts; b += SCAN_THREADS) {
        int64_t i = b + threadIdx.x;
        uint32_t v = i < nparts ? partials[i] : 0u;
        uint32_t total;
        uint32_t ex = block_exclusive_scan(v, waves, &total);
        if (i < nparts) partials[i] = carry + ex;
        carry += total;
    }
}

// Pass C: add the tile offsets.
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_add(uint32_t *__restrict__ out, int64_t n,
                                                           const uint32_t *__restrict__ partials) {
    const uint32_t off = partials[blockIdx.x];
    if (off == 0) return;
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        int64_t i = base + j * SCAN_THREADS + threadIdx.x;
        if (i < n) out[i] += off;
    }
}

inline int64_t scan_parts(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE; }

// Single-pass device scan with decoupled look-back (one launch instead of three).  Tiles take a
// dynamic id from an atomic ticket, so every tile's predecessors have started; a tile publishes
// its aggregate, then its inclusive prefix, in ONE 64-bit word {flag:2 | generation:30 | value:32}
// with agent-scope relaxed atomics (the payload is the flag: no separate release/acquire pair is
// needed).  One wave looks back over 64 predecessors at a time.  Spins are bounded; on timeout the
// tile records an error word and proceeds (wrong result, never a hang).
//
// No memset in front of a launch (round 6: a fill kernel costs ~5 us on the stream, and the radix path
// ran up to six per batch): every launch carries a generation, and a word of another generation reads
// as "not published yet"; the ticket is never reset -- the host passes how many tickets earlier
// launches took (tbase; 32-bit arithmetic, wraps).  The words live in their own buffer (LBState),
// zeroed when allocated (generation 0 is never a launch's) and again when the 30-bit generation wraps.
// (A self-cleaning variant -- the last workgroup to finish zeroing the words -- was measured first:
// its end-of-workgroup counter round trip made the segment kernel 40 -> 45 us.)
constexpr uint64_t LB_AGG = 1ull << 62;
constexpr uint64_t LB_PREFIX = 2ull << 62;
constexpr uint64_t LB_FLAGS = 3ull << 62;
constexpr uint32_t LB_GEN_MASK = (1u << 30) - 1;

// ctl: [0] tile ticket (never reset)
struct LBState {
    unsigned long long *status;
    uint32_t *ctl;
    uint32_t gen;        // this launch's generation, in [1, 2^30)
    uint32_t tbase;      // tickets taken by earlier launches
    uint32_t *err;       // pinned host word: 1 a look-back gave up its spin, 2 a ticket outside the grid
                         // (the batch's results are invalid; engine.hip, dev_err_synced)
};

__device__ inline void lookback_error(const LBState &L, uint32_t code) {
    __hip_atomic_store(L.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// This workgroup's tile id (call from every thread; thread 0 takes the ticket).  A ticket outside the
// grid (the host's count of earlier tickets out of step -- a launch that never ran) must not index the
// status words: the workgroup records the error and takes its block index (wrong results, reported to
// the host through L.err; never an out-of-bounds store).
__device__ inline uint32_t lookback_ticket(const LBState &L) {
    __shared__ uint32_t s_tid;
    if (threadIdx.x == 0) {
        uint32_t id = atomicAdd(&L.ctl[0], 1u) - L.tbase;
        if (id >= gridDim.x) {
            lookback_error(L, 2u);
            id = blockIdx.x;
        }
        s_tid = id;
    }
    __syncthreads();
    return s_tid;
}

// Decoupled look-back for tile b with aggregate `total`: wave 0 publishes the aggregate, sums
// predecessors 64 at a time until it meets an inclusive prefix, publishes its own prefix and
// leaves the exclusive prefix in *s_prefix (LDS).  Call from every thread of the block; a
// __syncthreads() must follow before *s_prefix is read.
__device__ inline void tile_lookback(int64_t b, uint32_t total, const LBState &L, uint32_t *s_prefix) {
    if (threadIdx.x >= WAVE) return;
    unsigned long long *status = L.status;
    const int lane = threadIdx.x;
    const uint64_t g = (uint64_t)L.gen << 32;
    uint32_t prefix = 0;
    if (b == 0) {
        if (lane == 0) __hip_atomic_store(&status[0], LB_PREFIX | g | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        if (lane == 0) __hip_atomic_store(&status[b], LB_AGG | g | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int64_t hi = b - 1;
        uint32_t spins = 0;
        for (;;) {
            const int64_t p = hi - lane;
            uint64_t st = p >= 0 ? __hip_atomic_load(&status[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : (LB_PREFIX | g);
            if (((st >> 32) & LB_GEN_MASK) != L.gen) st = 0;   // an earlier launch's word: not yet
            const uint64_t not_ready = __ballot((st & LB_FLAGS) == 0);
            const uint64_t is_prefix = __ballot((st & LB_FLAGS) == LB_PREFIX);
            const int first_prefix = is_prefix ? __ffsll((unsigned long long)is_prefix) - 1 : WAVE;
            const uint64_t need = first_prefix >= WAVE - 1 ? ~0ull : ((2ull << first_prefix) - 1);
            if (not_ready & need) {
                if (++spins > (1u << 22)) { if (lane == 0) lookback_error(L, 1u); break; }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            uint32_t v = (lane <= first_prefix) ? (uint32_t)st : 0u;
#pragma unroll
            for (int m = WAVE / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, WAVE);
            prefix += v;
            if (first_prefix < WAVE) break;
            hi -= WAVE;
        }
        if (lane == 0)
            __hip_atomic_store(&status[b], LB_PREFIX | g | (uint32_t)(prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) *s_prefix = prefix;
}

template <bool EXCLUSIVE>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_lookback(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                                int64_t n, LBState L) {
    __shared__ uint32_t tile[SCAN_TILE];
    __shared__ uint32_t waves[SCAN_THREADS / WAVE];
    __shared__ uint32_t s_prefix;
    const int64_t b = lookback_ticket(L);
    const int64_t base = b * SCAN_TILE;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int64_t i = base + j * SCAN_THREADS + threadIdx.x;
        tile[j * SCAN_THREADS + threadIdx.x] = i < n ? in[i] : 0u;
    }
    __syncthreads();
    uint32_t loc[SCAN_ITEMS];
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        loc[j] = tile[threadIdx.x * SCAN_ITEMS + j];
        sum += loc[j];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan(sum, waves, &total);
    tile_lookback(b, total, L, &s_prefix);
    __syncthreads();
    run += s_prefix;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const uint32_t x = loc[j];
        if (EXCLUSIVE) { tile[threadIdx.x * SCAN_ITEMS + j] = run; run += x; }
        else { run += x; tile[threadIdx.x * SCAN_ITEMS + j] = run; }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int64_t i = base + j * SCAN_THREADS + threadIdx.x;
        if (i < n) out[i] = tile[j * SCAN_THREADS + threadIdx.x];
    }
}


// ---------------------------------------------------------------- radix sort

inline int64_t sort_blocks(int64_t n) { return (n + SORT_TILE - 1) / SORT_TILE; }
inline int passes_for(int bits) { return bits <= 0 ? 1 : (bits + RADIX_BITS - 1) / RADIX_BITS; }
// digit-major histograms of all passes: hist[(p * RADIX + d) * nblocks + b]
inline int64_t hist_words(int64_t n, int passes) { return sort_blocks(n) * RADIX * passes; }

// Per-tile digit histograms of every pass, from one read of the keys.  The tile of block b is
// [b*SORT_TILE, (b+1)*SORT_TILE): the same tiling k_radix_scatter uses.
// One count per key digit.  When every active lane of the wave holds the same digit (a namespace-limiter
// key: one or a few namespaces for the whole batch) the first lane adds them all at once instead of 64
// lanes queueing atomics on one LDS word.
__device__ inline void tile_hist_accumulate(uint32_t (*h)[RADIX], uint32_t key, int passes) {
    const uint64_t act = __builtin_amdgcn_read_exec();
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
    if (__builtin_amdgcn_ballot_w64(key == k0) == act) {
        if ((uint64_t)1 << lane_id() == (act & (~act + 1)))
            for (int p = 0; p < passes; ++p)
                atomicAdd(&h[p][(k0 >> (p * RADIX_BITS)) & (RADIX - 1)], (uint32_t)__popcll(act));
        return;
    }
    for (int p = 0; p < passes; ++p) atomicAdd(&h[p][(key >> (p * RADIX_BITS)) & (RADIX - 1)], 1u);
}

__device__ inline void tile_hist_store(uint32_t (*h)[RADIX], uint32_t *hist, int passes, int64_t nblocks) {
    for (int p = 0; p < passes; ++p)
        for (int d = threadIdx.x; d < RADIX; d += blockDim.x)
            hist[((int64_t)p * RADIX + d) * nblocks + blockIdx.x] = h[p][d];
}

__global__ __launch_bounds__(SORT_THREADS) void k_radix_hist_pass(const uint32_t *__restrict__ keys, int64_t n,
                                                                  int shift, uint32_t *__restrict__ hist,
                                                                  int64_t nblocks) {
    __shared__ uint32_t h[RADIX];
    for (int d = threadIdx.x; d < RADIX; d += SORT_THREADS) h[d] = 0;
    const int64_t base = (int64_t)blockIdx.x * SORT_TILE;
    uint32_t k[SORT_ITEMS];                               // every load of the tile in flight at once
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const int64_t i = base + j * SORT_THREADS + threadIdx.x;
        k[j] = i < n ? keys[i] : 0u;
    }
    __syncthreads();
    // one LDS add per run of equal digits within a wave: a later pass reads the previous pass's output,
    // where a hot key's events are contiguous (a Zipf batch sent hundreds of same-address adds per tile
    // through one LDS bank before)
    const uint32_t lane = lane_id();
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; ++j) {
        const bool valid = base + j * SORT_THREADS + threadIdx.x < n;   // (a prefix of the wave's lanes)
        const uint32_t d = (k[j] >> shift) & (RADIX - 1);
        const uint32_t dp = __shfl_up(d, 1, WAVE);
        const bool head = valid && (lane == 0 || d != dp);
        const uint64_t hm = __ballot(head);
        const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
        if (head) {
            const uint64_t above = hm & ~((2ull << lane) - 1ull);    // (lane 63: 2 << 63 == 0, nothing above)
            const uint32_t end = above ? (uint32_t)__ffsll((long long)above) - 1 : nvalid;
            atomicAdd(&h[d], end - lane);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < RADIX; d += SORT_THREADS) hist[(int64_t)d * nblocks + blockIdx.x] = h[d];
}

}  // namespace sentinel
