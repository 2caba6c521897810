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

// ---------------------------------------------------------------- radix sort

inline int64_t sort_blocks(int64_t n) { return (n + SORT_TILE - 1) / SORT_TILE; }
inline int passes_for(int bits) { return bits <= 0 ? 1 : (bits + RADIX_BITS - 1) / RADIX_BITS; }
// digit-major histograms of all passes: hist[(p * RADIX + d) * nblocks + b]
inline int64_t hist_words(int64_t n, int passes) { return sort_blocks(n) * RADIX * passes; }

// Per-tile digit histograms of every pass, from one read of the keys.  The tile of block b is
// [b*SORT_TILE, (b+1)*SORT_TILE): the same tiling k_radix_scatter uses.
__device__ inline void tile_hist_accumulate(uint32_t (*h)[RADIX], uint32_t key, int passes) {
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
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * SORT_TILE;
#pragma unroll 4
    for (int j = 0; j < SORT_ITEMS; ++j) {
        int64_t i = base + j * SORT_THREADS + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & (RADIX - 1)], 1u);
    }
    __syncthreads();
    for (int d = threadIdx.x; d < RADIX; d += SORT_THREADS) hist[(int64_t)d * nblocks + blockIdx.x] = h[d];
}

}  // namespace sentinel
