// small.hpp -- a small flow batch (<= SM_MAX events) decided in ONE launch of ONE workgroup.
//
// The drop-in front doors (sentinel_batcher_*, the wire servers, sentinel_submit_flow_batch_host)
// hand over batches of tens to a few thousand requests, for which the large-batch pipelines are
// launch-bound: the sorted path is ~25 dependent launches + copies, ~130 us of GPU time per batch
// whatever its size (measured, profiles/r02_dropin).  Here one 512-thread workgroup
//   1. validates every event as k_part_prep does (DefaultTokenService.java:38-45, CFC:50-53) and
//      packs it (EventSrc::pack_fields), the sort key being (flow << 13 | arrival position);
//   2. sorts the keys in LDS (bitonic, padded to a power of two: invalid events sort last), so the
//      order is (flow, arrival) -- the order the radix sort produces;
//   3. finds the runs (one per flow) with a block scan of the head flags;
//   4. decides each run with one lane (part_run: the window header in VGPRs, closed-form epoch
//      segments, heterogeneous walk, the reference state machine for prioritized requests), the
//      verdicts landing in LDS;
//   5. writes the verdicts out in arrival order, coalesced, then (host callers) a completion flag
//      in pinned memory that the host polls: no stream synchronisation on the request path.
// The events and verdicts may live in pinned host memory (the kernel reads and writes them over
// the bus once each: no copy launches), the window state is the flow table both large paths use.
#pragma once

#include "partition.hpp"

namespace sentinel {

constexpr int SM_THREADS = 512;                   // 2 waves per SIMD: up to 256 VGPRs (part_run<16> spills at 128)
constexpr int SM_MAX = 4096;                      // events per launch (LDS: 3 x 32 KB + 16 KB)
constexpr int SM_ITEMS = SM_MAX / SM_THREADS;
constexpr int SM_POS_BITS = 13;
constexpr uint64_t SM_KEY_NONE = ~0ull;
static_assert((1 << SM_POS_BITS) > SM_MAX, "arrival position field");

template <int NMAX>
__global__ __launch_bounds__(SM_THREADS) void k_small_flow(KeyTable T, uint32_t n, EventSrc src, uint64_t *__restrict__ out,
                                                           int32_t nflows, const int32_t *__restrict__ route,
                                                           uint32_t *done) {
    __shared__ uint64_t s_key[SM_MAX];
    __shared__ uint64_t s_val[SM_MAX];
    __shared__ uint64_t s_out[SM_MAX];
    __shared__ uint32_t s_run[SM_MAX + 1];
    __shared__ int64_t s_waves[SM_THREADS / WAVE];
    __shared__ uint32_t s_nvalid;
    const uint32_t tid = threadIdx.x;
    uint32_t m = 1;
    while (m < n) m <<= 1;
    // (src arrives as a kernel argument: building the EventSrc in the kernel from pointer arguments
    // crashes ROCm 7.2's clang in SimplifyCFG)
    const Event *__restrict__ ev = src.ev;
    const uint8_t *__restrict__ fl = src.flags;
    const int64_t T0 = ev[0].ts;
    if (tid == 0) s_nvalid = 0;
    // 1. validation + packing (s_val by arrival position for now)
    for (uint32_t i = tid; i < m; i += SM_THREADS) {
        uint64_t key = SM_KEY_NONE, val = 0;
        if (i < n) {
            const Event e = ev[i];
            const uint8_t f = fl ? fl[i] : 0;
            int st = 127;
            if (e.idx == SENTINEL_IDX_BAD_ID || e.acquire <= 0) st = ST_BAD_REQUEST;      // DTS:38-40
            else if (e.idx < 0 || e.idx >= nflows) st = ST_NO_RULE_EXISTS;               // DTS:42-45
            else if (route && route[e.idx] == ROUTE_TOO_MANY) st = ST_TOO_MANY_REQUEST;  // CFC:50-53
            else if (e.ts < 0) st = ST_FAIL;                                              // NPE in LeapArray
            if (st == 127) {
                key = ((uint64_t)(uint32_t)e.idx << SM_POS_BITS) | i;
                val = src.pack_event(i, e, f, T0);
            } else {
                s_out[i] = pack_verdict(st, 0, 0);
            }
        }
        s_key[i] = key;
        s_val[i] = val;
    }
    __syncthreads();
    // 2. bitonic sort of s_key[0, m): pair t of stage (k, j) is (i, i + j), i = t with a zero bit
    // inserted at j; ascending where i & k == 0
    for (uint32_t k = 2; k <= m; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = tid; t < (m >> 1); t += SM_THREADS) {
                const uint32_t i = 2 * t - (t & (j - 1));
                const uint64_t a = s_key[i], b = s_key[i + j];
                if ((a > b) == ((i & k) == 0)) {
                    s_key[i] = b;
                    s_key[i + j] = a;
                }
            }
            __syncthreads();
        }
    }
    // 3. values into sorted order, run heads (thread t owns sorted positions [t*SM_ITEMS, +SM_ITEMS))
    uint64_t vv[SM_ITEMS];
    uint32_t heads = 0;
#pragma unroll
    for (int j = 0; j < SM_ITEMS; ++j) {
        const uint32_t i = tid * SM_ITEMS + j;
        vv[j] = 0;
        if (i < m) {
            const uint64_t k = s_key[i];
            if (k != SM_KEY_NONE) {
                vv[j] = s_val[(uint32_t)k & ((1u << SM_POS_BITS) - 1)];
                if (i == 0 || (s_key[i - 1] >> SM_POS_BITS) != (k >> SM_POS_BITS)) ++heads;
                if (i + 1 == m || s_key[i + 1] == SM_KEY_NONE) s_nvalid = i + 1;
            }
        }
    }
    int64_t nruns64 = 0;
    const uint32_t base = (uint32_t)block_exclusive_scan64((int64_t)heads, s_waves, &nruns64);   // (barriers)
    const uint32_t nruns = (uint32_t)nruns64;
    uint32_t r = base;
#pragma unroll
    for (int j = 0; j < SM_ITEMS; ++j) {
        const uint32_t i = tid * SM_ITEMS + j;
        if (i < m && s_key[i] != SM_KEY_NONE) {
            s_val[i] = vv[j];
            if (i == 0 || (s_key[i - 1] >> SM_POS_BITS) != (s_key[i] >> SM_POS_BITS)) s_run[r++] = i;
        }
    }
    if (tid == 0) s_run[nruns] = s_nvalid;
    __syncthreads();
    // 4. one lane per flow run, verdicts into LDS
    const Verdicts V{s_out, nullptr, 0};
    for (uint32_t q = tid; q < nruns; q += SM_THREADS) {
        const uint32_t q0 = s_run[q];
        part_run<NMAX>(T, (uint32_t)(s_key[q0] >> SM_POS_BITS), s_val, q0, s_run[q + 1], src, V, T0);
    }
    __syncthreads();
    // 5. verdicts in arrival order; then, if asked, a completion flag the host polls (every lane's
    // verdict stores are complete and visible system-wide before the release store of the flag)
    for (uint32_t i = tid; i < n; i += SM_THREADS) out[i] = s_out[i];
    if (done) {
        __threadfence_system();
        __syncthreads();
        if (tid == 0) __hip_atomic_store(done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace sentinel
