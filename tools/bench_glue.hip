// Bench support, not part of the engine: the 5conc workload's client traffic.  Batch s + 1 releases, at
// its release positions, the tokens batch s handed out at its acquire positions (bench.py, ConcWorkload):
// word 1 (token id) of event row rel_pos[i] (sentinel_concurrent_event_t, 3 words) <- word 0 (token id) of
// result row rel_src[i] of the previous batch (2 words).  One kernel with 32-bit positions instead of the
// two torch index kernels (index_select + index_copy_, 64-bit indices, ~60 us per 4M-event batch).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int GLUE_THREADS = 256;
constexpr int GLUE_ITEMS = 4;

__global__ __launch_bounds__(GLUE_THREADS) void k_forward_tokens(int64_t *__restrict__ ev_words,
                                                                 const int64_t *__restrict__ prev_words,
                                                                 const int32_t *__restrict__ rel_pos,
                                                                 const int32_t *__restrict__ rel_src, int64_t count) {
    const int64_t base = (int64_t)blockIdx.x * GLUE_THREADS * GLUE_ITEMS + threadIdx.x;
    int32_t d[GLUE_ITEMS], s[GLUE_ITEMS];
#pragma unroll
    for (int j = 0; j < GLUE_ITEMS; ++j) {
        const int64_t i = base + (int64_t)j * GLUE_THREADS;
        d[j] = i < count ? rel_pos[i] : -1;
        s[j] = i < count ? rel_src[i] : 0;
    }
    int64_t v[GLUE_ITEMS];
#pragma unroll
    for (int j = 0; j < GLUE_ITEMS; ++j) v[j] = d[j] >= 0 ? prev_words[(int64_t)s[j] * 2] : 0;
#pragma unroll
    for (int j = 0; j < GLUE_ITEMS; ++j)
        if (d[j] >= 0) ev_words[(int64_t)d[j] * 3 + 1] = v[j];
}

}  // namespace

extern "C" int bench_glue_forward_tokens(int64_t *ev_words, const int64_t *prev_words, const int32_t *rel_pos,
                                         const int32_t *rel_src, int64_t count, hipStream_t stream) {
    if (count <= 0) return 0;
    if (!ev_words || !prev_words || !rel_pos || !rel_src) return -1;
    const int64_t per = (int64_t)GLUE_THREADS * GLUE_ITEMS;
    const int64_t blocks = (count + per - 1) / per;
    if (blocks > 0x7fffffff) return -1;
    k_forward_tokens<<<dim3((unsigned)blocks), dim3(GLUE_THREADS), 0, stream>>>(ev_words, prev_words, rel_pos,
                                                                                rel_src, count);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
