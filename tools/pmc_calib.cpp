// pmc_calib.cpp -- known-byte access patterns for calibrating rocprofv3's memory-side request counters
// on gfx950 (HIP; build: hipcc -x hip, see below).  Each kernel moves a byte count fixed by its
// arguments; scripts/gpu_pmc_req.sh collects TCC_EA0_RDREQ{,_32B,_64B,_128B}_sum, TCC_BUBBLE_sum and
// TCC_EA0_WRREQ{,_64B}_sum per dispatch, and scripts/pmc_summary.py (--calib) prints requests x size
// against the known bytes, per pattern:
//   stream_read16     512 MiB read, 16 B per lane, consecutive lanes consecutive (a wave: 1 KiB run)
//   gather8           2^24 random 8-B reads from a 2 GiB table (each in its own line)
//   gather32          2^24 random 32-B aligned reads (one sector each) from the same table
//   gather64          2^23 random 64-B aligned reads (four lanes x 16 B)
//   stream_write16    512 MiB written, 16 B per lane, coalesced
//   scatter8          2^24 random 8-B writes into the 2 GiB table
//   scatter32         2^24 random 32-B aligned writes (two lanes x 16 B)
// The random patterns are the ones the engine's kernels issue (header and window gathers, verdict and
// record scatters), which the guide's x2 FETCH_SIZE correction (wide coalesced streams only) does not cover.
//   hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -o tools/pmc_calib tools/pmc_calib.cpp
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

__device__ inline uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

__global__ void stream_read16(const uint4 *__restrict__ a, int64_t n16, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void gather8(const uint64_t *__restrict__ t, uint64_t mask8, int64_t nreq, uint32_t *__restrict__ sink) {
    uint64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nreq; i += (int64_t)gridDim.x * blockDim.x)
        acc ^= t[mix((uint64_t)i) & mask8];
    if (acc == 0x9e3779b97f4a7c15ull) sink[0] = (uint32_t)acc;
}

__global__ void gather32(const uint4 *__restrict__ t, uint64_t mask32, int64_t nreq, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nreq; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t s = mix((uint64_t)i) & mask32;           // 32-B sector index
        const uint4 a = t[2 * s], b = t[2 * s + 1];
        acc ^= a.x ^ b.w;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

// four consecutive lanes read one 64-B block (16 B each)
__global__ void gather64(const uint4 *__restrict__ t, uint64_t mask64, int64_t nreq, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 4 * nreq; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t s = mix((uint64_t)(i >> 2)) & mask64;
        acc ^= t[4 * s + (i & 3)].y;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void stream_write16(uint4 *__restrict__ a, int64_t n16) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ void scatter8(uint64_t *__restrict__ t, uint64_t mask8, int64_t nreq) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nreq; i += (int64_t)gridDim.x * blockDim.x)
        t[mix((uint64_t)i + 77) & mask8] = (uint64_t)i;
}

// two consecutive lanes write one 32-B sector (16 B each)
__global__ void scatter32(uint4 *__restrict__ t, uint64_t mask32, int64_t nreq) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * nreq; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t s = mix((uint64_t)(i >> 1) + 99) & mask32;
        t[2 * s + (i & 1)] = make_uint4((uint32_t)i, 0u, 0u, 0u);
    }
}

int main() {
    const size_t SB = (size_t)512 << 20, TB = (size_t)2 << 30;
    void *s, *tb;
    uint32_t *sink;
    CK(hipMalloc(&s, SB));
    CK(hipMalloc(&tb, TB));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(s, 1, SB));
    CK(hipMemset(tb, 2, TB));
    CK(hipDeviceSynchronize());
    const int64_t nreq = (int64_t)1 << 24;
    const dim3 grid(256 * 8), block(256);
    for (int rep = 0; rep < 2; ++rep) {           // (the second pass of each is the one to read: warm TLB)
        stream_read16<<<grid, block>>>((const uint4 *)s, (int64_t)(SB / 16), sink);
        gather8<<<grid, block>>>((const uint64_t *)tb, TB / 8 - 1, nreq, sink);
        gather32<<<grid, block>>>((const uint4 *)tb, TB / 32 - 1, nreq, sink);
        gather64<<<grid, block>>>((const uint4 *)tb, TB / 64 - 1, nreq / 2, sink);
        stream_write16<<<grid, block>>>((uint4 *)s, (int64_t)(SB / 16));
        scatter8<<<grid, block>>>((uint64_t *)tb, TB / 8 - 1, nreq);
        scatter32<<<grid, block>>>((uint4 *)tb, TB / 32 - 1, nreq);
        CK(hipDeviceSynchronize());
    }
    printf("known bytes: stream_read16 %zu, gather8 %lld x 8 (lines: %lld), gather32 %lld x 32, gather64 %lld x 64, "
           "stream_write16 %zu, scatter8 %lld x 8, scatter32 %lld x 32\n",
           SB, (long long)nreq, (long long)nreq, (long long)nreq, (long long)nreq / 2, SB, (long long)nreq,
           (long long)nreq);
    return 0;
}
