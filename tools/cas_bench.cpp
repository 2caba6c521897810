// cas_bench.cpp -- the scattered 8-B atomic rate of gfx950 in isolation (HIP; build: hipcc -x hip, see
// below).  The shared count-min's HBM walk (k_pp_cm_walk) adds each (key, epoch) count to d cells with a
// returned compare-and-swap on a 640 MB sketch; this measures that access pattern alone, next to its
// non-returning and plain-store twins, on a table of the same size:
//   cas_ret     2^24 random 8-B atomicCAS (returned value used: the count-min retry loop)
//   add_noret   2^24 random 8-B atomicAdd, result unused (memory-side add, no round trip)
//   store8      2^24 random 8-B plain stores
//   load8       2^24 random 8-B loads
// Prints ops/s and ns per op for each, with 2048 x 256 threads (every op independent).
//   hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -o tools/cas_bench tools/cas_bench.cpp
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

__global__ void cas_ret(unsigned long long *t, uint64_t mask, int64_t nreq, uint32_t *sink) {
    uint32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nreq; i += (int64_t)gridDim.x * blockDim.x) {
        unsigned long long *c = t + (mix((uint64_t)i) & mask);
        unsigned long long x = *c;
        for (int k = 0; k < 8; ++k) {                       // (bounded: a contended slot gives up)
            const unsigned long long p = atomicCAS(c, x, x + 1);
            if (p == x) break;
            x = p;
        }
        acc ^= (uint32_t)x;
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

__global__ void add_noret(unsigned long long *t, uint64_t mask, int64_t nreq) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nreq; i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(t + (mix((uint64_t)i + 5) & mask), 1ull);
}

__global__ void store8(unsigned long long *t, uint64_t mask, int64_t nreq) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nreq; i += (int64_t)gridDim.x * blockDim.x)
        t[mix((uint64_t)i + 9) & mask] = (unsigned long long)i;
}

__global__ void load8(const unsigned long long *t, uint64_t mask, int64_t nreq, uint32_t *sink) {
    unsigned long long acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nreq; i += (int64_t)gridDim.x * blockDim.x)
        acc ^= t[mix((uint64_t)i + 13) & mask];
    if (acc == 0x9e3779b97f4a7c15ull) sink[0] = (uint32_t)acc;
}

int main() {
    const size_t TB = (size_t)640 << 20;                    // the 4cm sketch: 4 x 2^20 x 20 slots x 8 B
    const uint64_t mask = ((uint64_t)1 << 26) - 1;          // 2^26 slots x 8 B = 512 MiB of it addressed
    unsigned long long *t;
    uint32_t *sink;
    CK(hipMalloc(&t, TB));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(t, 0, TB));
    const int64_t nreq = (int64_t)1 << 24;
    const dim3 grid(2048), block(256);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char *name, auto &&f) {
        f();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < 5; ++r) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double s = ms * 1e-3 / 5;
        printf("%-10s %8.1f us  %7.2f Gops/s  %6.3f ns/op\n", name, s * 1e6, nreq / s / 1e9, s * 1e9 / nreq);
    };
    timeit("cas_ret", [&] { cas_ret<<<grid, block>>>(t, mask, nreq, sink); });
    timeit("add_noret", [&] { add_noret<<<grid, block>>>(t, mask, nreq); });
    timeit("store8", [&] { store8<<<grid, block>>>(t, mask, nreq); });
    timeit("load8", [&] { load8<<<grid, block>>>(t, mask, nreq, sink); });
    return 0;
}
