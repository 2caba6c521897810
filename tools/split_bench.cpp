// split_bench.cpp -- microbenchmark of the partition front (HIP; build: hipcc -x hip, see below).
//
// Times k_part_split (the one-sweep partition, partition.hpp) against the prep + scan + scatter front it
// replaces on the same device-generated config-3 batch (uniform flows, acquire 1), and checks that both
// produce the same range-ordered values and range starts.  Built with -DSENTINEL_SPLIT_STAMPS it also
// prints per-phase wall-clock spans of the split kernel's workgroups.
//   hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off [-DSENTINEL_SPLIT_STAMPS] \
//         -o tools/split_bench tools/split_bench.cpp
//   tools/split_bench [events=8388608] [flows=1000000] [reps=20]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/sentinel_amd.h"
#include "../sentinel_amd/csrc/partition.hpp"

using namespace sentinel;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

__global__ void k_gen(Event *ev, int64_t n, int32_t F, int64_t t0, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t h = mix64((uint64_t)i ^ seed);
    ev[i] = Event{(int32_t)(h % (uint64_t)F), 1, t0 + i / 8};
}

static int bits_for(int64_t nkeys) {
    int b = 1;
    while (((int64_t)1 << b) - 1 < nkeys) ++b;
    return b;
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 8 * 1024 * 1024;
    const int32_t F = argc > 2 ? atoi(argv[2]) : 1000000;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int fbits = bits_for(F);
    const uint32_t finvalid = (1u << fbits) - 1;
    const int lb = std::max(0, fbits - PART_MAX_BITS);
    const int32_t P = (int32_t)(((int64_t)F + (1 << lb) - 1) >> lb);
    const int pbits = bits_for(P - 1 > 0 ? P - 1 : 1);
    const int64_t nb = part_blocks(n), ng = (nb + PS_GROUP - 1) / PS_GROUP;
    int items = 0, G = 0;
    for (int it : {8, 16, 32}) {
        const int64_t g = (n + (int64_t)it * SP_THREADS - 1) / ((int64_t)it * SP_THREADS);
        if (g <= ncu) { items = it; G = (int)g; break; }
    }
    if (!items) { fprintf(stderr, "batch too large for one sweep\n"); return 1; }
    printf("n=%lld F=%d P=%d lb=%d items=%d G=%d CUs=%d\n", (long long)n, F, P, lb, items, G, ncu);

    Event *ev;
    uint64_t *out, *va, *vb;
    uint32_t *hist, *gsum, *ra, *rb, *col, *bar, *ctl, *err;
    unsigned long long *stat;
    CK(hipMalloc(&ev, n * sizeof(Event)));
    CK(hipMalloc(&out, n * 8));
    CK(hipMalloc(&va, n * 8));
    CK(hipMalloc(&vb, n * 8));
    CK(hipMalloc(&hist, (size_t)nb * P * 4 + 64));
    CK(hipMalloc(&gsum, ((size_t)ng * P + 2 * (size_t)P + 1) * 4));
    CK(hipMalloc(&rb, ((size_t)P + 1) * 4));
    CK(hipMalloc(&col, ((size_t)P * G + P) * 4));
    CK(hipMalloc(&bar, 64));
    CK(hipMalloc(&ctl, 64));
    CK(hipMalloc(&stat, 64));
    CK(hipHostMalloc(&err, 64, 0));
    *err = 0;
    CK(hipMemset(bar, 0, 64));
    ra = gsum + (size_t)ng * P;
    uint32_t *rtot = ra + P + 1;
    k_gen<<<(unsigned)((n + 255) / 256), 256>>>(ev, n, F, 1700000000000LL, 12345);
    CK(hipDeviceSynchronize());
    const EventSrc src{ev, nullptr, nullptr, false};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));

    auto old_front = [&] {
        k_part_prep<<<dim3((unsigned)nb), dim3(PP_THREADS)>>>(n, ev, F, nullptr, out, nullptr, finvalid, lb, hist, nb, P,
                                                              ctl, stat, nullptr);
        const dim3 g2((unsigned)ng, (unsigned)((P + PS_THREADS - 1) / PS_THREADS));
        k_part_colsum<<<g2, PS_THREADS>>>(hist, nb, P, gsum);
        k_part_colscan<<<(unsigned)((P + PC_THREADS / WAVE - 1) / (PC_THREADS / WAVE)), PC_THREADS>>>(gsum, ng, P, rtot);
        k_part_offsets<<<g2, PS_THREADS>>>(hist, nb, P, gsum, rtot, ra);
        k_part_scatter<<<dim3((unsigned)nb), dim3(PT_THREADS)>>>(nullptr, src, va, n, finvalid, lb, pbits, hist, nb, P, F);
    };
    uint32_t arrivals = 0;
    auto new_front = [&] {
        const uint32_t base = arrivals;
        arrivals += 2u * (uint32_t)G;
        if (items == 8)
            k_part_split<8><<<G, SP_THREADS>>>(n, src, F, out, lb, pbits, P, vb, rb, col, bar, base, err, ctl, stat);
        else if (items == 16)
            k_part_split<16><<<G, SP_THREADS>>>(n, src, F, out, lb, pbits, P, vb, rb, col, bar, base, err, ctl, stat);
        else
            k_part_split<32><<<G, SP_THREADS>>>(n, src, F, out, lb, pbits, P, vb, rb, col, bar, base, err, ctl, stat);
    };
    auto timeit = [&](const char *name, auto &&f) {
        f();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = 1000.0 * ms / reps;
        printf("%-28s %8.1f us  (%.2f TB/s on 24 B/event)\n", name, us, 24.0 * n / (us * 1e-6) / 1e12);
        return us;
    };
    timeit("prep + scan + scatter", old_front);
    timeit("k_part_split", new_front);
    if (*err) printf("BARRIER TIMEOUT\n");

    std::vector<uint64_t> ha(n), hb(n);
    std::vector<uint32_t> sa(P + 1), sb(P + 1);
    CK(hipMemcpy(ha.data(), va, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hb.data(), vb, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sa.data(), ra, (P + 1) * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sb.data(), rb, (P + 1) * 4, hipMemcpyDeviceToHost));
    const uint32_t nv = sa[P];
    int64_t bad = 0;
    for (int32_t d = 0; d <= P; ++d) bad += sa[d] != sb[d];
    for (uint32_t i = 0; i < nv; ++i) bad += ha[i] != hb[i];
    printf("valid %u, mismatches %lld -> %s\n", nv, (long long)bad, bad ? "DIFFERENT" : "identical");

#ifdef SENTINEL_SPLIT_STAMPS
    std::vector<unsigned long long> st((size_t)1024 * 8);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_split_stamp), st.size() * 8));
    unsigned long long t0 = ~0ull;
    for (int g = 0; g < G; ++g) t0 = std::min(t0, st[(size_t)g * 8]);
    const char *names[7] = {"read+validate+histogram", "publish+barrier1", "column scans", "barrier2", "range starts",
                            "first round's loads issued", "write-out rounds"};
    for (int ph = 0; ph < 7; ++ph) {
        double sum = 0, mx = 0;
        for (int g = 0; g < G; ++g) {
            const double d = (double)(st[(size_t)g * 8 + ph + 1] - st[(size_t)g * 8 + ph]) * 0.01;   // 100 MHz
            sum += d;
            mx = std::max(mx, d);
        }
        printf("  %-26s mean %7.2f us  max %7.2f us\n", names[ph], sum / G, mx);
    }
    double s0 = 0, e1 = 0;
    for (int g = 0; g < G; ++g) {
        s0 = std::max(s0, (double)(st[(size_t)g * 8] - t0) * 0.01);
        e1 = std::max(e1, (double)(st[(size_t)g * 8 + 7] - t0) * 0.01);
    }
    printf("  last workgroup start %.2f us, last end %.2f us\n", s0, e1);
    std::vector<unsigned long long> rs((size_t)1024 * 4);
    CK(hipMemcpyFromSymbol(rs.data(), HIP_SYMBOL(g_split_round), rs.size() * 8));
    const char *rn[4] = {"rank (+ next loads issued)", "wave offsets + digit scan", "stage", "write-out"};
    for (int ph = 0; ph < 4; ++ph) {
        double sum = 0;
        for (int g = 0; g < G; ++g) sum += (double)rs[(size_t)g * 4 + ph] * 0.01;
        printf("    rounds: %-26s mean %7.2f us (all rounds)\n", rn[ph], sum / G);
    }
#endif
    return bad ? 2 : 0;
}
