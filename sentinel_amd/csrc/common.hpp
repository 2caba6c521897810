// common.hpp -- device helpers shared by the gfx950 kernels of the token-decision engine.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sentinel {

constexpr int WAVE = 64;                 // CDNA wavefront width
constexpr int64_t EPOCH_ABSENT = -1;     // slot never created (LeapArray slot == null)
constexpr uint32_t KEY_INVALID = 0xFFFFFFFFu;

// ClusterFlowEvent ordinals (srv/flow/statistic/data/ClusterFlowEvent.java:22-52)
enum : int { EV_PASS = 0, EV_BLOCK = 1, EV_PASS_REQUEST = 2, EV_BLOCK_REQUEST = 3,
             EV_OCCUPIED_PASS = 4, EV_OCCUPIED_BLOCK = 5, EV_WAITING = 6, NEV = 7 };

// TokenResultStatus (core/cluster/TokenResultStatus.java:27-69)
enum : int8_t { ST_BAD_REQUEST = -4, ST_TOO_MANY_REQUEST = -2, ST_FAIL = -1, ST_OK = 0,
                ST_BLOCKED = 1, ST_SHOULD_WAIT = 2, ST_NO_RULE_EXISTS = 3 };

// Key kinds of the segmented-admission pipeline.
enum : uint8_t { KIND_CLUSTER = 0,   // ClusterFlowChecker (srv/flow/ClusterFlowChecker.java:55-112)
                 KIND_SIMPLE = 1,    // SimpleClusterFlowChecker (rls/flow/SimpleClusterFlowChecker.java:33-65)
                 KIND_LIMITER = 2,   // RequestLimiter.tryPass (srv/flow/statistic/limit/RequestLimiter.java:72-87)
                 KIND_PARAM = 3,     // ClusterParamFlowChecker single value (srv/flow/ClusterParamFlowChecker.java:42-87)
                 KIND_LOCAL_PARAM = 4 };   // ParamFlowChecker.passLocalCheck (pfc/.../ParamFlowChecker.java:78-202)

// Namespace routing of a rule (ClusterFlowChecker.allowProceed, CFC:50-53; GlobalRequestLimiter.tryPass,
// GRL:46-55): >= 0 is the namespace's limiter key.
constexpr int32_t ROUTE_TOO_MANY = -1;   // namespace == null -> TOO_MANY_REQUEST (GRL:47-49)
constexpr int32_t ROUTE_PLAIN = -2;      // no limiter for the namespace (GRL:51-53)

// JLS 5.1.3 double -> int: NaN -> 0, saturating.
__host__ __device__ inline int32_t java_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return 2147483647;
    if (d <= -2147483648.0) return (int32_t)0x80000000u;
    return (int32_t)d;
}

__host__ __device__ inline int64_t wrap_add(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a + (uint64_t)b);
}

__host__ __device__ inline int64_t wrap_mul(int64_t a, int64_t b) {
    return (int64_t)((uint64_t)a * (uint64_t)b);
}

// epoch(t) = floor(t / w) for 0 <= t < 2^53 without a 64-bit integer divide: the double quotient
// is within one of the true quotient (|err| <= t/w * 2^-52 < 1), fixed by one remainder check.
__device__ inline int64_t epoch_of(int64_t t, int32_t w, double rcp_w) {
    int64_t e = (int64_t)((double)t * rcp_w);
    int64_t r = t - e * (int64_t)w;
    if (r < 0) e -= 1;
    else if (r >= (int64_t)w) e += 1;
    return e;
}

// 64-bit finaliser (murmur3 fmix64): open-addressing slots and count-min columns.
__host__ __device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

// JLS 5.1.3 double -> long: NaN -> 0, saturating.
__host__ __device__ inline int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

constexpr uint64_t PKEY_EMPTY = 0xFFFFFFFFFFFFFFFFull;   // reserved param key (empty table slot)

// Batch counters that many workgroups add to (fresh inserts): one atomic per workgroup on a single
// address queues every workgroup of a launch at one memory channel, so the counter is striped over
// CNT_LANES lines by workgroup index and its readers sum the lanes (k_pfresh_publish, the engine).
constexpr int CNT_LANES = 64;
constexpr int CNT_STRIDE = 16;                                  // 128 B apart
constexpr size_t CNT_BYTES = (size_t)CNT_LANES * CNT_STRIDE * 8;
__device__ inline unsigned long long *cnt_lane(unsigned long long *c) {
    return c + (blockIdx.x & (CNT_LANES - 1)) * CNT_STRIDE;
}

// Find or insert `key` in an open-addressing table of 2^k slots; returns the slot or -1 (full).
// `fresh` (optional) counts the keys this call inserted.
__device__ inline int64_t slot_insert(unsigned long long *table, uint64_t mask, uint64_t key,
                                      unsigned long long *fresh = nullptr) {
    // A slot goes EMPTY -> key once and keeps it for the kernel's lifetime, so a plain load that sees
    // the key (or another key) is final and only an EMPTY slot needs the CAS: a hot key (Zipf values)
    // is found by reads, not by a queue of atomics on one address.  A stale EMPTY costs one CAS.
    uint64_t h = mix64(key) & mask;
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        const unsigned long long cur = table[h];
        if (cur == key) return (int64_t)h;
        if (cur == PKEY_EMPTY) {
            const unsigned long long prev = atomicCAS(&table[h], (unsigned long long)PKEY_EMPTY, (unsigned long long)key);
            if (prev == PKEY_EMPTY) {
                if (fresh) atomicAdd(cnt_lane(fresh), 1ull);
                return (int64_t)h;
            }
            if (prev == key) return (int64_t)h;
        }
        h = (h + 1) & mask;
    }
    return -1;
}

// slot_insert counting this thread's fresh inserts in a register (the kernel adds a workgroup's total
// to the global counter once: a global atomic per fresh key serialises a batch of new values on one
// address).
//
// The probe sequence is linear probing's (h, h + 1, ... mod capacity), read 8 slots (one aligned 64-B
// group, four 16-B loads in flight together) per memory round trip: at a load factor of 3/4 a fresh
// key's chain averages ~8 slots and its tail over a wave's 64 lanes runs to dozens, one dependent load
// each when probed slot by slot.  A CAS that loses to another key continues at the next slot (the
// group's copy may be stale there: the CAS is what decides).  Tables have >= 8 slots.
constexpr int PROBE_GROUP = 8;
__device__ inline int64_t slot_insert_counted(unsigned long long *table, uint64_t mask, uint64_t key, uint32_t &nfresh) {
    uint64_t h = mix64(key) & mask;
    uint32_t s = (uint32_t)h & (PROBE_GROUP - 1);
    uint64_t g = h & ~(uint64_t)(PROBE_GROUP - 1);
    for (uint64_t scanned = 0; scanned <= mask; scanned += PROBE_GROUP) {
        const ulonglong2 *gp = reinterpret_cast<const ulonglong2 *>(table + g);
        ulonglong2 v[PROBE_GROUP / 2];
#pragma unroll
        for (int q = 0; q < PROBE_GROUP / 2; ++q) v[q] = gp[q];
#pragma unroll
        for (int j = 0; j < PROBE_GROUP; ++j) {
            if ((uint32_t)j < s) continue;
            const unsigned long long cur = (j & 1) ? v[j >> 1].y : v[j >> 1].x;
            if (cur == key) return (int64_t)(g + j);
            if (cur == PKEY_EMPTY) {
                const unsigned long long prev = atomicCAS(&table[g + j], (unsigned long long)PKEY_EMPTY, (unsigned long long)key);
                if (prev == PKEY_EMPTY) { ++nfresh; return (int64_t)(g + j); }
                if (prev == key) return (int64_t)(g + j);
            }
        }
        s = 0;
        g = (g + PROBE_GROUP) & mask;
    }
    return -1;
}

// Adds every thread's `mine` to *global with one atomic per workgroup (`lds`: a zeroed shared word,
// all threads of the block call this).
__device__ inline void block_add_global(unsigned long long *global, uint32_t mine, uint32_t *lds) {
    if (mine) atomicAdd(lds, mine);
    __syncthreads();
    if (threadIdx.x == 0 && *lds && global) atomicAdd(cnt_lane(global), (unsigned long long)*lds);
}

// Read-only lookup; returns the slot or -1.
__device__ inline int64_t slot_find(const unsigned long long *table, uint64_t mask, uint64_t key) {
    if (!table) return -1;
    uint64_t h = mix64(key) & mask;
    for (uint64_t probes = 0; probes <= mask; ++probes) {
        const unsigned long long x = table[h];
        if (x == PKEY_EMPTY) return -1;
        if (x == key) return (int64_t)h;
        h = (h + 1) & mask;
    }
    return -1;
}

__device__ inline uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// popcount(mask & lanes-below-me)
// Lanes of the wave holding the same key d (valid lanes only): one ballot per key bit, each
// narrowing the candidate set to the lanes that agree on that bit (nbits <= MAXB).
template <int MAXB>
__device__ inline uint64_t match_peers(uint32_t d, bool valid, int nbits) {
    uint64_t peers = __builtin_amdgcn_ballot_w64(valid);
#pragma unroll
    for (int b = 0; b < MAXB; ++b) {
        if (b < nbits) {
            const uint64_t bal = __builtin_amdgcn_ballot_w64((d >> b) & 1u);
            const uint64_t flip = ((d >> b) & 1u) ? 0ull : ~0ull;
            peers &= bal ^ flip;
        }
    }
    return peers;
}

__device__ inline uint32_t mask_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

}  // namespace sentinel
