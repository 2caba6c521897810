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
// (K2 radix sort, arrival order kept) and one lane walks each flow's events in order.  The token
// cache is one open-addressing table in HBM shared by all lanes: inserts CAS an empty slot, a
// release turns its slot into a tombstone (only the owning flow's lane ever touches a token).
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

// Result record {token_id, status}: two 8-byte stores.
__device__ inline void put_conc(uint64_t *out, uint32_t i, int64_t token, int status) {
    out[2 * (uint64_t)i] = (uint64_t)token;
    out[2 * (uint64_t)i + 1] = (uint64_t)(uint32_t)status;
}

// DefaultTokenService.requestConcurrentToken validation (DTS:64-75, 89-91) and release lookup;
// sort key = flow index (acquire: the rule; release: the token's flow); pass-0 histograms.
__global__ __launch_bounds__(SORT_THREADS) void k_conc_prep(int64_t n, const ConcEvent *__restrict__ ev, int32_t nflows,
                                                            TokenTable TT, uint64_t *__restrict__ out,
                                                            uint32_t *__restrict__ fkey, uint32_t finvalid,
                                                            uint32_t *__restrict__ fhist, int64_t nblocks) {
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
            else k = (uint32_t)TT.flow_idx[h];
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

// One lane per flow: nowCalls in a register, the flow's acquires / releases in arrival order.
__global__ __launch_bounds__(256) void k_conc_process(BatchWork W, const ConcEvent *__restrict__ ev,
                                                      int32_t *__restrict__ now_calls, const double *__restrict__ thr,
                                                      const int64_t *__restrict__ flow_ids, TokenTable TT,
                                                      uint64_t id_base, uint64_t *__restrict__ out) {
    const int64_t g0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)*W.nseg;
    if (g0 >= S || (int64_t)*W.nvalid == 0) return;
    const uint32_t flow = W.seg_key[g0];
    if (g0 > 0 && W.seg_key[g0 - 1] == flow) return;
    int32_t now = now_calls[flow];
    const double threshold = thr[flow];
    for (int64_t g = g0; g < S; ++g) {
        if (g > g0 && W.seg_key[g] != flow) break;
        const uint32_t end = W.seg_start[g + 1];
        for (uint32_t i = W.seg_start[g]; i < end; ++i) {
            const uint32_t seq = (uint32_t)W.sval[i] & SEQ_MASK;
            const ConcEvent e = ev[seq];
            if (e.kind == CONC_ACQUIRE) {
                // CCFC:57-71: int + int (wraps) compared with the double threshold
                if ((double)(int32_t)((uint32_t)now + (uint32_t)e.acquire) > threshold) {
                    put_conc(out, seq, 0, ST_BLOCKED);
                    continue;
                }
                const uint64_t id = id_base + seq;                            // TokenCacheNode.java:59-70
                const int64_t h = slot_insert(TT.keys, TT.mask, id);
                if (h < 0) {                                                 // token cache full
                    put_conc(out, seq, 0, ST_FAIL);
                    continue;
                }
                TT.flow_id[h] = flow_ids[flow];
                TT.flow_idx[h] = (int32_t)flow;
                TT.acquire[h] = e.acquire;
                atomicAdd(&TT.counts[0], 1ull);
                now = (int32_t)((uint32_t)now + (uint32_t)e.acquire);
                put_conc(out, seq, (int64_t)id, ST_OK);
            } else {
                const int64_t h = token_find(TT, (uint64_t)e.token);         // CCFC:82-100
                if (h < 0) {                                                 // released earlier in this batch
                    put_conc(out, seq, 0, ST_ALREADY_RELEASE);
                    continue;
                }
                TT.keys[h] = TOKEN_TOMB;
                atomicAdd(&TT.counts[0], ~0ull);
                atomicAdd(&TT.counts[1], 1ull);
                now = (int32_t)((uint32_t)now - (uint32_t)TT.acquire[h]);
                put_conc(out, seq, 0, ST_RELEASE_OK);
            }
        }
    }
    now_calls[flow] = now;
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
