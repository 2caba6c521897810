// dropin_bench.cpp -- the drop-in TokenService path under concurrent callers, measured natively.
//
// Models the reference's cluster token server: Netty worker threads (io.netty.eventLoopThreads =
// 2 x cores, NettyTransportServer.java:53-54) each calling TokenService.requestToken synchronously per
// request (FlowRequestProcessor.java:36-45).  Here T native threads call sentinel_batcher_request_token
// (sync mode) -- or keep D requests in flight through sentinel_batcher_request_token_async (async
// mode, an event-loop front end) -- on BASELINE config-2 flows (10k flowIds, n=2 / 1000 ms, GLOBAL,
// count ~ U{10..1000}, Zipf(1.1) requests, timestamps = the wall clock like TimeUtil).  Prints one
// JSON line: decisions/s and per-call latency percentiles against the 20 ms client budget
// (ClusterConstants.java:44).
//
// usage: dropin_bench [--threads T] [--seconds S] [--flows F] [--max-batch B] [--max-wait-us W]
//                     [--mode sync|async] [--inflight D]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/sentinel_amd.h"

namespace {

using clk = std::chrono::steady_clock;

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
    uint64_t next() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

struct Slot {
    std::atomic<int> busy{0};
    int64_t start_ns = 0;
};

struct ThreadState {
    std::vector<uint32_t> lat_us10;   // latency in units of 0.1 us
    int64_t ok = 0, blocked = 0, other = 0;
    std::vector<Slot> slots;
    std::atomic<int64_t> done{0};
};

int64_t now_ns(clk::time_point t0) { return std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count(); }

void on_done(void *ctx, uint64_t tag, const sentinel_token_result_t *r);

struct Ctx {
    ThreadState *ts;
    clk::time_point t0;
};

void on_done(void *ctx, uint64_t tag, const sentinel_token_result_t *r) {
    Ctx *c = (Ctx *)ctx;
    ThreadState *ts = c->ts;
    Slot &sl = ts->slots[tag];
    const int64_t d = now_ns(c->t0) - sl.start_ns;
    ts->lat_us10.push_back((uint32_t)std::min<int64_t>(d / 100, 0xFFFFFFFF));   // dispatcher thread only
    if (r->status == SENTINEL_STATUS_OK) ts->ok++;
    else if (r->status == SENTINEL_STATUS_BLOCKED) ts->blocked++;
    else ts->other++;
    sl.busy.store(0, std::memory_order_release);
    ts->done.fetch_add(1, std::memory_order_release);
}

double pct(std::vector<uint32_t> &v, double q) {
    if (v.empty()) return 0.0;
    const size_t k = std::min(v.size() - 1, (size_t)std::ceil(q * v.size()) - (q * v.size() >= 1 ? 1 : 0));
    std::nth_element(v.begin(), v.begin() + k, v.end());
    return v[k] / 10.0;
}

}  // namespace

int main(int argc, char **argv) {
    int threads = 2 * (int)std::thread::hardware_concurrency(), seconds = 5, flows = 10000, max_batch = 4096;
    int max_wait_us = 20, inflight = 64;
    std::string mode = "sync";
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string a = argv[i];
        if (a == "--threads") threads = atoi(argv[i + 1]);
        else if (a == "--seconds") seconds = atoi(argv[i + 1]);
        else if (a == "--flows") flows = atoi(argv[i + 1]);
        else if (a == "--max-batch") max_batch = atoi(argv[i + 1]);
        else if (a == "--max-wait-us") max_wait_us = atoi(argv[i + 1]);
        else if (a == "--mode") mode = argv[i + 1];
        else if (a == "--inflight") inflight = atoi(argv[i + 1]);
    }
    sentinel_server_config_t cfg{1.0, 1.0};
    sentinel_engine_t *e = nullptr;
    if (sentinel_engine_create(0, &cfg, &e)) { fprintf(stderr, "engine: %s\n", sentinel_last_error()); return 1; }
    sentinel_namespace_t ns{1, 0, 30000.0};
    sentinel_set_namespaces(e, &ns, 1);
    std::vector<sentinel_flow_rule_t> rules(flows);
    Rng rr(2);
    for (int i = 0; i < flows; ++i)
        rules[i] = sentinel_flow_rule_t{i + 1, (double)(10 + rr.next() % 991), SENTINEL_THRESHOLD_GLOBAL, 2, 1000, 0,
                                        SENTINEL_CHECKER_CLUSTER, 0};
    if (sentinel_load_flow_rules(e, rules.data(), flows)) { fprintf(stderr, "rules: %s\n", sentinel_last_error()); return 1; }
    // Zipf(1.1) over the flows, ranks permuted
    std::vector<double> cdf(flows);
    double acc = 0;
    for (int i = 0; i < flows; ++i) cdf[i] = (acc += 1.0 / std::pow(i + 1.0, 1.1));
    for (double &c : cdf) c /= acc;
    std::vector<int64_t> perm(flows);
    for (int i = 0; i < flows; ++i) perm[i] = i + 1;
    Rng pr(7);
    for (int i = flows - 1; i > 0; --i) std::swap(perm[i], perm[pr.next() % (i + 1)]);
    sentinel_batcher_t *b = nullptr;
    if (sentinel_batcher_create(e, max_batch, max_wait_us, &b)) { fprintf(stderr, "batcher: %s\n", sentinel_last_error()); return 1; }
    // warm the path (first batches allocate workspaces)
    for (int i = 0; i < 50; ++i) {
        sentinel_token_result_t r;
        sentinel_batcher_request_token(b, 1, 1, 0, 1600000000000LL, &r);
    }
    const int64_t T0 = 1600000000000LL + 5000;
    std::vector<ThreadState> st(threads);
    std::vector<Ctx> ctx(threads);
    std::atomic<bool> go{false};
    const clk::time_point t0 = clk::now();
    const int64_t end_ns = (int64_t)seconds * 1000000000LL;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) {
        ctx[t] = Ctx{&st[t], t0};
        if (mode == "async") {
            st[t].slots = std::vector<Slot>(inflight);
            st[t].lat_us10.reserve(1 << 20);
        } else {
            st[t].lat_us10.reserve(1 << 20);
        }
        th.emplace_back([&, t] {
            Rng rng(100 + t);
            ThreadState &s = st[t];
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            size_t slot = 0;
            int64_t sent = 0;
            for (;;) {
                const int64_t n0 = now_ns(t0);
                if (n0 >= end_ns) break;
                const double u = rng.uni();
                const int64_t fid = perm[std::min<size_t>(std::upper_bound(cdf.begin(), cdf.end(), u) - cdf.begin(), flows - 1)];
                const int64_t ts = T0 + n0 / 1000000;                  // TimeUtil.currentTimeMillis()
                if (mode == "async") {
                    // next free slot (D in flight per thread)
                    for (;;) {
                        if (!s.slots[slot].busy.load(std::memory_order_acquire)) break;
                        slot = (slot + 1) % inflight;
                        if (slot == 0) std::this_thread::yield();
                    }
                    s.slots[slot].busy.store(1, std::memory_order_relaxed);
                    s.slots[slot].start_ns = now_ns(t0);
                    sentinel_batcher_request_token_async(b, fid, 1, 0, ts, on_done, &ctx[t], slot);
                    slot = (slot + 1) % inflight;
                    ++sent;
                } else {
                    sentinel_token_result_t r;
                    const int64_t a = now_ns(t0);
                    sentinel_batcher_request_token(b, fid, 1, 0, ts, &r);
                    s.lat_us10.push_back((uint32_t)std::min<int64_t>((now_ns(t0) - a) / 100, 0xFFFFFFFF));
                    if (r.status == SENTINEL_STATUS_OK) s.ok++;
                    else if (r.status == SENTINEL_STATUS_BLOCKED) s.blocked++;
                    else s.other++;
                }
            }
            if (mode == "async")
                while (s.done.load(std::memory_order_acquire) < sent) std::this_thread::yield();
        });
    }
    int64_t b0 = 0, r0 = 0;
    sentinel_batcher_stats(b, &b0, &r0);
    go.store(true, std::memory_order_release);
    for (auto &x : th) x.join();
    const double el = now_ns(t0) / 1e9;
    int64_t b1 = 0, r1 = 0;
    sentinel_batcher_stats(b, &b1, &r1);
    std::vector<uint32_t> all;
    int64_t ok = 0, blk = 0, oth = 0;
    for (auto &s : st) {
        all.insert(all.end(), s.lat_us10.begin(), s.lat_us10.end());
        ok += s.ok; blk += s.blocked; oth += s.other;
    }
    const int64_t n = (int64_t)all.size();
    const double p50 = pct(all, 0.50), p99 = pct(all, 0.99), p999 = pct(all, 0.999);
    const double mx = all.empty() ? 0.0 : *std::max_element(all.begin(), all.end()) / 10.0;
    printf("{\"bench\": \"dropin_batcher\", \"mode\": \"%s\", \"threads\": %d, \"inflight_per_thread\": %d, "
           "\"flows\": %d, \"max_batch\": %d, \"max_wait_us\": %d, \"seconds\": %.3f, \"requests\": %lld, "
           "\"decisions_per_s\": %.1f, \"latency_us\": {\"p50\": %.1f, \"p99\": %.1f, \"p999\": %.1f, \"max\": %.1f}, "
           "\"client_budget_ms\": 20, \"batches\": %lld, \"mean_batch\": %.1f, \"ok\": %lld, \"blocked\": %lld, "
           "\"other\": %lld}\n",
           mode.c_str(), threads, mode == "async" ? inflight : 1, flows, max_batch, max_wait_us, el, (long long)n,
           n / el, p50, p99, p999, mx, (long long)(b1 - b0), (double)(r1 - r0) / std::max<int64_t>(1, b1 - b0),
           (long long)ok, (long long)blk, (long long)oth);
    sentinel_batcher_destroy(b);
    sentinel_engine_destroy(e);
    return 0;
}
