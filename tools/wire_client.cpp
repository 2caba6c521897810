// wire_client.cpp -- load generator for the cluster token server's TCP wire protocol.
//
// Speaks the reference client's framing (NettyTransportClient: LengthFieldPrepender(2), request
// [i32 xid][i8 type=1][i64 flowId][i32 count][i8 prio], FlowRequestDataWriter) and reads responses
// [u16 len][i32 xid][i8 type][i8 status][i32 remaining][i32 waitInMs] (FlowResponseDataWriter).
// C connections, one thread each, keep D requests in flight (a cluster client multiplexes many
// callers over one Netty channel, NettyTransportClient.java:165-189); flows are BASELINE config 2
// (flowIds 1..F, Zipf(1.1) with ranks permuted).  Prints one JSON line: decisions/s and per-request
// latency percentiles (send -> response decoded) against the 20 ms client budget
// (ClusterConstants.java:44).
//
// usage: wire_client --port P [--host 127.0.0.1] [--conns C] [--inflight D] [--seconds S] [--flows F]
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

using clk = std::chrono::steady_clock;

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 1) {}
    uint64_t next() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

void put_be(uint8_t *p, uint64_t v, int bytes) {
    for (int i = bytes - 1; i >= 0; --i) { p[i] = (uint8_t)v; v >>= 8; }
}
uint64_t get_be(const uint8_t *p, int bytes) {
    uint64_t v = 0;
    for (int i = 0; i < bytes; ++i) v = (v << 8) | p[i];
    return v;
}

struct ConnStats {
    std::vector<uint32_t> lat_us10;
    int64_t ok = 0, blocked = 0, other = 0, bad = 0;
    bool failed = false;
};

constexpr int FLOW_FRAME = 2 + 4 + 1 + 8 + 4 + 1;     // 20 bytes on the wire
constexpr int FLOW_REPLY = 2 + 4 + 1 + 1 + 4 + 4;     // 16 bytes on the wire

double pct(std::vector<uint32_t> &v, double q) {
    if (v.empty()) return 0.0;
    size_t k = (size_t)std::ceil(q * v.size());
    k = k == 0 ? 0 : std::min(v.size() - 1, k - 1);
    std::nth_element(v.begin(), v.begin() + k, v.end());
    return v[k] / 10.0;
}

}  // namespace

int main(int argc, char **argv) {
    std::string host = "127.0.0.1";
    int port = 0, conns = 16, inflight = 256, seconds = 5, flows = 10000;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string a = argv[i];
        if (a == "--host") host = argv[i + 1];
        else if (a == "--port") port = atoi(argv[i + 1]);
        else if (a == "--conns") conns = atoi(argv[i + 1]);
        else if (a == "--inflight") inflight = atoi(argv[i + 1]);
        else if (a == "--seconds") seconds = atoi(argv[i + 1]);
        else if (a == "--flows") flows = atoi(argv[i + 1]);
    }
    if (port <= 0 || conns <= 0 || inflight <= 0 || flows <= 0) {
        fprintf(stderr, "usage: wire_client --port P [--conns C] [--inflight D] [--seconds S] [--flows F]\n");
        return 2;
    }
    std::vector<double> cdf(flows);
    double acc = 0;
    for (int i = 0; i < flows; ++i) cdf[i] = (acc += 1.0 / std::pow(i + 1.0, 1.1));
    for (double &c : cdf) c /= acc;
    std::vector<int64_t> perm(flows);
    for (int i = 0; i < flows; ++i) perm[i] = i + 1;
    Rng pr(7);
    for (int i = flows - 1; i > 0; --i) std::swap(perm[i], perm[pr.next() % (i + 1)]);

    const clk::time_point t0 = clk::now();
    auto now_ns = [&] { return std::chrono::duration_cast<std::chrono::nanoseconds>(clk::now() - t0).count(); };
    const int64_t end_ns = (int64_t)seconds * 1000000000LL;
    std::vector<ConnStats> st(conns);
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::thread> th;
    for (int c = 0; c < conns; ++c) {
        th.emplace_back([&, c] {
            ConnStats &s = st[c];
            s.lat_us10.reserve(1 << 20);
            const int fd = socket(AF_INET, SOCK_STREAM, 0);
            sockaddr_in sa{};
            sa.sin_family = AF_INET;
            sa.sin_port = htons((uint16_t)port);
            inet_pton(AF_INET, host.c_str(), &sa.sin_addr);
            int one = 1;
            if (fd < 0 || connect(fd, (sockaddr *)&sa, sizeof sa) != 0) {
                s.failed = true;
                ready.fetch_add(1);
                return;
            }
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
            Rng rng(1000 + c);
            std::vector<int64_t> start((size_t)inflight, 0);  // by xid % inflight (replies come in order)
            std::vector<uint8_t> out((size_t)inflight * FLOW_FRAME), in(1 << 16);
            size_t have = 0;
            int64_t sent = 0, recvd = 0;
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            bool sending = true;
            for (;;) {
                if (sending && now_ns() >= end_ns) sending = false;
                // top up to D in flight with one write
                if (sending && sent - recvd < inflight) {
                    size_t len = 0;
                    const int64_t t = now_ns();
                    while (sent - recvd < inflight) {
                        uint8_t *p = out.data() + len;
                        const double u = rng.uni();
                        const int64_t fid = perm[std::min<size_t>(std::upper_bound(cdf.begin(), cdf.end(), u) - cdf.begin(),
                                                                  (size_t)flows - 1)];
                        put_be(p, FLOW_FRAME - 2, 2);
                        put_be(p + 2, (uint32_t)sent, 4);
                        p[6] = 1;
                        put_be(p + 7, (uint64_t)fid, 8);
                        put_be(p + 15, 1, 4);
                        p[19] = 0;
                        start[(size_t)(sent % inflight)] = t;
                        len += FLOW_FRAME;
                        ++sent;
                    }
                    size_t off = 0;
                    while (off < len) {
                        const ssize_t w = send(fd, out.data() + off, len - off, MSG_NOSIGNAL);
                        if (w <= 0) { s.failed = true; break; }
                        off += (size_t)w;
                    }
                    if (s.failed) break;
                }
                if (!sending && recvd == sent) break;
                const ssize_t r = recv(fd, in.data() + have, in.size() - have, 0);
                if (r <= 0) { s.failed = true; break; }
                have += (size_t)r;
                size_t pos = 0;
                const int64_t t = now_ns();
                while (have - pos >= 2) {
                    const size_t flen = (size_t)get_be(in.data() + pos, 2);
                    if (have - pos < 2 + flen) break;
                    const uint8_t *b = in.data() + pos + 2;
                    if (flen >= 6) {
                        const int64_t xid = (int64_t)(uint32_t)get_be(b, 4);
                        const int8_t status = (int8_t)b[5];
                        if (xid != (recvd & 0xFFFFFFFFll)) s.bad++;
                        s.lat_us10.push_back((uint32_t)std::min<int64_t>((t - start[(size_t)(recvd % inflight)]) / 100,
                                                                         0xFFFFFFFF));
                        if (status == 0) s.ok++;
                        else if (status == 1) s.blocked++;
                        else s.other++;
                        ++recvd;
                    }
                    pos += 2 + flen;
                }
                memmove(in.data(), in.data() + pos, have - pos);
                have -= pos;
            }
            close(fd);
        });
    }
    while (ready.load() < conns) std::this_thread::yield();
    const int64_t tg = now_ns();
    go.store(true, std::memory_order_release);
    for (auto &x : th) x.join();
    const double el = (now_ns() - tg) / 1e9;
    std::vector<uint32_t> all;
    int64_t ok = 0, blk = 0, oth = 0, bad = 0, failed = 0;
    for (auto &s : st) {
        all.insert(all.end(), s.lat_us10.begin(), s.lat_us10.end());
        ok += s.ok; blk += s.blocked; oth += s.other; bad += s.bad; failed += s.failed;
    }
    const int64_t n = (int64_t)all.size();
    const double p50 = pct(all, 0.50), p99 = pct(all, 0.99), p999 = pct(all, 0.999);
    const double mx = all.empty() ? 0.0 : *std::max_element(all.begin(), all.end()) / 10.0;
    printf("{\"bench\": \"wire_client\", \"conns\": %d, \"inflight_per_conn\": %d, \"flows\": %d, \"seconds\": %.3f, "
           "\"requests\": %lld, \"decisions_per_s\": %.1f, \"latency_us\": {\"p50\": %.1f, \"p99\": %.1f, "
           "\"p999\": %.1f, \"max\": %.1f}, \"client_budget_ms\": 20, \"ok\": %lld, \"blocked\": %lld, "
           "\"other\": %lld, \"out_of_order\": %lld, \"failed_conns\": %lld}\n",
           conns, inflight, flows, el, (long long)n, n / el, p50, p99, p999, mx, (long long)ok, (long long)blk,
           (long long)oth, (long long)bad, (long long)failed);
    return failed ? 1 : 0;
}
