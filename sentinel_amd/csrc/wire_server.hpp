// wire_server.hpp -- the cluster token server's TCP front end, native (host code, included by
// engine.hip after the batcher).
//
// Replaces the reference's Netty transport (sentinel-cluster-server-default/.../server/):
//   framing   NettyTransportServer.java:89-92   LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2) in,
//                                               LengthFieldPrepender(2) out (big-endian u16 length)
//   requests  codec/DefaultRequestEntityDecoder.java:42-63 [i32 xid][i8 type][data];
//             PingRequestDataDecoder.java:29-39, FlowRequestDataDecoder.java:37-48,
//             ParamFlowRequestDataDecoder.java:35-90
//   responses codec/DefaultResponseEntityWriter.java:35-52, FlowResponseDataWriter.java:30-33,
//             PingResponseDataWriter.java:30-35
//   handling  handler/TokenServerHandler.java:61-106 (PING -> ConnectionManager.addConnection and
//             the namespace's connectedCount; FLOW / PARAM -> the processors, FlowRequestProcessor.java:36-53,
//             ParamFlowRequestProcessor.java:38-55)
// with the byte-level behaviour of sentinel_amd/wire.py (the Python front end, which the tests pin).
//
// Design: io_threads epoll loops own the connections (thread 0 also accepts); a loop decodes every
// frame of a read, stamps each request with the clock, and hands all the read's FLOW requests to the
// batcher in one call (sentinel_batcher_request_tokens_async); the batcher's dispatcher appends each
// verdict's response frame to its connection and, once per decided batch, flushes every touched
// connection with one send().  PARAM requests of a read are decided as one synchronous host batch
// on the loop; PINGs update the namespace's connection set and connectedCount at once (a PING's
// effect applies to the batches launched after it is read).
#pragma once

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <map>
#include <memory>
#include <set>

namespace {

namespace wire {

constexpr int MAX_FRAME = 1024;                      // LengthFieldBasedFrameDecoder maxFrameLength
constexpr int MSG_PING = 0, MSG_FLOW = 1, MSG_PARAM = 2;   // ClusterConstants.java:24-26
constexpr int8_t RESP_BAD = -1, RESP_OK = 0;                // ClusterConstants.java:31-32
enum { T_INT = 0, T_LONG, T_BYTE, T_DOUBLE, T_FLOAT, T_SHORT, T_BOOL, T_STRING };   // :34-41

inline uint64_t be(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 8) | p[i];
    return v;
}
inline void put_be(std::vector<uint8_t> &o, uint64_t v, int n) {
    for (int i = n - 1; i >= 0; --i) o.push_back((uint8_t)(v >> (8 * i)));
}

// Java's new String(bytes, UTF-8): malformed input becomes U+FFFD per maximal subpart; re-encoded,
// so two byte strings that decode to the same String intern to the same key.
inline std::string utf8_canonical(const uint8_t *s, size_t n) {
    std::string o;
    o.reserve(n);
    size_t i = 0;
    auto bad = [&] { o += "\xEF\xBF\xBD"; };
    while (i < n) {
        const uint8_t b = s[i];
        if (b < 0x80) { o.push_back((char)b); ++i; continue; }
        int len;
        uint8_t lo = 0x80, hi = 0xBF;
        if (b >= 0xC2 && b <= 0xDF) len = 2;
        else if (b == 0xE0) { len = 3; lo = 0xA0; }
        else if (b >= 0xE1 && b <= 0xEC) len = 3;
        else if (b == 0xED) { len = 3; hi = 0x9F; }
        else if (b >= 0xEE && b <= 0xEF) len = 3;
        else if (b == 0xF0) { len = 4; lo = 0x90; }
        else if (b >= 0xF1 && b <= 0xF3) len = 4;
        else if (b == 0xF4) { len = 4; hi = 0x8F; }
        else { bad(); ++i; continue; }
        size_t k = 1;
        for (; k < (size_t)len; ++k) {
            if (i + k >= n) break;
            const uint8_t c = s[i + k];
            const uint8_t l = k == 1 ? lo : 0x80, h = k == 1 ? hi : 0xBF;
            if (c < l || c > h) break;
        }
        if (k == (size_t)len) o.append((const char *)s + i, len);
        else bad();
        i += k;
    }
    return o;
}

// StringUtil.isBlank: every char Character.isWhitespace (the space separators except the no-break
// ones, \t \n \u000B \f \r, \u001C-\u001F) -- over canonical UTF-8 (utf8_canonical's output).
inline bool java_blank(const std::string &s) {
    const uint8_t *p = (const uint8_t *)s.data();
    size_t i = 0;
    while (i < s.size()) {
        uint32_t cp;
        const uint8_t b = p[i];
        if (b < 0x80) { cp = b; i += 1; }
        else if (b < 0xE0) { cp = ((b & 0x1Fu) << 6) | (p[i + 1] & 0x3Fu); i += 2; }
        else if (b < 0xF0) { cp = ((b & 0x0Fu) << 12) | ((p[i + 1] & 0x3Fu) << 6) | (p[i + 2] & 0x3Fu); i += 3; }
        else { return false; }                              // supplementary: never whitespace
        const bool ws = (cp >= 0x09 && cp <= 0x0D) || (cp >= 0x1C && cp <= 0x20) || cp == 0x1680 ||
                        (cp >= 0x2000 && cp <= 0x2006) || (cp >= 0x2008 && cp <= 0x200A) || cp == 0x2028 ||
                        cp == 0x2029 || cp == 0x205F || cp == 0x3000;
        if (!ws) return false;
    }
    return true;
}

}  // namespace wire

}  // namespace

// Injective (flowId, Java-typed value) -> 64-bit param key, dense from 1 (the all-ones key is
// reserved by the engine): the native counterpart of wire.py's ParamKeyInterner.
//
// Bounded: every entry remembers the last request time that used it.  Past max_entries, entries idle
// for longer than idle_ms are forgotten -- exact whenever idle_ms >= every param rule's interval: such
// a value has no valid bucket left (LeapArray.values keeps t - start <= interval, LeapArray.java:375-390),
// so its next request under a fresh key reads the same empty window the reference's CacheMaps give it
// (the engine reclaims the old key's slot as dead, param_table.hpp).  If a flood of distinct values
// inside the horizon still exceeds the cap, the least recently used entries go (the reference bounds
// the same per-rule maps by LRU eviction, ConcurrentLinkedHashMapWrapper.java:35-43: parity unpinned
// there, as for the engine's own tables).
struct sentinel_param_interner {
    struct Ent { uint64_t key; int64_t last; };
    std::mutex mu;
    std::unordered_map<std::string, Ent> ids;
    uint64_t next_id = 1;
    int64_t max_entries = (int64_t)1 << 23;
    int64_t idle_ms = 60000;
    int64_t now = INT64_MIN;                 // the newest request time seen
    int64_t evicted = 0;

    int64_t scans = 0;                       // full passes over the map (each frees >= cap / 4 entries)

    // Called when the map is full.  Every pass ends at or below the 3/4 low-water mark, so the next one
    // comes only after cap / 4 more inserts: O(1) amortised per insert even under a steady flood of
    // distinct values that expire one by one (an idle pass that freed a single entry used to leave the
    // map full, and every following insert rescanned it).
    void shrink_locked() {
        ++scans;
        const int64_t horizon = now == INT64_MIN ? INT64_MIN : now - idle_ms;
        for (auto it = ids.begin(); it != ids.end();) {
            if (it->second.last < horizon) { it = ids.erase(it); ++evicted; }
            else ++it;
        }
        const int64_t low = max_entries / 4 * 3;
        if ((int64_t)ids.size() <= low) return;
        // still above the low-water mark: least recently used first, down to it
        std::vector<int64_t> lasts;
        lasts.reserve(ids.size());
        for (auto &kv : ids) lasts.push_back(kv.second.last);
        const size_t drop = ids.size() - (size_t)low;
        std::nth_element(lasts.begin(), lasts.begin() + (drop - 1), lasts.end());
        const int64_t cut = lasts[drop - 1];
        size_t dropped = 0;
        for (auto it = ids.begin(); it != ids.end() && dropped < drop;) {
            if (it->second.last <= cut) { it = ids.erase(it); ++dropped; ++evicted; }
            else ++it;
        }
    }

    // canonical value: Java equals() semantics -- the type tag is part of the key, NaNs collapse to
    // doubleToLongBits / floatToIntBits' canonical NaN, booleans to 0 / 1, strings by their decoded text
    static bool canonical(int type, const uint8_t *v, int32_t len, std::string &out) {
        uint64_t x;
        switch (type) {
            case wire::T_INT: if (len != 4) return false; out.assign((const char *)v, 4); return true;
            case wire::T_LONG: if (len != 8) return false; out.assign((const char *)v, 8); return true;
            case wire::T_BYTE: if (len != 1) return false; out.assign((const char *)v, 1); return true;
            case wire::T_SHORT: if (len != 2) return false; out.assign((const char *)v, 2); return true;
            case wire::T_BOOL: if (len != 1) return false; out.assign(1, v[0] != 0 ? '\1' : '\0'); return true;
            case wire::T_DOUBLE:
                if (len != 8) return false;
                x = wire::be(v, 8);
                if ((x & 0x7FF0000000000000ull) == 0x7FF0000000000000ull && (x & 0x000FFFFFFFFFFFFFull)) x = 0x7FF8000000000000ull;
                out.clear();
                for (int i = 7; i >= 0; --i) out.push_back((char)(x >> (8 * i)));
                return true;
            case wire::T_FLOAT:
                if (len != 4) return false;
                x = wire::be(v, 4);
                if ((x & 0x7F800000u) == 0x7F800000u && (x & 0x007FFFFFu)) x = 0x7FC00000u;
                out.clear();
                for (int i = 3; i >= 0; --i) out.push_back((char)(x >> (8 * i)));
                return true;
            case wire::T_STRING: out = wire::utf8_canonical(v, (size_t)len); return true;
            default: return false;
        }
    }

    // ts: the request's time (INT64_MIN: the newest time seen so far)
    bool key(int64_t flow_id, int type, const uint8_t *v, int32_t len, uint64_t &k, int64_t ts = INT64_MIN) {
        std::string c;
        if (!canonical(type, v, len, c)) return false;
        std::string s(9, '\0');
        for (int i = 0; i < 8; ++i) s[i] = (char)((uint64_t)flow_id >> (8 * (7 - i)));
        s[8] = (char)type;
        s += c;
        std::lock_guard<std::mutex> g(mu);
        if (ts > now) now = ts;
        const int64_t t = ts == INT64_MIN ? now : ts;
        auto it = ids.find(s);
        if (it != ids.end()) {
            if (t > it->second.last) it->second.last = t;
            k = it->second.key;
            return true;
        }
        if ((int64_t)ids.size() >= max_entries) shrink_locked();
        k = next_id++;
        if (k == ~0ull) k = next_id++;              // (the reserved all-ones key: never reached in practice)
        ids.emplace(std::move(s), Ent{k, t});
        return true;
    }
};

struct sentinel_wire_server;

namespace {
namespace wire {

struct Conn {
    int fd = -1;
    int loop = 0;
    std::string addr;                   // "ip:port" (ConnectionManager's address)
    std::vector<uint8_t> rbuf;          // loop thread only
    size_t discard = 0;                 // bytes of a too-long frame still to skip (loop only)
    std::mutex wmu;                     // wbuf, want_out, closed, fd use for sends
    std::vector<uint8_t> wbuf;
    bool want_out = false;
    bool closed = false;
    std::atomic<bool> dirty{false};     // queued for the dispatcher's end-of-batch flush
    std::atomic<int> refs{1};           // the loop's + one per flow request in flight + flush list
};

inline void unref(Conn *c) {
    if (c->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete c;
}

struct Loop {
    int ep = -1;
    int evfd = -1;
    std::thread th;
    std::set<Conn *> conns;             // open connections of this loop (loop thread only)
};

}  // namespace wire
}  // namespace

struct sentinel_wire_server {
    sentinel_engine_t *e = nullptr;
    sentinel_batcher_t *b = nullptr;
    sentinel_param_interner *interner = nullptr;
    bool own_interner = false;
    sentinel_clock_fn clock = nullptr;
    void *clock_ctx = nullptr;
    int lfd = -1;
    int32_t port = 0;
    std::vector<std::unique_ptr<wire::Loop>> loops;
    std::atomic<bool> stopping{false};
    std::atomic<uint32_t> rr{0};
    std::map<std::string, int32_t> ns_index;
    std::mutex conn_mu;                 // ConnectionManager: namespace -> addresses
    std::map<std::string, std::set<std::string>> ns_conns;
    std::vector<wire::Conn *> flush;    // dispatcher thread only
    std::atomic<int64_t> n_flow{0}, n_param{0};
    std::atomic<int32_t> n_conns{0};

    int64_t now_ms() {
        if (clock) return clock(clock_ctx);
        return std::chrono::duration_cast<std::chrono::milliseconds>(
                   std::chrono::system_clock::now().time_since_epoch()).count();   // TimeUtil
    }

    // ---- sending (any thread; under the connection's wmu)
    void send_locked(wire::Conn *c) {
        if (c->closed) { c->wbuf.clear(); return; }
        size_t off = 0;
        while (off < c->wbuf.size()) {
            const ssize_t w = ::send(c->fd, c->wbuf.data() + off, c->wbuf.size() - off, MSG_NOSIGNAL);
            if (w > 0) { off += (size_t)w; continue; }
            if (w < 0 && errno == EINTR) continue;
            break;                                      // EAGAIN (or an error the loop will see)
        }
        c->wbuf.erase(c->wbuf.begin(), c->wbuf.begin() + off);
        const bool want = !c->wbuf.empty();
        if (want != c->want_out) {
            c->want_out = want;
            epoll_event ev{};
            ev.events = EPOLLIN | (want ? EPOLLOUT : 0);
            ev.data.ptr = c;
            (void)epoll_ctl(loops[c->loop]->ep, EPOLL_CTL_MOD, c->fd, &ev);
        }
    }

    // [u16 len][i32 xid][i8 type][i8 status] + `words` big-endian i32s (0: a BAD response, no data)
    static void response(std::vector<uint8_t> &o, int32_t xid, int type, int8_t status, int words, int32_t a = 0,
                         int32_t b2 = 0) {
        wire::put_be(o, (uint64_t)(6 + 4 * words), 2);
        wire::put_be(o, (uint32_t)xid, 4);
        o.push_back((uint8_t)type);
        o.push_back((uint8_t)status);
        if (words >= 1) wire::put_be(o, (uint32_t)a, 4);
        if (words >= 2) wire::put_be(o, (uint32_t)b2, 4);
    }

    // ---- the batcher's side: one response per decided flow request, one flush per batch
    static void on_flow(void *ctx, uint64_t tag, const sentinel_token_result_t *r) {
        ((sentinel_wire_server *)ctx)->flow_done(tag, r);
    }
    void flow_done(uint64_t tag, const sentinel_token_result_t *r);
    static void on_batch(void *ctx) { ((sentinel_wire_server *)ctx)->flush_all(); }
    void flush_all() {
        for (wire::Conn *c : flush) {
            {
                std::lock_guard<std::mutex> g(c->wmu);
                c->dirty.store(false, std::memory_order_relaxed);
                if (!c->want_out) send_locked(c);       // else the loop's EPOLLOUT drains it
            }
            wire::unref(c);
        }
        flush.clear();
    }

    // ---- the loop's side
    void close_conn(wire::Loop &L, wire::Conn *c) {
        {
            std::lock_guard<std::mutex> g(c->wmu);
            if (c->closed) return;
            c->closed = true;
            (void)epoll_ctl(L.ep, EPOLL_CTL_DEL, c->fd, nullptr);
            ::close(c->fd);
            c->wbuf.clear();
        }
        L.conns.erase(c);
        n_conns.fetch_sub(1);
        {   // ConnectionManager.removeConnection: every namespace that held the address
            std::lock_guard<std::mutex> g(conn_mu);
            for (auto &kv : ns_conns)
                if (kv.second.erase(c->addr)) set_count(kv.first, (int32_t)kv.second.size());
        }
        wire::unref(c);
    }
    void set_count(const std::string &ns, int32_t n) {
        auto it = ns_index.find(ns);
        if (it != ns_index.end()) (void)sentinel_set_connected_count(e, it->second, n);
    }

    void accept_all() {
        for (;;) {
            sockaddr_in sa{};
            socklen_t sl = sizeof sa;
            const int fd = accept4(lfd, (sockaddr *)&sa, &sl, SOCK_NONBLOCK | SOCK_CLOEXEC);
            if (fd < 0) {
                if (errno == EINTR) continue;
                return;
            }
            int one = 1;
            setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
            wire::Conn *c = new wire::Conn();
            c->fd = fd;
            char ip[64];
            inet_ntop(AF_INET, &sa.sin_addr, ip, sizeof ip);
            c->addr = std::string(ip) + ":" + std::to_string(ntohs(sa.sin_port));
            c->loop = (int)(rr.fetch_add(1) % loops.size());
            n_conns.fetch_add(1);
            // the owning loop registers it (its conns set is loop-private): hand over through epoll
            wire::Loop &L = *loops[c->loop];
            {
                std::lock_guard<std::mutex> g(pending_mu);
                pending.emplace_back(c->loop, c);
            }
            const uint64_t one64 = 1;
            (void)::write(L.evfd, &one64, 8);
        }
    }
    std::mutex pending_mu;
    std::vector<std::pair<int, wire::Conn *>> pending;

    void adopt(int li) {
        wire::Loop &L = *loops[li];
        std::vector<wire::Conn *> mine;
        {
            std::lock_guard<std::mutex> g(pending_mu);
            for (size_t i = 0; i < pending.size();) {
                if (pending[i].first == li) { mine.push_back(pending[i].second); pending.erase(pending.begin() + i); }
                else ++i;
            }
        }
        for (wire::Conn *c : mine) {
            L.conns.insert(c);
            epoll_event ev{};
            ev.events = EPOLLIN;
            ev.data.ptr = c;
            if (epoll_ctl(L.ep, EPOLL_CTL_ADD, c->fd, &ev) != 0) close_conn(L, c);
        }
    }

    bool on_readable(wire::Loop &L, wire::Conn *c);    // false: the connection was closed
    void run_loop(int li);
};

namespace {
namespace wire {

// Per-read scratch of a loop: the read's FLOW requests (one batcher call) and PARAM requests (one
// host batch), in arrival order.
struct ReadBatch {
    std::vector<int64_t> fid, fts;
    std::vector<int32_t> facq;
    std::vector<uint8_t> fprio;
    std::vector<uint64_t> ftag;
    std::vector<int64_t> pfid;
    std::vector<int32_t> pxid;
    std::vector<sentinel_param_multi_event_t> pev;
    std::vector<uint64_t> pvals;
    std::vector<int32_t> pnorule;                 // < 0: the flowId's lookup when decoded (NO_RULE / BAD_ID)
    std::unordered_map<int64_t, int32_t> prule_cache;   // flowId -> param rule index, this read
    void clear() {
        fid.clear(); fts.clear(); facq.clear(); fprio.clear(); ftag.clear();
        pfid.clear(); pxid.clear(); pev.clear(); pvals.clear(); pnorule.clear(); prule_cache.clear();
    }
};

}  // namespace wire
}  // namespace

// A flow request in flight (the batcher tag points to it): its connection (one reference held) and xid.
struct WireFlowTag {
    wire::Conn *c;
    int32_t xid;
};

inline void sentinel_wire_server::flow_done(uint64_t tag, const sentinel_token_result_t *r) {
    WireFlowTag *t = (WireFlowTag *)(uintptr_t)tag;
    wire::Conn *c = t->c;
    {
        std::lock_guard<std::mutex> g(c->wmu);
        if (!c->closed)
            response(c->wbuf, t->xid, wire::MSG_FLOW, (int8_t)r->status, 2, r->remaining, r->wait_in_ms);
    }
    delete t;
    if (!c->dirty.exchange(true, std::memory_order_acq_rel)) flush.push_back(c);   // keeps the request's ref
    else wire::unref(c);
}

inline bool sentinel_wire_server::on_readable(wire::Loop &L, wire::Conn *c) {
    uint8_t tmp[65536];
    bool eof = false;
    // at most 4 x 64 KB per readiness event (level-triggered: the rest raises the next one), so one
    // client streaming requests cannot hold this loop thread or grow its buffer without bound
    for (int reads = 0; reads < 4; ++reads) {
        const ssize_t r = ::recv(c->fd, tmp, sizeof tmp, 0);
        if (r > 0) { c->rbuf.insert(c->rbuf.end(), tmp, tmp + r); if ((size_t)r < sizeof tmp) break; continue; }
        if (r == 0) { eof = true; break; }
        if (errno == EINTR) continue;
        if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
        break;
    }
    static thread_local wire::ReadBatch B;
    B.clear();
    std::vector<uint8_t> &buf = c->rbuf;
    size_t pos = 0;
    std::vector<uint8_t> direct;                           // PING replies, written after the read
    const int64_t ts = now_ms();                           // TimeUtil at decode (one read = one instant)
    for (;;) {
        if (c->discard) {
            const size_t d = std::min(c->discard, buf.size() - pos);
            pos += d;
            c->discard -= d;
            if (c->discard) break;
        }
        if (buf.size() - pos < 2) break;
        const size_t len = (size_t)wire::be(&buf[pos], 2);
        if (len + 2 > (size_t)wire::MAX_FRAME) {            // TooLongFrameException: skip the frame
            pos += 2;
            c->discard = len;
            continue;
        }
        if (buf.size() - pos < 2 + len) break;
        const uint8_t *f = &buf[pos + 2];
        pos += 2 + len;
        if (len < 5) continue;                             // no xid + type: nothing decoded
        const int32_t xid = (int32_t)wire::be(f, 4);
        const int type = (int8_t)f[4];
        const uint8_t *d = f + 5;
        const size_t dl = len - 5;
        if (type == wire::MSG_PING) {
            // PingRequestDataDecoder: [i32 len][bytes]; blank / absent namespace -> BAD
            std::string ns;
            bool have = false;
            if (dl >= 4) {
                const int32_t L2 = (int32_t)wire::be(d, 4);
                if (L2 > 0 && dl > 4) {
                    if ((size_t)L2 > dl - 4) continue;    // readerIndex out of bounds: dropped
                    ns = wire::utf8_canonical(d + 4, (size_t)L2);
                    have = true;
                }
            }
            const bool blank = wire::java_blank(ns);
            if (!have || blank) {
                response(direct, xid, wire::MSG_PING, wire::RESP_BAD, 0);
                continue;
            }
            int32_t count;
            {
                std::lock_guard<std::mutex> g(conn_mu);
                auto &set = ns_conns[ns];
                set.insert(c->addr);
                count = (int32_t)set.size();
                set_count(ns, count);
            }
            response(direct, xid, wire::MSG_PING, wire::RESP_OK, 1, count);
        } else if (type == wire::MSG_FLOW) {
            if (dl < 12) continue;                         // null data: FlowRequestProcessor NPE, no reply
            B.fid.push_back((int64_t)wire::be(d, 8));
            B.facq.push_back((int32_t)wire::be(d + 8, 4));
            B.fprio.push_back(dl >= 13 && d[12] != 0);
            B.fts.push_back(ts);
            c->refs.fetch_add(1, std::memory_order_relaxed);
            B.ftag.push_back((uint64_t)(uintptr_t)new WireFlowTag{c, xid});
        } else if (type == wire::MSG_PARAM) {
            if (dl < 16) continue;                         // null data: no reply
            const int64_t fid = (int64_t)wire::be(d, 8);
            const int32_t cnt = (int32_t)wire::be(d + 8, 4);
            const int32_t amount = (int32_t)wire::be(d + 12, 4);
            if (amount <= 0) continue;                     // null data
            // no rule for the flowId: NO_RULE_EXISTS (DefaultTokenService.java:57-60) without interning
            // anything (untrusted values of unknown flowIds never reach the interner)
            auto rit = B.prule_cache.find(fid);
            if (rit == B.prule_cache.end()) {
                int32_t ridx = -1;
                if (sentinel_lookup_param_idx(e, 1, &fid, &ridx) != 0) ridx = SENTINEL_IDX_NO_RULE;
                rit = B.prule_cache.emplace(fid, ridx).first;
            }
            const bool has_rule = rit->second >= 0;
            size_t q = 16;
            bool ok = true;
            const size_t v0 = B.pvals.size();
            for (int32_t k = 0; k < amount && ok; ++k) {
                if (q + 1 > dl) { ok = false; break; }
                const int t = (int8_t)d[q++];
                int32_t w;
                switch (t) {
                    case wire::T_INT: case wire::T_FLOAT: w = 4; break;
                    case wire::T_LONG: case wire::T_DOUBLE: w = 8; break;
                    case wire::T_BYTE: case wire::T_BOOL: w = 1; break;
                    case wire::T_SHORT: w = 2; break;
                    case wire::T_STRING:
                        if (q + 4 > dl) { ok = false; continue; }
                        w = (int32_t)wire::be(d + q, 4);
                        q += 4;
                        if (w < 0) { ok = false; continue; }
                        break;
                    default: continue;                     // unknown type: only its byte consumed
                }
                if (q + (size_t)w > dl) { ok = false; break; }
                uint64_t key = 1;
                if (has_rule) interner->key(fid, t, d + q, w, key, ts);
                B.pvals.push_back(key);
                q += (size_t)w;
            }
            if (!ok) { B.pvals.resize(v0); continue; }   // truncated: Netty raises, nothing handled
            sentinel_param_multi_event_t pe{};
            pe.acquire = cnt;
            pe.ts = ts;
            pe.value_begin = (int32_t)v0;
            pe.value_count = (int32_t)(B.pvals.size() - v0);
            B.pev.push_back(pe);
            B.pfid.push_back(fid);
            B.pxid.push_back(xid);
            B.pnorule.push_back(has_rule ? 0 : rit->second);
        }
        // any other type: no decoder, nothing emitted
    }
    buf.erase(buf.begin(), buf.begin() + pos);
    // the read's flow requests -> the batcher in one call
    if (!B.fid.empty()) {
        n_flow.fetch_add((int64_t)B.fid.size());
        const int rc = sentinel_batcher_request_tokens_async(b, (int32_t)B.fid.size(), B.fid.data(), B.facq.data(),
                                                             B.fprio.data(), B.fts.data(), on_flow, this, B.ftag.data());
        if (rc) {                                          // batcher stopped: drop them
            for (uint64_t t : B.ftag) {
                WireFlowTag *w = (WireFlowTag *)(uintptr_t)t;
                wire::unref(w->c);
                delete w;
            }
        }
    }
    // the read's param requests -> one host batch
    if (!B.pev.empty()) {
        const int64_t n = (int64_t)B.pev.size();
        n_param.fetch_add(n);
        std::vector<int32_t> idx(n);
        std::vector<sentinel_verdict_t> out(n);
        int rc = sentinel_lookup_param_idx(e, n, B.pfid.data(), idx.data());
        // a flowId without a rule keeps its decode-time lookup: SENTINEL_IDX_BAD_ID for flowId <= 0 answers
        // BAD_REQUEST (DefaultTokenService.notValidRequest runs before the rule lookup), NO_RULE otherwise
        for (int64_t i = 0; i < n; ++i) B.pev[i].rule_idx = B.pnorule[i] < 0 ? B.pnorule[i] : idx[i];
        bool single = true;                                // every request one value: the single-value key walk
        for (int64_t i = 0; i < n && single; ++i) single = B.pev[i].value_count == 1;
        if (single) {
            // decide-order output (sentinel_submit_param_batch_ordered_host): verdict j answers request
            // seq[j]; each response carries its own xid (TokenServerHandler.java:61-81), so the read's
            // responses go out in the order the engine decided them
            std::vector<sentinel_param_event_t> sev(n);
            std::vector<uint32_t> seq(n);
            for (int64_t i = 0; i < n; ++i)
                sev[i] = sentinel_param_event_t{B.pev[i].rule_idx, B.pev[i].acquire, B.pev[i].ts,
                                                B.pvals[(size_t)B.pev[i].value_begin]};
            if (!rc) rc = sentinel_submit_param_batch_ordered_host(e, n, sev.data(), out.data(), seq.data());
            for (int64_t j = 0; j < n; ++j) {
                const int64_t i = rc ? j : (int64_t)seq[j];
                response(direct, B.pxid[i], wire::MSG_PARAM, rc ? (int8_t)SENTINEL_STATUS_FAIL : (int8_t)out[j].status, 2,
                         rc ? 0 : out[j].remaining, 0);
            }
        } else {
            if (!rc) rc = sentinel_submit_param_multi_batch_host(e, n, B.pev.data(), B.pvals.data(),
                                                                 (int64_t)B.pvals.size(), out.data());
            for (int64_t i = 0; i < n; ++i)
                response(direct, B.pxid[i], wire::MSG_PARAM, rc ? (int8_t)SENTINEL_STATUS_FAIL : (int8_t)out[i].status, 2,
                         rc ? 0 : out[i].remaining, 0);
        }
    }
    if (!direct.empty()) {
        std::lock_guard<std::mutex> g(c->wmu);
        c->wbuf.insert(c->wbuf.end(), direct.begin(), direct.end());
        if (!c->want_out) send_locked(c);
    }
    if (eof) {
        close_conn(L, c);
        return false;
    }
    return true;
}

inline void sentinel_wire_server::run_loop(int li) {
    wire::Loop &L = *loops[li];
    epoll_event evs[256];
    while (!stopping.load(std::memory_order_acquire)) {
        const int n = epoll_wait(L.ep, evs, 256, 100);
        for (int i = 0; i < n; ++i) {
            void *p = evs[i].data.ptr;
            if (p == nullptr) {                            // the listening socket (loop 0)
                accept_all();
                continue;
            }
            if (p == (void *)&L) {                         // eventfd: adopt new connections / stop
                uint64_t v;
                (void)::read(L.evfd, &v, 8);
                adopt(li);
                continue;
            }
            wire::Conn *c = (wire::Conn *)p;
            if ((evs[i].events & (EPOLLIN | EPOLLHUP | EPOLLERR)) && !on_readable(L, c)) continue;
            if (evs[i].events & EPOLLOUT) {
                std::lock_guard<std::mutex> g(c->wmu);
                send_locked(c);
            }
        }
    }
}

extern "C" {

int sentinel_param_interner_create(sentinel_param_interner_t **out) {
    if (!out) return fail(SENTINEL_E_INVALID, "null argument");
    *out = new sentinel_param_interner();
    return 0;
}

int sentinel_param_interner_destroy(sentinel_param_interner_t *it) {
    delete it;
    return 0;
}

int sentinel_param_interner_key(sentinel_param_interner_t *it, int64_t flow_id, int32_t type, const uint8_t *value,
                                int32_t len, uint64_t *key) {
    return sentinel_param_interner_key_at(it, flow_id, type, value, len, INT64_MIN, key);
}

int sentinel_param_interner_key_at(sentinel_param_interner_t *it, int64_t flow_id, int32_t type, const uint8_t *value,
                                   int32_t len, int64_t ts, uint64_t *key) {
    if (!it || !key || len < 0 || (len > 0 && !value)) return fail(SENTINEL_E_INVALID, "bad arguments");
    if (!it->key(flow_id, type, value, len, *key, ts)) return fail(SENTINEL_E_INVALID, "unsupported type or value width");
    return 0;
}

int sentinel_param_interner_set_limits(sentinel_param_interner_t *it, int64_t max_entries, int64_t idle_ms) {
    if (!it || max_entries < 4 || idle_ms < 0) return fail(SENTINEL_E_INVALID, "bad interner limits");
    std::lock_guard<std::mutex> g(it->mu);
    it->max_entries = max_entries;
    it->idle_ms = idle_ms;
    if ((int64_t)it->ids.size() > max_entries) it->shrink_locked();
    return 0;
}

int sentinel_param_interner_stats(sentinel_param_interner_t *it, int64_t *entries, int64_t *evicted) {
    if (!it) return fail(SENTINEL_E_INVALID, "null interner");
    std::lock_guard<std::mutex> g(it->mu);
    if (entries) *entries = (int64_t)it->ids.size();
    if (evicted) *evicted = it->evicted;
    return 0;
}

int sentinel_param_interner_scans(sentinel_param_interner_t *it, int64_t *scans) {
    if (!it || !scans) return fail(SENTINEL_E_INVALID, "null interner");
    std::lock_guard<std::mutex> g(it->mu);
    *scans = it->scans;
    return 0;
}

int sentinel_wire_server_create(sentinel_engine_t *e, const sentinel_wire_config_t *cfg, sentinel_wire_server_t **out) {
    if (!e || !cfg || !out || cfg->io_threads < 1 || cfg->io_threads > 64 || cfg->max_batch <= 0 || cfg->max_wait_us < 0 ||
        cfg->n_namespaces < 0 || (cfg->n_namespaces > 0 && !cfg->namespaces))
        return fail(SENTINEL_E_INVALID, "bad wire server config");
    auto *s = new sentinel_wire_server();
    s->e = e;
    s->clock = cfg->clock;
    s->clock_ctx = cfg->clock_ctx;
    s->interner = cfg->interner;
    if (!s->interner) {
        s->interner = new sentinel_param_interner();
        s->own_interner = true;
    }
    for (int32_t i = 0; i < cfg->n_namespaces; ++i)
        if (cfg->namespaces[i]) s->ns_index.emplace(cfg->namespaces[i], i);
    auto bail = [&](const std::string &m) {
        if (s->lfd >= 0) ::close(s->lfd);
        for (auto &L : s->loops) {
            if (L->ep >= 0) ::close(L->ep);
            if (L->evfd >= 0) ::close(L->evfd);
        }
        if (s->b) sentinel_batcher_destroy(s->b);
        if (s->own_interner) delete s->interner;
        delete s;
        return fail(SENTINEL_E_STATE, m);
    };
    if (sentinel_batcher_create(e, cfg->max_batch, cfg->max_wait_us, &s->b)) return bail(sentinel_last_error());
    sentinel_batcher_set_batch_hook(s->b, &sentinel_wire_server::on_batch, s);
    s->lfd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (s->lfd < 0) return bail("socket failed");
    int one = 1;
    setsockopt(s->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)cfg->port);
    if (inet_pton(AF_INET, cfg->host ? cfg->host : "127.0.0.1", &sa.sin_addr) != 1) return bail("bad host address");
    if (bind(s->lfd, (sockaddr *)&sa, sizeof sa) != 0) return bail(std::string("bind: ") + strerror(errno));
    if (listen(s->lfd, 1024) != 0) return bail("listen failed");
    socklen_t sl = sizeof sa;
    getsockname(s->lfd, (sockaddr *)&sa, &sl);
    s->port = ntohs(sa.sin_port);
    for (int32_t i = 0; i < cfg->io_threads; ++i) {
        auto L = std::make_unique<wire::Loop>();
        L->ep = epoll_create1(EPOLL_CLOEXEC);
        L->evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
        if (L->ep < 0 || L->evfd < 0) {
            s->loops.push_back(std::move(L));
            return bail("epoll / eventfd failed");
        }
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.ptr = L.get();
        epoll_ctl(L->ep, EPOLL_CTL_ADD, L->evfd, &ev);
        if (i == 0) {
            epoll_event lev{};
            lev.events = EPOLLIN;
            lev.data.ptr = nullptr;
            epoll_ctl(L->ep, EPOLL_CTL_ADD, s->lfd, &lev);
        }
        s->loops.push_back(std::move(L));
    }
    for (int32_t i = 0; i < cfg->io_threads; ++i) s->loops[i]->th = std::thread([s, i] { s->run_loop(i); });
    *out = s;
    return 0;
}

int32_t sentinel_wire_server_port(sentinel_wire_server_t *s) { return s ? s->port : -1; }

int sentinel_wire_server_stats(sentinel_wire_server_t *s, int64_t *flow_requests, int64_t *param_requests,
                               int64_t *batches, int32_t *connections) {
    if (!s) return fail(SENTINEL_E_INVALID, "null server");
    if (flow_requests) *flow_requests = s->n_flow.load();
    if (param_requests) *param_requests = s->n_param.load();
    if (batches) sentinel_batcher_stats(s->b, batches, nullptr);
    if (connections) *connections = s->n_conns.load();
    return 0;
}

int sentinel_wire_server_destroy(sentinel_wire_server_t *s) {
    if (!s) return 0;
    s->stopping.store(true, std::memory_order_release);
    for (auto &L : s->loops)
        if (L->th.joinable()) L->th.join();
    // requests still in flight are decided (their responses dropped) before the batcher returns
    for (auto &L : s->loops) {
        std::vector<wire::Conn *> cs(L->conns.begin(), L->conns.end());
        for (wire::Conn *c : cs) {
            std::lock_guard<std::mutex> g(c->wmu);
            if (!c->closed) {
                c->closed = true;
                ::close(c->fd);
            }
        }
    }
    sentinel_batcher_destroy(s->b);
    s->flush_all();
    for (auto &L : s->loops) {
        for (wire::Conn *c : std::vector<wire::Conn *>(L->conns.begin(), L->conns.end())) wire::unref(c);
        ::close(L->ep);
        ::close(L->evfd);
    }
    for (auto &p : s->pending) {
        ::close(p.second->fd);
        wire::unref(p.second);
    }
    ::close(s->lfd);
    if (s->own_interner) delete s->interner;
    delete s;
    return 0;
}

}  // extern "C"
