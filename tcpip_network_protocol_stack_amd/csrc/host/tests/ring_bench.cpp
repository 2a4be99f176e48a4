// ring_bench.cpp — receive-path rate of batched datagram I/O + GPU verify
// (SURVEY §8f rank 4).  A writer thread streams 64 Ki valid 1500-byte TCP/IPv4
// wire datagrams, `passes` times, over a SOCK_SEQPACKET socketpair; the
// receiver either only reads (the socket's own ceiling), reads then verifies
// one arena at a time (DatagramBatch), or reads into a ring of arenas on a
// reader thread while it verifies the previous one (DatagramRing).  Prints one
// JSON line per mode.  Needs a GPU.
//
// Transport `udp` streams the same datagrams as UDP payloads over 127.0.0.1
// instead (a real socket through the kernel's UDP/IP path, as the reference's
// endtoend relay carries datagrams): UDP has no end of stream and may
// drop, so the writer repeats an empty datagram (read_from's end marker) until
// the receiver stops, and the line reports what was sent and what arrived.
// `writers` > 1 splits the passes over that many writer threads on the same
// socket, so the sender side (which does the kernel's per-datagram work on
// loopback) stops being the ceiling and the receive path is measured.
// `readers` > 1 gives every reader its own socket, engine and ring on its own
// thread (writer k sends to socket k % readers; one port per socket stands in
// for SO_REUSEPORT's flow hashing, which would not let the bench end each
// socket's stream), to see whether the host side scales with reading threads.
// `tx` measures the transmit side instead (patch on the GPU, then send):
// one arena at a time vs a DatagramTxRing.
// `verify` times the engine side alone: [readers] threads verifying their
// own 24 MB arena `passes` times (how concurrent engines share PCIe).
// `tick` times the per-tick calls of a stack (1-256 datagrams per call)
// against the per-object CPU path on the drop-in types.
//   build/ring_bench [passes] [seqpacket|udp|tx|verify|unwrap|tick] [writers] [readers]
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "batch.h"
#include "batch_io.h"
#include "icsum.h"

namespace {

std::vector<std::string> make_wires(icsum::BatchEngine& eng, size_t n)
{
    TCPOverIPv4Adapter adapter;
    std::mt19937_64 rng(0x1071);
    std::vector<TCPMessage> msgs(n);
    for (auto& m : msgs) {
        m.sender.seqno = Wrap32{static_cast<uint32_t>(rng())};
        m.sender.payload.resize(1460);
        for (auto& c : m.sender.payload) c = static_cast<char>(rng());
        m.receiver.ackno = Wrap32{static_cast<uint32_t>(rng())};
        m.receiver.window_size = 65535;
    }
    std::vector<std::string> wires;
    wires.reserve(n);
    for (const auto& d : eng.wrap(adapter, msgs)) {
        std::string w;
        for (const auto& piece : serialize(d)) w += piece;
        wires.push_back(std::move(w));
    }
    return wires;
}

// one receiving socket and its writers' end-of-stream bookkeeping
struct Lane {
    int tx = -1, rx = -1;
    std::atomic<int> writers_left{0};
    std::atomic<bool> rx_done{false};
};

// the last writer of a lane ends its stream (close, or UDP end markers)
void writer(Lane& lane, const std::vector<std::string>& wires, size_t passes, bool udp)
{
    icsum::DatagramBatch txb(size_t(4) << 20);
    for (size_t p = 0; p < passes; ++p)
        for (size_t i = 0; i < wires.size();) {
            txb.clear();
            size_t j = i;
            for (; j < wires.size() && j - i < 1024 && txb.push(wires[j]); ++j) {
            }
            txb.write_to(lane.tx);
            i = j;
        }
    if (lane.writers_left.fetch_sub(1) != 1) return;
    if (udp)  // end marker: an empty datagram, repeated since UDP may drop it
        while (!lane.rx_done.load()) {
            (void)send(lane.tx, "", 0, 0);
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
    close(lane.tx);
}

// a connected pair of UDP sockets on 127.0.0.1: sv[0] sends, sv[1] receives
bool udp_pair(int sv[2])
{
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t len = sizeof a;
    sv[0] = socket(AF_INET, SOCK_DGRAM, 0);
    sv[1] = socket(AF_INET, SOCK_DGRAM, 0);
    if (sv[0] < 0 || sv[1] < 0) return false;
    if (bind(sv[1], reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) return false;
    if (getsockname(sv[1], reinterpret_cast<sockaddr*>(&a), &len) != 0) return false;
    return connect(sv[0], reinterpret_cast<sockaddr*>(&a), sizeof a) == 0;
}

void big_buffers(int fd)
{
    const int sz = 16 << 20;
    (void)setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
    (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
}

// `readers` receiving sockets (one receive() call each, on its own thread
// when readers > 1), writer k sending to socket k % readers
// shared: ONE receive() call on all sockets (one engine, one caller thread)
template <class Receive>
void run(const char* mode, const std::vector<std::string>& wires, size_t passes, bool udp, size_t writers,
         std::vector<std::unique_ptr<icsum::BatchEngine>>& engs, bool shared, Receive receive)
{
    const size_t readers = engs.size();
    const size_t callers = shared ? 1 : readers;
    std::vector<Lane> lanes(readers);
    int rcvbuf = 0;
    for (auto& l : lanes) {
        int sv[2];
        if (udp ? !udp_pair(sv) : socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) != 0) {
            std::perror(udp ? "udp socket" : "socketpair");
            std::exit(1);
        }
        l.tx = sv[0];
        l.rx = sv[1];
        big_buffers(l.tx);
        big_buffers(l.rx);
        socklen_t optlen = sizeof rcvbuf;
        (void)getsockopt(l.rx, SOL_SOCKET, SO_RCVBUF, &rcvbuf, &optlen);
    }
    for (size_t k = 0; k < writers; ++k) ++lanes[k % readers].writers_left;
    // each receiver sets up its arenas (page-locked allocations take tens of
    // ms) and then calls start(); the clock and the writers start once every
    // receiver is ready, so no UDP socket overflows while nobody can read it
    std::mutex mu;
    std::condition_variable cv;
    size_t ready = 0;
    bool go = false;
    auto start = [&] {
        std::unique_lock<std::mutex> lock(mu);
        ++ready;
        cv.notify_all();
        cv.wait(lock, [&] { return go; });
    };
    std::vector<size_t> got(callers, 0), accepted(callers, 0);
    std::vector<std::thread> rs;
    for (size_t r = 0; r < callers; ++r)
        rs.emplace_back([&, r] {
            std::vector<int> fds;
            for (size_t k = 0; k < readers; ++k)
                if (shared || k == r) fds.push_back(lanes[k].rx);
            got[r] = receive(fds, *engs[r], accepted[r], start);
            for (size_t k = 0; k < readers; ++k)
                if (shared || k == r) lanes[k].rx_done = true;
        });
    std::chrono::steady_clock::time_point t0;
    std::vector<std::thread> ws;
    {
        std::unique_lock<std::mutex> lock(mu);
        cv.wait(lock, [&] { return ready == callers; });
        t0 = std::chrono::steady_clock::now();
        for (size_t k = 0; k < writers; ++k)
            ws.emplace_back(writer, std::ref(lanes[k % readers]), std::cref(wires),
                            passes / writers + (k < passes % writers), udp);
        go = true;
    }
    cv.notify_all();
    for (auto& t : rs) t.join();
    const auto t1 = std::chrono::steady_clock::now();
    for (auto& w : ws) w.join();
    for (auto& l : lanes) close(l.rx);
    const double s = std::chrono::duration<double>(t1 - t0).count();
    size_t n = 0, acc = 0;
    for (size_t r = 0; r < callers; ++r) {
        n += got[r];
        acc += accepted[r];
    }
    const double bytes = double(n) * double(wires[0].size());
    const size_t sent = wires.size() * passes;
    std::printf("{\"transport\": \"%s\", \"writers\": %zu, \"readers\": %zu, \"mode\": \"%s\", \"sent\": %zu, "
                "\"datagrams\": %zu, \"accepted\": %zu, \"rcvbuf\": %d, \"seconds\": %.4f, \"Mdgram_s\": %.3f, "
                "\"GB_s\": %.3f}\n",
                udp ? "udp_loopback" : "seqpacket_socketpair", writers, readers, mode, sent, n, acc, rcvbuf, s,
                n / s / 1e6, bytes / s / 1e9);
    // UDP may drop (reported above); nothing may arrive corrupted or twice
    if ((udp ? n > sent : n != sent) || (acc != 0 && acc != n)) std::exit(2);
}

// transmit side over a SOCK_SEQPACKET socketpair: the caller fills arenas
// with serialized datagrams whose checksum fields are zero, patches them on
// the GPU and sends them, either in turn (patch_then_send) or through a
// DatagramTxRing whose writer thread sends arena k while the caller fills and
// patches arena k+1; a peer thread reads and checks every datagram
void tx_run(icsum::BatchEngine& eng, const std::vector<std::string>& wires, size_t passes, bool ring)
{
    constexpr size_t kBatch = 1 << 14;
    std::vector<std::string> zeroed(wires);
    for (auto& z : zeroed) z[10] = z[11] = z[36] = z[37] = 0;
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) != 0) {
        std::perror("socketpair");
        std::exit(1);
    }
    big_buffers(sv[0]);
    big_buffers(sv[1]);
    size_t heard = 0, same = 0;
    std::thread peer([&] {
        icsum::DatagramBatch rxb(size_t(32) << 20, kBatch);
        for (;;) {
            rxb.clear();
            const size_t k = rxb.read_from(sv[1], kBatch);
            for (size_t i = 0; i < k; ++i, ++heard) same += rxb[i] == wires[heard % wires.size()];
            if (k == 0 || rxb.ended()) break;
        }
    });
    std::unique_ptr<icsum::DatagramTxRing> tx;
    std::unique_ptr<icsum::DatagramBatch> one;
    if (ring)
        tx = std::make_unique<icsum::DatagramTxRing>(eng, sv[0], 3, size_t(32) << 20, kBatch);
    else
        one = std::make_unique<icsum::DatagramBatch>(eng, size_t(32) << 20, kBatch);
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t p = 0; p < passes; ++p)
        for (size_t i = 0; i < zeroed.size();) {
            icsum::DatagramBatch* b = ring ? tx->acquire() : one.get();
            if (!ring) b->clear();
            for (; i < zeroed.size() && b->push(zeroed[i]); ++i) {
            }
            if (ring) {
                tx->submit(b);
            } else {
                b->patch();
                b->write_to(sv[0]);
            }
        }
    if (ring) tx->flush();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    tx.reset();
    close(sv[0]);
    peer.join();
    close(sv[1]);
    const size_t sent = wires.size() * passes;
    std::printf("{\"transport\": \"seqpacket_socketpair\", \"mode\": \"%s\", \"sent\": %zu, \"datagrams\": %zu, "
                "\"intact\": %zu, \"seconds\": %.4f, \"Mdgram_s\": %.3f, \"GB_s\": %.3f}\n",
                ring ? "tx_ring_3x" : "patch_then_send", sent, heard, same, s, sent / s / 1e6,
                double(sent) * double(wires[0].size()) / s / 1e9);
    if (heard != sent || same != sent) std::exit(2);
}

}  // namespace

int main(int argc, char** argv)
{
    const size_t passes = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 4;
    const bool udp = argc > 2 && std::string(argv[2]) == "udp";
    if (argc > 2 && std::string(argv[2]) == "unwrap") {
        // receive side without a socket: one thread unwraps (GPU verify +
        // host field parse + the adapter's gates) a page-locked arena of
        // 16 Ki datagrams addressed to it, `passes` times
        icsum::BatchEngine eng(0);
        TCPOverIPv4Adapter a, b;
        a.config_mut().source = Address{"10.1.2.3", 4321};
        a.config_mut().destination = Address{"10.9.8.7", 80};
        b.config_mut().source = Address{"10.9.8.7", 80};
        b.config_mut().destination = Address{"10.1.2.3", 4321};
        std::mt19937_64 rng(0x1072);
        std::vector<TCPMessage> msgs(size_t(1) << 14);
        for (auto& m : msgs) {
            m.sender.seqno = Wrap32{static_cast<uint32_t>(rng())};
            m.sender.payload.resize(1460);
            for (auto& c : m.sender.payload) c = static_cast<char>(rng());
            m.receiver.ackno = Wrap32{static_cast<uint32_t>(rng())};
            m.receiver.window_size = 65535;
        }
        icsum::DatagramBatch arena(eng, size_t(32) << 20, msgs.size());
        for (const auto& d : eng.wrap(a, msgs)) {
            std::string w;
            for (const auto& piece : serialize(d)) w += piece;
            arena.push(w);
        }
        size_t ok = 0;
        for (const auto& m : arena.unwrap(b)) ok += m.has_value();  // staging allocated before the clock
        const auto t0 = std::chrono::steady_clock::now();
        for (size_t p = 0; p < passes; ++p)
            for (const auto& m : arena.unwrap(b)) ok += m.has_value();
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"mode\": \"unwrap_only\", \"passes\": %zu, \"arena_MB\": %.1f, \"ms_per_unwrap\": %.3f, "
                    "\"Mdgram_s\": %.3f, \"GB_s\": %.3f, \"accepted\": %zu}\n",
                    passes, arena.bytes() / 1e6, sec * 1e3 / double(passes),
                    double(passes) * double(arena.size()) / sec / 1e6,
                    double(passes) * double(arena.bytes()) / sec / 1e9, ok);
        return ok == (passes + 1) * arena.size() ? 0 : 2;
    }
    if (argc > 2 && std::string(argv[2]) == "tick") {
        // the stack's per-tick calls: the reference reads its TUN fd one
        // datagram per call (util/tuntap/tuntap_adapter.cpp:5-21) inside the
        // socket's event loop (util/tcp_minnow_socket/tcp_minnow_socket.h:
        // 138-164), so a tick carries a few datagrams.  Per tick of k MTU
        // datagrams: the arena's unwrap (GPU verify + host parse + gates) and
        // the engine's wrap, against the per-object path on the drop-in types
        // (parse + unwrap_tcp_in_ip, wrap_tcp_in_ip + serialize) on this core.
        // RING_TICK_SERVER=idle_us: the same with the resident tick server on.
        icsum::BatchEngine eng(0);
        const char* srv_env = std::getenv("RING_TICK_SERVER");
        const uint32_t srv_idle = srv_env ? uint32_t(std::strtoul(srv_env, nullptr, 10)) : 0u;
        if (srv_idle) eng.set_tick_server(srv_idle);
        // RING_TICK_SERVER_BLOCKS=1..8: the server's blocks (default 4: 64 datagrams)
        if (const char* blk = std::getenv("RING_TICK_SERVER_BLOCKS"))
            eng.set_tick_server_blocks(uint32_t(std::strtoul(blk, nullptr, 10)));
        TCPOverIPv4Adapter a, b;
        a.config_mut().source = Address{"10.1.2.3", 4321};
        a.config_mut().destination = Address{"10.9.8.7", 80};
        b.config_mut().source = Address{"10.9.8.7", 80};
        b.config_mut().destination = Address{"10.1.2.3", 4321};
        std::mt19937_64 rng(0x1073);
        std::vector<TCPMessage> msgs(256);
        for (auto& m : msgs) {
            m.sender.seqno = Wrap32{static_cast<uint32_t>(rng())};
            m.sender.payload.resize(1460);
            for (auto& c : m.sender.payload) c = static_cast<char>(rng());
            m.receiver.ackno = Wrap32{static_cast<uint32_t>(rng())};
            m.receiver.window_size = 65535;
        }
        auto p50 = [](std::vector<double> v) {
            std::sort(v.begin(), v.end());
            return v[v.size() / 2];
        };
        using clk = std::chrono::steady_clock;
        auto us = [](clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count(); };
        const size_t iters = passes < 50 ? 2000 : passes;
        for (size_t k : {1, 4, 16, 64, 256}) {
            const std::vector<TCPMessage> km(msgs.begin(), msgs.begin() + static_cast<std::ptrdiff_t>(k));
            icsum::DatagramBatch arena(eng, size_t(1) << 20, k);
            std::vector<std::string> wires;
            for (const auto& d : eng.wrap(a, km)) {
                std::string w;
                for (const auto& piece : serialize(d)) w += piece;
                arena.push(w);
                wires.push_back(w);
            }
            std::vector<double> t_unwrap, t_wrap, t_cpu_unwrap, t_cpu_wrap;
            size_t ok = 0, cpu_ok = 0;
            for (size_t it = 0; it < iters + 20; ++it) {
                auto t0 = clk::now();
                for (const auto& m : arena.unwrap(b)) ok += m.has_value();
                const double u = us(t0);
                t0 = clk::now();
                const auto dg = eng.wrap(a, km);
                const double w = us(t0);
                t0 = clk::now();
                for (const auto& wire : wires) {
                    InternetDatagram d;
                    if (parse(d, std::vector<std::string>{wire})) cpu_ok += b.unwrap_tcp_in_ip(d).has_value();
                }
                const double cu = us(t0);
                t0 = clk::now();
                size_t bytes = 0;
                for (const auto& m : km) {
                    const InternetDatagram d = a.wrap_tcp_in_ip(m);
                    for (const auto& piece : serialize(d)) bytes += piece.size();
                }
                const double cw = us(t0);
                if (dg.size() != k || bytes != k * 1500) return 3;
                if (it >= 20) {
                    t_unwrap.push_back(u);
                    t_wrap.push_back(w);
                    t_cpu_unwrap.push_back(cu);
                    t_cpu_wrap.push_back(cw);
                }
            }
            std::printf("{\"mode\": \"tick\", \"tick_server_idle_us\": %u, \"datagrams\": %zu, \"iters\": %zu, "
                        "\"unwrap_us\": %.2f, \"wrap_us\": %.2f, \"cpu_unwrap_us\": %.2f, \"cpu_wrap_us\": %.2f, "
                        "\"accepted\": %zu, \"cpu_accepted\": %zu}\n",
                        srv_idle, k, iters, p50(t_unwrap), p50(t_wrap), p50(t_cpu_unwrap), p50(t_cpu_wrap), ok, cpu_ok);
            std::fflush(stdout);
            if (ok != (iters + 20) * k || cpu_ok != ok) return 2;
        }
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "csum") {
        // BatchEngine::checksum over 16 Ki 1480-byte segments and
        // compute_checksums over 16 Ki TCP segments (1460-byte payloads)
        icsum::BatchEngine eng(0);
        std::mt19937_64 rng(0x1074);
        const size_t n = size_t(1) << 14;
        std::vector<std::string> raw(n, std::string(1480, '\0'));
        for (auto& r : raw)
            for (auto& c : r) c = static_cast<char>(rng());
        std::vector<std::string_view> views(raw.begin(), raw.end());
        std::vector<TCPSegment> segs(n);
        std::vector<IPv4Header> hdrs(n);
        for (size_t i = 0; i < n; ++i) {
            segs[i].message.sender.payload = raw[i].substr(0, 1460);
            segs[i].message.sender.seqno = Wrap32{static_cast<uint32_t>(rng())};
            hdrs[i].src = static_cast<uint32_t>(rng());
            hdrs[i].dst = static_cast<uint32_t>(rng());
            hdrs[i].len = 1500;
        }
        size_t sink = eng.checksum(views).size();
        eng.compute_checksums(segs, hdrs);
        auto t0 = std::chrono::steady_clock::now();
        for (size_t p = 0; p < passes; ++p) sink += eng.checksum(views)[p % n];
        const double s1 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        t0 = std::chrono::steady_clock::now();
        for (size_t p = 0; p < passes; ++p) eng.compute_checksums(segs, hdrs);
        const double s2 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"mode\": \"csum\", \"passes\": %zu, \"segments\": %zu, \"ms_per_checksum\": %.3f, "
                    "\"ms_per_compute_checksums\": %.3f, \"GB_s_checksum\": %.3f, \"sink\": %zu}\n",
                    passes, n, s1 * 1e3 / double(passes), s2 * 1e3 / double(passes),
                    double(passes) * double(n) * 1480.0 / s1 / 1e9, sink);
        return 0;
    }
    if (argc > 2 && std::string(argv[2]) == "wrap") {
        // transmit side without a socket: BatchEngine::wrap of 16 Ki messages
        // (1460-byte payloads) per call — payloads into the DMA arena, GPU
        // headers + checksums, InternetDatagrams back; const& (payloads
        // copied into the results) and rvalue (moved) overloads
        icsum::BatchEngine eng(0);
        TCPOverIPv4Adapter a;
        a.config_mut().source = Address{"10.1.2.3", 4321};
        a.config_mut().destination = Address{"10.9.8.7", 80};
        std::mt19937_64 rng(0x1073);
        std::vector<TCPMessage> msgs(size_t(1) << 14);
        for (auto& m : msgs) {
            m.sender.seqno = Wrap32{static_cast<uint32_t>(rng())};
            m.sender.payload.resize(1460);
            for (auto& c : m.sender.payload) c = static_cast<char>(rng());
            m.receiver.ackno = Wrap32{static_cast<uint32_t>(rng())};
            m.receiver.window_size = 65535;
        }
        size_t sink = eng.wrap(a, msgs).size();  // staging allocated before the clock
        auto t0 = std::chrono::steady_clock::now();
        for (size_t p = 0; p < passes; ++p) sink += eng.wrap(a, msgs).size();
        const double sec_ref = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        double sec_mv = 0;
        for (size_t p = 0; p < passes; ++p) {
            std::vector<TCPMessage> copy = msgs;  // outside the clock
            t0 = std::chrono::steady_clock::now();
            sink += eng.wrap(a, std::move(copy)).size();
            sec_mv += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        const double bytes = double(msgs.size()) * 1500.0;
        std::printf("{\"mode\": \"wrap\", \"passes\": %zu, \"datagrams\": %zu, \"ms_per_wrap\": %.3f, "
                    "\"ms_per_wrap_rvalue\": %.3f, \"Mdgram_s\": %.3f, \"GB_s\": %.3f, \"sink\": %zu}\n",
                    passes, msgs.size(), sec_ref * 1e3 / double(passes), sec_mv * 1e3 / double(passes),
                    double(passes) * double(msgs.size()) / sec_ref / 1e6, double(passes) * bytes / sec_ref / 1e9,
                    sink);
        return sink == (2 * passes + 1) * msgs.size() ? 0 : 2;
    }
    if (argc > 2 && std::string(argv[2]) == "verify") {
        // engine side alone: `readers` threads, each with its own engine and
        // a page-locked arena of 16 Ki datagrams, verify it `passes` times
        const size_t threads = std::max<size_t>(1, argc > 4 ? std::strtoul(argv[4], nullptr, 10) : 1);
        std::vector<std::unique_ptr<icsum::BatchEngine>> es;
        std::vector<std::unique_ptr<icsum::DatagramBatch>> bs;
        for (size_t r = 0; r < threads; ++r) es.push_back(std::make_unique<icsum::BatchEngine>(0));
        const auto wires = make_wires(*es[0], size_t(1) << 14);
        for (size_t r = 0; r < threads; ++r) {
            bs.push_back(std::make_unique<icsum::DatagramBatch>(*es[r], size_t(32) << 20, size_t(1) << 14));
            for (const auto& w : wires) bs[r]->push(w);
            (void)bs[r]->verify();  // staging allocated before the clock
        }
        std::atomic<size_t> bad{0};
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> ts;
        for (size_t r = 0; r < threads; ++r)
            ts.emplace_back([&, r] {
                for (size_t p = 0; p < passes; ++p)
                    for (uint8_t st : bs[r]->verify()) bad += st != ICS_ST_ACCEPT;
            });
        for (auto& t : ts) t.join();
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const double bytes = double(threads) * double(passes) * double(bs[0]->bytes());
        std::printf("{\"mode\": \"verify_only\", \"threads\": %zu, \"passes\": %zu, \"arena_MB\": %.1f, "
                    "\"ms_per_verify\": %.3f, \"GB_s\": %.3f}\n",
                    threads, passes, bs[0]->bytes() / 1e6, sec * 1e3 / double(passes),
                    bytes / sec / 1e9);
        return bad ? 2 : 0;
    }
    if (argc > 2 && std::string(argv[2]) == "tx") {
        icsum::BatchEngine eng(0);
        const auto wires = make_wires(eng, size_t(1) << 16);
        tx_run(eng, wires, passes, false);
        tx_run(eng, wires, passes, true);
        return 0;
    }
    const size_t readers = std::max<size_t>(1, argc > 4 ? std::strtoul(argv[4], nullptr, 10) : 1);
    // every socket needs a writer to end its stream
    const size_t writers = std::max<size_t>(readers, argc > 3 ? std::strtoul(argv[3], nullptr, 10) : 1);
    // one engine per receiving thread (a context is used by one thread)
    std::vector<std::unique_ptr<icsum::BatchEngine>> engs;
    for (size_t r = 0; r < readers; ++r) engs.push_back(std::make_unique<icsum::BatchEngine>(0));
    const auto wires = make_wires(*engs[0], size_t(1) << 16);
    constexpr size_t kBatch = 1 << 14;  // datagrams per arena (24 MB of 1500-byte datagrams)

    using Fds = const std::vector<int>&;
    run("read_only", wires, passes, udp, writers, engs, false, [&](Fds fds, icsum::BatchEngine& eng, size_t&, auto start) {
        const int fd = fds[0];
        icsum::DatagramBatch rxb(eng, size_t(32) << 20, kBatch);
        start();
        size_t n = 0;
        while (true) {
            rxb.clear();
            const size_t k = rxb.read_from(fd, kBatch);
            n += k;
            if (k == 0 || rxb.ended()) break;
        }
        return n;
    });
    run("read_then_verify", wires, passes, udp, writers, engs, false,
        [&](Fds fds, icsum::BatchEngine& eng, size_t& accepted, auto start) {
        const int fd = fds[0];
        icsum::DatagramBatch rxb(eng, size_t(32) << 20, kBatch);
        start();
        size_t n = 0;
        while (true) {
            rxb.clear();
            const size_t k = rxb.read_from(fd, kBatch);
            if (k) {
                for (uint8_t st : rxb.verify()) accepted += st == ICS_ST_ACCEPT;
                n += k;
            }
            if (k == 0 || rxb.ended()) break;
        }
        return n;
    });
    // one ring per socket (3 arenas, its own engine and caller thread), then
    // with several sockets one ring over all of them (2 * sockets + 1 arenas,
    // one engine, one caller)
    auto ring_receive = [&](Fds fds, icsum::BatchEngine& eng, size_t& accepted, auto start) {
        icsum::DatagramRing ring(eng, fds, 0, size_t(32) << 20, kBatch);
        start();
        size_t n = 0;
        while (icsum::DatagramBatch* b = ring.next()) {
            for (uint8_t st : b->verify()) accepted += st == ICS_ST_ACCEPT;
            n += b->size();
            ring.release(b);
        }
        return n;
    };
    // the ring alone (no GPU pass): its own hand-off cost against read_only
    run("ring_3x_only", wires, passes, udp, writers, engs, false,
        [&](Fds fds, icsum::BatchEngine& eng, size_t&, auto start) {
            icsum::DatagramRing ring(eng, fds, 0, size_t(32) << 20, kBatch);
            start();
            size_t n = 0;
            while (icsum::DatagramBatch* b = ring.next()) {
                n += b->size();
                ring.release(b);
            }
            return n;
        });
    run("ring_3x_verify", wires, passes, udp, writers, engs, false, ring_receive);
    if (readers > 1) run("ring_shared_verify", wires, passes, udp, writers, engs, true, ring_receive);
    return 0;
}
