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
//   build/ring_bench [passes] [seqpacket|udp] [writers]
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
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

std::atomic<bool> g_rx_done{false};
std::atomic<int> g_writers_left{0};

// the last writer to finish ends the stream (close, or UDP end markers)
void writer(int fd, const std::vector<std::string>& wires, size_t passes, bool udp)
{
    icsum::DatagramBatch txb(size_t(4) << 20);
    for (size_t p = 0; p < passes; ++p)
        for (size_t i = 0; i < wires.size();) {
            txb.clear();
            size_t j = i;
            for (; j < wires.size() && j - i < 1024 && txb.push(wires[j]); ++j) {
            }
            txb.write_to(fd);
            i = j;
        }
    if (g_writers_left.fetch_sub(1) != 1) return;
    if (udp)  // end marker: an empty datagram, repeated since UDP may drop it
        while (!g_rx_done.load()) {
            (void)send(fd, "", 0, 0);
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
    close(fd);
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

template <class Receive>
void run(const char* mode, const std::vector<std::string>& wires, size_t passes, bool udp, size_t writers,
         Receive receive)
{
    int sv[2];
    if (udp ? !udp_pair(sv) : socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) != 0) {
        std::perror(udp ? "udp socket" : "socketpair");
        std::exit(1);
    }
    big_buffers(sv[0]);
    big_buffers(sv[1]);
    int rcvbuf = 0;
    socklen_t optlen = sizeof rcvbuf;
    (void)getsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &rcvbuf, &optlen);
    g_rx_done = false;
    g_writers_left = static_cast<int>(writers);
    // the receiver sets up its arenas (page-locked allocations take tens of
    // ms) and then calls start(): the clock and the writers start there, so
    // a UDP socket does not overflow while nobody can read it yet
    std::chrono::steady_clock::time_point t0;
    std::vector<std::thread> ws;
    auto start = [&] {
        t0 = std::chrono::steady_clock::now();
        for (size_t k = 0; k < writers; ++k)
            ws.emplace_back(writer, sv[0], std::cref(wires), passes / writers + (k < passes % writers), udp);
    };
    size_t accepted = 0;
    const size_t got = receive(sv[1], accepted, start);
    g_rx_done = true;
    for (auto& w : ws) w.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    close(sv[1]);
    const double bytes = double(got) * double(wires[0].size());
    const size_t sent = wires.size() * passes;
    std::printf("{\"transport\": \"%s\", \"writers\": %zu, \"mode\": \"%s\", \"sent\": %zu, \"datagrams\": %zu, "
                "\"accepted\": %zu, \"rcvbuf\": %d, \"seconds\": %.4f, \"Mdgram_s\": %.3f, \"GB_s\": %.3f}\n",
                udp ? "udp_loopback" : "seqpacket_socketpair", writers, mode, sent, got, accepted, rcvbuf, s, got / s / 1e6,
                bytes / s / 1e9);
    // UDP may drop (reported above); nothing may arrive corrupted or twice
    if ((udp ? got > sent : got != sent) || (accepted != 0 && accepted != got)) std::exit(2);
}

}  // namespace

int main(int argc, char** argv)
{
    const size_t passes = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 4;
    const bool udp = argc > 2 && std::string(argv[2]) == "udp";
    const size_t writers = std::max<size_t>(1, argc > 3 ? std::strtoul(argv[3], nullptr, 10) : 1);
    icsum::BatchEngine eng(0);
    const auto wires = make_wires(eng, size_t(1) << 16);
    constexpr size_t kBatch = 1 << 14;  // datagrams per arena (24 MB of 1500-byte datagrams)

    run("read_only", wires, passes, udp, writers, [&](int fd, size_t&, auto start) {
        icsum::DatagramBatch rxb(eng, size_t(32) << 20, kBatch);
        start();
        size_t n = 0;
        while (true) {
            rxb.clear();
            const size_t k = rxb.read_from(fd, kBatch);
            if (k == 0) break;
            n += k;
        }
        return n;
    });
    run("read_then_verify", wires, passes, udp, writers, [&](int fd, size_t& accepted, auto start) {
        icsum::DatagramBatch rxb(eng, size_t(32) << 20, kBatch);
        start();
        size_t n = 0;
        while (true) {
            rxb.clear();
            const size_t k = rxb.read_from(fd, kBatch);
            if (k == 0) break;
            for (uint8_t st : rxb.verify()) accepted += st == ICS_ST_ACCEPT;
            n += k;
        }
        return n;
    });
    run("ring_3x_verify", wires, passes, udp, writers, [&](int fd, size_t& accepted, auto start) {
        icsum::DatagramRing ring(eng, fd, 3, size_t(32) << 20, kBatch);
        start();
        size_t n = 0;
        while (icsum::DatagramBatch* b = ring.next()) {
            for (uint8_t st : b->verify()) accepted += st == ICS_ST_ACCEPT;
            n += b->size();
            ring.release(b);
        }
        return n;
    });
    return 0;
}
