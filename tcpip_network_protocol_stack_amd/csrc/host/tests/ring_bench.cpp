// ring_bench.cpp — receive-path rate of batched datagram I/O + GPU verify
// (SURVEY §8f rank 4).  A writer thread streams 64 Ki valid 1500-byte TCP/IPv4
// wire datagrams, `passes` times, over a SOCK_SEQPACKET socketpair; the
// receiver either only reads (the socket's own ceiling), reads then verifies
// one arena at a time (DatagramBatch), or reads into a ring of arenas on a
// reader thread while it verifies the previous one (DatagramRing).  Prints one
// JSON line per mode.  Needs a GPU.
//   build/ring_bench [passes]
#include <sys/socket.h>
#include <unistd.h>

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

void writer(int fd, const std::vector<std::string>& wires, size_t passes)
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
    close(fd);
}

void big_buffers(int fd)
{
    const int sz = 16 << 20;
    (void)setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
    (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
}

template <class Receive>
void run(const char* mode, const std::vector<std::string>& wires, size_t passes, Receive receive)
{
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) != 0) {
        std::perror("socketpair");
        std::exit(1);
    }
    big_buffers(sv[0]);
    big_buffers(sv[1]);
    const auto t0 = std::chrono::steady_clock::now();
    std::thread w(writer, sv[0], std::cref(wires), passes);
    size_t accepted = 0;
    const size_t got = receive(sv[1], accepted);
    w.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    close(sv[1]);
    const double bytes = double(got) * double(wires[0].size());
    std::printf("{\"mode\": \"%s\", \"datagrams\": %zu, \"accepted\": %zu, \"seconds\": %.4f, "
                "\"Mdgram_s\": %.3f, \"GB_s\": %.3f}\n",
                mode, got, accepted, s, got / s / 1e6, bytes / s / 1e9);
    if (got != wires.size() * passes || (accepted != 0 && accepted != got)) std::exit(2);
}

}  // namespace

int main(int argc, char** argv)
{
    const size_t passes = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 4;
    icsum::BatchEngine eng(0);
    const auto wires = make_wires(eng, size_t(1) << 16);
    constexpr size_t kBatch = 1 << 14;  // datagrams per arena (24 MB of 1500-byte datagrams)

    run("read_only", wires, passes, [&](int fd, size_t&) {
        icsum::DatagramBatch rxb(eng, size_t(32) << 20, kBatch);
        size_t n = 0;
        while (true) {
            rxb.clear();
            const size_t k = rxb.read_from(fd, kBatch);
            if (k == 0) break;
            n += k;
        }
        return n;
    });
    run("read_then_verify", wires, passes, [&](int fd, size_t& accepted) {
        icsum::DatagramBatch rxb(eng, size_t(32) << 20, kBatch);
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
    run("ring_3x_verify", wires, passes, [&](int fd, size_t& accepted) {
        icsum::DatagramRing ring(eng, fd, 3, size_t(32) << 20, kBatch);
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
