// host_selftest.cpp — CPU checks of the drop-in types, driven line by line by
// tests/test_host_cpp.py with the golden fixtures of the real reference.
//   kat INIT HEX...                -> value (add(vector<string>) == add(vector<string_view>))
//   ipv4 HEX                       -> "ok computed pseudo" from IPv4Header::parse
//   tcpv HEX                       -> "ip_ok tcp_ok tcp_value ip_computed proto" (datagram parse path)
//   wrap SRC SPORT DST DPORT SEQ SYN FIN RST HASACK ACK WIN PAYLOADHEX -> wire hex
//   unwrap SRC SPORT DST DPORT HEX -> "1" if the adapter (source=SRC:SPORT) accepts, else "0"
//   io / ioudp / ioseq HEX...      -> DatagramBatch socket round trips (see below)
//   ringstress F P N               -> engine-less DatagramRing over F SEQPACKET streams, P passes of N
//                                     datagrams each: "got same_order lost_none"
//   txstress P N                   -> engine-less DatagramTxRing to a SEQPACKET stream:
//                                     "sent got same_order failed_patch_recovered"
//   parfor N T                     -> detail::parallel_ranges over [0, N) on T threads: "covered_once
//                                     worker_throw_seen caller_throw_seen"
//   pool N T J                     -> detail::WorkerPool(T - 1), J jobs of N items in T ranges each:
//                                     "covered_once_every_job worker_throw_seen caller_throw_seen"
// The stress commands run the rings' reader / writer threads (and parfor the
// thread pool) with no GPU, so the ASan+UBSan and TSan builds (make asan /
// make tsan) cover their locking.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <iostream>
#include <stdexcept>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include "batch_io.h"
#include "checksum.h"
#include "ipv4_datagram.h"
#include "par_for.h"
#include "parser.h"
#include "tcp_over_ip.h"
#include "tcp_segment.h"

namespace {
std::string unhex(const std::string& h)
{
    std::string s(h.size() / 2, '\0');
    for (size_t i = 0; i < s.size(); ++i) s[i] = static_cast<char>(std::stoi(h.substr(2 * i, 2), nullptr, 16));
    return s;
}
std::string tohex(const std::string& s)
{
    static const char* d = "0123456789abcdef";
    std::string r;
    for (unsigned char c : s) {
        r.push_back(d[c >> 4]);
        r.push_back(d[c & 15]);
    }
    return r;
}
std::string joined(const std::vector<std::string>& v)
{
    std::string r;
    for (auto& s : v) r += s;
    return r;
}
std::string ipstr(uint32_t a) { return Address::from_ipv4_numeric(a).ip(); }

// datagram k of stream f: [f][k, 4 bytes LE][(k*7+f) % 200 bytes of a pattern]
std::string stress_dgram(uint32_t f, uint32_t k)
{
    std::string d(5 + (k * 7 + f) % 200, '\0');
    d[0] = static_cast<char>(f);
    for (int b = 0; b < 4; ++b) d[1 + b] = static_cast<char>(k >> (8 * b));
    for (size_t i = 5; i < d.size(); ++i) d[i] = static_cast<char>(i * 31 + k);
    return d;
}
}  // namespace

int main()
{
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string cmd;
        in >> cmd;
        if (cmd == "pool") {
            size_t n = 0, t = 0, jobs = 0;
            in >> n >> t >> jobs;
            icsum::detail::WorkerPool pool(t > 0 ? t - 1 : 0);
            bool once = true;
            std::vector<std::atomic<int>> hits(n);
            for (size_t j = 0; j < jobs; ++j) {
                for (auto& h : hits) h.store(0, std::memory_order_relaxed);
                pool.run(n, t, [&](size_t i0, size_t i1) {
                    for (size_t i = i0; i < i1; ++i) hits[i].fetch_add(1, std::memory_order_relaxed);
                });
                once = once && std::all_of(hits.begin(), hits.end(), [](const std::atomic<int>& h) { return h.load() == 1; });
            }
            bool worker = false, caller = false;
            try {
                pool.run(n, t, [&](size_t i0, size_t) {
                    if (i0 > 0) throw std::runtime_error("worker");
                });
            } catch (const std::runtime_error& e) {
                worker = std::string(e.what()) == "worker";
            }
            try {
                pool.run(n, t, [&](size_t i0, size_t) {
                    if (i0 == 0) throw std::runtime_error("caller");
                });
            } catch (const std::runtime_error& e) {
                caller = std::string(e.what()) == "caller";
            }
            std::cout << once << " " << (worker || t <= 1 || n < 2) << " " << caller << "\n";
        } else if (cmd == "parfor") {
            size_t n = 0, t = 0;
            in >> n >> t;
            std::vector<std::atomic<int>> hits(n);
            icsum::detail::parallel_ranges(n, t, [&](size_t i0, size_t i1) {
                for (size_t i = i0; i < i1; ++i) hits[i].fetch_add(1, std::memory_order_relaxed);
            });
            bool once = std::all_of(hits.begin(), hits.end(), [](const std::atomic<int>& h) { return h.load() == 1; });
            // an exception in a worker's range and one in the caller's own
            // range (the first) both reach the caller, after every join
            bool worker = false, caller = false;
            try {
                icsum::detail::parallel_ranges(n, t, [&](size_t i0, size_t) {
                    if (i0 > 0) throw std::runtime_error("worker");
                });
            } catch (const std::runtime_error& e) {
                worker = std::string(e.what()) == "worker";
            }
            try {
                icsum::detail::parallel_ranges(n, t, [&](size_t i0, size_t) {
                    if (i0 == 0) throw std::runtime_error("caller");
                });
            } catch (const std::runtime_error& e) {
                caller = std::string(e.what()) == "caller";
            }
            std::cout << once << " " << (worker || t <= 1 || n < 2) << " " << caller << "\n";
        } else if (cmd == "kat") {
            uint64_t init = 0;
            in >> init;
            std::vector<std::string> pieces;
            std::string h;
            while (in >> h) pieces.push_back(h == "-" ? std::string{} : unhex(h));
            InternetChecksum a{static_cast<uint32_t>(init)}, b{static_cast<uint32_t>(init)};
            a.add(pieces);
            std::vector<std::string_view> views(pieces.begin(), pieces.end());
            b.add(views);
            if (a.value() != b.value()) return 2;
            std::cout << a.value() << "\n";
        } else if (cmd == "ipv4") {
            std::string h;
            in >> h;
            IPv4Header hd;
            const bool ok = parse(hd, std::vector<std::string>{unhex(h)});
            std::cout << ok << " " << hd.cksum << " " << (hd.ver == 4 ? hd.pseudo_checksum() : 0u) << "\n";
        } else if (cmd == "tcpv") {
            std::string h;
            in >> h;
            IPv4Datagram dg;
            const bool ip_ok = parse(dg, std::vector<std::string>{unhex(h)});
            TCPSegment seg;
            const uint32_t pseudo = dg.header.pseudo_checksum();
            const bool tcp_ok = parse(seg, dg.payload, pseudo);
            InternetChecksum c{pseudo};
            c.add(dg.payload);
            std::cout << ip_ok << " " << tcp_ok << " " << c.value() << " " << dg.header.cksum << " "
                      << +dg.header.proto << "\n";
        } else if (cmd == "wrap") {
            uint32_t src, dst, seq, ack;
            unsigned sport, dport, syn, fin, rst, has_ack, win;
            std::string ph;
            in >> src >> sport >> dst >> dport >> seq >> syn >> fin >> rst >> has_ack >> ack >> win >> ph;
            TCPOverIPv4Adapter A;
            A.config_mut().source = Address{ipstr(src), static_cast<uint16_t>(sport)};
            A.config_mut().destination = Address{ipstr(dst), static_cast<uint16_t>(dport)};
            TCPMessage m;
            m.sender.seqno = Wrap32{seq};
            m.sender.SYN = syn;
            m.sender.FIN = fin;
            m.sender.RST = rst;
            m.sender.payload = ph == "-" ? std::string{} : unhex(ph);
            if (has_ack) m.receiver.ackno = Wrap32{ack};
            m.receiver.window_size = static_cast<uint16_t>(win);
            std::cout << tohex(joined(serialize(A.wrap_tcp_in_ip(m)))) << "\n";
        } else if (cmd == "unwrap") {
            uint32_t src, dst;
            unsigned sport, dport;
            std::string h;
            in >> src >> sport >> dst >> dport >> h;
            TCPOverIPv4Adapter B;
            B.config_mut().source = Address{ipstr(src), static_cast<uint16_t>(sport)};
            B.config_mut().destination = Address{ipstr(dst), static_cast<uint16_t>(dport)};
            IPv4Datagram dg;
            bool ok = parse(dg, std::vector<std::string>{unhex(h)});
            ok = ok && B.unwrap_tcp_in_ip(dg).has_value();
            std::cout << ok << "\n";
        } else if (cmd == "io") {
            // DatagramBatch round trip through a SOCK_DGRAM socketpair:
            // push -> sendmmsg -> recvmmsg (compacted arena) -> same bytes
            std::vector<std::string> ws;
            std::string h;
            while (in >> h) ws.push_back(unhex(h));
            int sv[2];
            if (socketpair(AF_UNIX, SOCK_DGRAM, 0, sv) != 0) return 3;
            icsum::DatagramBatch tx(size_t(1) << 20), rx(size_t(1) << 22);
            size_t sent = 0, got = 0;
            bool same = true;
            for (size_t i = 0; i < ws.size();) {  // in rounds that fit the socket buffer
                tx.clear();
                size_t j = i;
                for (; j < ws.size() && j - i < 32 && tx.push(ws[j]); ++j) {
                }
                sent += tx.write_to(sv[0]);
                const size_t before = rx.size();
                got += rx.read_from(sv[1], j - i);
                for (size_t k = before; k < rx.size(); ++k) same = same && rx[k] == ws[k];
                i = j;
            }
            close(sv[0]);
            close(sv[1]);
            std::cout << sent << " " << got << " " << same << " " << rx.bytes() << "\n";
        } else if (cmd == "ioudp") {
            // UDP on 127.0.0.1: every wire, then an empty datagram (the end
            // marker DatagramRing's readers stop at), then one more wire;
            // read_from takes the wires before the marker, sets ended(), and
            // leaves the wire after it for the next read
            std::vector<std::string> ws;
            std::string h;
            while (in >> h) ws.push_back(unhex(h));
            sockaddr_in a{};
            a.sin_family = AF_INET;
            a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
            socklen_t alen = sizeof a;
            const int tx = socket(AF_INET, SOCK_DGRAM, 0), rxfd = socket(AF_INET, SOCK_DGRAM, 0);
            if (tx < 0 || rxfd < 0 || bind(rxfd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 ||
                getsockname(rxfd, reinterpret_cast<sockaddr*>(&a), &alen) != 0 ||
                connect(tx, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0)
                return 3;
            const int buf = 4 << 20;
            (void)setsockopt(rxfd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
            icsum::DatagramBatch txb(size_t(1) << 20), rx(size_t(1) << 22, 4096);
            for (const auto& w : ws) txb.push(w);
            const size_t sent = txb.write_to(tx);
            (void)send(tx, "", 0, 0);
            (void)send(tx, ws[0].data(), ws[0].size(), 0);
            size_t got = 0;
            bool same = true;
            while (!rx.ended() && got < ws.size()) {
                const size_t before = rx.size();
                got += rx.read_from(rxfd, ws.size() + 1);
                for (size_t k = before; k < rx.size(); ++k) same = same && rx[k] == ws[k];
            }
            const bool ended = rx.ended();
            rx.clear();
            const size_t after = rx.read_from(rxfd, 8);
            const bool next_ok = after == 1 && rx[0] == ws[0] && !rx.ended();
            close(tx);
            close(rxfd);
            std::cout << sent << " " << got << " " << same << " " << ended << " " << next_ok << "\n";
        } else if (cmd == "ioseq") {
            // SOCK_SEQPACKET stream: a writer thread sends every wire 4 times
            // and closes its end; read_from(64) until it returns 0
            std::vector<std::string> ws;
            std::string h;
            while (in >> h) ws.push_back(unhex(h));
            int sv[2];
            if (socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) != 0) return 3;
            size_t sent = 0;
            std::thread w([&] {
                icsum::DatagramBatch tx(size_t(1) << 20);
                for (int p = 0; p < 4; ++p)
                    for (const auto& x : ws) {
                        tx.clear();
                        tx.push(x);
                        sent += tx.write_to(sv[0]);
                    }
                close(sv[0]);
            });
            icsum::DatagramBatch rx(size_t(1) << 22, 64);
            size_t got = 0, reads = 0;
            bool same = true, ended_early = false;
            for (;;) {
                rx.clear();
                const size_t k = rx.read_from(sv[1], 64);
                ++reads;
                if (k == 0) break;
                ended_early = ended_early || (rx.ended() && got + k < 4 * ws.size());
                for (size_t i = 0; i < k; ++i) same = same && rx[i] == ws[(got + i) % ws.size()];
                got += k;
            }
            w.join();
            close(sv[1]);
            // ended() is set by the read that meets the end, never before
            std::cout << sent << " " << got << " " << same << " " << (reads > 1) << " "
                      << (rx.ended() && !ended_early) << "\n";
        } else if (cmd == "ringstress") {
            uint32_t F = 0, P = 0, N = 0;
            in >> F >> P >> N;
            std::vector<int> rd, wr;
            for (uint32_t f = 0; f < F; ++f) {
                int sv[2];
                if (socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) != 0) return 3;
                wr.push_back(sv[0]);
                rd.push_back(sv[1]);
            }
            std::vector<uint32_t> next(F, 0);
            bool same = true;
            size_t got = 0;
            {
                // small arenas and few datagrams per arena: many hand-overs
                icsum::DatagramRing ring(rd, 0, size_t(64) << 10, 64);
                std::vector<std::thread> ws;
                for (uint32_t f = 0; f < F; ++f)
                    ws.emplace_back([&, f] {
                        icsum::DatagramBatch tx(size_t(1) << 20, 256);
                        uint32_t k = 0;
                        for (uint32_t p = 0; p < P; ++p) {
                            for (uint32_t i = 0; i < N; i += 64) {
                                tx.clear();
                                for (uint32_t j = i; j < std::min(N, i + 64); ++j) tx.push(stress_dgram(f, k++));
                                tx.write_to(wr[f]);
                            }
                        }
                        close(wr[f]);
                    });
                while (icsum::DatagramBatch* b = ring.next()) {
                    for (size_t i = 0; i < b->size(); ++i) {
                        const std::string_view d = (*b)[i];
                        const uint32_t f = static_cast<uint8_t>(d[0]);
                        uint32_t k = 0;
                        for (int q = 0; q < 4; ++q) k |= uint32_t(static_cast<uint8_t>(d[1 + q])) << (8 * q);
                        same = same && f < F && k == next[f] && d == stress_dgram(f, k);
                        if (f < F) next[f] = k + 1;
                        ++got;
                    }
                    ring.release(b);
                }
                for (auto& t : ws) t.join();
            }
            bool all = true;
            for (uint32_t f = 0; f < F; ++f) all = all && next[f] == P * N;
            for (int fd : rd) close(fd);
            std::cout << got << " " << same << " " << all << "\n";
        } else if (cmd == "txstress") {
            uint32_t P = 0, N = 0;
            in >> P >> N;
            int sv[2];
            if (socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) != 0) return 3;
            size_t got = 0;
            bool same = true;
            std::thread r([&] {
                icsum::DatagramBatch rx(size_t(1) << 20, 256);
                for (;;) {
                    rx.clear();
                    const size_t k = rx.read_from(sv[1], 256);
                    if (k == 0) break;
                    for (size_t i = 0; i < k; ++i) same = same && rx[i] == stress_dgram(0, static_cast<uint32_t>(got + i));
                    got += k;
                }
            });
            size_t sent = 0;
            bool recovered = false;
            {
                icsum::DatagramTxRing tx(sv[0], 3, size_t(64) << 10, 64);
                // an engine-less arena cannot patch: submit() throws and the
                // arena goes back to the free list (4 more acquires than slots
                // would block forever if it leaked)
                int threw = 0;
                for (int t = 0; t < 4; ++t) {
                    icsum::DatagramBatch* b = tx.acquire();
                    b->push(stress_dgram(9, 9));
                    try {
                        tx.submit(b, true);
                    } catch (const std::logic_error&) {
                        ++threw;
                    }
                }
                recovered = threw == 4;
                uint32_t k = 0;
                for (uint32_t p = 0; p < P; ++p) {
                    for (uint32_t i = 0; i < N;) {
                        icsum::DatagramBatch* b = tx.acquire();
                        while (i < N && b->push(stress_dgram(0, k))) {
                            ++i;
                            ++k;
                        }
                        tx.submit(b, false);
                    }
                }
                tx.flush();
                sent = tx.sent();
            }
            shutdown(sv[0], SHUT_WR);
            r.join();
            close(sv[0]);
            close(sv[1]);
            std::cout << sent << " " << got << " " << same << " " << recovered << "\n";
        } else if (!cmd.empty()) {
            std::cerr << "unknown command " << cmd << "\n";
            return 1;
        }
    }
    return 0;
}
