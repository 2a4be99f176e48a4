// host_selftest.cpp — CPU checks of the drop-in types, driven line by line by
// tests/test_host_cpp.py with the golden fixtures of the real reference.
//   kat INIT HEX...                -> value (add(vector<string>) == add(vector<string_view>))
//   ipv4 HEX                       -> "ok computed pseudo" from IPv4Header::parse
//   tcpv HEX                       -> "ip_ok tcp_ok tcp_value ip_computed proto" (datagram parse path)
//   wrap SRC SPORT DST DPORT SEQ SYN FIN RST HASACK ACK WIN PAYLOADHEX -> wire hex
//   unwrap SRC SPORT DST DPORT HEX -> "1" if the adapter (source=SRC:SPORT) accepts, else "0"
#include <cstdio>
#include <iostream>
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
}  // namespace

int main()
{
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string cmd;
        in >> cmd;
        if (cmd == "kat") {
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
        } else if (!cmd.empty()) {
            std::cerr << "unknown command " << cmd << "\n";
            return 1;
        }
    }
    return 0;
}
