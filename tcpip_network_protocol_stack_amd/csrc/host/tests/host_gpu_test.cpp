// host_gpu_test.cpp — icsum::BatchEngine (GPU) against the per-object calls of
// the same drop-in types (CPU) on seeded random traffic.  Exit 0 = identical.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <map>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include "batch.h"
#include "batch_io.h"
#include "checksum.h"
#include "icsum.h"

namespace {
int failures = 0;
#define EXPECT(c)                                                     \
    do {                                                              \
        if (!(c)) {                                                   \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                               \
        }                                                             \
    } while (0)

std::string joined(const std::vector<std::string>& v)
{
    std::string r;
    for (auto& s : v) r += s;
    return r;
}
}  // namespace

int main()
{
    icsum::BatchEngine eng(0);
    std::mt19937_64 rng(0x1071);
    auto bytes = [&](size_t n) {
        std::string s(n, '\0');
        for (auto& c : s) c = static_cast<char>(rng());
        return s;
    };

    // checksum(): vs InternetChecksum per segment, odd lengths and empty ones
    std::vector<std::string> segs;
    std::vector<uint32_t> init;
    for (int i = 0; i < 5000; ++i) {
        segs.push_back(bytes(rng() % 3000));
        init.push_back(static_cast<uint32_t>(rng()));
    }
    std::vector<std::string_view> views(segs.begin(), segs.end());
    const auto v = eng.checksum(views, init);
    for (size_t i = 0; i < segs.size(); ++i) {
        InternetChecksum c{init[i]};
        c.add(std::string_view{segs[i]});
        EXPECT(v[i] == c.value());
    }

    // wrap(): vs wrap_tcp_in_ip per message
    TCPOverIPv4Adapter A, B;
    A.config_mut().source = Address{"10.1.2.3", 4321};
    A.config_mut().destination = Address{"10.9.8.7", 80};
    B.config_mut().source = Address{"10.9.8.7", 80};
    B.config_mut().destination = Address{"10.1.2.3", 4321};
    std::vector<TCPMessage> msgs;
    for (int i = 0; i < 2000; ++i) {
        TCPMessage m;
        m.sender.seqno = Wrap32{static_cast<uint32_t>(rng())};
        m.sender.SYN = rng() % 5 == 0;
        m.sender.FIN = rng() % 7 == 0;
        m.sender.payload = bytes(rng() % 1001);
        if (rng() % 3) m.receiver.ackno = Wrap32{static_cast<uint32_t>(rng())};
        m.receiver.window_size = static_cast<uint16_t>(rng());
        msgs.push_back(m);
    }
    const auto dgs = eng.wrap(A, msgs);
    std::vector<std::string> wires;
    for (size_t i = 0; i < msgs.size(); ++i) {
        const InternetDatagram ref = A.wrap_tcp_in_ip(msgs[i]);
        const auto want = joined(serialize(ref));
        wires.push_back(joined(serialize(dgs[i])));
        EXPECT(wires.back() == want);
        EXPECT(dgs[i].payload == ref.payload);  // the same pieces serialize(seg) gives
        EXPECT(dgs[i].header.len == ref.header.len && dgs[i].header.cksum == ref.header.cksum);
    }
    // device-side wrap through the other entry points: consuming the messages
    // (payloads moved, not copied), and the arena path (push_tcp + wrap, the
    // transmit ring's), both byte-equal to wrap_tcp_in_ip
    {
        std::vector<TCPMessage> moved = msgs;
        const auto dgs2 = eng.wrap(A, std::move(moved));
        for (size_t i = 0; i < msgs.size(); ++i) EXPECT(joined(serialize(dgs2[i])) == wires[i]);
        icsum::DatagramBatch tb(eng, size_t(8) << 20);
        for (const auto& m : msgs) EXPECT(tb.push_tcp(A, m));
        EXPECT(tb.wrap_pending());
        tb.wrap();
        EXPECT(!tb.wrap_pending());
        for (size_t i = 0; i < msgs.size(); ++i) EXPECT(tb[i] == wires[i]);
        icsum::DatagramBatch mixed(eng, size_t(1) << 20);
        EXPECT(mixed.push_tcp(A, msgs[0]) && mixed.push(wires[1]));
        bool threw = false;
        try {
            mixed.wrap();
        } catch (const std::logic_error&) {
            threw = true;
        }
        EXPECT(threw);
    }

    // compute_checksums(): TCP and IPv4 header batches
    {
        std::vector<TCPSegment> ts;
        std::vector<IPv4Header> hs;
        for (size_t i = 0; i < 300; ++i) {
            TCPSegment s;
            s.message = msgs[i];
            s.udinfo = {static_cast<uint16_t>(rng()), static_cast<uint16_t>(rng()), static_cast<uint16_t>(rng())};
            IPv4Header h;
            h.src = static_cast<uint32_t>(rng());
            h.dst = static_cast<uint32_t>(rng());
            h.len = static_cast<uint16_t>(40 + s.message.sender.payload.size());
            h.ttl = static_cast<uint8_t>(rng());
            h.id = static_cast<uint16_t>(rng());
            ts.push_back(s);
            hs.push_back(h);
        }
        auto ts_cpu = ts;
        auto hs_cpu = hs;
        eng.compute_checksums(ts, hs);
        eng.compute_checksums(std::span<IPv4Header>(hs));
        for (size_t i = 0; i < ts.size(); ++i) {
            ts_cpu[i].compute_checksum(hs_cpu[i].pseudo_checksum());
            hs_cpu[i].compute_checksum();
            EXPECT(ts[i].udinfo.cksum == ts_cpu[i].udinfo.cksum);
            EXPECT(hs[i].cksum == hs_cpu[i].cksum);
        }
    }

    // verify_raw() / unwrap_raw() / unwrap(): clean and one-bit-corrupted wires
    std::vector<std::string> rx;
    for (size_t i = 0; i < wires.size(); ++i) {
        std::string w = wires[i];
        if (i % 2) w[rng() % w.size()] ^= static_cast<char>(1u << (rng() % 8));
        rx.push_back(w);
    }
    std::vector<std::string_view> rxv(rx.begin(), rx.end());
    const auto st = eng.verify_raw(rxv);
    TCPOverIPv4Adapter Bcpu = B, Bgpu = B, Bgpu2 = B;
    const auto got = eng.unwrap_raw(Bgpu, rxv);
    std::vector<InternetDatagram> parsed(rx.size());
    std::vector<bool> ip_ok(rx.size());
    for (size_t i = 0; i < rx.size(); ++i) ip_ok[i] = parse(parsed[i], std::vector<std::string>{rx[i]});
    const auto got2 = eng.unwrap(Bgpu2, parsed);
    size_t accepted = 0;
    for (size_t i = 0; i < rx.size(); ++i) {
        TCPSegment seg;
        const bool tcp_ok = parse(seg, parsed[i].payload, parsed[i].header.pseudo_checksum());
        EXPECT(((st[i] & ICS_ST_IPV4_OK) != 0) == ip_ok[i]);
        EXPECT(((st[i] & (ICS_ST_TCP_CKSUM_OK | ICS_ST_TCP_HDR_OK)) == (ICS_ST_TCP_CKSUM_OK | ICS_ST_TCP_HDR_OK)) ==
               tcp_ok);
        const auto want = ip_ok[i] ? Bcpu.unwrap_tcp_in_ip(parsed[i]) : std::optional<TCPMessage>{};
        EXPECT(got[i].has_value() == want.has_value());
        if (ip_ok[i]) EXPECT(got2[i].has_value() == want.has_value());
        if (want) {
            ++accepted;
            EXPECT(got[i]->sender.payload == want->sender.payload);
            EXPECT(got[i]->sender.SYN == want->sender.SYN && got[i]->sender.FIN == want->sender.FIN);
            if (ip_ok[i] && got2[i]) {  // unwrap(InternetDatagram) — the same message, field by field
                EXPECT(got2[i]->sender.payload == want->sender.payload);
                EXPECT(got2[i]->sender.seqno == want->sender.seqno && got2[i]->receiver.ackno == want->receiver.ackno);
                EXPECT(got2[i]->sender.SYN == want->sender.SYN && got2[i]->sender.FIN == want->sender.FIN &&
                       got2[i]->sender.RST == want->sender.RST);
                EXPECT(got2[i]->receiver.window_size == want->receiver.window_size);
            }
        }
    }
    EXPECT(accepted >= wires.size() / 2);

    // unwrap_raw() at a batch size that takes the threaded field parse (8
    // ranges at >= 16 Ki datagrams, batch.cpp) with the adapter's gates in
    // datagram order: 20 000 wires from two peers and strangers, a third
    // one-bit corrupted, to a LISTENING adapter whose first clean SYN (from
    // peer 2) sits mid-batch; then to a connected adapter.  Every result must
    // equal the per-object unwrap_tcp_in_ip in the same order, field by field.
    {
        auto same_msg = [](const TCPMessage& a, const TCPMessage& b) {
            return a.sender.seqno == b.sender.seqno && a.sender.SYN == b.sender.SYN &&
                   a.sender.payload == b.sender.payload && a.sender.FIN == b.sender.FIN &&
                   a.sender.RST == b.sender.RST && a.receiver.ackno == b.receiver.ackno &&
                   a.receiver.window_size == b.receiver.window_size && a.receiver.RST == b.receiver.RST;
        };
        TCPOverIPv4Adapter p1, p2, stranger, wrongport;
        p1.config_mut().source = Address{"10.9.8.7", 80};
        p2.config_mut().source = Address{"10.5.5.5", 8080};
        stranger.config_mut().source = Address{"10.7.7.7", 80};
        wrongport.config_mut().source = Address{"10.9.8.7", 80};
        for (auto* a : {&p1, &p2, &stranger}) a->config_mut().destination = Address{"10.1.2.3", 4321};
        wrongport.config_mut().destination = Address{"10.1.2.3", 4322};
        const size_t N = 20000, kSyn = 8191;
        std::vector<std::string> big;
        for (size_t i = 0; i < N; ++i) {
            TCPMessage m;
            m.sender.seqno = Wrap32{static_cast<uint32_t>(rng())};
            m.sender.SYN = i == kSyn || (i > kSyn && rng() % 5 == 0);
            m.sender.RST = i != kSyn && rng() % 11 == 0;
            m.sender.FIN = rng() % 7 == 0;
            m.sender.payload = bytes(rng() % 600);
            if (rng() % 3) m.receiver.ackno = Wrap32{static_cast<uint32_t>(rng())};
            m.receiver.window_size = static_cast<uint16_t>(rng());
            const unsigned pick = static_cast<unsigned>(rng() % 20);
            TCPOverIPv4Adapter& from =
                i == kSyn ? p2 : (pick < 12 ? p1 : (pick < 16 ? p2 : (pick < 18 ? stranger : wrongport)));
            std::string w = joined(serialize(from.wrap_tcp_in_ip(m)));
            if (i != kSyn && i % 3 == 1) w[rng() % w.size()] ^= static_cast<char>(1u << (rng() % 8));
            big.push_back(w);
        }
        std::vector<std::string_view> bigv(big.begin(), big.end());
        TCPOverIPv4Adapter L;
        L.config_mut().source = Address{"0", 4321};
        L.set_listening(true);
        TCPOverIPv4Adapter C = A;  // 10.1.2.3:4321 connected to 10.9.8.7:80 (peer 1)
        for (int pass = 0; pass < 2; ++pass) {
            TCPOverIPv4Adapter Agpu = pass ? C : L, Acpu = pass ? C : L;
            const auto gotb = eng.unwrap_raw(Agpu, bigv);
            size_t acc = 0, before_syn = 0;
            for (size_t i = 0; i < N; ++i) {
                InternetDatagram d;
                std::optional<TCPMessage> want;
                if (parse(d, std::vector<std::string>{big[i]})) want = Acpu.unwrap_tcp_in_ip(d);
                EXPECT(gotb[i].has_value() == want.has_value());
                if (want && gotb[i]) {
                    EXPECT(same_msg(*gotb[i], *want));
                    ++acc;
                    if (i < kSyn) ++before_syn;
                }
            }
            EXPECT(Agpu.listening() == Acpu.listening());
            EXPECT(Agpu.config().destination == Acpu.config().destination);
            EXPECT(acc > N / 20);  // listening: only peer 2 (1/5 of the wires) after its SYN
            if (pass == 0) EXPECT(before_syn == 0 && !Agpu.listening());  // nothing before the first SYN
        }
    }

    // TCP data offsets 6..15 with valid checksums (options, or a header that
    // claims more than the segment holds: the reference's Parser skips to the
    // end without an error and the payload is empty): the batch field parse
    // must equal the per-object one
    {
        std::vector<std::string> opt;
        for (unsigned doff = 5; doff <= 15; ++doff)
            for (size_t plen : {size_t(0), size_t(3), size_t(4), size_t(10), size_t(41), size_t(60)}) {
                TCPMessage m;
                m.sender.seqno = Wrap32{static_cast<uint32_t>(rng())};
                m.sender.payload = bytes(plen);
                m.receiver.ackno = Wrap32{static_cast<uint32_t>(rng())};
                m.receiver.window_size = static_cast<uint16_t>(rng());
                std::string w = joined(serialize(A.wrap_tcp_in_ip(m)));
                w[20 + 12] = static_cast<char>(doff << 4);
                w[20 + 16] = w[20 + 17] = 0;
                IPv4Datagram d;
                EXPECT(parse(d, std::vector<std::string>{w}));
                InternetChecksum c{d.header.pseudo_checksum()};
                c.add(std::string_view{w}.substr(20));
                const uint16_t ck = c.value();
                w[20 + 16] = static_cast<char>(ck >> 8);
                w[20 + 17] = static_cast<char>(ck & 0xff);
                opt.push_back(w);
            }
        std::vector<std::string_view> optv(opt.begin(), opt.end());
        TCPOverIPv4Adapter Bg = B, Bc = B;
        const auto got_opt = eng.unwrap_raw(Bg, optv);
        size_t acc = 0;
        for (size_t i = 0; i < opt.size(); ++i) {
            IPv4Datagram d;
            std::optional<TCPMessage> want;
            if (parse(d, std::vector<std::string>{opt[i]})) want = Bc.unwrap_tcp_in_ip(d);
            EXPECT(got_opt[i].has_value() == want.has_value());
            if (want && got_opt[i]) {
                EXPECT(got_opt[i]->sender.payload == want->sender.payload);
                EXPECT(got_opt[i]->sender.seqno == want->sender.seqno);
                ++acc;
            }
        }
        EXPECT(acc == opt.size());  // every data offset >= 5 parses (payload empty past the end)
    }

    // batched datagram I/O: the same received wires through
    // a SOCK_DGRAM socketpair into a page-locked arena, unwrapped in place
    {
        int sv[2];
        EXPECT(socketpair(AF_UNIX, SOCK_DGRAM, 0, sv) == 0);
        icsum::DatagramBatch txb(size_t(1) << 20), rxb(eng, size_t(64) << 20);
        for (size_t i = 0; i < rx.size();) {
            txb.clear();
            size_t j = i;
            for (; j < rx.size() && j - i < 32 && txb.push(rx[j]); ++j) {
            }
            EXPECT(txb.write_to(sv[0]) == j - i);
            EXPECT(rxb.read_from(sv[1], j - i) == j - i);
            i = j;
        }
        close(sv[0]);
        close(sv[1]);
        EXPECT(rxb.size() == rx.size());
        TCPOverIPv4Adapter Bio = B;
        const auto got3 = rxb.unwrap(Bio);
        for (size_t i = 0; i < rx.size(); ++i) EXPECT(got3[i].has_value() == got[i].has_value());
        // transmit side: wires with both checksum fields zeroed, patched in the arena
        icsum::DatagramBatch out(eng, size_t(16) << 20);
        for (const auto& w : wires) {
            std::string z = w;
            z[10] = z[11] = 0;
            z[36] = z[37] = 0;
            EXPECT(out.push(z));
        }
        out.patch();
        for (size_t i = 0; i < wires.size(); ++i) EXPECT(out[i] == wires[i]);
    }
    // DatagramRing: a writer thread streams the received wires (8 passes) over
    // a SOCK_SEQPACKET socketpair and closes its end; the ring's reader fills
    // arenas while this thread verifies them; every datagram arrives once, in
    // order, with the status verify_raw() gave it
    {
        int sv[2];
        EXPECT(socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) == 0);
        constexpr size_t kPasses = 8;
        std::thread writer([&] {
            icsum::DatagramBatch txb(size_t(1) << 20);
            for (size_t p = 0; p < kPasses; ++p) {
                for (size_t i = 0; i < rx.size();) {
                    txb.clear();
                    size_t j = i;
                    for (; j < rx.size() && j - i < 64 && txb.push(rx[j]); ++j) {
                    }
                    txb.write_to(sv[0]);
                    i = j;
                }
            }
            close(sv[0]);
        });
        size_t seen = 0, batches = 0;
        {
            icsum::DatagramRing ring(eng, sv[1], 3, size_t(4) << 20, 700);
            while (icsum::DatagramBatch* b = ring.next()) {
                const auto vs = b->verify();
                for (size_t k = 0; k < vs.size(); ++k, ++seen) {
                    EXPECT((*b)[k] == rx[seen % rx.size()]);
                    EXPECT(vs[k] == st[seen % rx.size()]);
                }
                ++batches;
                ring.release(b);
            }
        }
        writer.join();
        close(sv[1]);
        EXPECT(seen == kPasses * rx.size());
        EXPECT(batches > 1);
        // destroyed while the stream is still open and idle: the reader stops
        // within its poll interval and leaves the socket usable
        EXPECT(socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) == 0);
        const auto t0 = std::chrono::steady_clock::now();
        { icsum::DatagramRing idle(eng, sv[1], 2, size_t(1) << 20, 64); }
        EXPECT(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2));
        EXPECT(send(sv[0], "x", 1, 0) == 1);
        char c = 0;
        EXPECT(recv(sv[1], &c, 1, 0) == 1 && c == 'x');
        close(sv[0]);
        close(sv[1]);
    }
    // DatagramRing over a UDP socket on 127.0.0.1 (the transport the
    // reference's endtoend relay uses): no end of stream and drops allowed,
    // so the writer repeats an empty datagram (the end marker) until the ring
    // stops; what arrives is an in-order subsequence of what was sent, every
    // datagram with the status verify_raw() gave it
    {
        int tx = socket(AF_INET, SOCK_DGRAM, 0), rxfd = socket(AF_INET, SOCK_DGRAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        socklen_t alen = sizeof a;
        const int buf = 4 << 20;
        (void)setsockopt(rxfd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
        EXPECT(tx >= 0 && rxfd >= 0);
        EXPECT(bind(rxfd, reinterpret_cast<sockaddr*>(&a), sizeof a) == 0);
        EXPECT(getsockname(rxfd, reinterpret_cast<sockaddr*>(&a), &alen) == 0);
        EXPECT(connect(tx, reinterpret_cast<sockaddr*>(&a), sizeof a) == 0);
        constexpr size_t kPasses = 8;
        std::atomic<bool> done{false};
        std::thread writer([&] {
            icsum::DatagramBatch txb(size_t(1) << 20);
            for (size_t p = 0; p < kPasses; ++p) {
                for (size_t i = 0; i < rx.size();) {
                    txb.clear();
                    size_t j = i;
                    for (; j < rx.size() && j - i < 64 && txb.push(rx[j]); ++j) {
                    }
                    txb.write_to(tx);
                    i = j;
                }
            }
            while (!done.load()) {
                (void)send(tx, "", 0, 0);
                std::this_thread::sleep_for(std::chrono::milliseconds(1));
            }
        });
        size_t seen = 0, pos = 0;
        bool ordered = true;
        {
            icsum::DatagramRing ring(eng, rxfd, 3, size_t(4) << 20, 700);
            while (icsum::DatagramBatch* b = ring.next()) {
                const auto vs = b->verify();
                for (size_t k = 0; k < vs.size(); ++k, ++seen) {
                    while (pos < kPasses * rx.size() && (*b)[k] != rx[pos % rx.size()]) ++pos;
                    ordered = ordered && pos < kPasses * rx.size();
                    if (ordered) EXPECT(vs[k] == st[pos % rx.size()]);
                    ++pos;
                }
                ring.release(b);
            }
        }
        done = true;
        writer.join();
        close(tx);
        close(rxfd);
        EXPECT(ordered);
        EXPECT(seen > 0 && seen <= kPasses * rx.size());
    }
    // one DatagramRing over two SOCK_SEQPACKET streams (one reader thread
    // each, shared arenas, one engine): every datagram of both streams
    // arrives exactly once, with the status verify_raw() gave its bytes
    {
        int a[2], c[2];
        EXPECT(socketpair(AF_UNIX, SOCK_SEQPACKET, 0, a) == 0);
        EXPECT(socketpair(AF_UNIX, SOCK_SEQPACKET, 0, c) == 0);
        constexpr size_t kPasses = 4;
        auto send_all = [&](int fd) {
            icsum::DatagramBatch txb(size_t(1) << 20);
            for (size_t p = 0; p < kPasses; ++p)
                for (size_t i = 0; i < rx.size();) {
                    txb.clear();
                    size_t j = i;
                    for (; j < rx.size() && j - i < 64 && txb.push(rx[j]); ++j) {
                    }
                    txb.write_to(fd);
                    i = j;
                }
            close(fd);
        };
        std::thread wa(send_all, a[0]), wc(send_all, c[0]);
        std::map<std::string, long> left;
        std::map<std::string, uint8_t> status;
        for (size_t i = 0; i < rx.size(); ++i) {
            left[rx[i]] += 2 * kPasses;
            status[rx[i]] = st[i];
        }
        size_t seen = 0;
        {
            icsum::DatagramRing ring(eng, std::vector<int>{a[1], c[1]}, 0, size_t(2) << 20, 300);
            while (icsum::DatagramBatch* b = ring.next()) {
                const auto vs = b->verify();
                for (size_t k = 0; k < vs.size(); ++k, ++seen) {
                    const std::string w((*b)[k]);
                    EXPECT(left.count(w) && --left[w] >= 0);
                    EXPECT(vs[k] == status[w]);
                }
                ring.release(b);
            }
        }
        wa.join();
        wc.join();
        close(a[1]);
        close(c[1]);
        EXPECT(seen == 2 * kPasses * rx.size());
        for (const auto& [w, n] : left) EXPECT(n == 0);
    }
    // DatagramTxRing: arenas of wires with both checksum fields zeroed are
    // patched on the GPU at submit(), arenas of messages (push_tcp) are
    // wrapped there (headers + checksums), and the ring's writer thread sends
    // them
    // over a SOCK_SEQPACKET socketpair; the peer reads exactly wrap_tcp_in_ip's
    // wires, in order
    {
        int sv[2];
        EXPECT(socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) == 0);
        constexpr size_t kPasses = 4, kPerArena = 50;
        std::vector<std::string> heard;
        std::thread peer([&] {
            icsum::DatagramBatch rxb(size_t(4) << 20, 1024);
            for (;;) {
                rxb.clear();
                const size_t k = rxb.read_from(sv[1], 1024);
                for (size_t i = 0; i < k; ++i) heard.emplace_back(rxb[i]);
                if (k == 0 || rxb.ended()) break;
            }
        });
        size_t sent = 0, arenas = 0;
        {
            icsum::DatagramTxRing tx(eng, sv[0], 3, size_t(1) << 20, kPerArena);
            for (size_t p = 0; p < kPasses; ++p)
                for (size_t i = 0; i < wires.size();) {
                    icsum::DatagramBatch* b = tx.acquire();
                    for (; i < wires.size() && b->size() < kPerArena; ++i) {
                        if (p % 2) {  // odd passes: messages, wrapped on the GPU at submit()
                            EXPECT(b->push_tcp(A, msgs[i]));
                            continue;
                        }
                        std::string z = wires[i];
                        z[10] = z[11] = 0;
                        z[36] = z[37] = 0;
                        EXPECT(b->push(z));
                    }
                    tx.submit(b);
                    ++arenas;
                }
            tx.flush();
            sent = tx.sent();
        }
        close(sv[0]);
        peer.join();
        close(sv[1]);
        EXPECT(sent == kPasses * wires.size());
        EXPECT(arenas > 3);
        EXPECT(heard.size() == kPasses * wires.size());
        for (size_t i = 0; i < heard.size() && i < kPasses * wires.size(); ++i) EXPECT(heard[i] == wires[i % wires.size()]);
    }
    // DatagramTxRing whose peer is gone: the writer's EPIPE (no SIGPIPE)
    // comes back from flush() / acquire(), and the destructor does not hang
    {
        int sv[2];
        EXPECT(socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) == 0);
        close(sv[1]);
        bool threw = false;
        const auto t0 = std::chrono::steady_clock::now();
        {
            icsum::DatagramTxRing tx(eng, sv[0], 2, size_t(1) << 20, 64);
            try {
                icsum::DatagramBatch* b = tx.acquire();
                EXPECT(b->push(wires[0]));
                tx.submit(b, false);
                tx.flush();
            } catch (const std::runtime_error&) {
                threw = true;
            }
        }
        EXPECT(threw);
        EXPECT(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2));
        close(sv[0]);
    }
    // a per-tick loop on the resident tick server: each tick verifies a few
    // received wires and wraps a few messages (the server's jobs: <= 64 on
    // its default 4 blocks, then <= 128 on 8), every result equal to the
    // per-object calls; then off again
    {
        eng.set_tick_server(5000);
        for (int t = 0; t < 300; ++t) {
            if (t == 200) eng.set_tick_server_blocks(8);
            const size_t most = t < 200 ? 64 : 128;
            const size_t k = 1 + static_cast<size_t>(rng() % most), at = static_cast<size_t>(rng() % (msgs.size() - k));
            std::vector<std::string_view> tw(wires.begin() + at, wires.begin() + at + k);
            const auto tst = eng.verify_raw(tw);
            for (size_t i = 0; i < k; ++i) EXPECT(tst[i] == ICS_ST_ACCEPT);
            const auto td = eng.wrap(A, std::span<const TCPMessage>(msgs.data() + at, k));
            for (size_t i = 0; i < k; ++i) EXPECT(joined(serialize(td[i])) == wires[at + i]);
            if (t % 50 == 49) std::this_thread::sleep_for(std::chrono::milliseconds(8));  // the server idles out
        }
        eng.set_tick_server(0);
        eng.set_tick_server_blocks(4);
    }
    std::printf("%s: %zu checksums, %zu wraps, %zu unwraps (%zu accepted)\n", failures ? "FAILED" : "OK",
                segs.size(), msgs.size(), rx.size(), accepted);
    return failures ? 1 : 0;
}
