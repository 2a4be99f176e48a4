// dropin_stack.cpp — drop-in proof.  The reference's own TCP stack sources
// (src/tcp_sender, src/tcp_receiver, src/reassembler, src/byte_stream,
// src/wrapping_integers; compiled in place from /root/reference, unchanged)
// run over THIS engine's TCPOverIPv4Adapter / IPv4Datagram / parser types:
// two peers move a bidirectional byte stream through wire datagrams with
// checksums computed and verified by the drop-in path (per object on the
// CPU, or per tick in one batch through icsum::BatchEngine with --gpu).
//
// BASELINE config 1 (the reference's own CPU case: 1 MiB through its stack,
// checksums via util/tcp_over_ip) is this program.  oracle/ref/Makefile builds
// the same source with -DICSUM_REFERENCE_UTIL against the reference's OWN util
// sources (oracle/_ref/stack_loop_ref), so the wall time printed here compares
// the reference path with the drop-in path on identical traffic.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <optional>
#include <random>
#include <string>
#include <vector>

#ifndef ICSUM_REFERENCE_UTIL
#include "batch.h"
#endif
#include "ipv4_datagram.h"
#include "tcp_over_ip.h"
#include "tcp_receiver.h"
#include "tcp_sender.h"

namespace {
struct Peer
{
    TCPSender sender;
    TCPReceiver receiver;
    TCPOverIPv4Adapter adapter{};
    Peer(uint32_t isn) : sender(ByteStream{64000}, Wrap32{isn}, 1000), receiver(Reassembler{ByteStream{64000}}) {}
};

std::string joined(const std::vector<std::string>& v)
{
    std::string r;
    for (auto& s : v) r += s;
    return r;
}
}  // namespace

int main(int argc, char** argv)
{
#ifdef ICSUM_REFERENCE_UTIL
    constexpr bool gpu = false;
    (void)argc;
    (void)argv;
#else
    const bool gpu = argc > 1 && std::strcmp(argv[1], "--gpu") == 0;
    std::unique_ptr<icsum::BatchEngine> eng;
    if (gpu) eng = std::make_unique<icsum::BatchEngine>(0);
#endif
    const auto t0 = std::chrono::steady_clock::now();
    Peer a(137), b(4242);
    a.adapter.config_mut().source = Address{"169.254.144.9", 5555};
    a.adapter.config_mut().destination = Address{"169.254.145.9", 80};
    b.adapter.config_mut().source = Address{"169.254.145.9", 80};
    b.adapter.config_mut().destination = Address{"169.254.144.9", 5555};

    std::mt19937_64 rng(7);
    std::string up(1 << 20, '\0'), down(300000, '\0');
    for (auto& c : up) c = static_cast<char>(rng());
    for (auto& c : down) c = static_cast<char>(rng());
    std::string got_up, got_down;
    size_t up_off = 0, down_off = 0, wires = 0, dropped = 0, wrap_mismatch = 0;

    for (int round = 0; round < 200000; ++round) {
        // application writes
        auto feed = [](Peer& p, const std::string& src, size_t& off) {
            auto& w = p.sender.writer();
            while (off < src.size() && w.available_capacity() > 0) {
                const size_t k = std::min<size_t>(w.available_capacity(), src.size() - off);
                w.push(src.substr(off, k));
                off += k;
            }
            if (off == src.size() && !w.is_closed()) w.close();
        };
        feed(a, up, up_off);
        feed(b, down, down_off);
        // each peer's transmissions this tick -> wire datagrams
        auto collect = [&](Peer& p) {
            std::vector<TCPMessage> msgs;
            auto tx = [&](const TCPSenderMessage& m) { msgs.push_back(TCPMessage{m, p.receiver.send()}); };
            p.sender.push(tx);
            p.sender.tick(1, tx);
            if (msgs.empty() && (p.receiver.send().ackno.has_value()))
                msgs.push_back(TCPMessage{p.sender.make_empty_message(), p.receiver.send()});
            std::vector<std::string> out;
#ifndef ICSUM_REFERENCE_UTIL
            if (gpu) {
                for (auto& d : eng->wrap(p.adapter, msgs)) out.push_back(joined(serialize(d)));
                // every GPU-wrapped datagram must equal the per-object wrap_tcp_in_ip's
                for (size_t i = 0; i < msgs.size(); ++i) {
                    const std::string want = joined(serialize(p.adapter.wrap_tcp_in_ip(msgs[i])));
                    if (out[i] != want && ++wrap_mismatch == 1) {
                        std::fprintf(stderr, "wrap mismatch (n=%zu, i=%zu, %zu vs %zu bytes)\n", msgs.size(), i,
                                     out[i].size(), want.size());
                        for (size_t k = 0; k < 48 && k < out[i].size(); ++k)
                            std::fprintf(stderr, "%02x%s", static_cast<unsigned char>(out[i][k]), k == 47 ? "\n" : "");
                        for (size_t k = 0; k < 48 && k < want.size(); ++k)
                            std::fprintf(stderr, "%02x%s", static_cast<unsigned char>(want[k]), k == 47 ? "\n" : "");
                    }
                }
                return out;
            }
#endif
            for (auto& m : msgs) out.push_back(joined(serialize(p.adapter.wrap_tcp_in_ip(m))));
            return out;
        };
        auto deliver = [&](Peer& p, const std::vector<std::string>& ws) {
            std::vector<std::optional<TCPMessage>> msgs;
#ifndef ICSUM_REFERENCE_UTIL
            if (gpu) {
                std::vector<std::string_view> v(ws.begin(), ws.end());
                msgs = eng->unwrap_raw(p.adapter, v);
            }
#endif
            if (!gpu) {
                for (auto& w : ws) {
                    IPv4Datagram dg;
                    msgs.push_back(parse(dg, std::vector<std::string>{w}) ? p.adapter.unwrap_tcp_in_ip(dg)
                                                                         : std::optional<TCPMessage>{});
                }
            }
            for (auto& m : msgs) {
                if (!m) {
                    ++dropped;
                    continue;
                }
                p.receiver.receive(m->sender);
                p.sender.receive(m->receiver);
            }
            wires += ws.size();
        };
        auto wa = collect(a), wb = collect(b);
        // corrupt one datagram in 50: the checksum must catch it, TCP retransmits
        for (auto* ws : {&wa, &wb})
            for (auto& w : *ws)
                if (rng() % 50 == 0) w[rng() % w.size()] ^= static_cast<char>(1u << (rng() % 8));
        deliver(b, wa);
        deliver(a, wb);
        auto drain = [](Peer& p, std::string& dst) {
            auto& r = p.receiver.reader();
            while (r.bytes_buffered()) {
                auto v = r.peek();
                dst.append(v);
                r.pop(v.size());
            }
        };
        drain(b, got_up);
        drain(a, got_down);
        if (b.receiver.reader().is_finished() && a.receiver.reader().is_finished()) break;
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const bool ok = got_up == up && got_down == down && wrap_mismatch == 0;
#ifdef ICSUM_REFERENCE_UTIL
    const char* path = "reference util";
#else
    const char* path = gpu ? "GPU batch" : "CPU";
#endif
    std::printf("%s: %s path, %zu + %zu bytes delivered bit-exact over %zu datagrams (%zu rejected) in %.1f ms\n",
                ok ? "OK" : "FAILED", path, got_up.size(), got_down.size(), wires, dropped, ms);
    return ok ? 0 : 1;
}
