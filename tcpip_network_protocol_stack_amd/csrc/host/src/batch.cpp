// batch.cpp — icsum::BatchEngine (see batch.h): packs objects into one
// contiguous wire buffer + offsets, runs one engine call, scatters results.
#include "batch.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "icsum.h"
#include "par_for.h"
#include "wire_internal.h"

namespace icsum {
namespace {

void check(int rc, const char* what)
{
    if (rc != ICS_OK) throw std::runtime_error(std::string(what) + ": " + ics_last_error());
}

}  // namespace

ics_tcp_msg wrap_fields(const FdAdapterConfig& cfg, const TCPMessage& msg)
{
    ics_tcp_msg m{};
    m.src = cfg.source.ipv4_numeric();
    m.dst = cfg.destination.ipv4_numeric();
    m.seqno = detail::raw_of(msg.sender.seqno);
    m.ackno = detail::raw_of(msg.receiver.ackno.value_or(Wrap32{0}));  // tcp_segment.cpp:86
    m.src_port = cfg.source.port();
    m.dst_port = cfg.destination.port();
    m.window = msg.receiver.window_size;
    m.flags = static_cast<uint8_t>((msg.receiver.ackno.has_value() ? ICS_TCP_ACK : 0U) |
                                   (msg.sender.RST || msg.receiver.RST ? ICS_TCP_RST : 0U) |
                                   (msg.sender.SYN ? ICS_TCP_SYN : 0U) | (msg.sender.FIN ? ICS_TCP_FIN : 0U));
    m.ttl = IPv4Header::DEFAULT_TTL;  // wrap_tcp_in_ip keeps the header defaults
    m.id = 0;
    return m;
}

uint8_t* BatchEngine::scratch(size_t bytes)
{
    if (bytes > scratch_cap_) {
        const size_t cap = std::max(bytes, scratch_cap_ * 2);
        if (scratch_) host_free(scratch_);
        scratch_ = nullptr;
        scratch_cap_ = 0;
        scratch_ = static_cast<uint8_t*>(host_alloc(cap));
        scratch_cap_ = cap;
    }
    return scratch_;
}

BatchEngine::BatchEngine(int device) : device_(device)
{
    check(ics_create(device, &ctx_), "ics_create");
}

BatchEngine::~BatchEngine()
{
    if (scratch_) ics_host_free(ctx_, scratch_);
    ics_destroy(ctx_);
}

template <typename Len, typename Put>
std::vector<uint64_t> BatchEngine::pack(size_t n, Len len, Put put)
{
    // item i's len(i) bytes at off[i] of the page-locked scratch arena, written
    // by put(i, dst) on the engine's workers: the *_host call then DMAs the
    // batch straight from it (no pageable staging copy)
    std::vector<uint64_t> off(n + 1, 0);
    for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + len(i);
    uint8_t* base = scratch(std::max<uint64_t>(off[n], 1));
    ranges(n, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) put(i, base + off[i]);
    });
    return off;
}

std::vector<uint16_t> BatchEngine::checksum(std::span<const std::string_view> segs, std::span<const uint32_t> init)
{
    if (!init.empty() && init.size() != segs.size()) throw std::invalid_argument("init size != segment count");
    std::vector<uint16_t> out(segs.size());
    if (segs.empty()) return out;
    const auto off = pack(
        segs.size(), [&](size_t i) { return segs[i].size(); },
        [&](size_t i, uint8_t* d) { std::memcpy(d, segs[i].data(), segs[i].size()); });
    check(ics_checksum_batch_host(ctx_, scratch_, off.data(), 0, 0, init.empty() ? nullptr : init.data(), out.data(),
                                  segs.size()),
          "ics_checksum_batch_host");
    return out;
}

void BatchEngine::compute_checksums(std::span<TCPSegment> segs, std::span<const IPv4Header> hdrs)
{
    if (hdrs.size() != segs.size()) throw std::invalid_argument("header count != segment count");
    if (segs.empty()) return;
    // serialize(seg)'s bytes — the 20-byte header with cksum = 0
    // (tcp_segment.cpp:111), then the payload — written straight into the arena
    std::vector<uint32_t> init(segs.size());
    const auto off = pack(
        segs.size(), [&](size_t i) { return 20 + segs[i].message.sender.payload.size(); },
        [&](size_t i, uint8_t* d) {
            segs[i].udinfo.cksum = 0;
            detail::tcp_header_bytes(segs[i], reinterpret_cast<char*>(d));
            const std::string& pl = segs[i].message.sender.payload;
            if (!pl.empty()) std::memcpy(d + 20, pl.data(), pl.size());
            init[i] = hdrs[i].pseudo_checksum();
        });
    std::vector<uint16_t> out(segs.size());
    check(ics_checksum_batch_host(ctx_, scratch_, off.data(), 0, 0, init.data(), out.data(), segs.size()),
          "ics_checksum_batch_host");
    for (size_t i = 0; i < segs.size(); ++i) segs[i].udinfo.cksum = out[i];
}

void BatchEngine::compute_checksums(std::span<IPv4Header> hdrs)
{
    if (hdrs.empty()) return;
    for (auto& h : hdrs)
        if (h.ver != 4) throw std::runtime_error("wrong IP version");  // serialize() would, like the reference
    const auto off = pack(
        hdrs.size(), [](size_t) { return size_t(IPv4Header::LENGTH); },
        [&](size_t i, uint8_t* d) {
            hdrs[i].cksum = 0;
            const std::string b = serialize(hdrs[i]).front();
            std::memcpy(d, b.data(), IPv4Header::LENGTH);
        });
    std::vector<uint16_t> ip(hdrs.size());
    check(ics_ipv4_tcp_batch_host(ctx_, scratch_, off.data(), 0, 0, hdrs.size(), ICS_MODE_COMPUTE, ip.data(), nullptr,
                                  nullptr),
          "ics_ipv4_tcp_batch_host");
    for (size_t i = 0; i < hdrs.size(); ++i) hdrs[i].cksum = ip[i];
}

std::vector<uint8_t> BatchEngine::verify_raw(std::span<const std::string_view> wires)
{
    std::vector<uint8_t> st(wires.size());
    if (wires.empty()) return st;
    const auto off = pack(
        wires.size(), [&](size_t i) { return wires[i].size(); },
        [&](size_t i, uint8_t* d) { std::memcpy(d, wires[i].data(), wires[i].size()); });
    check(ics_ipv4_tcp_batch_host(ctx_, scratch_, off.data(), 0, 0, wires.size(), ICS_MODE_VERIFY, nullptr, nullptr,
                                  st.data()),
          "ics_ipv4_tcp_batch_host");
    return st;
}

template <typename Msgs, typename Take>
std::vector<InternetDatagram> BatchEngine::wrap_impl(const TCPOverIPv4Adapter& adapter, Msgs& msgs, Take take_payload)
{
    // tcp_over_ip.cpp:69-88 for every message: each payload is copied ONCE,
    // to its final offset in a page-locked arena (after 40 bytes of header
    // room); one device pass sums it and serializes both headers with both
    // checksums (ics_tcp_wrap_batch_host) — no host-side serialize().
    const size_t n = msgs.size();
    std::vector<uint64_t> off(n + 1, 0);
    for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + 40 + msgs[i].sender.payload.size();
    uint8_t* arena = scratch(std::max<uint64_t>(off[n], 1));
    std::vector<ics_tcp_msg> rec(n);
    const FdAdapterConfig& cfg = adapter.config();
    // the payload copies into the arena and, after the device pass, the
    // results' construction (allocations, payload copies or moves) are
    // independent per message: split over the engine's workers
    ranges(n, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            const std::string& pl = msgs[i].sender.payload;
            if (!pl.empty()) std::memcpy(arena + off[i] + 40, pl.data(), pl.size());
            rec[i] = wrap_fields(cfg, msgs[i]);
        }
    });
    if (n) wrap_packed(arena, off.data(), rec.data(), n);
    std::vector<InternetDatagram> out(n);
    ranges(n, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            IPv4Header& h = out[i].header;  // the defaults wrap_tcp_in_ip keeps (ipv4_header.h)
            const uint8_t* w = arena + off[i];
            h.len = static_cast<uint16_t>((w[2] << 8) | w[3]);
            h.cksum = static_cast<uint16_t>((w[10] << 8) | w[11]);
            h.src = rec[i].src;
            h.dst = rec[i].dst;
            // serialize(seg)'s pieces: the 20-byte TCP header, then the payload
            // (Serializer::buffer, parser.h) when there is one
            out[i].payload.reserve(2);
            out[i].payload.emplace_back(reinterpret_cast<const char*>(w) + 20, 20);
            if (!msgs[i].sender.payload.empty()) out[i].payload.push_back(take_payload(msgs[i]));
        }
    });
    return out;
}

template <typename Fn>
void BatchEngine::ranges(size_t n, Fn&& fn)
{
    // up to 8 contiguous ranges of >= 2048 items on the engine's workers
    const size_t threads = std::min<size_t>({size_t(8), std::max(1u, std::thread::hardware_concurrency()),
                                             std::max<size_t>(1, n / 2048)});
    if (threads <= 1) {
        fn(size_t(0), n);
        return;
    }
    if (!pool_) pool_ = std::make_unique<detail::WorkerPool>(7);
    pool_->run(n, threads, fn);  // waits for every range, rethrows a range's exception
}

std::vector<InternetDatagram> BatchEngine::wrap(TCPOverIPv4Adapter& adapter, std::span<const TCPMessage> msgs)
{
    return wrap_impl(adapter, msgs, [](const TCPMessage& m) { return m.sender.payload; });
}

std::vector<InternetDatagram> BatchEngine::wrap(TCPOverIPv4Adapter& adapter, std::vector<TCPMessage>&& msgs)
{
    return wrap_impl(adapter, msgs, [](TCPMessage& m) { return std::move(m.sender.payload); });
}

void BatchEngine::wrap_packed(uint8_t* bytes, const uint64_t* offsets, const ics_tcp_msg* msgs, size_t n)
{
    if (n) check(ics_tcp_wrap_batch_host(ctx_, bytes, offsets, 0, 0, n, msgs), "ics_tcp_wrap_batch_host");
}

std::vector<std::optional<TCPMessage>> BatchEngine::unwrap(TCPOverIPv4Adapter& adapter,
                                                           std::span<const InternetDatagram> dgrams)
{
    // TCPSegment::parse's checksum (value() of pseudo + all payload bytes) on
    // the GPU for the whole batch (each datagram's payload pieces written into
    // the page-locked arena on the engine workers), then the field parse of
    // every datagram that passed (pure: on the workers, one payload copy out
    // of the arena) and the adapter's gates in datagram order on this thread
    const size_t n = dgrams.size();
    std::vector<std::optional<TCPMessage>> out(n);
    if (n == 0) return out;
    std::vector<uint32_t> init(n);
    const auto off = pack(
        n,
        [&](size_t i) {
            size_t b = 0;
            for (const auto& piece : dgrams[i].payload) b += piece.size();
            return b;
        },
        [&](size_t i, uint8_t* d) {
            for (const auto& piece : dgrams[i].payload) {
                std::memcpy(d, piece.data(), piece.size());
                d += piece.size();
            }
            init[i] = dgrams[i].header.pseudo_checksum();
        });
    std::vector<uint16_t> v(n);
    check(ics_checksum_batch_host(ctx_, scratch_, off.data(), 0, 0, init.data(), v.data(), n),
          "ics_checksum_batch_host");
    struct Parsed
    {
        bool ok = false;
        TCPSegment seg{};
    };
    std::vector<Parsed> parsed(n);
    ranges(n, [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i)
            if (v[i] == 0)
                parsed[i].ok = detail::parse_tcp_fields(
                    std::string_view{reinterpret_cast<const char*>(scratch_) + off[i], off[i + 1] - off[i]},
                    parsed[i].seg);
    });
    for (size_t i = 0; i < n; ++i) {
        const IPv4Header& h = dgrams[i].header;
        if (!detail::ip_gate(adapter, h) || v[i] != 0 || !parsed[i].ok) continue;
        out[i] = detail::tcp_gate(adapter, h, std::move(parsed[i].seg));
    }
    return out;
}

std::vector<std::optional<TCPMessage>> BatchEngine::unwrap_raw(TCPOverIPv4Adapter& adapter,
                                                               std::span<const std::string_view> wires)
{
    if (wires.empty()) return {};
    const auto off = pack(
        wires.size(), [&](size_t i) { return wires[i].size(); },
        [&](size_t i, uint8_t* d) { std::memcpy(d, wires[i].data(), wires[i].size()); });
    return unwrap_packed(adapter, scratch_, off.data(), wires.size());
}

std::vector<uint8_t> BatchEngine::verify_packed(const uint8_t* bytes, const uint64_t* offsets, size_t n)
{
    std::vector<uint8_t> st(n);
    if (n)
        check(ics_ipv4_tcp_batch_host(ctx_, const_cast<uint8_t*>(bytes), offsets, 0, 0, n, ICS_MODE_VERIFY, nullptr,
                                      nullptr, st.data()),
              "ics_ipv4_tcp_batch_host");
    return st;
}

void BatchEngine::patch_packed(uint8_t* bytes, const uint64_t* offsets, size_t n)
{
    if (n)
        check(ics_ipv4_tcp_batch_host(ctx_, bytes, offsets, 0, 0, n, ICS_MODE_PATCH, nullptr, nullptr, nullptr),
              "ics_ipv4_tcp_batch_host");
}

void BatchEngine::set_tick_server(uint32_t idle_us)
{
    check(ics_set_tick_server(ctx_, idle_us), "ics_set_tick_server");
}

void BatchEngine::set_tick_server_blocks(uint32_t blocks)
{
    check(ics_set_tick_server_blocks(ctx_, blocks), "ics_set_tick_server_blocks");
}

void* BatchEngine::host_alloc(size_t bytes)
{
    void* p = nullptr;
    check(ics_host_alloc(ctx_, &p, bytes), "ics_host_alloc");
    return p;
}

void BatchEngine::host_free(void* p) { ics_host_free(ctx_, p); }

std::vector<std::optional<TCPMessage>> BatchEngine::unwrap_packed(TCPOverIPv4Adapter& adapter, const uint8_t* bytes,
                                                                  const uint64_t* offsets, size_t n)
{
    // receive path from raw wire datagrams (a TUN / socket read batch):
    // IPv4 parse + TCP checksum verified on the GPU, fields parsed on the host
    const std::vector<uint8_t> st = verify_packed(bytes, offsets, n);
    // 1) field parse of every verified datagram: pure, so it runs on up to 8
    //    threads (contiguous ranges); 2) the adapter's gates in datagram
    //    order on this thread (tcp_gate's listen -> connected transition
    //    changes what ip_gate lets through for every later datagram)
    struct Parsed
    {
        bool ok = false;
        IPv4Header ip{};
        TCPSegment seg{};
    };
    std::vector<Parsed> parsed(n);
    auto parse_range = [&](size_t i0, size_t i1) {
        for (size_t i = i0; i < i1; ++i) {
            if ((st[i] & (ICS_ST_IPV4_OK | ICS_ST_TCP_CKSUM_OK | ICS_ST_TCP_HDR_OK)) !=
                (ICS_ST_IPV4_OK | ICS_ST_TCP_CKSUM_OK | ICS_ST_TCP_HDR_OK))
                continue;
            const std::string_view wire{reinterpret_cast<const char*>(bytes) + offsets[i],
                                        static_cast<size_t>(offsets[i + 1] - offsets[i])};
            IPv4Header& h = parsed[i].ip;
            // the 20 fixed header bytes, big-endian, read in place (IPV4_OK
            // implies at least 20 bytes); fields only, the GPU already
            // compared the header checksum
            auto u8 = [&](size_t k) { return static_cast<uint8_t>(wire[k]); };
            auto be16 = [&](size_t k) { return static_cast<uint16_t>((u8(k) << 8) | u8(k + 1)); };
            h.ver = u8(0) >> 4;
            h.hlen = u8(0) & 0x0f;
            h.tos = u8(1);
            h.len = be16(2);
            h.id = be16(4);
            const uint16_t fo = be16(6);
            h.df = (fo & 0x4000) != 0;
            h.mf = (fo & 0x2000) != 0;
            h.offset = fo & 0x1fff;
            h.ttl = u8(8);
            h.proto = u8(9);
            h.cksum = be16(10);
            h.src = (static_cast<uint32_t>(be16(12)) << 16) | be16(14);
            h.dst = (static_cast<uint32_t>(be16(16)) << 16) | be16(18);
            // all bytes after the options (ipv4_header.cpp:50, then the
            // datagram's remaining buffer as the TCP segment); a header
            // longer than the datagram leaves nothing, and the TCP parse
            // fails; the payload is copied once, straight from the batch
            const size_t hdr_bytes = static_cast<size_t>(h.hlen) * 4;
            parsed[i].ok = detail::parse_tcp_fields(
                hdr_bytes <= wire.size() ? wire.substr(hdr_bytes) : std::string_view{}, parsed[i].seg);
        }
    };
    ranges(n, parse_range);
    std::vector<std::optional<TCPMessage>> out(n);
    for (size_t i = 0; i < n; ++i) {
        if ((st[i] & (ICS_ST_IPV4_OK | ICS_ST_TCP_CKSUM_OK | ICS_ST_TCP_HDR_OK)) !=
            (ICS_ST_IPV4_OK | ICS_ST_TCP_CKSUM_OK | ICS_ST_TCP_HDR_OK))
            continue;
        if (!detail::ip_gate(adapter, parsed[i].ip)) continue;
        if (!parsed[i].ok) continue;
        out[i] = detail::tcp_gate(adapter, parsed[i].ip, std::move(parsed[i].seg));
    }
    return out;
}

}  // namespace icsum
