// icsum_wire.h — the stack's wire objects in one place: every type the
// checksum path reads, fills or hands to the MI355X engine.
//
// The reference spreads these over eight headers (util/tools/udinfo.h,
// tcp_sender_message.h, tcp_receiver_message.h, ipv4_datagram.h, tcp_config.h,
// fd_adapter.h, util/tcp_segment/tcp_segment.h, util/tcp_over_ip/tcp_over_ip.h).
// The stack's own sources #include those names, so each of them still exists
// in this directory as a one-line forwarder to this file; member names, member
// order (aggregate initialisation depends on it) and signatures are the
// reference's, so src/tcp_sender, src/tcp_receiver & co. compile unchanged.
//
// Byte map of one TCP-in-IPv4 datagram as the device kernels see it
// (k_ipv4_tcp, csrc/kernels/icsum_kernels.hip), with the member that owns
// each field:
//
//   IPv4 [0,20)   IPv4Header                     (ipv4_header.h)
//   TCP  [0,2)    UserDatagramInfo::src_port
//        [2,4)    UserDatagramInfo::dst_port
//        [4,8)    TCPSenderMessage::seqno        raw Wrap32
//        [8,12)   TCPReceiverMessage::ackno      0 when absent
//        [12]     data offset << 4               always 5 when serialized
//        [13]     flags  ACK 0x10  RST 0x04  SYN 0x02  FIN 0x01
//        [14,16)  TCPReceiverMessage::window_size
//        [16,18)  UserDatagramInfo::cksum        the engine's tcp_ck output
//        [18,20)  urgent pointer                 always 0
//        [20,..)  TCPSenderMessage::payload
#ifndef ICSUM_HOST_WIRE_H
#define ICSUM_HOST_WIRE_H

#include <cstddef>
#include <cstdint>
#include <optional>
#include <string>
#include <vector>

#include "address.h"
#include "ipv4_header.h"
#include "parser.h"
#include "wrapping_integers.h"

// =====================================================================
// Per-segment field holders (reference util/tools/*.h)
// =====================================================================

// Ports + the TCP checksum field; named after UDP in the reference
// (util/tools/udinfo.h:7-12).
struct UserDatagramInfo
{
    uint16_t src_port;
    uint16_t dst_port;
    uint16_t cksum;
};

// What the sending side puts in a segment (util/tools/tcp_sender_message.h:25-40).
struct TCPSenderMessage
{
    Wrap32 seqno{0};
    bool SYN{};
    std::string payload{};
    bool FIN{};
    bool RST{};

    // SYN and FIN each occupy one sequence number
    size_t sequence_length() const { return static_cast<size_t>(SYN) + payload.size() + static_cast<size_t>(FIN); }
};

// What the receiving side puts in a segment (util/tools/tcp_receiver_message.h:22-27).
struct TCPReceiverMessage
{
    std::optional<Wrap32> ackno{};
    uint16_t window_size{};
    bool RST{};
};

// util/tcp_segment/tcp_segment.h:10-14
struct TCPMessage
{
    TCPSenderMessage sender{};
    TCPReceiverMessage receiver{};
};

// =====================================================================
// Codec objects (implemented in src/tcp_segment.cpp; IPv4Header lives in
// ipv4_header.h)
// =====================================================================

// util/tcp_segment/tcp_segment.h:16-30.  parse() checks
// InternetChecksum{pseudo} over ALL bytes it is handed before reading a field;
// compute_checksum() stores the value the engine's COMPUTE mode produces.
struct TCPSegment
{
    TCPMessage message{};
    UserDatagramInfo udinfo{};

    void parse(Parser& parser, uint32_t datagram_layer_pseudo_checksum);
    void serialize(Serializer& serializer) const;
    void compute_checksum(uint32_t datagram_layer_pseudo_checksum);
};

// A header plus its payload pieces (util/tools/ipv4_datagram.h:10-34).  The
// pieces are kept as the Parser hands them over: no concatenation here.
struct IPv4Datagram
{
    IPv4Header header{};
    std::vector<std::string> payload{};

    void parse(Parser& parser)
    {
        header.parse(parser);
        parser.all_remaining(payload);
    }

    void serialize(Serializer& serializer) const
    {
        header.serialize(serializer);
        serializer.buffer(payload);
    }
};

using InternetDatagram = IPv4Datagram;

// =====================================================================
// Adapter configuration and the TCP-over-IPv4 adapter
// =====================================================================

// util/tools/tcp_config.h:11-27.  src/tcp_sender reads MAX_PAYLOAD_SIZE and
// the capacities; the values are the reference's.
class TCPConfig
{
  public:
    static constexpr size_t DEFAULT_CAPACITY = 64000;
    static constexpr size_t MAX_PAYLOAD_SIZE = 1000;
    static constexpr uint16_t TIMEOUT_DFLT = 1000;
    static constexpr unsigned MAX_RETX_ATTEMPTS = 8;

    uint16_t rt_timeout = TIMEOUT_DFLT;
    size_t recv_capacity = DEFAULT_CAPACITY;
    size_t send_capacity = DEFAULT_CAPACITY;
    Wrap32 isn{137};
};

// util/tools/tcp_config.h:30-42: the two endpoints the adapter filters on
// (loss rates are carried for source compatibility; nothing here drops).
class FdAdapterConfig
{
  public:
    Address source{"0", 0};
    Address destination{"0", 0};
    uint16_t loss_rate_dn = 0;
    uint16_t loss_rate_up = 0;
};

// util/tools/fd_adapter.h:13-38 reduced to its state: the endpoint
// configuration and the listen flag.  The file-descriptor / lossy-adapter
// runtime around it is outside this engine.
class FdAdapterBase
{
    FdAdapterConfig endpoints_{};
    bool listen_ = false;

  protected:
    FdAdapterConfig& config_mutable() { return endpoints_; }

  public:
    bool listening() const { return listen_; }
    void set_listening(const bool l) { listen_ = l; }
    const FdAdapterConfig& config() const { return endpoints_; }
    FdAdapterConfig& config_mut() { return endpoints_; }
    void tick(const size_t /*ms_since_last_tick*/) {}
};

// util/tcp_over_ip/tcp_over_ip.h:10-18.  Per-object calls run on the host
// (src/tcp_over_ip.cpp); icsum::BatchEngine::wrap / unwrap (batch.h) apply the
// same rules to whole batches with the checksums on the GPU.
class TCPOverIPv4Adapter : public FdAdapterBase
{
  public:
    std::optional<TCPMessage> unwrap_tcp_in_ip(const InternetDatagram& ip_dgram);
    InternetDatagram wrap_tcp_in_ip(const TCPMessage& msg);
};

#endif
