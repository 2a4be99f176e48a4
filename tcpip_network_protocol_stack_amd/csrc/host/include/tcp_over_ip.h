// tcp_over_ip.h — drop-in TCPOverIPv4Adapter (reference:
// util/tcp_over_ip/tcp_over_ip.h:10-18).  Per-object calls run on the host
// (src/tcp_over_ip.cpp) with the reference's rules; icsum::BatchEngine::wrap /
// unwrap (batch.h) apply the same rules to whole batches with the checksums
// on the GPU.  FdAdapterBase and IPv4Datagram are the reference's own
// (util/tools/fd_adapter.h, ipv4_datagram.h) when integrated.
#ifndef TCP_OVER_IP_H  // the reference header's guard
#define TCP_OVER_IP_H

#include <optional>

#include "fd_adapter.h"
#include "ipv4_datagram.h"
#include "tcp_segment.h"

class TCPOverIPv4Adapter : public FdAdapterBase
{
  public:
    std::optional<TCPMessage> unwrap_tcp_in_ip(const InternetDatagram& ip_dgram);
    InternetDatagram wrap_tcp_in_ip(const TCPMessage& msg);
};

#endif
