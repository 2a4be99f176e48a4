// tcp_over_ip.h — drop-in TCPOverIPv4Adapter (reference: util/tcp_over_ip/tcp_over_ip.h:10-18)
#ifndef ICSUM_HOST_TCP_OVER_IP_H
#define ICSUM_HOST_TCP_OVER_IP_H

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
