// address.h — standalone stand-in for the reference's Address
// (util/address/address.h:14-70), used only when this layer is built WITHOUT
// the reference tree (here and on the GPU box; see udinfo.h in this
// directory).  It is the part the TCP-over-IPv4 adapter needs: an IPv4
// address + port value type with the reference's signatures.  Integrated into
// the reference, the reference's own Address (sockaddr storage, resolution,
// Raw) is the one found and linked: the engine replaces nothing in it.
#ifndef ADDRESS_H  // the reference header's guard
#define ADDRESS_H

#include <cstdint>
#include <string>
#include <utility>

class Address
{
    uint32_t ip_ = 0;  // host order
    uint16_t port_ = 0;

  public:
    explicit Address(const std::string& ip, std::uint16_t port = 0);
    bool operator==(const Address& o) const { return ip_ == o.ip_ && port_ == o.port_; }
    bool operator!=(const Address& o) const { return !operator==(o); }
    std::pair<std::string, uint16_t> ip_port() const { return {ip(), port_}; }
    std::string ip() const;
    uint16_t port() const { return port_; }
    uint32_t ipv4_numeric() const { return ip_; }
    static Address from_ipv4_numeric(uint32_t ip_address);
    std::string to_string() const { return ip() + ":" + std::to_string(port_); }
};

#endif
