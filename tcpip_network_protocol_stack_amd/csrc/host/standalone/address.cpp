// address.cpp — numeric IPv4 Address (see address.h; reference util/address/address.cpp:124-146)
#include "address.h"

#include <arpa/inet.h>

#include <stdexcept>

Address::Address(const std::string& ip, std::uint16_t port) : port_(port)
{
    in_addr a{};
    // inet_aton accepts the shorthand forms ("0", "10.1") that the reference's
    // numeric getaddrinfo lookup accepts
    if (inet_aton(ip.c_str(), &a) == 0) throw std::runtime_error("Address: not a numeric IPv4 address: " + ip);
    ip_ = ntohl(a.s_addr);
}

std::string Address::ip() const
{
    in_addr a{};
    a.s_addr = htonl(ip_);
    char buf[INET_ADDRSTRLEN] = {};
    inet_ntop(AF_INET, &a, buf, sizeof buf);
    return buf;
}

Address Address::from_ipv4_numeric(uint32_t ip_address)
{
    Address a{"0", 0};
    a.ip_ = ip_address;
    return a;
}
