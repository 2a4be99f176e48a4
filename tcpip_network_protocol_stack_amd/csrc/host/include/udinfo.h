// udinfo.h — reference: util/tools/udinfo.h:7-12 (holds the TCP checksum field)
#ifndef ICSUM_HOST_UDINFO_H
#define ICSUM_HOST_UDINFO_H

#include <cstdint>

struct UserDatagramInfo
{
    uint16_t src_port;
    uint16_t dst_port;
    uint16_t cksum;
};

#endif
