// udinfo.h — standalone stand-in for the reference's util/tools/udinfo.h:7-12,
// used only when this layer is built WITHOUT the reference tree (here and on
// the GPU box).  Integrated into the reference, the reference's own header is
// the one found: the engine replaces no type in it.
#ifndef UDINFO_H
#define UDINFO_H

#include <cstdint>

// Ports + the TCP checksum field (named after UDP in the reference).
struct UserDatagramInfo
{
    uint16_t src_port;
    uint16_t dst_port;
    uint16_t cksum;
};

#endif
