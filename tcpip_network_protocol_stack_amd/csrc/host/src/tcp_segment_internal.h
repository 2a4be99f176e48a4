// tcp_segment_internal.h — not installed.  The field half of TCPSegment::parse,
// shared with the batch engine, which verifies checksums on the GPU first.
#pragma once

#include "tcp_segment.h"

namespace icsum::detail {
// tcp_segment.cpp:25-65: header fields, flags, data offset, payload
void parse_tcp_fields(Parser& parser, TCPSegment& seg);
uint32_t raw_of(const Wrap32& w);
}  // namespace icsum::detail
