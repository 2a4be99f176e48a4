// ref_shim.cpp — TEST INFRASTRUCTURE ONLY (bench.py cpu_baseline, kind "reference").
//
// A C-ABI wrapper over the reference's own InternetChecksum
// (util/tools/checksum.h:9-60, compiled from /root/reference by
// oracle/ref/Makefile into oracle/_ref/libref_icsum.so).  Per segment it does
// exactly what TCPSegment::compute_checksum does with the payload
// (tcp_segment.cpp:109-118): InternetChecksum{pseudo}.add(view).value().
#include <cstdint>
#include <string_view>
#include <thread>
#include <vector>

#include "checksum.h"

namespace {
void run(const uint8_t* bytes, const uint64_t* offsets, uint64_t stride, uint64_t seg_len,
         const uint32_t* init, uint16_t* out, uint64_t lo, uint64_t hi) {
  for (uint64_t i = lo; i < hi; ++i) {
    const uint64_t b = offsets ? offsets[i] : i * stride;
    const uint64_t e = offsets ? offsets[i + 1] : b + seg_len;
    InternetChecksum c{init ? init[i] : 0u};
    c.add(std::string_view{reinterpret_cast<const char*>(bytes) + b, size_t(e - b)});
    out[i] = c.value();
  }
}
}  // namespace

extern "C" int ref_checksum_batch(const uint8_t* bytes, const uint64_t* offsets, uint64_t stride,
                                  uint64_t seg_len, const uint32_t* init, uint16_t* out,
                                  uint64_t n, int threads) {
  if (threads <= 1 || n < uint64_t(threads)) {
    run(bytes, offsets, stride, seg_len, init, out, 0, n);
    return 0;
  }
  std::vector<std::thread> th;
  th.reserve(size_t(threads));
  for (int t = 0; t < threads; ++t)
    th.emplace_back(run, bytes, offsets, stride, seg_len, init, out, n * uint64_t(t) / uint64_t(threads),
                    n * uint64_t(t + 1) / uint64_t(threads));
  for (auto& x : th) x.join();
  return 0;
}
