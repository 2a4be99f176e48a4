// checksum.h — drop-in InternetChecksum (reference: util/tools/checksum.h:9-60).
//
// Same public surface and bit-exact semantics as the reference value type:
// bytes are big-endian 16-bit halves by their position in the add() stream
// (parity carried across add() calls), a uint32 accumulator that wraps mod
// 2^32, and value() = ~fold(sum).  Single objects stay on the CPU (a GPU
// launch would cost more than a 20-1500 byte sum); batches go to the MI355X
// engine through icsum::BatchEngine (batch.h) and the C-ABI (include/icsum.h).
//
// add() works 8 bytes at a time: for a little-endian 64-bit load w, the bytes
// at even offsets sum to the four 16-bit lanes of (w & 0x00FF00FF00FF00FF) and
// the odd ones to those of ((w >> 8) & ...); partial lane sums are folded into
// sum_ before they can overflow, so sum_ matches the byte loop exactly.
#ifndef CHECKSUM_H  // the reference header's guard
#define CHECKSUM_H

#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

class InternetChecksum
{
  private:
    uint32_t sum_;  // running sum, wraps mod 2^32 (checksum.h:12)
    bool parity_;   // true: the next byte is a low byte (checksum.h:13)

    static uint32_t lanes16(uint64_t x)
    {
        return static_cast<uint32_t>((x & 0xffffu) + ((x >> 16) & 0xffffu) + ((x >> 32) & 0xffffu) + (x >> 48));
    }

  public:
    explicit InternetChecksum(uint32_t sum = 0) : sum_(sum), parity_(false) {}

    void add(std::string_view data)
    {
        const auto* p = reinterpret_cast<const unsigned char*>(data.data());
        size_t n = data.size();
        if (parity_ && n) {  // finish the pending low byte
            sum_ += *p++;
            --n;
            parity_ = false;
        }
        uint64_t hi = 0, lo = 0;  // 4 lanes x 16 bits each; <= 257 adds per lane before a flush
        unsigned pending = 0;
        while (n >= 8) {
            uint64_t w;
            std::memcpy(&w, p, 8);
            hi += w & 0x00ff00ff00ff00ffull;         // bytes 0,2,4,6 -> high halves
            lo += (w >> 8) & 0x00ff00ff00ff00ffull;  // bytes 1,3,5,7 -> low halves
            p += 8;
            n -= 8;
            if (++pending == 256) {
                sum_ += (lanes16(hi) << 8) + lanes16(lo);
                hi = lo = 0;
                pending = 0;
            }
        }
        sum_ += (lanes16(hi) << 8) + lanes16(lo);
        for (size_t i = 0; i < n; ++i) {
            sum_ += parity_ ? p[i] : static_cast<uint32_t>(p[i]) << 8;
            parity_ = !parity_;
        }
    }

    uint16_t value() const
    {
        uint32_t r = sum_;
        while (r > 0xffff) r = (r >> 16) + (r & 0xffff);
        return static_cast<uint16_t>(~r);
    }

    void add(const std::vector<std::string>& data)
    {
        for (const auto& s : data) add(std::string_view{s});
    }

    void add(const std::vector<std::string_view>& data)
    {
        for (const auto v : data) add(v);
    }

    // engine interop (not in the reference): the raw running state, e.g. to
    // seed a device batch (ics_sum_batch) with a header computed on the host
    uint32_t raw_sum() const { return sum_; }
    bool odd() const { return parity_; }
};

#endif
