// wrapping_integers.h — the Wrap32 TYPE the checksum path serializes
// (reference: src/wrapping_integers/wrapping_integers.h:12-41).  Layout and
// interface match the reference so the stack's own src/ compiles against
// these headers; wrap()/unwrap() are the stack's logic (out of this engine's
// scope) and are defined by the stack's wrapping_integers.cpp when linked.
#ifndef WRAPPING_INTEGERS_H  // same guard as the stack's own header: either one defines Wrap32
#define WRAPPING_INTEGERS_H

#include <cstdint>

class Wrap32
{
  public:
    explicit Wrap32(uint32_t raw_value) : raw_value_(raw_value) {}
    static Wrap32 wrap(uint64_t n, Wrap32 zero_point);
    uint64_t unwrap(Wrap32 zero_point, uint64_t checkpoint) const;
    Wrap32 operator+(uint32_t n) const { return Wrap32{raw_value_ + n}; }
    bool operator==(const Wrap32& other) const { return raw_value_ == other.raw_value_; }

  protected:
    uint32_t raw_value_{};
};

#endif
