// parser.h — the stack's byte codec: Parser, Serializer, parse<T>(),
// serialize<T>() (reference util/tools/parser.h:17-289).
//
// Contract kept from the reference (the stack's code and its error handling
// depend on it):
//   * input and output are lists of std::string pieces; a value may straddle
//     two pieces;
//   * integers are big-endian; a read past the end sets the error flag and
//     leaves the destination untouched — Parser never throws on short input;
//   * all_remaining() hands the unread bytes over piece by piece (the first one
//     trimmed), buffer() views them without copying — TCPSegment::parse
//     checksums exactly those views;
//   * Serializer gathers integers in a pending piece and appends whole
//     strings as their own pieces, so a payload is moved, never re-copied.
//
// Representation (ours): the Parser owns the pieces in a vector and keeps a
// flat read cursor (piece index + offset into it).  Reads that fit in the
// current piece take one memcpy + byte swap instead of a byte loop.  The
// reference's nested BufferList and Parser::input() accessor are not part of
// this surface: nothing on the stack's path uses them.
#ifndef PARSER_H  // the reference header's guard
#define PARSER_H

#include <algorithm>
#include <concepts>
#include <cstdint>
#include <cstring>
#include <span>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace icsum::detail {
template <std::unsigned_integral T>
constexpr T from_big_endian(T v)
{
    if constexpr (sizeof(T) == 1) return v;
    else if constexpr (sizeof(T) == 2) return static_cast<T>(__builtin_bswap16(v));
    else if constexpr (sizeof(T) == 4) return static_cast<T>(__builtin_bswap32(v));
    else return static_cast<T>(__builtin_bswap64(v));
}
}  // namespace icsum::detail

class Parser
{
    std::vector<std::string> chunks_{};
    size_t cur_ = 0;         // index of the chunk the cursor is in
    size_t pos_ = 0;         // cursor offset inside chunks_[cur_]
    uint64_t remaining_ = 0; // unread bytes across all chunks
    bool error_ = false;

    // advance past exhausted chunks so chunks_[cur_] (if any) has unread bytes
    void normalise()
    {
        while (cur_ < chunks_.size() && pos_ >= chunks_[cur_].size()) {
            ++cur_;
            pos_ = 0;
        }
    }

    // copy n unread bytes (n <= remaining_) into dst and consume them
    void take(char* dst, size_t n)
    {
        while (n) {
            const std::string& c = chunks_[cur_];
            const size_t k = std::min(n, c.size() - pos_);
            std::memcpy(dst, c.data() + pos_, k);
            dst += k;
            n -= k;
            pos_ += k;
            remaining_ -= k;
            normalise();
        }
    }

    bool need(uint64_t n)
    {
        if (n > remaining_) error_ = true;
        return !error_;
    }

  public:
    explicit Parser(const std::vector<std::string>& input) : chunks_()
    {
        chunks_.reserve(input.size());
        for (const std::string& s : input) {
            if (s.empty()) continue;
            remaining_ += s.size();
            chunks_.push_back(s);
        }
    }

    bool has_error() const { return error_; }
    void set_error() { error_ = true; }

    // skip up to n bytes (clamped at the end of the input, never an error)
    void remove_prefix(size_t n)
    {
        uint64_t left = std::min<uint64_t>(n, remaining_);
        remaining_ -= left;
        while (left) {
            const size_t k = std::min<uint64_t>(left, chunks_[cur_].size() - pos_);
            pos_ += k;
            left -= k;
            normalise();
        }
        normalise();
    }

    template <std::unsigned_integral T>
    void integer(T& out)
    {
        if (!need(sizeof(T))) return;
        T raw;
        const std::string& c = chunks_[cur_];
        if (c.size() - pos_ >= sizeof(T)) {  // common case: one memcpy
            std::memcpy(&raw, c.data() + pos_, sizeof(T));
            pos_ += sizeof(T);
            remaining_ -= sizeof(T);
            normalise();
        } else {
            take(reinterpret_cast<char*>(&raw), sizeof(T));
        }
        out = icsum::detail::from_big_endian(raw);
    }

    void string(std::span<char> out)
    {
        if (!need(out.size())) return;
        take(out.data(), out.size());
    }

    void all_remaining(std::vector<std::string>& out)
    {
        out.clear();
        for (; cur_ < chunks_.size(); ++cur_, pos_ = 0) {
            std::string& c = chunks_[cur_];
            if (pos_) c.erase(0, pos_);
            if (!c.empty()) out.push_back(std::move(c));
        }
        chunks_.clear();
        cur_ = pos_ = 0;
        remaining_ = 0;
    }

    void all_remaining(std::string& out)
    {
        std::vector<std::string> parts;
        all_remaining(parts);
        if (parts.size() == 1) {
            out = std::move(parts[0]);
            return;
        }
        out.clear();
        out.reserve(remaining_bytes(parts));
        for (const std::string& p : parts) out += p;
    }

    std::vector<std::string_view> buffer() const
    {
        std::vector<std::string_view> views;
        if (remaining_ == 0) return views;
        views.reserve(chunks_.size() - cur_);
        views.emplace_back(chunks_[cur_].data() + pos_, chunks_[cur_].size() - pos_);
        for (size_t i = cur_ + 1; i < chunks_.size(); ++i) views.emplace_back(chunks_[i]);
        return views;
    }

  private:
    static size_t remaining_bytes(const std::vector<std::string>& parts)
    {
        size_t n = 0;
        for (const std::string& p : parts) n += p.size();
        return n;
    }
};

class Serializer
{
    std::vector<std::string> pieces_{};
    std::string pending_{};  // integers written since the last whole piece

  public:
    Serializer() = default;
    explicit Serializer(std::string&& buffer) : pending_(std::move(buffer)) {}

    template <std::unsigned_integral T>
    void integer(const T val)
    {
        const T be = icsum::detail::from_big_endian(val);  // the swap is its own inverse
        pending_.append(reinterpret_cast<const char*>(&be), sizeof(T));
    }

    void buffer(std::string buf)
    {
        flush();
        if (!buf.empty()) pieces_.push_back(std::move(buf));
    }

    void buffer(const std::vector<std::string>& bufs)
    {
        for (const std::string& b : bufs) buffer(b);
    }

    void flush()
    {
        if (pending_.empty()) return;
        pieces_.push_back(std::move(pending_));
        pending_.clear();
    }

    const std::vector<std::string>& output()
    {
        flush();
        return pieces_;
    }
};

// obj.serialize(Serializer&) -> its pieces
template <typename T>
std::vector<std::string> serialize(const T& obj)
{
    Serializer out;
    obj.serialize(out);
    return out.output();
}

// obj.parse(Parser&, extra...) over `buffers`; true iff no error was flagged
template <typename T, typename... Targs>
bool parse(T& obj, const std::vector<std::string>& buffers, Targs&&... Fargs)
{
    Parser in{buffers};
    obj.parse(in, std::forward<Targs>(Fargs)...);
    return !in.has_error();
}

#endif
