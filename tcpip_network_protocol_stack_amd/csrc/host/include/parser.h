// parser.h — drop-in Parser / Serializer (reference: util/tools/parser.h:17-289).
//
// Same API and error behaviour: Parser reads big-endian integers out of a
// list of string pieces and sets an error flag (never throws) on underflow;
// Serializer appends big-endian integers to a pending buffer and whole string
// pieces (taken by value, not copied twice) to its output list.  parse<T>() and
// serialize<T>() are the generic entry points the stack calls.
//
// Implementation differs from the reference: the parser keeps the pieces in a
// vector with a (piece, offset) cursor instead of a deque of owned strings.
#ifndef ICSUM_HOST_PARSER_H
#define ICSUM_HOST_PARSER_H

#include <algorithm>
#include <concepts>
#include <cstdint>
#include <cstring>
#include <span>
#include <stdexcept>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

class Parser
{
    class BufferList
    {
        std::vector<std::string> pieces_{};
        size_t piece_ = 0;   // first piece with unread bytes
        uint64_t skip_ = 0;  // bytes already consumed from pieces_[piece_]
        uint64_t size_ = 0;  // unread bytes in total

        void settle()
        {
            while (piece_ < pieces_.size() && skip_ == pieces_[piece_].size()) {
                ++piece_;
                skip_ = 0;
            }
        }

      public:
        explicit BufferList(const std::vector<std::string>& buffers)
        {
            for (const auto& b : buffers) append(b);
        }

        uint64_t size() const { return size_; }
        uint64_t serialized_length() const { return size_; }
        bool empty() const { return size_ == 0; }

        std::string_view peek() const
        {
            if (piece_ >= pieces_.size()) throw std::runtime_error("peek on empty BufferList");
            return std::string_view{pieces_[piece_]}.substr(skip_);
        }

        void remove_prefix(uint64_t len)
        {
            while (len > 0 && piece_ < pieces_.size()) {
                const uint64_t avail = pieces_[piece_].size() - skip_;
                const uint64_t take = std::min(len, avail);
                skip_ += take;
                size_ -= take;
                len -= take;
                settle();
            }
        }

        void dump_all(std::vector<std::string>& out)
        {
            out.clear();
            for (size_t i = piece_; i < pieces_.size(); ++i) {
                std::string s = std::move(pieces_[i]);
                if (i == piece_ && skip_) s.erase(0, skip_);
                if (!s.empty()) out.emplace_back(std::move(s));
            }
            pieces_.clear();
            piece_ = 0;
            skip_ = 0;
            size_ = 0;
        }

        void dump_all(std::string& out)
        {
            std::vector<std::string> parts;
            dump_all(parts);
            if (parts.size() == 1) {
                out = std::move(parts.front());
                return;
            }
            out.clear();
            for (const auto& s : parts) out.append(s);
        }

        std::vector<std::string_view> buffer() const
        {
            std::vector<std::string_view> r;
            if (empty()) return r;
            r.reserve(pieces_.size() - piece_);
            for (size_t i = piece_; i < pieces_.size(); ++i)
                r.push_back(std::string_view{pieces_[i]}.substr(i == piece_ ? skip_ : 0));
            return r;
        }

        void append(std::string str)
        {
            size_ += str.size();
            if (!str.empty()) pieces_.push_back(std::move(str));
            settle();
        }
    };

    BufferList input_;
    bool error_{};

    void check_size(size_t size)
    {
        if (size > input_.size()) error_ = true;
    }

  public:
    explicit Parser(const std::vector<std::string>& input) : input_(input) {}

    const BufferList& input() const { return input_; }
    bool has_error() const { return error_; }
    void set_error() { error_ = true; }
    void remove_prefix(size_t n) { input_.remove_prefix(n); }

    // big-endian unsigned integer; sets the error flag if too few bytes remain
    template <std::unsigned_integral T>
    void integer(T& out)
    {
        check_size(sizeof(T));
        if (has_error()) return;
        T v = 0;
        for (size_t i = 0; i < sizeof(T); ++i) {
            if constexpr (sizeof(T) > 1) v <<= 8;
            v |= static_cast<uint8_t>(input_.peek().front());
            input_.remove_prefix(1);
        }
        out = v;
    }

    void string(std::span<char> out)
    {
        check_size(out.size());
        if (has_error()) return;
        size_t done = 0;
        while (done < out.size()) {
            const auto view = input_.peek().substr(0, out.size() - done);
            std::memcpy(out.data() + done, view.data(), view.size());
            done += view.size();
            input_.remove_prefix(view.size());
        }
    }

    void all_remaining(std::vector<std::string>& out) { input_.dump_all(out); }
    void all_remaining(std::string& out) { input_.dump_all(out); }
    std::vector<std::string_view> buffer() const { return input_.buffer(); }
};

class Serializer
{
    std::vector<std::string> output_{};
    std::string buffer_{};

  public:
    Serializer() = default;
    explicit Serializer(std::string&& buffer) : buffer_(std::move(buffer)) {}

    template <std::unsigned_integral T>
    void integer(const T val)
    {
        for (size_t i = sizeof(T); i-- > 0;) buffer_.push_back(static_cast<char>(static_cast<uint8_t>(val >> (8 * i))));
    }

    void buffer(std::string buf)
    {
        flush();
        if (!buf.empty()) output_.push_back(std::move(buf));
    }

    void buffer(const std::vector<std::string>& bufs)
    {
        for (const auto& b : bufs) buffer(b);
    }

    void flush()
    {
        if (!buffer_.empty()) {
            output_.emplace_back(std::move(buffer_));
            buffer_.clear();
        }
    }

    const std::vector<std::string>& output()
    {
        flush();
        return output_;
    }
};

template <typename T>
std::vector<std::string> serialize(const T& obj)
{
    Serializer s;
    obj.serialize(s);
    return s.output();
}

template <typename T, typename... Targs>
bool parse(T& obj, const std::vector<std::string>& buffers, Targs&&... Fargs)
{
    Parser p{buffers};
    obj.parse(p, std::forward<Targs>(Fargs)...);
    return !p.has_error();
}

#endif
