// batch_io.cpp — icsum::DatagramBatch (see batch_io.h)
#include "batch_io.h"

#include <errno.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>

namespace icsum {
namespace {

bool is_datagram_socket(int fd)
{
    int type = 0;
    socklen_t len = sizeof type;
    return getsockopt(fd, SOL_SOCKET, SO_TYPE, &type, &len) == 0 && (type == SOCK_DGRAM || type == SOCK_SEQPACKET);
}

[[noreturn]] void sys_fail(const char* what)
{
    throw std::runtime_error(std::string(what) + ": " + std::strerror(errno));
}

}  // namespace

DatagramBatch::DatagramBatch(BatchEngine& engine, size_t capacity_bytes, size_t max_datagrams)
    : engine_(&engine), cap_(capacity_bytes), max_n_(max_datagrams)
{
    arena_ = static_cast<uint8_t*>(engine.host_alloc(cap_));
    off_.reserve(max_n_ + 1);
}

DatagramBatch::DatagramBatch(size_t capacity_bytes, size_t max_datagrams) : cap_(capacity_bytes), max_n_(max_datagrams)
{
    arena_ = static_cast<uint8_t*>(std::malloc(cap_ ? cap_ : 1));
    if (!arena_) throw std::bad_alloc();
    off_.reserve(max_n_ + 1);
}

DatagramBatch::~DatagramBatch()
{
    if (engine_)
        engine_->host_free(arena_);
    else
        std::free(arena_);
}

bool DatagramBatch::push(std::string_view wire)
{
    if (!room(wire.size())) return false;
    std::memcpy(arena_ + bytes(), wire.data(), wire.size());
    off_.push_back(bytes() + wire.size());
    return true;
}

size_t DatagramBatch::read_from(int fd, size_t max)
{
    size_t got = 0;
    if (is_datagram_socket(fd)) {
        // recvmmsg into kMaxDatagram slots carved from the arena's free tail,
        // then compact the datagrams back to back (offsets stay contiguous)
        while (got < max) {
            const size_t free_bytes = cap_ - bytes();
            const size_t k = std::min({max - got, max_n_ - size(), free_bytes / kMaxDatagram, size_t(1024)});
            if (k == 0) break;
            std::vector<mmsghdr> msgs(k);
            std::vector<iovec> iov(k);
            uint8_t* base = arena_ + bytes();
            for (size_t j = 0; j < k; ++j) {
                iov[j] = {base + j * kMaxDatagram, kMaxDatagram};
                msgs[j].msg_hdr = {};
                msgs[j].msg_hdr.msg_iov = &iov[j];
                msgs[j].msg_hdr.msg_iovlen = 1;
            }
            // the first call waits for one datagram only (a plain blocking
            // recvmmsg would wait until all k arrived), later calls take what
            // is already queued
            const int r = recvmmsg(fd, msgs.data(), static_cast<unsigned>(k), got ? MSG_DONTWAIT : MSG_WAITFORONE,
                                   nullptr);
            if (r < 0) {
                if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
                sys_fail("recvmmsg");
            }
            // a zero-length message ends the stream: at end of stream a
            // SOCK_SEQPACKET recvmmsg reports every remaining slot as an
            // empty message (an IPv4 datagram is never empty)
            int j = 0;
            for (; j < r && msgs[j].msg_len > 0; ++j) {
                const size_t len = msgs[j].msg_len;
                if (j) std::memmove(arena_ + bytes(), base + size_t(j) * kMaxDatagram, len);
                off_.push_back(bytes() + len);
            }
            got += size_t(j);
            if (j < r) {
                ended_ = true;
                break;
            }
            if (size_t(r) < k) break;
        }
        return got;
    }
    // packet fds (TUN): one datagram per read(), written in place
    while (got < max && room(kMaxDatagram)) {
        const ssize_t r = ::read(fd, arena_ + bytes(), kMaxDatagram);
        if (r < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
            sys_fail("read");
        }
        if (r == 0) {
            ended_ = true;
            break;
        }
        off_.push_back(bytes() + size_t(r));
        ++got;
    }
    return got;
}

size_t DatagramBatch::write_to(int fd) const
{
    const size_t n = size();
    if (is_datagram_socket(fd)) {
        size_t done = 0;
        while (done < n) {
            const size_t k = std::min<size_t>(n - done, 1024);
            std::vector<mmsghdr> msgs(k);
            std::vector<iovec> iov(k);
            for (size_t j = 0; j < k; ++j) {
                const size_t i = done + j;
                iov[j] = {arena_ + off_[i], static_cast<size_t>(off_[i + 1] - off_[i])};
                msgs[j].msg_hdr = {};
                msgs[j].msg_hdr.msg_iov = &iov[j];
                msgs[j].msg_hdr.msg_iovlen = 1;
            }
            const int r = sendmmsg(fd, msgs.data(), static_cast<unsigned>(k), MSG_NOSIGNAL);  // EPIPE, not SIGPIPE
            if (r < 0) {
                if (errno == EINTR) continue;
                sys_fail("sendmmsg");
            }
            done += size_t(r);
        }
        return done;
    }
    for (size_t i = 0; i < n; ++i) {
        const size_t len = static_cast<size_t>(off_[i + 1] - off_[i]);
        if (::write(fd, arena_ + off_[i], len) != static_cast<ssize_t>(len)) sys_fail("write");
    }
    return n;
}

std::vector<uint8_t> DatagramBatch::verify()
{
    if (!engine_) throw std::logic_error("DatagramBatch::verify needs an engine");
    return engine_->verify_packed(arena_, off_.data(), size());
}

std::vector<std::optional<TCPMessage>> DatagramBatch::unwrap(TCPOverIPv4Adapter& adapter)
{
    if (!engine_) throw std::logic_error("DatagramBatch::unwrap needs an engine");
    return engine_->unwrap_packed(adapter, arena_, off_.data(), size());
}

bool DatagramBatch::push_tcp(const TCPOverIPv4Adapter& adapter, const TCPMessage& msg)
{
    const std::string& pl = msg.sender.payload;
    if (!room(40 + pl.size())) return false;
    const uint64_t at = off_.back();
    if (!pl.empty()) std::memcpy(arena_ + at + 40, pl.data(), pl.size());
    off_.push_back(at + 40 + pl.size());
    msgs_.push_back(wrap_fields(adapter.config(), msg));
    return true;
}

void DatagramBatch::wrap()
{
    if (!engine_) throw std::logic_error("DatagramBatch::wrap needs an engine");
    if (msgs_.size() != size()) throw std::logic_error("DatagramBatch::wrap: datagrams not added by push_tcp");
    engine_->wrap_packed(arena_, off_.data(), msgs_.data(), size());
    msgs_.clear();
}

void DatagramBatch::patch()
{
    if (!engine_) throw std::logic_error("DatagramBatch::patch needs an engine");
    engine_->patch_packed(arena_, off_.data(), size());
}

namespace {
std::unique_ptr<DatagramBatch> make_arena(BatchEngine* engine, size_t capacity_bytes, size_t max_datagrams)
{
    return engine ? std::make_unique<DatagramBatch>(*engine, capacity_bytes, max_datagrams)
                  : std::make_unique<DatagramBatch>(capacity_bytes, max_datagrams);
}
}  // namespace

DatagramRing::DatagramRing(BatchEngine& engine, int fd, size_t slots, size_t capacity_bytes, size_t max_datagrams)
    : fds_{fd}, max_n_(max_datagrams)
{
    start(&engine, slots, capacity_bytes);
}

DatagramRing::DatagramRing(BatchEngine& engine, const std::vector<int>& fds, size_t slots, size_t capacity_bytes,
                           size_t max_datagrams)
    : fds_(fds), max_n_(max_datagrams)
{
    if (fds.empty()) throw std::invalid_argument("DatagramRing needs at least one fd");
    start(&engine, slots ? slots : 2 * fds.size() + 1, capacity_bytes);
}

DatagramRing::DatagramRing(int fd, size_t slots, size_t capacity_bytes, size_t max_datagrams)
    : fds_{fd}, max_n_(max_datagrams)
{
    start(nullptr, slots, capacity_bytes);
}

DatagramRing::DatagramRing(const std::vector<int>& fds, size_t slots, size_t capacity_bytes, size_t max_datagrams)
    : fds_(fds), max_n_(max_datagrams)
{
    if (fds.empty()) throw std::invalid_argument("DatagramRing needs at least one fd");
    start(nullptr, slots ? slots : 2 * fds.size() + 1, capacity_bytes);
}

void DatagramRing::start(BatchEngine* engine, size_t slots, size_t capacity_bytes)
{
    // every reader holds one arena while it fills it; one more keeps a
    // filled arena moving to the caller
    if (slots < fds_.size() + 1) throw std::invalid_argument("DatagramRing needs more slots than fds");
    for (size_t k = 0; k < slots; ++k) {
        arenas_.push_back(make_arena(engine, capacity_bytes, max_n_));
        free_.push_back(arenas_.back().get());
    }
    live_ = fds_.size();
    try {
        for (int fd : fds_) threads_.emplace_back([this, fd] { reader(fd); });
    } catch (...) {  // a thread failed to start: stop and join the ones that did
        {
            std::lock_guard<std::mutex> lock(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : threads_) t.join();
        throw;
    }
}

DatagramRing::~DatagramRing()
{
    {
        std::lock_guard<std::mutex> lock(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();  // each reader polls its fd and checks stop_ every 50 ms
}

void DatagramRing::reader(int fd)
{
    for (;;) {
        DatagramBatch* b = nullptr;
        {
            std::unique_lock<std::mutex> lock(mu_);
            cv_.wait(lock, [this] { return stop_ || !free_.empty(); });
            if (stop_) break;
            b = free_.front();
            free_.pop_front();
        }
        b->clear();
        bool end = false;
        try {
            // append until the arena is full, the stream ends, or the caller
            // waits with a non-empty arena here; poll with a timeout, looking
            // at stop_ in between, so the destructor never waits on a blocked
            // read (1 ms while holding datagrams, so an idle caller gets them)
            for (;;) {
                {
                    std::lock_guard<std::mutex> lock(mu_);
                    if (stop_ || (b->size() && waiting_)) break;
                }
                pollfd p{fd, POLLIN, 0};
                const int r = ::poll(&p, 1, b->size() ? 1 : 50);
                if (r < 0 && errno != EINTR) sys_fail("poll");
                if (r <= 0) continue;
                b->read_from(fd, max_n_ - b->size());
                if (b->ended()) {
                    end = true;
                    break;
                }
                if (b->full()) break;
            }
        } catch (...) {
            std::lock_guard<std::mutex> lock(mu_);
            if (!error_) error_ = std::current_exception();
            stop_ = true;  // the other readers stop too
            end = true;
        }
        std::lock_guard<std::mutex> lock(mu_);
        if (b->size())
            ready_.push_back(b);
        else
            free_.push_back(b);
        cv_.notify_all();
        if (end || stop_) break;
    }
    std::lock_guard<std::mutex> lock(mu_);
    if (--live_ == 0) eof_ = true;  // the stream ends with the last fd
    cv_.notify_all();
}

DatagramBatch* DatagramRing::next()
{
    std::unique_lock<std::mutex> lock(mu_);
    waiting_ = true;
    cv_.wait(lock, [this] { return !ready_.empty() || eof_; });
    waiting_ = false;
    if (!ready_.empty()) {
        DatagramBatch* b = ready_.front();
        ready_.pop_front();
        return b;
    }
    if (error_) std::rethrow_exception(error_);
    return nullptr;
}

void DatagramRing::release(DatagramBatch* batch)
{
    {
        std::lock_guard<std::mutex> lock(mu_);
        free_.push_back(batch);
    }
    cv_.notify_all();
}

DatagramTxRing::DatagramTxRing(BatchEngine& engine, int fd, size_t slots, size_t capacity_bytes,
                               size_t max_datagrams)
    : fd_(fd)
{
    start(&engine, slots, capacity_bytes, max_datagrams);
}

DatagramTxRing::DatagramTxRing(int fd, size_t slots, size_t capacity_bytes, size_t max_datagrams) : fd_(fd)
{
    start(nullptr, slots, capacity_bytes, max_datagrams);
}

void DatagramTxRing::start(BatchEngine* engine, size_t slots, size_t capacity_bytes, size_t max_datagrams)
{
    if (slots < 2) throw std::invalid_argument("DatagramTxRing needs at least 2 slots");
    for (size_t k = 0; k < slots; ++k) {
        arenas_.push_back(make_arena(engine, capacity_bytes, max_datagrams));
        free_.push_back(arenas_.back().get());
    }
    thread_ = std::thread([this] { writer(); });
}

DatagramTxRing::~DatagramTxRing()
{
    {
        std::unique_lock<std::mutex> lock(mu_);
        cv_.wait(lock, [this] { return (queued_.empty() && !busy_) || error_; });
        stop_ = true;
    }
    cv_.notify_all();
    thread_.join();
}

DatagramBatch* DatagramTxRing::acquire()
{
    std::unique_lock<std::mutex> lock(mu_);
    cv_.wait(lock, [this] { return !free_.empty() || error_; });
    if (error_) std::rethrow_exception(error_);
    DatagramBatch* b = free_.front();
    free_.pop_front();
    b->clear();
    return b;
}

void DatagramTxRing::submit(DatagramBatch* batch, bool patch)
{
    try {
        if (batch->wrap_pending())
            batch->wrap();  // the engine stays on the caller's thread
        else if (patch && batch->size())
            batch->patch();
    } catch (...) {
        // the arena goes back to the free list, so a failed patch does not
        // leak it (acquire() would otherwise block once every slot was lost)
        {
            std::lock_guard<std::mutex> lock(mu_);
            free_.push_back(batch);
        }
        cv_.notify_all();
        throw;
    }
    {
        std::lock_guard<std::mutex> lock(mu_);
        queued_.push_back(batch);
    }
    cv_.notify_all();
}

void DatagramTxRing::flush()
{
    std::unique_lock<std::mutex> lock(mu_);
    cv_.wait(lock, [this] { return (queued_.empty() && !busy_) || error_; });
    if (error_) std::rethrow_exception(error_);
}

size_t DatagramTxRing::sent() const
{
    std::lock_guard<std::mutex> lock(mu_);
    return sent_;
}

void DatagramTxRing::writer()
{
    for (;;) {
        DatagramBatch* b = nullptr;
        {
            std::unique_lock<std::mutex> lock(mu_);
            cv_.wait(lock, [this] { return stop_ || !queued_.empty(); });
            if (queued_.empty()) break;  // stop_ with nothing left to send
            b = queued_.front();
            queued_.pop_front();
            busy_ = true;
        }
        size_t n = 0;
        std::exception_ptr err;
        try {
            n = b->write_to(fd_);
        } catch (...) {
            err = std::current_exception();
        }
        {
            std::lock_guard<std::mutex> lock(mu_);
            sent_ += n;
            busy_ = false;
            free_.push_back(b);
            if (err && !error_) error_ = err;
        }
        cv_.notify_all();
        if (err) break;
    }
}

}  // namespace icsum
