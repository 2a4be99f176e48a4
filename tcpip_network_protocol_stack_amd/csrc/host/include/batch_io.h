// batch_io.h — batched datagram I/O for the engine.
//
// The reference reads one datagram per syscall into {20 B, 16 KiB} buffers
// (util/tuntap/tuntap_adapter.cpp:5-21 -> FileDescriptor::read,
// util/file_descriptor/file_descriptor.cpp:127-178, kReadBufferSize 16384 at
// file_descriptor.h:47) and checksums each one on the CPU.  A DatagramBatch
// is one arena of back-to-back wire datagrams + n+1 offsets, filled straight
// from a file descriptor (recvmmsg on datagram sockets, read() per datagram on
// TUN or other packet fds) and written back with sendmmsg / write(); with an
// engine it lives in page-locked memory, so verify / unwrap / patch DMA the
// arena with no staging copy.
#ifndef ICSUM_HOST_BATCH_IO_H
#define ICSUM_HOST_BATCH_IO_H

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <exception>
#include <memory>
#include <mutex>
#include <optional>
#include <string_view>
#include <thread>
#include <vector>

#include "batch.h"

namespace icsum {

class DatagramBatch
{
  public:
    static constexpr size_t kMaxDatagram = 16384 + 20;  // the reference's readv shape

    // page-locked arena from `engine` (GPU path)
    DatagramBatch(BatchEngine& engine, size_t capacity_bytes = size_t(64) << 20, size_t max_datagrams = 1 << 16);
    // ordinary memory (I/O only, no engine)
    explicit DatagramBatch(size_t capacity_bytes = size_t(64) << 20, size_t max_datagrams = 1 << 16);
    ~DatagramBatch();
    DatagramBatch(const DatagramBatch&) = delete;
    DatagramBatch& operator=(const DatagramBatch&) = delete;

    void clear()
    {
        off_.assign(1, 0);
        msgs_.clear();
        ended_ = false;
    }
    size_t size() const { return off_.size() - 1; }
    // no room for another datagram of the reference's maximum read size
    bool full() const { return !room(kMaxDatagram); }
    // the last read_from saw the end of the stream (0-byte read or message)
    bool ended() const { return ended_; }
    size_t bytes() const { return off_.back(); }
    std::string_view operator[](size_t i) const
    {
        return {reinterpret_cast<const char*>(arena_) + off_[i], static_cast<size_t>(off_[i + 1] - off_[i])};
    }
    const uint8_t* data() const { return arena_; }
    uint8_t* data() { return arena_; }
    const uint64_t* offsets() const { return off_.data(); }

    bool push(std::string_view wire);  // false when the arena is full
    // the transmit side without host serialization: 40 bytes of header room +
    // msg's payload (its only copy) appended; wrap() then has the engine write
    // both headers and checksums of every such datagram (wrap_tcp_in_ip,
    // tcp_over_ip.cpp:69-88, from `adapter`'s configuration).  False when full.
    bool push_tcp(const TCPOverIPv4Adapter& adapter, const TCPMessage& msg);
    // datagrams added by push_tcp are waiting for wrap() (which requires that
    // every datagram of the batch came from push_tcp)
    bool wrap_pending() const { return !msgs_.empty(); }

    // up to `max` datagrams from `fd` (non-blocking fds stop at EAGAIN;
    // blocking ones wait for the first datagram, then take what is queued);
    // returns the count read (0 at end of stream; on a socket an empty
    // message, which is what SOCK_SEQPACKET reads at end of stream, ends it)
    size_t read_from(int fd, size_t max);
    // every datagram to `fd`; returns the count written
    size_t write_to(int fd) const;

    // engine calls on the arena (require the engine constructor)
    std::vector<uint8_t> verify();
    std::vector<std::optional<TCPMessage>> unwrap(TCPOverIPv4Adapter& adapter);
    void patch();
    void wrap();

  private:
    BatchEngine* engine_ = nullptr;
    uint8_t* arena_ = nullptr;
    size_t cap_ = 0, max_n_ = 0;
    std::vector<uint64_t> off_{0};
    std::vector<ics_tcp_msg> msgs_{};  // one per push_tcp datagram
    bool ended_ = false;
    bool room(size_t n) const { return size() < max_n_ && bytes() + n <= cap_; }
};

// A ring of page-locked DatagramBatch arenas with a reader thread: while the
// caller runs batch k through the engine (verify / unwrap / patch), the reader
// fills arena k+1 from the fd, so socket reads overlap the PCIe + GPU pass.
// The reader keeps appending to its arena while the caller is busy and hands
// it over when it is full or as soon as the caller waits in next(): batches
// grow with the caller's pass time instead of one socket drain each, so the
// ring does not run out of free arenas (and a UDP socket does not overflow)
// behind a stream of small batches.
// The fd is the caller's and must be blocking (a socket, TUN or other packet
// fd); the reader polls it, reads once it is readable, and stops at end of
// stream (read_from returns 0: the peer closed).  The destructor stops and
// joins the reader within one 50 ms poll interval, and leaves the fd as it
// was.  Only the reader thread touches the fd; only the caller's thread
// touches the engine.  With several fds there is one reader thread per fd.
class DatagramRing
{
  public:
    DatagramRing(BatchEngine& engine, int fd, size_t slots = 3, size_t capacity_bytes = size_t(32) << 20,
                 size_t max_datagrams = 1 << 14);
    // several fds (e.g. SO_REUSEPORT sockets), one reader thread each, sharing
    // the arenas: next() returns filled arenas from any of them, so one caller
    // and one engine serve every socket; slots = 0 means 2 * fds + 1.  The
    // stream ends when every fd has ended.
    DatagramRing(BatchEngine& engine, const std::vector<int>& fds, size_t slots = 0,
                 size_t capacity_bytes = size_t(32) << 20, size_t max_datagrams = 1 << 14);
    // the same ring over ordinary-memory arenas, without an engine (I/O only:
    // the batches' verify / unwrap / patch throw); the host-only stress tests
    // and sanitizer builds run the ring's threading this way
    explicit DatagramRing(int fd, size_t slots = 3, size_t capacity_bytes = size_t(32) << 20,
                          size_t max_datagrams = 1 << 14);
    explicit DatagramRing(const std::vector<int>& fds, size_t slots = 0, size_t capacity_bytes = size_t(32) << 20,
                          size_t max_datagrams = 1 << 14);
    ~DatagramRing();
    DatagramRing(const DatagramRing&) = delete;
    DatagramRing& operator=(const DatagramRing&) = delete;

    // the next filled batch (blocks until one is ready), or nullptr once the
    // stream ended and every filled batch was taken; rethrows a reader error
    DatagramBatch* next();
    // hand a batch taken with next() back for refilling
    void release(DatagramBatch* batch);

  private:
    void start(BatchEngine* engine, size_t slots, size_t capacity_bytes);
    void reader(int fd);

    std::vector<int> fds_{};
    size_t max_n_, live_ = 0;
    std::vector<std::unique_ptr<DatagramBatch>> arenas_{};
    std::deque<DatagramBatch*> free_{}, ready_{};
    std::mutex mu_{};
    std::condition_variable cv_{};
    bool eof_ = false, stop_ = false, waiting_ = false;
    std::exception_ptr error_{};
    std::vector<std::thread> threads_{};
};

// The transmit side (the reference wraps each segment with wrap_tcp_in_ip,
// util/tcp_over_ip/tcp_over_ip.cpp:69-88, and writes it to the TUN fd, one
// write per datagram: util/tuntap/tuntap_adapter.h:39): the caller fills a
// page-locked arena with serialized datagrams, submit() patches both checksum
// fields of every datagram on the GPU (ICS_MODE_PATCH) on the caller's
// thread and queues the arena; a writer thread sends queued arenas with
// sendmmsg / write() while the caller fills and patches the next one.
class DatagramTxRing
{
  public:
    DatagramTxRing(BatchEngine& engine, int fd, size_t slots = 3, size_t capacity_bytes = size_t(32) << 20,
                   size_t max_datagrams = 1 << 14);
    // ordinary-memory arenas, no engine: submit(batch, false) only
    explicit DatagramTxRing(int fd, size_t slots = 3, size_t capacity_bytes = size_t(32) << 20,
                            size_t max_datagrams = 1 << 14);
    ~DatagramTxRing();  // flushes what was submitted, then stops the writer
    DatagramTxRing(const DatagramTxRing&) = delete;
    DatagramTxRing& operator=(const DatagramTxRing&) = delete;

    // an empty arena to fill (blocks while every arena is queued or being
    // sent); rethrows a writer error
    DatagramBatch* acquire();
    // queue an arena taken with acquire(): an arena filled with push_tcp is
    // wrapped on the GPU (headers + both checksums), one filled with push()
    // is patched (both checksum fields) when `patch`; if that throws, the
    // arena returns to the free list and the error propagates
    void submit(DatagramBatch* batch, bool patch = true);
    // wait until every submitted datagram was written; rethrows a writer error
    void flush();
    size_t sent() const;  // datagrams written so far

  private:
    void start(BatchEngine* engine, size_t slots, size_t capacity_bytes, size_t max_datagrams);
    void writer();

    int fd_;
    std::vector<std::unique_ptr<DatagramBatch>> arenas_{};
    std::deque<DatagramBatch*> free_{}, queued_{};
    mutable std::mutex mu_{};
    std::condition_variable cv_{};
    bool stop_ = false, busy_ = false;
    size_t sent_ = 0;
    std::exception_ptr error_{};
    std::thread thread_{};
};

}  // namespace icsum

#endif
