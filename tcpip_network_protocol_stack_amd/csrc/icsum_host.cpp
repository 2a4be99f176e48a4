// icsum_host.cpp — the host-memory (PCIe-inclusive) path behind the C-ABI's
// *_host entry points: batches in host memory are cut into chunks that fit
// the context's staging slots, and the slots take turns (one stream each) so
// the copies, the kernels and the host-side stores of consecutive chunks
// overlap.  The kernels are the device path's (icsum_dispatch.cpp's
// geometry choice); there is no CPU arithmetic beyond folding the pieces of a
// segment longer than a slot.
#include <algorithm>
#include <chrono>
#include <cstring>

#include "icsum_ctx.h"

namespace icsum::detail {
namespace {

// Is p page-locked host memory the DMA engines can read directly, and can a
// kernel address it at the same address (hipHostMalloc memory under the
// unified address space; a registered range mapped elsewhere is only DMA'd)?
struct Pinned {
  bool dma = false, kernel = false;
};
Pinned host_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory is not an error for us
    return {};
  }
  const bool host = a.type == hipMemoryTypeHost;
  return {host, host && a.devicePointer == p};
}

int ensure_staging(ics_ctx* ctx) {
  if (ctx->staged) return ICS_OK;
  for (int k = 0; k < ctx->nslots; ++k) {
    if (ctx->slot_prio)
      ICS_HIP(hipStreamCreateWithPriority(&ctx->st[k], hipStreamNonBlocking, ctx->slot_prio));
    else
      ICS_HIP(hipStreamCreateWithFlags(&ctx->st[k], hipStreamNonBlocking));
    ICS_HIP(hipEventCreateWithFlags(&ctx->ev[k], hipEventDisableTiming));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_in[k]), ctx->slot_bytes, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_in[k]), ctx->slot_bytes));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_off[k]), (ics_ctx::kSlotSegs + 1) * 8, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_off[k]), (ics_ctx::kSlotSegs + 1) * 8));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_init[k]), ics_ctx::kSlotSegs * 4, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_init[k]), ics_ctx::kSlotSegs * 4));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_out[k]), ics_ctx::kSlotSegs * 5, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_out[k]), ics_ctx::kSlotSegs * 5));
    // the zero-copy path hands these very addresses to kernels
    for (const void* h : {static_cast<const void*>(ctx->h_in[k]), static_cast<const void*>(ctx->h_off[k]),
                          static_cast<const void*>(ctx->h_init[k]), static_cast<const void*>(ctx->h_out[k])})
      if (!host_pinned(h).kernel) ctx->zero_copy_max = 0;
  }
  ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_flag), ics_ctx::kMaxSlots * 64, hipHostMallocCoherent));
  std::memset(ctx->h_flag, 0, ics_ctx::kMaxSlots * 64);
  if (!host_pinned(ctx->h_flag).kernel) ctx->zero_copy_max = 0;
  ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_ticket), ics_ctx::kMaxSlots * 64));
  // Zeroed and waited for before any slot launches: the slots' streams are
  // non-blocking (they would not wait for a null-stream memset), and a first
  // launch that read the tickets before the zeros landed (the allocation
  // reusing freed, non-zero memory) would never reach its last-block count —
  // the call failing with its completion word unwritten.
  ICS_HIP(hipMemsetAsync(ctx->d_ticket, 0, ics_ctx::kMaxSlots * 64, ctx->st[0]));
  if (ctx->poison_ticket)  // test hook: a ticket left non-zero (wait_flag recovers it)
    ICS_HIP(hipMemcpyAsync(ctx->d_ticket, &ctx->poison_ticket, 4, hipMemcpyHostToDevice, ctx->st[0]));
  ICS_HIP(hipStreamSynchronize(ctx->st[0]));
  ctx->staged = true;
  return ICS_OK;
}

int ensure_wrap_staging(ics_ctx* ctx) {
  if (ctx->wrap_staged) return ICS_OK;
  for (int k = 0; k < ctx->nslots; ++k) {
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_msg[k]), ics_ctx::kWrapSlotSegs * sizeof(ics_tcp_msg), 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_msg[k]), ics_ctx::kWrapSlotSegs * sizeof(ics_tcp_msg)));
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_hdr[k]), ics_ctx::kWrapSlotSegs * 40, 0));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_hdr[k]), ics_ctx::kWrapSlotSegs * 40));
    ICS_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->d_sums[k]), ics_ctx::kWrapSlotSegs * 4));
    if (!host_pinned(ctx->h_msg[k]).kernel || !host_pinned(ctx->h_hdr[k]).kernel) ctx->zero_copy_max = 0;
  }
  ctx->wrap_staged = true;
  return ICS_OK;
}

// One staged chunk of segments [i0, i1) covering bytes [b0, b1).  A segment
// longer than a staging slot goes through the slots as PIECES: chunks with
// piece = true, i1 = i0 + 1 and [b0, b1) a slot-sized part of that one
// segment (pos = the part's offset inside it).
struct Chunk {
  uint64_t i0, i1, b0, b1;
  bool piece = false, last = false;
  uint64_t pos = 0;
};

// Next chunk starting at segment i0 (whose first `pos` bytes were already
// staged as pieces) that fits the slot.  The offsets are the caller's host
// array: every one a chunk takes is checked monotone here (a decreasing
// pair would reach the kernels as a segment of ~2^64 bytes), in the loop
// that reads them anyway.
int not_monotone(uint64_t i) {
  return fail(ICS_ERR_INVALID, "offsets not monotone: offsets[%llu] > offsets[%llu]", (unsigned long long)i,
              (unsigned long long)(i + 1));
}

int next_chunk(const ics_ctx* ctx, const uint64_t* offsets, uint64_t stride, uint64_t seg_len, uint64_t n,
               uint64_t i0, uint64_t pos, bool allow_pieces, uint64_t cap_n, Chunk* c) {
  const uint64_t cap_b = ctx->slot_bytes;
  if (offsets && offsets[i0 + 1] < offsets[i0]) return not_monotone(i0);
  const uint64_t s0 = offsets ? offsets[i0] : i0 * stride;
  const uint64_t len0 = offsets ? offsets[i0 + 1] - s0 : seg_len;
  if (pos || len0 > cap_b) {  // segment i0 does not fit a slot: its next piece
    if (!allow_pieces)
      return fail(ICS_ERR_INVALID, "datagram %llu (%llu bytes) exceeds the %zu-byte staging slot",
                  (unsigned long long)i0, (unsigned long long)len0, ctx->slot_bytes);
    const uint64_t take = std::min<uint64_t>(cap_b, len0 - pos);
    *c = {i0, i0 + 1, s0 + pos, s0 + pos + take, true, pos + take == len0, pos};
    return ICS_OK;
  }
  if (!offsets) {
    const uint64_t per = std::max<uint64_t>(stride, seg_len);
    uint64_t k = per ? cap_b / per : cap_n;
    if (k == 0) k = 1;  // stride > slot but the segment itself fits
    k = std::min<uint64_t>({k, cap_n, n - i0});
    *c = {i0, i0 + k, i0 * stride, (i0 + k - 1) * stride + seg_len};
    return ICS_OK;
  }
  const uint64_t b0 = offsets[i0];
  uint64_t i1 = i0;
  while (i1 < n && i1 - i0 < cap_n && offsets[i1 + 1] - b0 <= cap_b) {
    if (offsets[i1 + 1] < offsets[i1]) return not_monotone(i1);
    ++i1;
  }
  *c = {i0, i1, b0, offsets[i1]};
  return ICS_OK;
}

// InternetChecksum::value() of a raw sum (util/tools/checksum.h:31-41)
uint16_t fold_value(uint32_t sum) {
  while (sum > 0xFFFFu) sum = (sum >> 16) + (sum & 0xFFFFu);
  return uint16_t(~sum & 0xFFFFu);
}

// A piece is summed on the device as sub-pieces of this many bytes (one lane
// group each, so a 32 MiB piece is 512 segments of work, not one long one);
// even, so every sub-piece starts with the piece's parity.
constexpr uint64_t kSubPiece = uint64_t(64) << 10;


// memcpy split over the context's copy workers: a single core copies pageable
// memory into the pinned slots at ~10-20 GB/s, below what PCIe Gen5 x16 moves
void par_memcpy(ics_ctx* ctx, void* dst, const void* src, size_t n) {
  constexpr size_t kMinPerThread = size_t(4) << 20;
  const size_t t = std::min<size_t>(ctx->copy_threads, std::max<size_t>(1, n / kMinPerThread));
  if (t <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  if (!ctx->copy_pool) ctx->copy_pool = std::make_unique<icsum::detail::WorkerPool>(ctx->copy_threads - 1);
  ctx->copy_pool->run(n, t, [=](size_t a, size_t b) {
    std::memcpy(static_cast<char*>(dst) + a, static_cast<const char*>(src) + a, b - a);
  });
}

// fn(j0, j1) over [0, m) datagrams on the copy workers (host-side stores into
// the caller's batch at retire), serially below 16 Ki datagrams per range
template <typename Fn>
void host_ranges(ics_ctx* ctx, uint64_t m, Fn&& fn) {
  constexpr uint64_t kMinPerThread = 16384;
  const size_t t = std::min<size_t>(ctx->copy_threads, std::max<uint64_t>(1, m / kMinPerThread));
  if (t <= 1) {
    fn(size_t(0), size_t(m));
    return;
  }
  if (!ctx->copy_pool) ctx->copy_pool = std::make_unique<icsum::detail::WorkerPool>(ctx->copy_threads - 1);
  ctx->copy_pool->run(m, t, fn);
}

// ICS_MODE_PATCH's stores (k_ipv4_tcp, mode 2) applied on the host from a
// COMPUTE pass's results: for every datagram of >= 20 bytes the IPv4
// checksum goes to bytes 10..11; when >= 18 bytes follow the header
// (4 * hlen clamped to [20, len]) the TCP checksum goes to bytes 16..17 of
// the TCP header.  Both big-endian.  `res` = the slot's results: m ip u16,
// m tcp u16, m status bytes.
void host_patch_fields(uint8_t* bytes, const uint64_t* offsets, uint64_t stride, uint64_t dlen, const Chunk& c,
                       const uint8_t* res, uint64_t j0, uint64_t j1) {
  const uint64_t m = c.i1 - c.i0;
  const uint16_t* ip = reinterpret_cast<const uint16_t*>(res);
  const uint16_t* tcp = ip + m;
  for (uint64_t j = j0; j < j1; ++j) {
    const uint64_t i = c.i0 + j;
    const uint64_t s = offsets ? offsets[i] : i * stride;
    const uint64_t len = offsets ? offsets[i + 1] - s : dlen;
    if (len < 20) continue;
    uint8_t* d = bytes + s;
    d[10] = uint8_t(ip[j] >> 8);
    d[11] = uint8_t(ip[j]);
    uint64_t off = 4u * (d[0] & 0x0fu);
    if (off < 20) off = 20;
    if (off > len) off = len;
    if (len - off >= 18) {
      d[off + 16] = uint8_t(tcp[j] >> 8);
      d[off + 17] = uint8_t(tcp[j]);
    }
  }
}

// Wait for a zero-copy chunk: spin on its completion word (written by the
// launch's last block, icsum_kernels.hip signal_done) for
// up to a millisecond — a zero-copy chunk is at most zero_copy_max bytes, tens
// of microseconds over PCIe — then block on the slot's stream, which also
// surfaces a kernel fault as a HIP error instead of a hang.  A launch that
// finished without writing the word found its block-count ticket non-zero at
// the start (no block drew the last ticket): the call fails, but the ticket
// is zeroed on the slot's stream first, so the next call on this slot counts
// from zero again instead of failing the same way for the context's life.
int wait_flag(ics_ctx* ctx, int k, uint64_t v) {
  const uint64_t* f = ctx->h_flag + 8 * k;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t i = 1;; ++i) {
    if (__atomic_load_n(f, __ATOMIC_ACQUIRE) >= v) return ICS_OK;
    if ((i & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(1)) break;
  }
  ICS_HIP(hipStreamSynchronize(ctx->st[k]));
  if (__atomic_load_n(f, __ATOMIC_ACQUIRE) >= v) return ICS_OK;
  ICS_HIP(hipMemsetAsync(ctx->d_ticket + 16 * k, 0, 64, ctx->st[k]));
  ICS_HIP(hipStreamSynchronize(ctx->st[k]));
  return fail(ICS_ERR_HIP, "host path: slot %d's completion word was not written (its ticket was reset)", k);
}

}  // namespace

void free_staging(ics_ctx* ctx) {
  (void)server_stop(ctx);
  if (ctx->st_srv) (void)hipStreamDestroy(ctx->st_srv);
  ctx->st_srv = nullptr;
  if (ctx->h_mb) (void)hipHostFree(ctx->h_mb);
  ctx->h_mb = nullptr;
  if (ctx->srv_words) (void)(ctx->srv_words_vram ? hipFree(ctx->srv_words) : hipHostFree(ctx->srv_words));
  ctx->srv_words = nullptr;
  ctx->srv_words_vram = false;
  for (int k = 0; k < ics_ctx::kMaxSlots; ++k) {
    if (ctx->d_srv_stage[k]) (void)hipFree(ctx->d_srv_stage[k]);
    ctx->d_srv_stage[k] = nullptr;
  }
  for (int k = 0; k < ics_ctx::kMaxSlots; ++k) {
    if (ctx->st[k]) (void)hipStreamSynchronize(ctx->st[k]);
    if (ctx->h_in[k]) (void)hipHostFree(ctx->h_in[k]);
    if (ctx->d_in[k]) (void)hipFree(ctx->d_in[k]);
    if (ctx->h_off[k]) (void)hipHostFree(ctx->h_off[k]);
    if (ctx->d_off[k]) (void)hipFree(ctx->d_off[k]);
    if (ctx->h_init[k]) (void)hipHostFree(ctx->h_init[k]);
    if (ctx->d_init[k]) (void)hipFree(ctx->d_init[k]);
    if (ctx->h_out[k]) (void)hipHostFree(ctx->h_out[k]);
    if (ctx->d_out[k]) (void)hipFree(ctx->d_out[k]);
    if (ctx->h_msg[k]) (void)hipHostFree(ctx->h_msg[k]);
    if (ctx->d_msg[k]) (void)hipFree(ctx->d_msg[k]);
    if (ctx->h_hdr[k]) (void)hipHostFree(ctx->h_hdr[k]);
    if (ctx->d_hdr[k]) (void)hipFree(ctx->d_hdr[k]);
    if (ctx->d_sums[k]) (void)hipFree(ctx->d_sums[k]);
    if (ctx->ev[k]) (void)hipEventDestroy(ctx->ev[k]);
    if (ctx->st[k]) (void)hipStreamDestroy(ctx->st[k]);
  }
  if (ctx->h_flag) (void)hipHostFree(ctx->h_flag);
  ctx->h_flag = nullptr;
  if (ctx->d_ticket) (void)hipFree(ctx->d_ticket);
  ctx->d_ticket = nullptr;
  ctx->staged = false;
  ctx->wrap_staged = false;
}

// ---- resident tick server (k_tick_server, icsum_launch.h TickMailbox) ----
namespace {

uint64_t mb_load(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
void mb_store(uint64_t* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
// stores into device memory through the BAR sit in the CPU's write-combining
// buffers until flushed: without this the server saw some jobs only after
// milliseconds, or not within 1 s (profiles/r6_probe_vram_mailbox*.jsonl)
void bar_flush(const ics_ctx* ctx) {
  if (ctx->srv_words_vram) __builtin_ia32_sfence();
}

// a posted tick: its parts' sequence numbers, part p in mailbox p (parts 0: none)
struct SrvTick {
  uint32_t seq[icsum::kSrvBlocksMax];
  uint32_t parts;
};

// every block of the grid launched last has left (block 0 leaves first, the
// others within a poll of seeing its `state`): only then may a new grid
// start, so no two blocks ever serve one mailbox
bool server_gone(const ics_ctx* ctx) {
  for (uint32_t b = 0; b < ctx->srv_grid; ++b)
    if (mb_load(&ctx->h_mb[b].state) != icsum::kSrvExited) return false;
  return true;
}

int server_launch(ics_ctx* ctx) {
  if (!ctx->h_mb) {
    const size_t sz = sizeof(icsum::TickMailbox) * icsum::kSrvBlocksMax;
    ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_mb), sz, hipHostMallocCoherent));
    std::memset(static_cast<void*>(ctx->h_mb), 0, sz);
    if (!host_pinned(ctx->h_mb).kernel) return fail(ICS_ERR_HIP, "tick server: mailbox not device-visible");
    const size_t wsz = sizeof(uint64_t) * icsum::kSrvWords * icsum::kSrvBlocksMax;
    if (ctx->srv_vram) {
      // every piece or none: a failed allocation falls back to page-locked words
      bool ok = hipExtMallocWithFlags(reinterpret_cast<void**>(&ctx->srv_words), wsz, hipDeviceMallocUncached) ==
                hipSuccess;
      for (int k = 0; ok && k < ics_ctx::kMaxSlots; ++k)
        ok = hipExtMallocWithFlags(reinterpret_cast<void**>(&ctx->d_srv_stage[k]), ics_ctx::kSrvStageBytes,
                                   hipDeviceMallocUncached) == hipSuccess;
      if (!ok) {
        (void)hipGetLastError();
        if (ctx->srv_words) (void)hipFree(ctx->srv_words);
        ctx->srv_words = nullptr;
        for (int k = 0; k < ics_ctx::kMaxSlots; ++k) {
          if (ctx->d_srv_stage[k]) (void)hipFree(ctx->d_srv_stage[k]);
          ctx->d_srv_stage[k] = nullptr;
        }
      } else {
        ctx->srv_words_vram = true;
        // zeroed by the host through the BAR like every later store (a
        // device memset could land after the first descriptor words)
        std::memset(ctx->srv_words, 0, wsz);
        bar_flush(ctx);
      }
    }
    if (!ctx->srv_words) {
      ICS_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->srv_words), wsz, hipHostMallocCoherent));
      std::memset(ctx->srv_words, 0, wsz);
    }
    ICS_HIP(hipStreamCreateWithFlags(&ctx->st_srv, hipStreamNonBlocking));
  }
  // each block reads its mailbox's `done` at start: the oldest job not done;
  // the exit word block 0 set when the last grid left goes back to 0
  mb_store(&ctx->srv_words[icsum::kSrvExit], 0);
  bar_flush(ctx);
  for (uint32_t b = 0; b < ctx->srv_blocks; ++b) mb_store(&ctx->h_mb[b].state, icsum::kSrvRunning);
  ICS_HIP(icsum::launch_tick_server(ctx->srv_words, ctx->h_mb, ctx->srv_blocks, ctx->d_zero, ctx->srv_idle_us,
                                    ctx->srv_pollers, ctx->st_srv));
  ctx->srv_grid = ctx->srv_blocks;
  ctx->srv_launched = true;
  ++ctx->n_srv_launches;
  return ICS_OK;
}

// (re)launch the grid when none runs; a grid part-way out is waited for
int server_ensure(ics_ctx* ctx) {
  if (ctx->srv_launched && mb_load(&ctx->h_mb[0].state) != icsum::kSrvExited) return ICS_OK;
  if (ctx->srv_launched) {
    const auto t0 = std::chrono::steady_clock::now();
    while (!server_gone(ctx))
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2))
        return fail(ICS_ERR_HIP, "tick server: blocks still resident 2 s after block 0 left");
  }
  return server_launch(ctx);
}

// The tick's descriptors, sub-job b (segments [16 b, 16 b + 16) of n) into
// mailbox b, each word stamped with that mailbox's sequence number (the
// server takes a job once every word it uses carries the number).  Mailbox 0
// goes last: when block 0 takes its part (restarting the idle clock that
// decides the grid's exit) the other parts are already posted.  A part the
// grid left without taking is taken by the relaunched grid (server_wait).
int server_post(ics_ctx* ctx, int op, int mode, const void* bytes, const uint32_t* init, void* res,
                const uint64_t* rel_off, uint64_t stride, uint64_t seg_len, uint32_t n, SrvTick* tick) {
  if (int rc = server_ensure(ctx)) return rc;
  const uint32_t parts = (n + icsum::kTickSegs - 1) / icsum::kTickSegs;
  // w[3..4]: the wrap's message records (device-visible); the checksum's
  // inits (the caller's host array) travel as words below, never as an address
  const uint64_t b = reinterpret_cast<uintptr_t>(bytes), ini = op == 2 ? reinterpret_cast<uintptr_t>(init) : 0,
                 r = reinterpret_cast<uintptr_t>(res);
  const bool inits = op == 0 && init;  // checksum inits: in the descriptor itself
  for (uint32_t p = parts; p-- > 0;) {
    const uint32_t k = ++ctx->srv_seq[p];
    const uint64_t stamp = uint64_t(k) << 32;
    uint64_t* w = ctx->srv_words + icsum::kSrvWords * p;
    auto put = [&](uint32_t i, uint64_t v32) {
      __atomic_store_n(&w[i], stamp | (v32 & 0xffffffffull), __ATOMIC_RELAXED);
    };
    const uint32_t j0 = p * icsum::kTickSegs, m = std::min(n - j0, icsum::kTickSegs);
    for (uint32_t j = 0; j < m; ++j) {
      const uint64_t s0 = rel_off ? rel_off[j0 + j] : (j0 + j) * stride;
      put(icsum::kSrvHead + 2 * j, s0);
      put(icsum::kSrvHead + 2 * j + 1, rel_off ? rel_off[j0 + j + 1] - s0 : seg_len);
    }
    if (inits)
      for (uint32_t j = 0; j < m; ++j) put(icsum::kSrvInit + j, init[j0 + j]);
    put(1, b);
    put(2, b >> 32);
    put(3, ini);
    put(4, ini >> 32);
    put(5, r);
    put(6, r >> 32);
    put(icsum::kSrvPart, j0 | (uint64_t(n) << 8));
    put(0, uint64_t(op) | (uint64_t(mode) << 4) | (uint64_t(m) << 8) | (uint64_t(inits) << 16));
    tick->seq[p] = k;
  }
  bar_flush(ctx);
  tick->parts = parts;
  ++ctx->n_srv_jobs;
  return ICS_OK;
}

// spin until the server reports every part of the tick done; a server that
// idled out (or hit its lifetime) before taking them is launched again, and
// it takes them
int server_wait(ics_ctx* ctx, const SrvTick& tick) {
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t p = 0;
  for (uint32_t i = 1;; ++i) {
    while (p < tick.parts && int32_t(uint32_t(mb_load(&ctx->h_mb[p].done)) - tick.seq[p]) >= 0) ++p;
    if (p == tick.parts) return ICS_OK;
    if ((i & 255) == 0) {
      if (mb_load(&ctx->h_mb[0].state) == icsum::kSrvExited && server_gone(ctx))
        if (int rc = server_launch(ctx)) return rc;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        (void)server_stop(ctx);
        ctx->srv_idle_us = 0;  // off: the calls after this one take the launches
        return fail(ICS_ERR_HIP, "tick server: job not done within 2 s (server turned off)");
      }
    }
  }
}

}  // namespace

int server_stop(ics_ctx* ctx) {
  if (!ctx->h_mb || !ctx->srv_launched) return ICS_OK;
  mb_store(&ctx->srv_words[icsum::kSrvQuit], 1);
  bar_flush(ctx);
  const hipError_t e = hipStreamSynchronize(ctx->st_srv);  // the server exits on the quit word
  mb_store(&ctx->srv_words[icsum::kSrvQuit], 0);
  bar_flush(ctx);
  ctx->srv_launched = false;
  if (e != hipSuccess) return fail(ICS_ERR_HIP, "tick server: %s", hipGetErrorString(e));
  return ICS_OK;
}

// kind 0: checksum batch (u16 out); kind 1: ipv4_tcp batch (ip u16, tcp u16, status u8);
// kind 2: tcp wrap (40 header bytes per datagram back, written into h_bytes).
// The slots take turns, one stream each: while the GPU moves and sums chunk
// k, the host prepares chunk k+1.  Pinned user buffers are DMA'd directly (no
// host copy); pageable ones are staged through the pinned slots by par_memcpy.
// A batch of at most ctx->zero_copy_max bytes in one chunk is not DMA'd at
// all: the kernel reads the pinned bytes, offsets, inits and messages over
// PCIe and writes its results into the pinned result area (one launch, one
// synchronisation).
namespace {

// ics_dispatch_info's "last call" fields for a host-memory call's launch
void note_host(ics_ctx* ctx, int kernel, int lps, int unroll) {
  ctx->last_kernel.store(kernel, std::memory_order_relaxed);
  ctx->last_lps.store(lps, std::memory_order_relaxed);
  ctx->last_unroll.store(unroll, std::memory_order_relaxed);
  ctx->last_plan.store(-1, std::memory_order_relaxed);
}

int run_pipeline(ics_ctx* ctx, int kind, void* h_bytes, const uint64_t* h_offsets, uint64_t stride,
                 uint64_t seg_len, const uint32_t* h_init, uint64_t n, int mode, uint16_t* out_a, uint16_t* out_b,
                 uint8_t* out_c, const ics_tcp_msg* h_msgs) {
  if (int rc = ensure_staging(ctx)) return rc;
  if (kind == 2)
    if (int rc = ensure_wrap_staging(ctx)) return rc;
  const Pinned pin = host_pinned(h_bytes);
  const bool direct = pin.dma;
  Chunk pending[ics_ctx::kMaxSlots];
  bool busy[ics_ctx::kMaxSlots] = {};
  uint64_t flag_of[ics_ctx::kMaxSlots] = {};  // zero-copy chunk: its completion word's value (0: event)
  SrvTick srv_of[ics_ctx::kMaxSlots] = {};    // a tick-server job: its parts' sequence numbers (parts 0: none)
  uint32_t piece_sum = 0;  // running sum of the long segment whose pieces are in flight
  auto retire = [&](int k) -> int {
    if (!busy[k]) return ICS_OK;
    if (srv_of[k].parts) {
      const SrvTick job = srv_of[k];
      srv_of[k].parts = 0;
      if (int rc = server_wait(ctx, job)) return rc;
    } else if (flag_of[k]) {
      if (int rc = wait_flag(ctx, k, flag_of[k])) return rc;
    } else {
      ICS_HIP(hipEventSynchronize(ctx->ev[k]));
    }
    const Chunk& c = pending[k];
    const uint64_t m = c.i1 - c.i0;
    if (c.piece) {
      // raw u32 sums of the piece's sub-pieces; uint32 addition is
      // associative, so sum_ of the whole segment = init + every part's sum
      // (each summed with its own start parity), wrap included
      const uint64_t parts = (c.b1 - c.b0 + kSubPiece - 1) / kSubPiece;
      const uint32_t* raw = reinterpret_cast<const uint32_t*>(ctx->h_out[k]);
      for (uint64_t j = 0; j < parts; ++j) piece_sum += raw[j];
      if (c.last) {
        out_a[c.i0] = fold_value((h_init ? h_init[c.i0] : 0u) + piece_sum);
        piece_sum = 0;
      }
    } else if (kind == 0) {
      std::memcpy(out_a + c.i0, ctx->h_out[k], m * 2);
    } else if (kind == 2 && mode == 1) {  // payload-only: headers to the caller's array
      std::memcpy(reinterpret_cast<uint8_t*>(out_c) + 40 * c.i0, ctx->h_hdr[k], m * 40);
    } else if (kind == 2) {  // 40 header bytes into each datagram of the caller's batch
      uint8_t* bytes = static_cast<uint8_t*>(h_bytes);
      host_ranges(ctx, m, [&](size_t j0, size_t j1) {
        for (uint64_t j = j0; j < j1; ++j) {
          const uint64_t i = c.i0 + j;
          const uint64_t s0 = h_offsets ? h_offsets[i] : i * stride;
          const uint64_t len = h_offsets ? h_offsets[i + 1] - s0 : seg_len;
          if (len >= 40) std::memcpy(bytes + s0, ctx->h_hdr[k] + 40 * j, 40);
        }
      });
    } else {
      if (out_a) std::memcpy(out_a + c.i0, ctx->h_out[k], m * 2);
      if (out_b) std::memcpy(out_b + c.i0, ctx->h_out[k] + m * 2, m * 2);
      if (out_c) std::memcpy(out_c + c.i0, ctx->h_out[k] + m * 4, m);
      if (mode == ICS_MODE_PATCH)  // scattered 2-byte stores into the caller's batch
        host_ranges(ctx, m, [&](size_t j0, size_t j1) {
          host_patch_fields(static_cast<uint8_t*>(h_bytes), h_offsets, stride, seg_len, c, ctx->h_out[k], j0, j1);
        });
    }
    busy[k] = false;
    return ICS_OK;
  };
  uint64_t i0 = 0, pos = 0;
  int slot = 0;
  while (i0 < n) {
    Chunk c;
    if (int rc = next_chunk(ctx, h_offsets, stride, seg_len, n, i0, pos, kind == 0,
                            kind == 2 ? ics_ctx::kWrapSlotSegs : ics_ctx::kSlotSegs, &c))
      return rc;
    if (int rc = retire(slot)) return rc;
    const uint64_t m = c.i1 - c.i0, nb = c.b1 - c.b0;
    const bool zc = !c.piece && c.i0 == 0 && c.i1 == n && nb <= ctx->zero_copy_max;
    (zc ? ctx->n_host_zc : ctx->n_host_dma).fetch_add(1, std::memory_order_relaxed);
    uint8_t* src = static_cast<uint8_t*>(h_bytes) + c.b0;
    if (zc ? !pin.kernel : !direct) {
      par_memcpy(ctx, ctx->h_in[slot], src, nb);
      src = ctx->h_in[slot];
    }
    hipStream_t st = ctx->st[slot];
    if (!zc) ICS_HIP(hipMemcpyAsync(ctx->d_in[slot], src, nb, hipMemcpyHostToDevice, st));
    // where the kernel finds the chunk's inputs and leaves its results
    uint8_t* const in = zc ? src : ctx->d_in[slot];
    uint8_t* const res = zc ? ctx->h_out[slot] : ctx->d_out[slot];
    auto h2d = [&](void* d, const void* h, size_t bytes, const void** where) -> hipError_t {
      *where = zc ? h : d;
      return zc ? hipSuccess : hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st);
    };
    auto d2h = [&](void* h, const void* d, size_t bytes) -> hipError_t {
      return zc ? hipSuccess : hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st);
    };
    if (c.piece) {
      // ics_sum_batch over the piece's sub-pieces: raw sums, parity = the
      // piece's offset in its segment (checksum.h:24-26 carried across add()s)
      const uint64_t parts = (nb + kSubPiece - 1) / kSubPiece;
      for (uint64_t j = 0; j <= parts; ++j) ctx->h_off[slot][j] = std::min<uint64_t>(j * kSubPiece, nb);
      uint8_t* odd = reinterpret_cast<uint8_t*>(ctx->h_init[slot]);
      std::memset(odd, int(c.pos & 1), parts);
      ICS_HIP(hipMemcpyAsync(ctx->d_off[slot], ctx->h_off[slot], (parts + 1) * 8, hipMemcpyHostToDevice, st));
      ICS_HIP(hipMemcpyAsync(ctx->d_init[slot], odd, parts, hipMemcpyHostToDevice, st));
      const icsum::SegSpec sp{ctx->d_in[slot], ctx->d_off[slot], 0, 0, parts, ctx->d_zero};
      ICS_HIP(icsum::launch_checksum(sp, nullptr, reinterpret_cast<const uint8_t*>(ctx->d_init[slot]),
                                     ctx->d_out[slot], 1, geometry_for(ctx, kSubPiece), 0, st));
      ICS_HIP(hipMemcpyAsync(ctx->h_out[slot], ctx->d_out[slot], parts * 4, hipMemcpyDeviceToHost, st));
      ICS_HIP(hipEventRecord(ctx->ev[slot], st));
      flag_of[slot] = 0;
      pending[slot] = c;
      busy[slot] = true;
      if (c.last) {
        i0 = c.i1;
        pos = 0;
      } else {
        pos = c.pos + nb;
      }
      slot = (slot + 1) % ctx->nslots;
      continue;
    }
    const uint64_t* d_off = nullptr;
    if (h_offsets) {
      for (uint64_t j = 0; j <= m; ++j) ctx->h_off[slot][j] = h_offsets[c.i0 + j] - c.b0;
      const void* w = nullptr;
      ICS_HIP(h2d(ctx->d_off[slot], ctx->h_off[slot], (m + 1) * 8, &w));
      d_off = static_cast<const uint64_t*>(w);
    }
    icsum::SegSpec sp{in, d_off, stride, seg_len, m, ctx->d_zero};
    // zero-copy: the launch itself stores the completion word (one launch per
    // call, DESIGN.md §6 "Per-tick host batches"); staged: an event
    flag_of[slot] = zc ? ++ctx->flag_ticket : 0;
    if (zc) sp.done = icsum::Done{ctx->d_ticket + 16 * slot, ctx->h_flag + 8 * slot, flag_of[slot]};
    const uint64_t avg = h_offsets ? nb / m : seg_len;
    const icsum::Geometry g = geometry_for(ctx, avg);
    // a zero-copy tick of a few segments with offsets: the offsets travel in
    // the kernel arguments (k_tick), not as a dependent PCIe read
    const bool tick = zc && h_offsets && kind != 2 && m <= icsum::kTickSegs && ctx->tick_inline;
    const bool srv =
        zc && m <= icsum::kTickSegs * ctx->srv_blocks && ctx->srv_idle_us && (h_offsets || nb < (1u << 31));
    if (srv) {  // the resident tick server takes it: no launch
      if (int rc = server_ensure(ctx)) return rc;
      const uint32_t* d_init = nullptr;  // checksum: the inits; wrap: the message records
      void* out = res;
      int dev_mode = mode == ICS_MODE_PATCH ? ICS_MODE_COMPUTE : mode;  // PATCH: fields written at retire
      const void* bytes_in = in;
      // srv_vram: the tick's bytes (and the wrap's records) written into
      // device memory through the BAR, so the server reads nothing over PCIe
      const uint64_t rec_at = (nb + 15) & ~uint64_t(15);
      const bool stage = ctx->srv_words_vram && rec_at + m * sizeof(ics_tcp_msg) <= ics_ctx::kSrvStageBytes;
      if (stage) {
        std::memcpy(ctx->d_srv_stage[slot], in, nb);
        bytes_in = ctx->d_srv_stage[slot];
      }
      if (kind == 0 && h_init) {
        d_init = h_init + c.i0;  // copied into the descriptor (server_post)
      } else if (kind == 2) {
        uint8_t* recs = stage ? ctx->d_srv_stage[slot] + rec_at : ctx->h_msg[slot];
        std::memcpy(recs, h_msgs + c.i0, m * sizeof(ics_tcp_msg));
        d_init = reinterpret_cast<const uint32_t*>(recs);
        out = ctx->h_hdr[slot];
        dev_mode = mode;  // 1: payload only (headers apart)
      }
      if (stage) bar_flush(ctx);  // the staged bytes land before any descriptor word
      if (int rc = server_post(ctx, kind, dev_mode, bytes_in, d_init, out, h_offsets ? ctx->h_off[slot] : nullptr,
                               stride, seg_len, uint32_t(m), &srv_of[slot]))
        return rc;
      note_host(ctx, ICS_K_TICK_SERVER, 16, 8);
    } else if (tick) {
      const uint32_t* d_init = nullptr;
      if (kind == 0 && h_init) {
        std::memcpy(ctx->h_init[slot], h_init + c.i0, m * 4);
        d_init = reinterpret_cast<const uint32_t*>(ctx->h_init[slot]);
      }
      uint16_t* a = reinterpret_cast<uint16_t*>(res);
      const int dev_mode = mode == ICS_MODE_PATCH ? ICS_MODE_COMPUTE : mode;  // PATCH: fields written at retire
      ICS_HIP(icsum::launch_tick(in, ctx->h_off[slot], uint32_t(m), kind == 0 ? 0 : 1, d_init, a, dev_mode, a, a + m,
                                 res + m * 4, ctx->d_zero, sp.done, st));
      note_host(ctx, ICS_K_TICK, 16, 8);
    } else if (kind == 2) {
      std::memcpy(ctx->h_msg[slot], h_msgs + c.i0, m * sizeof(ics_tcp_msg));
      const void* msgs = nullptr;
      ICS_HIP(h2d(ctx->d_msg[slot], ctx->h_msg[slot], m * sizeof(ics_tcp_msg), &msgs));
      uint8_t* hdr = zc ? ctx->h_hdr[slot] : ctx->d_hdr[slot];
      ICS_HIP(icsum::launch_tcp_wrap(sp, static_cast<const icsum::TcpMsg*>(msgs), reinterpret_cast<uint32_t*>(hdr),
                                     nullptr, nullptr, mode == 1,
                                     wrap_two_pass(ctx, true, m) ? ctx->d_sums[slot] : nullptr, ipv4_geometry(g),
                                     0, st));
      ICS_HIP(d2h(ctx->h_hdr[slot], ctx->d_hdr[slot], m * 40));
      note_host(ctx, wrap_two_pass(ctx, true, m) ? ICS_K_WRAP_2PASS : ICS_K_WRAP, ipv4_geometry(g).lps,
                ipv4_geometry(g).unroll);
    } else if (kind == 0) {
      const uint32_t* d_init = nullptr;
      if (h_init) {
        std::memcpy(ctx->h_init[slot], h_init + c.i0, m * 4);
        const void* w = nullptr;
        ICS_HIP(h2d(ctx->d_init[slot], ctx->h_init[slot], m * 4, &w));
        d_init = static_cast<const uint32_t*>(w);
      }
      ICS_HIP(icsum::launch_checksum(sp, d_init, nullptr, res, 0, g, 0, st));
      ICS_HIP(d2h(ctx->h_out[slot], ctx->d_out[slot], m * 2));
      note_host(ctx, g.mode == icsum::kModeTiny ? ICS_K_TINY : g.segs > 1 ? ICS_K_SMALL : ICS_K_CHECKSUM, g.lps,
                g.unroll);
    } else {
      uint16_t* a = reinterpret_cast<uint16_t*>(res);
      uint16_t* b = a + m;
      uint8_t* s = res + m * 4;
      // PATCH from host memory: the device computes (COMPUTE gives the very
      // values PATCH stores) and only the 5-byte results come back; the two
      // fields are written into the caller's bytes on the host at retire,
      // instead of copying every patched byte back over PCIe
      const int dev_mode = mode == ICS_MODE_PATCH ? ICS_MODE_COMPUTE : mode;
      const icsum::Geometry gi = h_offsets ? ipv4_geometry(g) : ipv4_fixed_geometry(ctx, ipv4_geometry(g), seg_len);
      ICS_HIP(icsum::launch_ipv4_tcp(sp, dev_mode, a, b, s, gi, 0, st));
      ICS_HIP(d2h(ctx->h_out[slot], ctx->d_out[slot], m * 5));
      note_host(ctx, ICS_K_IPV4, gi.lps, gi.unroll);
    }
    if (!zc) ICS_HIP(hipEventRecord(ctx->ev[slot], st));
    pending[slot] = c;
    busy[slot] = true;
    i0 = c.i1;
    slot = (slot + 1) % ctx->nslots;
  }
  for (int k = 0; k < ctx->nslots; ++k)  // oldest first
    if (int rc = retire((slot + k) % ctx->nslots)) return rc;
  return bounds_verdict(ctx->st[0], ICS_OK);
}

}  // namespace

int host_pipeline(ics_ctx* ctx, int kind, void* h_bytes, const uint64_t* h_offsets,
                  uint64_t stride, uint64_t seg_len, const uint32_t* h_init, uint64_t n, int mode,
                  uint16_t* out_a, uint16_t* out_b, uint8_t* out_c, const ics_tcp_msg* h_msgs) {
  std::lock_guard<std::mutex> lock(ctx->mu);
  const int rc = run_pipeline(ctx, kind, h_bytes, h_offsets, stride, seg_len, h_init, n, mode, out_a, out_b, out_c,
                              h_msgs);
  // an error after chunks were enqueued (a later datagram larger than a slot,
  // a failed launch or copy) leaves copies — or zero-copy kernels reading the
  // caller's page-locked bytes — in flight: drain every slot before the
  // caller sees the error and frees or reuses its buffers
  if (rc != ICS_OK && ctx->staged)
    for (int k = 0; k < ctx->nslots; ++k)
      if (ctx->st[k]) (void)hipStreamSynchronize(ctx->st[k]);
  return rc;
}

}  // namespace icsum::detail
