/*
 * icsum.h — C-ABI of the MI355X Internet-checksum engine (libicsum.so).
 *
 * This is the drop-in boundary for the one per-byte transform the reference
 * stack (qmmzzdx/tcpip_network_protocol_stack) implements itself: the RFC-1071
 * one's-complement 16-bit sum over IPv4 headers and TCP segments.  Every entry
 * point below replaces a batch of calls to a reference C++ routine; the
 * reference has no C ABI of its own (its "interface" is the C++ header surface,
 * SURVEY.md §8b), so each declaration cites the reference function whose
 * semantics it reproduces bit for bit.
 *
 * Conventions
 *   - All functions return ICS_OK (0) or a negative ICS_ERR_* code.  No C++
 *     exception ever crosses this boundary; the message of the last failure on
 *     the calling thread is available from ics_last_error().
 *   - d_* pointers are device (HBM) pointers on the context's GPU; h_* pointers
 *     are host pointers.  `stream` is a hipStream_t (NULL = the legacy default
 *     stream of the context's device).  Device-pointer calls are asynchronous
 *     with respect to the host: they enqueue on `stream` and return.
 *   - Segment addressing (used by every batch call):
 *       d_offsets != NULL : segment i = bytes[d_offsets[i], d_offsets[i+1])
 *                           (n+1 monotone uint64 offsets; starts may be odd /
 *                           unaligned — byte roles are relative to each start;
 *                           the *_host calls reject decreasing h_offsets with
 *                           ICS_ERR_INVALID, the device calls trust them and
 *                           libicsum_debug.so reports them)
 *       d_offsets == NULL : segment i = bytes[i*stride, i*stride + seg_len)
 *   - Byte bases (d_bytes, d_dgrams, d_payloads, h_bytes, ...) may lie at ANY
 *     address, as InternetChecksum::add takes any string_view
 *     (util/tools/checksum.h:20-28): e.g. the IPv4 datagrams of a frame arena
 *     14 bytes in.  Loads stay inside the 16-byte-aligned blocks that hold a
 *     segment's bytes (never outside the pages of the batch).  Only the
 *     record arrays d_msgs / d_hdrs must be 4-byte aligned (ICS_ERR_INVALID
 *     otherwise); fixed stride == length == 64 B runs the dense kernel only
 *     from a 16-byte-aligned base (same results either way).
 *   - A context is bound to one device and may be used from several host
 *     threads (launch calls are thread-safe; the host-memory *_host calls
 *     serialise on an internal staging lock).
 */
#ifndef ICSUM_H
#define ICSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ICS_ABI_VERSION 2 /* 2: ics_dispatch_info_t gained the host-pipeline counters */

/* ---- status codes ------------------------------------------------------ */
#define ICS_OK 0
#define ICS_ERR_INVALID (-1)     /* bad argument (null pointer, bad mode, ...) */
#define ICS_ERR_HIP (-2)         /* HIP runtime error (message has details) */
#define ICS_ERR_NOMEM (-3)       /* device / pinned allocation failed */
#define ICS_ERR_NODEVICE (-4)    /* no GPU / device index out of range */

/* ---- per-datagram status bits written by ics_ipv4_tcp_batch ------------ */
/* IPv4Header::parse success: ver==4, hlen>=5, recomputed == given
 * (util/ipv4_header/ipv4_header.cpp:9-59).  In COMPUTE/PATCH mode: ver==4 &&
 * hlen>=5 only (nothing to compare). */
#define ICS_ST_IPV4_OK 0x01u
/* TCP checksum: VERIFY = InternetChecksum{pseudo}.add(all bytes after the IPv4
 * header).value()==0 (util/tcp_segment/tcp_segment.cpp:11-18);
 * COMPUTE/PATCH = the TCP checksum field lies inside the datagram (patchable). */
#define ICS_ST_TCP_CKSUM_OK 0x02u
/* TCP header parse: >=20 bytes after the IPv4 header and data offset >= 5
 * (tcp_segment.cpp:25-65). */
#define ICS_ST_TCP_HDR_OK 0x04u
/* proto == IPv4Header::PROTO_TCP (util/tcp_over_ip/tcp_over_ip.cpp:26-29). */
#define ICS_ST_PROTO_TCP 0x08u
/* all of the above: the datagram would pass unwrap_tcp_in_ip's parse steps. */
#define ICS_ST_ACCEPT 0x0Fu

/* ---- modes of ics_ipv4_tcp_batch ---------------------------------------- */
#define ICS_MODE_COMPUTE 0 /* IPv4Header::compute_checksum + TCPSegment::compute_checksum */
#define ICS_MODE_VERIFY 1  /* IPv4Header::parse + TCPSegment::parse checksum checks */
#define ICS_MODE_PATCH 2   /* COMPUTE, then write both checksum fields in place */

typedef struct ics_ctx ics_ctx;

/* ---- lifecycle ---------------------------------------------------------- */
const char* ics_version(void);
int ics_abi_version(void);
int ics_device_count(int* count);
/* One context per GPU.  Allocates the context's staging resources lazily. */
int ics_create(int device, ics_ctx** out);
int ics_destroy(ics_ctx* ctx);
int ics_device_of(const ics_ctx* ctx, int* device);
/* Message of the last failing call made by this thread ("" if none). */
const char* ics_last_error(void);

/* ---- a1-a4: InternetChecksum over a batch of segments ------------------ */
/* d_out[i] = InternetChecksum{init_i}.add(segment_i).value()
 *   replaces util/tools/checksum.h:17 (ctor), :20-28 (add), :31-41 (value);
 *   the TCP use is util/tcp_segment/tcp_segment.cpp:109-118 with init_i =
 *   IPv4Header::pseudo_checksum() (ipv4_header.cpp:103-110).
 * d_init == NULL means init_i = 0.  Bit-exact for every length, including the
 * reference's uint32 wrap above 131074 bytes of 0xFF. */
int ics_checksum_batch(ics_ctx* ctx, const void* d_bytes, const uint64_t* d_offsets,
                       uint64_t stride, uint64_t seg_len, const uint32_t* d_init,
                       uint16_t* d_out, uint64_t n, void* stream);

/* Unfolded running sum, for multi-piece add() chains (checksum.h:44-59, parity
 * carried across pieces): d_sum[i] = sum_ after InternetChecksum{init_i} has
 * had add(segment_i) applied with parity_ = d_odd[i] (0/1; NULL = all 0).
 * Chain pieces by feeding d_sum back as d_init and (len & 1) ^ odd as d_odd;
 * fold with ics_fold_batch or on the host. */
int ics_sum_batch(ics_ctx* ctx, const void* d_bytes, const uint64_t* d_offsets,
                  uint64_t stride, uint64_t seg_len, const uint32_t* d_init,
                  const uint8_t* d_odd, uint32_t* d_sum, uint64_t n, void* stream);

/* Dispatch of offsets batches (d_offsets != NULL) in ics_checksum_batch /
 * ics_sum_batch.  BINNED measures the length mix on the device and a one-block
 * plan kernel picks, per batch: split into length bins (each run with the lane
 * geometry that suits it), or the whole batch in one launch with 64/32-lane
 * groups (long segments dominate), 16-lane groups (short and MTU-sized) or
 * the small-segment body (ACK-sized);
 * SINGLE runs one launch with the long-segment geometry.  AUTO (default) =
 * BINNED for batches of >= 65536 segments.  Results are identical; only the
 * speed differs.  Per context; not a reference interface. */
#define ICS_BINNING_AUTO (-1)
#define ICS_BINNING_SINGLE 0
#define ICS_BINNING_BINNED 1
int ics_set_binning(ics_ctx* ctx, int mode);

/* d_out[i] = InternetChecksum::value() of a raw sum (checksum.h:31-41). */
int ics_fold_batch(ics_ctx* ctx, const uint32_t* d_sum, uint16_t* d_out, uint64_t n,
                   void* stream);

/* ---- a7/a8/a10/a11/a13: fused IPv4 + TCP over raw datagrams ------------- */
/* Each segment is one raw IPv4 datagram (wire bytes, header first).  Per
 * datagram, in one pass over its bytes:
 *   ip_ck  = IPv4Header::compute_checksum() of the parsed fields
 *            (ipv4_header.cpp:113-123: 20 serialized bytes, cksum=0, flag bit
 *            0x8000 dropped, options never summed)
 *   pseudo = IPv4Header::pseudo_checksum() (ipv4_header.cpp:103-110)
 *   tcp_ck = COMPUTE/PATCH: TCPSegment::compute_checksum(pseudo) over the bytes
 *            after the IPv4 header with the TCP checksum field read as 0
 *            (tcp_segment.cpp:109-118)
 *            VERIFY: InternetChecksum{pseudo}.add(all bytes after the IPv4
 *            header).value() (tcp_segment.cpp:11-18; 0 means valid)
 *   status = ICS_ST_* bits above.
 * PATCH additionally stores ip_ck / tcp_ck big-endian into the datagram
 * (the checksum fields wrap_tcp_in_ip fills, tcp_over_ip.cpp:69-88).
 * Datagrams shorter than 20 bytes get ip_ck = tcp_ck = status = 0.
 * Any of d_ip_ck / d_tcp_ck / d_status may be NULL. */
int ics_ipv4_tcp_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets,
                       uint64_t stride, uint64_t dgram_len, uint64_t n, int mode,
                       uint16_t* d_ip_ck, uint16_t* d_tcp_ck, uint8_t* d_status,
                       void* stream);

/* ---- router forwarding batch (src/router/router.cpp:43-50) -------------- */
/* For each raw datagram whose IPv4 header parses (ver 4, hlen>=5, checksum
 * valid): if ttl <= 1 the datagram is dropped (d_status[i] = 0, bytes
 * untouched); else ttl-- and the header checksum is recomputed with
 * IPv4Header::compute_checksum() semantics and written in place
 * (d_status[i] = 1).  Unparseable datagrams get d_status[i] = 0. */
int ics_router_ttl_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets,
                         uint64_t stride, uint64_t dgram_len, uint64_t n,
                         uint8_t* d_status, void* stream);

/* The same router step with the forwarded headers apart: the datagrams are
 * only read, and the 20 bytes Router::route's send_datagram serializes as the
 * header piece (router.cpp:39-66 -> ipv4_header.cpp:62-86: ttl - 1, the
 * recomputed checksum, the reserved flag bit dropped, no options) go to
 * d_hdrs + 20 * i, 4-byte aligned, one coalesced array.  Datagram i on the
 * wire = d_hdrs[20 i .. 20 i + 20) followed by its payload piece, the bytes
 * after the parsed header: [start + 4 hlen, end) (ipv4_header.cpp:50).
 * d_status[i] as ics_router_ttl_batch; a dropped or unparseable datagram's 20
 * header bytes are zero.  A forwarded header equals the first 20 bytes the
 * in-place call leaves. */
int ics_router_ttl_headers(ics_ctx* ctx, const void* d_dgrams, const uint64_t* d_offsets,
                           uint64_t stride, uint64_t dgram_len, uint64_t n, void* d_hdrs,
                           uint8_t* d_status, void* stream);

/* ---- a14 / §8(f) rank 2: device-side wrap_tcp_in_ip -------------------- */
/* The fields of one TCPMessage as TCPOverIPv4Adapter::wrap_tcp_in_ip
 * (util/tcp_over_ip/tcp_over_ip.cpp:69-88) puts them on the wire.  28 bytes. */
typedef struct ics_tcp_msg {
  uint32_t src, dst;   /* IPv4Header::src / dst, host order (FdAdapterConfig source / destination) */
  uint32_t seqno;      /* TCPSenderMessage::seqno, raw Wrap32 value */
  uint32_t ackno;      /* raw ackno; 0 when the message has none (tcp_segment.cpp:86) */
  uint16_t src_port, dst_port;
  uint16_t window;     /* TCPReceiverMessage::window_size */
  uint8_t flags;       /* ICS_TCP_* bits, as tcp_segment.cpp:92-97 derives them */
  uint8_t ttl;         /* IPv4Header::ttl (DEFAULT_TTL = 128 in wrap_tcp_in_ip) */
  uint16_t id;         /* IPv4Header::id (0 in wrap_tcp_in_ip) */
  uint16_t reserved;   /* 0 */
} ics_tcp_msg;
#define ICS_TCP_FIN 0x01u
#define ICS_TCP_SYN 0x02u
#define ICS_TCP_RST 0x04u /* sender.RST || receiver.RST */
#define ICS_TCP_ACK 0x10u /* receiver.ackno present */

/* Datagram i = bytes [off_i, off_i+1) (or fixed stride / dgram_len) holds 40
 * bytes of room for the headers followed by message i's payload, already in
 * place.  In one pass per datagram the engine sums the payload and writes the
 * serialized IPv4 header (ipv4_header.cpp:62-86: ver 4, hlen 5, tos 0,
 * len = datagram length mod 2^16, id, DF, ttl, proto 6, checksum, src, dst)
 * and TCP header (tcp_segment.cpp:76-106: ports, seqno, ackno, data offset 5,
 * flags, window, checksum, urgent 0) with both checksums
 * (TCPSegment::compute_checksum(pseudo_checksum()), then
 * IPv4Header::compute_checksum(), tcp_over_ip.cpp:83-84): the wire bytes of
 * serialize(wrap_tcp_in_ip(msg)), with no host-side serialization.
 * Datagrams shorter than 40 bytes are left untouched (checksums 0).
 * d_ip_ck / d_tcp_ck (optional) receive the two checksums. */
int ics_tcp_wrap_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets, uint64_t stride,
                       uint64_t dgram_len, uint64_t n, const ics_tcp_msg* d_msgs, uint16_t* d_ip_ck,
                       uint16_t* d_tcp_ck, void* stream);

/* The same wrap with the headers kept apart — the two pieces an
 * InternetDatagram holds (util/tools/ipv4_datagram.h:10-34: header, then the
 * serialized segment) and what a writev/sendmmsg iovec pair sends: segment i
 * of d_payloads is message i's payload ALONE (no header room); the 40 header
 * bytes of datagram i go to d_hdrs + 40*i (4-byte aligned), written as one
 * coalesced array instead of into the payload stream.  Datagram i on the wire
 * = d_hdrs[40 i .. 40 i + 40) followed by payload i.  From 2^18 datagrams up
 * the engine runs two launches on `stream` (payload sums, then the headers),
 * faster than storing headers inside the payload stream;
 * d_msgs must be 4-byte aligned (both wrap calls). */
int ics_tcp_wrap_headers(ics_ctx* ctx, const void* d_payloads, const uint64_t* d_offsets, uint64_t stride,
                         uint64_t payload_len, uint64_t n, const ics_tcp_msg* d_msgs, void* d_hdrs,
                         uint16_t* d_ip_ck, uint16_t* d_tcp_ck, void* stream);

/* ---- several batches in one launch -------------------------------------- */
/* The receive and transmit paths hand the engine a stream of small batches —
 * one per event-loop tick or per filled arena (the reference reads its TUN fd
 * one datagram per call, util/tuntap/tuntap_adapter.cpp:5-21, inside the
 * socket's event loop, util/tcp_minnow_socket/tcp_minnow_socket.h:138-164).
 * Each launch pays a fixed ramp and drain of a few microseconds, so k such
 * batches queued together run as ONE launch per kernel shape (batches of up
 * to 16 per launch): results identical to k calls of ics_checksum_batch /
 * ics_ipv4_tcp_batch on the same arguments, in any order (the batches must
 * not overlap where PATCH writes).  Fixed-stride batches take the geometry
 * their length picks; offsets batches take the unplanned default (no
 * binning: call ics_checksum_batch for one large mixed batch).  The
 * descriptor arrays are host memory, read before the call returns. */
typedef struct ics_seg_batch {
  const void* bytes;         /* d_bytes of ics_checksum_batch */
  const uint64_t* offsets;   /* d_offsets (NULL: fixed stride) */
  uint64_t stride, seg_len, n;
  const uint32_t* init;      /* d_init (NULL = 0) */
  uint16_t* out;             /* d_out */
} ics_seg_batch;
int ics_checksum_batchv(ics_ctx* ctx, const ics_seg_batch* batches, uint32_t k, void* stream);

typedef struct ics_dgram_batch {
  void* dgrams;              /* d_dgrams of ics_ipv4_tcp_batch */
  const uint64_t* offsets;   /* d_offsets (NULL: fixed stride) */
  uint64_t stride, dgram_len, n;
  uint16_t* ip_ck;           /* each output may be NULL */
  uint16_t* tcp_ck;
  uint8_t* status;
} ics_dgram_batch;
int ics_ipv4_tcp_batchv(ics_ctx* ctx, const ics_dgram_batch* batches, uint32_t k, int mode, void* stream);

/* ---- host-memory variants (PCIe-inclusive path) ------------------------ */
/* Same semantics as ics_checksum_batch / ics_ipv4_tcp_batch on host
 * buffers; ics_checksum_batch_host takes segments of any length (longer than
 * a staging slot: summed piecewise, parity carried, as add() chains do).  The engine stages through pinned memory in chunks (page-locked
 * caller buffers are DMA'd directly) and pipelines H2D / kernel / D2H on its
 * slot streams; returns when the outputs are complete.  PATCH on host
 * memory: the device computes the two checksums and the engine writes the
 * two fields into h_dgrams on the host (same bytes as the device PATCH). */
int ics_checksum_batch_host(ics_ctx* ctx, const void* h_bytes, const uint64_t* h_offsets,
                            uint64_t stride, uint64_t seg_len, const uint32_t* h_init,
                            uint16_t* h_out, uint64_t n);
int ics_ipv4_tcp_batch_host(ics_ctx* ctx, void* h_dgrams, const uint64_t* h_offsets,
                            uint64_t stride, uint64_t dgram_len, uint64_t n, int mode,
                            uint16_t* h_ip_ck, uint16_t* h_tcp_ck, uint8_t* h_status);
/* ics_tcp_wrap_batch on host memory (e.g. a page-locked DatagramBatch arena
 * the payloads were copied into once): the payload bytes go to the device,
 * only the 40 header bytes per datagram come back and are written into
 * h_dgrams.  Synchronous. */
int ics_tcp_wrap_batch_host(ics_ctx* ctx, void* h_dgrams, const uint64_t* h_offsets, uint64_t stride,
                            uint64_t dgram_len, uint64_t n, const ics_tcp_msg* h_msgs);
/* ics_tcp_wrap_headers on host memory: payloads in, 40 header bytes per
 * datagram out into h_hdrs.  Synchronous. */
int ics_tcp_wrap_headers_host(ics_ctx* ctx, const void* h_payloads, const uint64_t* h_offsets, uint64_t stride,
                              uint64_t payload_len, uint64_t n, const ics_tcp_msg* h_msgs, void* h_hdrs);

/* Resident tick server (not a reference interface).  idle_us > 0: the
 * zero-copy *_host calls of at most 16 x blocks segments (checksum, fused
 * IPv4 in any mode, both wraps; fixed stride or offsets) are taken by a
 * kernel of `blocks` blocks that stays resident on the context's GPU between
 * calls and reads each call's job from mailboxes in page-locked memory (16
 * segments per block) — no kernel launch per call.  It leaves after idle_us
 * microseconds without a call (the next call launches it again) or on
 * ics_set_tick_server(ctx, 0) / ics_destroy.  While it is resident the
 * device is busy: hipDeviceSynchronize waits until it leaves.  Results are
 * identical to the launched path.  0 (default): off. */
int ics_set_tick_server(ics_ctx* ctx, uint32_t idle_us);
/* The server's blocks, 1..8 (default 4: ticks of up to 64 segments).  Each
 * resident block keeps one CU and one poll of its mailbox in flight over
 * PCIe; a tick of at most 16 segments costs the same with any number.
 * Takes effect at the server's next launch (a running server is stopped). */
int ics_set_tick_server_blocks(ics_ctx* ctx, uint32_t blocks);

/* ---- device memory helpers for FFI callers without an allocator -------- */
int ics_malloc(ics_ctx* ctx, void** d_ptr, size_t bytes);
int ics_free(ics_ctx* ctx, void* d_ptr);
/* Page-locked host memory: batches in it are DMA'd by the *_host calls with
 * no staging copy (the receive/transmit rings of a batched TUN/socket path). */
int ics_host_alloc(ics_ctx* ctx, void** h_ptr, size_t bytes);
int ics_host_free(ics_ctx* ctx, void* h_ptr);
int ics_memcpy_htod(ics_ctx* ctx, void* d_dst, const void* h_src, size_t bytes, void* stream);
int ics_memcpy_dtoh(ics_ctx* ctx, void* h_dst, const void* d_src, size_t bytes, void* stream);
int ics_stream_synchronize(ics_ctx* ctx, void* stream);

/* ---- diagnostics (not a reference interface) ----------------------------- */
/* Which launch the last batch call on this context issued, and the plan
 * cache's counters since ics_create: a caller can check that its steady-state
 * batches hit the cached plan (and tests check which kernel ran).  Racy
 * snapshots when several threads share the context. */
#define ICS_K_CHECKSUM 1         /* k_checksum: one lane group per segment */
#define ICS_K_SMALL 2            /* k_checksum_small: several short segments per lane group */
#define ICS_K_TINY 3             /* k_checksum_tiny: one lane per segment */
#define ICS_K_DENSE 4            /* k_checksum_dense: fixed stride == length in {32, 64, 128} */
#define ICS_K_TWOCLASS 5         /* k_checksum_twoclass: short segments one per lane, long ones 16 lanes */
#define ICS_K_BINNED 6           /* the length-binning passes + bin launches */
#define ICS_K_IPV4 7             /* k_ipv4_tcp */
#define ICS_K_IPV4_TWOCLASS 8    /* k_ipv4_twoclass */
#define ICS_K_WRAP 9             /* k_tcp_wrap, one pass */
#define ICS_K_WRAP_2PASS 10      /* k_tcp_wrap (payload sums) + k_tcp_hdr */
#define ICS_K_ROUTER 11          /* k_router_ttl */
#define ICS_K_BATCHV 12          /* several batches in one launch (ics_*_batchv) */
#define ICS_K_TILE 13            /* k_span: an offsets batch as one packed stream, S (1..63) segments per wave */
#define ICS_K_ROUTER_HDRS 14     /* k_router_hdrs: the router step, forwarded headers apart */
#define ICS_K_TICK 15            /* k_tick: a zero-copy *_host tick of <= 16 offsets segments, offsets in the kernel arguments */
#define ICS_K_TICK_SERVER 16     /* the resident tick server took the tick (ics_set_tick_server) */
/* last_lps / last_unroll by kernel:
 *   ICS_K_CHECKSUM .. ICS_K_WRAP_2PASS  lanes per segment / loads in flight per lane
 *   ICS_K_TWOCLASS, ICS_K_IPV4_TWOCLASS  long-segment lanes (16) / segments per wave (16 or 32; 8 only under ICSUM_FORCE twoclass=8)
 *   ICS_K_BATCHV  the ICS_BV_* shape of the last launch group / batches in the call
 *   ICS_K_TILE    segments per wave S / ICS_TILE_* operation; S is chosen per
 *                 call, clamp(20 KiB / mean segment length, 1, 63) from the
 *                 cached plan (ICSUM_FORCE span_segs pins it)
 *   ICS_K_ROUTER, ICS_K_ROUTER_HDRS  0 / 0
 *   ICS_K_TICK, ICS_K_TICK_SERVER  16 / 8 (a 16-lane group per segment, one block) */
#define ICS_BV_DENSE64 0 /* fixed stride == length == 64 B, 16-byte aligned */
#define ICS_BV_TINY 1    /* one lane per segment (ACK-sized fixed lengths) */
#define ICS_BV_SMALL 2   /* 4-lane groups, two segments in flight */
#define ICS_BV_LINE16 3  /* 16-lane line grid */
#define ICS_BV_LINE64 4  /* 64-lane line grid */
#define ICS_BV_LANE1 5   /* fused IPv4 kernel, one lane per ACK-sized datagram */
#define ICS_TILE_CHECKSUM 0
#define ICS_TILE_IPV4 1
#define ICS_TILE_WRAP 2
#define ICS_TILE_WRAP_APART 3
typedef struct ics_dispatch_info_t {
  uint64_t plan_hits;      /* lookups that found this batch's landed plan */
  uint64_t plan_misses;    /* lookups that did not (first call, plan still in flight) */
  uint64_t plan_requests;  /* plan kernels queued behind launches */
  int32_t last_kernel;     /* ICS_K_* of the last call's main launch (0: none yet) */
  int32_t last_lps;        /* its lanes per segment (other kernels: see the table above) */
  int32_t last_unroll;     /* its loads in flight per lane (other kernels: see the table above) */
  int32_t last_plan;       /* the cached plan it followed (k_bin_plan ids 0-3), -1 none */
  uint64_t host_zero_copy; /* *_host calls whose batch the kernel read in place (one chunk, no DMA) */
  uint64_t host_dma_chunks; /* staged chunks (and long-segment pieces) the *_host calls DMA'd */
} ics_dispatch_info_t;
int ics_dispatch_info(const ics_ctx* ctx, ics_dispatch_info_t* info);

#ifdef __cplusplus
}
#endif

#endif /* ICSUM_H */
