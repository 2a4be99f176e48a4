// icsum_api.cpp — the C-ABI of libicsum.so (declared in include/icsum.h).
//
// Thin, exception-free layer: argument validation, device binding, error
// strings, and the extern "C" entry points.  Which kernel runs a batch is
// icsum_dispatch.cpp's business, the host-memory pipeline icsum_host.cpp's;
// all arithmetic happens in the HIP kernels (kernels/icsum_kernels.hip) and
// there is no CPU fallback — without a usable GPU every call returns an error.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <new>
#include <string>
#include <thread>

#include "icsum_ctx.h"
#include "icsum_workload.h"

namespace icsum::detail {

namespace {
thread_local std::string g_err;
}  // namespace

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(e == hipErrorOutOfMemory ? ICS_ERR_NOMEM : ICS_ERR_HIP, "%s: %s (%d)", what,
              hipGetErrorString(e), int(e));
}

const char* last_error() { return g_err.c_str(); }

int bind(ics_ctx* ctx) {
  if (!ctx) return fail(ICS_ERR_INVALID, "null context");
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != ctx->device) ICS_HIP(hipSetDevice(ctx->device));
  return ICS_OK;
}

int bounds_verdict(hipStream_t st, int rc) {
  if (rc != ICS_OK || !icsum::bounds_checked_build()) return rc;
  uint32_t flags = 0;
  uint64_t what = 0;
  ICS_HIP(icsum::bounds_take(st, &flags, &what));
  if (flags)
    return fail(ICS_ERR_INVALID,
                "bounds check: %s%s%s (first: %s 0x%llx)", (flags & 1u) ? "load outside a segment's envelope " : "",
                (flags & 2u) ? "offsets not monotone " : "", (flags & 4u) ? "header load past a datagram " : "",
                (flags & 2u) && !(flags & 5u) ? "segment" : "address", (unsigned long long)what);
  return ICS_OK;
}

}  // namespace icsum::detail

using namespace icsum::detail;

extern "C" {

const char* ics_version(void) {
  return icsum::bounds_checked_build() ? "icsum 0.2.0 (gfx950, bounds-checked debug build)" : "icsum 0.2.0 (gfx950)";
}
int ics_abi_version(void) { return ICS_ABI_VERSION; }
const char* ics_last_error(void) { return last_error(); }

int ics_device_count(int* count) {
  if (!count) return fail(ICS_ERR_INVALID, "null count");
  *count = 0;
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e == hipErrorNoDevice || (e == hipSuccess && c == 0)) return ICS_OK;
  ICS_HIP(e);
  *count = c;
  return ICS_OK;
}

int ics_create(int device, ics_ctx** out) {
  if (!out) return fail(ICS_ERR_INVALID, "null output pointer");
  *out = nullptr;
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess || c == 0) return fail(ICS_ERR_NODEVICE, "no GPU available (%s)", hipGetErrorString(e));
  if (device < 0 || device >= c) return fail(ICS_ERR_NODEVICE, "device %d out of range [0,%d)", device, c);
  ICS_HIP(hipSetDevice(device));
  ics_ctx* ctx = new (std::nothrow) ics_ctx();
  if (!ctx) return fail(ICS_ERR_NOMEM, "context allocation failed");
  ctx->device = device;
  if (int rc = apply_force(ctx, std::getenv("ICSUM_FORCE"))) {
    delete ctx;
    return rc;
  }
  if (hipMalloc(&ctx->d_zero, 64) != hipSuccess || hipMemset(ctx->d_zero, 0, 64) != hipSuccess) {
    delete ctx;
    return fail(ICS_ERR_NOMEM, "device allocation failed");
  }
  {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    ctx->copy_threads = std::max<size_t>(1, env_u32("ICSUM_COPY_THREADS", std::min(8u, hw)));
  }
  if (hipEventCreateWithFlags(&ctx->scratch.ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipFree(ctx->d_zero);
    delete ctx;
    return fail(ICS_ERR_HIP, "event creation failed");
  }
  {  // the plan cache's words; coherent: the plan kernel's store reaches host memory without a flush
    void* p = nullptr;
    if (hipHostMalloc(&p, 8 * ics_ctx::kPlanSlots, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess) {
      ctx->plan_host = static_cast<uint64_t*>(p);
      for (int k = 0; k < ics_ctx::kPlanSlots; ++k) ctx->plan_host[k] = ~uint64_t(0);
      void* dp = nullptr;
      if (hipHostGetDevicePointer(&dp, p, 0) == hipSuccess) {
        ctx->plan_host_dev = static_cast<uint64_t*>(dp);
      } else {
        (void)hipHostFree(p);
        ctx->plan_host = nullptr;
      }
    }
    (void)hipGetLastError();
  }
  ctx->nslots = int(std::min<uint32_t>(std::max<uint32_t>(env_u32("ICSUM_HOST_SLOTS", 3), 2), ics_ctx::kMaxSlots));
  ctx->slot_bytes = size_t(std::max<uint32_t>(env_u32("ICSUM_HOST_SLOT_MB", 32), 1)) << 20;
  *out = ctx;
  return ICS_OK;
}

int ics_destroy(ics_ctx* ctx) {
  if (!ctx) return ICS_OK;
  if (bind(ctx) == ICS_OK) {
    free_staging(ctx);
    if (ctx->d_zero) (void)hipFree(ctx->d_zero);
    if (ctx->plan_host) (void)hipHostFree(ctx->plan_host);
    ctx->scratch.release();
  }
  delete ctx;
  return ICS_OK;
}

int ics_dispatch_info(const ics_ctx* ctx, ics_dispatch_info_t* info) {
  if (!ctx || !info) return fail(ICS_ERR_INVALID, "null argument");
  info->plan_hits = ctx->n_hits.load(std::memory_order_relaxed);
  info->plan_misses = ctx->n_misses.load(std::memory_order_relaxed);
  info->plan_requests = ctx->n_replans.load(std::memory_order_relaxed);
  info->last_kernel = ctx->last_kernel.load(std::memory_order_relaxed);
  info->last_lps = ctx->last_lps.load(std::memory_order_relaxed);
  info->last_unroll = ctx->last_unroll.load(std::memory_order_relaxed);
  info->last_plan = ctx->last_plan.load(std::memory_order_relaxed);
  info->host_zero_copy = ctx->n_host_zc.load(std::memory_order_relaxed);
  info->host_dma_chunks = ctx->n_host_dma.load(std::memory_order_relaxed);
  return ICS_OK;
}

int ics_device_of(const ics_ctx* ctx, int* device) {
  if (!ctx || !device) return fail(ICS_ERR_INVALID, "null argument");
  *device = ctx->device;
  return ICS_OK;
}

int ics_checksum_batch(ics_ctx* ctx, const void* d_bytes, const uint64_t* d_offsets, uint64_t stride,
                       uint64_t seg_len, const uint32_t* d_init, uint16_t* d_out, uint64_t n,
                       void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_bytes || !d_out) return fail(ICS_ERR_INVALID, "null device buffer");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_bytes), d_offsets, stride, seg_len, n, ctx->d_zero};
  return bounds_verdict(static_cast<hipStream_t>(stream),
                        checksum_device(ctx, sp, d_init, nullptr, d_out, 0, static_cast<hipStream_t>(stream)));
}

int ics_sum_batch(ics_ctx* ctx, const void* d_bytes, const uint64_t* d_offsets, uint64_t stride,
                  uint64_t seg_len, const uint32_t* d_init, const uint8_t* d_odd, uint32_t* d_sum,
                  uint64_t n, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_bytes || !d_sum) return fail(ICS_ERR_INVALID, "null device buffer");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_bytes), d_offsets, stride, seg_len, n, ctx->d_zero};
  return bounds_verdict(static_cast<hipStream_t>(stream),
                        checksum_device(ctx, sp, d_init, d_odd, d_sum, 1, static_cast<hipStream_t>(stream)));
}

int ics_set_binning(ics_ctx* ctx, int mode) {
  if (!ctx) return fail(ICS_ERR_INVALID, "null context");
  if (mode < ICS_BINNING_AUTO || mode > ICS_BINNING_BINNED) return fail(ICS_ERR_INVALID, "bad binning mode %d", mode);
  ctx->bin = mode;
  return ICS_OK;
}

int ics_set_tick_server(ics_ctx* ctx, uint32_t idle_us) {
  if (int rc = bind(ctx)) return rc;
  if (idle_us > 10000000u) return fail(ICS_ERR_INVALID, "tick server idle time %u us above 10 s", idle_us);
  std::lock_guard<std::mutex> lock(ctx->mu);  // the *_host calls' lock: no job in flight
  const int rc = icsum::detail::server_stop(ctx);  // a running server keeps its old idle time: restart it
  ctx->srv_idle_us = idle_us;
  return rc;
}

int ics_set_tick_server_blocks(ics_ctx* ctx, uint32_t blocks) {
  if (int rc = bind(ctx)) return rc;
  if (blocks < 1 || blocks > icsum::kSrvBlocksMax)
    return fail(ICS_ERR_INVALID, "tick server blocks %u outside 1..%u", blocks, icsum::kSrvBlocksMax);
  std::lock_guard<std::mutex> lock(ctx->mu);
  const int rc = icsum::detail::server_stop(ctx);  // the next tick launches the new grid
  ctx->srv_blocks = blocks;
  return rc;
}

int ics_fold_batch(ics_ctx* ctx, const uint32_t* d_sum, uint16_t* d_out, uint64_t n, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_sum || !d_out) return fail(ICS_ERR_INVALID, "null device buffer");
  ICS_HIP(icsum::launch_fold(d_sum, d_out, n, static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int ics_ipv4_tcp_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets, uint64_t stride,
                       uint64_t dgram_len, uint64_t n, int mode, uint16_t* d_ip_ck,
                       uint16_t* d_tcp_ck, uint8_t* d_status, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (mode < ICS_MODE_COMPUTE || mode > ICS_MODE_PATCH) return fail(ICS_ERR_INVALID, "bad mode %d", mode);
  if (n == 0) return ICS_OK;
  if (!d_dgrams) return fail(ICS_ERR_INVALID, "null datagram buffer");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_dgrams), d_offsets, stride, dgram_len, n, ctx->d_zero};
  return bounds_verdict(static_cast<hipStream_t>(stream),
                        ipv4_device(ctx, sp, mode, d_ip_ck, d_tcp_ck, d_status, static_cast<hipStream_t>(stream)));
}

int ics_tcp_wrap_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets, uint64_t stride,
                       uint64_t dgram_len, uint64_t n, const ics_tcp_msg* d_msgs, uint16_t* d_ip_ck,
                       uint16_t* d_tcp_ck, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_dgrams || !d_msgs) return fail(ICS_ERR_INVALID, "null device buffer");
  if (reinterpret_cast<uintptr_t>(d_msgs) & 3u) return fail(ICS_ERR_INVALID, "message records not 4-byte aligned");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_dgrams), d_offsets, stride, dgram_len, n, ctx->d_zero};
  // the stack's segments are <= 1000 B of payload (TCPConfig::MAX_PAYLOAD_SIZE): the
  // 16-lane line grid of MTU-sized datagrams unless a fixed length says otherwise
  hipStream_t st = static_cast<hipStream_t>(stream);
  return bounds_verdict(st, wrap_device(ctx, sp, d_msgs, nullptr, d_ip_ck, d_tcp_ck, false, 1040, st));
}

int ics_tcp_wrap_headers(ics_ctx* ctx, const void* d_payloads, const uint64_t* d_offsets, uint64_t stride,
                         uint64_t payload_len, uint64_t n, const ics_tcp_msg* d_msgs, void* d_hdrs,
                         uint16_t* d_ip_ck, uint16_t* d_tcp_ck, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_payloads || !d_msgs || !d_hdrs) return fail(ICS_ERR_INVALID, "null device buffer");
  if (reinterpret_cast<uintptr_t>(d_msgs) & 3u) return fail(ICS_ERR_INVALID, "message records not 4-byte aligned");
  if (reinterpret_cast<uintptr_t>(d_hdrs) & 3u) return fail(ICS_ERR_INVALID, "header array not 4-byte aligned");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_payloads), d_offsets, stride, payload_len, n, ctx->d_zero};
  hipStream_t st = static_cast<hipStream_t>(stream);
  return bounds_verdict(st, wrap_device(ctx, sp, d_msgs, static_cast<uint32_t*>(d_hdrs), d_ip_ck, d_tcp_ck, true,
                                        1000, st));
}

int ics_checksum_batchv(ics_ctx* ctx, const ics_seg_batch* batches, uint32_t k, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (k == 0) return ICS_OK;
  if (!batches) return fail(ICS_ERR_INVALID, "null batch array");
  for (uint32_t j = 0; j < k; ++j)
    if (batches[j].n && (!batches[j].bytes || !batches[j].out))
      return fail(ICS_ERR_INVALID, "batch %u: null device buffer", j);
  hipStream_t st = static_cast<hipStream_t>(stream);
  return bounds_verdict(st, checksum_batchv_device(ctx, batches, k, st));
}

int ics_ipv4_tcp_batchv(ics_ctx* ctx, const ics_dgram_batch* batches, uint32_t k, int mode, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (mode < ICS_MODE_COMPUTE || mode > ICS_MODE_PATCH) return fail(ICS_ERR_INVALID, "bad mode %d", mode);
  if (k == 0) return ICS_OK;
  if (!batches) return fail(ICS_ERR_INVALID, "null batch array");
  for (uint32_t j = 0; j < k; ++j)
    if (batches[j].n && !batches[j].dgrams) return fail(ICS_ERR_INVALID, "batch %u: null datagram buffer", j);
  hipStream_t st = static_cast<hipStream_t>(stream);
  return bounds_verdict(st, ipv4_batchv_device(ctx, batches, k, mode, st));
}

int ics_tcp_wrap_headers_host(ics_ctx* ctx, const void* h_payloads, const uint64_t* h_offsets, uint64_t stride,
                              uint64_t payload_len, uint64_t n, const ics_tcp_msg* h_msgs, void* h_hdrs) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!h_payloads || !h_msgs || !h_hdrs) return fail(ICS_ERR_INVALID, "null host buffer");
  return host_pipeline(ctx, 2, const_cast<void*>(h_payloads), h_offsets, stride, payload_len, nullptr, n, 1,
                       nullptr, nullptr, static_cast<uint8_t*>(h_hdrs), h_msgs);
}

int ics_tcp_wrap_batch_host(ics_ctx* ctx, void* h_dgrams, const uint64_t* h_offsets, uint64_t stride,
                            uint64_t dgram_len, uint64_t n, const ics_tcp_msg* h_msgs) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!h_dgrams || !h_msgs) return fail(ICS_ERR_INVALID, "null host buffer");
  return host_pipeline(ctx, 2, h_dgrams, h_offsets, stride, dgram_len, nullptr, n, 0, nullptr, nullptr, nullptr,
                       h_msgs);
}

int ics_router_ttl_batch(ics_ctx* ctx, void* d_dgrams, const uint64_t* d_offsets, uint64_t stride,
                         uint64_t dgram_len, uint64_t n, uint8_t* d_status, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_dgrams || !d_status) return fail(ICS_ERR_INVALID, "null device buffer");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_dgrams), d_offsets, stride, dgram_len, n, ctx->d_zero};
  return bounds_verdict(static_cast<hipStream_t>(stream),
                        router_device(ctx, sp, nullptr, d_status, static_cast<hipStream_t>(stream)));
}

int ics_router_ttl_headers(ics_ctx* ctx, const void* d_dgrams, const uint64_t* d_offsets, uint64_t stride,
                           uint64_t dgram_len, uint64_t n, void* d_hdrs, uint8_t* d_status, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!d_dgrams || !d_hdrs || !d_status) return fail(ICS_ERR_INVALID, "null device buffer");
  if (reinterpret_cast<uintptr_t>(d_hdrs) & 3u) return fail(ICS_ERR_INVALID, "header array not 4-byte aligned");
  const icsum::SegSpec sp{static_cast<const uint8_t*>(d_dgrams), d_offsets, stride, dgram_len, n, ctx->d_zero};
  return bounds_verdict(static_cast<hipStream_t>(stream),
                        router_device(ctx, sp, static_cast<uint32_t*>(d_hdrs), d_status,
                                      static_cast<hipStream_t>(stream)));
}

int ics_checksum_batch_host(ics_ctx* ctx, const void* h_bytes, const uint64_t* h_offsets,
                            uint64_t stride, uint64_t seg_len, const uint32_t* h_init,
                            uint16_t* h_out, uint64_t n) {
  if (int rc = bind(ctx)) return rc;
  if (n == 0) return ICS_OK;
  if (!h_bytes || !h_out) return fail(ICS_ERR_INVALID, "null host buffer");
  return host_pipeline(ctx, 0, const_cast<void*>(h_bytes), h_offsets, stride, seg_len, h_init, n, 0,
                       h_out, nullptr, nullptr);
}

int ics_ipv4_tcp_batch_host(ics_ctx* ctx, void* h_dgrams, const uint64_t* h_offsets, uint64_t stride,
                            uint64_t dgram_len, uint64_t n, int mode, uint16_t* h_ip_ck,
                            uint16_t* h_tcp_ck, uint8_t* h_status) {
  if (int rc = bind(ctx)) return rc;
  if (mode < ICS_MODE_COMPUTE || mode > ICS_MODE_PATCH) return fail(ICS_ERR_INVALID, "bad mode %d", mode);
  if (n == 0) return ICS_OK;
  if (!h_dgrams) return fail(ICS_ERR_INVALID, "null host buffer");
  return host_pipeline(ctx, 1, h_dgrams, h_offsets, stride, dgram_len, nullptr, n, mode, h_ip_ck,
                       h_tcp_ck, h_status);
}

int ics_malloc(ics_ctx* ctx, void** d_ptr, size_t bytes) {
  if (int rc = bind(ctx)) return rc;
  if (!d_ptr) return fail(ICS_ERR_INVALID, "null output pointer");
  ICS_HIP(hipMalloc(d_ptr, bytes ? bytes : 1));
  return ICS_OK;
}

int ics_free(ics_ctx* ctx, void* d_ptr) {
  if (int rc = bind(ctx)) return rc;
  if (d_ptr) ICS_HIP(hipFree(d_ptr));
  return ICS_OK;
}

int ics_host_alloc(ics_ctx* ctx, void** h_ptr, size_t bytes) {
  if (int rc = bind(ctx)) return rc;
  if (!h_ptr) return fail(ICS_ERR_INVALID, "null output pointer");
  ICS_HIP(hipHostMalloc(h_ptr, bytes ? bytes : 1, 0));
  return ICS_OK;
}

int ics_host_free(ics_ctx* ctx, void* h_ptr) {
  if (int rc = bind(ctx)) return rc;
  if (h_ptr) ICS_HIP(hipHostFree(h_ptr));
  return ICS_OK;
}

int ics_memcpy_htod(ics_ctx* ctx, void* d_dst, const void* h_src, size_t bytes, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (!bytes) return ICS_OK;
  ICS_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int ics_memcpy_dtoh(ics_ctx* ctx, void* h_dst, const void* d_src, size_t bytes, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (!bytes) return ICS_OK;
  ICS_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int ics_stream_synchronize(ics_ctx* ctx, void* stream) {
  if (int rc = bind(ctx)) return rc;
  ICS_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

// ---- synthetic workloads (icsum_workload.h) -----------------------------

int icsw_fill_bytes(ics_ctx* ctx, void* d_bytes, uint64_t nbytes, uint64_t seed, uint64_t pos0,
                    void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (nbytes && !d_bytes) return fail(ICS_ERR_INVALID, "null device buffer");
  ICS_HIP(icsum::launch_fill_bytes(static_cast<uint8_t*>(d_bytes), nbytes, seed, pos0,
                                   static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int icsw_pseudo_inits(ics_ctx* ctx, uint32_t* d_init, const uint64_t* d_offsets, uint64_t seg_len,
                      uint64_t n, uint64_t seed, uint64_t index0, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n && !d_init) return fail(ICS_ERR_INVALID, "null device buffer");
  ICS_HIP(icsum::launch_pseudo_inits(d_init, d_offsets, seg_len, n, seed, index0,
                                     static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

int icsw_ipv4_tcp_headers(ics_ctx* ctx, void* d_dgrams, uint64_t stride, uint64_t dgram_len,
                          uint64_t n, uint64_t seed, uint64_t index0, void* stream) {
  if (int rc = bind(ctx)) return rc;
  if (n && !d_dgrams) return fail(ICS_ERR_INVALID, "null device buffer");
  if (dgram_len < 20) return fail(ICS_ERR_INVALID, "datagram length %llu < 20", (unsigned long long)dgram_len);
  ICS_HIP(icsum::launch_ipv4_tcp_headers(static_cast<uint8_t*>(d_dgrams), stride, dgram_len, n, seed,
                                         index0, static_cast<hipStream_t>(stream)));
  return ICS_OK;
}

static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t icsw_mixed_len(uint64_t seed, uint64_t i) {
  const uint64_t m = mix64((seed ^ 0x3C3C3C3C3C3C3C3Cull) + (i + 1) * 0x9E3779B97F4A7C15ull);
  const unsigned e = 6u + unsigned(m % 10u);
  return (1ull << e) + ((m >> 8) & ((1ull << e) - 1));
}

int icsw_mixed_offsets(uint64_t* h_offsets, uint64_t n, uint64_t seed) {
  if (!h_offsets) return fail(ICS_ERR_INVALID, "null offsets");
  h_offsets[0] = 0;
  for (uint64_t i = 0; i < n; ++i) h_offsets[i + 1] = h_offsets[i] + icsw_mixed_len(seed, i);
  return ICS_OK;
}

}  // extern "C"
