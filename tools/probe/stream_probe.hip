// stream_probe.hip — dev tool: the sustained HBM read ceiling on this box.
// An "ideal" read kernel (every lane streams 16-byte non-temporal loads of a
// flat buffer, 8 in flight, one sum per lane) launched back to back, next to
// the same number of ics_checksum_batch launches on the NS workload.  Run under
// `rocprofv3 --kernel-trace` to read per-dispatch durations.
//   hipcc --offload-arch=gfx950 -O3 -I../../include stream_probe.hip ../../tcpip_network_protocol_stack_amd/libicsum.so -o stream_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "icsum.h"
#include "icsum_workload.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_ideal_read(const u32x4* __restrict__ p, uint64_t nvec,
                                                    uint32_t* __restrict__ out) {
  const uint64_t tid = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t step = uint64_t(gridDim.x) * 256;
  uint32_t acc = 0;
  for (uint64_t i = tid; i < nvec; i += step * 8) {
    u32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t j = i + u * step;
      v[u] = j < nvec ? __builtin_nontemporal_load(p + j) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[0] = acc;  // keep the loads live
}

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  const uint64_t n = 1 << 20, L = 1500, nbytes = n * L;
  ics_ctx* ctx = nullptr;
  if (ics_create(0, &ctx) != ICS_OK) {
    fprintf(stderr, "ics_create: %s\n", ics_last_error());
    return 1;
  }
  void *d = nullptr, *init = nullptr, *out = nullptr;
  CK(hipMalloc(&d, nbytes));
  CK(hipMalloc(&init, n * 4));
  CK(hipMalloc(&out, n * 4));
  icsw_fill_bytes(ctx, d, nbytes, 0x10710000, 0, nullptr);
  icsw_pseudo_inits(ctx, static_cast<uint32_t*>(init), nullptr, L, n, 0x10710000, 0, nullptr);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int round = 0; round < 2; ++round) {
    for (int which = 0; which < 2; ++which) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a, nullptr));
      for (int r = 0; r < reps; ++r) {
        if (which == 0)
          hipLaunchKernelGGL(k_ideal_read, dim3(8192), dim3(256), 0, nullptr, (const u32x4*)d, nbytes / 16,
                             (uint32_t*)out);
        else
          ics_checksum_batch(ctx, d, nullptr, L, L, (const uint32_t*)init, (uint16_t*)out, n, nullptr);
      }
      CK(hipEventRecord(b, nullptr));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("round %d %-14s %d launches: %.1f us/launch = %.1f GB/s\n", round,
             which ? "icsum NS" : "ideal read", reps, ms * 1e3 / reps, nbytes / (ms * 1e-3 / reps) / 1e9);
    }
  }
  ics_destroy(ctx);
  return 0;
}
