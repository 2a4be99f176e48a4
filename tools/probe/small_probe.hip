// small_probe.hip — dev tool: the floor for a SMALL device-resident batch.
// How long does the best plain read of 64 MiB (+ 4 MiB of per-segment words,
// + a 2 MiB u16 write) take on MI355X, launched back to back over 6 rotated
// copies so every launch streams from HBM (not the 256 MiB Infinity Cache)?
// Variants: loads per lane (1/2/4 dwordx4), block size, and one or two
// extra streams like config 3's init / out arrays.
//   hipcc --offload-arch=gfx950 -O3 small_probe.hip -o small_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// every lane reads U consecutive-by-wave 16-byte chunks (chunk = base + u * 64
// lanes), optionally one init word per 4 lanes and writes one u16 per 4 lanes
template <int U, bool META>
__global__ void k_read(const u32x4* __restrict__ p, const uint32_t* __restrict__ init,
                       uint16_t* __restrict__ out, uint64_t nvec) {
  const uint64_t wave = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t base = wave * 64 * U + lane;
  uint32_t acc = 0;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t j = base + uint64_t(u) * 64;
    v[u] = j < nvec ? __builtin_nontemporal_load(p + j) : u32x4{0, 0, 0, 0};
  }
  uint32_t i0 = 0;
  if (META) i0 = init[base >> 2];
#pragma unroll
  for (int u = 0; u < U; ++u) acc += __builtin_amdgcn_udot4(v[u].x ^ v[u].y, 0x01010101u, v[u].z + v[u].w, false);
  acc += i0;
  if (META) {
    if ((lane & 3) == 3) out[base >> 2] = uint16_t(acc);
  } else if (acc == 0x12345678u) {
    out[0] = 1;
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr int kCopies = 6;

template <int U, bool META>
int run(int block, u32x4** bufs, uint32_t** inits, uint16_t* out, uint64_t nbytes, hipEvent_t a, hipEvent_t b) {
  const uint64_t nvec = nbytes / 16;
  const uint64_t threads = nvec / U;
  const uint32_t blocks = uint32_t((threads + block - 1) / block);
  const int reps = 60;
  float best = 1e30f;
  for (int round = 0; round < 5; ++round) {
    CK(hipEventRecord(a, nullptr));
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL((k_read<U, META>), dim3(blocks), dim3(block), 0, nullptr, bufs[r % kCopies],
                         inits[r % kCopies], out, nvec);
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  const double us = best * 1e3 / reps;
  printf("{\"bytes\": %llu, \"loads_per_lane\": %d, \"meta\": %d, \"block\": %d, \"blocks\": %u, "
         "\"us\": %.2f, \"GBs\": %.1f}\n",
         (unsigned long long)nbytes, U, int(META), block, blocks, us, nbytes / us / 1e3);
  return 0;
}

int main() {
  const uint64_t nbytes = uint64_t(64) << 20;  // config 3: 1 M x 64 B
  u32x4* bufs[kCopies];
  uint32_t* inits[kCopies];
  uint16_t* out = nullptr;
  for (int c = 0; c < kCopies; ++c) {
    CK(hipMalloc(&bufs[c], nbytes));
    CK(hipMemset(bufs[c], c + 1, nbytes));
    CK(hipMalloc(&inits[c], nbytes / 16));
    CK(hipMemset(inits[c], c, nbytes / 16));
  }
  CK(hipMalloc(&out, nbytes / 32));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // settle the clocks: ~200 ms of reads
  for (int r = 0; r < 20000; ++r)
    hipLaunchKernelGGL((k_read<2, false>), dim3(8192), dim3(256), 0, nullptr, bufs[r % kCopies], inits[0], out,
                       nbytes / 16);
  CK(hipDeviceSynchronize());
  int rc = 0;
  for (int block : {256, 512, 1024}) {
    rc |= run<1, false>(block, bufs, inits, out, nbytes, a, b);
    rc |= run<2, false>(block, bufs, inits, out, nbytes, a, b);
    rc |= run<4, false>(block, bufs, inits, out, nbytes, a, b);
    rc |= run<8, false>(block, bufs, inits, out, nbytes, a, b);
    rc |= run<1, true>(block, bufs, inits, out, nbytes, a, b);
    rc |= run<2, true>(block, bufs, inits, out, nbytes, a, b);
    rc |= run<4, true>(block, bufs, inits, out, nbytes, a, b);
  }
  // a larger batch for the ramp: 256 MiB (1 copy repeated is MALL-resident; use 4 of the 6 back to back)
  return rc;
}
