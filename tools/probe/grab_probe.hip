// Dev probe (round 5): one-round streaming tails.  A 131 MB buffer (the stack
// tick's transmit payloads) read by 1024 persistent blocks of four waves
// (4 KiB windows, three in flight, NT loads) split into tiles of TB bytes,
// each wave a quarter of its tile: tiles assigned statically (tile =
// block + k * grid) or grabbed from a global counter (atomicAdd, the last
// block resets it).  Also the same bytes as one-shot waves (no tiles).
// One JSON line per (assignment, tile bytes): us per launch (HIP events, 20
// launches, median of 5), fraction of 8 TB/s.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                    \
  do {                                                           \
    hipError_t e = (x);                                          \
    if (e != hipSuccess) {                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                              \
    }                                                            \
  } while (0)
constexpr uint32_t kWin = 4096;

__device__ __forceinline__ void load_win(const uint8_t* base, uint64_t off, uint64_t end, u32x4 (&v)[4]) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t left = end > off ? end - off : 0;
  const uint32_t len = uint32_t(left < kWin ? left : kWin);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base + (off < end ? off : 0)), 0, int(len), 0x00020000);
#pragma unroll
  for (int u = 0; u < 4; ++u)
    v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16u, u * 1024, 2));
}

template <bool DYN>
__global__ __launch_bounds__(256) void k_tiles(const uint8_t* __restrict__ buf, uint64_t nbytes, uint64_t tb,
                                               uint32_t* __restrict__ ctr, uint32_t* __restrict__ out) {
  __shared__ uint32_t s_tile;
  const uint32_t wv = threadIdx.x >> 6;
  const uint64_t ntiles = (nbytes + tb - 1) / tb;
  uint32_t acc = 0;
  uint64_t t = blockIdx.x;
  for (;;) {
    if (DYN) {
      if (threadIdx.x == 0) s_tile = atomicAdd(ctr, 1u);
      __syncthreads();
      t = s_tile;
      __syncthreads();
    }
    if (t >= ntiles) break;
    const uint64_t lo = t * tb, hi = std::min(lo + tb, nbytes);
    const uint64_t q = ((hi - lo + 4 * kWin - 1) / (4 * kWin)) * kWin;
    const uint64_t qlo = std::min(lo + wv * q, hi), qhi = std::min(qlo + q, hi);
    u32x4 b0[4], b1[4], b2[4];
    load_win(buf, qlo, qhi, b0);
    load_win(buf, qlo + kWin, qhi, b1);
    load_win(buf, qlo + 2 * kWin, qhi, b2);
    for (uint64_t o = qlo; o < qhi; o += 3 * kWin) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += b0[u].x + b0[u].y + b0[u].z + b0[u].w;
      load_win(buf, o + 3 * kWin, qhi, b0);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += b1[u].x + b1[u].y + b1[u].z + b1[u].w;
      load_win(buf, o + 4 * kWin, qhi, b1);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += b2[u].x + b2[u].y + b2[u].z + b2[u].w;
      load_win(buf, o + 5 * kWin, qhi, b2);
    }
    if (!DYN) t += gridDim.x;
  }
  out[uint64_t(blockIdx.x) * 256 + threadIdx.x] = acc;
  if (DYN) {  // the last block resets the counter for the next launch
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      if (atomicAdd(ctr + 1, 1u) == gridDim.x - 1) {
        ctr[0] = 0;
        ctr[1] = 0;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_oneshot(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                 uint32_t* __restrict__ out) {
  const uint64_t w = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  u32x4 b[4];
  load_win(buf, w * kWin, nbytes, b);
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) acc += b[u].x + b[u].y + b[u].z + b[u].w;
  out[(uint64_t(blockIdx.x) * 256 + threadIdx.x) & ((1u << 20) - 1)] = acc;
}

int main() {
  const uint64_t nbytes = 141543414;
  uint8_t* buf[2];
  uint32_t *out, *ctr;
  for (auto& p : buf) {
    CK(hipMalloc(&p, nbytes + 4096));
    CK(hipMemset(p, 1, nbytes + 4096));
  }
  CK(hipMalloc(&out, (1u << 20) * 4 + 1024 * 256 * 4));
  CK(hipMalloc(&ctr, 64));
  CK(hipMemset(ctr, 0, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](auto launch, const char* name, uint64_t tb, int b2b) {
    for (int i = 0; i < 20; ++i) launch(i);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int round = 0; round < (b2b ? 5 : 30); ++round) {
      if (!b2b) CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < (b2b ? 20 : 1); ++i) launch(i);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1000.f / (b2b ? 20.f : 1.f));
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2];
    std::printf("{\"run\": \"%s\", \"tile_kib\": %llu, \"timing\": \"%s\", \"us\": %.2f, \"frac\": %.4f}\n", name,
                (unsigned long long)(tb >> 10), b2b ? "b2b" : "alone", us, nbytes / us / 1e3 / 8000.0);
    std::fflush(stdout);
  };
  for (int b2b = 1; b2b >= 0; --b2b) {
    time([&](int i) {
      hipLaunchKernelGGL(k_oneshot, dim3(uint32_t((nbytes + 4 * kWin - 1) / (4 * kWin))), dim3(256), 0, 0, buf[i & 1],
                         nbytes, out);
    }, "oneshot", 4096, b2b);
    for (uint64_t tb : {uint64_t(32) << 10, uint64_t(64) << 10, uint64_t(138) << 10}) {
      const uint64_t ntiles = (nbytes + tb - 1) / tb;
      const uint32_t grid = uint32_t(std::min<uint64_t>(ntiles, 1024));
      time([&](int i) {
        hipLaunchKernelGGL(k_tiles<false>, dim3(grid), dim3(256), 0, 0, buf[i & 1], nbytes, tb, ctr, out);
      }, "static", tb, b2b);
      time([&](int i) {
        hipLaunchKernelGGL(k_tiles<true>, dim3(grid), dim3(256), 0, 0, buf[i & 1], nbytes, tb, ctr, out);
      }, "dynamic", tb, b2b);
    }
  }
  return 0;
}
