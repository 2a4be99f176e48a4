// Dev probe (round 5): HBM read bandwidth of a streaming wave as a function
// of the bytes it keeps in flight and of the waves per CU — the same shape as
// the tile launches' stream (4 KiB windows per wave, four dwordx4
// non-temporal buffer loads per lane per window, D register sets = D windows
// in flight, every dword added so nothing is dead; per-wave result stores, no
// atomics).  The grid is persistent (blocks_per_cu x 256 CUs, all resident:
// dynamic LDS caps the blocks per CU) and sweeps the 807 MB buffer
// (1 M x 770 B) in window order.  One JSON line per (D, blocks per CU):
// us per launch (HIP events, 20 launches, median of 5), fraction of 8 TB/s.
// Build: hipcc --offload-arch=gfx950 -O3 pattern_probe.hip -o pattern_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                     \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

constexpr uint32_t kWin = 4096;

// LANE64: lane L loads bytes [64 L + 16 u, +16) (lane-contiguous); PIECES:
// instruction u, lane group g = L / 16 loads [1024 g + 256 u + 16 (L % 16), +16)
// (four 256-byte pieces per instruction, k_checksum's 16-lane line grid)
template <int AUX = 2, bool LANE64 = false, bool PIECES = false>
__device__ __forceinline__ void load_win(const uint8_t* base, uint64_t off, uint64_t end, u32x4 (&v)[4]) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t left = end > off ? end - off : 0;
  const uint32_t len = uint32_t(left < kWin ? left : kWin);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base + (off < end ? off : 0)), 0, int(len), 0x00020000);
#pragma unroll
  for (int u = 0; u < 4; ++u)
    v[u] = __builtin_bit_cast(
        u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                   rs, LANE64 ? lane * 64u : PIECES ? (lane >> 4) * 1024u + (lane & 15u) * 16u : lane * 16u,
                   LANE64 ? u * 16 : PIECES ? u * 256 : u * 1024, AUX));
}

// one-shot waves: wave w reads windows [w D, (w + 1) D) (contiguous D x 4 KiB)
// and exits; the hardware dispatcher keeps the CUs full
template <int D, int AUX>
__global__ __launch_bounds__(256) void k_oneshot(const uint8_t* __restrict__ buf, uint64_t nbytes,
                                                 uint32_t* __restrict__ out) {
  const uint64_t w = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  u32x4 b[D][4];
#pragma unroll
  for (int d = 0; d < D; ++d) load_win<AUX>(buf, (w * D + d) * kWin, nbytes, b[d]);
  uint32_t acc = 0;
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += b[d][u].x + b[d][u].y + b[d][u].z + b[d][u].w;
  out[(uint64_t(blockIdx.x) * 256 + threadIdx.x) & ((8u << 16) - 1)] = acc;
}

template <int D, int AUX = 2, bool LANE64 = false, bool XCD = false, bool PIECES = false>
__global__ __launch_bounds__(256) void k_pattern(const uint8_t* __restrict__ buf_all, uint64_t nbytes_all,
                                                 uint32_t* __restrict__ out) {
  extern __shared__ uint32_t pad[];
  const uint32_t wv = threadIdx.x >> 6;
  // XCD: block b runs on XCD b % 8 (round-robin dispatch); each XCD sweeps
  // its own contiguous eighth of the buffer
  const uint32_t nx = XCD ? 8u : 1u, x = XCD ? blockIdx.x % 8u : 0u;
  const uint64_t part = (nbytes_all / nx) & ~uint64_t(kWin - 1);
  const uint8_t* buf = buf_all + x * part;
  const uint64_t nbytes = x + 1 == nx ? nbytes_all - x * part : part;
  const uint64_t waves = uint64_t(gridDim.x / nx) * 4, first = uint64_t(blockIdx.x / nx) * 4 + wv;
  const uint64_t st = waves * kWin;
  uint32_t acc = 0;
  u32x4 b[D][4];
#pragma unroll
  for (int d = 0; d < D; ++d) load_win<AUX, LANE64, PIECES>(buf, (first + d * waves) * kWin, nbytes, b[d]);
  for (uint64_t o = first * kWin; o < nbytes; o += D * st) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += b[d][u].x + b[d][u].y + b[d][u].z + b[d][u].w;
      load_win<AUX, LANE64, PIECES>(buf, o + (D + d) * st, nbytes, b[d]);
    }
  }
  if (acc == 0x12345678u) pad[threadIdx.x] = acc;  // never true; keeps pad referenced
  out[uint64_t(blockIdx.x) * 256 + threadIdx.x] = acc;
}

int main() {
  const uint64_t nbytes = (uint64_t(1) << 20) * 770;
  uint8_t* buf[2];
  uint32_t* out;
  for (auto& p : buf) {
    CK(hipMalloc(&p, nbytes + 4096));
    CK(hipMemset(p, 1, nbytes + 4096));
  }
  CK(hipMalloc(&out, (8u << 16) * 4 + 8 * 256 * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  using K = void (*)(const uint8_t*, uint64_t, uint32_t*);
  struct Run {
    const char* name;
    K k;
    int d, bpc;  // bpc 0: one-shot grid, all blocks the data needs
  } runs[] = {{"persist_nt", k_pattern<3, 2>, 3, 4}, {"persist_nt_pieces", k_pattern<3, 2, false, false, true>, 3, 4},
              {"persist_nt", k_pattern<3, 2>, 3, 5}, {"persist_nt_pieces", k_pattern<3, 2, false, false, true>, 3, 5},
              {"persist_nt", k_pattern<2, 2>, 2, 6}, {"persist_nt_pieces", k_pattern<2, 2, false, false, true>, 2, 6}};
  for (const Run& r : runs) {
    const uint32_t grid = r.bpc ? uint32_t(r.bpc) * 256 : uint32_t((nbytes / kWin + 4 * r.d - 1) / (4 * r.d));
    const size_t lds = r.bpc ? (160 * 1024) / r.bpc - 1024 : 0;
    if (lds)
      CK(hipFuncSetAttribute(reinterpret_cast<const void*>(r.k), hipFuncAttributeMaxDynamicSharedMemorySize,
                             int(lds)));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(r.k, dim3(grid), dim3(256), lds, 0, buf[i & 1], nbytes, out);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int round = 0; round < 5; ++round) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(r.k, dim3(grid), dim3(256), lds, 0, buf[i & 1], nbytes, out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1000.f / 20.f);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[2];
    std::printf("{\"run\": \"%s\", \"windows\": %d, \"blocks_per_cu\": %d, \"grid\": %u, \"us\": %.2f, \"frac\": %.4f}\n",
                r.name, r.d, r.bpc, grid, us, nbytes / us / 1e3 / 8000.0);
    std::fflush(stdout);
  }
  return 0;
}
