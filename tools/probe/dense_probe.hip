// dense_probe.hip — dev tool: where config 3's dense kernel (1 M x 64 B
// segments + a u32 init per segment + a u16 out per segment) loses against
// the north-star stream.  Same memory pattern as k_checksum_dense (4 lanes per
// 64-byte segment, one dwordx4 per lane per segment, init read by the group,
// out written by its last lane), in three launch structures:
//   oneshot<S>   every wave handles S x 16 segments and exits (shipped: S = 4)
//   stride<S>    a capped grid, every wave loops over S x 16-segment tiles
//   stride_pf<S> the same loop with the next tile's loads issued before the
//                current tile is reduced
// each with and without the init / out streams (META), over 6 rotated copies
// so every launch streams from HBM; then tile layouts (k_layout), load policy
// and XCD runs (k_policy), occupancy caps (dynamic LDS) and consolidated
// metadata access (k_meta2).  Prints one JSON line per variant
// (profiles/r3_dense_probe.jsonl, DESIGN.md §6 "Config 3's ceiling").
//   hipcc --offload-arch=gfx950 -O3 dense_probe.hip -o dense_probe
//   ./dense_probe [segments_log2 = 20] [name filter]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;
constexpr int kCopies = 6;

__device__ __forceinline__ uint32_t reduce4(uint32_t x) {  // sum over the 4 lanes of a segment
  x += __shfl_xor(x, 1);
  x += __shfl_xor(x, 2);
  return x;
}

__device__ __forceinline__ uint32_t chunk_sum(u32x4 v) {
  return __builtin_amdgcn_udot4(v.x ^ v.y, 0x01010101u, v.z + v.w, false);
}

template <bool META>
__device__ __forceinline__ void finish(uint32_t acc, uint32_t i0, uint16_t* out, uint64_t seg, uint64_t n,
                                       uint32_t lane) {
  const uint32_t s = reduce4(acc) + i0;
  if (META) {
    if (seg < n && (lane & 3) == 3) out[seg] = uint16_t(s);
  } else if (s == 0x9E3779B9u) {
    out[0] = 1;
  }
}

// tile = 16 segments per wave-instruction x S: wave w's segments [w*16*S, (w+1)*16*S)
template <int S, bool META>
__global__ __launch_bounds__(kBlock) void k_oneshot(const u32x4* __restrict__ p, const uint32_t* __restrict__ init,
                                                    uint16_t* __restrict__ out, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  const uint64_t seg0 = wave * 16 * S + (lane >> 2);
  const uint64_t nch = n * 4;
  u32x4 v[S];
  uint32_t i0[S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const uint64_t c = (seg0 + uint64_t(k) * 16) * 4 + (lane & 3);
    v[k] = __builtin_nontemporal_load(p + (c < nch ? c : nch - 1));
    const uint64_t s = seg0 + uint64_t(k) * 16;
    i0[k] = META ? init[s < n ? s : n - 1] : 0u;
  }
#pragma unroll
  for (int k = 0; k < S; ++k) finish<META>(chunk_sum(v[k]), i0[k], out, seg0 + uint64_t(k) * 16, n, lane);
}

template <int S, bool META>
__global__ __launch_bounds__(kBlock) void k_stride(const u32x4* __restrict__ p, const uint32_t* __restrict__ init,
                                                   uint16_t* __restrict__ out, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = uint64_t(gridDim.x) * (kBlock / 64);
  const uint64_t nch = n * 4;
  for (uint64_t wave = (uint64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6; wave * 16 * S < n; wave += waves) {
    const uint64_t seg0 = wave * 16 * S + (lane >> 2);
    u32x4 v[S];
    uint32_t i0[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const uint64_t c = (seg0 + uint64_t(k) * 16) * 4 + (lane & 3);
      v[k] = __builtin_nontemporal_load(p + (c < nch ? c : nch - 1));
      const uint64_t s = seg0 + uint64_t(k) * 16;
      i0[k] = META ? init[s < n ? s : n - 1] : 0u;
    }
#pragma unroll
    for (int k = 0; k < S; ++k) finish<META>(chunk_sum(v[k]), i0[k], out, seg0 + uint64_t(k) * 16, n, lane);
  }
}

template <int S, bool META>
__global__ __launch_bounds__(kBlock) void k_stride_pf(const u32x4* __restrict__ p, const uint32_t* __restrict__ init,
                                                      uint16_t* __restrict__ out, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = uint64_t(gridDim.x) * (kBlock / 64);
  const uint64_t nch = n * 4;
  uint64_t wave = (uint64_t(blockIdx.x) * kBlock + threadIdx.x) >> 6;
  u32x4 v[S];
  uint32_t i0[S];
  auto load = [&](uint64_t w) {
    const uint64_t seg0 = w * 16 * S + (lane >> 2);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const uint64_t c = (seg0 + uint64_t(k) * 16) * 4 + (lane & 3);
      v[k] = __builtin_nontemporal_load(p + (c < nch ? c : nch - 1));
      const uint64_t s = seg0 + uint64_t(k) * 16;
      i0[k] = META ? init[s < n ? s : n - 1] : 0u;
    }
  };
  if (wave * 16 * S >= n) return;
  load(wave);
  for (;;) {
    uint32_t acc[S], ii[S];
#pragma unroll
    for (int k = 0; k < S; ++k) {
      acc[k] = chunk_sum(v[k]);
      ii[k] = i0[k];
    }
    const uint64_t cur = wave;
    wave += waves;
    const bool more = wave * 16 * S < n;
    if (more) load(wave);
    const uint64_t seg0 = cur * 16 * S + (lane >> 2);
#pragma unroll
    for (int k = 0; k < S; ++k) finish<META>(acc[k], ii[k], out, seg0 + uint64_t(k) * 16, n, lane);
    if (!more) break;
  }
}

// Layout family: a wave's tile is 64 lanes x 16 B x U; lane groups of G lanes
// each walk a contiguous G*16*U-byte region of it, instruction u reading G*16
// bytes at region + u*G*16 (G = 64: the wave-contiguous dense layout; G = 16,
// U = 8: the north-star kernel's lane-group walk).  Every 4 consecutive lanes
// of an instruction cover one 64-byte segment.  REMAP: XCD-aware block order
// (consecutive tiles on one XCD), as the engine's block_order.
template <int G, int U, bool META, bool REMAP>
__global__ __launch_bounds__(kBlock) void k_layout(const u32x4* __restrict__ p, const uint32_t* __restrict__ init,
                                                   uint16_t* __restrict__ out, uint64_t n) {
  const uint32_t lane = threadIdx.x & 63, g = lane / G, l = lane % G;
  uint32_t blk = blockIdx.x;
  if (REMAP && (gridDim.x & 7u) == 0) blk = (blk & 7u) * (gridDim.x >> 3) + (blk >> 3);
  const uint64_t wave = (uint64_t(blk) * kBlock + threadIdx.x) >> 6;
  const uint64_t nch = n * 4;
  const uint64_t c0 = wave * 64 * U + uint64_t(g) * G * U + l;  // 16-byte chunk index of instruction 0
  u32x4 v[U];
  uint32_t i0[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t c = c0 + uint64_t(u) * G;
    v[u] = __builtin_nontemporal_load(p + (c < nch ? c : nch - 1));
    const uint64_t s = c >> 2;
    i0[u] = META ? init[s < n ? s : n - 1] : 0u;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) finish<META>(chunk_sum(v[u]), i0[u], out, (c0 + uint64_t(u) * G) >> 2, n, lane);
}

// Load policy study (layout G = 64, U = 4): POL 0 all non-temporal, 1 all
// default (cache-allocating), 2 instruction 0 default and the rest NT.  RUN:
// XCD runs of 2^RUN blocks as the engine's block_order (0: hardware order).
template <int POL, int RUN, bool META>
__global__ __launch_bounds__(kBlock) void k_policy(const u32x4* __restrict__ p, const uint32_t* __restrict__ init,
                                                   uint16_t* __restrict__ out, uint64_t n) {
  constexpr int U = 4;
  extern __shared__ uint32_t lds_cap[];
  const uint32_t lane = threadIdx.x & 63;
  if (n == 0) lds_cap[threadIdx.x] = 0;  // keeps the dynamic LDS (an occupancy cap) referenced
  uint32_t blk = blockIdx.x;
  const uint32_t nblk = gridDim.x;
  if (RUN && nblk >= 16) {
    const uint32_t fl = 31u - uint32_t(__builtin_clz(nblk >> 3));
    const uint32_t lc = fl < uint32_t(RUN) ? fl : uint32_t(RUN);
    const uint32_t full = (nblk >> (lc + 3)) << (lc + 3);
    if (blk < full) {
      const uint32_t k = blk >> 3, x = blk & 7u;
      blk = ((k >> lc) << (lc + 3)) + (x << lc) + (k & ((1u << lc) - 1u));
    }
  }
  const uint64_t wave = (uint64_t(blk) * kBlock + threadIdx.x) >> 6;
  const uint64_t nch = n * 4;
  const uint64_t c0 = wave * 64 * U + lane;
  u32x4 v[U];
  uint32_t i0[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t c = c0 + uint64_t(u) * 64;
    const u32x4* q = p + (c < nch ? c : nch - 1);
    v[u] = (POL == 1 || (POL == 2 && u == 0)) ? *q : __builtin_nontemporal_load(q);
    const uint64_t s = c >> 2;
    i0[u] = META ? init[s < n ? s : n - 1] : 0u;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) finish<META>(chunk_sum(v[u]), i0[u], out, (c0 + uint64_t(u) * 64) >> 2, n, lane);
}

// Consolidated metadata: one 256-byte init load per wave (lane L: segment L
// of the wave's 64), distributed to the 4 lanes of each segment by lane
// shuffles, and the 64 results gathered into lane L for ONE 128-byte store
// per wave (instead of 4 init loads of 64 B and 4 stores of 32 B).
template <int RUN, int OUTW>
__global__ __launch_bounds__(kBlock) void k_meta2(const u32x4* __restrict__ p, const uint32_t* __restrict__ init,
                                                  uint16_t* __restrict__ out, uint64_t n) {
  constexpr int U = 4;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t blk = blockIdx.x;
  const uint32_t nblk = gridDim.x;
  if (RUN && nblk >= 16) {
    const uint32_t fl = 31u - uint32_t(__builtin_clz(nblk >> 3));
    const uint32_t lc = fl < uint32_t(RUN) ? fl : uint32_t(RUN);
    const uint32_t full = (nblk >> (lc + 3)) << (lc + 3);
    if (blk < full) {
      const uint32_t k = blk >> 3, x = blk & 7u;
      blk = ((k >> lc) << (lc + 3)) + (x << lc) + (k & ((1u << lc) - 1u));
    }
  }
  const uint64_t wave = (uint64_t(blk) * kBlock + threadIdx.x) >> 6;
  const uint64_t nch = n * 4;
  const uint64_t c0 = wave * 64 * U + lane;
  const uint64_t myseg = wave * 64 + lane;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint64_t c = c0 + uint64_t(u) * 64;
    v[u] = __builtin_nontemporal_load(p + (c < nch ? c : nch - 1));
  }
  const uint32_t iall = init[myseg < n ? myseg : n - 1];
  uint32_t mine = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t s = reduce4(chunk_sum(v[u]));      // lanes 4k..4k+3: segment u*16 + k
    const uint32_t g = __shfl(s, int((lane & 15) * 4));  // lane L: segment u*16 + L%16
    if ((lane >> 4) == uint32_t(u)) mine = g;
  }
  const uint32_t sum = mine + iall;
  if (OUTW == 2) {
    if (myseg < n) out[myseg] = uint16_t(sum);
  } else {  // pairs of u16 in one u32 from the even lanes (32 x 4 B)
    const uint32_t hi = __shfl_down(sum, 1);
    if ((lane & 1) == 0 && myseg + 1 < n)
      reinterpret_cast<uint32_t*>(out)[myseg >> 1] = (sum & 0xFFFFu) | (hi << 16);
    else if ((lane & 1) == 0 && myseg < n)
      out[myseg] = uint16_t(sum);
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

typedef void (*KFn)(const u32x4*, const uint32_t*, uint16_t*, uint64_t);

struct Variant {
  const char* name;
  KFn fn;
  int segs_per_wave;  // 16 * S
  uint32_t grid_cap;  // 0: one wave per tile (oneshot)
  bool meta;
  uint32_t lds = 0;   // dynamic LDS bytes per block: caps blocks per CU (160 KiB of LDS per CU)
};

static float time_variant(const Variant& v, u32x4** bufs, uint32_t** inits, uint16_t* out, uint64_t n,
                          hipEvent_t a, hipEvent_t b) {
  const uint64_t waves = (n + v.segs_per_wave - 1) / v.segs_per_wave;
  uint64_t blocks = (waves + kBlock / 64 - 1) / (kBlock / 64);
  if (v.grid_cap && blocks > v.grid_cap) blocks = v.grid_cap;
  const int reps = 30;
  for (int i = 0; i < 12; ++i)
    hipLaunchKernelGGL(v.fn, dim3(uint32_t(blocks)), dim3(kBlock), v.lds, nullptr, bufs[i % kCopies], inits[i % kCopies],
                       out, n);
  CK(hipDeviceSynchronize());
  float ts[5];
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a, nullptr));
    for (int i = 0; i < reps; ++i)
      hipLaunchKernelGGL(v.fn, dim3(uint32_t(blocks)), dim3(kBlock), v.lds, nullptr, bufs[i % kCopies],
                         inits[i % kCopies], out, n);
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ts[r] = ms * 1e3f / reps;
  }
  for (int i = 0; i < 5; ++i)  // median of 5
    for (int j = i + 1; j < 5; ++j)
      if (ts[j] < ts[i]) {
        const float t = ts[i];
        ts[i] = ts[j];
        ts[j] = t;
      }
  return ts[2];
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 20;
  const uint64_t n = uint64_t(1) << lg;
  const uint64_t nbytes = n * 64;
  u32x4* bufs[kCopies];
  uint32_t* inits[kCopies];
  uint16_t* out;
  for (int c = 0; c < kCopies; ++c) {
    CK(hipMalloc(&bufs[c], nbytes));
    CK(hipMemset(bufs[c], 0x5A + c, nbytes));
    CK(hipMalloc(&inits[c], n * 4));
    CK(hipMemset(inits[c], c, n * 4));
  }
  CK(hipMalloc(&out, n * 2));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const Variant vs[] = {
      // structure (study "dense")
      {"oneshot4", k_oneshot<4, true>, 64, 0, true},
      {"oneshot4_nometa", k_oneshot<4, false>, 64, 0, false},
      {"oneshot8", k_oneshot<8, true>, 128, 0, true},
      {"oneshot16", k_oneshot<16, true>, 256, 0, true},
      {"stride4_g2048", k_stride<4, true>, 64, 2048, true},
      {"stride4_g4096", k_stride<4, true>, 64, 4096, true},
      {"stride4_g8192", k_stride<4, true>, 64, 8192, true},
      {"stride4_g4096_nometa", k_stride<4, false>, 64, 4096, false},
      {"stridepf4_g2048", k_stride_pf<4, true>, 64, 2048, true},
      {"stridepf4_g4096", k_stride_pf<4, true>, 64, 4096, true},
      {"stridepf2_g4096", k_stride_pf<2, true>, 32, 4096, true},
      {"stridepf8_g2048", k_stride_pf<8, true>, 128, 2048, true},
      {"stridepf4_g4096_nometa", k_stride_pf<4, false>, 64, 4096, false},
      // tile layout (study "dense2"; r = eighths remap)
      {"L64u4r", k_layout<64, 4, true, true>, 64, 0, true},
      {"L16u4", k_layout<16, 4, true, false>, 64, 0, true},
      {"L16u4r", k_layout<16, 4, true, true>, 64, 0, true},
      {"L16u8", k_layout<16, 8, true, false>, 128, 0, true},
      {"L16u8r", k_layout<16, 8, true, true>, 128, 0, true},
      {"L4u4r", k_layout<4, 4, true, true>, 64, 0, true},
      {"L4u8", k_layout<4, 8, true, false>, 128, 0, true},
      {"L4u8r", k_layout<4, 8, true, true>, 128, 0, true},
      {"L8u8r", k_layout<8, 8, true, true>, 128, 0, true},
      {"L64u4r_nometa", k_layout<64, 4, false, true>, 64, 0, false},
      {"L16u8r_nometa", k_layout<16, 8, false, true>, 128, 0, false},
      {"L4u8r_nometa", k_layout<4, 8, false, true>, 128, 0, false},
      // load policy and XCD runs (study "dense3")
      {"nt_hw", k_policy<0, 0, true>, 64, 0, true},
      {"nt_run10", k_policy<0, 10, true>, 64, 0, true},
      {"dflt_hw", k_policy<1, 0, true>, 64, 0, true},
      {"dflt_run10", k_policy<1, 10, true>, 64, 0, true},
      {"mix_hw", k_policy<2, 0, true>, 64, 0, true},
      {"mix_run10", k_policy<2, 10, true>, 64, 0, true},
      {"nt_hw_nometa", k_policy<0, 0, false>, 64, 0, false},
      {"nt_run10_nometa", k_policy<0, 10, false>, 64, 0, false},
      {"dflt_hw_nometa", k_policy<1, 0, false>, 64, 0, false},
      {"dflt_run10_nometa", k_policy<1, 10, false>, 64, 0, false},
      {"mix_run10_nometa", k_policy<2, 10, false>, 64, 0, false},
      // occupancy cap (study "dense4")
      {"nt_run10_lds20k", k_policy<0, 10, true>, 64, 0, true, 20 << 10},
      {"nt_run10_lds40k", k_policy<0, 10, true>, 64, 0, true, 40 << 10},
      {"nt_run10_lds54k", k_policy<0, 10, true>, 64, 0, true, 54 << 10},
      {"nt_run10_lds80k", k_policy<0, 10, true>, 64, 0, true, 80 << 10},
      {"nt_run10_nometa_lds20k", k_policy<0, 10, false>, 64, 0, false, 20 << 10},
      {"nt_run10_nometa_lds40k", k_policy<0, 10, false>, 64, 0, false, 40 << 10},
      {"nt_run10_nometa_lds54k", k_policy<0, 10, false>, 64, 0, false, 54 << 10},
      {"nt_run10_nometa_lds80k", k_policy<0, 10, false>, 64, 0, false, 80 << 10},
      // consolidated metadata (study "dense5")
      {"meta2_run10", k_meta2<10, 2>, 64, 0, true, 0},
      {"meta2_run10_w4", k_meta2<10, 4>, 64, 0, true, 0},
      {"meta2_hw", k_meta2<0, 2>, 64, 0, true, 0},
      {"meta2_run10_lds20k", k_meta2<10, 2>, 64, 0, true, 20 << 10},
  };





  const char* only = argc > 2 ? argv[2] : nullptr;  // run the variants whose name contains this
  for (int round = 0; round < 2; ++round)
    for (const Variant& v : vs) {
      if (only && !strstr(v.name, only)) continue;
      const float us = time_variant(v, bufs, inits, out, n, a, b);
      if (round == 0) continue;  // first pass: clocks settle
      const double meta = v.meta ? double(n) * 6 : 0.0;
      printf("{\"segments\": %llu, \"variant\": \"%s\", \"us\": %.2f, \"frac_seg_bytes\": %.4f, "
             "\"frac_all_bytes\": %.4f}\n",
             (unsigned long long)n, v.name, us, double(nbytes) / (us * 1e-6) / 8e12,
             (double(nbytes) + meta) / (us * 1e-6) / 8e12);
      fflush(stdout);
    }
  return 0;
}
