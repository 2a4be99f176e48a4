// Dev probe (round 5): why does the fixed-stride k_checksum stream 1 M x 770
// / 1500 B segments at 91-94 % of 8 TB/s while 4 KiB-window streams (k_span,
// pattern_probe) stop at 84-87 %?  One-shot waves, every byte summed, one
// store per 16 lanes, non-temporal buffer loads; the same bytes read three ways:
//   seg16:  k_checksum's shape — four 16-lane groups per wave, group g reads
//           segment 4 w + g: its loads u = 0..U-1 at 256 u (a 256-byte piece
//           per group per instruction, four segments per instruction);
//   flat:   wave w reads the same four segments' bytes as one contiguous
//           range, 1 KiB per instruction (lane l: 1024 u + 16 l);
//   flat4k: as flat, but each wave's range is rounded to whole 4 KiB windows
//           of the buffer (pattern_probe's one-shot shape).
// seg16 on 1500-byte segments: 6 loads per lane (U = 6), flat: ceil(6000 /
// 1024) = 6; 770-byte segments: U = 4 / 4.  One 4-byte store per 16 lanes.  One JSON line per (shape, L):
// us per launch (HIP events around 20 launches, median of 5), fraction of
// 8 TB/s.  Build: hipcc --offload-arch=gfx950 -O3 footprint_probe.hip -o footprint_probe
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

template <int U>
__device__ __forceinline__ uint32_t sum_loads(const uint8_t* base, uint32_t len, uint32_t voff, uint32_t step) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, int(len), 0x00020000);
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, int(u * step), 2));
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  return acc;
}

// the same loads as global_load ... nt (k_checksum's load16<true>), the
// range's end clamped instead of the buffer resource's range check
template <int U>
__device__ __forceinline__ uint32_t sum_loads_g(const uint8_t* base, uint32_t len, uint32_t voff, uint32_t step) {
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t o = voff + uint32_t(u) * step;
    v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + (o < len ? o : 0u)));
    if (o >= len) v[u] = u32x4{0u, 0u, 0u, 0u};
  }
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  return acc;
}

// k_checksum's mode 3 (range_sums_line_primed), sums only: the group's chunk
// grid anchored on the 128-byte line holding the start, the head and tail
// chunks loaded first with the default policy by lanes 0 and 1, the slots
// non-temporal (clamped to the tail chunk), head / tail masked out of them
template <int U, bool BUF>
__device__ __forceinline__ uint32_t line_primed(const uint8_t* base, uint64_t s, uint64_t e, uint32_t lane) {
  const uint64_t a0 = s & ~uint64_t(127);
  const uint32_t nch = uint32_t((e - a0 + 15) >> 4), cs = uint32_t(s - a0) >> 4, lastc = nch - 1;
  const u32x4* p = reinterpret_cast<const u32x4*>(base + a0);
  const u32x4 bnd = p[lane == 1 ? lastc : cs];
  u32x4 v[U];
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4*>(p), 0, int(nch * 16u), 0x00020000);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t cc = lane + 16u * u;
    if (BUF)
      v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, cc * 16u, 0, 2));
    else
      v[u] = __builtin_nontemporal_load(p + (cc < lastc ? cc : lastc));
  }
  uint32_t acc = lane < 2 ? bnd.x + bnd.y + bnd.z + bnd.w : 0u;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t cc = lane + 16u * u;
    const uint32_t keep = (cc > cs && cc < lastc) ? ~0u : 0u;
    acc += (v[u].x + v[u].y + v[u].z + v[u].w) & keep;
  }
  return acc;
}

// SHAPE 0 seg16, 1 flat, 2 flat4k, 3 flat (global loads), 4 flat4k (global
// loads), 5 seg16 line-primed (global), 6 seg16 line-primed (buffer slots),
// 7 quarters: the wave's flat range (four segments' bytes) cut in four
// quarters at 16-byte chunks, group g streaming quarter g at 256 B per
// instruction (buffer loads); 8 the same with the quarters cut at 128-byte
// lines and the range's start on a line; 9 / 10: 7 / 8 with global loads;
// 11: 10 with each group's first and last chunk loaded first with the
// default (L2-allocating) policy by its lanes 0 / 1 (mode 3's priming);
// 12: flat with global loads, primed the same way per wave
template <int SHAPE, int U>
__global__ __launch_bounds__(256) void k_probe(const uint8_t* __restrict__ buf, uint64_t n, uint32_t L,
                                               uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t w = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  uint32_t acc = 0;
  if (SHAPE == 0) {
    const uint64_t seg = w * 4 + (lane >> 4);
    if (seg < n) acc = sum_loads<U>(buf + seg * L, L, (lane & 15u) * 16u, 256u);
  } else if (SHAPE == 1) {
    const uint64_t s0 = w * 4 * L, e0 = std::min<uint64_t>(n * L, s0 + 4ull * L);
    if (s0 < e0) acc = sum_loads<U>(buf + s0, uint32_t(e0 - s0), lane * 16u, 1024u);
  } else if (SHAPE == 2) {
    const uint64_t per = uint64_t(U) * 1024, s0 = w * per, e0 = std::min<uint64_t>(n * L, s0 + per);
    if (s0 < e0) acc = sum_loads<U>(buf + s0, uint32_t(e0 - s0), lane * 16u, 1024u);
  } else if (SHAPE == 3) {
    const uint64_t s0 = w * 4 * L, e0 = std::min<uint64_t>(n * L, s0 + 4ull * L);
    if (s0 < e0) acc = sum_loads_g<U>(buf + s0, uint32_t(e0 - s0), lane * 16u, 1024u);
  } else if (SHAPE == 4) {
    const uint64_t per = uint64_t(U) * 1024, s0 = w * per, e0 = std::min<uint64_t>(n * L, s0 + per);
    if (s0 < e0) acc = sum_loads_g<U>(buf + s0, uint32_t(e0 - s0), lane * 16u, 1024u);
  } else if (SHAPE == 12) {
    const uint64_t s0 = w * 4 * L, e0 = std::min<uint64_t>(n * L, s0 + 4ull * L);
    if (s0 < e0) {
      const u32x4* pr = reinterpret_cast<const u32x4*>(buf + s0);
      const uint32_t last = uint32_t((e0 - s0 - 1) >> 4);
      const u32x4 bnd = pr[lane == 1 ? last : 0u];
      acc = sum_loads_g<U>(buf + s0, uint32_t(e0 - s0), lane * 16u, 1024u) + (lane < 2 ? bnd.x : 0u);
    }
  } else if (SHAPE == 5 || SHAPE == 6) {
    const uint64_t seg = w * 4 + (lane >> 4);
    if (seg < n) acc = line_primed<U, SHAPE == 6>(buf, seg * L, seg * L + L, lane & 15u);
  } else {
    const uint64_t s0r = w * 4 * L, e0 = std::min<uint64_t>(n * L, s0r + 4ull * L);
    const bool lines = SHAPE == 8 || SHAPE == 10 || SHAPE == 11;
    const uint64_t s0 = lines ? (s0r & ~uint64_t(127)) : (s0r & ~uint64_t(15));
    if (s0 < e0) {
      const uint64_t unit = lines ? 128 : 16;
      const uint64_t q = ((e0 - s0 + 4 * unit - 1) / (4 * unit)) * unit;  // quarter length
      const uint64_t g = lane >> 4, qs = s0 + g * q, qe = std::min<uint64_t>(e0, qs + q);
      if (SHAPE == 11 && qe > qs) {
        const u32x4* pr = reinterpret_cast<const u32x4*>(buf + qs);
        const uint32_t last = uint32_t((qe - qs - 1) >> 4);
        const u32x4 bnd = pr[(lane & 15u) == 1 ? last : 0u];
        acc = (lane & 15u) < 2 ? bnd.x : 0u;
      }
      if (SHAPE == 9 || SHAPE == 10 || SHAPE == 11)
        acc += sum_loads_g<U>(buf + qs, uint32_t(qe > qs ? qe - qs : 0), (lane & 15u) * 16u, 256u);
      else
        acc = sum_loads<U>(buf + qs, uint32_t(qe > qs ? qe - qs : 0), (lane & 15u) * 16u, 256u);
    }
  }
  // one store per 16 lanes (k_checksum writes 2 bytes per segment)
  if ((lane & 15u) == 0) out[(w * 4 + (lane >> 4)) & ((1u << 20) - 1)] = acc;
}

int main() {
  const uint64_t n = uint64_t(1) << 20;
  const uint64_t cap = n * 1500 + 8192;
  uint8_t* buf[2];
  uint32_t* out;
  for (auto& p : buf) {
    CK(hipMalloc(&p, cap));
    CK(hipMemset(p, 1, cap));
  }
  CK(hipMalloc(&out, (1u << 20) * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  using K = void (*)(const uint8_t*, uint64_t, uint32_t, uint32_t*);
  struct Run {
    const char* name;
    K k;
    uint32_t L;
    int shape, u;
  } runs[] = {{"seg16", k_probe<0, 6>, 1500, 0, 6}, {"flat", k_probe<1, 6>, 1500, 1, 6},
              {"flat4k", k_probe<2, 6>, 1500, 2, 6}, {"seg16", k_probe<0, 4>, 770, 0, 4},
              {"flat", k_probe<1, 4>, 770, 1, 4},    {"flat4k", k_probe<2, 4>, 770, 2, 4},
              {"flat4k_1win", k_probe<2, 4>, 1024, 2, 4},
              {"flat_global", k_probe<3, 6>, 1500, 3, 6}, {"flat4k_global", k_probe<4, 6>, 1500, 4, 6},
              {"flat_global", k_probe<3, 4>, 770, 3, 4},  {"flat4k_global", k_probe<4, 4>, 770, 4, 4},
              {"line_primed_global", k_probe<5, 7>, 1500, 5, 7}, {"line_primed_buffer", k_probe<6, 7>, 1500, 6, 7},
              {"line_primed_global", k_probe<5, 4>, 770, 5, 4},  {"line_primed_buffer", k_probe<6, 4>, 770, 6, 4},
              {"quarters", k_probe<7, 6>, 1500, 7, 6}, {"quarters_lines", k_probe<8, 7>, 1500, 8, 7},
              {"quarters", k_probe<7, 4>, 770, 7, 4},  {"quarters_lines", k_probe<8, 4>, 770, 8, 4},
              {"quarters_global", k_probe<9, 6>, 1500, 9, 6}, {"quarters_lines_global", k_probe<10, 7>, 1500, 10, 7},
              {"quarters_global", k_probe<9, 4>, 770, 9, 4},  {"quarters_lines_global", k_probe<10, 4>, 770, 10, 4},
              {"quarters_lines_global_primed", k_probe<11, 7>, 1500, 11, 7},
              {"quarters_lines_global_primed", k_probe<11, 4>, 770, 11, 4},
              {"flat_global_primed", k_probe<12, 6>, 1500, 12, 6}, {"flat_global_primed", k_probe<12, 4>, 770, 12, 4}};
  for (const Run& r : runs) {
    const uint64_t bytes = n * r.L;
    const uint64_t waves = (r.shape == 2 || r.shape == 4) ? (bytes + uint64_t(r.u) * 1024 - 1) / (uint64_t(r.u) * 1024) : (n + 3) / 4;
    const uint32_t grid = uint32_t((waves + 3) / 4);
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(r.k, dim3(grid), dim3(256), 0, 0, buf[i & 1], n, r.L, out);
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int round = 0; round < 5; ++round) {
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(r.k, dim3(grid), dim3(256), 0, 0, buf[i & 1], n, r.L, out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1000.f / 20.f);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[2];
    std::printf("{\"shape\": \"%s\", \"L\": %u, \"loads_per_lane\": %d, \"grid\": %u, \"us\": %.2f, \"frac\": %.4f}\n",
                r.name, r.L, r.u, grid, us, bytes / us / 1e3 / 8000.0);
    std::fflush(stdout);
  }
  return 0;
}
