// patch_probe.hip — dev tool: what in-place checksum patching costs on
// MI355X, by store shape and cache policy.  Config 2 (64 Ki x 1500 B
// datagrams) read once per launch, 6 rotated copies (HBM, not the Infinity
// Cache); per datagram the group leader writes either nothing, the two 2-byte
// checksum fields (bytes 10 and 36, what ICS_MODE_PATCH does), or the 16- /
// 32- / 64-byte aligned blocks that contain them (whole-granule writes the
// memory side does not have to merge).  Policies: default (write-back: the
// lines stay dirty in the XCD's L2 until the end-of-kernel release writes them
// back), nt (streaming), sc1 (write-through: relaxed agent-scope atomic store /
// buffer store with aux sc1).  The written values are junk: only time matters.
//   hipcc --offload-arch=gfx950 -O3 patch_probe.hip -o patch_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kLps = 16;  // lanes per datagram
constexpr uint32_t kLen = 1500;
constexpr int kCopies = 6;

enum Policy { kDefault = 0, kNt = 1, kSc1 = 2 };

template <int POL>
__device__ __forceinline__ void st16(uint16_t* p, uint16_t v) {
  if (POL == kNt)
    __builtin_nontemporal_store(v, p);
  else if (POL == kSc1)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}

template <int POL>
__device__ __forceinline__ void st128(u32x4* p, u32x4 v) {
  if (POL == kNt) {
    __builtin_nontemporal_store(v, p);
  } else if (POL == kSc1) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, 0, 16, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, 0, 0, 16);  // aux 16 = sc1
  } else {
    *p = v;
  }
}

// STORE: 0 none, 2 two shorts, 16 / 32 / 64 aligned blocks
template <int STORE, int POL>
__global__ __launch_bounds__(256) void k_patch(uint8_t* __restrict__ d, uint64_t n, uint32_t* __restrict__ sink) {
  const uint64_t g = (uint64_t(blockIdx.x) * 256 + threadIdx.x) / kLps;
  const uint32_t lane = threadIdx.x % kLps;
  if (g >= n) return;
  const uint64_t s = g * kLen, a0 = s & ~uint64_t(15), e = s + kLen;
  const uint32_t nch = uint32_t((e - a0 + 15) >> 4);
  const u32x4* p = reinterpret_cast<const u32x4*>(d + a0);
  uint32_t acc = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint32_t c = lane + u * kLps;
    const u32x4 v = __builtin_nontemporal_load(p + (c < nch ? c : nch - 1));
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (lane == kLps - 1) {
    if (STORE == 2) {
      st16<POL>(reinterpret_cast<uint16_t*>(d + s + 10), uint16_t(acc));
      st16<POL>(reinterpret_cast<uint16_t*>(d + s + 36), uint16_t(acc >> 16));
    } else if (STORE >= 16) {
      const uint64_t f[2] = {s + 10, s + 36};
      uint64_t last = ~uint64_t(0);
      for (int k = 0; k < 2; ++k) {
        const uint64_t b = f[k] & ~uint64_t(STORE - 1);
        if (b == last) continue;  // both fields in one block: one write
        last = b;
        u32x4* q = reinterpret_cast<u32x4*>(d + b);
        for (int j = 0; j < STORE / 16; ++j) st128<POL>(q + j, u32x4{acc, acc + 1, acc + 2, acc + 3});
      }
    } else if (acc == 0x12345678u) {
      sink[0] = acc;
    }
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

template <int STORE, int POL = kDefault>
int run(uint8_t** bufs, uint32_t* sink, uint64_t n, hipEvent_t a, hipEvent_t b) {
  const uint32_t blocks = uint32_t((n * kLps + 255) / 256);
  const int reps = 60;
  float best = 1e30f;
  for (int round = 0; round < 5; ++round) {
    CK(hipEventRecord(a, nullptr));
    for (int r = 0; r < reps; ++r)
      hipLaunchKernelGGL((k_patch<STORE, POL>), dim3(blocks), dim3(256), 0, nullptr, bufs[r % kCopies], n, sink);
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  static const char* pol[] = {"default", "nt", "sc1"};
  printf("{\"store\": %d, \"policy\": \"%s\", \"us\": %.2f}\n", STORE, pol[POL], best * 1e3 / reps);
  return 0;
}

int main() {
  const uint64_t n = 1 << 16, bytes = n * kLen + 64;
  uint8_t* bufs[kCopies];
  uint32_t* sink = nullptr;
  for (int c = 0; c < kCopies; ++c) {
    CK(hipMalloc(&bufs[c], bytes));
    CK(hipMemset(bufs[c], c + 1, bytes));
  }
  CK(hipMalloc(&sink, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 10000; ++r)  // settle clocks
    hipLaunchKernelGGL((k_patch<0, kDefault>), dim3(4096), dim3(256), 0, nullptr, bufs[r % kCopies], n, sink);
  CK(hipDeviceSynchronize());
  int rc = 0;
  for (int pass = 0; pass < 2 && !rc; ++pass) {
    rc |= run<0>(bufs, sink, n, a, b);
    rc |= run<2>(bufs, sink, n, a, b);
    rc |= run<2, kNt>(bufs, sink, n, a, b);
    rc |= run<2, kSc1>(bufs, sink, n, a, b);
    rc |= run<16>(bufs, sink, n, a, b);
    rc |= run<16, kNt>(bufs, sink, n, a, b);
    rc |= run<16, kSc1>(bufs, sink, n, a, b);
    rc |= run<32>(bufs, sink, n, a, b);
    rc |= run<64>(bufs, sink, n, a, b);
    rc |= run<64, kSc1>(bufs, sink, n, a, b);
  }
  return rc;
}
