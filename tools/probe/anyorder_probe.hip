// anyorder_probe.hip — dev tool: does a launch with hipExtAnyOrderLaunch on
// gfx950 start before the previous launch in the same stream has drained?
// Two independent streaming reads (200 MB and 140 MB, like a stack tick's
// receive VERIFY and transmit wrap), launched in turn on one stream, timed
// with events around 20 pairs; the second launch plain vs any-order.  Also
// checks the ordering a caller relies on: a device write launched (plain)
// before the pair is seen by both kernels.
//   hipcc --offload-arch=gfx950 -O3 anyorder_probe.hip -o anyorder_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ p, uint64_t n, const uint32_t* flag,
                                              uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const uint64_t step = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += step) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[1] = *flag;  // what the earlier plain write left
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_set(uint32_t* flag, uint32_t v) { *flag = v; }

int main() {
  const uint64_t na = 200ull << 20, nb = 140ull << 20;
  u32x4 *a, *b;
  uint32_t *flag, *oa, *ob;
  CK(hipMalloc(&a, na));
  CK(hipMalloc(&b, nb));
  CK(hipMalloc(&flag, 4));
  CK(hipMalloc(&oa, 8));
  CK(hipMalloc(&ob, 8));
  CK(hipMemset(a, 1, na));
  CK(hipMemset(b, 2, nb));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(2048), blk(256);
  for (int variant = 0; variant < 3; ++variant) {
    for (int round = 0; round < 4; ++round) {
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < 20; ++i) {
        hipLaunchKernelGGL(k_set, dim3(1), dim3(1), 0, st, flag, uint32_t(round * 100 + i + 1));
        if (variant == 2) {  // one kernel only: the read of a (for the sum of the parts)
          hipLaunchKernelGGL(k_read, grid, blk, 0, st, a, na / 16, flag, oa);
          continue;
        }
        hipLaunchKernelGGL(k_read, grid, blk, 0, st, a, na / 16, flag, oa);
        hipExtLaunchKernelGGL(k_read, grid, blk, 0, st, nullptr, nullptr, variant == 1 ? hipExtAnyOrderLaunch : 0,
                              static_cast<const u32x4*>(b), nb / 16, static_cast<const uint32_t*>(flag), ob);
      }
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      uint32_t ha[2] = {0, 0}, hb[2] = {0, 0};
      CK(hipMemcpy(ha, oa, 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hb, ob, 8, hipMemcpyDeviceToHost));
      const uint32_t want = uint32_t(round * 100 + 20);
      printf("{\"variant\": \"%s\", \"round\": %d, \"us_per_pair\": %.2f, \"flag_seen_a\": %u, \"flag_seen_b\": %u, "
             "\"want\": %u}\n",
             variant == 0 ? "plain" : variant == 1 ? "second_any_order" : "first_only", round, ms * 1000.0f / 20.0f,
             ha[1], variant == 2 ? want : hb[1], want);
    }
  }
  return 0;
}
