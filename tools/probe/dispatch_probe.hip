// dispatch_probe.hip — dev tool: what an "empty" launch costs on MI355X (every
// block reads one plan word and exits), by block size and by whether the word
// is read at all.  Question it answers: is the cost of a launch whose blocks
// find no work per workgroup, per wave, or the latency of the plan load?
//   hipcc --offload-arch=gfx950 -O3 dispatch_probe.hip -o dispatch_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int BLOCK, bool LOAD>
__global__ __launch_bounds__(BLOCK) void k_empty(const uint32_t* __restrict__ plan, uint32_t* __restrict__ out) {
  uint32_t w = 0;
  if (LOAD) w = plan[0];  // uniform: scalar load
  if (w != 0) out[blockIdx.x * BLOCK + threadIdx.x] = w;  // never taken (plan = 0)
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <int BLOCK, bool LOAD>
int run(const uint32_t* plan, uint32_t* out, uint64_t threads, hipEvent_t a, hipEvent_t b) {
  const uint32_t blocks = uint32_t(threads / BLOCK);
  const int reps = 20;
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k_empty<BLOCK, LOAD>), dim3(blocks), dim3(BLOCK), 0, nullptr, plan, out);
  CK(hipEventRecord(a, nullptr));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((k_empty<BLOCK, LOAD>), dim3(blocks), dim3(BLOCK), 0, nullptr, plan, out);
  CK(hipEventRecord(b, nullptr));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"block\": %d, \"load\": %d, \"blocks\": %u, \"waves\": %llu, \"us_per_launch\": %.2f, "
         "\"ns_per_block\": %.4f, \"ns_per_wave\": %.4f}\n",
         BLOCK, int(LOAD), blocks, (unsigned long long)(threads / 64), ms * 1e3 / reps,
         ms * 1e6 / reps / blocks, ms * 1e6 / reps / (threads / 64));
  return 0;
}

int main() {
  uint32_t *plan = nullptr, *out = nullptr;
  CK(hipMalloc(&plan, 256));
  CK(hipMemset(plan, 0, 256));
  CK(hipMalloc(&out, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint64_t threads = uint64_t(1) << 27;  // 2 M segments x 64 lanes (bimodal's last-bin launch)
  int rc = 0;
  for (int pass = 0; pass < 2 && !rc; ++pass) {
    rc |= run<256, true>(plan, out, threads, a, b);
    rc |= run<256, false>(plan, out, threads, a, b);
    rc |= run<512, true>(plan, out, threads, a, b);
    rc |= run<1024, true>(plan, out, threads, a, b);
    rc |= run<1024, false>(plan, out, threads, a, b);
    rc |= run<64, true>(plan, out, threads / 4, a, b);  // one wave per block, a quarter of the waves
  }
  return rc;
}
