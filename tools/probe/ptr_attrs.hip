#include <hip/hip_runtime.h>
#include <cstdio>
int main() {
  for (unsigned fl : {hipDeviceMallocUncached, hipDeviceMallocFinegrained, hipDeviceMallocDefault}) {
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, 4096, fl) != hipSuccess) { printf("{\"flag\": %u, \"alloc\": false}\n", fl); continue; }
    hipPointerAttribute_t a{};
    hipError_t e = hipPointerGetAttributes(&a, p);
    printf("{\"flag\": %u, \"rc\": %d, \"type\": %d, \"hostPointer_eq\": %d, \"hostPointer_null\": %d, \"devicePointer_eq\": %d, \"isManaged\": %d, \"allocationFlags\": %u}\n",
           fl, int(e), int(a.type), a.hostPointer == p, a.hostPointer == nullptr, a.devicePointer == p, int(a.isManaged), a.allocationFlags);
    (void)hipFree(p);
  }
  void* q = nullptr; (void)hipMalloc(&q, 4096);
  hipPointerAttribute_t a{}; (void)hipPointerGetAttributes(&a, q);
  printf("{\"hipMalloc\": 1, \"type\": %d, \"hostPointer_eq\": %d, \"hostPointer_null\": %d}\n", int(a.type), a.hostPointer == q, a.hostPointer == nullptr);
  return 0;
}
