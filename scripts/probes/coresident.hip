// Probe: how many workgroups that each need a whole CU's LDS (one per CU) are co-resident?
// Each workgroup arrives on a counter and spins (bounded, ~0.2 s) until `n` have arrived.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256, 1) void arrive_wait(unsigned* cnt, unsigned n, unsigned* ok) {
  extern __shared__ float lds[];
  lds[threadIdx.x] = 0.f;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n && spins < (1u << 20)) {
      __builtin_amdgcn_s_sleep(2);
      ++spins;
    }
    if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n)
      __hip_atomic_fetch_add(ok, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (lds[threadIdx.x ^ 1] != 0.f) cnt[1] = 1;
}

int main(int argc, char** argv) {
  size_t lds = argc > 1 ? (size_t)atol(argv[1]) : 100 * 1024;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int per = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)arrive_wait, 256, lds);
  printf("CUs %d, occupancy per CU %d at %zu B LDS\n", cus, per, lds);
  unsigned *cnt, *ok;
  hipMalloc(&cnt, 256);
  hipMalloc(&ok, 256);
  for (int n : {128, 192, 224, 240, 248, 252, 254, 255, 256}) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(cnt, 0, 256);
      hipMemset(ok, 0, 256);
      hipDeviceSynchronize();
      arrive_wait<<<n, 256, lds>>>(cnt, n, ok);
      hipDeviceSynchronize();
      unsigned h = 0;
      hipMemcpy(&h, ok, 4, hipMemcpyDeviceToHost);
      printf("grid %3d rep %d: %u of %d saw all arrive\n", n, rep, h, n);
    }
  }
  return 0;
}
