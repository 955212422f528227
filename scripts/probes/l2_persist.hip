// Probe: does a buffer stay in the XCD L2s across dependent kernel launches?
// Each workgroup (1 per CU, blockIdx -> XCD round-robin, so the slice -> XCD mapping is the same
// every launch) streams a fixed slice of the buffer; per-launch time from HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void stream_kernel(const float4* __restrict__ buf, long n4,
                                                     float* __restrict__ out) {
  const long per = n4 / gridDim.x;
  const float4* p = buf + per * blockIdx.x;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (long i = threadIdx.x; i < per; i += 256) {
    const float4 v = p[i];
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 12345.678f) out[blockIdx.x] = s;  // keep the loads alive
}

int main() {
  float* out;
  hipMalloc(&out, 4096 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (long mb : {4L, 8L, 16L, 24L, 32L, 48L, 64L, 128L, 512L}) {
    const long bytes = mb << 20;
    float4* buf;
    hipMalloc(&buf, bytes);
    hipMemset(buf, 0, bytes);
    for (int grid : {256, 1024}) {
      for (int w = 0; w < 3; ++w) stream_kernel<<<grid, 256>>>(buf, bytes / 16, out);
      hipDeviceSynchronize();
      const int reps = 50;
      hipEventRecord(e0);
      for (int r = 0; r < reps; ++r) stream_kernel<<<grid, 256>>>(buf, bytes / 16, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = 1000.0 * ms / reps;
      printf("%4ld MB grid %4d: %8.2f us/launch  %6.2f TB/s\n", mb, grid, us, bytes / (us * 1e-6) / 1e12);
    }
    hipFree(buf);
  }
  return 0;
}
