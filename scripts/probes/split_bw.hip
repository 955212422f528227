// Probe: what bounds the operand split (gemm.hip split_frag32_kernel, row-major source)?
// 64 MB fp32 [32768][512] -> 64 MB fragment-major hi/lo f16 image.  Times, with HIP events:
//   copy4   : float4 copy of the same bytes (the streaming floor)
//   split   : the production indexing (one 8-element group per thread)
//   splitN  : N groups per thread, all loads issued before the conversions and stores
//   split_nt: as split, nontemporal stores
// each alone (back to back) and right behind a kernel that rewrites the source (dirty lines).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split8(const float* v, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = (_Float16)v[j];
    hi[j] = h;
    lo[j] = (_Float16)((v[j] - (float)h) * 2048.0f);
  }
}

__global__ __launch_bounds__(256) void fill(float* p, long n, float s) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n / 4; i += (long)gridDim.x * 256)
    reinterpret_cast<float4*>(p)[i] = float4{s, s * 0.5f, s * 0.25f, -s};
}

__global__ __launch_bounds__(256) void copy4(const float4* __restrict__ s, float4* __restrict__ d, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) d[i] = s[i];
}

// production mapping (row-major source): thread -> (tile, quad, row, group), NG groups per thread
template <int NG, bool NT>
__global__ __launch_bounds__(256) void split_k(const float* __restrict__ src, long rs, int ntile, int nkc,
                                               _Float16* __restrict__ dst, float sc) {
  const int G8 = nkc * 2;
  const long total = (long)ntile * 32 * G8;
  const long stride = (long)gridDim.x * 256;
  for (long base = blockIdx.x * 256L + threadIdx.x; base < total; base += stride * NG) {
    float v[NG][8];
    long rr_[NG];
    int g_[NG];
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const long idx = base + n * stride;
      const int gq = (int)(idx & 3);
      const long rest = idx >> 2;
      const int rr = (int)(rest & 31);
      const long tq = rest >> 5;
      const unsigned q4 = (unsigned)(G8 >> 2);
      const long t = (long)((unsigned)tq / q4);
      const int quad = (int)(tq - t * (long)q4);
      rr_[n] = t * 32 + rr;
      g_[n] = quad * 4 + gq;
      if (idx < total) {
        const float4* q = reinterpret_cast<const float4*>(src + rr_[n] * rs + 8 * g_[n]);
        const float4 a = q[0], b = q[1];
        v[n][0] = a.x; v[n][1] = a.y; v[n][2] = a.z; v[n][3] = a.w;
        v[n][4] = b.x; v[n][5] = b.y; v[n][6] = b.z; v[n][7] = b.w;
      }
    }
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const long idx = base + n * stride;
      if (idx >= total) break;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[n][e] *= sc;
      f16x8 hi, lo;
      split8(v[n], hi, lo);
      const long r = rr_[n];
      const int g8 = g_[n];
      const long blk = ((r >> 5) * nkc + (g8 >> 1)) * 2;
      const int lane = (int)(r & 31) + 32 * (g8 & 1);
      if (NT) {
        __builtin_nontemporal_store(hi, reinterpret_cast<f16x8*>(dst + blk * 512 + lane * 8));
        __builtin_nontemporal_store(lo, reinterpret_cast<f16x8*>(dst + (blk + 1) * 512 + lane * 8));
      } else {
        *reinterpret_cast<f16x8*>(dst + blk * 512 + lane * 8) = hi;
        *reinterpret_cast<f16x8*>(dst + (blk + 1) * 512 + lane * 8) = lo;
      }
    }
  }
}

// tile-local mapping: a workgroup owns a 32-row tile x 64 k (4 chunks = 8 KB of output, contiguous);
// thread (row, group of 8): reads 32 B, the 8 threads of a row read 256 B contiguous
template <int NG>
__global__ __launch_bounds__(256) void split_tile(const float* __restrict__ src, long rs, int ntile, int nkc,
                                                  _Float16* __restrict__ dst, float sc) {
  const int tid = threadIdx.x;
  const int rr = tid >> 3, g = tid & 7;
  const int cpb = nkc / 4;  // 64-k column blocks per tile
  const long units = (long)ntile * cpb;
  for (long u0 = blockIdx.x; u0 < units; u0 += (long)gridDim.x * NG) {
    float v[NG][8];
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const long u = u0 + (long)n * gridDim.x;
      if (u < units) {
        const long t = u / cpb;
        const int cb = (int)(u - t * cpb);
        const float4* q = reinterpret_cast<const float4*>(src + (t * 32 + rr) * rs + cb * 64 + g * 8);
        const float4 a = q[0], b = q[1];
        v[n][0] = a.x; v[n][1] = a.y; v[n][2] = a.z; v[n][3] = a.w;
        v[n][4] = b.x; v[n][5] = b.y; v[n][6] = b.z; v[n][7] = b.w;
      }
    }
#pragma unroll
    for (int n = 0; n < NG; ++n) {
      const long u = u0 + (long)n * gridDim.x;
      if (u >= units) break;
      const long t = u / cpb;
      const int cb = (int)(u - t * cpb);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[n][e] *= sc;
      f16x8 hi, lo;
      split8(v[n], hi, lo);
      const int g8 = cb * 8 + g;
      const long blk = (t * nkc + (g8 >> 1)) * 2;
      const int lane = rr + 32 * (g8 & 1);
      *reinterpret_cast<f16x8*>(dst + blk * 512 + lane * 8) = hi;
      *reinterpret_cast<f16x8*>(dst + (blk + 1) * 512 + lane * 8) = lo;
    }
  }
}

int main() {
  const int M = 32768, K = 512, ntile = M / 32, nkc = K / 16;
  const long n = (long)M * K;
  float* src;
  _Float16* dst;
  float* other;
  hipMalloc(&src, n * 4);
  hipMalloc(&dst, n * 4);
  hipMalloc(&other, n * 4);
  fill<<<4096, 256>>>(src, n, 1.f);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const long total = (long)ntile * 32 * nkc * 2;
  auto launch = [&](int which, bool dirty) -> float {
    const int reps = 20;
    float sum = 0.f;
    for (int r = 0; r < reps + 2; ++r) {
      if (dirty) fill<<<4096, 256>>>(src, n, 1.f + r);
      else fill<<<4096, 256>>>(other, n, 1.f + r);  // same boundary, clean source
      hipEventRecord(e0);
      switch (which) {
        case 0: copy4<<<8192, 256>>>((const float4*)src, (float4*)dst, n / 4); break;
        case 1: split_k<1, false><<<(int)std::min<long>((total + 255) / 256, 8192), 256>>>(src, K, ntile, nkc, dst, 1.f); break;
        case 2: split_k<2, false><<<4096, 256>>>(src, K, ntile, nkc, dst, 1.f); break;
        case 3: split_k<4, false><<<2048, 256>>>(src, K, ntile, nkc, dst, 1.f); break;
        case 4: split_k<1, true><<<(int)std::min<long>((total + 255) / 256, 8192), 256>>>(src, K, ntile, nkc, dst, 1.f); break;
        case 5: split_tile<1><<<8192, 256>>>(src, K, ntile, nkc, dst, 1.f); break;
        case 6: split_tile<2><<<4096, 256>>>(src, K, ntile, nkc, dst, 1.f); break;
        case 7: split_tile<4><<<2048, 256>>>(src, K, ntile, nkc, dst, 1.f); break;
        case 8: copy4<<<2048, 256>>>((const float4*)src, (float4*)dst, n / 4); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (r >= 2) sum += ms;
    }
    return sum / reps * 1000.f;
  };
  const char* names[] = {"copy4 8192wg", "split (prod)", "split NG2", "split NG4", "split nt", "tile NG1", "tile NG2",
                         "tile NG4", "copy4 2048wg"};
  for (int round = 0; round < 2; ++round)
    for (int w = 0; w < 9; ++w) {
      const float clean = launch(w, false), dirty = launch(w, true);
      printf("%-14s clean %7.1f us (%5.2f TB/s)  dirty-source %7.1f us (%5.2f TB/s)\n", names[w], clean,
             2.0 * n * 4 / clean / 1e6, dirty, 2.0 * n * 4 / dirty / 1e6);
    }
  hipError_t err = hipGetLastError();
  printf("status %s\n", hipGetErrorString(err));
  return 0;
}
