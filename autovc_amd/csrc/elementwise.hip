// Bandwidth-bound kernels of the Generator: column reductions, BatchNorm statistics /
// normalisation / backward, the layout glue around the encoder bottleneck (concat, down- and
// up-sampling of the content codes), the reconstruction losses and the fused
// clip + Adam + EMA optimizer pass.  All of them stream time-major [T*B][C] rows with
// consecutive lanes on consecutive channels (coalesced), and every reduction is two-pass with
// a fixed summation order (deterministic, fp64 final combine).
#include <algorithm>
#include <cmath>

#include "kernels.h"
#include "elementwise.h"

namespace avc {
namespace {

inline int ew_blocks(long n, int per = 256) { return (int)std::max<long>(1, std::min<long>((n + per - 1) / per, 16384)); }

__device__ __forceinline__ float act_fwd(float a, int act) {
  if (act == AVC_ACT_RELU) return a < 0.f ? 0.f : a;  // NaN propagates, as torch.relu
  if (act == AVC_ACT_TANH) return tanhf(a);
  return a;
}
// derivative of act at pre-activation a
__device__ __forceinline__ float act_bwd(float a, int act) {
#pragma clang fp contract(off)
  if (act == AVC_ACT_RELU) return a > 0.f ? 1.f : 0.f;
  if (act == AVC_ACT_TANH) {
    const float t = tanhf(a);
    return 1.f - t * t;
  }
  return 1.f;
}

// The BatchNorm backward's per-element expressions, written once with contraction off so every
// pass that forms them (reduce, apply, the split-writing apply of round 4) gets the same bits
// whatever the compiler would fuse in each kernel:
//   x^ = (y - mu) * is,  dA = dout * act'(x^ g + b),  dy = g is (dA - k1 - x^ k2)  (train) | g is dA
__device__ __forceinline__ float bnb_xhat(float y, float mu, float is) {
#pragma clang fp contract(off)
  return (y - mu) * is;
}
__device__ __forceinline__ float bnb_da(float d, float xh, float g, float bt, int act) {
#pragma clang fp contract(off)
  return d * act_bwd(xh * g + bt, act);
}
__device__ __forceinline__ float bnb_dy(float dA, float xh, float g, float is, float k1, float k2, int training) {
#pragma clang fp contract(off)
  return training ? g * is * (dA - k1 - xh * k2) : g * is * dA;
}

// ---- column sums -------------------------------------------------------------------------
__global__ void colsum_partial_kernel(int M, int N, const float* __restrict__ X, long ld,
                                      int rows_per, float* __restrict__ part) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int m0 = blockIdx.y * rows_per, m1 = min(M, m0 + rows_per);
  float s = 0.f;
  for (int m = m0; m < m1; ++m) s += X[(long)m * ld + n];
  part[(long)blockIdx.y * N + n] = s;
}

// 64 columns per block, the 16 waves split the R partial rows; fp64 combine through LDS.
__global__ __launch_bounds__(1024) void colsum_final_kernel(int R, int N, const float* __restrict__ part,
                                                            float* __restrict__ out, int accumulate,
                                                            float* __restrict__ out2) {
  __shared__ double red[16][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + cl;
  double s = 0.0;
  if (n < N) {
    // four partial rows loaded ahead of their adds (same addition order: bit-identical sums)
    int r = grp;
    for (; r + 48 < R; r += 64) {
      const float a = part[(long)r * N + n], b = part[(long)(r + 16) * N + n];
      const float c = part[(long)(r + 32) * N + n], e = part[(long)(r + 48) * N + n];
      s += a; s += b; s += c; s += e;
    }
    for (; r < R; r += 16) s += part[(long)r * N + n];
  }
  red[grp][cl] = s;
  __syncthreads();
  if (grp != 0 || n >= N) return;
  double t = 0.0;
#pragma unroll
  for (int g = 0; g < 16; ++g) t += red[g][cl];
  out[n] = accumulate ? out[n] + (float)t : (float)t;
  if (out2) out2[n] = accumulate ? out2[n] + (float)t : (float)t;  // a second sink (LSTM b_ih / b_hh)
}

void colsum_geometry(int M, int N, int& R, int& rows_per) {
  const int cb = (N + 255) / 256;
  R = std::max(1, std::min(M, std::max(1, 1024 / cb)));
  rows_per = (M + R - 1) / R;
  R = (M + rows_per - 1) / rows_per;
}

// ---- BatchNorm ---------------------------------------------------------------------------
// 64 channels per block; the 4 waves split the partial-sum slabs, combine in fp64 through LDS.
__global__ __launch_bounds__(256) void bn_finalize_kernel(int C, int nparts, int part_rows, const float* __restrict__ stats,
                                                          double count, int training, float momentum,
                                                          float eps, float* __restrict__ rmean,
                                                          float* __restrict__ rvar,
                                                          float* __restrict__ mean_out,
                                                          float* __restrict__ invstd_out,
                                                          unsigned* __restrict__ amax_init) {
  __shared__ double red[3][4][64];
  if (amax_init && blockIdx.x == 0 && threadIdx.x < 2) amax_init[threadIdx.x] = threadIdx.x ? 0x46800000u : 0u;
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  if (training) {
    // partial p covers rows [p * part_rows, min(M, (p + 1) * part_rows)) (gemm.hip bn_tile_stats)
    const long M = (long)count;
    double s = 0.0, a1 = 0.0, a2 = 0.0;
    if (c < C) {
      // partials p = grp, grp + 4, ... combined in order (the fused-BN epilogue's order, gemm.hip
      // bnf_epilogue: same bits); the shift K (partial 0's mean) comes with the first batch.  The
      // loads go out kB partials per thread at a time, the next batch's before the current one is
      // combined: the combine is a chain of dependent fp64 adds, the loads a round trip each batch,
      // and with 4 per batch the C3 call (256 partials x 512 channels on 8 workgroups) took 24.6 us
      // in round trips (round 4); 16 per batch takes four.
      constexpr int kB = 16;
      const double inv_pr = 1.0 / (double)part_rows;
      const double inv_last = 1.0 / (double)(M - (long)(nparts - 1) * part_rows);  // the short last partial
      const float S0 = stats[c];
      float Sv[kB], Qv[kB];
      // (clamped, unconditional loads: see bn_bwd_final_kernel; partials past nparts are skipped)
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        const long p = min(grp + 4 * u, nparts - 1);
        Sv[u] = stats[(p * 2 + 0) * C + c];
        Qv[u] = stats[(p * 2 + 1) * C + c];
      }
      const double K = (double)S0 * (nparts == 1 ? inv_last : inv_pr);
      for (int p0 = grp; p0 < nparts; p0 += 4 * kB) {
        float Sn[kB], Qn[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
          const long p = min(p0 + 4 * kB + 4 * u, nparts - 1);
          Sn[u] = stats[(p * 2 + 0) * C + c];
          Qn[u] = stats[(p * 2 + 1) * C + c];
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) {
          const int p = p0 + 4 * u;
          if (p < nparts) {
            const long n = min((long)part_rows, M - (long)p * part_rows);
            bn_combine(Sv[u], Qv[u], n, p == nparts - 1 ? inv_last : inv_pr, K, s, a1, a2);
          }
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) {
          Sv[u] = Sn[u];
          Qv[u] = Qn[u];
        }
      }
    }
    red[0][grp][cl] = s;
    red[1][grp][cl] = a1;
    red[2][grp][cl] = a2;
    __syncthreads();
    if (grp != 0 || c >= C) return;
    s = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    a1 = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
    a2 = red[2][0][cl] + red[2][1][cl] + red[2][2][cl] + red[2][3][cl];
    const double mean = s / count;
    const double e1 = a1 / count;
    double var = a2 / count - e1 * e1;
    if (var < 0.0) var = 0.0;
    mean_out[c] = (float)mean;
    invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (rmean) rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    if (rvar) {
      const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
      rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
    }
  } else if (grp == 0 && c < C) {
    mean_out[c] = rmean[c];
    invstd_out[c] = (float)(1.0 / sqrt((double)rvar[c] + (double)eps));
  }
}

// Each thread owns one channel quad (its mean/invstd/gamma/beta stay in registers) and walks
// rows; consecutive threads cover consecutive quads of a row (coalesced float4 streams).
__global__ __launch_bounds__(256) void bn_apply_kernel(long M, int C, const float* __restrict__ y,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int act,
                                                       const float* __restrict__ residual,
                                                       float* __restrict__ out,
                                                       unsigned* __restrict__ range_flag,
                                                       unsigned* __restrict__ amax_out) {
  const int Q = C / 4;
  const long nthreads = (long)gridDim.x * blockDim.x;
  const long gt = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long rows_per_pass = nthreads / Q;
  const int q = (int)(gt % Q);
  // leftover threads would revisit rows (out may alias y): they skip the loop (but take part in
  // the block's max reduction)
  const long r0 = gt / Q < rows_per_pass ? gt / Q : M;
  float amax = 0.f;
  float sc[4], sh[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = 4 * q + e;
    sc[e] = invstd[c] * gamma[c];
    sh[e] = beta[c] - mean[c] * sc[e];
  }
  // kRows rows per pass, all loads issued before any store (out may alias y: every element is
  // read and written by the same thread, so loading ahead is safe), so the loads overlap
  constexpr int kRows = 8;
  for (long rb = r0; rb < M; rb += kRows * rows_per_pass) {
    float4 v[kRows], rr[kRows];
#pragma unroll
    for (int u = 0; u < kRows; ++u) {
      const long r = rb + u * rows_per_pass;
      if (r < M) {
        v[u] = reinterpret_cast<const float4*>(y)[r * Q + q];
        if (residual) rr[u] = reinterpret_cast<const float4*>(residual)[r * Q + q];
      }
    }
#pragma unroll
    for (int u = 0; u < kRows; ++u) {
      const long r = rb + u * rows_per_pass;
      if (r >= M) break;
      float o[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = act_fwd(o[e] * sc[e] + sh[e], act);
      if (residual) {
        o[0] += rr[u].x; o[1] += rr[u].y; o[2] += rr[u].z; o[3] += rr[u].w;
      }
      if (range_flag) {  // the consumer contraction skips its range scan (see bn_apply_frag_kernel)
        bool over = false;
#pragma unroll
        for (int e = 0; e < 4; ++e) over |= fabsf(o[e]) >= 65504.f && fabsf(o[e]) < __builtin_inff();
        if (over) __hip_atomic_store(range_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      reinterpret_cast<float4*>(out)[r * Q + q] = make_float4(o[0], o[1], o[2], o[3]);
      if (amax_out) amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
    }
  }
  if (amax_out) {
    __shared__ float red[4];
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      amax_update(amax_out, m);
      amax_update(amax_out + 1, fmaxf(m, 16384.f));
    }
  }
}

// bn_apply with the output also split for the next contraction: thread -> (32-row tile, group
// quad, row, 8-channel group) exactly as gemm.hip's split_frag32_kernel walks a row-major source,
// same arithmetic as bn_apply_kernel, same hi / lo split (lo scaled by 2^11); padding rows and
// channels (to 32-row tiles and 32-deep K) are written as zeros.
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
constexpr int kBnFragLdsC = 1024;
__global__ __launch_bounds__(256) void bn_apply_frag_kernel(long M, int C, int nkc, long ntile,
                                                            const float* __restrict__ y,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, int act,
                                                            const float* __restrict__ residual,
                                                            float* __restrict__ out,
                                                            _Float16* __restrict__ frag,
                                                            unsigned* __restrict__ range_flag,
                                                            unsigned* __restrict__ amax_out) {
  const int G8 = nkc * 2;
  float amax = 0.f;  // max |out| of this thread's elements (amax_out: see bn_apply_kernel)
  const long total = ntile * 32 * G8;
  // per-channel scale / shift formed once per workgroup in LDS (same expressions as
  // bn_apply_kernel), so the element loop issues two float4 loads instead of 32 parameter loads
  __shared__ float s_sc[kBnFragLdsC], s_sh[kBnFragLdsC];
  const bool lds = C <= kBnFragLdsC;
  if (lds) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float sc = invstd[c] * gamma[c];
      s_sc[c] = sc;
      s_sh[c] = beta[c] - mean[c] * sc;
    }
    __syncthreads();
  }
  const unsigned q4 = (unsigned)(G8 >> 2);
  // item idx -> (row r, 8-channel group g8): tile-quad major, then row, then group (4 per quad)
  auto coords = [&](long idx, long& r, int& g8) {
    const int gq = (int)(idx & 3);
    const long rest = idx >> 2;
    const int rr = (int)(rest & 31);
    const long tq = rest >> 5;
    // 32-bit division where the tile-quad index fits (always, below 2^32 quads)
    const long t = tq < 0xffffffffL ? (long)((unsigned)tq / q4) : tq / (long)q4;
    const int quad = (int)(tq - t * (long)q4);
    r = t * 32 + rr;
    g8 = quad * 4 + gq;
  };
  // IT items per thread per pass, all loads issued before any store (the grid is capped when max
  // words are recorded, so each thread walks several items: without this they go one round trip
  // at a time)
  constexpr int IT = 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long base = blockIdx.x * (long)blockDim.x + threadIdx.x; base < total; base += IT * stride) {
    float4 ya[IT], yb[IT], ra[IT], rb[IT];
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const long idx = base + u * stride;
      long r;
      int g8;
      coords(idx, r, g8);
      const int k0 = 8 * g8;
      if (idx < total && r < M && k0 < C) {  // C % 8 == 0: a group is all in or all out
        const float4* q = reinterpret_cast<const float4*>(y + r * C + k0);
        ya[u] = q[0];
        yb[u] = q[1];
        if (residual) {
          const float4* rq = reinterpret_cast<const float4*>(residual + r * C + k0);
          ra[u] = rq[0];
          rb[u] = rq[1];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < IT; ++u) {
      const long idx = base + u * stride;
      if (idx >= total) break;
      long r;
      int g8;
      coords(idx, r, g8);
      const int k0 = 8 * g8;
      float o[8];
      if (r < M && k0 < C) {
        o[0] = ya[u].x; o[1] = ya[u].y; o[2] = ya[u].z; o[3] = ya[u].w;
        o[4] = yb[u].x; o[5] = yb[u].y; o[6] = yb[u].z; o[7] = yb[u].w;
        if (lds) {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = act_fwd(o[e] * s_sc[k0 + e] + s_sh[k0 + e], act);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int c = k0 + e;
            const float sc = invstd[c] * gamma[c];
            const float sh = beta[c] - mean[c] * sc;
            o[e] = act_fwd(o[e] * sc + sh, act);
          }
        }
        if (residual) {
          o[0] += ra[u].x; o[1] += ra[u].y; o[2] += ra[u].z; o[3] += ra[u].w;
          o[4] += rb[u].x; o[5] += rb[u].y; o[6] += rb[u].z; o[7] += rb[u].w;
        }
        if (out) {
          float4* oq = reinterpret_cast<float4*>(out + r * C + k0);
          oq[0] = make_float4(o[0], o[1], o[2], o[3]);
          oq[1] = make_float4(o[4], o[5], o[6], o[7]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = 0.f;
      }
      h16x8 hi, lo;
      bool over = false;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        amax = fmaxf(amax, fabsf(o[j]));
        const _Float16 h = (_Float16)o[j];
        hi[j] = h;
        lo[j] = (_Float16)((o[j] - (float)h) * 2048.0f);
        over |= fabsf(o[j]) >= 65504.f && fabsf(o[j]) < __builtin_inff();
      }
      // range guard of the conv -> conv hand-over: a finite activation the f16 split cannot hold
      // (a BatchNorm affine far outside any trained range) is reported to the host (pinned word),
      // and the next call on the context fails with AVC_ERR_DEVICE
      if (over && range_flag) __hip_atomic_store(range_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const long blk = ((r >> 5) * nkc + (g8 >> 1)) * 2;
      const int lane = (int)(r & 31) + 32 * (g8 & 1);
      *reinterpret_cast<h16x8*>(frag + blk * 512 + lane * 8) = hi;
      *reinterpret_cast<h16x8*>(frag + (blk + 1) * 512 + lane * 8) = lo;
    }
  }
  if (amax_out) {
    __shared__ float red[4];
    for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      amax_update(amax_out, m);
      amax_update(amax_out + 1, fmaxf(m, 16384.f));
    }
  }
}

// partial sums over a row range of dA = d_out * act'(a) and dA * xhat  -> part[r][2][C]
__global__ void bn_bwd_reduce_kernel(int M, int C, const float* __restrict__ dout,
                                     const float* __restrict__ y, const float* __restrict__ mean,
                                     const float* __restrict__ invstd,
                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                     int act, int rows_per, float* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int m0 = blockIdx.y * rows_per, m1 = min(M, m0 + rows_per);
  const float mu = mean[c], is = invstd[c], g = gamma[c], bt = beta[c];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll 4
  for (int m = m0; m < m1; ++m) {
    const long i = (long)m * C + c;
    const float xh = bnb_xhat(y[i], mu, is);
    const float dA = bnb_da(dout[i], xh, g, bt, act);
    s1 += dA;
    s2 += dA * xh;
  }
  part[((long)blockIdx.y * 2 + 0) * C + c] = s1;
  part[((long)blockIdx.y * 2 + 1) * C + c] = s2;
}

// BnBound (bn_backward_frag): also bound max |dy| before dy exists, so the pass that writes dy can
// write it already split.  From the reduce pass's per-channel signed max / min of dA and max |x^|
// (mpart):
//   |dy_c| = |g_c is_c (dA - k1_c - x^ k2_c)| <= |g_c is_c| (max(maxdA_c - k1_c, k1_c - mindA_c) + max|x^|_c |k2_c|),
// maximised over the channels into *bound (pre-zeroed).  The split's power-of-two scale then
// comes from the bound instead of the exact max: a bound above the max by 2^k only moves the
// operand k binades down inside f16's range, which leaves hi / lo (and so the product, unscaled
// exactly) unchanged for every element above 2^-13 of the scaled max.  The signed range keeps the
// bound tight when dA is mostly its channel mean k1 (round 4 used max|dA| + |k1|, which exceeds
// the true max by |k1| / |dA - k1| there: many binades for a mean-dominated gradient).
struct BnBound {
  const float* mpart = nullptr;  // [R][3][C] per-block max dA, min dA, max |x^|
  const float* gamma = nullptr;
  const float* invstd = nullptr;
  float inv_count = 0.f;
  int training = 0;
  unsigned* bound = nullptr;     // max over c of the bound above (float bits)
};

__global__ __launch_bounds__(1024) void bn_bwd_final_kernel(int R, int C, const float* __restrict__ part,
                                                            float* __restrict__ sums, float* __restrict__ d_gamma,
                                                            float* __restrict__ d_beta, int accumulate,
                                                            unsigned* __restrict__ amax, BnBound bb) {
  __shared__ double red[2][16][64];
  __shared__ float redm[3][16][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  if (amax && blockIdx.x == 0 && threadIdx.x == 0) *amax = 0u;  // bn_bwd_apply_cols_kernel raises it
  const int c = blockIdx.x * 64 + cl;
  double s1 = 0.0, s2 = 0.0;
  float m1 = -INFINITY, m0 = INFINITY, m2 = 0.f;  // max dA, min dA, max |x^|
  if (c < C) {
    // rows r = grp, grp + 16, ... summed in that order; kB rows' loads in flight per batch (the
    // sums are a dependent fp64 chain: one load round trip per row took 17 us per C3 call)
    constexpr int kB = 8;
    for (int r0 = grp; r0 < R; r0 += 16 * kB) {
      float a[kB], b[kB];
      // (unconditional loads of a clamped row, masked below: a load under `r < R` compiles to a
      // branch that waits for it, one round trip per row -- 53 us per C3 call measured)
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        const long rc = min(r0 + 16 * u, R - 1);
        a[u] = part[(rc * 2 + 0) * C + c];
        b[u] = part[(rc * 2 + 1) * C + c];
      }
      if (bb.bound) {
        float x1[kB], x0[kB], x2[kB];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
          const long rc = min(r0 + 16 * u, R - 1);  // (a repeated row leaves max / min unchanged)
          x1[u] = bb.mpart[(rc * 3 + 0) * C + c];
          x0[u] = bb.mpart[(rc * 3 + 1) * C + c];
          x2[u] = bb.mpart[(rc * 3 + 2) * C + c];
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) {
          m1 = fmaxf(m1, x1[u]);
          m0 = fminf(m0, x0[u]);
          m2 = fmaxf(m2, x2[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < kB; ++u)
        if (r0 + 16 * u < R) {
          s1 += a[u];
          s2 += b[u];
        }
    }
  }
  red[0][grp][cl] = s1;
  red[1][grp][cl] = s2;
  redm[0][grp][cl] = m1;
  redm[1][grp][cl] = m2;
  redm[2][grp][cl] = m0;
  __syncthreads();
  if (grp != 0 || c >= C) return;
  double t1 = 0.0, t2 = 0.0;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    t1 += red[0][g][cl];
    t2 += red[1][g][cl];
    m1 = fmaxf(m1, redm[0][g][cl]);
    m2 = fmaxf(m2, redm[1][g][cl]);
    m0 = fminf(m0, redm[2][g][cl]);
  }
  sums[c] = (float)t1;
  sums[C + c] = (float)t2;
  if (d_beta) d_beta[c] = accumulate ? d_beta[c] + (float)t1 : (float)t1;
  if (d_gamma) d_gamma[c] = accumulate ? d_gamma[c] + (float)t2 : (float)t2;
  if (bb.bound) {
    // the apply pass's own k1 / k2 (sums as float, times 1 / M); a few ulps of slack for the
    // rounding of the apply's expression
    const float k1 = bb.training ? (float)t1 * bb.inv_count : 0.f, k2 = bb.training ? (float)t2 * bb.inv_count : 0.f;
    const float rng = fmaxf(fmaxf(m1 - k1, k1 - m0), 0.f);  // max |dA - k1| over the channel's rows
    const float b = fabsf(bb.gamma[c] * bb.invstd[c]) * (rng + m2 * fabsf(k2)) * 1.0001f;
    atomicMax(bb.bound, __float_as_uint(b));  // non-negative floats order as their bits
  }
}

__global__ void bn_bwd_apply_kernel(long M, int C, const float* __restrict__ dout,
                                    const float* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ invstd,
                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                    int act, int training, const float* __restrict__ sums,
                                    float inv_count, float* __restrict__ dy) {
  const long total = M * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float is = invstd[c], g = gamma[c];
    const float xh = bnb_xhat(y[i], mean[c], is);
    const float dA = bnb_da(dout[i], xh, g, beta[c], act);
    const float v = bnb_dy(dA, xh, g, is, training ? sums[c] * inv_count : 0.f,
                           training ? sums[C + c] * inv_count : 0.f, training);
    dy[i] = v;
  }
}

// bn_bwd_apply_kernel by columns: thread = channel c walking a row range (per-channel constants in
// registers, coalesced along channels), also producing the column partial sums of dy (the conv
// bias gradient, part[blockIdx.y][c]) and max |dy| (the backward products' operand scale) so no
// separate pass re-reads dy for them.
__global__ __launch_bounds__(256) void bn_bwd_apply_cols_kernel(int M, int C, const float* __restrict__ dout,
                                                                const float* __restrict__ y,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, int act,
                                                                int training, const float* __restrict__ sums,
                                                                float inv_count, int rows_per, float* __restrict__ dy,
                                                                float* __restrict__ part, unsigned* __restrict__ amax) {
  __shared__ float red[4];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  float cs = 0.f, mx = 0.f;
  if (c < C) {
    const int m0 = blockIdx.y * rows_per, m1 = min(M, m0 + rows_per);
    const float is = invstd[c], g = gamma[c], mu = mean[c], bt = beta[c];
    const float k1 = training ? sums[c] * inv_count : 0.f, k2 = training ? sums[C + c] * inv_count : 0.f;
#pragma unroll 4
    for (int m = m0; m < m1; ++m) {
      const long i = (long)m * C + c;
      const float xh = bnb_xhat(y[i], mu, is);
      const float dA = bnb_da(dout[i], xh, g, bt, act);
      const float v = bnb_dy(dA, xh, g, is, k1, k2, training);
      dy[i] = v;
      cs += v;
      mx = fmaxf(mx, fabsf(v));
    }
    if (part) part[(long)blockIdx.y * C + c] = cs;
  }
  if (amax) {
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) amax_update(amax, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

// The two BN-backward passes with float4 streams: thread = (row phase, channel quad); the
// P = 256 / (C/4) phases interleave the rows of the block's range and are combined through LDS
// in a fixed order.  Needs C % 4 == 0, C <= 1024 and 16-byte aligned dout / y / dy.
struct BnQuad {
  float mu[4], is[4], g[4], bt[4];
};
__device__ __forceinline__ void bn_quad_load(BnQuad& k, int c0, const float* mean, const float* invstd,
                                             const float* gamma, const float* beta) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    k.mu[e] = mean[c0 + e];
    k.is[e] = invstd[c0 + e];
    k.g[e] = gamma[c0 + e];
    k.bt[e] = beta[c0 + e];
  }
}

__global__ __launch_bounds__(256) void bn_bwd_reduce4_kernel(int M, int C, const float* __restrict__ dout,
                                                             const float* __restrict__ y, const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int act, int rows_per,
                                                             float* __restrict__ part, float* __restrict__ mpart,
                                                             unsigned* __restrict__ zero_word) {
  __shared__ float4 red[2][256];
  // (bn_backward_frag: the bound word the final kernel raises, zeroed here, a launch before)
  if (zero_word && blockIdx.y == 0 && threadIdx.x == 0) *zero_word = 0u;
  const int Q = C >> 2, P = 256 / Q;
  const int ph = threadIdx.x / Q, q = threadIdx.x - ph * Q;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  // (mpart) max dA, min dA, max |xh|
  float mx1[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, mn1[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
  float mx2[4] = {0.f, 0.f, 0.f, 0.f};
  if (ph < P) {
    BnQuad k;
    bn_quad_load(k, 4 * q, mean, invstd, gamma, beta);
    const int m0 = blockIdx.y * rows_per, m1 = min(M, m0 + rows_per);
#pragma unroll 8
    for (int m = m0 + ph; m < m1; m += P) {
      const long i4 = (long)m * Q + q;
      const float4 yv = reinterpret_cast<const float4*>(y)[i4];
      const float4 dv = reinterpret_cast<const float4*>(dout)[i4];
      const float yy[4] = {yv.x, yv.y, yv.z, yv.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = bnb_xhat(yy[e], k.mu[e], k.is[e]);
        const float dA = bnb_da(dd[e], xh, k.g[e], k.bt[e], act);
        s1[e] += dA;
        s2[e] += dA * xh;
        mx1[e] = fmaxf(mx1[e], dA);
        mn1[e] = fminf(mn1[e], dA);
        mx2[e] = fmaxf(mx2[e], fabsf(xh));
      }
    }
  }
  red[0][threadIdx.x] = make_float4(s1[0], s1[1], s1[2], s1[3]);
  red[1][threadIdx.x] = make_float4(s2[0], s2[1], s2[2], s2[3]);
  __syncthreads();
  if (ph == 0) {
    float4 a = red[0][q], b = red[1][q];
    for (int p = 1; p < P; ++p) {
      const float4 u = red[0][p * Q + q], v = red[1][p * Q + q];
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
      b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
    }
    reinterpret_cast<float4*>(part + ((long)blockIdx.y * 2 + 0) * C)[q] = a;
    reinterpret_cast<float4*>(part + ((long)blockIdx.y * 2 + 1) * C)[q] = b;
  }
  if (!mpart) return;
  __syncthreads();
  red[0][threadIdx.x] = make_float4(mx1[0], mx1[1], mx1[2], mx1[3]);
  red[1][threadIdx.x] = make_float4(mx2[0], mx2[1], mx2[2], mx2[3]);
  __syncthreads();
  if (ph == 0) {
    float4 a = red[0][q], b = red[1][q];
    for (int p = 1; p < P; ++p) {
      const float4 u = red[0][p * Q + q], v = red[1][p * Q + q];
      a.x = fmaxf(a.x, u.x); a.y = fmaxf(a.y, u.y); a.z = fmaxf(a.z, u.z); a.w = fmaxf(a.w, u.w);
      b.x = fmaxf(b.x, v.x); b.y = fmaxf(b.y, v.y); b.z = fmaxf(b.z, v.z); b.w = fmaxf(b.w, v.w);
    }
    reinterpret_cast<float4*>(mpart + ((long)blockIdx.y * 3 + 0) * C)[q] = a;
    reinterpret_cast<float4*>(mpart + ((long)blockIdx.y * 3 + 2) * C)[q] = b;
  }
  __syncthreads();
  red[0][threadIdx.x] = make_float4(mn1[0], mn1[1], mn1[2], mn1[3]);
  __syncthreads();
  if (ph != 0) return;
  float4 a = red[0][q];
  for (int p = 1; p < P; ++p) {
    const float4 u = red[0][p * Q + q];
    a.x = fminf(a.x, u.x); a.y = fminf(a.y, u.y); a.z = fminf(a.z, u.z); a.w = fminf(a.w, u.w);
  }
  reinterpret_cast<float4*>(mpart + ((long)blockIdx.y * 3 + 1) * C)[q] = a;
}

__global__ __launch_bounds__(256) void bn_bwd_apply4_kernel(int M, int C, const float* __restrict__ dout,
                                                            const float* __restrict__ y, const float* __restrict__ mean,
                                                            const float* __restrict__ invstd,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, int act, int training,
                                                            const float* __restrict__ sums, float inv_count,
                                                            int rows_per, float* __restrict__ dy,
                                                            float* __restrict__ part, unsigned* __restrict__ amax) {
  __shared__ float4 red[256];
  __shared__ float redm[4];
  const int Q = C >> 2, P = 256 / Q;
  const int ph = threadIdx.x / Q, q = threadIdx.x - ph * Q;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  float mx = 0.f;
  if (ph < P) {
    BnQuad k;
    bn_quad_load(k, 4 * q, mean, invstd, gamma, beta);
    float k1[4], k2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      k1[e] = training ? sums[4 * q + e] * inv_count : 0.f;
      k2[e] = training ? sums[C + 4 * q + e] * inv_count : 0.f;
    }
    const int m0 = blockIdx.y * rows_per, m1 = min(M, m0 + rows_per);
#pragma unroll 4
    for (int m = m0 + ph; m < m1; m += P) {
      const long i4 = (long)m * Q + q;
      const float4 yv = reinterpret_cast<const float4*>(y)[i4];
      const float4 dv = reinterpret_cast<const float4*>(dout)[i4];
      const float yy[4] = {yv.x, yv.y, yv.z, yv.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xh = bnb_xhat(yy[e], k.mu[e], k.is[e]);
        const float dA = bnb_da(dd[e], xh, k.g[e], k.bt[e], act);
        o[e] = bnb_dy(dA, xh, k.g[e], k.is[e], k1[e], k2[e], training);
        cs[e] += o[e];
        mx = fmaxf(mx, fabsf(o[e]));
      }
      reinterpret_cast<float4*>(dy)[i4] = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  if (part) {
    red[threadIdx.x] = make_float4(cs[0], cs[1], cs[2], cs[3]);
    __syncthreads();
    if (ph == 0) {
      float4 a = red[q];
      for (int p = 1; p < P; ++p) {
        const float4 u = red[p * Q + q];
        a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
      }
      reinterpret_cast<float4*>(part + (long)blockIdx.y * C)[q] = a;
    }
  }
  if (amax) {
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if ((threadIdx.x & 63) == 0) redm[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) amax_update(amax, fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3])));
  }
}

// bn_bwd_apply4_kernel writing dy already split (bn_backward_frag; round 4): the two fragment
// images the conv backward's products stream -- dy as the dgrad product's A (rows = frames, k =
// channels) and dy^T as the weight gradient's A (rows = channels, k = frames), both in
// split_frag32_kernel's layout and scaled by the power of two of the bound from
// bn_bwd_final_kernel (BnBound) -- instead of an fp32 dy that a max scan and two split passes
// re-read.  Workgroup = 32 frames x 128 channels: dy (same expressions as bn_bwd_apply4_kernel)
// into an LDS tile, its column sums (the conv bias gradient's partials, one row per 32 frames),
// then the tile's blocks of both images.  Needs C % 4 == 0.
__device__ __forceinline__ void bwd_split8(const float* v, h16x8& hi, h16x8& lo) {  // split8 (gemm.hip)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = (_Float16)v[j];
    hi[j] = h;
    lo[j] = (_Float16)((v[j] - (float)h) * 2048.0f);
  }
}
__device__ __forceinline__ float pow2_of_bound(const unsigned* w) {  // split_scale_of (gemm.hip)
  const float m = __uint_as_float(*w);
  if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, 15 - e);
}

__global__ __launch_bounds__(256) void bn_bwd_apply_frag_kernel(int M, int C, const float* __restrict__ dout,
                                                                const float* __restrict__ y,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, int act, int training,
                                                                const float* __restrict__ sums, float inv_count,
                                                                const unsigned* __restrict__ bound,
                                                                _Float16* __restrict__ imgA, int nkcA,
                                                                _Float16* __restrict__ imgT, int nkcT,
                                                                float* __restrict__ part) {
  constexpr int TR = 32, TC = 128, LD = TC + 4;
  __shared__ __attribute__((aligned(16))) float tile[TR][LD];
  __shared__ float4 csr[4][32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cg = blockIdx.x, rt = blockIdx.y;
  const int c0 = cg * TC, r0 = rt * TR;
  const int q = tid & 31, ph = tid >> 5;  // channel quad of the group, row phase (8)
  const int c = c0 + 4 * q;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    BnQuad k;
    bn_quad_load(k, c, mean, invstd, gamma, beta);
    float k1[4], k2[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      k1[e] = training ? sums[c + e] * inv_count : 0.f;
      k2[e] = training ? sums[C + c + e] * inv_count : 0.f;
    }
#pragma unroll
    for (int i = 0; i < TR / 8; ++i) {
      const int r = ph + 8 * i, m = r0 + r;
      float o[4] = {0.f, 0.f, 0.f, 0.f};
      if (m < M) {
        const long i4 = ((long)m * C + c) >> 2;
        const float4 yv = reinterpret_cast<const float4*>(y)[i4];
        const float4 dv = reinterpret_cast<const float4*>(dout)[i4];
        const float yy[4] = {yv.x, yv.y, yv.z, yv.w}, dd[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = bnb_xhat(yy[e], k.mu[e], k.is[e]);
          const float dA = bnb_da(dd[e], xh, k.g[e], k.bt[e], act);
          o[e] = bnb_dy(dA, xh, k.g[e], k.is[e], k1[e], k2[e], training);
          cs[e] += o[e];
        }
      }
      *reinterpret_cast<float4*>(&tile[r][4 * q]) = make_float4(o[0], o[1], o[2], o[3]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < TR / 8; ++i) *reinterpret_cast<float4*>(&tile[ph + 8 * i][4 * q]) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // column sums over the 32 frames in a fixed order: the two phases of a wave, then the 4 waves
#pragma unroll
  for (int e = 0; e < 4; ++e) cs[e] += __shfl_xor(cs[e], 32);
  if (lane < 32) csr[w][q] = make_float4(cs[0], cs[1], cs[2], cs[3]);
  __syncthreads();
  if (part && tid < 32 && c < C) {
    float4 a = csr[0][q];
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) {
      const float4 u = csr[ww][q];
      a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    }
    *reinterpret_cast<float4*>(part + (long)rt * C + c) = a;
  }
  const float sc = pow2_of_bound(bound);
  // dy as the dgrad product's A: block (row tile rt, 16-channel chunk kc), lane l = row l & 31,
  // channels 8 (l >> 5) .. + 7 of the chunk
  for (int it = tid; it < (TC / 16) * 64; it += 256) {
    const int kcl = it >> 6, kc = cg * (TC / 16) + kcl;
    if (kc >= nkcA) continue;
    const int l = it & 63, r = l & 31, k0 = kcl * 16 + 8 * (l >> 5);
    const float4 a = *reinterpret_cast<const float4*>(&tile[r][k0]);
    const float4 b = *reinterpret_cast<const float4*>(&tile[r][k0 + 4]);
    const float v[8] = {a.x * sc, a.y * sc, a.z * sc, a.w * sc, b.x * sc, b.y * sc, b.z * sc, b.w * sc};
    h16x8 hi, lo;
    bwd_split8(v, hi, lo);
    const long blk = ((long)rt * nkcA + kc) * 2;
    *reinterpret_cast<h16x8*>(imgA + blk * 512 + l * 8) = hi;
    *reinterpret_cast<h16x8*>(imgA + (blk + 1) * 512 + l * 8) = lo;
  }
  // dy^T as the weight gradient's A: block (channel tile ct, 16-frame chunk 2 rt + j), lane l =
  // channel l & 31 of the tile, frames 8 (l >> 5) .. + 7 of the chunk
  const int ntc = (C + 31) / 32;
  for (int it = tid; it < (TC / 32) * 2 * 64; it += 256) {
    const int ctl = it >> 7, j = (it >> 6) & 1, ct = cg * (TC / 32) + ctl;
    if (ct >= ntc) continue;
    const int l = it & 63, cl = ctl * 32 + (l & 31), rb = j * 16 + 8 * (l >> 5);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[rb + e][cl] * sc;
    h16x8 hi, lo;
    bwd_split8(v, hi, lo);
    const long blk = ((long)ct * nkcT + 2 * rt + j) * 2;
    *reinterpret_cast<h16x8*>(imgT + blk * 512 + l * 8) = hi;
    *reinterpret_cast<h16x8*>(imgT + (blk + 1) * 512 + l * 8) = lo;
  }
}

// ---- layout glue -------------------------------------------------------------------------
__global__ void frames_from_mel_kernel(int T, int B, int cm, const float* __restrict__ x, int ce,
                                       const float* __restrict__ emb, float* __restrict__ out) {
  const int C = cm + ce;
  const long total = (long)T * B * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c, b, t;
    if (total <= 0x7fffffffL) {  // 32-bit divisions (a 64-bit one is a long software sequence)
      const unsigned u = (unsigned)i, r = u / (unsigned)C;
      c = (int)(u - r * (unsigned)C);
      t = (int)(r / (unsigned)B);
      b = (int)(r - (unsigned)t * (unsigned)B);
    } else {
      c = (int)(i % C);
      const long r = i / C;
      b = (int)(r % B), t = (int)(r / B);
    }
    out[i] = c < cm ? x[((long)b * cm + c) * T + t] : emb[(long)b * ce + (c - cm)];
  }
}

// frames_from_mel straight into the first encoder conv's split operand (round 4):
// frames_guard_kernel takes the range guard of the input itself (max |x| over the mel and the
// embedding: a quarter of the frames' bytes) into w[0] = max, w[1] = max(max, 2^14) (pre-zeroed);
// frames_frag_kernel then writes the [T*B][cm+ce] frames directly as the fragment image
// split_frag32_kernel would make of them with that guard's scale (GemmDesc::a_frag_guard): the
// frames' fp32 store, their range scan and the split pass are gone, and the bits are the same.
__global__ __launch_bounds__(256) void frames_guard_kernel(const float* __restrict__ x, long nx,
                                                           const float* __restrict__ emb, long ne,
                                                           float* __restrict__ partial, unsigned* __restrict__ ticket,
                                                           unsigned* __restrict__ w) {
  // (guard_scan_kernel's one-launch form over two sources: every block writes its maximum to
  // partial[blockIdx]; the last block to take a ticket writes the words -- no zeroing launch)
  __shared__ float red[4];
  __shared__ bool last;
  float m = 0.f;
  const long stride = (long)gridDim.x * 256, gid = blockIdx.x * 256L + threadIdx.x;
  if ((nx & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    // (round 6) the mel as float4 with four loads in flight, then the embedding: the scalar walk
    // below went one dependent round trip per element (10.6 us for a C2 batch)
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const long n4 = nx >> 2;
    long i = gid;
    for (; i + 3 * stride < n4; i += 4 * stride) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = x4[i + u * stride];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
    for (; i < n4; i += stride) {
      const float4 v = x4[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
    for (long j = gid; j < ne; j += stride) m = fmaxf(m, fabsf(emb[j]));
  } else {
    for (long i = gid; i < nx + ne; i += stride) m = fmaxf(m, fabsf(i < nx ? x[i] : emb[i - nx]));
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(partial + blockIdx.x, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    last = atomicInc(ticket, gridDim.x - 1) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  float v = 0.f;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += 256)
    v = fmaxf(v, __hip_atomic_load(partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    w[0] = __float_as_uint(v);
    w[1] = __float_as_uint(fmaxf(v, 16384.f));
  }
}

__global__ __launch_bounds__(256) void frames_frag_kernel(int T, int B, int cm, const float* __restrict__ x, int ce,
                                                          const float* __restrict__ emb, int nkc, long ntile,
                                                          const unsigned* __restrict__ guard,
                                                          _Float16* __restrict__ frag) {
  const int C = cm + ce, G8 = nkc * 2;
  const float sc = pow2_of_bound(guard);  // split_scale_of: 1 below 2^15
  const long total = ntile * 32 * G8, M = (long)T * B;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    // item -> (row r, 8-channel group g8), rows fastest within a tile: a wave writes 64 lanes of
    // one fragment block pair
    const long tile = idx / (32L * G8);
    const int rem = (int)(idx - tile * 32L * G8), g8 = rem >> 5, rr = rem & 31;
    const long r = tile * 32 + rr;
    float v[8];
    if (r < M) {
      const int t = (int)(r / B), b = (int)(r - (long)t * B);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 8 * g8 + e;
        v[e] = (c < cm ? x[((long)b * cm + c) * T + t] : c < C ? emb[(long)b * ce + (c - cm)] : 0.f) * sc;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
    }
    h16x8 hi, lo;
    bwd_split8(v, hi, lo);
    const long blk = (tile * nkc + (g8 >> 1)) * 2;
    const int lane = rr + 32 * (g8 & 1);
    *reinterpret_cast<h16x8*>(frag + blk * 512 + lane * 8) = hi;
    *reinterpret_cast<h16x8*>(frag + (blk + 1) * 512 + lane * 8) = lo;
  }
}

// frames_guard_kernel and frames_frag_kernel in ONE launch for T % 4 == 0, B % 32 == 0 (round 6):
// a thread takes 4 consecutive frames of one batch row and 8-channel group (one float4 per channel;
// lanes take consecutive b, so a wave writes whole 512-B runs of a block).  The image is written with
// scale 1 -- what the guard gives whenever max |x| < 2^15, i.e. for every mel in [0, 1] and unit-norm
// embedding -- while each workgroup also takes the max of the values it split; the last workgroup
// to take a ticket forms the guard words and, only if the guard's scale is not 1, re-writes the
// whole image with that scale itself (correct, slow, never taken for normalised inputs).  Every
// other workgroup's stores precede its ticket (fence), so the re-write lands last.  Same words,
// same image as the two kernels; one launch and one pass fewer.
__global__ __launch_bounds__(256) void frames_frag_guard_kernel(int T, int B, int cm, const float* __restrict__ x,
                                                                int ce, const float* __restrict__ emb, int nkc,
                                                                float* __restrict__ partial,
                                                                unsigned* __restrict__ ticket, unsigned* __restrict__ w,
                                                                _Float16* __restrict__ frag) {
  __shared__ float red[4];
  __shared__ bool last;
  const int C = cm + ce, G8 = nkc * 2, T4 = T >> 2;
  const long total = (long)T4 * G8 * B;
  auto item = [&](long idx, float sc, float& m) {
    const int b = (int)(idx % B);
    const long rest = idx / B;
    const int g8 = (int)(rest % G8), t4 = (int)(rest / G8);
    float v[4][8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = 8 * g8 + e;
      if (c < cm) {
        const float4 q = *reinterpret_cast<const float4*>(x + ((long)b * cm + c) * T + 4 * t4);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fmaxf(fabsf(q.z), fabsf(q.w))));
        v[0][e] = q.x * sc; v[1][e] = q.y * sc; v[2][e] = q.z * sc; v[3][e] = q.w * sc;
      } else {
        const float ev = c < C ? emb[(long)b * ce + (c - cm)] : 0.f;
        m = fmaxf(m, fabsf(ev));
        v[0][e] = v[1][e] = v[2][e] = v[3][e] = ev * sc;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long r = (long)(4 * t4 + u) * B + b;
      h16x8 hi, lo;
      bwd_split8(v[u], hi, lo);
      const long blk = ((r >> 5) * nkc + (g8 >> 1)) * 2;
      const int lane = (int)(r & 31) + 32 * (g8 & 1);
      *reinterpret_cast<h16x8*>(frag + blk * 512 + lane * 8) = hi;
      *reinterpret_cast<h16x8*>(frag + (blk + 1) * 512 + lane * 8) = lo;
    }
  };
  float m = 0.f;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) item(idx, 1.f, m);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(partial + blockIdx.x, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    last = atomicInc(ticket, gridDim.x - 1) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  float v = 0.f;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += 256)
    v = fmaxf(v, __hip_atomic_load(partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const unsigned w1 = __float_as_uint(fmaxf(v, 16384.f));
  if (threadIdx.x == 0) {
    w[0] = __float_as_uint(v);
    w[1] = w1;
  }
  const float sc = pow2_of_bound(&w1);
  if (sc != 1.f) {  // out of the split's range: the whole image again, with the guard's scale
    float unused = 0.f;
    for (long idx = threadIdx.x; idx < total; idx += 256) item(idx, sc, unused);
  }
}

// d_x[b][c][t] (+)= d_frames[(t*B+b)*ld + c]
__global__ void mel_grad_kernel(int T, int B, int cm, const float* __restrict__ df, int ld,
                                float* __restrict__ dx, int accumulate) {
  const long total = (long)B * cm * T;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int t = (int)(i % T);
    const long bc = i / T;
    const int c = (int)(bc % cm), b = (int)(bc / cm);
    const float v = df[((long)t * B + b) * ld + c];
    dx[i] = accumulate ? dx[i] + v : v;
  }
}

__global__ void emb_grad_kernel(int T, int B, int cm, int ce, const float* __restrict__ df, int ld,
                                float* __restrict__ demb, int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * ce) return;
  const int b = i / ce, c = i % ce;
  double s = 0.0;
  for (int t = 0; t < T; ++t) s += df[((long)t * B + b) * ld + cm + c];
  demb[i] = accumulate ? demb[i] + (float)s : (float)s;
}

// grid y = 1 or 2: a second (frames, mel) pair in the same launch (the Generator's mel and mel_post)
__global__ void mel_from_frames_kernel(int T, int B, int cm, const float* __restrict__ fr,
                                       float* __restrict__ mel, const float* __restrict__ fr1,
                                       float* __restrict__ mel1) {
  if (blockIdx.y) fr = fr1, mel = mel1;
  const long total = (long)B * cm * T;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int t, c, b;
    if (total <= 0x7fffffffL) {  // 32-bit divisions
      const unsigned u = (unsigned)i, bc = u / (unsigned)T;
      t = (int)(u - bc * (unsigned)T);
      b = (int)(bc / (unsigned)cm);
      c = (int)(bc - (unsigned)b * (unsigned)cm);
    } else {
      t = (int)(i % T);
      const long bc = i / T;
      c = (int)(bc % cm), b = (int)(bc / cm);
    }
    mel[i] = fr[((long)t * B + b) * cm + c];
  }
}

// codes[b][32*i + d]: i < nA -> forward half at t = 32i+31; else backward half at t = 32(i-nA)
__global__ void codes_kernel(int T, int B, const float* __restrict__ enc, float* __restrict__ codes,
                             int backward, int accumulate, float* __restrict__ denc) {
  const int nA = T / 32, nB = (T + 31) / 32, L = 32 * (nA + nB);
  const long total = (long)B * L;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int b = (int)(idx / L), q = (int)(idx % L);
    const int i = q >> 5, d = q & 31;
    long src;
    if (i < nA) src = ((long)(32 * i + 31) * B + b) * 64 + d;
    else src = ((long)(32 * (i - nA)) * B + b) * 64 + 32 + d;
    if (!backward) codes[idx] = enc[src];
    else denc[src] = accumulate ? denc[src] + codes[idx] : codes[idx];
  }
}

__global__ void decoder_input_kernel(int T, int B, const float* __restrict__ enc, int ce,
                                     const float* __restrict__ ctrg, float* __restrict__ out,
                                     unsigned* __restrict__ range_flag) {
  const int C = 64 + ce, nA = T / 32;
  const long total = (long)T * B * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c, b, t;
    if (total <= 0x7fffffffL) {  // 32-bit divisions
      const unsigned u = (unsigned)i, r = u / (unsigned)C;
      c = (int)(u - r * (unsigned)C);
      t = (int)(r / (unsigned)B);
      b = (int)(r - (unsigned)t * (unsigned)B);
    } else {
      c = (int)(i % C);
      const long r = i / C;
      b = (int)(r % B), t = (int)(r / B);
    }
    float v;
    if (c < 32) {
      const int blk = min(t / 32, nA - 1);
      v = enc[((long)(32 * blk + 31) * B + b) * 64 + c];
    } else if (c < 64) {
      v = enc[((long)(32 * (t / 32)) * B + b) * 64 + c];
    } else {
      v = ctrg[(long)b * ce + (c - 64)];
      // the codes are LSTM outputs (|h| < 1); the target embedding is the caller's: range-check it
      // for the consumer's f16 split (see bn_apply_kernel)
      if (range_flag && fabsf(v) >= 65504.f && fabsf(v) < __builtin_inff())
        __hip_atomic_store(range_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    out[i] = v;
  }
}

// decoder_input_kernel four channels per thread (C % 4 == 0), also writing the content codes where
// `codes` is given (round 6: the whole-Generator forward's codes_kernel folded in -- each code
// element is the decoder input's value at frame 32 i + 31 (forward stream) or 32 i (backward
// stream), written by the one thread that reads it).  Same values as decoder_input_kernel and
// codes_kernel.
__global__ void decoder_input4_kernel(int T, int B, const float* __restrict__ enc, int ce,
                                      const float* __restrict__ ctrg, float* __restrict__ out,
                                      unsigned* __restrict__ range_flag, float* __restrict__ codes) {
  const int C = 64 + ce, C4 = C >> 2, nA = T / 32, L = 32 * (nA + (T + 31) / 32);
  const long total = (long)T * B * C4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / C4;
    const int c0 = 4 * (int)(i - r * C4), t = (int)(r / B), b = (int)(r - (long)t * B);
    float4 v;
    if (c0 < 32) {
      const int blk = min(t / 32, nA - 1);
      v = *reinterpret_cast<const float4*>(enc + ((long)(32 * blk + 31) * B + b) * 64 + c0);
      if (codes && (t & 31) == 31 && t / 32 < nA)
        *reinterpret_cast<float4*>(codes + (long)b * L + (t / 32) * 32 + c0) = v;
    } else if (c0 < 64) {
      v = *reinterpret_cast<const float4*>(enc + ((long)(32 * (t / 32)) * B + b) * 64 + c0);
      if (codes && (t & 31) == 0)
        *reinterpret_cast<float4*>(codes + (long)b * L + (nA + t / 32) * 32 + (c0 - 32)) = v;
    } else {
      v = *reinterpret_cast<const float4*>(ctrg + (long)b * ce + (c0 - 64));
      if (range_flag) {  // (see decoder_input_kernel)
        bool over = false;
        over |= fabsf(v.x) >= 65504.f && fabsf(v.x) < __builtin_inff();
        over |= fabsf(v.y) >= 65504.f && fabsf(v.y) < __builtin_inff();
        over |= fabsf(v.z) >= 65504.f && fabsf(v.z) < __builtin_inff();
        over |= fabsf(v.w) >= 65504.f && fabsf(v.w) < __builtin_inff();
        if (over) __hip_atomic_store(range_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    *reinterpret_cast<float4*>(out + r * C + c0) = v;
  }
}

// one thread per (b, stream s in {fwd,bwd}, code index i, dim d)
__global__ void decoder_input_bwd_kernel(int T, int B, int ce, const float* __restrict__ dd,
                                         float* __restrict__ denc) {
  const int C = 64 + ce, nA = T / 32, nB = (T + 31) / 32;
  const long total = (long)B * (nA + nB) * 32;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int d = (int)(idx & 31);
    const long rest = idx >> 5;
    const int q = (int)(rest % (nA + nB)), b = (int)(rest / (nA + nB));
    int t0, t1, col, trow;
    if (q < nA) {  // forward code q covers [32q, 32q+32) (last one also the tail)
      t0 = 32 * q;
      t1 = (q == nA - 1) ? T : 32 * q + 32;
      col = d;
      trow = 32 * q + 31;
    } else {
      const int j = q - nA;
      t0 = 32 * j;
      t1 = min(T, 32 * j + 32);
      col = 32 + d;
      trow = 32 * j;
    }
    float s = 0.f;
    for (int t = t0; t < t1; ++t) s += dd[((long)t * B + b) * C + col];
    denc[((long)trow * B + b) * 64 + col] += s;
  }
}

// out[c][tau] = mean over slices i covering tau of frames[i][c][tau - i*step], skipping NaNs
// (model.py:428-437: NaN padding + nanmean)
__global__ void overlap_average_kernel(int M, int C, int N, int step, const float* __restrict__ fr,
                                       float* __restrict__ out) {
  const int L = (M - 1) * step + N;
  const long total = (long)C * L;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx / L), tau = (int)(idx % L);
    float s = 0.f;
    int cnt = 0;
    for (int i = 0; i < M; ++i) {
      const int k = tau - i * step;
      if (k < 0 || k >= N) continue;
      const float v = fr[((long)i * C + c) * N + k];
      if (v != v) continue;
      s += v;
      ++cnt;
    }
    out[idx] = cnt ? s / (float)cnt : __int_as_float(0x7fc00000);
  }
}

// d fr[i][c][k] = d_out[c][i*step + k] / (non-NaN slices covering that column), 0 for a NaN
// entry: torch's nanmean backward (nansum / count) for the paste of model.py:428-437
__global__ void overlap_average_backward_kernel(int M, int C, int N, int step, const float* __restrict__ fr,
                                                const float* __restrict__ dout, float* __restrict__ dfr) {
  const int L = (M - 1) * step + N;
  const long total = (long)M * C * N;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int i = (int)(idx / ((long)C * N));
    const int c = (int)((idx / N) % C);
    const int tau = i * step + (int)(idx % N);
    const float v = fr[idx];
    if (v != v) {
      dfr[idx] = 0.f;
      continue;
    }
    int cnt = 0;
    for (int j = 0; j < M; ++j) {
      const int k = tau - j * step;
      if (k < 0 || k >= N) continue;
      const float w = fr[((long)j * C + c) * N + k];
      if (w == w) ++cnt;
    }
    dfr[idx] = dout[(long)c * L + tau] / (float)cnt;
  }
}

// ---- losses ------------------------------------------------------------------------------
__global__ void loss_partial_kernel(int kind, long n, const float* __restrict__ a,
                                    const float* __restrict__ b, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float d = a[i] - b[i];
    s += kind == 0 ? (double)(d * d) : (double)fabsf(d);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// one block of 256: strided partial sums, then a fixed-order tree (deterministic)
__global__ __launch_bounds__(256) void loss_final_kernel(int nparts, const double* __restrict__ part, double inv_n,
                                                         float* __restrict__ out, int accumulate) {
  __shared__ double red[256];
  double s = 0.0;
  for (int p = threadIdx.x; p < nparts; p += 256) s += part[p];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const float v = (float)(red[0] * inv_n);
  out[0] = accumulate ? out[0] + v : v;
}

__global__ void loss_grad_kernel(int kind, long n, const float* __restrict__ a,
                                 const float* __restrict__ b, const float* __restrict__ dscale,
                                 float scale, float* __restrict__ ga, float* __restrict__ gb,
                                 int accumulate) {
  const float sc = scale * (dscale ? dscale[0] : 1.f);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float d = a[i] - b[i];
    float g;
    if (kind == 0) g = 2.f * d * sc;
    else g = (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) * sc;
    if (ga) ga[i] = accumulate ? ga[i] + g : g;
    if (gb) gb[i] = accumulate ? gb[i] - g : -g;
  }
}

// ---- optimizer ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sumsq_partial_kernel(long n, const float* __restrict__ g,
                                                            double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  const long n4 = (reinterpret_cast<uintptr_t>(g) & 15) == 0 ? n / 4 : 0;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = g4[i];
    s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (long i = 4 * n4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const double v = g[i];
    s += v * v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// one block of 256: strided partial sums, then a fixed-order tree (deterministic)
__global__ __launch_bounds__(256) void clip_coef_kernel(int nparts, const double* __restrict__ part, float max_norm,
                                                        float* __restrict__ norm_out, float* __restrict__ coef,
                                                        unsigned* __restrict__ skips, int step, float lr, float b1,
                                                        float b2) {
  __shared__ double red[256];
  double s = 0.0;
  for (int p = threadIdx.x; p < nparts; p += 256) s += part[p];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const float norm = (float)sqrt(red[0]);
  if (norm_out) norm_out[0] = norm;
  float c = 1.f;
  if (max_norm > 0.f) {
    c = max_norm / (norm + 1e-6f);
    if (c > 1.f) c = 1.f;
  }
  coef[0] = c;
  // a non-finite norm (a persistent recurrence that gave up writes NaN; in data-parallel training
  // the NaN reaches every rank through the all-reduce): the update below is skipped
  coef[1] = isfinite(norm) ? 0.f : 1.f;
  // device count of skipped updates (avc_clip_adam_ema_dev): Adam's bias correction of this update
  // uses step - skips, so the host never has to wait for the norm to know the step
  unsigned sk = skips ? *skips : 0u;
  if (skips && !isfinite(norm)) *skips = ++sk;
  coef[2] = __uint_as_float(sk);
  // the bias corrections of effective step max(1, step - sk), formed here in double as the host
  // forms its table (clip_adam_ema): adam_ema_kernel takes these where sk is past the table, so
  // any number of skipped updates between two settles keeps torch.optim.Adam's step
  const int st = (int)max(1L, (long)step - (long)sk);
  coef[3] = (float)((double)lr / (1.0 - pow((double)b1, (double)st)));
  coef[4] = (float)sqrt(1.0 - pow((double)b2, (double)st));
}

constexpr int kAdamTab = 8;
struct AdamArgs {
  float c, lr, b1, b2, eps, wd, step_size, bc2_sqrt, ema_decay, ema_keep;
  int clip;
  int guard;  // coef[1] holds the skip flag of clip_coef_kernel
  int tabled;  // step_size / bc2_sqrt from the tables below, indexed by the device skip count coef[2]
               // (coef[3] / coef[4], formed by clip_coef_kernel, past the table's end)
  float ss[kAdamTab], bc[kAdamTab];  // the host's values for effective steps step, step - 1, ...
};

// ema_decay * avg + keep * p with both products rounded (HIP's __fmul_rn is a plain multiply, so
// without this the compiler may contract the sum into an fma: measured 4-ulp EMA drift vs torch)
__device__ __forceinline__ float ema_blend(float decay, float avg, float keep, float p) {
#pragma clang fp contract(off)
  return decay * avg + keep * p;
}

// one element of the fused clip + Adam + EMA update (torch.optim.Adam's foreach arithmetic)
__device__ __forceinline__ void adam_elem(const AdamArgs& a, float& pi, float& gi, float& mi, float& vi,
                                          float& ei, bool has_e) {
  if (a.clip) gi *= a.c;
  float gw = gi;
  if (a.wd != 0.f) gw += a.wd * pi;
  mi = mi + (1.f - a.b1) * (gw - mi);  // torch foreach Adam: exp_avg.lerp_(g, 1-b1)
  vi = a.b2 * vi + (1.f - a.b2) * gw * gw;
  const float denom = sqrtf(vi) / a.bc2_sqrt + a.eps;
  pi -= a.step_size * (mi / denom);
  // torch: ema_decay * avg + (1 - ema_decay) * flat  (two rounded products, one rounded sum;
  // 1 - ema_decay formed in double on the host like the Python scalar)
  if (has_e) ei = ema_blend(a.ema_decay, ei, a.ema_keep, pi);
}

// float4 form over the first n4 * 4 elements (all five arrays 16-byte aligned), scalar tail
__global__ __launch_bounds__(256) void adam_ema_kernel(long n, long n4, float* __restrict__ p, float* __restrict__ g,
                                                       float* __restrict__ m, float* __restrict__ v,
                                                       float* __restrict__ ema, const float* __restrict__ coef,
                                                       AdamArgs a) {
  if (a.guard && coef[1] != 0.f) return;  // non-finite gradient norm: parameters, moments, EMA kept
  a.c = a.clip ? coef[0] : 1.f;
  if (a.tabled) {
    // table entry k by selects: a dynamic index into the by-value arguments put the whole struct
    // in scratch, and every element's update read its scalars from there (adam 218 -> 297 us at C3)
    // (k >= kAdamTab: the device's own values for step - k)
    const unsigned k = __float_as_uint(coef[2]);
    float ss = coef[3], bc = coef[4];
#pragma unroll
    for (int j = 0; j < kAdamTab; ++j) {
      ss = k == (unsigned)j ? a.ss[j] : ss;
      bc = k == (unsigned)j ? a.bc[j] : bc;
    }
    a.step_size = ss;
    a.bc2_sqrt = bc;
  }
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 p4 = reinterpret_cast<float4*>(p)[i], g4 = reinterpret_cast<float4*>(g)[i];
    float4 m4 = reinterpret_cast<float4*>(m)[i], v4 = reinterpret_cast<float4*>(v)[i];
    const bool he = ema != nullptr;
    float4 e4 = he ? reinterpret_cast<float4*>(ema)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    adam_elem(a, p4.x, g4.x, m4.x, v4.x, e4.x, he);
    adam_elem(a, p4.y, g4.y, m4.y, v4.y, e4.y, he);
    adam_elem(a, p4.z, g4.z, m4.z, v4.z, e4.z, he);
    adam_elem(a, p4.w, g4.w, m4.w, v4.w, e4.w, he);
    if (a.clip) reinterpret_cast<float4*>(g)[i] = g4;
    reinterpret_cast<float4*>(m)[i] = m4;
    reinterpret_cast<float4*>(v)[i] = v4;
    reinterpret_cast<float4*>(p)[i] = p4;
    if (ema) reinterpret_cast<float4*>(ema)[i] = e4;
  }
  for (long i = 4 * n4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) {
    float pi = p[i], gi = g[i], mi = m[i], vi = v[i], ei = ema ? ema[i] : 0.f;
    adam_elem(a, pi, gi, mi, vi, ei, ema != nullptr);
    if (ema) ema[i] = ei;
    if (a.clip) g[i] = gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

}  // namespace

// ---- internal API --------------------------------------------------------------------------
size_t colsum_scratch(int M, int N) {
  int R, rp;
  colsum_geometry(M, N, R, rp);
  return (size_t)R * N * sizeof(float) + 256;
}

int colsum(avc_context* ctx, int M, int N, const float* X, long ld, float* out, int accumulate,
           hipStream_t s, float* out2) {
  int R, rp;
  colsum_geometry(M, N, R, rp);
  Scratch sc(ctx);
  AVC_TAKE(part, float, (size_t)R * N, sc);
  colsum_partial_kernel<<<dim3((N + 255) / 256, R), 256, 0, s>>>(M, N, X, ld, rp, part);
  colsum_final_kernel<<<(N + 63) / 64, 1024, 0, s>>>(R, N, part, out, accumulate, out2);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int bn_finalize(int C, int nparts, int part_rows, const float* stats, double count, int training, float momentum,
                float eps, float* rmean, float* rvar, float* mean, float* invstd, hipStream_t s,
                unsigned* amax_init) {
  bn_finalize_kernel<<<(C + 63) / 64, 256, 0, s>>>(C, nparts, part_rows, stats, count, training, momentum,
                                                   eps, rmean, rvar, mean, invstd, amax_init);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int bn_apply(long M, int C, const float* y, const float* mean, const float* invstd,
             const float* gamma, const float* beta, int act, const float* residual, float* out,
             hipStream_t s, _Float16* frag, unsigned* range_flag, unsigned* amax_out) {
  AVC_CHECK_ARG(C % 4 == 0, "bn_apply: channels must be a multiple of 4");
  if (frag) {
    AVC_CHECK_ARG(C % 8 == 0, "bn_apply: the split output needs channels in multiples of 8");
    const int nkc = (C + 31) / 32 * 2;
    const long ntile = (M + 31) / 32;
    const long total = ntile * 32 * nkc * 2;
    // with max words every workgroup ends in an atomic max on one word: fewer, longer workgroups
    bn_apply_frag_kernel<<<(int)std::min<long>((total + 255) / 256, amax_out ? 512 : 8192), 256, 0, s>>>(
        M, C, nkc, ntile, y, mean, invstd, gamma, beta, act, residual, out, frag, range_flag, amax_out);
    AVC_LAUNCH_CHECK();
    return AVC_OK;
  }
  // ~4 float4 per thread; every thread owns one channel quad for the whole launch
  const long Q = C / 4;
  // with max words every workgroup ends in an atomic max on one word: fewer, longer workgroups
  const long threads = std::max<long>(256, std::min<long>(M * Q / 4, (amax_out ? 512L : 2048L) * 256));
  const long blocks = (threads + 255) / 256;
  bn_apply_kernel<<<(int)blocks, 256, 0, s>>>(M, C, y, mean, invstd, gamma, beta, act, residual, out, range_flag,
                                              amax_out);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

namespace {
// row blocks of the BN backward (a function of the shape only: callers size the bias partials
// with bn_backward_rows): ~64 rows per block
bool bn_vec_ok(int C, const float* dout, const float* y, const float* dy) {
  return C % 4 == 0 && C <= 1024 && aligned16(dout) && aligned16(y) && aligned16(dy);
}
void bn_geometry(int M, int C, int& R, int& rows_per) {
  if (C % 4 != 0 || C > 1024) {
    colsum_geometry(M, C, R, rows_per);
    return;
  }
  R = std::max(1, std::min(512, (M + 63) / 64));
  rows_per = (M + R - 1) / R;
  R = (M + rows_per - 1) / rows_per;
}
}  // namespace

size_t bn_backward_scratch(int M, int C) {
  int R, rp;
  bn_geometry(M, C, R, rp);
  return (size_t)R * 2 * C * sizeof(float) + 2 * C * sizeof(float) + 512;
}


int bn_backward(avc_context* ctx, int M, int C, const float* dout, const float* y,
                const float* mean, const float* invstd, const float* gamma, const float* beta,
                int act, int training, float* d_gamma, float* d_beta, int accumulate, float* dy,
                hipStream_t s, float* dy_colpart, unsigned* dy_amax) {
  const bool vec = bn_vec_ok(C, dout, y, dy);
  int R, rp;
  bn_geometry(M, C, R, rp);
  Scratch sc(ctx);
  AVC_TAKE(part, float, (size_t)R * 2 * C, sc);
  AVC_TAKE(sums, float, (size_t)2 * C, sc);
  if (vec) {
    bn_bwd_reduce4_kernel<<<dim3(1, R), 256, 0, s>>>(M, C, dout, y, mean, invstd, gamma, beta, act, rp, part, nullptr, nullptr);
  } else {
    bn_bwd_reduce_kernel<<<dim3((C + 255) / 256, R), 256, 0, s>>>(M, C, dout, y, mean, invstd, gamma,
                                                                  beta, act, rp, part);
  }
  bn_bwd_final_kernel<<<(C + 63) / 64, 1024, 0, s>>>(R, C, part, sums, d_gamma, d_beta, accumulate, dy_amax, BnBound{});
  if (vec) {
    bn_bwd_apply4_kernel<<<dim3(1, R), 256, 0, s>>>(M, C, dout, y, mean, invstd, gamma, beta, act, training, sums,
                                                    1.f / (float)M, rp, dy, dy_colpart, dy_amax);
  } else if (dy_colpart || dy_amax) {
    bn_bwd_apply_cols_kernel<<<dim3((C + 255) / 256, R), 256, 0, s>>>(M, C, dout, y, mean, invstd, gamma, beta,
                                                                      act, training, sums, 1.f / (float)M, rp, dy,
                                                                      dy_colpart, dy_amax);
  } else {
    bn_bwd_apply_kernel<<<ew_blocks((long)M * C), 256, 0, s>>>(M, C, dout, y, mean, invstd, gamma,
                                                                beta, act, training, sums,
                                                                1.f / (float)M, dy);
  }
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int bn_backward_rows(int M, int C) {
  int R, rp;
  bn_geometry(M, C, R, rp);
  return R;
}

bool bn_backward_frag_ok(int M, int C, const float* dout, const float* y) {
  return C % 4 == 0 && C <= 1024 && aligned16(dout) && aligned16(y) && M > 0;
}

int bn_backward_frag(avc_context* ctx, int M, int C, const float* dout, const float* y, const float* mean,
                     const float* invstd, const float* gamma, const float* beta, int act, int training,
                     float* d_gamma, float* d_beta, int accumulate, _Float16* imgA, _Float16* imgT,
                     unsigned* bound, hipStream_t s, float* dy_colpart) {
  AVC_CHECK_ARG(bn_backward_frag_ok(M, C, dout, y), "bn_backward_frag: C must be a multiple of 4 (<= 1024), rows 16-B aligned");
  int R, rp;
  bn_geometry(M, C, R, rp);
  Scratch sc(ctx);
  AVC_TAKE(part, float, (size_t)R * 2 * C, sc);
  AVC_TAKE(mpart, float, (size_t)R * 3 * C, sc);
  AVC_TAKE(sums, float, (size_t)2 * C, sc);
  bn_bwd_reduce4_kernel<<<dim3(1, R), 256, 0, s>>>(M, C, dout, y, mean, invstd, gamma, beta, act, rp, part, mpart, bound);
  BnBound bb;
  bb.mpart = mpart; bb.gamma = gamma; bb.invstd = invstd; bb.inv_count = 1.f / (float)M;
  bb.training = training; bb.bound = bound;
  bn_bwd_final_kernel<<<(C + 63) / 64, 1024, 0, s>>>(R, C, part, sums, d_gamma, d_beta, accumulate, nullptr, bb);
  const int nkcA = (C + 31) / 32 * 2, nkcT = (M + 31) / 32 * 2;
  bn_bwd_apply_frag_kernel<<<dim3((C + 127) / 128, (M + 31) / 32), 256, 0, s>>>(
      M, C, dout, y, mean, invstd, gamma, beta, act, training, sums, 1.f / (float)M, bound, imgA, nkcA, imgT, nkcT,
      dy_colpart);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int bn_backward_frag_rows(int M) { return (M + 31) / 32; }

size_t bn_backward_frag_scratch(int M, int C) { return bn_backward_scratch(M, C) + (size_t)bn_backward_rows(M, C) * 3 * C * sizeof(float) + 256; }

int colsum_finish(int R, int N, const float* part, float* out, int accumulate, hipStream_t s) {
  colsum_final_kernel<<<(N + 63) / 64, 1024, 0, s>>>(R, N, part, out, accumulate, nullptr);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int frames_from_mel(int T, int B, int cm, const float* x, int ce, const float* emb, float* out,
                    hipStream_t s) {
  frames_from_mel_kernel<<<ew_blocks((long)T * B * (cm + ce)), 256, 0, s>>>(T, B, cm, x, ce, emb, out);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int frames_from_mel_frag(avc_context* ctx, int T, int B, int cm, const float* x, int ce, const float* emb,
                         _Float16* frag, unsigned* guard, hipStream_t s) {
  if (!ctx->guard_ticket) {  // (as guard_scan: the first use happens eagerly, before any capture)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    AVC_HIP(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) {
      set_error("frames range guard: ticket not allocated before graph capture");
      return AVC_ERR_WORKSPACE;
    }
    AVC_HIP(hipMalloc(&ctx->guard_ticket, 256));
    AVC_HIP(hipMemsetAsync(ctx->guard_ticket, 0, 256, s));
    AVC_HIP(hipStreamSynchronize(s));
  }
  Scratch sc(ctx);
  const int nkc0 = (cm + ce + 31) / 32 * 2;
  if (T % 4 == 0 && B % 32 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const long total4 = (long)(T / 4) * nkc0 * 2 * B;
    const int blocks = (int)std::min<long>((total4 + 255) / 256, 8192);
    AVC_TAKE(partm, float, blocks, sc);
    frames_frag_guard_kernel<<<blocks, 256, 0, s>>>(T, B, cm, x, ce, emb, nkc0, partm, ctx->guard_ticket, guard, frag);
    AVC_LAUNCH_CHECK();
    return AVC_OK;
  }
  AVC_TAKE(part, float, 256, sc);
  const long nx = (long)B * cm * T, ne = (long)B * ce;
  frames_guard_kernel<<<(int)std::max<long>(1, std::min<long>((nx + ne + 1023) / 1024, 256)), 256, 0, s>>>(
      x, nx, emb, ne, part, ctx->guard_ticket, guard);
  const int nkc = (cm + ce + 31) / 32 * 2;
  const long ntile = ((long)T * B + 31) / 32, total = ntile * 32 * nkc * 2;
  frames_frag_kernel<<<(int)std::min<long>((total + 255) / 256, 8192), 256, 0, s>>>(T, B, cm, x, ce, emb, nkc, ntile,
                                                                                   guard + 1, frag);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int frames_from_mel_backward(int T, int B, int cm, int ce, const float* df, int ld, float* dx,
                             float* demb, int accumulate, hipStream_t s) {
  if (dx) mel_grad_kernel<<<ew_blocks((long)B * cm * T), 256, 0, s>>>(T, B, cm, df, ld, dx, accumulate);
  if (demb && ce > 0)
    emb_grad_kernel<<<(B * ce + 255) / 256, 256, 0, s>>>(T, B, cm, ce, df, ld, demb, accumulate);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

// Stream-ordered zeroing by a kernel of our own.  hipMemsetAsync is NOT used anywhere in the
// library: on ROCm 7.2 a memset issued ahead of a persistent (spin-waiting) launch was measured to
// land out of order with it (stale counters -> wrong recurrence outputs in the first calls of a
// process; scripts/persist_repeat.py "modes"), while a kernel is ordered like every other launch.
__global__ void zero_bytes_kernel(unsigned char* __restrict__ p, size_t n, unsigned v) {
  const size_t n16 = n / 16;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    reinterpret_cast<uint4*>(p)[i] = make_uint4(v, v, v, v);
  const size_t tail = n16 * 16 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tail < n) p[tail] = (unsigned char)(v >> (8 * (tail & 3)));
}

// fill with a repeated 32-bit pattern (zero_async's kernel); p 16-byte aligned
int fill_async(void* p, size_t bytes, unsigned v, hipStream_t s) {
  if (bytes == 0) return AVC_OK;
  AVC_CHECK_ARG(p != nullptr && (reinterpret_cast<uintptr_t>(p) & 15) == 0, "fill_async: NULL or unaligned");
  const size_t n16 = bytes / 16;
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>((n16 + 255) / 256, 2048));
  zero_bytes_kernel<<<blocks, 256, 0, s>>>(static_cast<unsigned char*>(p), bytes, v);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int zero_async(void* p, size_t bytes, hipStream_t s) { return fill_async(p, bytes, 0u, s); }

constexpr int kZeroPool = 16384;  // words (64 KiB)

unsigned* zeroed_words(avc_context* ctx, int n, hipStream_t s) {
  if (n <= 0 || n > 64) {
    set_error("zeroed_words: 1..64 words");
    return nullptr;
  }
  const int take = (n + 15) / 16 * 16;  // 64-byte granules
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess) cs = hipStreamCaptureStatusActive;
  if (!ctx->zpool) {
    if (hipMalloc(&ctx->zpool, kZeroPool * sizeof(unsigned)) != hipSuccess) {
      ctx->zpool = nullptr;
      set_error("zeroed_words: hipMalloc failed");
      return nullptr;
    }
    ctx->zpool_next = kZeroPool;  // forces the first zeroing below
  }
  if (ctx->zpool_next + take > kZeroPool) {
    if (zero_async(ctx->zpool, kZeroPool * sizeof(unsigned), s) != AVC_OK) return nullptr;
    ctx->zpool_next = 0;
  }
  unsigned* p = ctx->zpool + ctx->zpool_next;
  ctx->zpool_next += take;
  if (cs != hipStreamCaptureStatusNone && zero_async(p, take * sizeof(unsigned), s) != AVC_OK) return nullptr;
  return p;
}

int mel_from_frames(int T, int B, int cm, const float* fr, float* mel, hipStream_t s, const float* fr1,
                    float* mel1) {
  mel_from_frames_kernel<<<dim3(ew_blocks((long)B * cm * T), fr1 ? 2 : 1), 256, 0, s>>>(T, B, cm, fr, mel, fr1, mel1);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int codes_from_encoder(int T, int B, const float* enc, float* codes, hipStream_t s) {
  AVC_CHECK_ARG(T >= 32, "content codes need T >= 32 frames (model.py:99 cat of an empty list)");
  const long total = (long)B * 32 * (T / 32 + (T + 31) / 32);
  codes_kernel<<<ew_blocks(total), 256, 0, s>>>(T, B, enc, codes, 0, 0, nullptr);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int codes_from_encoder_backward(int T, int B, const float* dcodes, float* denc, int accumulate,
                                hipStream_t s) {
  AVC_CHECK_ARG(T >= 32, "content codes need T >= 32 frames");
  if (!accumulate) AVC_TRY(zero_async(denc, sizeof(float) * (size_t)T * B * 64, s));
  const long total = (long)B * 32 * (T / 32 + (T + 31) / 32);
  codes_kernel<<<ew_blocks(total), 256, 0, s>>>(T, B, nullptr, const_cast<float*>(dcodes), 1, 1, denc);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int decoder_input(int T, int B, const float* enc, int ce, const float* ctrg, float* out,
                  hipStream_t s, unsigned* range_flag, float* codes) {
  AVC_CHECK_ARG(T >= 32, "decoder input needs T >= 32 frames (model.py:115-119)");
  const auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (ce % 4 == 0 && a16(enc) && a16(ctrg) && a16(out) && (!codes || a16(codes))) {
    decoder_input4_kernel<<<ew_blocks((long)T * B * ((64 + ce) / 4)), 256, 0, s>>>(T, B, enc, ce, ctrg, out,
                                                                                   range_flag, codes);
    AVC_LAUNCH_CHECK();
    return AVC_OK;
  }
  if (codes) AVC_TRY(codes_from_encoder(T, B, enc, codes, s));
  decoder_input_kernel<<<ew_blocks((long)T * B * (64 + ce)), 256, 0, s>>>(T, B, enc, ce, ctrg, out, range_flag);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int decoder_input_backward(int T, int B, int ce, const float* dd, float* denc, int accumulate,
                           hipStream_t s) {
  AVC_CHECK_ARG(T >= 32, "decoder input needs T >= 32 frames");
  if (!accumulate) AVC_TRY(zero_async(denc, sizeof(float) * (size_t)T * B * 64, s));
  const long total = (long)B * (T / 32 + (T + 31) / 32) * 32;
  decoder_input_bwd_kernel<<<ew_blocks(total), 256, 0, s>>>(T, B, ce, dd, denc);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int overlap_average(int M, int C, int N, int step, const float* fr, float* out, hipStream_t s) {
  AVC_CHECK_ARG(M >= 1 && C >= 1 && N >= 1 && step >= 0, "overlap_average: bad shape");
  const long total = (long)C * ((M - 1) * step + N);
  overlap_average_kernel<<<ew_blocks(total), 256, 0, s>>>(M, C, N, step, fr, out);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int overlap_average_backward(int M, int C, int N, int step, const float* fr, const float* dout, float* dfr,
                             hipStream_t s) {
  AVC_CHECK_ARG(M >= 1 && C >= 1 && N >= 1 && step >= 0, "overlap_average_backward: bad shape");
  const long total = (long)M * C * N;
  overlap_average_backward_kernel<<<ew_blocks(total), 256, 0, s>>>(M, C, N, step, fr, dout, dfr);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

size_t loss_scratch() { return 1024 * sizeof(double) + 256; }

int loss_forward(avc_context* ctx, int kind, size_t n, const float* a, const float* b,
                 float* out, int accumulate, hipStream_t s) {
  AVC_CHECK_ARG(kind == 0 || kind == 1, "loss kind must be 0 (MSE) or 1 (L1)");
  AVC_CHECK_ARG(n > 0, "loss over an empty tensor");
  Scratch sc(ctx);
  const int nb = (int)std::min<size_t>(1024, (n + 255) / 256);
  AVC_TAKE(part, double, (size_t)nb, sc);
  loss_partial_kernel<<<nb, 256, 0, s>>>(kind, (long)n, a, b, part);
  loss_final_kernel<<<1, 256, 0, s>>>(nb, part, 1.0 / (double)n, out, accumulate);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int loss_backward(int kind, size_t n, const float* a, const float* b, const float* dscale,
                  float* ga, float* gb, int accumulate, hipStream_t s) {
  AVC_CHECK_ARG(kind == 0 || kind == 1, "loss kind must be 0 (MSE) or 1 (L1)");
  loss_grad_kernel<<<ew_blocks((long)n), 256, 0, s>>>(kind, (long)n, a, b, dscale,
                                                      1.0f / (float)n, ga, gb, accumulate);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

size_t optimizer_scratch() { return 2048 * sizeof(double) + 512; }

int clip_adam_ema(avc_context* ctx, size_t n, float* p, float* g, float* m, float* v, float* ema,
                  float lr, float b1, float b2, float eps, float wd, int step, float max_norm,
                  double ema_decay, float* norm_out, hipStream_t s, unsigned* skips) {
  AVC_CHECK_ARG(step >= 1, "adam step counter starts at 1");
  AVC_CHECK_ARG(!skips || max_norm > 0.f || norm_out, "adam skip count: needs the gradient norm");
  Scratch sc(ctx);
  const int nb = (int)std::min<size_t>(2048, (n + 255) / 256);
  AVC_TAKE(part, double, (size_t)nb, sc);
  AVC_TAKE(coef, float, 8, sc);
  const bool need_norm = max_norm > 0.f || norm_out != nullptr;
  if (need_norm) {
    sumsq_partial_kernel<<<nb, 256, 0, s>>>((long)n, g, part);
    clip_coef_kernel<<<1, 256, 0, s>>>(nb, part, max_norm, norm_out, coef, skips, step, lr, b1, b2);
  }
  AdamArgs a{};
  a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd;
  // torch.optim.Adam's bias corrections in double (Python floats), for this step and, with a
  // device skip count, for the steps it would be after k skipped updates
  for (int k = 0; k < kAdamTab; ++k) {
    const int st = std::max(1, step - k);
    const double bc1 = 1.0 - std::pow((double)b1, st);
    const double bc2 = 1.0 - std::pow((double)b2, st);
    a.ss[k] = (float)(lr / bc1);
    a.bc[k] = (float)std::sqrt(bc2);
  }
  a.step_size = a.ss[0];
  a.bc2_sqrt = a.bc[0];
  a.tabled = skips ? 1 : 0;
  a.ema_decay = (float)ema_decay;
  a.ema_keep = (float)(1.0 - ema_decay);
  a.clip = max_norm > 0.f ? 1 : 0;
  a.guard = need_norm ? 1 : 0;
  const bool al = aligned16(p) && aligned16(g) && aligned16(m) && aligned16(v) && (!ema || aligned16(ema));
  const long n4 = al ? (long)n / 4 : 0;
  adam_ema_kernel<<<ew_blocks(std::max<long>(n4, (long)n - 4 * n4)), 256, 0, s>>>((long)n, n4, p, g, m, v, ema, coef, a);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

}  // namespace avc
