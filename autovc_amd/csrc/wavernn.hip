// WaveRNN vocoder `generate` (autovc/wavernn/model.py:214-329,
// autovc/wavernn/distribution.py:87-123) on gfx950.
//
// The work splits into a parallel prologue and a strictly sequential sample loop:
//   * up-sampling (model.py:34-93, eval-mode BN): MelResNet as frame-row kernels, the mel's
//     Stretch2d + (1, 2s+1) smoothing as three stencil passes; the aux features stay at frame
//     rate (the ×275 stretch is an index, never materialised), the fold into target + 2·overlap
//     rows (model.py:296-339) is an index too;
//   * the input layer's mel / aux part, which does not depend on the sampled signal, is
//     contracted for every sample position up front (pI = W_I[:, 1:] · [m; a1] + b_I); per step
//     only W_I[:, 0] · x_prev remains;
//   * the loop: per sample step five dependent launches over every fold row at once — GRU1,
//     GRU2, fc1, fc2, fc3 + sampling — captured into a hipGraph in chunks of kChunk steps and
//     replayed.  The step index lives in device memory (the sampling kernel's last workgroup
//     advances it), so one captured chunk serves every position.  Each step streams ~17 MB of
//     weights, spread over 128-256 workgroups so that each pulls at most ~50 KB from its XCD's L2;
//     with a stable block -> XCD placement an XCD keeps its eighth of the weights L2-resident
//     across steps.  What bounds a step is the chain of five kernel boundaries (~1.3 us each,
//     MI355X_MICROARCH.md 'boundary') plus each kernel's load -> reduce -> store latency.
//   * sampling uses a counter-based stream (splitmix64 of (row, step, draw)), restated by the
//     oracle, in place of torch's global RNG; the cross-fade and fade-out (model.py:316-329,
//     341-399) run in float64 like the reference's numpy.
#include <algorithm>
#include <cmath>

#include "kernels.h"
#include "timing.h"

namespace avc {
namespace {

inline int ew(long n) { return (int)std::max<long>(1, std::min<long>((n + 255) / 256, 65536)); }

// ---- up-sampling network ------------------------------------------------------------------

// (80, T) channel-major mel -> the generate() padding (2 zero frames each side, model.py:250)
// in both layouts the next kernels read: time-major [T+2p][C] and channel-major [C][T+2p].
__global__ void wr_pad_mel_kernel(int C, int T, int pad, const float* __restrict__ mel, float* __restrict__ tm,
                                  float* __restrict__ cm) {
  const int Tp = T + 2 * pad;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < (long)C * Tp; idx += (long)gridDim.x * 256) {
    const int c = (int)(idx / Tp), q = (int)(idx - (long)c * Tp);
    const float v = (q >= pad && q < pad + T) ? mel[(long)c * T + q - pad] : 0.f;
    cm[idx] = v;
    tm[(long)q * C + c] = v;
  }
}

// One MelResNet layer over frame rows (model.py:24-31, 41-49):
//   out[t][n] = act(bn_eval(sum_{k, tap} W[n][k][tap] · in[t + tap][k] + bias[n])) (+ res[t][n])
// with valid (unpadded) taps: Tout = Tin - taps + 1.  BN eval as alpha·x + beta
// (alpha = gamma / sqrt(var + eps), beta = beta - mean·alpha), then ReLU, then the residual.
__global__ void wr_frame_layer_kernel(int Tout, int Cin, int Cout, int taps, const float* __restrict__ in,
                                      const float* __restrict__ W, const float* __restrict__ bias,
                                      const float* __restrict__ g, const float* __restrict__ b,
                                      const float* __restrict__ rm, const float* __restrict__ rv, int relu,
                                      const float* __restrict__ res, float* __restrict__ out) {
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < (long)Tout * Cout; idx += (long)gridDim.x * 256) {
    const int t = (int)(idx / Cout), n = (int)(idx - (long)t * Cout);
    const float* w = W + (long)n * Cin * taps;
    float s = 0.f;
    for (int k = 0; k < Cin; ++k) {
#pragma unroll 1
      for (int tap = 0; tap < taps; ++tap) s = fmaf(w[k * taps + tap], in[(long)(t + tap) * Cin + k], s);
    }
    if (bias) s += bias[n];
    if (g) {
      const float alpha = g[n] / sqrtf(rv[n] + 1e-5f);
      s = s * alpha + (b[n] - rm[n] * alpha);
    }
    if (relu) s = fmaxf(s, 0.f);
    if (res) s += res[idx];
    out[idx] = s;
  }
}

// Stretch2d(s, 1) + Conv2d(1, 1, (1, 2s+1), padding (0, s)) along time (model.py:52-63, 79-92):
//   out[c][j] = sum_u w[u] · xs[c][j + u - s],  xs[c][q] = in[c][q / s] for 0 <= q < Lin·s, else 0.
// final != 0: write the cropped (indent on both sides), time-major [Lout - 2·indent][C] result.
__global__ void wr_stretch_conv_kernel(int C, int Lin, int s, const float* __restrict__ w, const float* __restrict__ in,
                                       float* __restrict__ out, int final_crop, int indent) {
  const long Lout = (long)Lin * s;
  const long Lw = final_crop ? Lout - 2L * indent : Lout;
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < (long)C * Lw; idx += (long)gridDim.x * 256) {
    long j;
    int c;
    if (final_crop) {
      const long q = idx / C;
      c = (int)(idx - q * C);
      j = q + indent;
    } else {
      c = (int)(idx / Lout);
      j = idx - (long)c * Lout;
    }
    const float* row = in + (long)c * Lin;
    float acc = 0.f;
    for (int u = 0; u <= 2 * s; ++u) {
      const long q = j + u - s;
      const float v = (q >= 0 && q < Lout) ? row[q / s] : 0.f;
      acc = fmaf(w[u], v, acc);
    }
    out[idx] = acc;
  }
}

// pI[src][q][u] = b_I[u] + W_I[u][1:1+F] · m[src][q] + W_I[u][1+F:1+F+A] · aux[src][q / hop][0:A],
// for q < Ltot; row q = Ltot holds b_I alone (fold padding: m = aux = 0, model.py:318-321).
__global__ void wr_input_proj_kernel(int nsrc, long Ltot, int H, int F, int A, int hop, int Tf, int auxd,
                                     const float* __restrict__ m, const float* __restrict__ auxf,
                                     const float* __restrict__ WI, const float* __restrict__ bI,
                                     float* __restrict__ pI) {
  const int K = 1 + F + A;
  const long rows = (long)nsrc * (Ltot + 1);
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < rows * H; idx += (long)gridDim.x * 256) {
    const long rq = idx / H;
    const int u = (int)(idx - rq * H);
    const int src = (int)(rq / (Ltot + 1));
    const long q = rq - (long)src * (Ltot + 1);
    float s = 0.f;
    if (q < Ltot) {
      const float* w = WI + (long)u * K + 1;
      const float* mv = m + ((long)src * Ltot + q) * F;
      for (int k = 0; k < F; ++k) s = fmaf(w[k], mv[k], s);
      const float* av = auxf + ((long)src * Tf + q / hop) * auxd;
      for (int k = 0; k < A; ++k) s = fmaf(w[F + k], av[k], s);
    }
    pI[idx] = s + bI[u];
  }
}

// The same pI, tiled: a workgroup forms 64 position rows x 64 units (4 x 4 per thread) with the
// operand chunks (32 k) staged in LDS; every output's FMA chain runs over k in the order above
// (m, then aux; padding rows q = Ltot multiply zeros into +0), so the bits are
// wr_input_proj_kernel's.  (The per-thread form re-read each row of m and W_I from memory for
// every output: 42 ms per 10 s utterance, 7 % of generate().)
__global__ __launch_bounds__(256) void wr_input_proj_tiled_kernel(int nsrc, long Ltot, int H, int F, int A, int hop,
                                                                  int Tf, int auxd, const float* __restrict__ m,
                                                                  const float* __restrict__ auxf,
                                                                  const float* __restrict__ WI,
                                                                  const float* __restrict__ bI,
                                                                  float* __restrict__ pI) {
  constexpr int TR = 64, TU = 64, KC = 32;
  __shared__ float xs[TR][KC + 1];
  __shared__ float ws[TU][KC + 1];
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  const long rows = (long)nsrc * (Ltot + 1);
  const long r0 = (long)blockIdx.x * TR;
  const int u0 = blockIdx.y * TU;
  const int KF = F + A, Kw = 1 + F + A;
  float acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = 0.f;
  for (int k0 = 0; k0 < KF; k0 += KC) {
    for (int e = tid; e < TR * KC; e += 256) {
      const int rr = e / KC, kk = e - rr * KC, k = k0 + kk;
      const long rq = r0 + rr;
      float x = 0.f;
      if (rq < rows && k < KF) {
        const int src = (int)(rq / (Ltot + 1));
        const long q = rq - (long)src * (Ltot + 1);
        if (q < Ltot)
          x = k < F ? m[((long)src * Ltot + q) * F + k] : auxf[((long)src * Tf + q / hop) * auxd + (k - F)];
      }
      xs[rr][kk] = x;
    }
    for (int e = tid; e < TU * KC; e += 256) {
      const int uu = e / KC, kk = e - uu * KC, k = k0 + kk, u = u0 + uu;
      ws[uu][kk] = (u < H && k < KF) ? WI[(long)u * Kw + 1 + k] : 0.f;
    }
    __syncthreads();
    const int kn = min(KC, KF - k0);
    for (int kk = 0; kk < kn; ++kk) {
      float xv[4], wv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) xv[a] = xs[ty * 4 + a][kk];
#pragma unroll
      for (int b = 0; b < 4; ++b) wv[b] = ws[tx * 4 + b][kk];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = fmaf(wv[b], xv[a], acc[a][b]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const long rq = r0 + ty * 4 + a;
    if (rq >= rows) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int u = u0 + tx * 4 + b;
      if (u < H) pI[rq * H + u] = acc[a][b] + bI[u];
    }
  }
}

// ---- the sample loop ------------------------------------------------------------------------

struct WrStep {
  int R, L, H, Fc, A, NC, auxd, hop, Tf;
  long Ltot, stride;      // stride = target + overlap (batched), 0 = one source row per fold row
  int batched, mol, teacher;
  unsigned long long seed;
  int* step;              // current step (device); advanced by wr_out_kernel's last workgroup
  int* done;              // arrivals of wr_out_kernel's workgroups in the current step
  const float* pI;        // [nsrc][Ltot + 1][H]
  const float* auxf;      // [nsrc][Tf][auxd] frame-rate aux features
  const float* WI; long wi_ld;  // I.weight: column 0 multiplies x_prev
  const float* wi0;       // I.weight[:, 0], contiguous
  const float *Wih1, *Whh1, *bih1, *bhh1, *Wih2, *Whh2, *bih2, *bhh2;
  const float *W1, *b1, *W2, *b2, *W3, *b3;
  float *x_prev, *h1, *h2, *t1, *t2, *y1, *y2;  // h1 / h2: [2][R][H] (step parity)
  float* out;             // [R][L] samples
  float* logits;          // teacher mode: [R][L][NC]
  const float* x_tf;      // teacher mode: [R][L] previous samples
};

__device__ __forceinline__ int cur_step(const WrStep& a) {
  return __hip_atomic_load(a.step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// source row and position of fold row r at step i (valid positions < Ltot; fold padding reads
// the pI row Ltot and zero aux)
__device__ __forceinline__ void fold_pos(const WrStep& a, int r, int i, int& src, long& q) {
  src = a.batched ? 0 : r;
  q = a.batched ? (long)r * a.stride + i : (long)i;
  if (q > a.Ltot) q = a.Ltot;
}

__device__ __forceinline__ float aux_at(const WrStep& a, int src, long q, int k) {
  return q < a.Ltot ? a.auxf[((long)src * a.Tf + q / a.hop) * a.auxd + k] : 0.f;
}

// the previous sample a step consumes: the last draw, or (teacher-forced, model.py:195-197) the
// given sequence at the same index
__device__ __forceinline__ float xprev_at(const WrStep& a, int r, int i) {
  return a.teacher ? a.x_tf[(long)r * a.L + i] : a.x_prev[r];
}

constexpr int kRC = 24;  // fold rows per LDS chunk
constexpr int kKJ = 9;   // K <= 64 * kKJ = 576 (staging capacity)
constexpr int kJ4 = 3;   // float4 k4 = lane + 64 j4, j4 < kJ4 (K / 4 <= 192)
constexpr int kRP = 65;  // padded row of the partial-sum transpose (conflict-free column sums)

// Inputs of the step's contractions (model.py:263-278): K = Kv + A, the vector part, then its
// aux slice a2 / a3 / a4 (xI and the hidden states have no aux part).
enum WrIn : int { IN_XI = 0, IN_H1 = 1, IN_T1A2 = 2, IN_H2 = 3, IN_T2A3 = 4, IN_Y1A4 = 5 };

// Stage rows [rb, rb + kRC) of input `which` (K elements each, K % 4 == 0) into xs[kRC][K] as
// float4s: stage_load brings every float4 of the chunk into registers, stage_store then writes
// LDS, so all loads of a kernel (weights, both inputs, epilogue operands) are in flight together;
// rows past R are zero.
constexpr int kStage4 = (kRC * 576 / 4 + 255) / 256;  // float4s per thread (K <= 576)
__device__ __forceinline__ void stage_load(const WrStep& a, int which, int i, int rb, int K, float4 (&v)[kStage4]) {
  const int cur = i & 1, K4 = K >> 2, H = a.H;
#pragma unroll
  for (int m = 0; m < kStage4; ++m) {
    const int e = threadIdx.x + 256 * m;
    const int rr = e / K4, k = 4 * (e - rr * K4), r = rb + rr;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rr < kRC && r < a.R) {
      int src;
      long q;
      fold_pos(a, r, i, src, q);
      const float* p = nullptr;
      switch (which) {
        case IN_XI: {
          const float4 pi = *reinterpret_cast<const float4*>(a.pI + ((long)src * (a.Ltot + 1) + q) * H + k);
          const float4 w0 = *reinterpret_cast<const float4*>(a.wi0 + k);
          const float xp = xprev_at(a, r, i);
          x = make_float4(fmaf(w0.x, xp, pi.x), fmaf(w0.y, xp, pi.y), fmaf(w0.z, xp, pi.z), fmaf(w0.w, xp, pi.w));
          break;
        }
        case IN_H1: p = a.h1 + ((long)cur * a.R + r) * H + k; break;
        case IN_H2: p = a.h2 + ((long)cur * a.R + r) * H + k; break;
        case IN_T1A2: p = k < H ? a.t1 + (long)r * H + k : nullptr; break;
        case IN_T2A3: p = k < H ? a.t2 + (long)r * H + k : nullptr; break;
        default: p = k < a.Fc ? a.y1 + (long)r * a.Fc + k : nullptr; break;
      }
      if (which != IN_XI) {
        if (p) {
          x = *reinterpret_cast<const float4*>(p);
        } else if (q < a.Ltot) {  // the layer's aux slice
          const int kv = which == IN_Y1A4 ? a.Fc : H;
          const int off = (which == IN_T1A2 ? 1 : which == IN_T2A3 ? 2 : 3) * a.A + (k - kv);
          x = *reinterpret_cast<const float4*>(a.auxf + ((long)src * a.Tf + q / a.hop) * a.auxd + off);
        }
      }
    }
    v[m] = x;
  }
}
__device__ __forceinline__ void stage_store(int K, const float4 (&v)[kStage4], float* xs) {
  const int K4 = K >> 2;
#pragma unroll
  for (int m = 0; m < kStage4; ++m) {
    const int e = threadIdx.x + 256 * m;
    if (e < kRC * K4) reinterpret_cast<float4*>(xs)[e] = v[m];
  }
}

// This wave's NG output rows against the kRC staged rows: lane holds float4 k4 = lane + 64 j4 of
// each row's weights (wv) and reads the same float4 of every staged row; acc[g][rr].
template <int NG>
__device__ __forceinline__ void rows_dot(const float4 (&wv)[NG][kJ4], const float* xs, int K, int lane,
                                         float (&acc)[NG][kRC]) {
  const int K4 = K >> 2;
  const float4* xs4 = reinterpret_cast<const float4*>(xs);
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int rr = 0; rr < kRC; ++rr) acc[g][rr] = 0.f;
#pragma unroll
  for (int j = 0; j < kJ4; ++j) {
    const int k4 = lane + 64 * j;
    if (k4 < K4) {
#pragma unroll
      for (int rr = 0; rr < kRC; ++rr) {
        const float4 x = xs4[rr * K4 + k4];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          float t = acc[g][rr];
          t = fmaf(wv[g][j].x, x.x, t);
          t = fmaf(wv[g][j].y, x.y, t);
          t = fmaf(wv[g][j].z, x.z, t);
          acc[g][rr] = fmaf(wv[g][j].w, x.w, t);
        }
      }
    }
  }
}

// float4 k4 of weight row `row` (K % 4 == 0), zero past K
__device__ __forceinline__ float4 wrow4(const float* W, long row, int K, int k4) {
  return k4 < (K >> 2) ? reinterpret_cast<const float4*>(W + row * K)[k4] : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Lane partials -> sums: every lane writes its NG x kRC partials as a column of red[w][.][lane],
// then thread t sums row t over the 64 lanes (fixed order) into sums[t] (t < 4 * NG * kRC).
template <int NG>
__device__ __forceinline__ void reduce_lanes(const float (&acc)[NG][kRC], int w, int lane, float* red,
                                             float* sums) {
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int rr = 0; rr < kRC; ++rr) red[((w * NG + g) * kRC + rr) * kRP + lane] = acc[g][rr];
  __syncthreads();
  for (int t = threadIdx.x; t < 4 * NG * kRC; t += 256) {
    const float* row = red + t * kRP;
    float s = 0.f;
#pragma unroll 8
    for (int l = 0; l < 64; ++l) s += row[l];
    sums[t] = s;
  }
  __syncthreads();
}

// torch's GRUCell epilogue for one (unit, row) from the summed gate products (gi / gh without
// biases): the new h; shared by the per-step kernel and the persistent loop (contraction off, so
// both form the same bits)
__device__ __forceinline__ float gru_cell(const float* gi, const float* gh, const float (&ebi)[3], const float (&ebh)[3],
                                          float ehp) {
#pragma clang fp contract(off)
  const float gi_r = gi[0] + ebi[0], gi_z = gi[kRC] + ebi[1], gi_n = gi[2 * kRC] + ebi[2];
  const float gh_r = gh[0] + ebh[0], gh_z = gh[kRC] + ebh[1], gh_n = gh[2 * kRC] + ebh[2];
  const float rg = sigmoidf_(gh_r + gi_r), zg = sigmoidf_(gh_z + gi_z);
  const float ng = tanhf(gi_n + gh_n * rg);
  return (ehp - ng) * zg + ng;
}

// GRU layer WHICH (1: rnn1 on xI; 2: rnn2 on [t1, a2]) for two hidden units per workgroup.
// Waves 0/1: the input gates (r, z, n rows) of units u0 / u0+1, waves 2/3: their hidden gates.
// torch's GRU cell order (aten RNN.cpp GRUCell): r = σ(gh_r + gi_r), z = σ(gh_z + gi_z),
// n = tanh(gi_n + gh_n·r), h' = (h − n)·z + n.
template <int WHICH>
__global__ __launch_bounds__(256) void wr_gru_kernel(WrStep a) {
  const int i = cur_step(a);
  if (i >= a.L) return;
  constexpr int KI = 576;  // staging row capacity (checked on the host: H + A <= 576)
  __shared__ float smem[kRC * (KI + 512) > 4 * 3 * kRC * kRP ? kRC * (KI + 512) : 4 * 3 * kRC * kRP];
  __shared__ float sums[4 * 3 * kRC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int H = a.H, R = a.R;
  const int u0 = blockIdx.x * 2;
  const int u = u0 + (w & 1);
  const bool hid = w >= 2;
  const int Kin = WHICH == 1 ? H : H + a.A;
  const int K = hid ? H : Kin;
  const float* W = hid ? (WHICH == 1 ? a.Whh1 : a.Whh2) : (WHICH == 1 ? a.Wih1 : a.Wih2);
  const int cur = i & 1;
  float4 wv[3][kJ4];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int j = 0; j < kJ4; ++j) wv[g][j] = wrow4(W, (long)g * H + u, K, lane + 64 * j);
  float* xin = smem;             // [kRC][Kin]
  float* xh = smem + kRC * Kin;  // [kRC][H]
  const float* bi = WHICH == 1 ? a.bih1 : a.bih2;
  const float* bh = WHICH == 1 ? a.bhh1 : a.bhh2;
  float* hb = WHICH == 1 ? a.h1 : a.h2;
  for (int rb = 0; rb < R; rb += kRC) {
    // epilogue operands of thread (unit uu, row rr), fetched with the staging loads
    const int nr = min(kRC, R - rb);
    const int uu = tid & 1, rr0 = tid >> 1, un = u0 + uu, r0 = rb + rr0;
    const bool ep = tid < 2 * nr;
    float ebi[3], ebh[3], ehp = 0.f, ex = 0.f;
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      ebi[g] = bi[g * H + un];
      ebh[g] = bh[g * H + un];
    }
    if (ep) {
      ehp = hb[((long)cur * R + r0) * H + un];
      if (WHICH == 1) {
        int src;
        long q;
        fold_pos(a, r0, i, src, q);
        ex = fmaf(a.wi0[un], xprev_at(a, r0, i), a.pI[((long)src * (a.Ltot + 1) + q) * H + un]);
      } else {
        ex = a.t1[(long)r0 * H + un];
      }
    }
    {
      float4 v0[kStage4], v1[kStage4];
      stage_load(a, WHICH == 1 ? IN_XI : IN_T1A2, i, rb, Kin, v0);
      stage_load(a, WHICH == 1 ? IN_H1 : IN_H2, i, rb, H, v1);
      stage_store(Kin, v0, xin);
      stage_store(H, v1, xh);
    }
    __syncthreads();
    float acc[3][kRC];
    rows_dot<3>(wv, hid ? xh : xin, K, lane, acc);
    __syncthreads();  // staged rows fully read: the partial transpose reuses the space
    reduce_lanes<3>(acc, w, lane, smem, sums);
    if (ep) {
      const float* gi = sums + (uu * 3) * kRC + rr0;        // wave uu: input gates
      const float* gh = sums + ((2 + uu) * 3) * kRC + rr0;  // wave 2 + uu: hidden gates
      const float hn = gru_cell(gi, gh, ebi, ebh, ehp);
      hb[((long)(cur ^ 1) * R + r0) * H + un] = hn;
      // x = I(...) + h1 (model.py:269) after rnn1, x + h2 (model.py:273) after rnn2
      (WHICH == 1 ? a.t1 : a.t2)[(long)r0 * H + un] = ex + hn;
    }
    __syncthreads();
  }
}

// fc1 / fc2 (model.py:274-278): y = relu(W · [v, a] + b), v = t2 (WHICH 1, a = a3) or y1
// (WHICH 2, a = a4); two output rows per wave, eight per workgroup.
template <int WHICH>
__global__ __launch_bounds__(256) void wr_fc_kernel(WrStep a) {
  const int i = cur_step(a);
  if (i >= a.L) return;
  __shared__ float smem[kRC * 576 > 4 * 2 * kRC * kRP ? kRC * 576 : 4 * 2 * kRC * kRP];
  __shared__ float sums[4 * 2 * kRC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int Kv = WHICH == 1 ? a.H : a.Fc, K = Kv + a.A;
  const float* W = WHICH == 1 ? a.W1 : a.W2;
  const float* bias = WHICH == 1 ? a.b1 : a.b2;
  float* y = WHICH == 1 ? a.y1 : a.y2;
  const int n0 = blockIdx.x * 8 + 2 * w;
  float4 wv[2][kJ4];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int j = 0; j < kJ4; ++j) wv[g][j] = wrow4(W, min(n0 + g, a.Fc - 1), K, lane + 64 * j);
  for (int rb = 0; rb < a.R; rb += kRC) {
    {
      float4 v0[kStage4];
      stage_load(a, WHICH == 1 ? IN_T2A3 : IN_Y1A4, i, rb, K, v0);
      stage_store(K, v0, smem);
    }
    __syncthreads();
    float acc[2][kRC];
    rows_dot<2>(wv, smem, K, lane, acc);
    __syncthreads();
    reduce_lanes<2>(acc, w, lane, smem, sums);
    const int nr = min(kRC, a.R - rb);
    for (int t = tid; t < 8 * nr; t += 256) {  // (output row, fold row)
      const int o = t / nr, rr = t - o * nr, n = blockIdx.x * 8 + o;
      if (n < a.Fc) y[(long)(rb + rr) * a.Fc + n] = fmaxf(sums[o * kRC + rr] + bias[n], 0.f);
    }
    __syncthreads();
  }
}

// counter-based uniform in [1e-5, 1 - 1e-5] (oracle/wavernn_oracle.py:uniforms, the same bits)
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float uniform_draw(unsigned long long seed, int r, int i, int d) {
  const unsigned long long base = mix64((seed + 1ull) * 0x9E3779B97F4A7C15ull);
  const unsigned long long ctr = ((unsigned long long)r << 40) | ((unsigned long long)(unsigned)i << 8) | (unsigned)d;
  const unsigned long long z = mix64(ctr * 0x9E3779B97F4A7C15ull + base);
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  return __fadd_rn(1e-5f, __fmul_rn(0.99998f, u));
}

// The sample of fold row r at step i from its logits lg (model.py:279-315, distribution.py:87-123),
// called by every thread of the workgroup; thread 0 returns it.  Teacher-forced calls store the
// logits and return the given sample.  MOL: lanes k < nr form the Gumbel-perturbed mixture logits
// and lane nr the logistic draw's log-odds side by side (LDS tk[0..nr]); thread 0 then takes the
// first maximum (torch.max) and forms the sample -- each value by the expression the serial form
// used, so the bits are unchanged.  Shared by the per-step kernel and the persistent loop
// (contraction off).  tk: >= 32 floats of LDS.
__device__ __forceinline__ float wr_sample(const WrStep& a, int r, int i, const float* lg, float* tk) {
#pragma clang fp contract(off)
  const int NC = a.NC, tid = threadIdx.x;
  const long o = (long)r * a.L + i;
  float x = 0.f;
  if (a.teacher) {
    if (tid == 0) {
      for (int c = 0; c < NC; ++c) a.logits[o * NC + c] = lg[c];
      x = a.x_tf[o];  // (unused by the next step, which reads x_tf itself)
    }
  } else if (a.mol) {
    const int nr = NC / 3;
    if (tid < nr) {
      const float u = uniform_draw(a.seed, r, i, tid);
      tk[tid] = lg[tid] - logf(-logf(u));
    } else if (tid == nr) {
      const float u = uniform_draw(a.seed, r, i, nr);
      tk[nr] = logf(u) - logf(1.0f - u);
    }
    __syncthreads();
    if (tid == 0) {
      int best = 0;
      float bv = 0.f;
      for (int k = 0; k < nr; ++k) {  // Gumbel-max mixture choice; first maximum wins (torch.max)
        const float t = tk[k];
        if (k == 0 || t > bv) { bv = t; best = k; }
      }
      const float mean = lg[nr + best];
      const float ls = fmaxf(lg[2 * nr + best], -32.236191301916641f);  // log(1e-14)
      x = mean + expf(ls) * tk[nr];
      x = fminf(fmaxf(x, -1.f), 1.f);
    }
  } else if (tid == 0) {  // RAW: Categorical(softmax) by inverse CDF, 2k / (n_classes - 1) - 1
    float mx = lg[0];
    for (int c = 1; c < NC; ++c) mx = fmaxf(mx, lg[c]);
    float sum = 0.f;  // (each exp is formed twice, the same bits both times: no indexed array)
    for (int c = 0; c < NC; ++c) sum += expf(lg[c] - mx);
    const float u = uniform_draw(a.seed, r, i, 0);
    float cdf = 0.f;
    int k = 0;
    for (int c = 0; c < NC; ++c) { cdf += expf(lg[c] - mx) / sum; if (cdf < u) k = c + 1; }
    k = min(k, NC - 1);
    x = 2.f * (float)k / ((float)NC - 1.f) - 1.f;
  }
  return x;
}

// fc3 + sampling (model.py:279-315; distribution.py:87-123), one workgroup per fold row; the last
// workgroup to finish advances the step counter for the next launch.
__global__ __launch_bounds__(256) void wr_out_kernel(WrStep a) {
  const int i = cur_step(a);
  if (i >= a.L) return;
  __shared__ float red[4 * 8 * kRP];
  __shared__ float lg[64];  // [0, 32) logits, [32, 64) wr_sample's tk
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = blockIdx.x, Fc = a.Fc, NC = a.NC;
  float4 yv[kJ4];
#pragma unroll
  for (int j = 0; j < kJ4; ++j) yv[j] = wrow4(a.y2, r, Fc, lane + 64 * j);
  // class c = w + 4 m (m < 8, NC <= 32): lanes over float4 k, one transpose-reduction through LDS
  float acc[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const float4* wr = reinterpret_cast<const float4*>(a.W3 + (long)min(w + 4 * m, NC - 1) * Fc);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kJ4; ++j) {
      const float4 v = wr[min(lane + 64 * j, (Fc >> 2) - 1)];  // yv is zero past Fc
      s = fmaf(v.x, yv[j].x, s);
      s = fmaf(v.y, yv[j].y, s);
      s = fmaf(v.z, yv[j].z, s);
      s = fmaf(v.w, yv[j].w, s);
    }
    acc[m] = s;
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) red[(w * 8 + m) * kRP + lane] = acc[m];
  __syncthreads();
  if (tid < 32) {
    const int ww = tid & 3, m = tid >> 2, c = ww + 4 * m;
    if (c < NC) {
      const float* row = red + (ww * 8 + m) * kRP;
      float s = 0.f;
#pragma unroll 8
      for (int l = 0; l < 64; ++l) s += row[l];
      lg[c] = s + a.b3[c];
    }
  }
  __syncthreads();
  const float x = wr_sample(a, r, i, lg, lg + 32);
  if (tid == 0) {
    const long o = (long)r * a.L + i;
    a.out[o] = x;
    a.x_prev[r] = x;
    if (atomicAdd(a.done, 1) == a.R - 1) {  // every workgroup has read this step: advance it
      __hip_atomic_store(a.done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.step, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
__global__ void wr_column_kernel(int n, long ld, const float* __restrict__ W, float* __restrict__ col) {
  for (int k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) col[k] = W[(long)k * ld];
}

__global__ void wr_init_state_kernel(int R, int H, int Fc, int* step, int* done, float* x_prev, float* h1,
                                     float* h2) {
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < 2L * R * H; idx += (long)gridDim.x * 256) {
    h1[idx] = 0.f;
    h2[idx] = 0.f;
    if (idx < R) x_prev[idx] = 0.f;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *step = 0;
    *done = 0;
  }
}

// ---- the persistent sample loop (avc_wavernn_persist) ---------------------------------------
//
// All L steps in ONE launch of G = H / 2 workgroups (one per CU; every one resident, checked on
// the host) instead of five launches per step.  Workgroup w does what blockIdx w does in the
// per-step kernels, with the same arithmetic, so the two paths agree bit for bit:
//   every w:              GRU1 and GRU2 for hidden units 2w, 2w + 1;
//   w < nfc:              fc1 rows [8w, 8w + 8)                  (role FC1)
//   nfc <= w < 2 nfc:     fc2 rows [8(w - nfc), 8(w - nfc) + 8)  (role FC2)
//   2 nfc <= w < 2nfc+R:  fc3 + sampling of fold row w - 2 nfc  (role OUT)
// A GRU's hidden-gate products W_hh h_{i-1} do not depend on the sample just drawn: they are
// formed early (the 'hid' phase: step i+1's sums, kept in LDS) while fc1 / fc2 / fc3 of step i
// run, each role placing them where it waits anyway.  The chain of a step is then GRU1's input
// gates -> GRU2's input gates -> fc1 -> fc2 -> fc3 + sampling: five in-launch hand-offs.
// Hand-offs follow the LSTM recurrences' counter form (cdna_hip_programming.md Guideline 16):
// payload stored write-through (sc1), every storing wave drains, barrier, one 8-lane add to the
// stage's 8 counter replicas; a consumer polls its replica relaxed, barrier, and EVERY load of
// handed-off bytes is an sc1 load.  Counters are a ring of kWrRing steps per stage that is never
// reset: launch E's target for step i (ring slot k = i % kWrRing) is ((E - 1) n_k + i / kWrRing
// + 1) P, n_k the steps of slot k per launch, P the stage's producers; E comes from a ticket each
// workgroup takes at start, as in the recurrences.  Write-after-read: each buffer rewritten at
// step i + 1 was read at step i by workgroups that counted in on a counter the writer has waited
// for.  Every spin is bounded; a launch that gives up writes its remaining samples
// as NaN and the call reports AVC_ERR_DEVICE.
constexpr int kWrRing = 16, kWrStages = 5, kWrRep = 8, kWrLine = 32;
constexpr int kWrMaxChunks = 4;  // fold rows <= kWrMaxChunks * kRC
constexpr long kWrCntWords = (long)kWrStages * kWrRing * kWrRep * kWrLine;
enum : int { WR_NONE = 0, WR_FC1 = 1, WR_FC2 = 2, WR_OUT = 3 };
enum : int { S_GRU1 = 0, S_GRU2 = 1, S_FC1 = 2, S_FC2 = 3, S_OUT = 4 };
// LDS (floats): staging | partial transpose | hidden sums [2][chunks][6 kRC] | input / fc sums |
// previous h [2][chunks][2 kRC] | own t1 [chunks][2 kRC] | logits | flags
constexpr int kWrXs = 0, kWrRed = kWrXs + kRC * 576, kWrShid = kWrRed + 8 * kRC * kRP;
constexpr int kWrSin = kWrShid + 2 * kWrMaxChunks * 6 * kRC, kWrHprev = kWrSin + 8 * kRC;
constexpr int kWrT1 = kWrHprev + 2 * kWrMaxChunks * 2 * kRC, kWrLg = kWrT1 + kWrMaxChunks * 2 * kRC;
constexpr int kWrFlags = kWrLg + 64, kWrLdsFloats = kWrFlags + 8;

struct WrLoop {
  WrStep a;
  int G, nfc, nchk;
  unsigned* cnt;                  // [stage][ring][replica] lines (never reset)
  unsigned* tmo;                  // give-up word: epoch of the last launch that gave up
  unsigned long long* tickets;    // one per workgroup per launch
  unsigned* fail_host;            // the context's pinned failure word
  unsigned spin_limit;
  unsigned long long* stamps;     // diagnostics (avc_debug_wavernn_stamps): [G][nstamp][16] realtime
  int nstamp;                     // steps stamped
};

typedef __attribute__((address_space(1))) unsigned wr_gu32;
typedef unsigned wr_u32x4 __attribute__((ext_vector_type(4)));
__device__ unsigned g_wr_giveups = 0;

// sc1 (write-through / L2-bypassing) accesses of handed-off bytes: base is uniform, off in floats
__device__ __forceinline__ float4 ld4_sc1(const float* base, long off) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
  const wr_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off * 4), 0, 16 /*sc1*/);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ float ld_sc1(const float* base, long off) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(off * 4), 0, 16 /*sc1*/));
}
__device__ __forceinline__ void st_sc1(float* base, long off, float v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)(off * 4), 0, 16 /*sc1*/);
}

__device__ __forceinline__ long wr_cidx(int S, int i, int rep) {
  return (((long)S * kWrRing + i % kWrRing) * kWrRep + rep) * kWrLine;
}
__device__ __forceinline__ unsigned wr_target(const WrLoop& p, int S, int i, unsigned E) {
  const int k = i % kWrRing;
  const unsigned nk = (unsigned)((p.a.L - k + kWrRing - 1) / kWrRing);
  const unsigned P = S <= S_GRU2 ? (unsigned)p.G : S <= S_FC2 ? (unsigned)p.nfc : (unsigned)p.a.R;
  return ((E - 1u) * nk + (unsigned)(i / kWrRing) + 1u) * P;
}

// One lane waits for stage S of step i (wrap-safe relaxed agent-scope polls of its replica);
// false = gave up, or another workgroup of this launch did (the give-up word, every 64 polls).
__device__ __forceinline__ bool wr_poll(const WrLoop& p, int S, int i, unsigned E) {
  wr_gu32* c = (wr_gu32*)(p.cnt + wr_cidx(S, i, blockIdx.x % kWrRep));
  wr_gu32* t = (wr_gu32*)p.tmo;
  const unsigned target = wr_target(p, S, i, E);
  for (unsigned spins = 0;; ++spins) {
    if ((int)(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) >= 0) return true;
    if ((spins & 63) == 63 && __hip_atomic_load(t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == E) return false;
    if (spins >= p.spin_limit) {
      const unsigned old = __hip_atomic_fetch_max(t, E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old != E) {  // first to give up in this launch (tag 0x40000000: the vocoder loop)
        const unsigned n = atomicAdd(&g_wr_giveups, 1u) + 1u;
        if (p.fail_host)
          __hip_atomic_store(p.fail_host, 0x40000000u | n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// the whole workgroup waits (thread 0 polls; the verdict goes through one of 4 LDS words in turn,
// so a word is rewritten only after barriers every reader has passed)
__device__ __forceinline__ bool wr_wait(const WrLoop& p, int S, int i, unsigned E, int* flags, int& nw) {
  int* f = flags + (nw++ & 3);
  if (threadIdx.x == 0) {
    *f = wr_poll(p, S, i, E) ? 1 : 0;
    // diagnostics: when the wait ended (slot 3 op + 1 of the loop step; flags[6] / [7] = op, step)
    if (p.stamps && flags[7] >= 0 && flags[7] < p.nstamp)
      p.stamps[((long)blockIdx.x * p.nstamp + flags[7]) * 24 + 3 * flags[6] + 1] = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  return *f != 0;
}

// every storing wave drains its sc1 stores, barrier, one 8-lane add to the stage's replicas
__device__ __forceinline__ void wr_publish(const WrLoop& p, int S, int i) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < kWrRep)
    __hip_atomic_fetch_add((wr_gu32*)(p.cnt + wr_cidx(S, i, threadIdx.x)), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Loop staging of rows [rb, rb + kRC) of input `which` (stage_load's layout and values): _pre
// issues the loads of bytes no workgroup of the launch writes (pI, the aux slices) before the
// wait, _post the handed-off part (sc1) after it; IN_XI forms pI + W_I[:, 0] x_prev as stage_load.
__device__ __forceinline__ void lstage_pre(const WrStep& a, int which, int i, int rb, int K, int tid, float4 (&v)[kStage4]) {
  const int K4 = K >> 2, H = a.H;
#pragma unroll
  for (int m = 0; m < kStage4; ++m) {
    const int e = tid + 256 * m;
    const int rr = e / K4, k = 4 * (e - rr * K4), r = rb + rr;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rr < kRC && r < a.R) {
      int src;
      long q;
      fold_pos(a, r, i, src, q);
      if (which == IN_XI) {
        x = *reinterpret_cast<const float4*>(a.pI + ((long)src * (a.Ltot + 1) + q) * H + k);
      } else if (which != IN_H1 && which != IN_H2) {
        const int kv = which == IN_Y1A4 ? a.Fc : H;
        if (k >= kv && q < a.Ltot) {
          const int off = (which == IN_T1A2 ? 1 : which == IN_T2A3 ? 2 : 3) * a.A + (k - kv);
          x = *reinterpret_cast<const float4*>(a.auxf + ((long)src * a.Tf + q / a.hop) * a.auxd + off);
        }
      }
    }
    v[m] = x;
  }
}
__device__ __forceinline__ void lstage_post(const WrStep& a, int which, int i, int rb, int K, int tid, float4 (&v)[kStage4]) {
  const int K4 = K >> 2, H = a.H, cur = i & 1;
#pragma unroll
  for (int m = 0; m < kStage4; ++m) {
    const int e = tid + 256 * m;
    const int rr = e / K4, k = 4 * (e - rr * K4), r = rb + rr;
    if (rr < kRC && r < a.R) {
      switch (which) {
        case IN_XI: {
          const float4 pi = v[m];
          const float4 w0 = *reinterpret_cast<const float4*>(a.wi0 + k);
          const float xp = a.teacher ? a.x_tf[(long)r * a.L + i] : ld_sc1(a.x_prev, r);
          v[m] = make_float4(fmaf(w0.x, xp, pi.x), fmaf(w0.y, xp, pi.y), fmaf(w0.z, xp, pi.z), fmaf(w0.w, xp, pi.w));
          break;
        }
        case IN_H1: v[m] = ld4_sc1(a.h1, ((long)cur * a.R + r) * H + k); break;
        case IN_H2: v[m] = ld4_sc1(a.h2, ((long)cur * a.R + r) * H + k); break;
        case IN_T1A2: if (k < H) v[m] = ld4_sc1(a.t1, (long)r * H + k); break;
        case IN_T2A3: if (k < H) v[m] = ld4_sc1(a.t2, (long)r * H + k); break;
        default: if (k < a.Fc) v[m] = ld4_sc1(a.y1, (long)r * a.Fc + k); break;
      }
    }
  }
}

__device__ __forceinline__ void lstage_store(int K, int tid, const float4 (&v)[kStage4], float* xs) {
  const int K4 = K >> 2;
#pragma unroll
  for (int m = 0; m < kStage4; ++m) {
    const int e = tid + 256 * m;
    if (e < kRC * K4) reinterpret_cast<float4*>(xs)[e] = v[m];
  }
}

// rows_dot over the NR staged rows [rr0, rr0 + NR): each (output row, staged row) partial is formed
// in rows_dot's order (j ascending, x y z w), so the sums are the per-step kernels' bits
template <int NG, int NR>
__device__ __forceinline__ void rows_dot_part(const float4 (&wv)[NG][kJ4], const float* xs, int K, int lane, int rr0,
                                              float (&acc)[NG][NR]) {
  const int K4 = K >> 2;
  const float4* xs4 = reinterpret_cast<const float4*>(xs);
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) acc[g][rr] = 0.f;
#pragma unroll
  for (int j = 0; j < kJ4; ++j) {
    const int k4 = lane + 64 * j;
    if (k4 < K4) {
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) {
        const float4 x = xs4[(rr0 + rr) * K4 + k4];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          float t = acc[g][rr];
          t = fmaf(wv[g][j].x, x.x, t);
          t = fmaf(wv[g][j].y, x.y, t);
          t = fmaf(wv[g][j].z, x.z, t);
          acc[g][rr] = fmaf(wv[g][j].w, x.w, t);
        }
      }
    }
  }
}

// The six gate rows of units u0, u0 + 1 (wave w: unit w >> 1's three rows against staged rows
// [12 (w & 1), + 12)) against one staged chunk v: sums[(uu * 3 + g) * kRC + rr] into dst
__device__ __forceinline__ void gru_chunk_sums(const float4 (&wv)[3][kJ4], const float4 (&v)[kStage4], int K, float* xs,
                                               float* red, float* dst, int tid, int lane, int w) {
  lstage_store(K, tid, v, xs);
  __syncthreads();
  float acc[3][12];
  rows_dot_part<3, 12>(wv, xs, K, lane, 12 * (w & 1), acc);
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int rr = 0; rr < 12; ++rr) red[(((w >> 1) * 3 + g) * kRC + 12 * (w & 1) + rr) * kRP + lane] = acc[g][rr];
  __syncthreads();
  if (tid < 6 * kRC) {
    const float* row = red + tid * kRP;
    float s = 0.f;
#pragma unroll 8
    for (int l = 0; l < 64; ++l) s += row[l];
    dst[tid] = s;
  }
  __syncthreads();
}

// Step i's hidden-gate sums of BOTH layers (W_hh1 h1_{i-1}, W_hh2 h2_{i-1}) for units u0, u0 + 1,
// kept in LDS for the input phases: the two layers' h rows are loaded together (one round trip),
// then multiplied one after the other.
__device__ __forceinline__ bool hid_phase(const WrLoop& p, int i, unsigned E, float* sm, int& nw) {
  const WrStep& a = p.a;
  int tid = threadIdx.x;  // (opaque per phase: see gru_phase)
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, w = tid >> 6;
  const int H = a.H, u0 = blockIdx.x * 2;
  int* flags = reinterpret_cast<int*>(sm + kWrFlags);
  float4 wv1[3][kJ4], wv2[3][kJ4];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int j = 0; j < kJ4; ++j) {
      wv1[g][j] = wrow4(a.Whh1, (long)g * H + u0 + (w >> 1), H, lane + 64 * j);
      wv2[g][j] = wrow4(a.Whh2, (long)g * H + u0 + (w >> 1), H, lane + 64 * j);
    }
  if (i >= 1 && !(wr_wait(p, S_GRU1, i - 1, E, flags, nw) && wr_wait(p, S_GRU2, i - 1, E, flags, nw))) return false;
  for (int c = 0; c < p.nchk; ++c) {
    const int rb = c * kRC;
    float4 v1[kStage4], v2[kStage4];
    lstage_pre(a, IN_H1, i, rb, H, tid, v1);
    lstage_pre(a, IN_H2, i, rb, H, tid, v2);
    lstage_post(a, IN_H1, i, rb, H, tid, v1);
    lstage_post(a, IN_H2, i, rb, H, tid, v2);
    gru_chunk_sums(wv1, v1, H, sm + kWrXs, sm + kWrRed, sm + kWrShid + c * 6 * kRC, tid, lane, w);
    gru_chunk_sums(wv2, v2, H, sm + kWrXs, sm + kWrRed, sm + kWrShid + (kWrMaxChunks + c) * 6 * kRC, tid, lane, w);
  }
  return true;
}

// One GRU phase of step i for units u0, u0 + 1: HID = the hidden gates (W_hh h_{i-1}; sums kept
// for the input phase), else the input gates, the cell and the hand-off of h_i and t1 / t2.
// Wave w multiplies unit w >> 1's three gate rows against staged rows [12 (w & 1), + 12).
template <int WHICH, bool HID>
__device__ __forceinline__ bool gru_phase(const WrLoop& p, int i, unsigned E, float* sm, int& nw, const float (&ebi)[3],
                          const float (&ebh)[3]) {
  const WrStep& a = p.a;
  // (the thread index goes through an empty asm per phase, so the lane-dependent index math of
  // every phase is formed inside it instead of being hoisted out of the step loop into scratch)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, w = tid >> 6;
  const int H = a.H, R = a.R, u0 = blockIdx.x * 2;
  const int K = HID ? H : (WHICH == 1 ? H : H + a.A);
  const int which = HID ? (WHICH == 1 ? IN_H1 : IN_H2) : (WHICH == 1 ? IN_XI : IN_T1A2);
  const float* W = HID ? (WHICH == 1 ? a.Whh1 : a.Whh2) : (WHICH == 1 ? a.Wih1 : a.Wih2);
  float* xs = sm + kWrXs;
  float* red = sm + kWrRed;
  float* sin_ = sm + kWrSin;
  int* flags = reinterpret_cast<int*>(sm + kWrFlags);
  float4 wv[3][kJ4];
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int j = 0; j < kJ4; ++j) wv[g][j] = wrow4(W, (long)g * H + u0 + (w >> 1), K, lane + 64 * j);
  float4 v[kStage4];
  lstage_pre(a, which, i, 0, K, tid, v);
  // producers: HID waits for h_{i-1} of its own layer; GRU1's input gates for the sample of step
  // i - 1, GRU2's for t1 of step i
  const int wS = HID ? (WHICH == 1 ? S_GRU1 : S_GRU2) : (WHICH == 1 ? S_OUT : S_GRU1);
  const int wi = (HID || WHICH == 1) ? i - 1 : i;
  if (wi >= 0 && !wr_wait(p, wS, wi, E, flags, nw)) return false;
  for (int c = 0; c < p.nchk; ++c) {
    const int rb = c * kRC;
    const int nr = min(kRC, R - rb);
    if (c > 0) lstage_pre(a, which, i, rb, K, tid, v);
    // GRU1's epilogue operands (the new sample, pI, W_I[:, 0]) issued with the staging loads
    float xpe = 0.f, pie = 0.f, w0e = 0.f;
    if (!HID && WHICH == 1 && tid < 2 * nr) {
      const int r0 = rb + (tid >> 1), un = u0 + (tid & 1);
      int src;
      long q;
      fold_pos(a, r0, i, src, q);
      xpe = a.teacher ? a.x_tf[(long)r0 * a.L + i] : ld_sc1(a.x_prev, r0);
      pie = a.pI[((long)src * (a.Ltot + 1) + q) * H + un];
      w0e = a.wi0[un];
    }
    lstage_post(a, which, i, rb, K, tid, v);
    gru_chunk_sums(wv, v, K, xs, red, HID ? sm + kWrShid + ((WHICH - 1) * kWrMaxChunks + c) * 6 * kRC : sin_, tid,
                   lane, w);
    if (!HID) {
      if (tid < 2 * nr) {
        const int uu = tid & 1, rr0 = tid >> 1, un = u0 + uu, r0 = rb + rr0;
        const float* sh = sm + kWrShid + ((WHICH - 1) * kWrMaxChunks + c) * 6 * kRC;
        float* hp = sm + kWrHprev + ((WHICH - 1) * kWrMaxChunks + c) * 2 * kRC + tid;
        float* t1o = sm + kWrT1 + c * 2 * kRC + tid;
        const float hn = gru_cell(sin_ + uu * 3 * kRC + rr0, sh + uu * 3 * kRC + rr0, ebi, ebh, *hp);
        *hp = hn;
        const float ex = WHICH == 1 ? fmaf(w0e, xpe, pie) : *t1o;
        const float tv = ex + hn;
        if (WHICH == 1) *t1o = tv;
        st_sc1(WHICH == 1 ? a.h1 : a.h2, ((long)((i & 1) ^ 1) * R + r0) * H + un, hn);
        st_sc1(WHICH == 1 ? a.t1 : a.t2, (long)r0 * H + un, tv);
      }
    }
  }
  if (!HID) wr_publish(p, WHICH == 1 ? S_GRU1 : S_GRU2, i);
  return true;
}

// fc1 / fc2 of step i for rows [8f, 8f + 8) (wr_fc_kernel's arithmetic)
template <int WHICH>
__device__ __forceinline__ bool fc_phase(const WrLoop& p, int f, int i, unsigned E, float* sm, int& nw) {
  const WrStep& a = p.a;
  int tid = threadIdx.x;  // (opaque per phase: see gru_phase)
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, w = tid >> 6;
  const int Kv = WHICH == 1 ? a.H : a.Fc, K = Kv + a.A;
  const float* W = WHICH == 1 ? a.W1 : a.W2;
  const float* bias = WHICH == 1 ? a.b1 : a.b2;
  float* y = WHICH == 1 ? a.y1 : a.y2;
  float* xs = sm + kWrXs;
  float* sums = sm + kWrSin;
  int* flags = reinterpret_cast<int*>(sm + kWrFlags);
  // wave w: output rows [4 (w & 1), + 4) of the 8 against staged rows [12 (w >> 1), + 12) -- the
  // per-step kernel's (output row, fold row) partials with half its LDS reads per wave
  const int og = 4 * (w & 1), rh = 12 * (w >> 1);
  float4 wv[4][kJ4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int j = 0; j < kJ4; ++j) wv[g][j] = wrow4(W, min(f * 8 + og + g, a.Fc - 1), K, lane + 64 * j);
  const int which = WHICH == 1 ? IN_T2A3 : IN_Y1A4;
  float4 v[kStage4];
  lstage_pre(a, which, i, 0, K, tid, v);
  if (!wr_wait(p, WHICH == 1 ? S_GRU2 : S_FC1, i, E, flags, nw)) return false;
  for (int c = 0; c < p.nchk; ++c) {
    const int rb = c * kRC;
    const int nr = min(kRC, a.R - rb);
    if (c > 0) lstage_pre(a, which, i, rb, K, tid, v);
    // the epilogue thread's bias (one (output row, fold row) per thread: 8 nr <= 192), issued with
    // the staging loads
    const int o = tid / nr, n = f * 8 + o;
    const bool ep = tid < 8 * nr && n < a.Fc;
    const float bz = ep ? bias[n] : 0.f;
    lstage_post(a, which, i, rb, K, tid, v);
    lstage_store(K, tid, v, xs);
    __syncthreads();
    float acc[4][12];
    rows_dot_part<4, 12>(wv, xs, K, lane, rh, acc);
    float* red = sm + kWrRed;
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 12; ++r) red[((og + g) * kRC + rh + r) * kRP + lane] = acc[g][r];
    __syncthreads();
    if (tid < 8 * kRC) {  // reduce_lanes' fixed-order 64-lane sums, sums[o * kRC + rr]
      const float* row = red + tid * kRP;
      float sacc = 0.f;
#pragma unroll 8
      for (int l = 0; l < 64; ++l) sacc += row[l];
      sums[tid] = sacc;
    }
    __syncthreads();
    if (ep) {
      const int rr = tid - o * nr;
      st_sc1(y, (long)(rb + rr) * a.Fc + n, fmaxf(sums[o * kRC + rr] + bz, 0.f));
    }
    __syncthreads();
  }
  wr_publish(p, WHICH == 1 ? S_FC1 : S_FC2, i);
  return true;
}

// fc3 + sampling of fold row r at step i (wr_out_kernel's arithmetic)
__device__ __forceinline__ bool out_phase(const WrLoop& p, int r, int i, unsigned E, float* sm, int& nw) {
  const WrStep& a = p.a;
  int tid = threadIdx.x;  // (opaque per phase: see gru_phase)
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, w = tid >> 6;
  const int Fc = a.Fc, NC = a.NC;
  float* red = sm + kWrRed;
  float* lg = sm + kWrLg;
  int* flags = reinterpret_cast<int*>(sm + kWrFlags);
  float4 w3[8][kJ4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int j = 0; j < kJ4; ++j)
      w3[m][j] = reinterpret_cast<const float4*>(a.W3 + (long)min(w + 4 * m, NC - 1) * Fc)[min(lane + 64 * j, (Fc >> 2) - 1)];
  const int cb3 = (tid & 3) + 4 * (tid >> 2);
  const float b3v = tid < 32 && cb3 < NC ? a.b3[cb3] : 0.f;
  if (!wr_wait(p, S_FC2, i, E, flags, nw)) return false;
  float4 yv[kJ4];
#pragma unroll
  for (int j = 0; j < kJ4; ++j)
    yv[j] = lane + 64 * j < (Fc >> 2) ? ld4_sc1(a.y2, (long)r * Fc + 4 * (lane + 64 * j)) : make_float4(0.f, 0.f, 0.f, 0.f);
  float acc[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kJ4; ++j) {
      s = fmaf(w3[m][j].x, yv[j].x, s);
      s = fmaf(w3[m][j].y, yv[j].y, s);
      s = fmaf(w3[m][j].z, yv[j].z, s);
      s = fmaf(w3[m][j].w, yv[j].w, s);
    }
    acc[m] = s;
  }
#pragma unroll
  for (int m = 0; m < 8; ++m) red[(w * 8 + m) * kRP + lane] = acc[m];
  __syncthreads();
  if (tid < 32) {
    const int ww = tid & 3, m = tid >> 2, c = ww + 4 * m;
    if (c < NC) {
      const float* row = red + (ww * 8 + m) * kRP;
      float s = 0.f;
#pragma unroll 8
      for (int l = 0; l < 64; ++l) s += row[l];
      lg[c] = s + b3v;
    }
  }
  __syncthreads();
  const float x = wr_sample(a, r, i, lg, lg + 32);
  if (tid == 0) {
    a.out[(long)r * a.L + i] = x;
    st_sc1(a.x_prev, r, x);
  }
  wr_publish(p, S_OUT, i);
  return true;
}

__global__ __launch_bounds__(256, 1) void wr_loop_kernel(WrLoop p) {
  extern __shared__ float wr_sm[];
  const WrStep& a = p.a;
  const int tid = threadIdx.x, L = a.L;
  int* flags = reinterpret_cast<int*>(wr_sm + kWrFlags);
  if (tid == 0) {  // this launch's epoch
    const unsigned long long tk = __hip_atomic_fetch_add(p.tickets, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flags[4] = (int)(unsigned)(tk / (unsigned long long)p.G + 1ull);
    flags[7] = -1;
  }
  for (int t = tid; t < kWrLg - kWrHprev; t += 256) wr_sm[kWrHprev + t] = 0.f;  // h_{-1} = 0
  __syncthreads();
  const unsigned E = (unsigned)flags[4];
  int nw = 0;
  const int wg = blockIdx.x, nfc = p.nfc;
  const int role = wg < nfc ? WR_FC1 : wg < 2 * nfc ? WR_FC2 : wg < 2 * nfc + a.R ? WR_OUT : WR_NONE;
  // the epilogue thread's biases (unit u0 + (tid & 1)), fixed for the launch
  const int un = 2 * wg + (tid & 1);
  float ebi1[3], ebh1[3], ebi2[3], ebh2[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    ebi1[g] = a.bih1[g * a.H + un];
    ebh1[g] = a.bhh1[g * a.H + un];
    ebi2[g] = a.bih2[g * a.H + un];
    ebh2[g] = a.bhh2[g * a.H + un];
  }
  // per step: GRU1 and GRU2 input phases of step i, then the role's ops; HID forms step i + 1's
  // hidden sums of both layers (skipped after the last step), placed where the role would wait
  // anyway: FC1 after its product, FC2 and OUT before waiting for theirs.  One op list walked by one
  // switch, so every phase is instantiated once.
  enum : int { OP_HID = 0, OP_IN1 = 2, OP_IN2 = 3, OP_FC1 = 4, OP_FC2 = 5, OP_OUT = 6 };
  // the role's op list, packed 4 bits per op (no indexed array: it would live in scratch)
  const unsigned seq = role == WR_FC1   ? (OP_IN1 | OP_IN2 << 4 | OP_FC1 << 8 | OP_HID << 12)
                       : role == WR_FC2 ? (OP_IN1 | OP_IN2 << 4 | OP_HID << 8 | OP_FC2 << 12)
                       : role == WR_OUT ? (OP_IN1 | OP_IN2 << 4 | OP_HID << 8 | OP_OUT << 12)
                                        : (OP_IN1 | OP_IN2 << 4 | OP_HID << 8);
  const int nops = role == WR_NONE ? 3 : 4;
  bool ok = true;
  int i = -1;  // step -1: only the hidden sums of step 0 (h_{-1} = 0)
  for (; ok && i < L; ++i) {
    for (int o = 0; o < nops && ok; ++o) {
      const int op = (int)((seq >> (4 * o)) & 15u);
      const bool hid = op == OP_HID;
      if (hid ? i + 1 >= L : i < 0) continue;
      const bool stamp = p.stamps && i >= 0 && i < p.nstamp && tid == 0;
      if (tid == 0) {  // (read by wr_wait's stamp, same thread)
        flags[6] = op;
        flags[7] = i;
      }
      if (stamp) p.stamps[((long)wg * p.nstamp + i) * 24 + 3 * op] = __builtin_amdgcn_s_memrealtime();
      switch (op) {
        case OP_HID: ok = hid_phase(p, i + 1, E, wr_sm, nw); break;
        case OP_IN1: ok = gru_phase<1, false>(p, i, E, wr_sm, nw, ebi1, ebh1); break;
        case OP_IN2: ok = gru_phase<2, false>(p, i, E, wr_sm, nw, ebi2, ebh2); break;
        case OP_FC1: ok = fc_phase<1>(p, wg, i, E, wr_sm, nw); break;
        case OP_FC2: ok = fc_phase<2>(p, wg - nfc, i, E, wr_sm, nw); break;
        default: ok = out_phase(p, wg - 2 * nfc, i, E, wr_sm, nw); break;
      }
      if (stamp) p.stamps[((long)wg * p.nstamp + i) * 24 + 3 * op + 2] = __builtin_amdgcn_s_memrealtime();
    }
    if (!ok) break;
  }
  // gave up at step i: the row's remaining samples (and teacher-forced logits) are NaN, so a
  // timed-out launch never returns plausible audio (the call reports it)
  if (!ok && role == WR_OUT && tid == 0) {
    const int r = wg - 2 * nfc;
    const float nan = __builtin_nanf("");
    for (int k = max(i, 0); k < L; ++k) {
      a.out[(long)r * L + k] = nan;
      if (a.teacher)
        for (int c = 0; c < a.NC; ++c) a.logits[((long)r * L + k) * a.NC + c] = nan;
    }
  }
}

int g_wr_proj_tiled = 1;  // avc_wavernn_proj_tiled(): the LDS-tiled input projection (same bits)
int g_wr_persist = 1;  // avc_wavernn_persist(): 1 (default) = the persistent sample loop where eligible
int g_wr_inject = 0;   // avc_debug_wavernn_inject(): loop launches left that give up at once
int g_wr_fallbacks = 0;  // avc_wavernn_fallbacks(): loop launches that gave up and were re-run per step
unsigned long long* g_wr_stamps = nullptr;  // avc_debug_wavernn_stamps(): next loop launch's stamps
int g_wr_nstamp = 0;

// workgroups of wr_loop_kernel the device holds at once (occupancy x CUs), cached per device
int wr_loop_capacity() {
  static int cap = -1, cap_dev = -1;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (cap >= 0 && dev == cap_dev) return cap;
  const void* fn = (const void*)wr_loop_kernel;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kWrLdsFloats * 4);
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, kWrLdsFloats * 4) != hipSuccess) {
    (void)hipGetLastError();
    per_cu = 0;
  }
  cap = per_cu * coresident_cus();
  cap_dev = dev;
  return cap;
}

// the loop's shape limits: fold rows in <= kWrMaxChunks staging chunks, one workgroup per role
// (fc1, fc2, each fold row's sampling) besides the GRU units, every workgroup resident
bool wr_loop_eligible(const WrStep& a) {
  const int G = a.H / 2, nfc = (a.Fc + 7) / 8;
  return g_wr_persist && a.R <= kWrMaxChunks * kRC && 2 * nfc + a.R <= G && a.L >= 1 && G <= wr_loop_capacity();
}

// gave_up: set when THIS launch abandoned a bounded wait (a workgroup was not resident, e.g. CUs
// held by another process); its samples are NaN and the caller re-runs the call on the per-step path.
// A failure an earlier call left on the context is returned as before, with gave_up false.
int wr_loop_run(avc_context* ctx, const WrStep& a, hipStream_t s, double macs, unsigned long long* stamps,
                bool* gave_up) {
  *gave_up = false;
  AVC_TRY(persist_guard(ctx));
  const int G = a.H / 2;
  unsigned* region = nullptr;
  // counter layout key: every quantity a wait target depends on -- the steps per launch L and each
  // stage's producer count (G, nfc, R); a region shared by two layouts would leave one layout's
  // arrivals under the other's epoch targets
  const int nfc = (a.Fc + 7) / 8;
  AVC_TRY(coresident_region(ctx, 5, a.L, a.R * 1024 + nfc, G, (size_t)kWrCntWords, s, &region));
  WrLoop p{};
  p.a = a;
  p.G = G;
  p.nfc = nfc;
  p.nchk = (a.R + kRC - 1) / kRC;
  p.tickets = reinterpret_cast<unsigned long long*>(region);  // region layout: lstm_persist.hip
  p.tmo = region + 32;
  p.cnt = region + 64;
  p.fail_host = host_flags(ctx);
  if (!p.fail_host) return AVC_ERR_HIP;
  p.spin_limit = coresident_spin_limit();
  if (g_wr_inject > 0) {  // test hook: this launch gives up at its first unmet poll
    --g_wr_inject;
    p.spin_limit = 0;
  }
  p.stamps = stamps;
  p.nstamp = stamps ? g_wr_nstamp : 0;
  void* args[] = {&p};
  hipEvent_t ev = timing_begin(TC_WAVERNN, s);
  AVC_TRY(coresident_dispatch(ctx, (const void*)wr_loop_kernel, dim3(G), dim3(256), args, kWrLdsFloats * 4, s));
  if (ev) timing_end(TC_WAVERNN, ev, s, (double)a.L * 2.0 * macs * a.R, (double)a.L * 4.0 * macs);
  AVC_HIP(hipStreamSynchronize(s));
  const int rc = persist_guard(ctx);  // this launch gave up: its samples are NaN
  *gave_up = rc == AVC_ERR_DEVICE;
  return rc;
}

// numpy.linspace(a, b, n)[k] in float64: a + k·(b - a)/(n - 1), the last point exactly b
__device__ __forceinline__ double linspace_at(double a, double b, int n, int k) {
  if (n == 1) return a;
  if (k == n - 1) return b;
  return a + (double)k * ((b - a) / (double)(n - 1));
}

// xfade_and_unfold + crop + 20-hop fade-out (model.py:316-329, 341-399) in float64, then float32
__global__ void wr_unfold_kernel(int R, int L, int batched, int target, int overlap, long wave_len, int fade_n,
                                 const float* __restrict__ y, float* __restrict__ wave) {
  for (long q = blockIdx.x * 256L + threadIdx.x; q < wave_len; q += (long)gridDim.x * 256) {
    double v = 0.0;
    if (batched) {
      const long stride = (long)target + overlap;
      const int silence = overlap / 2, fade = overlap - silence;
      long b0 = (q - L) / stride;
      if (b0 < 0) b0 = 0;
      for (long b = b0; b < R; ++b) {
        const long p = q - b * stride;
        if (p < 0) break;
        if (p >= L) continue;
        double s = (double)y[b * L + p];
        if (p < overlap) s *= p < silence ? 0.0 : sqrt(0.5 * (1.0 + linspace_at(-1.0, 1.0, fade, (int)p - silence)));
        if (p >= L - overlap) {
          const long pp = p - (L - overlap);
          s *= pp < silence ? 1.0 : sqrt(0.5 * (1.0 - linspace_at(-1.0, 1.0, fade, (int)(pp - silence))));
        }
        v += s;
      }
    } else {
      v = (double)y[q];
    }
    const long tail0 = wave_len - fade_n;
    if (q >= tail0 && tail0 >= 0) v *= linspace_at(1.0, 0.0, fade_n, (int)(q - tail0));
    wave[q] = (float)v;
  }
}

constexpr int kChunk = 32;  // sample steps per captured graph

// the five launches of one sample step
int launch_step(const WrStep& a, hipStream_t s) {
  wr_gru_kernel<1><<<a.H / 2, 256, 0, s>>>(a);
  wr_gru_kernel<2><<<a.H / 2, 256, 0, s>>>(a);
  wr_fc_kernel<1><<<(a.Fc + 7) / 8, 256, 0, s>>>(a);
  wr_fc_kernel<2><<<(a.Fc + 7) / 8, 256, 0, s>>>(a);
  wr_out_kernel<<<a.R, 256, 0, s>>>(a);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

// Parameter order: the float tensors of WaveRNN.state_dict() (step and num_batches_tracked left out).
enum : int {
  W_CONV_IN = 0, W_BN0 = 1, W_LAYERS = 5, W_PER_LAYER = 10,
};

struct WrDims {
  int F, C, A4, RB, H, Fc, NC, pad, f0, f1, f2;
  int base_after_layers() const { return W_LAYERS + W_PER_LAYER * RB; }
  int count() const { return base_after_layers() + 2 + 3 + 2 + 8 + 6; }
};

int check_dims(const WrDims& d) {
  AVC_CHECK_ARG(d.F > 0 && d.F <= 512 && d.C > 0 && d.A4 > 0 && d.A4 % 4 == 0 && d.RB >= 0 && d.RB <= 64,
                "wavernn: feat_dims, compute_dims, res_out_dims (multiple of 4) or res_blocks out of range");
  AVC_CHECK_ARG(d.H >= 64 && d.H <= 512 && d.H % 2 == 0 && d.H + d.A4 / 4 <= 64 * kKJ && d.Fc >= 8 &&
                    d.Fc + d.A4 / 4 <= 64 * kKJ,
                "wavernn: need 64 <= rnn_dims <= 512 (even) and rnn_dims + aux_dims, fc_dims + aux_dims <= 576");
  AVC_CHECK_ARG(d.H % 4 == 0 && d.Fc % 4 == 0 && (d.A4 / 4) % 4 == 0,
                "wavernn: rnn_dims, fc_dims and res_out_dims / 4 must be multiples of 4 (float4 staging)");
  AVC_CHECK_ARG(d.NC > 0 && d.NC <= 32, "wavernn: n_classes must be 1..32 (MOL 30, RAW 2 * bits)");
  AVC_CHECK_ARG(d.pad >= 0 && d.f0 > 0 && d.f1 > 0 && d.f2 > 0, "wavernn: bad pad / upsample factors");
  return AVC_OK;
}

// Up-sampling of a generate() input (1, F, T) with the padding generate applies:
// m [Ltot][F], auxf [T][A4] (frame rate), Ltot = T·hop.  Scratch from sc.
// add_pad = 0: the mel already carries `pad` context frames on both sides (the reference's
// forward(x, mels), model.py:186): then Ltot = (T - 2 pad)·hop and auxf has T - 2 pad frames.
int upsample(avc_context* ctx, Scratch& sc, const WrDims& d, int T, const float* mel, const float* const* P,
             float* m, float* auxf, hipStream_t s, int add_pad = 1) {
  (void)ctx;
  const int padf = add_pad ? d.pad : 0;
  const int Tp = T + 2 * padf, k = 2 * d.pad + 1;
  AVC_CHECK_ARG(Tp - 2 * d.pad >= 1, "wavernn: need at least one mel frame beyond the context");
  AVC_TAKE(tm, float, (size_t)Tp * d.F, sc);
  AVC_TAKE(cm, float, (size_t)Tp * d.F, sc);
  wr_pad_mel_kernel<<<ew((long)d.F * Tp), 256, 0, s>>>(d.F, T, padf, mel, tm, cm);
  // MelResNet: conv_in (valid, k = 2 pad + 1) -> BN -> relu, res blocks, conv_out (model.py:34-49)
  const int Tr = Tp - k + 1;  // frames of the aux features (== T when generate pads)
  AVC_TAKE(xa, float, (size_t)Tr * d.C, sc);
  AVC_TAKE(xb, float, (size_t)Tr * d.C, sc);
  AVC_TAKE(xc, float, (size_t)Tr * d.C, sc);
  wr_frame_layer_kernel<<<ew((long)Tr * d.C), 256, 0, s>>>(Tr, d.F, d.C, k, tm, P[W_CONV_IN], nullptr, P[W_BN0],
                                                          P[W_BN0 + 1], P[W_BN0 + 2], P[W_BN0 + 3], 1, nullptr, xa);
  for (int l = 0; l < d.RB; ++l) {
    const float* const* q = P + W_LAYERS + W_PER_LAYER * l;
    wr_frame_layer_kernel<<<ew((long)Tr * d.C), 256, 0, s>>>(Tr, d.C, d.C, 1, xa, q[0], nullptr, q[2], q[3], q[4],
                                                            q[5], 1, nullptr, xb);
    wr_frame_layer_kernel<<<ew((long)Tr * d.C), 256, 0, s>>>(Tr, d.C, d.C, 1, xb, q[1], nullptr, q[6], q[7], q[8],
                                                            q[9], 0, xa, xc);
    std::swap(xa, xc);
  }
  const int o = d.base_after_layers();
  wr_frame_layer_kernel<<<ew((long)Tr * d.A4), 256, 0, s>>>(Tr, d.C, d.A4, 1, xa, P[o], P[o + 1], nullptr, nullptr,
                                                           nullptr, nullptr, 0, nullptr, auxf);
  // mel: three stretch + smoothing passes, the last one cropped and time-major (model.py:86-93)
  const int fs[3] = {d.f0, d.f1, d.f2};
  const long hop = (long)d.f0 * d.f1 * d.f2;
  const long L1 = (long)Tp * fs[0], L2 = L1 * fs[1];
  AVC_TAKE(s1, float, (size_t)d.F * L1, sc);
  AVC_TAKE(s2, float, (size_t)d.F * L2, sc);
  wr_stretch_conv_kernel<<<ew((long)d.F * L1), 256, 0, s>>>(d.F, Tp, fs[0], P[o + 2], cm, s1, 0, 0);
  wr_stretch_conv_kernel<<<ew((long)d.F * L2), 256, 0, s>>>(d.F, (int)L1, fs[1], P[o + 3], s1, s2, 0, 0);
  wr_stretch_conv_kernel<<<ew((long)d.F * Tr * hop), 256, 0, s>>>(d.F, (int)L2, fs[2], P[o + 4], s2, m, 1,
                                                                  (int)(d.pad * hop));
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

size_t upsample_scratch(const WrDims& d, int T) {
  const size_t Tp = T + 2 * d.pad, hop = (size_t)d.f0 * d.f1 * d.f2;
  return 4 * (2 * Tp * d.F + 3 * (size_t)T * d.C + (size_t)d.F * Tp * d.f0 + (size_t)d.F * Tp * d.f0 * d.f1) +
         8 * 256;
}

}  // namespace
}  // namespace avc

using namespace avc;

extern "C" {

int avc_wavernn_param_count(int res_blocks) { return W_LAYERS + W_PER_LAYER * res_blocks + 2 + 3 + 2 + 8 + 6; }

int avc_wavernn_upsample(avc_context* ctx, const int* dims, int T, const float* const* params, const float* mel,
                         float* m, float* aux, void* stream) {
  AVC_CHECK_ARG(ctx && dims && params && mel && m && aux, "NULL pointer");
  const WrDims d{dims[0], dims[1], dims[2], dims[3], dims[4], dims[5], dims[6], dims[7], dims[8], dims[9], dims[10]};
  AVC_TRY(check_dims(d));
  for (int k = 0; k < d.count(); ++k) AVC_CHECK_ARG(params[k] != nullptr, "wavernn: NULL parameter");
  AVC_TRY(ensure_arena(ctx, upsample_scratch(d, T)));
  Scratch sc(ctx);
  return upsample(ctx, sc, d, T, mel, params, m, aux, reinterpret_cast<hipStream_t>(stream));
}

int avc_wavernn_generate(avc_context* ctx, const int* dims, int T, const float* const* params, const float* mel,
                         int batched, int target, int overlap, int mol, unsigned long long seed,
                         const float* x_teacher, float* logits, float* samples, float* wave, void* stream) {
  // the stamp buffer (avc_debug_wavernn_stamps) belongs to this call only, whichever path it takes:
  // a later loop launch never writes into a buffer the caller may have freed since
  unsigned long long* const stamps = g_wr_stamps;
  g_wr_stamps = nullptr;
  AVC_CHECK_ARG(ctx && dims && params && mel, "NULL pointer");
  const WrDims d{dims[0], dims[1], dims[2], dims[3], dims[4], dims[5], dims[6], dims[7], dims[8], dims[9], dims[10]};
  AVC_TRY(check_dims(d));
  for (int k = 0; k < d.count(); ++k) AVC_CHECK_ARG(params[k] != nullptr, "wavernn: NULL parameter");
  AVC_CHECK_ARG(T >= 1, "wavernn: need at least one mel frame");
  AVC_CHECK_ARG(!batched || (target > 0 && overlap > 0), "wavernn: batched generation needs target, overlap > 0");
  AVC_CHECK_ARG(!x_teacher || logits, "wavernn: teacher-forced mode writes logits");
  const long hop = (long)d.f0 * d.f1 * d.f2;
  // generate() pads `pad` zero frames on both sides; teacher-forced calls are the reference's
  // forward(x, mels), whose mel carries real context frames there instead
  const int add_pad = x_teacher ? 0 : 1;
  const int Tf = add_pad ? T : T - 2 * d.pad;
  AVC_CHECK_ARG(Tf >= 1, "wavernn: forward(x, mels) needs more than 2 * pad mel frames");
  const long Ltot = (long)Tf * hop;
  const int A = d.A4 / 4;
  // fold geometry (model.py:311-324): rows of target + 2 overlap positions, stride target + overlap
  long R = 1, L = Ltot, stride = 0;
  if (batched) {
    R = (Ltot - overlap) / (target + overlap);
    const long ext = R * (overlap + target) + overlap;
    if (Ltot - ext != 0) ++R;
    L = (long)target + 2 * overlap;
    stride = (long)target + overlap;
  }
  AVC_CHECK_ARG(R >= 1 && R <= 65535 && L <= (1L << 30), "wavernn: sequence too long for one call");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t H = d.H;
  const size_t need = upsample_scratch(d, T) + 4 * ((size_t)Ltot * d.F + (size_t)T * d.A4 + (Ltot + 1) * H +
                                                    (size_t)R * (1 + 7 * H + 2 * d.Fc) + (size_t)R * L) +
                      32 * 256;
  AVC_TRY(ensure_arena(ctx, need));
  Scratch sc(ctx);
  AVC_TAKE(m, float, (size_t)Ltot * d.F, sc);
  AVC_TAKE(auxf, float, (size_t)Tf * d.A4, sc);
  {
    Scratch up(ctx);
    AVC_TRY(upsample(ctx, up, d, T, mel, params, m, auxf, s, add_pad));
  }
  const int o = d.base_after_layers() + 5;  // I.weight
  AVC_TAKE(pI, float, (size_t)(Ltot + 1) * H, sc);
  if (g_wr_proj_tiled)
    wr_input_proj_tiled_kernel<<<dim3((unsigned)((Ltot + 1 + 63) / 64), (unsigned)((d.H + 63) / 64)), 256, 0, s>>>(
        1, Ltot, d.H, d.F, A, (int)hop, Tf, d.A4, m, auxf, params[o], params[o + 1], pI);
  else
    wr_input_proj_kernel<<<ew((Ltot + 1) * (long)H), 256, 0, s>>>(1, Ltot, d.H, d.F, A, (int)hop, Tf, d.A4, m, auxf,
                                                                params[o], params[o + 1], pI);
  AVC_LAUNCH_CHECK();
  AVC_TAKE(ctr, int, 64, sc);
  AVC_TAKE(wi0, float, H, sc);
  wr_column_kernel<<<ew(d.H), 256, 0, s>>>(d.H, 1 + d.F + A, params[o], wi0);
  AVC_TAKE(x_prev, float, R, sc);
  AVC_TAKE(h1, float, 2 * R * H, sc);
  AVC_TAKE(h2, float, 2 * R * H, sc);
  AVC_TAKE(t1, float, R * H, sc);
  AVC_TAKE(t2, float, R * H, sc);
  AVC_TAKE(y1, float, (size_t)R * d.Fc, sc);
  AVC_TAKE(y2, float, (size_t)R * d.Fc, sc);
  float* out = samples;
  if (!out) {
    out = sc.take<float>((size_t)R * L);
    if (!out) return AVC_ERR_WORKSPACE;
  }
  WrStep a{};
  a.R = (int)R; a.L = (int)L; a.H = d.H; a.Fc = d.Fc; a.A = A; a.NC = d.NC; a.auxd = d.A4; a.hop = (int)hop;
  a.Tf = Tf; a.Ltot = Ltot; a.stride = stride; a.batched = batched ? 1 : 0; a.mol = mol ? 1 : 0;
  a.teacher = x_teacher ? 1 : 0; a.seed = seed;
  a.step = ctr; a.done = ctr + 32;
  a.pI = pI; a.auxf = auxf; a.WI = params[o]; a.wi_ld = 1 + d.F + A; a.wi0 = wi0;
  a.Wih1 = params[o + 2]; a.Whh1 = params[o + 3]; a.bih1 = params[o + 4]; a.bhh1 = params[o + 5];
  a.Wih2 = params[o + 6]; a.Whh2 = params[o + 7]; a.bih2 = params[o + 8]; a.bhh2 = params[o + 9];
  a.W1 = params[o + 10]; a.b1 = params[o + 11]; a.W2 = params[o + 12]; a.b2 = params[o + 13];
  a.W3 = params[o + 14]; a.b3 = params[o + 15];
  a.x_prev = x_prev; a.h1 = h1; a.h2 = h2; a.t1 = t1; a.t2 = t2; a.y1 = y1; a.y2 = y2;
  a.out = out; a.logits = logits; a.x_tf = x_teacher;
  wr_init_state_kernel<<<ew(2 * R * (long)H), 256, 0, s>>>((int)R, d.H, d.Fc, a.step, a.done, x_prev, h1, h2);
  AVC_LAUNCH_CHECK();
  // the sequential loop: chunks of kChunk steps captured once into a graph and replayed
  if (!ctx->capture_stream) AVC_HIP(hipStreamCreateWithFlags(&ctx->capture_stream, hipStreamNonBlocking));
  hipStream_t cs = ctx->capture_stream;
  const long chunks = (L + kChunk - 1) / kChunk;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  // per-step algorithmic work of every fold row (timing class "wavernn"): GRU1 6·H·H, GRU2
  // 3·H·(H + A) + 3·H·H, fc1 Fc·(H + A), fc2 Fc·(Fc + A), fc3 NC·Fc MACs, every weight read once
  // per step
  const double macs = 6.0 * H * H + 3.0 * H * (H + A) + 3.0 * H * H + (double)d.Fc * (H + A) +
                      (double)d.Fc * (d.Fc + A) + (double)d.NC * d.Fc;
  bool per_step = !wr_loop_eligible(a);
  if (!per_step) {
    bool gave_up = false;
    const int rc = wr_loop_run(ctx, a, s, macs, stamps, &gave_up);
    if (rc != AVC_OK && !gave_up) return rc;
    if (gave_up) {
      // The loop needs all rnn_dims / 2 workgroups resident at once; with CUs held elsewhere it gave
      // up (persist_guard has reset the counter regions).  The per-step graph path forms the same
      // sums in the same order (bit-identical samples), so the call is re-run there from a fresh state.
      ++g_wr_fallbacks;
      wr_init_state_kernel<<<ew(2 * R * (long)H), 256, 0, s>>>((int)R, d.H, d.Fc, a.step, a.done, x_prev, h1, h2);
      AVC_LAUNCH_CHECK();
      per_step = true;
    }
  }
  if (!per_step) {
  } else if (chunks > 1) {
    AVC_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed));
    int rc = AVC_OK;
    for (int k = 0; k < kChunk && rc == AVC_OK; ++k) rc = launch_step(a, cs);
    const hipError_t e = hipStreamEndCapture(cs, &graph);
    if (rc != AVC_OK) {
      if (graph) (void)hipGraphDestroy(graph);
      return rc;
    }
    AVC_HIP(e);
    const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
      (void)hipGraphDestroy(graph);
      AVC_HIP(ei);
    }
    for (long c = 0; c < chunks; ++c) {
      hipEvent_t ev = timing_begin(TC_WAVERNN, s);
      const hipError_t el = hipGraphLaunch(exec, s);
      if (ev) timing_end(TC_WAVERNN, ev, s, kChunk * 2.0 * macs * R, kChunk * 4.0 * macs);
      if (el != hipSuccess) {
        (void)hipGraphExecDestroy(exec);
        (void)hipGraphDestroy(graph);
        AVC_HIP(el);
      }
    }
    // generate() returns a host waveform anyway: wait here, then release the graph
    const hipError_t es = hipStreamSynchronize(s);
    (void)hipGraphExecDestroy(exec);
    (void)hipGraphDestroy(graph);
    AVC_HIP(es);
  } else {
    for (long k = 0; k < L; ++k) AVC_TRY(launch_step(a, s));
  }
  if (wave && !x_teacher) {
    const long wave_len = (long)(T - 1) * hop;
    AVC_CHECK_ARG(wave_len >= 20 * hop, "wavernn: generate() fades out the last 20 hops; need T >= 21 frames");
    wr_unfold_kernel<<<ew(wave_len), 256, 0, s>>>((int)R, (int)L, batched ? 1 : 0, target, overlap, wave_len,
                                                  (int)(20 * hop), out, wave);
    AVC_LAUNCH_CHECK();
  }
  return AVC_OK;
}

int avc_wavernn_proj_tiled(int on) {
  AVC_CHECK_ARG(on == 0 || on == 1, "avc_wavernn_proj_tiled: on must be 0 or 1");
  avc::g_wr_proj_tiled = on;
  return AVC_OK;
}

int avc_wavernn_persist(int on) {
  AVC_CHECK_ARG(on == 0 || on == 1, "avc_wavernn_persist: on must be 0 or 1");
  avc::g_wr_persist = on;
  return AVC_OK;
}

int avc_debug_wavernn_inject(int launches) {
  AVC_CHECK_ARG(launches >= 0, "avc_debug_wavernn_inject: launches must be >= 0");
  avc::g_wr_inject = launches;
  return AVC_OK;
}

// Diagnostics: the next loop launch writes s_memrealtime stamps (100 MHz) of its first `steps`
// steps into buf [rnn_dims / 2][steps][24] (u64; per op: start, wait done, end).
int avc_debug_wavernn_stamps(void* buf, int steps) {
  AVC_CHECK_ARG(steps >= 0 && (buf || steps == 0), "avc_debug_wavernn_stamps: bad arguments");
  avc::g_wr_stamps = static_cast<unsigned long long*>(buf);
  avc::g_wr_nstamp = steps;
  return AVC_OK;
}

int avc_wavernn_fallbacks(void) { return avc::g_wr_fallbacks; }

int avc_wavernn_persist_eligible(int rows, int rnn_dims, int fc_dims) {
  avc::WrStep a{};
  a.R = rows; a.H = rnn_dims; a.Fc = fc_dims; a.L = 1;
  const int on = avc::g_wr_persist;
  avc::g_wr_persist = 1;
  const bool ok = avc::wr_loop_eligible(a);
  avc::g_wr_persist = on;
  return ok ? 1 : 0;
}

// Rows and steps of a generate() call (so the caller can size `samples` [rows][steps]).
int avc_wavernn_fold_shape(long n_positions, int batched, int target, int overlap, long* rows, long* steps) {
  AVC_CHECK_ARG(rows && steps && n_positions > 0, "wavernn_fold_shape: bad arguments");
  if (!batched) {
    *rows = 1;
    *steps = n_positions;
    return AVC_OK;
  }
  AVC_CHECK_ARG(target > 0 && overlap > 0, "wavernn_fold_shape: target, overlap > 0");
  long R = (n_positions - overlap) / (target + overlap);
  if (n_positions - (R * (overlap + target) + overlap) != 0) ++R;
  *rows = R;
  *steps = (long)target + 2 * overlap;
  return AVC_OK;
}

}  // extern "C"
