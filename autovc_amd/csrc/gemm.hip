// fp32 MFMA GEMM for gfx950 (v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulate).
//
// Block = 256 threads = 4 waves in a 2x2 layout; block tile BM x BN, K-step BK = 32.  Each
// wave owns a (BM/2) x (BN/2) sub-tile as TM x TN 32x32 accumulators.  Operand tiles are
// staged global -> registers -> LDS in a k-major image ([BK][BM+4]) so that the per-lane MFMA
// fragment reads (lane l reads column l&31 of row k) are conflict-free ds_read_b32, and
// double-buffered so the next tile's global loads are in flight during the MFMAs of the
// current one (one barrier per K-step).  The row-shift in the A/B addressing implements the
// Conv1d taps implicitly (no im2col buffer): in time-major frame rows a shift of one frame is
// a shift of B rows, and rows outside the sequence read as the zero padding.
#include "gemm.h"
#include "timing.h"

namespace avc {

namespace {

constexpr int BK = 32;
typedef float f32x16 __attribute__((ext_vector_type(16)));

// branch-free masked operand load: the address is clamped to the (valid) operand base when the
// element is outside the problem/padding, and the value replaced by zero.
__device__ __forceinline__ float4 sel4(bool ok, float4 v) {
  return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}

__device__ __forceinline__ float act_apply(float v, int act) {
  if (act == AVC_ACT_RELU) return v > 0.f ? v : 0.f;
  if (act == AVC_ACT_TANH) return tanhf(v);
  return v;
}

template <int BM, int BN, int WM, int WN, int AT, int BT>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(GemmDesc d, int tilesM, int tilesN,
                                                            int kt_per_tap, int kps, int nsplit,
                                                            float* __restrict__ slab) {
  constexpr int NT = 64 * WM * WN;            // threads
  constexpr int PA = BM + 4, PB = BN + 4;     // padded k-major LDS rows (16-B aligned)
  constexpr int WTM = BM / WM, WTN = BN / WN; // wave tile
  constexpr int TM = WTM / 32, TN = WTN / 32; // 32x32 MFMA tiles per wave
  constexpr int NA = BM * BK / 4 / NT, NB = BN * BK / 4 / NT;  // float4 staged per thread
  static_assert(NA * NT * 4 == BM * BK && NB * NT * 4 == BN * BK, "tile/thread mismatch");
  __shared__ __attribute__((aligned(16))) float lds[2 * BK * (PA + PB)];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;

  // XCD-aware bijective remap: blocks sharing an XCD (bid % 8) get consecutive tiles, i.e.
  // the same A row-panel, so the panel is served from that XCD's L2.
  const int nwg = tilesM * tilesN;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  const int tm = wgid / tilesN, tn = wgid - tm * tilesN;
  const int z = blockIdx.y % d.nz, split = blockIdx.y / d.nz;

  // kernel-argument fields copied to scalars (a lambda capturing `d` would force it to scratch)
  const int M = d.M, N = d.N, Kc = d.Kc;
  const float* __restrict__ Ab = d.A + (long)z * d.a_zoff;
  const float* __restrict__ Bb = d.B;
  const long lda = d.lda, ldb = d.ldb, a_rows = d.a_rows, b_rows = d.b_rows;
  const long a_shift0 = d.a_shift0, a_tapshift = d.a_tapshift, b_tapoff = d.b_tapoff;
  const long bshift = d.b_shift0 + (long)z * d.b_zshift;
  const int ktotal = d.ntaps * kt_per_tap;
  const int kt0 = split * kps;
  const int kt1 = min(ktotal, kt0 + kps);

  f32x16 acc[TM][TN], cmp[TM][TN];
  f32x16 zero16;
#pragma unroll
  for (int e = 0; e < 16; ++e) zero16[e] = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[i][j] = zero16;
      cmp[i][j] = zero16;
    }

  float4 ra[NA], rb[NB];

  // Staging maps.  K-contiguous operand (A row-major / B^T): element idx -> (row, k-quad) with
  // 32 consecutive lanes on 32 consecutive rows (conflict-free ds_write_b32 into the k-major
  // image).  MN-contiguous operand: idx -> (k-row, quad of 4 consecutive rows/cols), one
  // ds_write_b128 per float4.
#define AVC_KC_ROW(IDX) (((IDX) & 31) + 32 * ((IDX) >> 8))
#define AVC_KC_KQ(IDX) (((IDX) >> 5) & 7)

#define AVC_LOAD_TILE(KT)                                                                       \
  {                                                                                             \
    const int tau = (KT) / kt_per_tap;                                                          \
    const int k0 = ((KT) - tau * kt_per_tap) * BK;                                              \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                            \
      const int idx = tid + NT * i;                                                             \
      if (AT == 0) {                                                                            \
        const int m = tm * BM + AVC_KC_ROW(idx), k = k0 + 4 * AVC_KC_KQ(idx);                   \
        const long srow = (long)m + a_shift0 + (long)tau * a_tapshift;                          \
        const bool ok = m < M && k < Kc && srow >= 0 && srow < a_rows;                          \
        ra[i] = sel4(ok, *reinterpret_cast<const float4*>(Ab + (ok ? srow * lda + k : 0)));    \
      } else {                                                                                  \
        const int mq = idx % (BM / 4), krow = idx / (BM / 4);                                   \
        const int m = tm * BM + 4 * mq, k = k0 + krow;                                          \
        const bool ok = m < M && k < Kc;                                                        \
        ra[i] = sel4(ok, *reinterpret_cast<const float4*>(Ab + (ok ? (long)k * lda + m : 0))); \
      }                                                                                         \
    }                                                                                           \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                            \
      const int idx = tid + NT * i;                                                             \
      if (BT == 0) {                                                                            \
        const int nq = idx % (BN / 4), krow = idx / (BN / 4);                                   \
        const int n = tn * BN + 4 * nq, k = k0 + krow;                                          \
        const long srow = (long)k + bshift;                                                     \
        const bool ok = n < N && k < Kc && srow >= 0 && srow < b_rows;                          \
        rb[i] = sel4(ok, *reinterpret_cast<const float4*>(Bb + (ok ? (long)tau * b_tapoff + srow * ldb + n : 0))); \
      } else {                                                                                  \
        const int n = tn * BN + AVC_KC_ROW(idx), k = k0 + 4 * AVC_KC_KQ(idx);                   \
        const bool ok = n < N && k < Kc;                                                        \
        rb[i] = sel4(ok, *reinterpret_cast<const float4*>(Bb + (ok ? (long)tau * b_tapoff + (long)n * ldb + k : 0))); \
      }                                                                                         \
    }                                                                                           \
  }

#define AVC_STORE_TILE(BUF)                                                                     \
  {                                                                                             \
    float* As = lds + (BUF) * BK * (PA + PB);                                                   \
    float* Bs = As + BK * PA;                                                                   \
    _Pragma("unroll") for (int i = 0; i < NA; ++i) {                                            \
      const int idx = tid + NT * i;                                                             \
      if (AT == 0) {                                                                            \
        const int r = AVC_KC_ROW(idx), kq = AVC_KC_KQ(idx);                                     \
        As[(4 * kq + 0) * PA + r] = ra[i].x;                                                    \
        As[(4 * kq + 1) * PA + r] = ra[i].y;                                                    \
        As[(4 * kq + 2) * PA + r] = ra[i].z;                                                    \
        As[(4 * kq + 3) * PA + r] = ra[i].w;                                                    \
      } else {                                                                                  \
        const int mq = idx % (BM / 4), krow = idx / (BM / 4);                                   \
        *reinterpret_cast<float4*>(As + krow * PA + 4 * mq) = ra[i];                            \
      }                                                                                         \
    }                                                                                           \
    _Pragma("unroll") for (int i = 0; i < NB; ++i) {                                            \
      const int idx = tid + NT * i;                                                             \
      if (BT == 0) {                                                                            \
        const int nq = idx % (BN / 4), krow = idx / (BN / 4);                                   \
        *reinterpret_cast<float4*>(Bs + krow * PB + 4 * nq) = rb[i];                            \
      } else {                                                                                  \
        const int c = AVC_KC_ROW(idx), kq = AVC_KC_KQ(idx);                                     \
        Bs[(4 * kq + 0) * PB + c] = rb[i].x;                                                    \
        Bs[(4 * kq + 1) * PB + c] = rb[i].y;                                                    \
        Bs[(4 * kq + 2) * PB + c] = rb[i].z;                                                    \
        Bs[(4 * kq + 3) * PB + c] = rb[i].w;                                                    \
      }                                                                                         \
    }                                                                                           \
  }

  if (kt0 < kt1) AVC_LOAD_TILE(kt0);
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    AVC_STORE_TILE(buf);
    __syncthreads();
    if (kt + 1 < kt1) AVC_LOAD_TILE(kt + 1);
    const float* As = lds + buf * BK * (PA + PB);
    const float* Bs = As + BK * PA;
    // Each K-tile (32 products) is accumulated by a fresh MFMA chain and added to the running
    // total with Kahan compensation: a single fp32 FMA chain over K = 2560 (Conv1d, 5 taps x 512)
    // is ~8x less accurate than oneDNN's blocked CPU accumulation, and the train-mode BatchNorms
    // of the postnet amplify that error into mel_post (DESIGN.md "Numerics").
    f32x16 part[TM][TN];
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int kr = 2 * s + (lane >> 5);
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[kr * PA + wm * WTM + 32 * i + (lane & 31)];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[kr * PB + wn * WTN + 32 * j + (lane & 31)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], s == 0 ? zero16 : part[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float y = part[i][j][e] - cmp[i][j][e];
          const float t = acc[i][j][e] + y;
          cmp[i][j][e] = (t - acc[i][j][e]) - y;
          acc[i][j][e] = t;
        }
  }
#undef AVC_LOAD_TILE
#undef AVC_STORE_TILE
#undef AVC_KC_ROW
#undef AVC_KC_KQ

  // ---- epilogue -------------------------------------------------------------------------
  const int row_base = tm * BM + wm * WTM + 4 * (lane >> 5);
  const int col_base = tn * BN + wn * WTN + (lane & 31);
  if (nsplit > 1) {
    float* out = slab + ((long)(split * d.nz + z) * d.M) * d.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = col_base + 32 * j;
        if (col >= d.N) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
          if (row < d.M) out[(long)row * d.N + col] = acc[i][j][e];
        }
      }
    return;
  }

  float* __restrict__ C = d.C + (long)z * d.c_zoff;
  float csum[TN], csq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    csum[j] = 0.f;
    csq[j] = 0.f;
    const int col = col_base + 32 * j;
    const bool colok = col < d.N;
    float bias = 0.f;
    if (colok) {
      if (d.bias0) bias += d.bias0[col];
      if (d.bias1) bias += d.bias1[col];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
        if (!colok || row >= d.M) continue;
        const float v = act_apply(acc[i][j][e] + bias, d.act);
        float* p = C + (long)row * d.ldc + (long)col * d.ldc_col;
        if (d.accumulate) *p += v; else *p = v;
        csum[j] += v;
        csq[j] += v * v;
      }
  }

  if (d.stats) {
    __syncthreads();  // LDS operand tiles are dead now; reuse them for the column reduction
    float* red = lds;  // [WM][2 (sum,sq)][BN]
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      float s = csum[j] + __shfl_xor(csum[j], 32);
      float s2 = csq[j] + __shfl_xor(csq[j], 32);
      if (lane < 32) {
        const int cl = wn * WTN + 32 * j + lane;
        red[(wm * 2 + 0) * BN + cl] = s;
        red[(wm * 2 + 1) * BN + cl] = s2;
      }
    }
    __syncthreads();
    for (int cl = tid; cl < BN; cl += NT) {
      const int col = tn * BN + cl;
      if (col < d.N) {
        float s = 0.f, s2 = 0.f;
#pragma unroll
        for (int r = 0; r < WM; ++r) {
          s += red[(r * 2 + 0) * BN + cl];
          s2 += red[(r * 2 + 1) * BN + cl];
        }
        d.stats[((long)tm * 2 + 0) * d.N + col] = s;
        d.stats[((long)tm * 2 + 1) * d.N + col] = s2;
      }
    }
  }
}

__global__ void splitk_reduce_kernel(GemmDesc d, int nsplit, const float* __restrict__ slab) {
  const long total = (long)d.nz * d.M * d.N;
  const long MN = (long)d.M * d.N;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int z = (int)(idx / MN);
    const long rem = idx - z * MN;
    const int m = (int)(rem / d.N), n = (int)(rem - (long)m * d.N);
    float s = 0.f;
    for (int sp = 0; sp < nsplit; ++sp) s += slab[((long)sp * d.nz + z) * MN + rem];
    if (d.bias0) s += d.bias0[n];
    if (d.bias1) s += d.bias1[n];
    s = act_apply(s, d.act);
    float* p = d.C + (long)z * d.c_zoff + (long)m * d.ldc + (long)n * d.ldc_col;
    if (d.accumulate) *p += s; else *p = s;
  }
}

struct Plan {
  int bm, bn, tilesM, tilesN, kt_per_tap, ktotal, nsplit, kps;
};

Plan make_plan(const GemmDesc& d, int force_split) {
  Plan p;
  const bool big = (long)d.M * d.N >= 256L * 128 * 128 / 2;
  p.bm = big ? 128 : 64;
  p.bn = big ? 128 : 64;
  p.tilesM = (d.M + p.bm - 1) / p.bm;
  p.tilesN = (d.N + p.bn - 1) / p.bn;
  p.kt_per_tap = (d.Kc + BK - 1) / BK;
  p.ktotal = p.kt_per_tap * d.ntaps;
  const long blocks = (long)p.tilesM * p.tilesN * d.nz;
  int ns = 1;
  if (force_split > 0) {
    ns = force_split;
  } else if (!d.stats && blocks < 256 && p.ktotal >= 16) {
    ns = (int)((512 + blocks - 1) / blocks);
    ns = std::min(ns, p.ktotal / 8);
    ns = std::min(ns, 32);
    ns = std::max(ns, 1);
  }
  p.kps = (p.ktotal + ns - 1) / ns;
  p.nsplit = (p.ktotal + p.kps - 1) / p.kps;
  if (p.nsplit < 1) p.nsplit = 1;
  return p;
}

template <int BM, int BN, int WM, int WN>
void launch(const GemmDesc& d, const Plan& p, float* slab, hipStream_t s) {
  dim3 grid(p.tilesM * p.tilesN, d.nz * p.nsplit);
  constexpr int NT = 64 * WM * WN;
  const int code = d.a_trans * 2 + d.b_trans;
  if (code == 0)
    gemm_kernel<BM, BN, WM, WN, 0, 0><<<grid, NT, 0, s>>>(d, p.tilesM, p.tilesN, p.kt_per_tap, p.kps, p.nsplit, slab);
  else if (code == 1)
    gemm_kernel<BM, BN, WM, WN, 0, 1><<<grid, NT, 0, s>>>(d, p.tilesM, p.tilesN, p.kt_per_tap, p.kps, p.nsplit, slab);
  else if (code == 2)
    gemm_kernel<BM, BN, WM, WN, 1, 0><<<grid, NT, 0, s>>>(d, p.tilesM, p.tilesN, p.kt_per_tap, p.kps, p.nsplit, slab);
  else
    gemm_kernel<BM, BN, WM, WN, 1, 1><<<grid, NT, 0, s>>>(d, p.tilesM, p.tilesN, p.kt_per_tap, p.kps, p.nsplit, slab);
}

}  // namespace

int gemm_stats_rows(int M, int N) {
  GemmDesc d;
  d.M = M;
  d.N = N;
  d.Kc = 32;
  return make_plan(d, 1).bm;
}

size_t gemm_scratch_bytes(const GemmDesc& d) {
  Plan p = make_plan(d, 0);
  if (p.nsplit <= 1) return 0;
  return (size_t)p.nsplit * d.nz * d.M * d.N * sizeof(float) + 256;
}

int gemm_run(avc_context* ctx, GemmDesc d, hipStream_t stream, int force_split) {
  AVC_CHECK_ARG(d.M > 0 && d.N > 0 && d.Kc > 0 && d.ntaps > 0 && d.nz > 0, "gemm: empty problem");
  AVC_CHECK_ARG(d.Kc % 4 == 0 || (d.a_trans == 1 && d.b_trans == 0),
                "gemm: reduction dim must be a multiple of 4 for K-contiguous operands");
  AVC_CHECK_ARG(d.a_trans == 0 || d.M % 4 == 0, "gemm: M must be a multiple of 4 (A^T)");
  AVC_CHECK_ARG(d.b_trans == 1 || d.N % 4 == 0, "gemm: N must be a multiple of 4 (B)");
  AVC_CHECK_ARG(d.lda % 4 == 0 && d.ldb % 4 == 0, "gemm: leading dims must be multiples of 4");
  AVC_CHECK_ARG(aligned16(d.A) && aligned16(d.B), "gemm: operands must be 16-byte aligned");
  AVC_CHECK_ARG(d.a_trans == 0 || (d.ntaps == 1 || d.a_tapshift == 0), "gemm: taps need A row-major");
  if (d.a_rows == 0) d.a_rows = d.a_trans ? d.Kc : d.M;
  if (d.b_rows == 0) d.b_rows = d.b_trans ? d.N : d.Kc;
  Plan p = make_plan(d, force_split);
  if (d.stats) p.nsplit = 1, p.kps = p.ktotal;
  d.stats_bm = p.bm;
  Scratch sc(ctx);
  float* slab = nullptr;
  if (p.nsplit > 1) {
    slab = sc.take<float>((size_t)p.nsplit * d.nz * d.M * d.N);
    if (!slab) return AVC_ERR_WORKSPACE;
  }
  hipEvent_t ev = timing_begin(TC_GEMM, stream);
  if (p.bm == 128) launch<128, 128, 2, 4>(d, p, slab, stream);
  else launch<64, 64, 2, 2>(d, p, slab, stream);
  AVC_LAUNCH_CHECK();
  if (ev) {
    const double flops = 2.0 * d.M * d.N * (double)d.Kc * d.ntaps * d.nz;
    const double bytes = 4.0 * ((double)d.M * d.Kc * d.ntaps + (double)d.Kc * d.N * d.ntaps + (double)d.M * d.N) * d.nz;
    timing_end(TC_GEMM, ev, stream, flops, bytes);
  }
  if (p.nsplit > 1) {
    const long total = (long)d.nz * d.M * d.N;
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    splitk_reduce_kernel<<<blocks, 256, 0, stream>>>(d, p.nsplit, slab);
    AVC_LAUNCH_CHECK();
  }
  return AVC_OK;
}

}  // namespace avc
