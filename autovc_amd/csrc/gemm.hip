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
#include <type_traits>
#include <vector>

#include "gemm.h"
#include "timing.h"

namespace avc {

namespace {

constexpr int BK = 32;
#ifndef AVC_GEMM_NOLOAD
#define AVC_GEMM_NOLOAD 0  // diagnostic build only (-DAVC_GEMM_NOLOAD=1): gemm16f skips its LDS-DMA
#endif
#ifndef AVC_GEMM_DIAG_NOREAD
#define AVC_GEMM_DIAG_NOREAD 0  // diagnostic: gemm16f reads its fragments from LDS once, not per K-tile
#endif
#ifndef AVC_GEMM_DIAG_NOBAR
#define AVC_GEMM_DIAG_NOBAR 0  // diagnostic (wrong results): gemm16f skips its per-K-tile barrier
#endif
#ifndef AVC_GEMM_DIAG_NOMFMA
#define AVC_GEMM_DIAG_NOMFMA 0  // diagnostic (wrong results): gemm16f skips its MFMAs (loads, reads, barriers kept)
#endif
#ifndef AVC_GEMM_DIAG_NOEPI
#define AVC_GEMM_DIAG_NOEPI 0  // diagnostic (wrong results): gemm16f returns right after its K loop
#endif
#ifndef AVC_GEMM_DIAG_EPI
#define AVC_GEMM_DIAG_EPI 0  // diagnostic (wrong results): bnf_epilogue pieces skipped, bit 1 the column-tile
                             // wait, bit 2 the partials' combine, bit 4 the tile staging, bit 8 the outputs
#endif
#ifndef AVC_GEMM_DMA_SPREAD
// gemm16f issues the next K-tile's LDS-DMA over the first AVC_GEMM_DMA_SPREAD chunks of the current
// one, between their fragment reads and MFMAs, instead of all DPW pieces right after the barrier
// (round 6: 2 measured -2.4 % on the C2 conv, -2.5 % at C5; 4 less; the pieces after the chunk's
// MFMAs, interleaved with them by sched_group_barrier, or starting at chunk 1, no better; same
// bytes, same bits)
#define AVC_GEMM_DMA_SPREAD 2
#endif
#ifndef AVC_GEMM_DIAG_NOKAHAN
#define AVC_GEMM_DIAG_NOKAHAN 0  // diagnostic: gemm16f folds 128-k partials with a plain add
#endif
typedef float f32x16 __attribute__((ext_vector_type(16)));

// branch-free masked operand load: the address is clamped to the (valid) operand base when the
// element is outside the problem/padding, and the value replaced by zero.
__device__ __forceinline__ float4 sel4(bool ok, float4 v) {
  return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}

#ifndef AVC_GEMM_DIAG_NOACT
#define AVC_GEMM_DIAG_NOACT 0  // diagnostic (wrong results for act != none): act_apply is the identity
#endif
__device__ __forceinline__ float act_apply(float v, int act) {
  if (AVC_GEMM_DIAG_NOACT) return v;
  if (act == AVC_ACT_RELU) return v < 0.f ? 0.f : v;  // NaN propagates, as torch.relu
  if (act == AVC_ACT_TANH) return tanhf(v);
  if (act == AVC_ACT_DBNORM) {
    const float db = 20.f * log10f(fmaxf(1e-5f, v));
    return fminf(fmaxf((db + 100.f) / 100.f, 0.f), 1.f);
  }
  return v;
}

#ifdef AVC_GEMM_EPI_STAMPS
// diagnostic build only: s_memtime per (workgroup, phase) of the fused-BN epilogue, thread 0,
// launches of 256 workgroups (the 512-column convs at B = 64, T = 128; the last one wins)
__device__ unsigned long long g_epi_st[1024][10];
#define AVC_EPI_STAMP(k)                                                                          \
  do {                                                                                            \
    unsigned long long _t;                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (threadIdx.x == 0 && gridDim.x == 256) g_epi_st[blockIdx.x][k] = _t;                     \
  } while (0)
#else
#define AVC_EPI_STAMP(k) do { } while (0)
#endif

// rows of ld floats starting at p are 16-B aligned pieces (store_tile_rows' float4 form)
__device__ __forceinline__ bool g_tile_rows_ok(const float* p, long ld, int unit) {
  return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && (ld & 3) == 0 && unit == 1;
}

// ---- fused BatchNorm epilogue (BnFuse): the column-tile barrier ------------------------------
__device__ unsigned g_bnf_giveups = 0;  // sticky count of timed-out fused launches
typedef __attribute__((address_space(1))) unsigned bnf_gu32;

// One lane waits until *p reaches target (wrap-safe relaxed agent-scope polls, as the persistent
// LSTM kernels' wait_ge_ctl); false = gave up, or another workgroup of this launch (epoch E) did.
// A give-up is reported to the context's pinned word with the top bit set, so its numbers never
// collide with the persistent recurrences' failure numbers (persist_guard compares for change).
__device__ bool bnf_wait(unsigned* p, unsigned target, const BnFuse& bf, unsigned E) {
  bnf_gu32* gp = (bnf_gu32*)p;
  bnf_gu32* gt = (bnf_gu32*)bf.tmo;
  for (unsigned spins = 0;; ++spins) {
    // the give-up word is read beside every poll (one round trip for both): a workgroup that
    // arrives after another one gave up never takes the barrier as passed
    const unsigned v = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned g = __hip_atomic_load(gt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (g == E) return false;
    if ((int)(v - target) >= 0) return true;
    if (spins >= bf.spin_limit) {
      const unsigned old = __hip_atomic_fetch_max(gt, E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old != E) {
        const unsigned n = atomicAdd(&g_bnf_giveups, 1u) + 1u;
        if (bf.fail_host)
          __hip_atomic_store(bf.fail_host, 0x80000000u | n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Tile order: workgroup ids are XCD-contiguous (wgid ranges per XCD), and within them bands of 8
// tile rows are walked column by column, so the ~32 workgroups an XCD runs at once cover an 8 x 4
// block and the next ones reuse the same 8 row tiles from that XCD's L2 while the column tiles
// stream through once (row-major order re-fetched every column tile per row: 51 % L2 hits on
// the 8192 x 4096 x 512 LSTM input product).
__device__ __forceinline__ void tile_of(int wgid, int tilesM, int tilesN, int& tm, int& tn) {
  constexpr int G = 8;
  const int band = G * tilesN;
  const int group = wgid / band, first = group * G;
  const int gsize = min(tilesM - first, G);
  const int local = wgid - group * band;
  tm = first + local % gsize;
  tn = local / gsize;
}

// power-of-two operand scale for the split-f16 products: max |x| -> [2^14, 2^15)
__device__ __forceinline__ float split_scale_of(const unsigned* amax) {
  if (!amax) return 1.f;
  const float m = __uint_as_float(*amax);
  if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, 15 - e);
}

__device__ __forceinline__ float split_unscale(const unsigned* amax_a, const unsigned* amax_b) {
  return 1.f / (split_scale_of(amax_a) * split_scale_of(amax_b));
}

// BatchNorm column partials of one output tile (train mode).  Per column and partial (PARTS = 1:
// the tile's rows; 2: the two 128-row halves of a 256-row tile, make_plan's stats granularity):
// stats[part][0][col] = S, the sum of the column's valid rows, and stats[part][1][col] = Q, the sum
// of squares about the partial's mean S / n.  One pass: each wave sums its rows of a column shifted
// by k, the wave's first row of that column (a lane shuffle away), so S_w = S1 + n_w k and
// Q_w = S2 - S1^2 / n_w carry no cancellation beyond ((mean - k) / std)^2 -- a sample lies within a
// few standard deviations of its mean; the wave rows of a partial are then merged exactly (Chan:
// Q = sum Q_w + sum n_w (S_w / n_w - S / n)^2).  So the variance never comes out of
// E[x^2] - E[x]^2 with fp32 sums: at B = 1 a decoder conv channel's mean is ~17 standard deviations
// and that difference cost ~2^-12 relative in the variance (dec.conv0 5.9e-5 local error against
// fp32 CPU's 6.9e-6).  bn_finalize_kernel combines the partials in fp64 about a common
// shift.  val(i, j, e) = act(acc + bias) as the epilogue stored it (RAW: acc already holds it).
// Every producer (the three GEMM epilogues, the fused BN one) goes through here, so fused and
// unfused chains form the same bits.  SC1: write-through stores (the fused BN's in-launch
// hand-off).  red: >= 2 WM BN floats of LDS, free.
template <int BM, int BN, int WM, int WTN, int TM, int TN, int PARTS, bool RAW, bool SC1>
__device__ __forceinline__ void bn_tile_stats(const GemmDesc& d, const f32x16 (&acc)[TM][TN], const float (&bias)[TN],
                                              float* red, int tm, int tn, int wm, int wn, int lane, int tid, int NT,
                                              int row_base, int col_base) {
  static_assert(PARTS == 1 || (BM == 256 && WM % 2 == 0), "two 128-row partials per 256-row tile");
  constexpr int PR = BM / PARTS, WPP = WM / PARTS, WTM = BM / WM;  // rows / wave rows per partial
  const int M = d.M, N = d.N, act = d.act;
  const auto srs = __builtin_amdgcn_make_buffer_rsrc(d.stats, 0, 0x7fffffff, 0x00020000);
  auto put = [&](long idx, float v) {
    if (SC1) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), srs, (int)(idx * 4), 0, 16 /*sc1*/);
    else d.stats[idx] = v;
  };
  // this wave row's valid rows (its first row, row_base of lane 0, is tm * BM + wm * WTM)
  const long wrow0 = (long)tm * BM + (long)wm * WTM;
  const float nw = (float)max(0L, min((long)WTM, (long)M - wrow0));
  float cs[TN], cq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + 32 * j;
    // the shift: element (0, j, 0) of lane (lane & 31) holds row wrow0 of this lane's column
    const float v00 = RAW ? acc[0][j][0] : act_apply(acc[0][j][0] + bias[j], act);
    const float k = __shfl(v00, lane & 31);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
        if (col >= N || row >= M) continue;
        const float dv = (RAW ? acc[i][j][e] : act_apply(acc[i][j][e] + bias[j], act)) - k;
        s1 += dv;
        s2 = fmaf(dv, dv, s2);
      }
    s1 += __shfl_xor(s1, 32);
    s2 += __shfl_xor(s2, 32);
    // the wave row's (S_w, Q_w) of this column
    cs[j] = nw > 0.f ? fmaf(nw, k, s1) : 0.f;
    cq[j] = nw > 0.f ? fmaxf(s2 - s1 * (s1 / nw), 0.f) : 0.f;
  }
  __syncthreads();  // (the LDS operand ring is dead)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    if (lane < 32) {
      red[(wm * 2 + 0) * BN + wn * WTN + 32 * j + lane] = cs[j];
      red[(wm * 2 + 1) * BN + wn * WTN + 32 * j + lane] = cq[j];
    }
  }
  __syncthreads();
  for (int cl = tid; cl < BN; cl += NT) {
    const int col = tn * BN + cl;
    if (col >= N) continue;
#pragma unroll
    for (int sp = 0; sp < PARTS; ++sp) {
      const long part = (long)tm * PARTS + sp;
      if (part * PR >= M) break;
      const float n = (float)min((long)PR, (long)M - part * PR);
      float S = 0.f;
#pragma unroll
      for (int r = sp * WPP; r < (sp + 1) * WPP; ++r) S += red[(r * 2 + 0) * BN + cl];
      const float m = S / n;
      float Q = 0.f;
#pragma unroll
      for (int r = sp * WPP; r < (sp + 1) * WPP; ++r) {  // Chan's merge of the wave rows
        const float nr = (float)max(0L, min((long)WTM, (long)M - ((long)tm * BM + (long)r * WTM)));
        if (nr > 0.f) {
          const float dm = red[(r * 2 + 0) * BN + cl] / nr - m;
          Q += red[(r * 2 + 1) * BN + cl] + nr * dm * dm;
        }
      }
      put((part * 2 + 0) * N + col, S);
      put((part * 2 + 1) * N + col, Q);
    }
  }
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
  int tm, tn;
  tile_of(wgid, tilesM, tilesN, tm, tn);
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
  float biasv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + 32 * j;
    float bias = 0.f;
    if (col < d.N) {
      if (d.bias0) bias += d.bias0[col];
      if (d.bias1) bias += d.bias1[col];
    }
    biasv[j] = bias;
  }
  {  // (the fallback kernels keep the per-element stores)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + 32 * j;
    const bool colok = col < d.N;
    const float bias = biasv[j];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
        if (!colok || row >= d.M) continue;
        const float v = act_apply(acc[i][j][e] + bias, d.act);
        float* p = C + (long)row * d.ldc + (long)col * d.ldc_col;
        if (d.accumulate) *p += v; else *p = v;
      }
  }
  }

  if (d.stats)  // (the LDS operand tiles are dead now: the column reduction reuses them)
    bn_tile_stats<BM, BN, WM, WTN, TM, TN, 1, false, false>(d, acc, biasv, lds, tm, tn, wm, wn, lane, tid, NT,
                                                            row_base, col_base);
}

// ---- split-fp16 ("3xf16") GEMM for forward products ------------------------------------
//
// Operands are split while they are staged into LDS: x = hi + lo/2^11 with hi = f16(x) and
// lo = f16((x - hi) * 2^11) (the pre-scaled low part stays out of the f16 subnormal range for
// |x| > ~6e-5).  v_mfma_f32_32x32x16_f16 accumulates hi.hi into a per-128-k partial that is
// Kahan-added into the running sum (the same compensation the fp32 kernel uses), and the two
// cross terms hi.lo + lo.hi into a separate fp32 accumulator scaled by 2^11.  3 f16 products run
// 5.3x faster than one fp32 MFMA; the error matches the compensated fp32 kernel.
// Forward operands are range-guarded like the pre-split path below (amax_a / amax_b guard words,
// scale exactly 1 in the normal range).
//
// Block: NT = 64*WM*WN threads; each thread stages one octet (8 consecutive k) of A and of B
// per 32-deep K-tile.  LDS holds MFMA fragment images: [tile32][ksub16][hi|lo][64 lanes][16 B],
// so every fragment read is one conflict-free ds_read_b128 at lane*16.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split8(const float* v, f16x8& hi, f16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 h = (_Float16)v[j];
    hi[j] = h;
    lo[j] = (_Float16)((v[j] - (float)h) * 2048.0f);
  }
}

template <int BM, int BN, int WM, int WN, int BT>
__global__ __launch_bounds__(64 * WM * WN) void gemm16_kernel(GemmDesc d, int tilesM, int tilesN,
                                                              int kt_per_tap, int kps, int nsplit,
                                                              float* __restrict__ slab) {
  constexpr int NT = 64 * WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(BM * 4 == NT && BN * 4 == NT, "one A octet and one B octet per thread");
  constexpr int AIMG = (BM / 32) * 2 * 2 * 1024;  // bytes per buffer
  constexpr int BIMG = (BN / 32) * 2 * 2 * 1024;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * (AIMG + BIMG)];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int nwg = tilesM * tilesN;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  int tm, tn;
  tile_of(wgid, tilesM, tilesN, tm, tn);
  const int z = blockIdx.y % d.nz, split = blockIdx.y / d.nz;

  const int M = d.M, N = d.N, Kc = d.Kc;
  const float* __restrict__ Ab = d.A + (long)z * d.a_zoff;
  const float* __restrict__ Bb = d.B;
  const long lda = d.lda, ldb = d.ldb, a_rows = d.a_rows, b_rows = d.b_rows;
  const long a_shift0 = d.a_shift0, a_tapshift = d.a_tapshift, b_tapoff = d.b_tapoff;
  const long bshift = d.b_shift0 + (long)z * d.b_zshift;
  const int ktotal = d.ntaps * kt_per_tap;
  const int kt0 = split * kps;
  const int kt1 = min(ktotal, kt0 + kps);

  // staging coordinates: K-contiguous operand -> (row = t>>2, octet = t&3) (a row's 128 B are
  // read by 4 neighbouring lanes); MN-contiguous B -> (column = t % BN, octet = t / BN)
  const int ar = tid >> 2, aoct = tid & 3;
  const int am = tm * BM + ar;
  const int bc = BT ? (tid >> 2) : (tid % BN);
  const int boct = BT ? (tid & 3) : (tid / BN);
  const int bn_ = tn * BN + bc;
  // fragment-image slot of this thread's octets (tile, ksub, lane)
  const int a_slot = ((ar >> 5) * 2 + (aoct >> 1)) * 2048 + ((ar & 31) + 32 * (aoct & 1)) * 16;
  const int b_slot = ((bc >> 5) * 2 + (boct >> 1)) * 2048 + ((bc & 31) + 32 * (boct & 1)) * 16;

  float va[8], vb[8];
  // range guard (forward products, see guard_init_kernel): exactly 1 unless max |x| >= 2^15
  const float sa = split_scale_of(d.amax_a), sb = split_scale_of(d.amax_b);
#define AVC16_LOAD(KT)                                                                           \
  {                                                                                              \
    const int tau = (KT) / kt_per_tap;                                                           \
    const int k0 = ((KT) - tau * kt_per_tap) * BK;                                               \
    {                                                                                            \
      const int k = k0 + 8 * aoct;                                                               \
      const long srow = (long)am + a_shift0 + (long)tau * a_tapshift;                            \
      const bool rok = am < M && srow >= 0 && srow < a_rows;                                     \
      const bool ok0 = rok && k < Kc, ok1 = rok && k + 4 < Kc;                                   \
      const float4 x0 = sel4(ok0, *reinterpret_cast<const float4*>(Ab + (ok0 ? srow * lda + k : 0)));     \
      const float4 x1 = sel4(ok1, *reinterpret_cast<const float4*>(Ab + (ok1 ? srow * lda + k + 4 : 0))); \
      va[0] = x0.x; va[1] = x0.y; va[2] = x0.z; va[3] = x0.w;                                    \
      va[4] = x1.x; va[5] = x1.y; va[6] = x1.z; va[7] = x1.w;                                    \
    }                                                                                            \
    if (BT) {                                                                                    \
      const int k = k0 + 8 * boct;                                                               \
      const bool ok0 = bn_ < N && k < Kc, ok1 = bn_ < N && k + 4 < Kc;                           \
      const float* bp = Bb + (long)tau * b_tapoff + (long)bn_ * ldb + k;                         \
      const float4 x0 = sel4(ok0, *reinterpret_cast<const float4*>(ok0 ? bp : Bb));              \
      const float4 x1 = sel4(ok1, *reinterpret_cast<const float4*>(ok1 ? bp + 4 : Bb));          \
      vb[0] = x0.x; vb[1] = x0.y; vb[2] = x0.z; vb[3] = x0.w;                                    \
      vb[4] = x1.x; vb[5] = x1.y; vb[6] = x1.z; vb[7] = x1.w;                                    \
    } else {                                                                                     \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                            \
        const int k = k0 + 8 * boct + j;                                                         \
        const long srow = (long)k + bshift;                                                      \
        const bool ok = bn_ < N && k < Kc && srow >= 0 && srow < b_rows;                         \
        const float x = Bb[ok ? (long)tau * b_tapoff + srow * ldb + bn_ : 0];                    \
        vb[j] = ok ? x : 0.f;                                                                    \
      }                                                                                          \
    }                                                                                            \
  }
#define AVC16_STORE(BUF)                                                                         \
  {                                                                                              \
    unsigned char* Ai = lds + (BUF) * (AIMG + BIMG);                                             \
    unsigned char* Bi = Ai + AIMG;                                                               \
    f16x8 hi, lo;                                                                                \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) { va[j] *= sa; vb[j] *= sb; }                  \
    split8(va, hi, lo);                                                                          \
    *reinterpret_cast<f16x8*>(Ai + a_slot) = hi;                                                 \
    *reinterpret_cast<f16x8*>(Ai + a_slot + 1024) = lo;                                          \
    split8(vb, hi, lo);                                                                          \
    *reinterpret_cast<f16x8*>(Bi + b_slot) = hi;                                                 \
    *reinterpret_cast<f16x8*>(Bi + b_slot + 1024) = lo;                                          \
  }

  f32x16 zero16;
#pragma unroll
  for (int e = 0; e < 16; ++e) zero16[e] = 0.f;
  f32x16 acc[TM][TN], cmp[TM][TN], part[TM][TN], crs[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = cmp[i][j] = part[i][j] = crs[i][j] = zero16;

  constexpr int KB = 4;  // K-tiles (128 k) per compensated partial
  if (kt0 < kt1) AVC16_LOAD(kt0);
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    AVC16_STORE(buf);
    __syncthreads();
    if (kt + 1 < kt1) AVC16_LOAD(kt + 1);
    const unsigned char* Ai = lds + buf * (AIMG + BIMG);
    const unsigned char* Bi = Ai + AIMG;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      f16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const unsigned char* p = Ai + ((wm * TM + i) * 2 + s) * 2048 + lane * 16;
        ah[i] = *reinterpret_cast<const f16x8*>(p);
        al[i] = *reinterpret_cast<const f16x8*>(p + 1024);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const unsigned char* p = Bi + ((wn * TN + j) * 2 + s) * 2048 + lane * 16;
        bh[j] = *reinterpret_cast<const f16x8*>(p);
        bl[j] = *reinterpret_cast<const f16x8*>(p + 1024);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], part[i][j], 0, 0, 0);
          crs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], crs[i][j], 0, 0, 0);
          crs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], crs[i][j], 0, 0, 0);
        }
    }
    if ((kt - kt0) % KB == KB - 1 || kt + 1 == kt1) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float y = part[i][j][e] - cmp[i][j][e];
            const float t = acc[i][j][e] + y;
            cmp[i][j][e] = (t - acc[i][j][e]) - y;
            acc[i][j][e] = t;
          }
          part[i][j] = zero16;
        }
    }
  }
#undef AVC16_LOAD
#undef AVC16_STORE
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = (acc[i][j][e] - cmp[i][j][e]) + crs[i][j][e] * (1.0f / 2048.0f);
  if (d.split_scale && nsplit == 1) {  // split-K partials stay scaled; splitk_reduce_kernel unscales
    const float us = split_unscale(d.amax_a, d.amax_b);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] *= us;
  }

  // ---- epilogue (32x32 C layout: col = lane&31, row = (e&3) + 8(e>>2) + 4(lane>>5)) --------
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
  float biasv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + 32 * j;
    float bias = 0.f;
    if (col < d.N) {
      if (d.bias0) bias += d.bias0[col];
      if (d.bias1) bias += d.bias1[col];
    }
    biasv[j] = bias;
  }
  {  // (the fallback kernels keep the per-element stores)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + 32 * j;
    const bool colok = col < d.N;
    const float bias = biasv[j];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
        if (!colok || row >= d.M) continue;
        const float v = act_apply(acc[i][j][e] + bias, d.act);
        float* p = C + (long)row * d.ldc + (long)col * d.ldc_col;
        if (d.accumulate) *p += v; else *p = v;
      }
  }
  }
  if (d.stats)
    bn_tile_stats<BM, BN, WM, WTN, TM, TN, 1, false, false>(d, acc, biasv, reinterpret_cast<float*>(lds), tm, tn, wm,
                                                            wn, lane, tid, NT, row_base, col_base);
}

// ---- output tile through LDS (round 6) ------------------------------------------------------
// The per-element epilogue (one 4-B store per accumulator element, the activation picked by a
// runtime switch per element, 64-bit address arithmetic per element) took about as long as the K
// loop itself: the C2 forward's GEMM class measured 66 -> 36 us per launch with every epilogue
// skipped.  Here the tile's values -- act(acc + bias), the same expression -- go to
// LDS once (the operand ring is dead by then), and the tile leaves as whole rows of 16-B pieces
// (one wave instruction writes 1 KiB: two 128-column rows); an accumulating product reads the old
// row pieces and adds in the same order.  Same values, same bits.  Requires a row-major C
// (ldc_col = 1) with 16-B aligned rows; other layouts keep the per-element form.
template <int ACT>
__device__ __forceinline__ float act_k(float v) { return act_apply(v, ACT); }

template <int BM, int BN, int TM, int TN, int NT, int ACT>
__device__ __forceinline__ void tile_to_lds(float* tile, const f32x16 (&acc)[TM][TN], const float (&bias)[TN], int rl0,
                                            int cl0) {
  constexpr int TP = BN + 4;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        tile[(rl0 + 32 * i + (e & 3) + 8 * (e >> 2)) * TP + cl0 + 32 * j] = act_k<ACT>(acc[i][j][e] + bias[j]);
}

template <int BM, int BN, int TM, int TN, int NT>
__device__ __forceinline__ void store_tile_rows(float* __restrict__ C, long ldc, int M, int N, int row0, int col0,
                                                const f32x16 (&acc)[TM][TN], const float (&bias)[TN], int act,
                                                bool accumulate, unsigned char* lds, int rl0, int cl0, int tid) {
  constexpr int TP = BN + 4, C4 = BN / 4;
  float* tile = reinterpret_cast<float*>(lds);
  __syncthreads();  // (every wave is done with the LDS operand ring)
  switch (act) {  // once, not per element
    case AVC_ACT_RELU: tile_to_lds<BM, BN, TM, TN, NT, AVC_ACT_RELU>(tile, acc, bias, rl0, cl0); break;
    case AVC_ACT_TANH: tile_to_lds<BM, BN, TM, TN, NT, AVC_ACT_TANH>(tile, acc, bias, rl0, cl0); break;
    case AVC_ACT_DBNORM: tile_to_lds<BM, BN, TM, TN, NT, AVC_ACT_DBNORM>(tile, acc, bias, rl0, cl0); break;
    default: tile_to_lds<BM, BN, TM, TN, NT, AVC_ACT_NONE>(tile, acc, bias, rl0, cl0); break;
  }
  __syncthreads();
  for (int it = tid; it < BM * C4; it += NT) {
    const int rl = it / C4, c4 = it - rl * C4;
    const int row = row0 + rl, col = col0 + 4 * c4;
    if (row >= M || col >= N) continue;
    const float4 v = *reinterpret_cast<const float4*>(tile + rl * TP + 4 * c4);
    float* p = C + (long)row * ldc + col;
    if (col + 4 <= N) {
      float4 o = v;
      if (accumulate) {
        const float4 q = *reinterpret_cast<const float4*>(p);
        o = make_float4(q.x + v.x, q.y + v.y, q.z + v.z, q.w + v.w);
      }
      *reinterpret_cast<float4*>(p) = o;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
      for (int e = 0; e < N - col; ++e) p[e] = accumulate ? p[e] + vv[e] : vv[e];
    }
  }
}

// ---- split-f16 GEMM on pre-split fragment-major operands ("gemm16f") ---------------------
//
// Both operands are first split once into the fragment-major layout of v_mfma_f32_32x32x16_f16
// (split_frag32_kernel): for every 32-row tile t and 16-deep chunk c, two 1 KiB blocks (hi,
// lo) hold exactly what the 64 lanes of one operand load: lane l = r + 32q gets row 32t + r,
// k = 16c + 8q .. +7.  Block (t, c, hl) sits at ((t*nkc + c)*2 + hl) KiB; rows are padded to a
// multiple of 32 and K to a multiple of 32 with zeros.  The GEMM then streams whole 1 KiB blocks
// global -> LDS with LDS-DMA (buffer_load ... lds: no VGPRs, no conversion ALU, no bank
// conflicts), three stages deep with counted vmcnt and raw barriers, and reads every fragment
// with one conflict-free ds_read_b128 at lane*16.  Row tiles outside the operand (Conv1d zero
// padding; tap shifts must be multiples of 32 rows) fall outside the buffer descriptor and
// land as zeros.
__global__ __launch_bounds__(256) void split_frag32_kernel(const float* __restrict__ src, long rs,
                                                           long ks, int R, int K, int ntile, int nkc,
                                                           _Float16* __restrict__ dst,
                                                           const unsigned* __restrict__ amax = nullptr,
                                                           long src_tap = 0, long dst_tap = 0) {
  // grid y enumerates the taps of a multi-tap operand (one launch for all of them)
  src += blockIdx.y * src_tap;
  dst += blockIdx.y * dst_tap;
  const int G8 = nkc * 2;  // 8-element groups per row (a multiple of 4)
  const float sc = split_scale_of(amax);
  const long total = (long)ntile * 32 * G8;
  const bool vec = ks == 1 && (rs & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    long r;
    int g8;
    if (ks == 1) {
      // row-major source: thread -> (tile, 32-k group quad, row, group) with the group fastest, so
      // a wave reads 16 rows x 128 B and each of its stores writes two 256-B runs (whole lines)
      const int gq = (int)(idx & 3);
      const long rest = idx >> 2;
      const int rr = (int)(rest & 31);
      const long tq = rest >> 5;  // tile * (G8/4) + quad
      // 32-bit divisions whenever the indices fit (a 64-bit division is a long software sequence)
      const unsigned q4 = (unsigned)(G8 >> 2);
      const long t = tq < 0xffffffffL ? (long)((unsigned)tq / q4) : tq / (long)q4;
      const int quad = (int)(tq - t * (long)q4);
      r = t * 32 + rr;
      g8 = quad * 4 + gq;
    } else {        // transposed source (column stride 1): consecutive threads take consecutive rows
      const long rows = (long)ntile * 32;
      g8 = idx < 0xffffffffL && rows < 0xffffffffL ? (int)((unsigned)idx / (unsigned)rows) : (int)(idx / rows);
      r = idx - (long)g8 * rows;
    }
    float v[8];
    const int k0 = 8 * g8;
    if (vec && r < R && k0 + 8 <= K) {
      const float4* q = reinterpret_cast<const float4*>(src + r * rs + k0);
      const float4 a = q[0], b = q[1];
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + e;
        v[e] = (r < R && k < K) ? src[r * rs + (long)k * ks] : 0.f;
      }
    }
    if (amax) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= sc;
    }
    f16x8 hi, lo;
    split8(v, hi, lo);
    const long blk = ((r >> 5) * nkc + (g8 >> 1)) * 2;
    const int lane = (int)(r & 31) + 32 * (g8 & 1);
    *reinterpret_cast<f16x8*>(dst + blk * 512 + lane * 8) = hi;
    *reinterpret_cast<f16x8*>(dst + (blk + 1) * 512 + lane * 8) = lo;
  }
}

// A Conv1d weight's five tap images in one pass (GemmDesc::b_conv; split_frag32_kernel's layout,
// scale and split8, so the same bits): one wave per 1 KiB block pair (32 rows x 16 k), lane
// l -> row 32t + (l & 31), k = 16c + 8(l >> 5) .. +7, every tap of those 8 k read at once and each
// tap's hi / lo written as whole 1 KiB blocks.  MODE 1 (forward, N = cout, K = cin): element
// (n, k, tau) = W[n][k][tau], a lane's 40 floats contiguous; MODE 2 (dgrad, N = cin, K = cout):
// W[k][n][4 - tau], 32 lanes reading 640 contiguous bytes per k.  (split_frag32_kernel walked
// the weight with the row as the fast index: each lane strided 10 KB from its neighbour, 8 us per
// 512 x 512 weight.)
template <int MODE>
__global__ __launch_bounds__(64) void split_convw_kernel(const float* __restrict__ W, int N, int K, int ntile, int nkc,
                                                         _Float16* __restrict__ dst, long tapstride,
                                                         const unsigned* __restrict__ amax) {
  const int l = threadIdx.x;
  const int t = blockIdx.x / nkc, c = blockIdx.x - (blockIdx.x / nkc) * nkc;
  const int n = 32 * t + (l & 31), k0 = 16 * c + 8 * (l >> 5);
  const float sc = split_scale_of(amax);
  float f[8][5];
  if (MODE == 1 && n < N && k0 + 8 <= K && (K & 3) == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0) {
    const float4* q = reinterpret_cast<const float4*>(W + ((long)n * K + k0) * 5);
    float4 r[10];
#pragma unroll
    for (int u = 0; u < 10; ++u) r[u] = q[u];
    const float* rf = reinterpret_cast<const float*>(r);
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int tau = 0; tau < 5; ++tau) f[e][tau] = rf[e * 5 + tau];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + e;
      const bool ok = n < N && k < K;
#pragma unroll
      for (int tau = 0; tau < 5; ++tau)
        f[e][tau] = !ok ? 0.f : (MODE == 1 ? W[((long)n * K + k) * 5 + tau] : W[((long)k * N + n) * 5 + 4 - tau]);
    }
  }
  const long blk = ((long)t * nkc + c) * 2;
#pragma unroll
  for (int tau = 0; tau < 5; ++tau) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = f[e][tau];
    if (amax) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= sc;
    }
    f16x8 hi, lo;
    split8(v, hi, lo);
    _Float16* o = dst + tau * tapstride + blk * 512 + l * 8;
    *reinterpret_cast<f16x8*>(o) = hi;
    *reinterpret_cast<f16x8*>(o + 512) = lo;
  }
}

// max |x| over a rows x cols region (row stride ld) into *out (float bits; out pre-zeroed).
// Contiguous regions stream as float4; strided ones walk rows per block (no 64-bit division).
__global__ __launch_bounds__(256) void absmax_vec_kernel(const float4* __restrict__ src, long n4,
                                                         const float* __restrict__ tail, int ntail,
                                                         unsigned* __restrict__ out) {
  __shared__ float red[4];
  float m = 0.f;
  // eight independent loads in flight per thread per iteration
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + 7 * stride < n4; i += 8 * stride) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
  }
  for (; i < n4; i += stride) {
    const float4 v = src[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
  }
  if (blockIdx.x == 0 && (int)threadIdx.x < ntail) m = fmaxf(m, fabsf(tail[threadIdx.x]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) amax_update(out, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

__global__ __launch_bounds__(256) void absmax_rows_kernel(const float* __restrict__ src, long rows, int cols,
                                                          long ld, unsigned* __restrict__ out) {
  __shared__ float red[4];
  float m = 0.f;
  if ((cols & 3) == 0 && (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    // flattened (row, float4 column) index: narrow regions (cols = 32 of a 64-wide row) still
    // keep every lane busy
    const int c4n = cols >> 2;
    const long n = rows * c4n;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L) {
      const long r = i / c4n;
      const int c = (int)(i - r * c4n);
      const float4 v = *reinterpret_cast<const float4*>(src + r * ld + 4 * c);
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  } else {
    for (long r = blockIdx.x; r < rows; r += gridDim.x)
      for (int c = threadIdx.x; c < cols; c += 256) m = fmaxf(m, fabsf(src[r * ld + c]));
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) amax_update(out, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// Every workgroup of a max scan ends in one atomic max on the same word, and workgroups that finish
// together all take it (the running max has not risen yet): the grid is capped at kMaxScanBlocks
// (2048 workgroups made a 64 MB scan take ~37 us, mostly serialised atomics); the loop keeps four
// loads in flight per thread instead.
constexpr long kMaxScanBlocks = 256;
// ... and a small scan takes at least 4096 float4 per workgroup (16 per thread, two batches of
// eight loads): each workgroup's atomic costs ~35 ns serialised on the one word, so a 5 MB weight
// spread over 256 workgroups spent most of its 9-13 us in atomics (round 6)
inline long scan_blocks(long n4) { return std::max<long>(1, std::min<long>((n4 + 4095) / 4096, kMaxScanBlocks)); }
inline void absmax2d(const float* src, long rows, long cols, long ld, unsigned* out, hipStream_t s) {
  if (ld == cols && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
    const long n = rows * cols, n4 = n / 4;
    absmax_vec_kernel<<<(int)scan_blocks(n4), 256, 0, s>>>(
        reinterpret_cast<const float4*>(src), n4, src + 4 * n4, (int)(n - 4 * n4), out);
  } else {
    const long blocks = (cols % 4 == 0 && ld % 4 == 0) ? (rows * (cols / 4) + 1023) / 1024 : rows;
    absmax_rows_kernel<<<(int)std::max<long>(1, std::min<long>(blocks, kMaxScanBlocks)), 256, 0, s>>>(src, rows, (int)cols,
                                                                                            ld, out);
  }
}

// gemm16f's per-column epilogue operands, loaded at kernel start so their latency hides behind
// the main loop: this lane's bias per column block (biasv, summed as every epilogue sums it) and,
// with the fused BatchNorm (bn), for threads tid < BN column tid's gamma, beta, running mean and
// running var (par).
template <int BN, int TN>
__device__ __forceinline__ void bnf_prefetch(const GemmDesc& d, int tn, int tid, int col_base, float (&biasv)[TN],
                                             float (&par)[4], bool bn) {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + 32 * j;
    float bias = 0.f;
    if (col < d.N) {
      if (d.bias0) bias += d.bias0[col];
      if (d.bias1) bias += d.bias1[col];
    }
    biasv[j] = bias;
  }
  const BnFuse& bf = d.bnf;
  const int col = tn * BN + tid;
  par[0] = par[1] = par[2] = par[3] = 0.f;
  if (bn && tid < BN && col < d.N) {
    par[0] = bf.gamma[col];
    par[1] = bf.beta[col];
    if (bf.rmean) par[2] = bf.rmean[col];
    if (bf.rvar) par[3] = bf.rvar[col];
  }
}

// Fused BatchNorm epilogue of gemm16f (GemmDesc::bnf, see gemm.h).  Every expression that forms a
// value is the one the unfused chain uses (this kernel's epilogue for y and the column partials,
// bn_finalize_kernel for mean / invstd and the running statistics, bn_apply(_frag) for the
// output and its split), in the same order, so both chains give the same bits.
// LDS (bytes): [0, 8K) column partials [2 WM][BN] f32; [8K, 20K) fp64 sums [3][4][BN];
// [20K, 21K) scale / shift [2][BN]; 21K flag; [22K, ..) the tile [BM][BN + 4] f32.
template <int BM, int BN, int WM, int WTN, int TM, int TN, int NT>
__device__ __forceinline__ void bnf_epilogue(const GemmDesc& d, f32x16 (&acc)[TM][TN], unsigned char* lds, int tm,
                                             int tn, int tilesM, int wm, int lane, int tid, int row_base,
                                             int col_base, unsigned long long ticket, const float (&biasv)[TN],
                                             const float (&par)[4]) {
  static_assert(NT == 4 * BN, "the finalize step takes 4 threads per column (bn_finalize_kernel)");
  const BnFuse& bf = d.bnf;
  float* red = reinterpret_cast<float*>(lds);
  double* dred = reinterpret_cast<double*>(lds + 8192);
  float* s_sc = reinterpret_cast<float*>(lds + 20480);
  float* s_sh = s_sc + BN;
  int* flag = reinterpret_cast<int*>(lds + 21504);
  float* tile = reinterpret_cast<float*>(lds + 22528);
  constexpr int TP = BN + 4;
  const int wn = (col_base - tn * BN - (lane & 31)) / WTN;
  AVC_EPI_STAMP(1);
  // (1) y = A.B + bias (biasv: bnf_prefetch; d.act is none, gemm_bnf_ok), kept in registers
  // (stored only where the caller keeps y_pre)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + 32 * j;
    const bool colok = col < d.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
        if (!colok || row >= d.M) continue;
        const float v = acc[i][j][e] + biasv[j];
        acc[i][j][e] = v;
        if (d.C) d.C[(long)row * d.ldc + col] = v;
      }
  }
  bool ok = true;
  if (bf.training) {
    // (2) this tile's column partials exactly as the unfused epilogue forms them (bn_tile_stats),
    // stored write-through, drained, then this workgroup counts itself in on its column tile
    const float nob[TN] = {};
    const int wm_ = wm, wn_ = wn;
    AVC_EPI_STAMP(2);
    bn_tile_stats<BM, BN, WM, WTN, TM, TN, 1, true, true>(d, acc, nob, red, tm, tn, wm_, wn_, lane, tid, NT, row_base,
                                                          col_base);
    AVC_EPI_STAMP(3);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    AVC_EPI_STAMP(4);
    if (tid == 0) {
      const unsigned E = (unsigned)(ticket / (unsigned long long)bf.nwg) + 1u;
      __hip_atomic_fetch_add((bnf_gu32*)(bf.cnt + tn * 32), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = (AVC_GEMM_DIAG_EPI & 1) ? 1 : (bnf_wait(bf.cnt + tn * 32, E * (unsigned)tilesM, bf, E) ? 1 : 0);
    }
    __syncthreads();
    AVC_EPI_STAMP(5);
    ok = flag[0] != 0;
    // (3) this workgroup's columns' partials over every tile, combined in bn_finalize_kernel's
    // order (4 thread groups over the partial rows p = grp, grp + 4, ..., then the 4 group sums
    // left to right) and form (bn_combine)
    const auto srs = __builtin_amdgcn_make_buffer_rsrc(d.stats, 0, tilesM * 2 * d.N * 4, 0x00020000);
    const int grp = tid / BN, cl = tid - grp * BN, col = tn * BN + cl;
    // (4 rows of loads in flight per thread: a variant that requested all 16 rows of a thread
    // before its first add measured 0.08 ms slower per C2 forward)
    double s = 0.0, a1 = 0.0, a2 = 0.0;
    if (col < d.N && !(AVC_GEMM_DIAG_EPI & 2)) {
      // (bn_finalize_kernel's order and loads: K with the first batch, the next batch's loads issued
      // before the current one is combined)
      const double inv_pr = 1.0 / (double)BM;
      const double inv_last = 1.0 / (double)(d.M - (tilesM - 1) * BM);  // the short last partial
      // (partials past tilesM lie past the descriptor's range and load as zeros: no branch, whose
      // wait would serialise the batch's loads)
      auto ld = [&](int p, int h) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(srs, ((p * 2 + h) * d.N + col) * 4, 0, 16));
      };
      const float S0 = ld(0, 0);
      float Sv[4], Qv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        Sv[u] = ld(grp + 4 * u, 0);
        Qv[u] = ld(grp + 4 * u, 1);
      }
      const double K = (double)S0 * (tilesM == 1 ? inv_last : inv_pr);
      for (int p0 = grp; p0 < tilesM; p0 += 16) {
        float Sn[4], Qn[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          Sn[u] = ld(p0 + 16 + 4 * u, 0);
          Qn[u] = ld(p0 + 16 + 4 * u, 1);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int p = p0 + 4 * u;
          if (p < tilesM) {
            const long n = min(BM, d.M - p * BM);
            bn_combine(Sv[u], Qv[u], n, p == tilesM - 1 ? inv_last : inv_pr, K, s, a1, a2);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          Sv[u] = Sn[u];
          Qv[u] = Qn[u];
        }
      }
    }
    dred[(0 * 4 + grp) * BN + cl] = s;
    dred[(1 * 4 + grp) * BN + cl] = a1;
    dred[(2 * 4 + grp) * BN + cl] = a2;
    __syncthreads();
    AVC_EPI_STAMP(6);
  }
  // (4) per-column scale and shift (bn_finalize_kernel, then bn_apply's sc / sh); par = gamma,
  // beta, running mean, running var of column tid (bnf_prefetch)
  if (tid < BN) {
    const int col = tn * BN + tid;
    if (col < d.N) {
      float mf, isf;
      if (bf.training) {
        const double s = dred[0 * BN + tid] + dred[1 * BN + tid] + dred[2 * BN + tid] + dred[3 * BN + tid];
        const double a1 = dred[4 * BN + tid] + dred[5 * BN + tid] + dred[6 * BN + tid] + dred[7 * BN + tid];
        const double a2 = dred[8 * BN + tid] + dred[9 * BN + tid] + dred[10 * BN + tid] + dred[11 * BN + tid];
        const double mean = s / bf.count;
        const double e1 = a1 / bf.count;
        double var = a2 / bf.count - e1 * e1;
        if (var < 0.0) var = 0.0;
        mf = (float)mean;
        isf = (float)(1.0 / sqrt(var + (double)bf.eps));
        if (!ok) mf = __builtin_nanf("");  // gave up: this launch's outputs are NaN, never plausible
        if (tm == 0 && ok) {
          if (bf.mean) bf.mean[col] = mf;
          if (bf.invstd) bf.invstd[col] = isf;
          if (bf.rmean) bf.rmean[col] = (float)((1.0 - bf.momentum) * par[2] + bf.momentum * mean);
          if (bf.rvar) {
            const double unb = bf.count > 1.0 ? var * bf.count / (bf.count - 1.0) : var;
            bf.rvar[col] = (float)((1.0 - bf.momentum) * par[3] + bf.momentum * unb);
          }
        }
      } else {
        mf = par[2];
        isf = (float)(1.0 / sqrt((double)par[3] + (double)bf.eps));
        if (tm == 0) {
          if (bf.mean) bf.mean[col] = mf;
          if (bf.invstd) bf.invstd[col] = isf;
        }
      }
      const float sc = isf * par[0];
      s_sc[tid] = sc;
      s_sh[tid] = par[1] - mf * sc;
    }
  }
  // (5) the pre-BN tile into LDS, so each output item is one row's 8 consecutive columns
  AVC_EPI_STAMP(7);
  const int rl0 = row_base - tm * BM, cl0 = col_base - tn * BN;
  if (!(AVC_GEMM_DIAG_EPI & 4)) {
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) tile[(rl0 + 32 * i + (e & 3) + 8 * (e >> 2)) * TP + cl0 + 32 * j] = acc[i][j][e];
  }
  __syncthreads();
  AVC_EPI_STAMP(8);
  if (AVC_GEMM_DIAG_EPI & 8) return;
  // (6) BN + act (+ residual) per item (32-row block, 16-deep chunk, lane): a wave's fragment
  // stores cover whole 1 KiB blocks.  Items past N inside the image's K padding are zeros, as
  // bn_apply_frag writes them.
  constexpr int NCH16 = BN / 16, ITEMS = (BM / 32) * NCH16 * 64;
  const long fr_rows = ((long)d.M + 31) / 32 * 32;
  const int kpad = bf.nkc_out * 16;
  // (the act switch taken once, outside the item loop)
  auto items = [&](auto actc) {
    constexpr int ACT = decltype(actc)::value;
    bool over = false;
    for (int it = tid; it < ITEMS; it += NT) {
      const int l = it & 63, blk = it >> 6;
      const int c16 = blk % NCH16, rb = blk / NCH16;
      const int rl = rb * 32 + (l & 31), cl8 = c16 * 16 + 8 * (l >> 5);
      const long row = (long)tm * BM + rl;
      const int col = tn * BN + cl8;
      float o[8];
      if (row < d.M && col < d.N) {
        const float4 a = *reinterpret_cast<const float4*>(tile + rl * TP + cl8);
        const float4 b = *reinterpret_cast<const float4*>(tile + rl * TP + cl8 + 4);
        o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
        o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  #pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = act_k<ACT>(o[e] * s_sc[cl8 + e] + s_sh[cl8 + e]);
        if (bf.residual) {
          const float4* rq = reinterpret_cast<const float4*>(bf.residual + row * d.N + col);
          const float4 ra = rq[0], rb4 = rq[1];
          o[0] += ra.x; o[1] += ra.y; o[2] += ra.z; o[3] += ra.w;
          o[4] += rb4.x; o[5] += rb4.y; o[6] += rb4.z; o[7] += rb4.w;
        }
        if (bf.out) {
          float4* oq = reinterpret_cast<float4*>(bf.out + row * d.N + col);
          oq[0] = make_float4(o[0], o[1], o[2], o[3]);
          oq[1] = make_float4(o[4], o[5], o[6], o[7]);
        }
      } else {
  #pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = 0.f;
      }
  #pragma unroll
      for (int e = 0; e < 8; ++e) over |= fabsf(o[e]) >= 65504.f && fabsf(o[e]) < __builtin_inff();
      if (bf.frag && row < fr_rows && col < kpad) {
        f16x8 hi, lo;
  #pragma unroll
        for (int e = 0; e < 8; ++e) {
          const _Float16 h = (_Float16)o[e];
          hi[e] = h;
          lo[e] = (_Float16)((o[e] - (float)h) * 2048.0f);
        }
        const long fb = ((row >> 5) * bf.nkc_out + (col >> 4)) * 2;
        const int fl = (int)(row & 31) + 32 * ((col >> 3) & 1);
        *reinterpret_cast<f16x8*>(bf.frag + fb * 512 + fl * 8) = hi;
        *reinterpret_cast<f16x8*>(bf.frag + (fb + 1) * 512 + fl * 8) = lo;
      }
    }
    return over;
  };
  bool over;
  switch (bf.act) {
    case AVC_ACT_RELU: over = items(std::integral_constant<int, AVC_ACT_RELU>{}); break;
    case AVC_ACT_TANH: over = items(std::integral_constant<int, AVC_ACT_TANH>{}); break;
    case AVC_ACT_DBNORM: over = items(std::integral_constant<int, AVC_ACT_DBNORM>{}); break;
    default: over = items(std::integral_constant<int, AVC_ACT_NONE>{}); break;
  }
  if (over && bf.range_flag) __hip_atomic_store(bf.range_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#ifdef AVC_GEMM_EPI_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  AVC_EPI_STAMP(9);
}

struct Frag16Args {
  const _Float16* As; int a_ntile, a_nkc; long a_shift0, a_tapshift;  // shifts in rows (x32)
  const _Float16* Bs; int b_ntile, b_nkc; long b_tapstride;            // halves per tap
  int b_shift0_c, b_zshift_c;  // B K-shift of product z in 16-deep chunks (weight gradients)
};

// OCC = 2: two workgroups per CU (waves capped at 128 VGPRs): the 128-k partials are folded
// into the accumulator with a plain add instead of Kahan-compensated ones (no cmp registers).
// KH = 0 (round 3, the default configuration): the same plain fold at one workgroup per CU.  Each
// 128-k partial is already a fresh MFMA chain, so the fold adds 20 roundings to a K = 2560 sum;
// measured: the C2 conv 92 -> 84 us, and every forward / gradient / loss-curve parity test keeps
// its margin.
// BNF = 1: the fused BatchNorm epilogue (GemmDesc::bnf; one K split, co-resident grid).
template <int BM, int BN, int WM, int WN, int NS, int KC, int OCC = 1, int KH = 1, int BNF = 0>
__global__ __launch_bounds__(64 * WM * WN, OCC * WM * WN / 4) void gemm16f_kernel(GemmDesc d, Frag16Args f, int tilesM,
                                                               int tilesN, int kt_per_tap, int kps,
                                                               int nsplit, float* __restrict__ slab) {
  constexpr int NT = 64 * WM * WN, NWAVE = WM * WN;
  // fused BN, train mode: this launch's ticket (its epoch), taken now so its latency hides
  // behind the main loop
  unsigned long long bnf_ticket = 0;
  if constexpr (BNF) {
    if (d.bnf.training && threadIdx.x == 0)
      bnf_ticket = __hip_atomic_fetch_add(d.bnf.tickets, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int ABLK = (BM / 32) * KC * 2, BBLK = (BN / 32) * KC * 2;  // 1 KiB blocks per K-tile (KC kc x hi/lo)
  constexpr int NBLK = ABLK + BBLK;
  static_assert(NBLK % NWAVE == 0, "blocks per K-tile must split evenly over the waves");
  constexpr int DPW = NBLK / NWAVE;  // LDS-DMA instructions per wave per K-tile
  constexpr int STAGE = NBLK * 1024;
  static_assert(!BNF || 18432 + BM * (BN + 4) * 4 <= NS * STAGE, "fused BN: the tile does not fit the ring's LDS");
  constexpr bool kTileFits = BM * (BN + 4) * 4 <= NS * STAGE;  // (store_tile_rows stages the tile in the ring)
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // NS stages

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w % WN;
  const int nwg = tilesM * tilesN;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (bid >> 3);
  int tm, tn;
  if constexpr (BNF) {
    // fused BN: the barrier group of column tile tn (its tilesM row tiles) is the contiguous
    // dispatch range [tn * tilesM, (tn + 1) * tilesM), dealt evenly over the XCDs, so a group needs
    // only its own tilesM workgroups resident, never the whole grid (bnf_epilogue).
    // Inside the group, dispatch index l = bid - tn * tilesM lands on XCD l % 8 (round-robin), and
    // that XCD takes the contiguous band of tilesM / 8 row tiles starting at (l % 8) * tilesM / 8,
    // the same band under every column tile.  The conv taps shift A by +-1 / +-2 frames (+-B rows),
    // i.e. into the neighbouring row tile, which is then in the same band and the same L2.
    // (Round 4 mapped tm = l, which dealt row tiles x, x + 8, ... to XCD x: every tap's neighbour
    // tile sat in another XCD's L2, +46 % fetched bytes at C2.)  Speed only: any bijection is correct.
    tn = bid / tilesM;
    const int l = bid - tn * tilesM;
    tm = (!d.bnf.band || (tilesM & 7)) ? l : (l & 7) * (tilesM >> 3) + (l >> 3);
    (void)wgid;
  } else {
    tile_of(wgid, tilesM, tilesN, tm, tn);
  }
  const int split = blockIdx.y % nsplit, z = blockIdx.y / nsplit;
  const int ktotal = d.ntaps * kt_per_tap;
  const int kt0 = split * kps;
  const int kt1 = min(ktotal, kt0 + kps);
  if constexpr (BNF) AVC_EPI_STAMP(0);
  // the epilogue's per-column operands, loaded now so their latency hides behind the main loop
  float bnf_bias[TN], bnf_par[4];
  bnf_prefetch<BN, TN>(d, tn, tid, tn * BN + wn * WTN + (lane & 31), bnf_bias, bnf_par, BNF != 0);

  const auto ars = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(f.As), 0,
                                                     f.a_ntile * f.a_nkc * 2048, 0x00020000);
  const auto brs = __builtin_amdgcn_make_buffer_rsrc(const_cast<_Float16*>(f.Bs), 0,
                                                     (int)(d.ntaps * f.b_tapstride * 2), 0x00020000);
  // Out-of-range blocks get an offset past the descriptor's num_records: the bounds check (on
  // the VGPR offset; the SGPR offset is not range-checked) makes the DMA land zeros.
  constexpr unsigned kOut = 0x7FFFFF00u;
  const int a_ntile = f.a_ntile, a_nkc = f.a_nkc, b_ntile = f.b_ntile, b_nkc = f.b_nkc;
  const long a_shift0 = f.a_shift0, a_tapshift = f.a_tapshift, b_tapstride = f.b_tapstride;
  const int bzs = f.b_shift0_c + z * f.b_zshift_c;  // uniform per workgroup

  // issue the LDS-DMA of K-tile kt into stage st: this wave's DPW blocks of the NBLK
#define AVC16F_ISSUE(KT, ST)                                                                      \
  {                                                                                               \
    const int tau = (KT) / kt_per_tap;                                                            \
    const int kc0 = ((KT) - tau * kt_per_tap) * KC;                                               \
    unsigned char* const stage_base = lds + (ST) * STAGE;                                         \
    _Pragma("unroll") for (int i = 0; i < DPW; ++i) {                                             \
      const int b = w * DPW + i;                                                                  \
      unsigned char* dst = stage_base + b * 1024;                                                 \
      if (b < ABLK) {                                                                             \
        const int rt = b / (2 * KC), kc = (b >> 1) % KC, hl = b & 1;                              \
        const long src_tile = (long)tm * (BM / 32) + rt + (a_shift0 + (long)tau * a_tapshift) / 32; \
        const bool ok = src_tile >= 0 && src_tile < a_ntile && kc0 + kc < a_nkc;                 \
        const unsigned off = ok ? (unsigned)(((src_tile * a_nkc + kc0 + kc) * 2 + hl) * 1024) : kOut; \
        if (!AVC_GEMM_NOLOAD)                                                                     \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (__attribute__((address_space(3))) void*)dst, 16, \
                                                 off + lane * 16, 0, 0, 0);                       \
      } else {                                                                                    \
        const int bb = b - ABLK;                                                                  \
        const int ct = bb / (2 * KC), kc = (bb >> 1) % KC, hl = bb & 1;                           \
        const int src_tile = tn * (BN / 32) + ct;                                                 \
        const int bkc = kc0 + kc + bzs;                                                           \
        const bool ok = src_tile < b_ntile && bkc >= 0 && bkc < b_nkc;                            \
        const unsigned off = ok ? (unsigned)(tau * b_tapstride * 2 +                              \
                                             ((long)(src_tile * b_nkc + bkc) * 2 + hl) * 1024) : kOut; \
        if (!AVC_GEMM_NOLOAD)                                                                     \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (__attribute__((address_space(3))) void*)dst, 16, \
                                                 off + lane * 16, 0, 0, 0);                       \
      }                                                                                           \
    }                                                                                             \
  }

  f32x16 zero16;
#pragma unroll
  for (int e = 0; e < 16; ++e) zero16[e] = 0.f;
  f32x16 acc[TM][TN], cmp[TM][TN], part[TM][TN], crs[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = cmp[i][j] = part[i][j] = crs[i][j] = zero16;

  // Fast issue (round 3).  The macro above spends ~300 scalar instructions of index math per
  // K-tile per wave, and the CU's one scalar unit issues at most one per cycle for all 8 waves:
  // 2 x 348 per SIMD per K-tile against 1536 cycles of MFMA work was the kernel's bound.  Here
  // every piece's VGPR offset (tile row / column, hi / lo, lane, and the conv tap's shift) is
  // formed once per tap, and a K-tile adds one SGPR offset (its 16-deep chunk index; buffer
  // bounds checks see the VGPR part only, so out-of-range pieces stay at kOut).  Same bytes,
  // same LDS image: bit-identical.  Waves whose pieces straddle A and B, and K-tiles that run
  // past K, keep the macro.
  const bool wave_a = (w + 1) * DPW <= ABLK, wave_b = w * DPW >= ABLK;
  unsigned voff[DPW];
  int itau = kt0 / kt_per_tap, ikin = kt0 - itau * kt_per_tap;  // the next K-tile to issue
  int vtau = -1;                                                 // the tap voff was formed for
  // (macros, not lambdas: a lambda here left the kernel's host-side handle undefined)
#define AVC16F_SETTAP(TAU)                                                                        \
  {                                                                                               \
    _Pragma("unroll") for (int i = 0; i < DPW; ++i) {                                             \
      const int b = w * DPW + i;                                                                  \
      if (wave_a) {                                                                               \
        const int rt = b / (2 * KC), kc = (b >> 1) % KC, hl = b & 1;                              \
        const long src_tile = (long)tm * (BM / 32) + rt + (a_shift0 + (long)(TAU) * a_tapshift) / 32; \
        voff[i] = src_tile >= 0 && src_tile < a_ntile                                             \
                      ? (unsigned)(((src_tile * a_nkc + kc) * 2 + hl) * 1024) + lane * 16 : kOut; \
      } else {                                                                                    \
        const int bb = b - ABLK;                                                                  \
        const int ct = bb / (2 * KC), kc = (bb >> 1) % KC, hl = bb & 1;                           \
        const int src_tile = tn * (BN / 32) + ct;                                                 \
        voff[i] = src_tile < b_ntile                                                              \
                      ? (unsigned)((TAU) * b_tapstride * 2 + ((long)(src_tile * b_nkc + kc) * 2 + hl) * 1024) + lane * 16 \
                      : kOut;                                                                     \
      }                                                                                           \
    }                                                                                             \
    vtau = (TAU);                                                                                 \
  }
#define AVC16F_FAST_ISSUE(KT, ST)                                                                 \
  {                                                                                               \
    const int kc0f = ikin * KC;                                                                   \
    const bool inside = wave_a ? kc0f + KC <= a_nkc : (wave_b && kc0f + bzs >= 0 && kc0f + KC + bzs <= b_nkc); \
    if (!inside) {                                                                                \
      AVC16F_ISSUE(KT, ST)                                                                        \
    } else {                                                                                      \
      if (itau != vtau) AVC16F_SETTAP(itau)                                                       \
      unsigned char* const fbase = lds + (ST) * STAGE;                                            \
      const int so = (wave_a ? kc0f : kc0f + bzs) * 2048;                                         \
      _Pragma("unroll") for (int i = 0; i < DPW; ++i) {                                           \
        unsigned char* dst = fbase + (w * DPW + i) * 1024;                                        \
        const unsigned vo = voff[i]; /* (an array element as the builtin's argument drops the  \
                                        kernel's host-side handle: ROCm 7.2 hipcc) */             \
        if (AVC_GEMM_NOLOAD) {                                                                    \
        } else if (wave_a) {                                                                      \
          __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (__attribute__((address_space(3))) void*)dst, 16, vo, so, 0, 0); \
        } else {                                                                                  \
          __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (__attribute__((address_space(3))) void*)dst, 16, vo, so, 0, 0); \
        }                                                                                         \
      }                                                                                           \
    }                                                                                             \
    if (++ikin == kt_per_tap) {                                                                   \
      ikin = 0;                                                                                   \
      ++itau;                                                                                     \
    }                                                                                             \
  }

  // (the spread form: the fast path's pieces [lo, hi) of the K-tile set up by AVC16F_SPREAD_BEGIN)
#define AVC16F_SPREAD_BEGIN(KT, ST)                                                               \
  {                                                                                               \
    const int kc0f = ikin * KC;                                                                   \
    sp_inside = wave_a ? kc0f + KC <= a_nkc : (wave_b && kc0f + bzs >= 0 && kc0f + KC + bzs <= b_nkc); \
    if (!sp_inside) {                                                                             \
      AVC16F_ISSUE(KT, ST)                                                                        \
    } else {                                                                                      \
      if (itau != vtau) AVC16F_SETTAP(itau)                                                       \
      sp_base = lds + (ST) * STAGE;                                                               \
      sp_so = (wave_a ? kc0f : kc0f + bzs) * 2048;                                                \
    }                                                                                             \
    if (++ikin == kt_per_tap) {                                                                   \
      ikin = 0;                                                                                   \
      ++itau;                                                                                     \
    }                                                                                             \
  }
#define AVC16F_SPREAD_PIECES(LO, HI)                                                              \
  _Pragma("unroll") for (int i = (LO); i < (HI); ++i) {                                           \
    unsigned char* dst = sp_base + (w * DPW + i) * 1024;                                          \
    const unsigned vo = voff[i];                                                                  \
    if (wave_a)                                                                                   \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (__attribute__((address_space(3))) void*)dst, 16, vo, sp_so, 0, 0); \
    else                                                                                          \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (__attribute__((address_space(3))) void*)dst, 16, vo, sp_so, 0, 0); \
  }
  // (every piece must be issued inside this K-tile's chunk loop: SPREAD <= KC, or the burst)
  constexpr int SPR = AVC_GEMM_DMA_SPREAD > 0 && AVC_GEMM_DMA_SPREAD <= KC &&
                              DPW % (AVC_GEMM_DMA_SPREAD > 0 ? AVC_GEMM_DMA_SPREAD : 1) == 0
                          ? AVC_GEMM_DMA_SPREAD : 0;
  bool sp_inside = false;
  unsigned char* sp_base = lds;
  int sp_so = 0;
  constexpr int KB = 8 / KC;  // K-tiles (128 k) per compensated partial
  f16x8 fah[2][TM], fal[2][TM], fbh[2][TN], fbl[2][TN];  // fragment double buffer
  // NS-stage ring: NS-1 K-tiles in flight ahead of the one being consumed
#pragma unroll
  for (int pre = 0; pre < NS - 1; ++pre)  // (not `i`: the macro's own loop variable)
    if (kt0 + pre < kt1) AVC16F_FAST_ISSUE(kt0 + pre, pre);
  for (int kt = kt0; kt < kt1; ++kt) {
    const int st = (kt - kt0) % NS;
    // this wave's blocks of tile kt have landed once at most the later tiles' DPW each are pending
    const int ahead = min(NS - 2, kt1 - kt - 1);
    if (ahead >= 3) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * DPW) : "memory");
    } else if (ahead == 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DPW) : "memory");
    } else if (ahead == 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (AVC_GEMM_DIAG_NOBAR) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const bool issue_next = kt + NS - 1 < kt1;
    if constexpr (SPR == 0) {
      if (issue_next) AVC16F_FAST_ISSUE(kt + NS - 1, (kt + NS - 1 - kt0) % NS);
    } else {
      sp_inside = false;
      if (issue_next) AVC16F_SPREAD_BEGIN(kt + NS - 1, (kt + NS - 1 - kt0) % NS);
    }
    const unsigned char* Ai = lds + st * STAGE;
    const unsigned char* Bi = Ai + ABLK * 1024;
    // Fragments of chunk s + 1 are read while chunk s's MFMAs issue (two register buffers), and
    // the MFMAs go in passes over the accumulators (hi.hi for every tile, then hi.lo, then
    // lo.hi): no MFMA waits on a just-issued LDS read or on the MFMA right before it.  Each
    // accumulator still sees hi.hi, hi.lo, lo.hi per chunk in the same order (bit-identical).
#define AVC16F_FRAGS(S, BUF)                                                                      \
    _Pragma("unroll") for (int i = 0; i < TM; ++i) {                                              \
      const unsigned char* p = Ai + (((wm * TM + i) * KC + (S)) * 2) * 1024 + lane * 16;          \
      fah[BUF][i] = *reinterpret_cast<const f16x8*>(p);                                           \
      fal[BUF][i] = *reinterpret_cast<const f16x8*>(p + 1024);                                    \
    }                                                                                             \
    _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                              \
      const unsigned char* p = Bi + (((wn * TN + j) * KC + (S)) * 2) * 1024 + lane * 16;          \
      fbh[BUF][j] = *reinterpret_cast<const f16x8*>(p);                                           \
      fbl[BUF][j] = *reinterpret_cast<const f16x8*>(p + 1024);                                    \
    }
    if (!AVC_GEMM_DIAG_NOREAD || kt == kt0) { AVC16F_FRAGS(0, 0) }
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      if (s + 1 < KC && (!AVC_GEMM_DIAG_NOREAD || kt == kt0)) { AVC16F_FRAGS(s + 1, (s + 1) & 1) }
      if constexpr (SPR > 0) {
        if (s < SPR && sp_inside && !AVC_GEMM_NOLOAD) AVC16F_SPREAD_PIECES(s * (DPW / SPR), (s + 1) * (DPW / SPR))
      }
      // pin the order: without it the scheduler sinks the next chunk's reads back under these
      // MFMAs and every pass waits on lgkmcnt(0) again
      __builtin_amdgcn_sched_barrier(0);
      const int cb = s & 1;
      if (AVC_GEMM_DIAG_NOMFMA) {  // (diagnostic: the fragments stay live, no MFMA)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            crs[i][j][0] += (float)fah[cb][i][0] + (float)fal[cb][i][1] + (float)fbh[cb][j][2] + (float)fbl[cb][j][3];
      } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if constexpr (KH == 2) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[cb][i], fbh[cb][j], acc[i][j], 0, 0, 0);
          else part[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[cb][i], fbh[cb][j], part[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          crs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fah[cb][i], fbl[cb][j], crs[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          crs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(fal[cb][i], fbh[cb][j], crs[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#undef AVC16F_FRAGS
#undef AVC16F_SPREAD_PIECES
    if (KH != 2 && ((kt - kt0) % KB == KB - 1 || kt + 1 == kt1)) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            if constexpr (KH == 1 && OCC == 1 && !AVC_GEMM_DIAG_NOKAHAN) {
              const float y = part[i][j][e] - cmp[i][j][e];
              const float t = acc[i][j][e] + y;
              cmp[i][j][e] = (t - acc[i][j][e]) - y;
              acc[i][j][e] = t;
            } else {
              acc[i][j][e] += part[i][j][e];
            }
          }
          part[i][j] = zero16;
        }
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        acc[i][j][e] = (KH == 1 && OCC == 1 ? acc[i][j][e] - cmp[i][j][e] : acc[i][j][e]) + crs[i][j][e] * (1.0f / 2048.0f);
#undef AVC16F_ISSUE
#undef AVC16F_SETTAP
#undef AVC16F_FAST_ISSUE
#undef AVC16F_SPREAD_BEGIN
  if (AVC_GEMM_DIAG_NOEPI) {  // (diagnostic: keep every sum live, skip every epilogue)
    float keep = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) keep += acc[i][j][e];
    if (keep == 1.2345f && threadIdx.x == 9999) d.C[0] = keep;
    return;
  }
  if (d.split_scale && nsplit == 1) {  // split-K partials stay scaled; splitk_reduce_kernel unscales
    const float us = split_unscale(d.amax_a, d.amax_b);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] *= us;
  }

  // ---- epilogue (32x32 C layout: col = lane&31, row = (e&3) + 8(e>>2) + 4(lane>>5)) --------
  const int row_base = tm * BM + wm * WTM + 4 * (lane >> 5);
  const int col_base = tn * BN + wn * WTN + (lane & 31);
  if (nsplit > 1) {
    float* out = slab + ((long)split * d.nz + z) * d.M * d.N;
    if (kTileFits && g_tile_rows_ok(out, d.N, 1)) {  // (round 6: through LDS, whole rows; same values)
      const float zb[TN] = {};
      store_tile_rows<BM, BN, TM, TN, NT>(out, d.N, d.M, d.N, tm * BM, tn * BN, acc, zb, AVC_ACT_NONE, false, lds,
                                          row_base - tm * BM, col_base - tn * BN, tid);
      return;
    }
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
  if constexpr (BNF) {
    bnf_epilogue<BM, BN, WM, WTN, TM, TN, NT>(d, acc, lds, tm, tn, tilesM, wm, lane, tid, row_base, col_base,
                                              bnf_ticket, bnf_bias, bnf_par);
    return;
  }
  float* __restrict__ C = d.C + (long)z * d.c_zoff;
  const float (&biasv)[TN] = bnf_bias;
  if (kTileFits && d.ldc_col == 1 && g_tile_rows_ok(C, d.ldc, 1)) {  // (round 6: through LDS, whole rows; same values)
    store_tile_rows<BM, BN, TM, TN, NT>(C, d.ldc, d.M, d.N, tm * BM, tn * BN, acc, biasv, d.act, d.accumulate != 0,
                                        lds, row_base - tm * BM, col_base - tn * BN, tid);
  } else {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col_base + 32 * j;
    const bool colok = col < d.N;
    const float bias = biasv[j];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = row_base + 32 * i + (e & 3) + 8 * (e >> 2);
        if (!colok || row >= d.M) continue;
        const float v = act_apply(acc[i][j][e] + bias, d.act);
        float* p = C + (long)row * d.ldc + (long)col * d.ldc_col;
        if (d.accumulate) *p += v; else *p = v;
      }
  }
  }
  if (d.stats)
    bn_tile_stats<BM, BN, WM, WTN, TM, TN, BM == 256 ? 2 : 1, false, false>(
        d, acc, biasv, reinterpret_cast<float*>(lds), tm, tn, wm, wn, lane, tid, NT, row_base, col_base);
}

// splitk_reduce_kernel for the common case (one product, row-major C, N % 4 == 0): a thread sums
// 4 consecutive columns of one row over the splits (float4 streams); grid.y walks row blocks.
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(GemmDesc d, int nsplit, const float* __restrict__ slab,
                                                             int rows_per_block) {
  const int n4 = d.N >> 2;
  const long MN = (long)d.M * d.N;
  const float us = d.split_scale ? split_unscale(d.amax_a, d.amax_b) : 1.f;
  const int r1 = min(d.M, (int)(blockIdx.y + 1) * rows_per_block);
  for (int i = threadIdx.x; ; i += 256) {
    const int m = blockIdx.y * rows_per_block + i / n4, c4 = i - (i / n4) * n4;
    if (m >= r1) break;
    const long off = (long)m * d.N + 4 * c4;
    float4 a = *reinterpret_cast<const float4*>(slab + off);
    for (int sp = 1; sp < nsplit; ++sp) {
      const float4 b = *reinterpret_cast<const float4*>(slab + sp * MN + off);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = 4 * c4 + e;
      float t = v[e] * us;
      if (d.bias0) t += d.bias0[n];
      if (d.bias1) t += d.bias1[n];
      v[e] = act_apply(t, d.act);
    }
    float* p = d.C + (long)m * d.ldc + 4 * c4;
    if (d.accumulate) {
      const float4 o = *reinterpret_cast<const float4*>(p);
      v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
    }
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// The same reduction for few output rows (weight gradients of narrow layers: M = 4H = 128): one
// row chunk per block (rpb rows x N/4 float4 = tasks <= 256/G), and G thread groups sum
// interleaved K-splits, combined through LDS in a fixed order (deterministic).
__global__ __launch_bounds__(256) void splitk_reduce4g_kernel(GemmDesc d, int nsplit, const float* __restrict__ slab,
                                                              int rows_per_block, int G) {
  __shared__ float4 part[256];
  const int n4 = d.N >> 2;
  const long MN = (long)d.M * d.N;
  const int tasks = rows_per_block * n4;
  const int g = threadIdx.x / tasks;
  const int i = threadIdx.x - g * tasks;
  const int m = blockIdx.y * rows_per_block + i / n4, c4 = i - (i / n4) * n4;
  const long off = (long)m * d.N + 4 * c4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (g < G && m < d.M) {
    for (int sp = g; sp < nsplit; sp += G) {
      const float4 b = *reinterpret_cast<const float4*>(slab + sp * MN + off);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
  }
  part[threadIdx.x] = a;
  __syncthreads();
  if (g != 0 || m >= d.M) return;
  for (int gg = 1; gg < G; ++gg) {
    const float4 b = part[gg * tasks + i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  const float us = d.split_scale ? split_unscale(d.amax_a, d.amax_b) : 1.f;
  float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int n = 4 * c4 + e;
    float t = v[e] * us;
    if (d.bias0) t += d.bias0[n];
    if (d.bias1) t += d.bias1[n];
    v[e] = act_apply(t, d.act);
  }
  float* p = d.C + (long)m * d.ldc + 4 * c4;
  if (d.accumulate) {
    const float4 o = *reinterpret_cast<const float4*>(p);
    v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
  }
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
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
    if (d.split_scale) s *= split_unscale(d.amax_a, d.amax_b);
    if (d.bias0) s += d.bias0[n];
    if (d.bias1) s += d.bias1[n];
    s = act_apply(s, d.act);
    float* p = d.C + (long)z * d.c_zoff + (long)m * d.ldc + (long)n * d.ldc_col;
    if (d.accumulate) *p += s; else *p = s;
  }
}

// avc_gemm_tune(): forward (prec16) products on 0 = the fp32 kernel, 1 = gemm16 (operands split
// while staged), 2 = gemm16f on pre-split fragment-major operands where eligible (default);
// 3 = as 2 for forward products but backward (split_scale) products on the fp32 kernel
int g_gemm16 = 2;

struct Plan {
  int bm, bn, tilesM, tilesN, kt_per_tap, ktotal, nsplit, kps;
};

int g_plan_rounds = 1;  // avc_gemm_plan_rounds(): round-aware split-K count for long-K products

Plan make_plan(const GemmDesc& d, int force_split) {
  Plan p;
  // long-K products (weight gradients: K = T*B rows) take 128x128 tiles and split K until the
  // grid has ~4 workgroups per CU
  const bool longk = (long)d.Kc * d.ntaps >= 8192 && d.M >= 128 && d.N >= 128;
  const bool big = (long)d.M * d.N > 256L * 128 * 128 / 2 || longk;
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
  } else if (!d.stats && longk && blocks < 1024) {
    ns = (int)((1024 + blocks - 1) / blocks);
    ns = std::min(ns, p.ktotal / 16);
    ns = std::min(ns, 32);
    ns = std::max(ns, 1);
    if (g_plan_rounds) {
      // round-aware split (round 5, avc_gemm_plan_rounds): the grid runs in rounds of one
      // workgroup per CU, so a split count whose grid spills a few workgroups into an extra round
      // pays that whole round (the conv weight gradients: 80 tiles x 13 splits = 1040 workgroups,
      // 4.06 rounds on 256 CUs).  Among ns / 2 .. 2 ns, take the count that minimises rounds x
      // K-steps per split, plus each split's slab write + read (~0.75 us per 32-deep K-step,
      // ~5 TB/s for the slab)
      const int cus = std::max(1, coresident_cus());
      const double slab_us = (double)d.M * d.N * d.nz * 8.0 / 5.0e6;
      double best = 1e30;
      int pick = ns;
      for (int n = std::max(1, ns / 2); n <= std::min({2 * ns, 32, std::max(1, p.ktotal / 16)}); ++n) {
        const long rounds = (blocks * n + cus - 1) / cus;
        const long kps = (p.ktotal + n - 1) / n;
        const double cost = (double)rounds * kps * 0.75 + n * slab_us;
        if (cost < best - 1e-9) {
          best = cost;
          pick = n;
        }
      }
      ns = pick;
    }
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

inline long frag_ntile(long rows) { return (rows + 31) / 32; }
inline int frag_nkc(int K) { return (K + 31) / 32 * 2; }
inline size_t frag_bytes(long rows, int K) { return (size_t)frag_ntile(rows) * frag_nkc(K) * 2048; }

bool frag16_eligible(const GemmDesc& d) {
  if (!d.prec16 || d.a_zoff != 0) return false;
  if (g_gemm16 != 2 && !(g_gemm16 == 3 && !d.split_scale)) return false;
  if (d.a_trans) {
    if (d.ntaps != 1 || d.a_shift0 != 0) return false;
  } else if (d.a_shift0 % 32 != 0 || (d.ntaps > 1 && d.a_tapshift % 32 != 0)) {
    return false;
  }
  const bool bshift = d.b_shift0 != 0 || d.b_zshift != 0;
  if (bshift && (d.b_trans || d.b_shift0 % 16 != 0 || d.b_zshift % 16 != 0 || d.ntaps != 1)) return false;
  if (d.nz > 1 && !bshift) return false;
  return d.b_trans || bshift || d.b_rows >= d.Kc;
}

// rows of the B operand's source that its fragments cover
inline long frag16_b_krows(const GemmDesc& d) {
  const long b_rows = d.b_rows ? d.b_rows : (d.b_trans ? d.N : d.Kc);
  if (d.b_trans) return d.Kc;
  if (d.b_shift0 != 0 || d.b_zshift != 0) return b_rows;
  return std::min<long>(d.Kc, b_rows);
}

size_t frag16_scratch(const GemmDesc& d) {
  const long a_rows = d.a_trans ? d.M : (d.a_rows ? d.a_rows : d.M);
  return frag_bytes(a_rows, d.Kc) + (size_t)d.ntaps * frag_bytes(d.N, (int)frag16_b_krows(d)) + 2048;
}

// avc_gemm_config(): tile/ring variant of gemm16f; 8 (= 1 with the plain fold of the 128-k
// partials) is the default since round 3 (1 in rounds 1-2).  Late round 3: 9 / 10 (256 x 128 tiles)
// and 11 (8 with the hi.hi products in one MFMA chain over K) were 0-3 % faster on single GEMMs but
// moved the C3 step by < 0.1 ms (34.68 vs 34.72 ms) while 10 / 11 double the product's error
// against float64 (1.9e-7 -> 3.9e-7 on the 8192 x 4096 x 512 product), so 8 stays
int g_gemm_cfg = 8;

template <int BM, int BN, int WM, int WN, int NS, int KC, int OCC = 1, int KH = 1>
void launch16f_cfg(const GemmDesc& d, const Frag16Args& f, const Plan& p, float* slab, hipStream_t s) {
  constexpr int NBLK = (BM / 32) * KC * 2 + (BN / 32) * KC * 2;
  const size_t lds = (size_t)NS * NBLK * 1024;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm16f_kernel<BM, BN, WM, WN, NS, KC, OCC, KH>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  // K-tiles of KC 16-deep chunks; the split-K plan is re-cut in these units (every split
  // writes its slab, an empty range writes zeros)
  const int kt_per_tap = (f.a_nkc + KC - 1) / KC;
  const int ktotal = d.ntaps * kt_per_tap;
  const int kps = (ktotal + p.nsplit - 1) / p.nsplit;
  // tiles of this instance (the plan's are 128 x 128 for every big product; a 256-row instance
  // halves tilesM and keeps the plan's split-K count)
  const int tilesM = (d.M + BM - 1) / BM, tilesN = (d.N + BN - 1) / BN;
  dim3 grid(tilesM * tilesN, d.nz * p.nsplit);
  gemm16f_kernel<BM, BN, WM, WN, NS, KC, OCC, KH><<<grid, 64 * WM * WN, lds, s>>>(d, f, tilesM, tilesN, kt_per_tap,
                                                                        kps, p.nsplit, slab);
}

void launch16f_128(const GemmDesc& d, const Frag16Args& f, const Plan& p, float* slab, hipStream_t s) {
  switch (g_gemm_cfg) {
    case 1: launch16f_cfg<128, 128, 4, 2, 2, 4>(d, f, p, slab, s); break;
    case 2: launch16f_cfg<128, 128, 4, 2, 3, 3>(d, f, p, slab, s); break;
    case 3: launch16f_cfg<128, 128, 2, 4, 4, 2>(d, f, p, slab, s); break;
    case 4: launch16f_cfg<128, 128, 2, 4, 2, 4>(d, f, p, slab, s); break;
    case 5: launch16f_cfg<128, 128, 4, 2, 3, 2>(d, f, p, slab, s); break;
    case 6: launch16f_cfg<128, 128, 4, 2, 2, 2, 2>(d, f, p, slab, s); break;
    case 7: launch16f_cfg<128, 128, 4, 2, 2, 4, 2>(d, f, p, slab, s); break;
    case 8: launch16f_cfg<128, 128, 4, 2, 2, 4, 1, 0>(d, f, p, slab, s); break;  // cfg 1, plain fold
    case 9: launch16f_cfg<256, 128, 4, 2, 3, 2, 1, 0>(d, f, p, slab, s); break;  // 256-row tiles
    case 10: launch16f_cfg<256, 128, 4, 2, 3, 2, 1, 2>(d, f, p, slab, s); break;  // ... hi.hi into one chain
    case 11: launch16f_cfg<128, 128, 4, 2, 2, 4, 1, 2>(d, f, p, slab, s); break;  // 8 with hi.hi into one chain
    default: launch16f_cfg<128, 128, 4, 2, 4, 2>(d, f, p, slab, s); break;
  }
}

template <int BM, int BN, int WM, int WN>
void launch16(const GemmDesc& d, const Plan& p, float* slab, hipStream_t s) {
  dim3 grid(p.tilesM * p.tilesN, d.nz * p.nsplit);
  constexpr int NT = 64 * WM * WN;
  if (d.b_trans)
    gemm16_kernel<BM, BN, WM, WN, 1><<<grid, NT, 0, s>>>(d, p.tilesM, p.tilesN, p.kt_per_tap, p.kps, p.nsplit, slab);
  else
    gemm16_kernel<BM, BN, WM, WN, 0><<<grid, NT, 0, s>>>(d, p.tilesM, p.tilesN, p.kt_per_tap, p.kps, p.nsplit, slab);
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

size_t gemm_bfrag_bytes(const GemmDesc& d) { return (size_t)d.ntaps * frag_bytes(d.N, d.Kc) + 256; }

namespace {
// the range-guard word behind a prepared B operand's fragments
unsigned* bfrag_guard_word(const GemmDesc& d, const _Float16* bf) {
  return reinterpret_cast<unsigned*>(const_cast<char*>(reinterpret_cast<const char*>(bf)) +
                                     (size_t)d.ntaps * frag_bytes(d.N, d.Kc));
}

// max |B| over all taps of a forward product's B operand into a guard word
// max |x| over the taps of a multi-tap operand (rows x cols each, row stride ld, taps tapoff
// apart): one scan when the taps tile one dense block, else one per tap
void absmax_taps(const float* src, int ntaps, long tapoff, long rows, long cols, long ld, unsigned* out,
                 hipStream_t s) {
  if (ntaps > 1 && ld == cols && tapoff == rows * cols) {
    absmax2d(src, rows * ntaps, cols, ld, out, s);
    return;
  }
  for (int tau = 0; tau < ntaps; ++tau) absmax2d(src + (long)tau * tapoff, rows, cols, ld, out, s);
}

// where the B split reads element (n, k) of tap tau: p[n * rs + k * ks + tau * tap]
struct BSrc {
  const float* p;
  long rs, ks, tap;
};
BSrc b_src(const GemmDesc& d) {
  if (d.b_conv == 1) return {d.B, 5L * d.Kc, 5, 1};
  if (d.b_conv == 2) return {d.B + 4, 5, 5L * d.N, -1};
  return {d.B, d.b_trans ? d.ldb : 1, d.b_trans ? 1 : d.ldb, d.b_tapoff};
}

// the B operand's split into its tap images: a Conv1d weight through split_convw_kernel (one
// pass, whole-block stores), any other through split_frag32_kernel
void split_b(const GemmDesc& d, int K, long ntile, int nkc, _Float16* dst, long tapstride, const unsigned* amax,
             hipStream_t s) {
  if (d.b_conv && d.ntaps == 5) {
    const unsigned blocks = (unsigned)(ntile * nkc);
    if (d.b_conv == 1)
      split_convw_kernel<1><<<blocks, 64, 0, s>>>(d.B, d.N, K, (int)ntile, nkc, dst, tapstride, amax);
    else
      split_convw_kernel<2><<<blocks, 64, 0, s>>>(d.B, d.N, K, (int)ntile, nkc, dst, tapstride, amax);
    return;
  }
  const long tb = ntile * 32 * nkc * 2;
  const BSrc bsrc = b_src(d);
  split_frag32_kernel<<<dim3((int)std::min<long>((tb + 255) / 256, 8192), d.ntaps), 256, 0, s>>>(
      bsrc.p, bsrc.rs, bsrc.ks, d.N, K, (int)ntile, nkc, dst, amax, bsrc.tap, tapstride);
}

void absmax_b(const GemmDesc& d, unsigned* w, hipStream_t s) {
  if (d.b_conv) {  // the whole weight, one contiguous scan
    absmax2d(d.B, 1, 5L * d.N * d.Kc, 5L * d.N * d.Kc, w, s);
    return;
  }
  const long b_rows = d.b_rows ? d.b_rows : (d.b_trans ? d.N : d.Kc);
  const long kb = d.b_trans ? d.Kc : std::min<long>(d.Kc, b_rows);
  if (d.b_trans) absmax_taps(d.B, d.ntaps, d.b_tapoff, d.N, kb, d.ldb, w, s);
  else absmax_taps(d.B, d.ntaps, d.b_tapoff, kb, d.N, d.ldb, w, s);
}
}  // namespace

// Range guard of the forward split: a guard word starts at 2^14 and takes the
// operand's max |x| (atomicMax on float bits), so split_scale_of() returns exactly 1 unless
// max |x| >= 2^15, and otherwise the power of two that brings it into [2^14, 2^15): overflow-free
// splits for any magnitude, bit-identical results in the normal range.
__global__ void guard_init_kernel(unsigned* w, int n) {
  if ((int)threadIdx.x < n) w[threadIdx.x] = 0x46800000u;  // 16384.0f
}

// The same guard word in ONE launch (no initialisation kernel): every block writes its maximum
// to partial[blockIdx], and the last block to take a ticket (atomicInc wraps the per-context
// ticket back to 0, so it is ready for the next scan) writes max(all, 2^14) to *out.
constexpr int kGuardBlocks = 256;  // partial words of the guard scan (one per workgroup; each takes a ticket atomic, 1024 measured slower)
__global__ __launch_bounds__(256) void guard_scan_kernel(const float* __restrict__ src, long rows, int cols,
                                                         long ld, float* __restrict__ partial,
                                                         unsigned* __restrict__ ticket, unsigned* __restrict__ out) {
  __shared__ float red[4];
  __shared__ bool last;
  float m = 0.f;
  if (ld == cols && (reinterpret_cast<uintptr_t>(src) & 15) == 0 && (cols & 3) == 0) {
    const long n4 = rows * cols / 4;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    const long stride = (long)gridDim.x * 256;
    long i = blockIdx.x * 256L + threadIdx.x;
    for (; i + 7 * stride < n4; i += 8 * stride) {  // eight loads in flight
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = s4[i + u * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    }
    for (; i < n4; i += stride) {
      const float4 v = s4[i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  } else {
    for (long r = blockIdx.x; r < rows; r += gridDim.x)
      for (int c = threadIdx.x; c < cols; c += 256) m = fmaxf(m, fabsf(src[r * ld + c]));
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(partial + blockIdx.x, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    last = atomicInc(ticket, gridDim.x - 1) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  float v = 16384.f;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += 256)
    v = fmaxf(v, __hip_atomic_load(partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) *out = __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

int gemm_prepare_bfrag(const GemmDesc& d, _Float16* dst, hipStream_t stream) {
  const long b_ntile = frag_ntile(d.N);
  const int nkc = frag_nkc(d.Kc);
  const long tapstride = b_ntile * nkc * 1024;  // halves
  const long b_rows = d.b_rows ? d.b_rows : (d.b_trans ? d.N : d.Kc);
  unsigned* guard = bfrag_guard_word(d, dst);
  guard_init_kernel<<<1, 64, 0, stream>>>(guard, 1);
  absmax_b(d, guard, stream);
  split_b(d, d.b_trans ? d.Kc : (int)std::min<long>(d.Kc, b_rows), b_ntile, nkc, dst, tapstride, guard, stream);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int gemm_absmax(const float* src, long rows, long cols, long ld, unsigned* out, hipStream_t stream) {
  AVC_TRY(zero_async(out, sizeof(unsigned), stream));
  absmax2d(src, rows, cols, ld, out, stream);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

size_t gemm_afrag_bytes(long rows, int K) { return frag_bytes(rows, K); }

// Raw split-K partial products of two operands already split into the fragment-major layout
// (split_frag32_kernel): slab[split][M][N] = A_frag(M x K) . B_frag(N x K)^T, no scale, no
// epilogue.  The BPTT recurrence (lstm.hip) reduces the slabs in its own epilogue.
int gemm_frag_partials(int M, int N, int K, const _Float16* As, const _Float16* Bs, int tile, int nsplit,
                       float* slab, hipStream_t s) {
  AVC_CHECK_ARG(M > 0 && N > 0 && K > 0 && As && Bs && slab && nsplit >= 1 && (tile == 64 || tile == 128),
                "gemm_frag_partials: bad arguments");
  GemmDesc d;
  d.M = M; d.N = N; d.Kc = K; d.ntaps = 1;
  Frag16Args f{};
  f.As = As; f.a_ntile = (int)frag_ntile(M); f.a_nkc = frag_nkc(K); f.a_shift0 = 0; f.a_tapshift = 0;
  f.Bs = Bs; f.b_ntile = (int)frag_ntile(N); f.b_nkc = frag_nkc(K);
  f.b_tapstride = (long)f.b_ntile * f.b_nkc * 1024;  // halves: the descriptor covers all of B
  Plan p{};
  p.bm = p.bn = tile;
  p.tilesM = (M + tile - 1) / tile;
  p.tilesN = (N + tile - 1) / tile;
  p.nsplit = nsplit;
  if (tile == 128) launch16f_cfg<128, 128, 4, 2, 2, 4>(d, f, p, slab, s);
  else launch16f_cfg<64, 64, 2, 2, 4, 2>(d, f, p, slab, s);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

// split a [R][K] row-major fp32 matrix (row stride rs) into the fragment-major layout, scaled
// by the power of two split_scale_of(amax) (amax NULL: unscaled)
// One read of a row-major [R][C] operand (R % 32 == 0, C % 64 == 0) writes BOTH of its scaled
// split images: dst_a as the A operand of a product with K = C (rows R: split_frag32_kernel's
// row-major layout) and dst_t as the A^T operand of a product with K = R (rows C: its transposed
// layout).  Workgroup = a 32 x 64 block staged through LDS; every element is scaled and split by
// the expressions split_frag32_kernel uses, so both images are its bits.  (The LSTM backward's dG:
// the dX product reads it as A, the two weight-gradient products as A^T; two split passes read the
// 512 MB operand twice.)
__global__ __launch_bounds__(256) void split_frag32_dual_kernel(const float* __restrict__ src, long ld, int R, int C,
                                                                const unsigned* __restrict__ amax,
                                                                _Float16* __restrict__ dst_a,
                                                                _Float16* __restrict__ dst_t,
                                                                const unsigned* __restrict__ amax_t) {
  // (amax_t: the A^T image's own scale; the tile holds the unscaled values, each image multiplies
  // by its scale once, as split_frag32_kernel does)
  __shared__ float tile[32][65];
  const int tid = threadIdx.x;
  const long bt = blockIdx.x;        // 32-row block
  const int bc = (int)blockIdx.y;    // 64-column block
  const float sc = split_scale_of(amax), sct = split_scale_of(amax_t);
  const int nkc_a = C / 16, nkc_t = R / 16;
  {  // A image: thread = (row rr, 8-column group g)
    const int rr = tid >> 3, g = tid & 7;
    const long r = bt * 32 + rr;
    const float4* q = reinterpret_cast<const float4*>(src + r * ld + (long)bc * 64 + 8 * g);
    const float4 a = q[0], b = q[1];
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[rr][8 * g + e] = v[e];
    if (amax) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= sc;
    }
    f16x8 hi, lo;
    split8(v, hi, lo);
    const int g8 = bc * 8 + g;
    const long blk = ((r >> 5) * nkc_a + (g8 >> 1)) * 2;
    const int lane = (int)(r & 31) + 32 * (g8 & 1);
    *reinterpret_cast<f16x8*>(dst_a + blk * 512 + lane * 8) = hi;
    *reinterpret_cast<f16x8*>(dst_a + (blk + 1) * 512 + lane * 8) = lo;
  }
  __syncthreads();
  {  // A^T image: thread = (column c, 8-row group q)
    const int c = tid & 63, q = tid >> 6;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = tile[8 * q + e][c];
    if (amax_t) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= sct;
    }
    f16x8 hi, lo;
    split8(v, hi, lo);
    const long r = (long)bc * 64 + c;
    const long g8 = bt * 4 + q;
    const long blk = ((r >> 5) * nkc_t + (g8 >> 1)) * 2;
    const int lane = (int)(r & 31) + 32 * (int)(g8 & 1);
    *reinterpret_cast<f16x8*>(dst_t + blk * 512 + lane * 8) = hi;
    *reinterpret_cast<f16x8*>(dst_t + (blk + 1) * 512 + lane * 8) = lo;
  }
}

bool gemm_split_dual_ok(long R, long C, long ld) {
  return R > 0 && C > 0 && R % 32 == 0 && C % 64 == 0 && ld % 4 == 0 && R / 32 < 0x7fffffffL && C / 64 <= 65535;
}

int gemm_split_dual2(const float* src, long ld, long R, int C, const unsigned* amax_a, const unsigned* amax_t,
                     _Float16* dst_a, _Float16* dst_t, hipStream_t s) {
  AVC_CHECK_ARG(gemm_split_dual_ok(R, C, ld) && (reinterpret_cast<uintptr_t>(src) & 15) == 0,
                "gemm_split_dual: needs rows % 32 == 0, columns % 64 == 0 and 16-byte aligned rows");
  split_frag32_dual_kernel<<<dim3((unsigned)(R / 32), (unsigned)(C / 64)), 256, 0, s>>>(src, ld, (int)R, C, amax_a,
                                                                                       dst_a, dst_t, amax_t);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int gemm_split_dual(const float* src, long ld, long R, int C, const unsigned* amax, _Float16* dst_a, _Float16* dst_t,
                    hipStream_t s) {
  return gemm_split_dual2(src, ld, R, C, amax, amax, dst_a, dst_t, s);
}

int gemm_split_frag(const float* src, long rs, int R, int K, const unsigned* amax, _Float16* dst, hipStream_t s) {
  const long ntile = frag_ntile(R);
  const int nkc = frag_nkc(K);
  const long total = ntile * 32 * nkc * 2;
  split_frag32_kernel<<<(int)std::min<long>((total + 255) / 256, 8192), 256, 0, s>>>(src, rs, 1, R, K, (int)ntile,
                                                                                   nkc, dst, amax);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}
int gemm_split_frag_t(const float* src, long ld, long R, int C, const unsigned* amax, _Float16* dst, hipStream_t s) {
  AVC_CHECK_ARG(R > 0 && C > 0 && R < 0x7fffffffL, "gemm_split_frag_t: bad shape");
  const long ntile = frag_ntile(C);
  const int nkc = frag_nkc((int)R);
  const long total = ntile * 32 * nkc * 2;
  split_frag32_kernel<<<(int)std::min<long>((total + 255) / 256, 8192), 256, 0, s>>>(src, 1, ld, C, (int)R, (int)ntile,
                                                                                   nkc, dst, amax);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}
bool gemm_frag_eligible(const GemmDesc& d) { return frag16_eligible(d); }

size_t gemm_scratch_bytes(const GemmDesc& d) {
  Plan p = make_plan(d, 0);
  size_t s = p.nsplit <= 1 ? 0 : (size_t)p.nsplit * d.nz * d.M * d.N * sizeof(float) + 256;
  if (d.prec16) s += frag16_scratch(d);
  return s;
}

namespace {
int guard_scan(avc_context* ctx, const float* src, long rows, long cols, long ld, float* part, unsigned* out,
               hipStream_t s) {
  if (!ctx->guard_ticket) {  // first use happens eagerly (graphs are captured on a later call)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    AVC_HIP(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) {
      set_error("range guard: ticket not allocated before graph capture");
      return AVC_ERR_WORKSPACE;
    }
    AVC_HIP(hipMalloc(&ctx->guard_ticket, 256));
    AVC_HIP(hipMemsetAsync(ctx->guard_ticket, 0, 256, s));
    AVC_HIP(hipStreamSynchronize(s));
  }
  const long n4 = rows * cols / 4;
  const int blocks = (int)std::min<long>(scan_blocks(n4), kGuardBlocks);
  guard_scan_kernel<<<blocks, 256, 0, s>>>(src, rows, (int)cols, ld, part, ctx->guard_ticket, out);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}
}  // namespace

// ---- fused BatchNorm epilogue: eligibility and launch ------------------------------------
int g_bnf = 1;  // avc_bn_fuse()
int g_bnf_band = 1;  // avc_bn_fuse_band(): XCD-contiguous row bands in the fused instance's dispatch order
int g_bnf_inject = 0;  // avc_debug_bnf_inject(): train-mode fused launches left that give up at once

namespace {
// the two gemm16f instances the plans pick (128 x 128: avc_gemm_config 8; 64 x 64), BNF = 1
const void* bnf_fn(int bm) {
  if (bm == 128) return reinterpret_cast<const void*>(&gemm16f_kernel<128, 128, 4, 2, 2, 4, 1, 0, 1>);
  return reinterpret_cast<const void*>(&gemm16f_kernel<64, 64, 2, 2, 4, 2, 1, 1, 1>);
}
size_t bnf_lds(int bm) { return bm == 128 ? 2 * 64 * 1024 : 4 * 16 * 1024; }
int bnf_threads(int bm) { return bm == 128 ? 512 : 256; }

// workgroups of the instance the device holds at once (occupancy API x CUs), per device
int bnf_capacity(int bm) {
  struct Entry { const void* fn; int dev, cap; };
  static std::vector<Entry> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const void* fn = bnf_fn(bm);
  for (const auto& e : cache)
    if (e.fn == fn && e.dev == dev) return e.cap;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bnf_lds(bm));
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, bnf_threads(bm), bnf_lds(bm)) != hipSuccess) {
    (void)hipGetLastError();
    per_cu = 0;
  }
  const int cap = per_cu * coresident_cus();
  cache.push_back({fn, dev, cap});
  return cap;
}

int launch16f_bnf(avc_context* ctx, GemmDesc d, Frag16Args f, const Plan& p, hipStream_t s) {
  d.bnf.band = g_bnf_band;
  const int bm = p.bm;
  const int KC = bm == 128 ? 4 : 2;
  int kt_per_tap = (f.a_nkc + KC - 1) / KC;
  int kps = d.ntaps * kt_per_tap, nsplit = 1;
  int tilesM = (d.M + bm - 1) / bm, tilesN = (d.N + bm - 1) / bm;
  const int nwg = tilesM * tilesN;
  AVC_CHECK_ARG(tilesM <= bnf_capacity(bm), "fused BatchNorm GEMM: a column tile's workgroups are not co-resident");
  const void* fn = bnf_fn(bm);
  float* slab = nullptr;
  void* args[] = {&d, &f, &tilesM, &tilesN, &kt_per_tap, &kps, &nsplit, &slab};
  if (!d.bnf.training) {  // eval mode: no barrier, an ordinary launch
    AVC_HIP(hipLaunchKernel(fn, dim3(nwg), dim3(bnf_threads(bm)), args, bnf_lds(bm), s));
    return AVC_OK;
  }
  unsigned* region = nullptr;
  AVC_TRY(coresident_region(ctx, 4, tilesM, tilesN, nwg, (size_t)tilesN * 32, s, &region));
  unsigned* flags = host_flags(ctx);
  if (!flags) return AVC_ERR_HIP;
  d.bnf.tickets = reinterpret_cast<unsigned long long*>(region);  // region layout: lstm_persist.hip
  d.bnf.tmo = region + 32;
  d.bnf.cnt = region + 64;
  d.bnf.fail_host = flags;
  d.bnf.spin_limit = coresident_spin_limit();
  if (g_bnf_inject > 0) {  // test hook: this launch's barrier gives up at its first unmet poll
    --g_bnf_inject;
    d.bnf.spin_limit = 0;
  }
  d.bnf.nwg = nwg;
  return coresident_dispatch(ctx, fn, dim3(nwg), dim3(bnf_threads(bm)), args, bnf_lds(bm), s);
}
}  // namespace

bool gemm_bnf_ok(const GemmDesc& d, bool training) {
  if (!g_bnf || !d.prec16 || d.split_scale || !frag16_eligible(d) || d.nz != 1 || d.accumulate || d.ldc_col != 1 ||
      d.act != AVC_ACT_NONE || d.N % 8 != 0)
    return false;
  Plan p = make_plan(d, 0);
  if (training) p.nsplit = 1;  // a stats product never splits K (gemm_run)
  if (p.nsplit != 1 || p.bm != p.bn) return false;
  if (p.bm == 128 && g_gemm_cfg != 8) return false;  // the fused 128 x 128 instance: configuration 8
  // The invariant the barrier needs: one column tile's tilesM workgroups (a contiguous dispatch
  // range) resident at once.  avc_bn_fuse(1) also keeps the fused form to grids that are one
  // co-resident wave; 2 takes it wherever a single group fits (multi-wave grids, e.g. C3's 1024).
  const int cap = bnf_capacity(p.bm);
  if (p.tilesM > cap) return false;
  return g_bnf == 2 || p.tilesM * p.tilesN <= cap;
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
  Frag16Args fa{};
  const bool frag = frag16_eligible(d);
  AVC_CHECK_ARG(!d.b_conv || (frag && d.ntaps == 5 && !d.b_trans && d.b_rows == d.Kc),
                "gemm: a Conv1d-layout B operand needs the split-f16 fragment path");
  const bool scaled_product = d.split_scale != 0;
  if (!frag) {  // only the split-f16 path scales its operands
    d.split_scale = 0;
    d.amax_a = d.amax_b = nullptr;
  }
  if (frag && !scaled_product) {
    // forward product: range guard (see guard_init_kernel).  B from gemm_prepare_bfrag carries
    // its guard word; an A handed over pre-split (bn_apply's fragment output) was range-checked
    // by its producer; every other operand is scanned here unless its bound is known.
    unsigned* gw = sc.take<unsigned>(64);
    float* part = sc.take<float>(kGuardBlocks);
    if (!gw || !part) return AVC_ERR_WORKSPACE;
    d.amax_a = nullptr;
    if (!d.a_frag && !d.a_guard && d.A && d.A == ctx->xhint.x) {  // (XHintScope: x's producer's words)
      if (ctx->xhint.amax) d.a_guard = ctx->xhint.amax + 1;
      else if (ctx->xhint.unit) d.a_bound = 1.f;
    }
    if (d.a_frag && d.a_frag_guard) {
      d.amax_a = d.a_frag_guard;  // the image's own scale (its producer range-checked A)
    } else if (d.a_guard && !d.a_frag) {
      d.amax_a = d.a_guard;
    } else if (!d.a_frag && !(d.a_bound > 0.f && d.a_bound < 32768.f) && !range_checked(ctx, d.A)) {
      AVC_TRY(guard_scan(ctx, d.A, d.a_rows, d.Kc, d.lda, part, gw, stream));
      d.amax_a = gw;
    }
    if (d.b_frag) {
      d.amax_b = bfrag_guard_word(d, d.b_frag);
    } else if (d.b_conv || (d.ntaps == 1 && d.b_trans && d.ldb == d.Kc)) {
      // a contiguous B (a conv weight, or one [N][K] matrix): the one-launch guard scan (round 5;
      // the same word as guard_init + absmax_b)
      const long n = d.b_conv ? 5L * d.N * d.Kc : (long)d.N * d.Kc;
      AVC_TRY(guard_scan(ctx, d.B, 1, n, n, part, gw + 1, stream));
      d.amax_b = gw + 1;
    } else {
      guard_init_kernel<<<1, 64, 0, stream>>>(gw + 1, 1);
      absmax_b(d, gw + 1, stream);
      d.amax_b = gw + 1;
    }
    d.split_scale = 1;  // the epilogue unscales by 1 / (scale_a * scale_b): exactly 1 in range
  }
  if (frag) {
    // split both operands once into the fragment-major layout gemm16f_kernel streams
    if (scaled_product) {  // power-of-two operand scales from max |A|, max |B| (device side)
      unsigned* amax = zeroed_words(ctx, 2, stream);
      if (!amax) return AVC_ERR_WORKSPACE;
      if (!d.amax_a) {
        if (d.a_trans) absmax2d(d.A, d.Kc, d.M, d.lda, amax, stream);
        else absmax2d(d.A, d.a_rows, d.Kc, d.lda, amax, stream);
        d.amax_a = amax;
      }
      if (!d.amax_b) {
        const long kb = frag16_b_krows(d);
        if (d.b_conv) absmax_b(d, amax + 1, stream);
        else if (d.b_trans) absmax_taps(d.B, d.ntaps, d.b_tapoff, d.N, d.Kc, d.ldb, amax + 1, stream);
        else absmax_taps(d.B, d.ntaps, d.b_tapoff, kb, d.N, d.ldb, amax + 1, stream);
        d.amax_b = amax + 1;
      }
    }
    const long a_src_rows = d.a_trans ? d.M : d.a_rows;
    const long a_ntile = frag_ntile(a_src_rows);
    const int nkc = frag_nkc(d.Kc);
    const long b_ntile = frag_ntile(d.N);
    const long b_krows = frag16_b_krows(d);
    const int b_nkc = frag_nkc((int)b_krows);
    const _Float16* as = d.a_frag;
    // an A split by an earlier product with the same scale (a_frag_out -> a_frag_scaled) is reused
    const bool reuse_a = as && d.a_frag_scaled && scaled_product && d.amax_a;
    if (!reuse_a && (!as || scaled_product || d.a_trans)) {
      _Float16* at = d.a_frag_out ? d.a_frag_out : sc.take<_Float16>(frag_bytes(a_src_rows, d.Kc) / 2);
      if (!at) return AVC_ERR_WORKSPACE;
      const long ta = a_ntile * 32 * nkc * 2;
      split_frag32_kernel<<<(int)std::min<long>((ta + 255) / 256, 8192), 256, 0, stream>>>(
          d.A, d.a_trans ? 1 : d.lda, d.a_trans ? d.lda : 1, (int)a_src_rows, d.Kc, (int)a_ntile, nkc, at, d.amax_a);
      as = at;
    }
    const long tapstride = b_ntile * b_nkc * 1024;  // halves
    const _Float16* bs = (scaled_product && !(d.b_frag_scaled && d.amax_b)) ? nullptr : d.b_frag;
    if (!bs) {
      _Float16* tmp = sc.take<_Float16>((size_t)d.ntaps * frag_bytes(d.N, (int)b_krows) / 2);
      if (!tmp) return AVC_ERR_WORKSPACE;
      split_b(d, (int)b_krows, b_ntile, b_nkc, tmp, tapstride, d.amax_b, stream);
      bs = tmp;
    }
    AVC_LAUNCH_CHECK();
    fa.As = as; fa.a_ntile = (int)a_ntile; fa.a_nkc = nkc;
    fa.a_shift0 = d.a_shift0; fa.a_tapshift = d.a_tapshift;
    fa.Bs = bs; fa.b_ntile = (int)b_ntile; fa.b_nkc = b_nkc; fa.b_tapstride = tapstride;
    fa.b_shift0_c = (int)(d.b_shift0 / 16); fa.b_zshift_c = (int)(d.b_zshift / 16);
  }
  const bool staged16 = !frag && d.prec16 && !scaled_product && !d.a_trans && g_gemm16;
  if (staged16) {  // forward product on the staged-split kernel: the same range guard
    unsigned* gw = sc.take<unsigned>(64);
    float* part = sc.take<float>(kGuardBlocks);
    if (!gw || !part) return AVC_ERR_WORKSPACE;
    d.amax_a = nullptr;
    if (d.a_guard) {
      d.amax_a = d.a_guard;
    } else if (!(d.a_bound > 0.f && d.a_bound < 32768.f) && !range_checked(ctx, d.A)) {
      AVC_TRY(guard_scan(ctx, d.A, d.a_rows, d.Kc, d.lda, part, gw, stream));
      d.amax_a = gw;
    }
    guard_init_kernel<<<1, 64, 0, stream>>>(gw + 1, 1);
    absmax_b(d, gw + 1, stream);
    d.amax_b = gw + 1;
    d.split_scale = 1;
  }
  AVC_CHECK_ARG(!d.bnf.on || (frag && p.nsplit == 1 && p.bm == p.bn && (p.bm == 64 || g_gemm_cfg == 8) &&
                              (d.stats != nullptr) == (d.bnf.training != 0)),
                "gemm: fused BatchNorm requested for a product that cannot take it (gemm_bnf_ok)");
  hipEvent_t ev = timing_begin(TC_GEMM, stream);
  if (frag && d.bnf.on) {
    const int rc = launch16f_bnf(ctx, d, fa, p, stream);
    if (rc != AVC_OK) return rc;
  } else if (frag) {
    if (p.bm == 128) launch16f_128(d, fa, p, slab, stream);
    else launch16f_cfg<64, 64, 2, 2, 4, 2>(d, fa, p, slab, stream);
  } else if (staged16) {
    if (p.bm == 128) launch16<128, 128, 4, 2>(d, p, slab, stream);
    else launch16<64, 64, 2, 2>(d, p, slab, stream);
  } else if (p.bm == 128) {
    launch<128, 128, 2, 4>(d, p, slab, stream);
  } else {
    launch<64, 64, 2, 2>(d, p, slab, stream);
  }
  AVC_LAUNCH_CHECK();
  if (ev) {
    const double flops = 2.0 * d.M * d.N * (double)d.Kc * d.ntaps * d.nz;
    const double bytes = 4.0 * ((double)d.M * d.Kc * d.ntaps + (double)d.Kc * d.N * d.ntaps + (double)d.M * d.N) * d.nz;
    timing_end(TC_GEMM, ev, stream, flops, bytes);
  }
  if (p.nsplit > 1) {
    const long total = (long)d.nz * d.M * d.N;
    const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
    if (d.nz == 1 && d.ldc_col == 1 && d.N % 4 == 0 && d.ldc % 4 == 0 && aligned16(d.C)) {
      const int n4 = d.N / 4;
      int rpb = std::max(1, 1024 / n4);  // ~4 float4 per thread
      if ((d.M + rpb - 1) / rpb < 256 && n4 <= 128) {
        // too few row chunks to fill the chip: one row chunk per block, K-splits across threads
        rpb = std::max(1, std::min(256 / n4, d.M / 256));
        int G = 1;
        while (2 * G * rpb * n4 <= 256 && 2 * G <= p.nsplit) G *= 2;
        splitk_reduce4g_kernel<<<dim3(1, (d.M + rpb - 1) / rpb), 256, 0, stream>>>(d, p.nsplit, slab, rpb, G);
      } else {
        splitk_reduce4_kernel<<<dim3(1, (d.M + rpb - 1) / rpb), 256, 0, stream>>>(d, p.nsplit, slab, rpb);
      }
    } else {
      splitk_reduce_kernel<<<blocks, 256, 0, stream>>>(d, p.nsplit, slab);
    }
    AVC_LAUNCH_CHECK();
  }
  return AVC_OK;
}

}  // namespace avc

extern "C" int avc_gemm_tune(int mode) {
  if (mode < 0 || mode > 3) {
    avc::set_error("avc_gemm_tune: mode must be 0..3");
    return AVC_ERR_INVALID;
  }
  avc::g_gemm16 = mode;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_gemm_config(int cfg) {
  if (cfg < 0 || cfg > 11) {
    avc::set_error("avc_gemm_config: cfg must be 0..11");
    return AVC_ERR_INVALID;
  }
  avc::g_gemm_cfg = cfg;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_gemm_plan_rounds(int on) {
  if (on != 0 && on != 1) {
    avc::set_error("avc_gemm_plan_rounds: 0 or 1");
    return AVC_ERR_INVALID;
  }
  avc::g_plan_rounds = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_bn_fuse_band(int on) {
  if (on != 0 && on != 1) {
    avc::set_error("avc_bn_fuse_band: on must be 0 or 1");
    return AVC_ERR_INVALID;
  }
  avc::g_bnf_band = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_bn_fuse(int on) {
  if (on < 0 || on > 2) {
    avc::set_error("avc_bn_fuse: on must be 0, 1 or 2");
    return AVC_ERR_INVALID;
  }
  avc::g_bnf = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}

#ifdef AVC_GEMM_EPI_STAMPS
extern "C" int avc_debug_epi_stamps(unsigned long long* host) {  // (diagnostic build) [1024][10]
  AVC_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(avc::g_epi_st), sizeof(avc::g_epi_st), 0, hipMemcpyDeviceToHost));
  return AVC_OK;
}
#endif

extern "C" int avc_debug_bnf_inject(int launches) {
  if (launches < 0) {
    avc::set_error("avc_debug_bnf_inject: launches must be >= 0");
    return AVC_ERR_INVALID;
  }
  avc::g_bnf_inject = launches;
  return AVC_OK;
}
