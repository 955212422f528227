// LSTM forward recurrence on split-fp16 MFMA for gfx950 (decoder lstm1 / lstm2, H >= 64).
//
// Why: one time step of decoder.lstm2 (both layers, B = 64) is a [64 x 3072] . [3072 x 4096]
// product — 1.6 GFLOP against 50 MB of weights.  In fp32 MFMA (64 FLOP/clk/SIMD) that alone is
// >= 10 us per step; worse, with one 16-column tile per workgroup every workgroup re-reads the
// whole h operand, so the per-CU load path (~70 GB/s per CU from L2) was the real limit.
//
// What:
//   * "3xf16" products: every operand x (pre-scaled by a power of two) is stored as
//     hi = f16(x), lo = f16(x - hi) and a dot product is accumulated in fp32 by
//     v_mfma_f32_16x16x32_f16 as hi.hi + hi.lo + lo.hi (16x the fp32 MFMA rate per product, 3
//     products).  hi+lo carries 22 significant bits; the dropped lo.lo term is 2^-22 relative;
//     both are below the fp32 accumulation error of a K = 1024..2048 chain.
//     Weights are scaled per gate row so |w| < 2^15, h (|h| < 1) by 2^15: no fp16 overflow and no
//     subnormal lo terms that matter.  Unscaling is one multiply per gate in the epilogue.
//   * tile = 64 batch rows x 64 gate rows (16 hidden units x 4 gates) per workgroup, so h is
//     re-read 4H/64 times instead of 4H/16; the K range is split over the workgroup's 4 waves
//     (LDS reduction) and over `nks` workgroups, whose fp32 slabs the last-arriving workgroup
//     sums in a fixed order (write-through `sc1` slab stores, agent-scope ticket, `sc1` slab
//     loads: cdna_hip_programming.md, in-launch split-K reduction) before running the gate
//     epilogue.  Deterministic: the sum order never depends on arrival order.
//
// Split operands are stored FRAGMENT-MAJOR: for every 16-row tile t and 32-deep chunk c of a
// [rows][K] matrix, two 1 KiB blocks (hi, then lo) hold exactly what the 64 lanes of a
// v_mfma_f32_16x16x32_f16 operand load: lane l = r + 16q gets row 16t + r, k = 32c + 8q .. +7
// (8 halves, 16 B).  Block (t, c, hl) starts at ((t*nck + c)*2 + hl) KiB, nck = K/32.  Every
// operand load is then one contiguous 1 KiB wave instruction (8 full 128-B lines) instead of a
// 16-row x 64-B "fragment-shaped" gather, which ran the per-CU load path at ~11 B/cycle.
#include <algorithm>

#include "kernels.h"
#include "timing.h"

namespace avc {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#ifdef AVC_STAMPS
__device__ unsigned long long* g_sstamps = nullptr;
#define AVC_STAMP(slot)                                                                           \
  do {                                                                                            \
    unsigned long long _t;                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (g_sstamps && lane == 0) {                                                                 \
      const long wid = ((long)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + w;       \
      if (wid < 65536) g_sstamps[wid * 8 + (slot)] = _t;                                          \
    }                                                                                             \
  } while (0)
#else
#define AVC_STAMP(slot) do { } while (0)
#endif

constexpr float kHScale = 32768.0f;           // h is stored as h * 2^15
constexpr float kHUnscale = 1.0f / 32768.0f;

__host__ __device__ __forceinline__ int perm_to_orig(int p, int H) {
  const int blk = p >> 4, g = (p >> 2) & 3, u = p & 3;
  return g * H + blk * 4 + u;
}

__device__ __forceinline__ void split16(float v, _Float16& hi, _Float16& lo) {
  hi = (_Float16)v;
  lo = (_Float16)(v - (float)hi);
}

// Split rows of a weight matrix: dst row p (of R = 4H, permuted gate order when perm != 0) is
// [A[src(p)][0:Da] | Bm[src(p)][0:Db]] scaled by 2^(15 - e), e = exponent of the row's max |w|;
// winv[p] = 2^(e - 15) * 2^-15 undoes both scalings.  One workgroup per row.
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ A, int Da,
                                                         const float* __restrict__ Bm, int Db,
                                                         int H, int perm,
                                                         _Float16* __restrict__ dst,
                                                         float* __restrict__ winv, int Kp = 0) {
  const int p = blockIdx.x, tid = threadIdx.x;
  const int o = perm ? perm_to_orig(p, H) : p;
  const int K = Da + Db;
  if (Kp < K) Kp = K;  // columns [K, Kp) are written as zeros (K padded to whole chunks per wave)
  const float* ra = A + (long)o * Da;
  const float* rb = Bm ? Bm + (long)o * Db : nullptr;
  float m = 0.f;
  for (int k = tid; k < K; k += 256) m = fmaxf(m, fabsf(k < Da ? ra[k] : rb[k - Da]));
  __shared__ float red[256];
  red[tid] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] = fmaxf(red[tid], red[tid + s]);
    __syncthreads();
  }
  int e = 0;
  if (red[0] > 0.f) (void)frexpf(red[0], &e);  // max < 2^e
  const float sc = ldexpf(1.0f, 15 - e);
  if (tid == 0) winv[p] = ldexpf(1.0f, e - 15) * kHUnscale;
  const int nck = Kp >> 5;
  _Float16* d = dst + (long)(p >> 4) * nck * 1024 + (p & 15) * 8;
  for (int k = tid; k < Kp; k += 256) {
    const float v = k >= K ? 0.f : (k < Da ? ra[k] : rb[k - Da]) * sc;
    _Float16 hi, lo;
    split16(v, hi, lo);
    _Float16* q = d + (k >> 5) * 1024 + ((k & 31) >> 3) * 128 + (k & 7);
    q[0] = hi;
    q[512] = lo;
  }
}

// per-gate-row bias vector in permuted order: dst[p] = a[orig(p)] (+ b[orig(p)])
__global__ void perm_bias_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                 float* __restrict__ dst, int H) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < 4 * H) dst[p] = a[perm_to_orig(p, H)] + (b ? b[perm_to_orig(p, H)] : 0.f);
}

struct SplitSlot {
  int K, K0, kslice, nks, ncb;
  int mode;                            // 0: LSTM step epilogue; 1: projection, h_out[b][p] = acc*winv + gx
  // fragment-major split operands; ld* = 32-deep chunks per 16-row tile of that matrix
  const unsigned char* A; long lda;    // reduction operand, columns [0, K0); ntile 16-row tiles
  const unsigned char* A1; long lda1;  // columns [K0, K); NULL source = zeros
  int ntile;                           // 16-row tiles present in A / A1 (ceil(B/16))
  const unsigned char* W; long ldw;    // weights [4H][K] (permuted gate order)
  const float* winv;                   // [4H] unscale per gate row
  const float* gx; long ldgx;          // input projection (+biases) per batch row; ldgx 0 = shared row
  const float* c_prev;                 // NULL = zero state
  float* c_out;
  float* h_out; long ldh;              // fp32 h (the layer output)
  _Float16* hs_out; long ldhs;         // split h for the next step (fragment-major, H/32 chunks)
  float* gates_out;                    // training: [B][4H] activated gates (permuted order)
  float* slab;                         // [nrb][ncb][nks][64*64] fp32 partials
  int* cnt;                            // [nrb][ncb] tickets, zero before the launch
};

// A launch runs up to three independent slots side by side: workgroups [0, nb[0]) slot 0,
// the next nb[1] slot 1, the last nb[2] slot 2.
struct SplitArgs {
  int B, H;
  int nb[3];
  SplitSlot s[3];
};

// NC = 16-column gate blocks (4 hidden units x 4 gates) per workgroup tile: 4 for the wide
// split-K tiles of decoder.lstm2, 1 for the narrow full-K tiles of lstm1 (no slab hand-off).
template <int NW, int NCH, int NC, int RT>
__global__ __launch_bounds__(NW * 64, 2) void lstm_split_step_kernel(SplitArgs a) {
  constexpr int MB = 16 * RT;      // batch rows per workgroup (RT 16-row tiles)
  constexpr int TW = 16 * NC;      // tile width (gate rows)
  constexpr int RP = TW + 4;       // LDS row stride (floats): conflict-free partial writes
  constexpr int TSZ = MB * TW;     // floats per tile partial
  extern __shared__ float part[];  // [NW][64][RP] + flag
  constexpr int NT = NW * 64;
  constexpr int NPAIR = MB * NC;   // (row, 16-column block) pairs of the tile
  constexpr int PP = (NPAIR + NT - 1) / NT;  // pairs per thread in the epilogue
  // wave index through readfirstlane: the buffer descriptors below must be provably uniform, or
  // hipcc wraps every buffer load in a waterfall loop
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lq = lane >> 4;
  const int bx = blockIdx.x;
  const int L = bx < a.nb[0] ? 0 : (bx < a.nb[0] + a.nb[1] ? 1 : 2);
  const SplitSlot& S = L == 0 ? a.s[0] : (L == 1 ? a.s[1] : a.s[2]);
  const int lb = bx - (L >= 1 ? a.nb[0] : 0) - (L == 2 ? a.nb[1] : 0);
  const int nks = S.nks;
  const int cb = lb / nks, ks = lb - cb * nks;
  const int rb = blockIdx.y;
  const int B = a.B, H = a.H;
  AVC_STAMP(0);

  // Epilogue ownership (wide tiles): thread t handles (row, blk) pairs t + NT*i; a pair's 4 float4
  // columns blk*16 + 4g (gate g, units 0..3) hold all four gates of 4 hidden units.  Its
  // operands are fetched before the MFMA phase so that their latency hides under it.
  f32x4 gxv[PP][4], wiv[PP][4], cpv[PP];
  if constexpr (!(NC == 1 && NW == 4))
#pragma unroll
  for (int i = 0; i < PP; ++i) {
    const int pr = min(tid + NT * i, NPAIR - 1), row = pr / NC, blk = pr % NC;
    const int b = min(rb * MB + row, B - 1);
    const int p0 = cb * TW + blk * 16;
    const float* gxr = S.gx + (long)b * S.ldgx + p0;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      gxv[i][g] = *reinterpret_cast<const f32x4*>(gxr + 4 * g);
      wiv[i][g] = *reinterpret_cast<const f32x4*>(S.winv + p0 + 4 * g);
    }
    // unconditional load (a NULL c_prev reads winv instead and is zeroed after): a conditional
    // load would make hipcc drain vmcnt to 0 at the join, before the MFMA loads are issued
    const bool hasc = S.c_prev != nullptr;
    const float* cpp = hasc ? S.c_prev + (long)b * H + cb * 4 * NC + blk * 4 : S.winv;
    const f32x4 cv = *reinterpret_cast<const f32x4*>(cpp);
    cpv[i] = hasc ? cv : f32x4{0.f, 0.f, 0.f, 0.f};
  }

  f32x4 acc[RT][NC];
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int n = 0; n < NC; ++n) acc[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int kw = NCH * 32;  // == S.kslice / NW (host-checked)
  const int k0 = ks * S.kslice + w * kw;
  const bool second = k0 >= S.K0;
  const unsigned char* src = second ? S.A1 : S.A;
  if (src != nullptr) {
    // buffer loads, one 1 KiB block per wave instruction: the lane offset (lane*16) is the only
    // VGPR; tile / chunk offsets are SGPRs.  Row tiles past ntile fall outside the descriptor's
    // range and read as zero (rows of a partial tile are computed and never stored).
    const long nck = second ? S.lda1 : S.lda;
    const int kc0 = (second ? k0 - S.K0 : k0) >> 5;
    const long hbase = ((long)rb * RT * nck + kc0) * 2048;
    const auto hrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(src) + hbase, 0, (int)((long)S.ntile * nck * 2048 - hbase), 0x00020000);
    const long wbase = ((long)cb * NC * S.ldw + (k0 >> 5)) * 2048;
    const auto wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(S.W) + wbase, 0, (int)(NC * S.ldw * 2048), 0x00020000);
    const int hvo = lane * 16, wvo = lane * 16;
    const int hrow16 = (int)nck * 2048, wrow16 = (int)S.ldw * 2048;

    f16x8 hA[RT][2], wA[NC][2], hB[RT][2], wB[NC][2];
#define AVC_LD(RS, VO, SO) __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(RS, VO, SO, 0))
#define AVC_LOAD(HV, WV, C)                                                                       \
  _Pragma("unroll") for (int r = 0; r < RT; ++r) {                                                \
    HV[r][0] = AVC_LD(hrs, hvo, r * hrow16 + (C) * 2048);                                         \
    HV[r][1] = AVC_LD(hrs, hvo, r * hrow16 + (C) * 2048 + 1024);                                  \
  }                                                                                               \
  _Pragma("unroll") for (int n = 0; n < NC; ++n) {                                                \
    WV[n][0] = AVC_LD(wrs, wvo, n * wrow16 + (C) * 2048);                                         \
    WV[n][1] = AVC_LD(wrs, wvo, n * wrow16 + (C) * 2048 + 1024);                                  \
  }
#define AVC_MFMA(HV, WV)                                                                          \
  _Pragma("unroll") for (int r = 0; r < RT; ++r)                                                  \
    _Pragma("unroll") for (int n = 0; n < NC; ++n) {                                              \
      acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][1], WV[n][0], acc[r][n], 0, 0, 0); \
      acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][0], WV[n][1], acc[r][n], 0, 0, 0); \
      acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][0], WV[n][0], acc[r][n], 0, 0, 0); \
    }
#define AVC_PIN __builtin_amdgcn_sched_barrier(0);
    if constexpr (NC == 1 && NCH <= 4) {
      // narrow tile: every chunk of the wave's K range in flight at once (40 VGPRs per chunk),
      // consumed in issue order under counted waits
      f16x8 hC[NCH][RT][2], wC[NCH][NC][2];
#pragma unroll
      for (int c = 0; c < NCH; ++c) { AVC_LOAD(hC[c], wC[c], c) }
#ifdef AVC_STAMPS
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      AVC_STAMP(1);
#endif
      AVC_PIN
#pragma unroll
      for (int c = 0; c < NCH; ++c) { AVC_MFMA(hC[c], wC[c]) }
    } else {
    // register double buffer, program order pinned (see lstm.hip: the scheduler otherwise sinks
    // the next chunk's loads under the current MFMAs and the waitcnt pass drains to zero)
    AVC_LOAD(hA, wA, 0)
#ifdef AVC_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    AVC_STAMP(1);
#endif
    // fully unrolled (NCH is a template parameter): in a runtime loop hipcc's waitcnt pass
    // merges the two buffers' pending loads at the back edge and waits for the just-issued ones
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c + 1 < NCH) {
        if (c & 1) { AVC_LOAD(hA, wA, c + 1) } else { AVC_LOAD(hB, wB, c + 1) }
      }
      AVC_PIN
      if (c & 1) { AVC_MFMA(hB, wB) } else { AVC_MFMA(hA, wA) }
      AVC_PIN
    }
    }
#undef AVC_PIN
#undef AVC_MFMA
#undef AVC_LOAD
#undef AVC_LD
  }
  AVC_STAMP(2);

  // Narrow tiles (NC = 1, 4 waves): 64 rows x 4 hidden units = 256 cells, one per thread, summed
  // straight from the wave partials (the host never splits K for them).
  if constexpr (NC == 1 && NW == 4) {
    const int row = min(tid >> 2, MB - 1), u = tid & 3;
    const bool live = (tid >> 2) < MB;
    const int b = rb * MB + row;
    const int bc = min(b, B - 1);
    const int p0 = cb * 16 + u;
    const float* gxr = S.gx + (long)bc * S.ldgx + p0;
    float gxs[4], wis[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      gxs[g] = gxr[4 * g];
      wis[g] = S.winv[p0 + 4 * g];
    }
    const int j = cb * 4 + u;
    const bool hasc = S.c_prev != nullptr;
    const float cpl = *(hasc ? S.c_prev + (long)bc * H + j : S.winv);
    const float cp = hasc ? cpl : 0.f;
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int e = 0; e < 4; ++e) part[w * MB * RP + (r * 16 + 4 * lq + e) * RP + l15] = acc[r][0][e];
    __syncthreads();
    AVC_STAMP(3);
    float z[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float v = part[row * RP + 4 * g + u];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) v += part[ww * MB * RP + row * RP + 4 * g + u];
      z[g] = fmaf(v, wis[g], gxs[g]);  // explicit fmas: the persistent kernel forms the same values
    }
    AVC_STAMP(5);
    if (live && b < B) {
      const float ig = gate_sigmoid(z[0]), fg = gate_sigmoid(z[1]), gg = gate_tanh(z[2]), og = gate_sigmoid(z[3]);
      const float cn = fmaf(fg, cp, ig * gg);
      const float hv = og * gate_tanh(cn);
      S.c_out[(long)b * H + j] = cn;
      S.h_out[(long)b * S.ldh + j] = hv;
      if (S.hs_out) {
        _Float16 hi, lo;
        split16(hv * kHScale, hi, lo);
        _Float16* hs = S.hs_out + ((long)(b >> 4) * S.ldhs + (j >> 5)) * 1024 +
                       ((b & 15) + 16 * ((j & 31) >> 3)) * 8 + (j & 7);
        hs[0] = hi;
        hs[512] = lo;
      }
      if (S.gates_out) {
        float* go = S.gates_out + (long)b * 4 * H + p0;
        go[0] = ig;
        go[4] = fg;
        go[8] = gg;
        go[12] = og;
      }
    }
    AVC_STAMP(6);
    return;
  }

  // wave partials -> LDS; C layout of 16x16: column lane&15, rows 4(lane>>4) + e
  float* mine = part + w * MB * RP;
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int n = 0; n < NC; ++n)
#pragma unroll
      for (int e = 0; e < 4; ++e) mine[(r * 16 + 4 * lq + e) * RP + n * 16 + l15] = acc[r][n][e];
  __syncthreads();

  f32x4 sum[PP][4];
#pragma unroll
  for (int i = 0; i < PP; ++i) {
    const int pr = min(tid + NT * i, NPAIR - 1), row = pr / NC, blk = pr % NC;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int off = row * RP + blk * 16 + 4 * g;
      f32x4 v = *reinterpret_cast<const f32x4*>(part + off);
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) v += *reinterpret_cast<const f32x4*>(part + ww * MB * RP + off);
      sum[i][g] = v;
    }
  }
  AVC_STAMP(3);

  if (nks > 1) {
    // publish this workgroup's slab (write-through), take a ticket; the last one reduces.
    // Slab element (row, col) of split s at s*TSZ + row*TW + col.
    const long tile = (long)rb * S.ncb + cb;
    float* slab0 = S.slab + tile * nks * TSZ;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(slab0, 0, nks * TSZ * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < PP; ++i) {
      const int pr = tid + NT * i, row = pr / NC, blk = pr % NC;
      if (pr >= NPAIR) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, sum[i][g]), rsrc,
                                               (ks * TSZ + row * TW + blk * 16 + 4 * g) * 4, 0, 16 /*sc1*/);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(part + NW * MB * RP);
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(S.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = old;
    }
    __syncthreads();
    AVC_STAMP(4);
    if (*flag != nks - 1) return;
    // fixed order s = 0..nks-1, up to 8 slabs in flight per pass
#pragma unroll
    for (int i = 0; i < PP; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) sum[i][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < nks; s0 += 4) {
      f32x4 v[4][PP][4];
#pragma unroll
      for (int s1 = 0; s1 < 4; ++s1)
#pragma unroll
        for (int i = 0; i < PP; ++i) {
          const int pr = min(tid + NT * i, NPAIR - 1), row = pr / NC, blk = pr % NC;
#pragma unroll
          for (int g = 0; g < 4; ++g)
            v[s1][i][g] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                rsrc, ((s0 + s1) * TSZ + row * TW + blk * 16 + 4 * g) * 4, 0, 16 /*sc1*/));
        }
#pragma unroll
      for (int s1 = 0; s1 < 4; ++s1)
        if (s0 + s1 < nks)
#pragma unroll
          for (int i = 0; i < PP; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) sum[i][g] += v[s1][i][g];
    }
  }
  AVC_STAMP(5);

  if (S.mode == 1) {
    // projection slot: the input product of the next layer, scaled and biased, no gate math
#pragma unroll
    for (int i = 0; i < PP; ++i) {
      const int pr = tid + NT * i, row = pr / NC, blk = pr % NC;
      const int b = rb * MB + row;
      if (pr >= NPAIR || b >= B) continue;
      float* o = S.h_out + (long)b * S.ldh + cb * TW + blk * 16;
#pragma unroll
      for (int g = 0; g < 4; ++g) *reinterpret_cast<f32x4*>(o + 4 * g) = sum[i][g] * wiv[i][g] + gxv[i][g];
    }
    AVC_STAMP(6);
    return;
  }

  // gate epilogue, 4 hidden units per (row, blk) pair
#pragma unroll
  for (int i = 0; i < PP; ++i) {
    const int pr = tid + NT * i, row = pr / NC, blk = pr % NC;
    const int b = rb * MB + row;
    if (pr >= NPAIR || b >= B) continue;
    const int j0 = cb * 4 * NC + blk * 4;
    f32x4 cn, hv, ig, fg, gg, og;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      // hardware exp/rcp gate math with a polynomial tanh near 0 (common.h: gate_tanh): the plain
      // 1 - 2 / (e^2x + 1) form lost ~1e-7 absolute there, which the train-mode postnet amplified
      // past the 1e-4 mel bar.  Explicit fmas so the persistent kernel forms identical values.
      ig[u] = gate_sigmoid(fmaf(sum[i][0][u], wiv[i][0][u], gxv[i][0][u]));
      fg[u] = gate_sigmoid(fmaf(sum[i][1][u], wiv[i][1][u], gxv[i][1][u]));
      gg[u] = gate_tanh(fmaf(sum[i][2][u], wiv[i][2][u], gxv[i][2][u]));
      og[u] = gate_sigmoid(fmaf(sum[i][3][u], wiv[i][3][u], gxv[i][3][u]));
      cn[u] = fmaf(fg[u], cpv[i][u], ig[u] * gg[u]);
      hv[u] = og[u] * gate_tanh(cn[u]);
    }
    *reinterpret_cast<f32x4*>(S.c_out + (long)b * H + j0) = cn;
    *reinterpret_cast<f32x4*>(S.h_out + (long)b * S.ldh + j0) = hv;
    if (S.hs_out) {
      typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
      f16x4 hi, lo;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        _Float16 h1, l1;
        split16(hv[u] * kHScale, h1, l1);
        hi[u] = h1;
        lo[u] = l1;
      }
      _Float16* hs = S.hs_out + ((long)(b >> 4) * S.ldhs + (j0 >> 5)) * 1024 +
                     ((b & 15) + 16 * ((j0 & 31) >> 3)) * 8 + (j0 & 7);
      *reinterpret_cast<f16x4*>(hs) = hi;
      *reinterpret_cast<f16x4*>(hs + 512) = lo;
    }
    if (S.gates_out) {
      float* go = S.gates_out + (long)b * 4 * H + cb * TW + blk * 16;
      *reinterpret_cast<f32x4*>(go) = ig;
      *reinterpret_cast<f32x4*>(go + 4) = fg;
      *reinterpret_cast<f32x4*>(go + 8) = gg;
      *reinterpret_cast<f32x4*>(go + 12) = og;
    }
  }
  AVC_STAMP(6);
}

int g_split_kslice = 0;  // avc_lstm_split_tune() overrides (0 = automatic)
int g_split_nc = 0;
int g_split_rows64 = 0;  // 1: never use 32-row workgroups

// K-slice per workgroup: start at min(K, 1024); halve while the launch has fewer than 128
// workgroups and each wave keeps >= 2 chunks of 32 (measured: scripts/sweep_split.py; the slab
// hand-off costs more than the extra per-CU bytes of a longer K range).
void choose_kslices(int nslots, const int* K, const int* ncb, int nrb, int NW, int* kslice) {
  for (int L = 0; L < nslots; ++L) kslice[L] = std::min(K[L], 1024);
  if (g_split_kslice) {
    for (int L = 0; L < nslots; ++L)
      kslice[L] = std::max(32 * NW, std::min(K[L], g_split_kslice));
  } else {
    for (;;) {
      long wgs = 0;
      for (int L = 0; L < nslots; ++L) wgs += (long)ncb[L] * (K[L] / kslice[L]) * nrb;
      if (wgs >= 128) break;
      bool changed = false;
      for (int L = 0; L < nslots; ++L)
        if (kslice[L] / NW >= 128 && kslice[L] % 2 == 0) { kslice[L] /= 2; changed = true; }
      if (!changed) break;
    }
  }
  // per-wave range: a power-of-two number of 32-deep chunks (1..8), the same for every slot
  int kw = 256;
  for (int L = 0; L < nslots; ++L) kw = std::min(kw, kslice[L] / NW);
  int p2 = 32;
  while (p2 * 2 <= kw) p2 *= 2;
  for (int L = 0; L < nslots; ++L) {
    kslice[L] = p2 * NW;
    while (K[L] % kslice[L] != 0) kslice[L] /= 2;  // K % (64 NW) == 0 ends this at >= 32 NW
  }
  int m = kslice[0];
  for (int L = 1; L < nslots; ++L) m = std::min(m, kslice[L]);
  for (int L = 0; L < nslots; ++L) kslice[L] = m;  // powers of two times 32 NW: m divides every K
}

int pick_nw(int K) { return K % 128 == 0 ? 4 : 2; }

#ifdef AVC_STAMPS
void* g_sstamp_buf = nullptr;
long g_sstamp_target = -1, g_sstamp_count = 0;
#endif

void launch_split(int NW, int NC, int RT, dim3 grid, const SplitArgs& a, hipStream_t s) {
  const size_t lds = (size_t)NW * 16 * RT * (16 * NC + 4) * sizeof(float) + 16;
#ifdef AVC_STAMPS
  const bool rec = g_sstamp_count++ == g_sstamp_target && g_sstamp_buf;
  if (rec) (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sstamps), &g_sstamp_buf, sizeof(void*), 0, hipMemcpyHostToDevice, s);
#endif
  hipEvent_t ev = timing_begin(TC_LSTM_STEP_FWD, s);
  // every active slot uses the same per-wave K range (choose_kslices keeps kslice/NW equal)
  const int first = a.nb[0] > 0 ? 0 : (a.nb[1] > 0 ? 1 : 2);
  const int nch = a.s[first].kslice / NW / 32;
#define AVC_SPLIT_LAUNCH(NWV, NCV, RTV)                                                           \
  switch (nch) {                                                                                  \
    case 1: lstm_split_step_kernel<NWV, 1, NCV, RTV><<<grid, NWV * 64, lds, s>>>(a); break;       \
    case 2: lstm_split_step_kernel<NWV, 2, NCV, RTV><<<grid, NWV * 64, lds, s>>>(a); break;       \
    case 4: lstm_split_step_kernel<NWV, 4, NCV, RTV><<<grid, NWV * 64, lds, s>>>(a); break;       \
    default: lstm_split_step_kernel<NWV, 8, NCV, RTV><<<grid, NWV * 64, lds, s>>>(a); break;      \
  }
  if (NW == 4) {
    if (NC == 4) { AVC_SPLIT_LAUNCH(4, 4, 4) }
    else if (RT == 2) { AVC_SPLIT_LAUNCH(4, 1, 2) }
    else { AVC_SPLIT_LAUNCH(4, 1, 4) }
  } else {
    if (NC == 4) { AVC_SPLIT_LAUNCH(2, 4, 4) } else { AVC_SPLIT_LAUNCH(2, 1, 4) }
  }
#undef AVC_SPLIT_LAUNCH
  if (ev) {
    double flops = 0.0, bytes = 0.0;
    for (int L = 0; L < 3; ++L) {
      if (a.nb[L] == 0) continue;
      const SplitSlot& S = a.s[L];
      const double kk = (S.A ? S.K0 : 0) + (S.A1 ? S.K - S.K0 : 0);
      flops += 2.0 * a.B * kk * 4.0 * a.H;
      // algorithmic bytes: split weights (4 B per element), the split h operand once, the input
      // projection rows, and the fp32 c/h state + split h written (or the projection output)
      bytes += 4.0 * 4.0 * (double)a.H * S.K + 4.0 * a.B * kk;
      if (S.mode == 1) {
        bytes += 4.0 * a.B * 4.0 * a.H;
      } else {
        bytes += (S.ldgx ? 4.0 * a.B * 4.0 * a.H : 0.0) + 4.0 * a.B * a.H * ((S.c_prev ? 1 : 0) + 3);
      }
    }
    timing_end(TC_LSTM_STEP_FWD, ev, s, flops, bytes);
  }
#ifdef AVC_STAMPS
  if (rec) {
    static void* null_ptr = nullptr;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sstamps), &null_ptr, sizeof(void*), 0, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
  }
#endif
}

inline int ew_blocks(long n) { return (int)std::min<long>((n + 255) / 256, 8192); }

inline size_t al(size_t b) { return (b + 255) & ~size_t(255); }

}  // namespace

// Cached split-f16 copy of a (permuted) input-projection weight for the gemm16f path, rebuilt
// when the weight itself was rebuilt this call.
int attach_bfrag(avc_context* ctx, GemmDesc& g, const void* key, bool rebuilt, hipStream_t s) {
  if (ctx->prep_version < 0) return AVC_OK;
  bool fb = true;
  auto* bf = static_cast<_Float16*>(prep_buffer(ctx, PREP_LSTM_WIH_BFRAG, key, nullptr, gemm_bfrag_bytes(g), &fb));
  if (!bf) return AVC_OK;
  if (fb || rebuilt) AVC_TRY(gemm_prepare_bfrag(g, bf, s));
  g.b_frag = bf;
  return AVC_OK;
}

bool lstm_split_supported(int H, int din) { return H % 64 == 0 && din % 4 == 0; }

size_t lstm_split_forward_scratch(int T, int B, int din, int H, int nlayers) {
  const size_t f = sizeof(float);
  const size_t TB = (size_t)T * B;
  const int nrb = (B + 63) / 64;
  size_t s = al(TB * 4 * H * f);                                  // gx
  s += al((size_t)4 * H * din * f) + 2 * al((size_t)4 * H * f);  // permuted W_ih, biases
  s += al((size_t)4 * H * H * 2 * 2) + al((size_t)4 * H * f);    // split W_hh + winv
  if (nlayers == 2) s += 2 * al((size_t)4 * H * H * 2 * 2) + 3 * al((size_t)4 * H * f) + al((size_t)2 * B * 4 * H * f);
  const size_t Bp = (size_t)(B + 15) / 16 * 16;
  s += (size_t)nlayers * (2 * al(Bp * H * 2 * 2) + 2 * al((size_t)B * H * f));  // h splits, c
  // slabs: at most K/128 splits of every 64-column tile, per slot
  s += (size_t)(nlayers + 1) * al((size_t)nrb * (4 * H / 64) * (2 * H / 128 + 1) * 4096 * f);
  s += al((size_t)(T + 2) * 3 * nrb * (4 * H / 64) * sizeof(int));
  if (nlayers == 2 && B <= 64 && (H == 512 || H == 1024)) s += lstm2_persist_scratch(T, B, H, din);
  if (nlayers == 1 && B <= 256 && (H == 512 || H == 1024)) s += lstm1_persist_scratch(T, B, H, din);
  GemmDesc d;
  d.M = (int)TB; d.N = 4 * H; d.Kc = din; d.prec16 = 1;
  return s + gemm_scratch_bytes(d) + 4096;
}

// W_ih split for an input slot of a persistent recurrence (split_rows_kernel layout, K padded with
// zero columns to inproj_kpad(din)), cached per weights version like the other derived weights.
int split_wih(avc_context* ctx, Scratch& sc, const float* w_ih, int H, int din, InProj& ip, hipStream_t s) {
  const int Kp = inproj_kpad(din);
  bool fresh;
  _Float16* ws = prep_or_scratch<_Float16>(ctx, sc, PREP_LSTM_WIH_SPLIT, w_ih, nullptr,
                                           (size_t)4 * H * Kp * 2 + 8 * H, &fresh);
  if (!ws) return AVC_ERR_WORKSPACE;
  float* winv = reinterpret_cast<float*>(ws + (size_t)4 * H * Kp * 2);
  if (fresh) split_rows_kernel<<<4 * H, 256, 0, s>>>(w_ih, din, nullptr, 0, H, 1, ws, winv, Kp);
  AVC_LAUNCH_CHECK();
  ip.w_s = ws;
  ip.winv = winv;
  return AVC_OK;
}

// One layer (lstm.hip: lstm_forward_impl's contract).  x [T*B][din] (ldx), y [T*B][ldy].
int lstm_split_forward_impl(avc_context* ctx, int T, int B, int din, int H, int reverse,
                            const float* x, int ldx, const float* w_ih, const float* w_hh,
                            const float* b_ih, const float* b_hh, float* y, int ldy,
                            float* saved_gates, float* saved_c, hipStream_t s, _Float16* y_frag) {
  AVC_CHECK_ARG(lstm_split_supported(H, din), "lstm split path: H must be a multiple of 32, >= 64");
  Scratch sc(ctx);
  const long TB = (long)T * B;
  AVC_TAKE(gx, float, (size_t)TB * 4 * H, sc);
  bool f_wih, f_b, f_whh;
  float* wih_p = prep_or_scratch<float>(ctx, sc, PREP_LSTM_WIH, w_ih, nullptr, (size_t)4 * H * din, &f_wih);
  float* b_p = prep_or_scratch<float>(ctx, sc, PREP_LSTM_BIAS, b_ih, b_hh, (size_t)4 * H, &f_b);
  // split W_hh (fragment-major, 4H*H*2 halves) followed by its per-row unscale (4H floats)
  _Float16* whh_s = prep_or_scratch<_Float16>(ctx, sc, PREP_LSTM_WHH, w_hh, nullptr,
                                              (size_t)4 * H * H * 2 + 8 * H, &f_whh);
  if (!wih_p || !b_p || !whh_s) return AVC_ERR_WORKSPACE;
  float* winv = reinterpret_cast<float*>(whh_s + (size_t)4 * H * H * 2);
  const int ntile = (B + 15) / 16;
  const long hsz = (long)ntile * 16 * H * 2;  // halves per split-h buffer
  AVC_TAKE(hs, _Float16, (size_t)2 * hsz, sc);
  float* cpp = nullptr;
  if (!saved_c) {
    AVC_TAKE(tmp, float, (size_t)2 * B * H, sc);
    cpp = tmp;
  }
  // W_ih is consumed by the fp32 GEMM in permuted row order: reuse the split kernel's permutation
  // through a plain gather (lstm.hip's permute_rows_kernel lives in that translation unit).
  if (f_whh) split_rows_kernel<<<4 * H, 256, 0, s>>>(w_hh, H, nullptr, 0, H, 1, whh_s, winv);
  if (f_b) perm_bias_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(b_ih, b_hh, b_p, H);
  AVC_LAUNCH_CHECK();
  if (f_wih) AVC_TRY(permute_rows(w_ih, wih_p, H, din, s));  // cached: kept valid for either path
  if (!reverse && ldy == H && lstm1_inproj_eligible(T, B, H, din) && ldx % 4 == 0 && aligned16(x)) {
    // the recurrence and its input projection (an input slot on the CUs the batch groups leave
    // idle) as one weight-stationary launch
    InProj ip{x, (long)ldx, din, nullptr, nullptr, b_p};
    AVC_TRY(split_wih(ctx, sc, w_ih, H, din, ip, s));
    return lstm1_persist_forward(ctx, T, B, H, gx, whh_s, winv, y, saved_gates, saved_c, s, &ip, y_frag);
  }
  GemmDesc g;
  g.M = (int)TB; g.N = 4 * H; g.Kc = din;
  g.A = x; g.lda = ldx; g.a_rows = TB;
  g.b_trans = 1; g.ldb = din; g.B = wih_p; g.bias0 = b_p;
  g.C = gx; g.ldc = 4 * H;
  g.prec16 = 1;
  AVC_TRY(attach_bfrag(ctx, g, w_ih, f_wih, s));
  AVC_TRY(gemm_run(ctx, g, s));
  if (!reverse && ldy == H && lstm1_persist_eligible(T, B, H))  // the recurrence as one launch
    return lstm1_persist_forward(ctx, T, B, H, gx, whh_s, winv, y, saved_gates, saved_c, s, nullptr, y_frag);

  const int NW = pick_nw(H);
  // narrow full-K tiles when they alone fill the chip (no slab hand-off: one memory round trip
  // less per step); otherwise 64-column tiles with the K range split over workgroups
  int NC = (4 * H / 16) * ((B + 63) / 64) >= 96 && H <= 512 ? 1 : 4;
  if (g_split_nc) NC = g_split_nc;
  // narrow tiles: 32-row workgroups when 64-row ones would leave CUs idle (h bytes per CU halve)
  const int RT = (NC == 1 && NW == 4 && (4 * H / 16) * ((B + 63) / 64) < 256 && B > 32 && !g_split_rows64) ? 2 : 4;
  const int nrb = (B + 16 * RT - 1) / (16 * RT);
  const int ncb = 4 * H / (16 * NC);
  int K[1] = {H}, nc[1] = {ncb}, ksl[1];
  if (NC == 1) {  // narrow tiles reduce the whole K range in one workgroup
    ksl[0] = H;
    while ((ksl[0] / NW) > 256 || (ksl[0] / NW) % 32 != 0 || ((ksl[0] / NW / 32) & (ksl[0] / NW / 32 - 1))) ksl[0] /= 2;
  } else {
    choose_kslices(1, K, nc, nrb, NW, ksl);
  }
  const int nks = H / ksl[0];
  float* slab = nullptr;
  int* cnt = nullptr;
  if (nks > 1) {
    AVC_TAKE(sl, float, (size_t)nrb * ncb * nks * 1024 * NC, sc);
    AVC_TAKE(ct, int, (size_t)T * nrb * ncb, sc);
    AVC_TRY(zero_async(ct, sizeof(int) * T * nrb * ncb, s));
    slab = sl;
    cnt = ct;
  }
  dim3 grid(ncb * nks, nrb);
  for (int st = 0; st < T; ++st) {
    const int t = reverse ? T - 1 - st : st;
    const int tp = reverse ? t + 1 : t - 1;
    SplitArgs a{};
    a.B = B; a.H = H; a.nb[0] = (int)grid.x;
    SplitSlot& S = a.s[0];
    S.K = H; S.K0 = H; S.kslice = ksl[0]; S.nks = nks; S.ncb = ncb;
    S.A = st > 0 ? reinterpret_cast<const unsigned char*>(hs + (long)((st - 1) & 1) * hsz) : nullptr;
    S.lda = H / 32;
    S.ntile = ntile;
    S.W = reinterpret_cast<const unsigned char*>(whh_s);
    S.ldw = H / 32;
    S.winv = winv;
    S.gx = gx + (long)t * B * 4 * H;
    S.ldgx = 4L * H;
    if (saved_c) {
      S.c_prev = st > 0 ? saved_c + (long)tp * B * H : nullptr;
      S.c_out = saved_c + (long)t * B * H;
    } else {
      S.c_prev = st > 0 ? cpp + (long)((st - 1) & 1) * B * H : nullptr;
      S.c_out = cpp + (long)(st & 1) * B * H;
    }
    S.h_out = y + (long)t * B * ldy;
    S.ldh = ldy;
    S.hs_out = st < T - 1 ? hs + (long)(st & 1) * hsz : nullptr;
    S.ldhs = H / 32;
    S.gates_out = saved_gates ? saved_gates + (long)t * B * 4 * H : nullptr;
    S.slab = slab;
    S.cnt = cnt ? cnt + (long)st * nrb * ncb : nullptr;
    launch_split(NW, NC, RT, grid, a, s);
  }
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

// Two stacked layers as a three-slot wavefront (lstm.hip: lstm2_forward_impl's contract).  Launch
// st runs, side by side,
//   slot 0: layer 0 at t = st            (h0_{st-1} . W_hh0^T + Gx0[st]),
//   slot 1: layer 1's input product for t = st-1:  Gx1 = h0_{st-1} . W_ih1^T + b_ih1 + b_hh1,
//   slot 2: layer 1 at t = st-2          (h1_{st-3} . W_hh1^T + Gx1[st-2]),
// so 2T recurrent steps take T+2 launches and every slot reduces K = H inside one workgroup
// (no cross-workgroup slab hand-off).
int lstm2_split_forward_impl(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                             const float* const* w0, const float* const* w1, float* y0, float* y1,
                             float* g0, float* c0, float* g1, float* c1, hipStream_t s, _Float16* y1_frag) {
  AVC_CHECK_ARG(lstm_split_supported(H, din), "lstm2 split path: H must be a multiple of 64");
  Scratch sc(ctx);
  const long TB = (long)T * B;
  const int NC = 4;
  const int nrb = (B + 63) / 64, ncb = 4 * H / (16 * NC);
  AVC_TAKE(gx, float, (size_t)TB * 4 * H, sc);
  bool f_wih, f_b0, f_b1, f_w0, f_w1i, f_w1h;
  float* wih_p = prep_or_scratch<float>(ctx, sc, PREP_LSTM_WIH, w0[0], nullptr, (size_t)4 * H * din, &f_wih);
  float* b0_p = prep_or_scratch<float>(ctx, sc, PREP_LSTM_BIAS, w0[2], w0[3], (size_t)4 * H, &f_b0);
  float* b1_p = prep_or_scratch<float>(ctx, sc, PREP_LSTM_BIAS, w1[2], w1[3], (size_t)4 * H, &f_b1);
  const size_t wsz = (size_t)4 * H * H * 2 + 8 * H;  // split weights + per-row unscale
  _Float16* w0_s = prep_or_scratch<_Float16>(ctx, sc, PREP_LSTM_WHH, w0[1], nullptr, wsz, &f_w0);
  _Float16* w1i_s = prep_or_scratch<_Float16>(ctx, sc, PREP_LSTM_WHH, w1[0], nullptr, wsz, &f_w1i);
  _Float16* w1h_s = prep_or_scratch<_Float16>(ctx, sc, PREP_LSTM_WHH, w1[1], nullptr, wsz, &f_w1h);
  if (!wih_p || !b0_p || !b1_p || !w0_s || !w1i_s || !w1h_s) return AVC_ERR_WORKSPACE;
  float* winv0 = reinterpret_cast<float*>(w0_s + (size_t)4 * H * H * 2);
  float* winv1i = reinterpret_cast<float*>(w1i_s + (size_t)4 * H * H * 2);
  float* winv1h = reinterpret_cast<float*>(w1h_s + (size_t)4 * H * H * 2);
  AVC_TAKE(gx1, float, (size_t)2 * B * 4 * H, sc);
  const int ntile = (B + 15) / 16;
  const long hsz = (long)ntile * 16 * H * 2;  // halves per split-h buffer
  AVC_TAKE(hs0, _Float16, (size_t)2 * hsz, sc);
  AVC_TAKE(hs1, _Float16, (size_t)2 * hsz, sc);
  if (f_w0) split_rows_kernel<<<4 * H, 256, 0, s>>>(w0[1], H, nullptr, 0, H, 1, w0_s, winv0);
  if (f_w1i) split_rows_kernel<<<4 * H, 256, 0, s>>>(w1[0], H, nullptr, 0, H, 1, w1i_s, winv1i);
  if (f_w1h) split_rows_kernel<<<4 * H, 256, 0, s>>>(w1[1], H, nullptr, 0, H, 1, w1h_s, winv1h);
  if (f_b0) perm_bias_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(w0[2], w0[3], b0_p, H);
  if (f_b1) perm_bias_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(w1[2], w1[3], b1_p, H);
  AVC_LAUNCH_CHECK();
  if (f_wih) AVC_TRY(permute_rows(w0[0], wih_p, H, din, s));  // cached: kept valid for either path
  if (lstm2_inproj_eligible(T, B, H, din) && ldx % 4 == 0 && aligned16(x)) {
    // the whole recurrence AND layer 0's input projection as one weight-stationary launch: the
    // projection runs per time step on the CUs the recurrence leaves idle (slot 3)
    InProj ip{x, (long)ldx, din, nullptr, nullptr, b0_p};
    AVC_TRY(split_wih(ctx, sc, w0[0], H, din, ip, s));
    return lstm2_persist_forward(ctx, T, B, H, gx, w0_s, winv0, w1i_s, winv1i, w1h_s, winv1h, b1_p,
                                 y0, y1, g0, c0, g1, c1, s, &ip, y1_frag);
  }
  GemmDesc g;
  g.M = (int)TB; g.N = 4 * H; g.Kc = din;
  g.A = x; g.lda = ldx; g.a_rows = TB;
  g.b_trans = 1; g.ldb = din; g.B = wih_p; g.bias0 = b0_p;
  g.C = gx; g.ldc = 4 * H;
  g.prec16 = 1;
  AVC_TRY(attach_bfrag(ctx, g, w0[0], f_wih, s));
  AVC_TRY(gemm_run(ctx, g, s));
  if (lstm2_persist_eligible(T, B, H))  // the whole recurrence as one weight-stationary launch
    return lstm2_persist_forward(ctx, T, B, H, gx, w0_s, winv0, w1i_s, winv1i, w1h_s, winv1h, b1_p,
                                 y0, y1, g0, c0, g1, c1, s, nullptr, y1_frag);

  float* cpp0 = nullptr;
  float* cpp1 = nullptr;
  if (!c0) {
    AVC_TAKE(tmp, float, (size_t)4 * B * H, sc);
    cpp0 = tmp;
    cpp1 = tmp + 2L * B * H;
  }
  const int NW = pick_nw(H);
  int K[1] = {H}, nc[1] = {3 * ncb}, ksl[1];
  choose_kslices(1, K, nc, nrb, NW, ksl);
  const int nks = H / ksl[0];
  float* slab[3] = {nullptr, nullptr, nullptr};
  int* cnt = nullptr;
  const long cstride = 3L * nrb * ncb;
  if (nks > 1) {
    for (int L = 0; L < 3; ++L) {
      AVC_TAKE(sl, float, (size_t)nrb * ncb * nks * 1024 * NC, sc);
      slab[L] = sl;
    }
    AVC_TAKE(ct, int, (size_t)(T + 2) * cstride, sc);
    AVC_TRY(zero_async(ct, sizeof(int) * (T + 2) * cstride, s));
    cnt = ct;
  }
  auto hs0p = [&](int t) { return hs0 + (long)(t & 1) * hsz; };
  auto hs1p = [&](int t) { return hs1 + (long)(t & 1) * hsz; };
  auto fill = [&](SplitSlot& S, int L, int st) {
    S.K = H; S.K0 = H; S.kslice = ksl[0]; S.nks = nks; S.ncb = ncb;
    S.lda = H / 32; S.ntile = ntile; S.ldw = H / 32; S.ldhs = H / 32;
    S.slab = slab[L];
    S.cnt = cnt ? cnt + (long)st * cstride + (long)L * nrb * ncb : nullptr;
  };
  const int nbl = ncb * nks;
  for (int st = 0; st <= T + 1; ++st) {
    SplitArgs a{};
    a.B = B; a.H = H;
    // slot 0: layer 0 at t0 = st
    const int t0 = st;
    if (t0 < T) {
      SplitSlot& S = a.s[0];
      fill(S, 0, st);
      S.mode = 0;
      S.A = t0 > 0 ? reinterpret_cast<const unsigned char*>(hs0p(t0 - 1)) : nullptr;
      S.W = reinterpret_cast<const unsigned char*>(w0_s);
      S.winv = winv0;
      S.gx = gx + (long)t0 * B * 4 * H;
      S.ldgx = 4L * H;
      if (c0) {
        S.c_prev = t0 > 0 ? c0 + (long)(t0 - 1) * B * H : nullptr;
        S.c_out = c0 + (long)t0 * B * H;
      } else {
        S.c_prev = t0 > 0 ? cpp0 + (long)((t0 - 1) & 1) * B * H : nullptr;
        S.c_out = cpp0 + (long)(t0 & 1) * B * H;
      }
      S.h_out = y0 + (long)t0 * B * H;
      S.ldh = H;
      S.hs_out = hs0p(t0);
      S.gates_out = g0 ? g0 + (long)t0 * B * 4 * H : nullptr;
      a.nb[0] = nbl;
    }
    // slot 1: layer-1 input product for tp = st - 1
    const int tp = st - 1;
    if (tp >= 0 && tp < T) {
      SplitSlot& S = a.s[1];
      fill(S, 1, st);
      S.mode = 1;
      S.A = reinterpret_cast<const unsigned char*>(hs0p(tp));
      S.W = reinterpret_cast<const unsigned char*>(w1i_s);
      S.winv = winv1i;
      S.gx = b1_p;
      S.ldgx = 0;
      S.h_out = gx1 + (long)(tp & 1) * B * 4 * H;
      S.ldh = 4L * H;
      a.nb[1] = nbl;
    }
    // slot 2: layer 1 at t1 = st - 2
    const int t1 = st - 2;
    if (t1 >= 0 && t1 < T) {
      SplitSlot& S = a.s[2];
      fill(S, 2, st);
      S.mode = 0;
      S.A = t1 > 0 ? reinterpret_cast<const unsigned char*>(hs1p(t1 - 1)) : nullptr;
      S.W = reinterpret_cast<const unsigned char*>(w1h_s);
      S.winv = winv1h;
      S.gx = gx1 + (long)(t1 & 1) * B * 4 * H;
      S.ldgx = 4L * H;
      if (c1) {
        S.c_prev = t1 > 0 ? c1 + (long)(t1 - 1) * B * H : nullptr;
        S.c_out = c1 + (long)t1 * B * H;
      } else {
        S.c_prev = t1 > 0 ? cpp1 + (long)((t1 - 1) & 1) * B * H : nullptr;
        S.c_out = cpp1 + (long)(t1 & 1) * B * H;
      }
      S.h_out = y1 + (long)t1 * B * H;
      S.ldh = H;
      S.hs_out = t1 < T - 1 ? hs1p(t1) : nullptr;
      S.gates_out = g1 ? g1 + (long)t1 * B * 4 * H : nullptr;
      a.nb[2] = nbl;
    }
    launch_split(NW, NC, 4, dim3(a.nb[0] + a.nb[1] + a.nb[2], nrb), a, s);
  }
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

}  // namespace avc

#ifdef AVC_STAMPS
extern "C" int avc_debug_stamps_split(void* buf, long target_launch) {
  avc::g_sstamp_buf = buf;
  avc::g_sstamp_target = target_launch;
  avc::g_sstamp_count = 0;
  return AVC_OK;
}
#endif

extern "C" int avc_lstm_split_tune(int kslice, int col_blocks, int rows64) {
  if (kslice < 0 || kslice % 32 != 0) {
    avc::set_error("avc_lstm_split_tune: kslice must be a non-negative multiple of 32");
    return AVC_ERR_INVALID;
  }
  if (!(col_blocks == 0 || col_blocks == 1 || col_blocks == 4)) {
    avc::set_error("avc_lstm_split_tune: col_blocks must be 0, 1 or 4");
    return AVC_ERR_INVALID;
  }
  avc::g_split_kslice = kslice;
  ++avc::g_config_epoch;
  avc::g_split_nc = col_blocks;
  avc::g_split_rows64 = rows64 ? 1 : 0;
  return AVC_OK;
}
