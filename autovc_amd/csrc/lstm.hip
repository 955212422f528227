// LSTM layer forward / backward-through-time for gfx950.
//
// Gate math follows nn.LSTM (gates i,f,g,o; c' = f*c + i*g; h' = o*tanh(c'); zero initial
// state) as used by the reference at encoder.py:51, decoder.py:37 and decoder.py:53.
//
// Large H (512, 1024 — decoder lstm1/lstm2):
//   * the input projection for all T steps is one MFMA GEMM (gemm.hip) into Gx [T*B][4H];
//   * each time step is ONE fused launch: the recurrent product h_{t-1} . W_hh^T on fp32 MFMA
//     (16x16x4, the K range split over the block's waves, reduced through LDS) with the gate
//     nonlinearities and the c/h update in the epilogue.  To let one block own complete gate
//     quadruples, W_hh/W_ih rows are permuted so that gate-columns of 4 hidden units are
//     adjacent: permuted p = blk*16 + gate*4 + u  <->  PyTorch row gate*H + blk*4 + u.
//   * backward: one fused launch per step computes dh_rec = dG_{t+1} . W_hh (MFMA, W_hh^T
//     permuted copy) and the gate/cell gradients; weight gradients are three GEMMs over all
//     steps afterwards.
// Small H (32 — encoder BiLSTM): one single-wave workgroup per (utterance, direction) walks
//   all T steps with W_hh held in registers and h broadcast through LDS (latency-bound path).
#include <mutex>
#include <algorithm>

#include "kernels.h"
#include "timing.h"

namespace avc {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Diagnostic build only (-DAVC_STAMPS): per-wave s_memtime stamps at phase boundaries of the
// step kernel, written to a debug buffer nothing else reads.  The shipped build has none.
#ifdef AVC_STAMPS
__device__ unsigned long long* g_stamps = nullptr;
#define AVC_STAMP(slot)                                                                           \
  do {                                                                                            \
    unsigned long long _t;                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (g_stamps && lane == 0) {                                                                  \
      const long wid = ((long)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + w;       \
      if (wid < 65536) g_stamps[wid * 8 + (slot)] = _t;                                           \
    }                                                                                             \
  } while (0)
#else
#define AVC_STAMP(slot) do { } while (0)
#endif

__host__ __device__ __forceinline__ int perm_to_orig(int p, int H) {
  const int blk = p >> 4, g = (p >> 2) & 3, u = p & 3;
  return g * H + blk * 4 + u;
}

__global__ void permute_rows_kernel(const float* __restrict__ src, float* __restrict__ dst, int H,
                                    int D) {
  const long total = 4L * H * D;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int p = (int)(idx / D);
    const int c = (int)(idx - (long)p * D);
    dst[idx] = src[(long)perm_to_orig(p, H) * D + c];
  }
}

// dst[p][0:Da] = A[orig(p)][:], dst[p][Da:Da+Db] = Bm[orig(p)][:]   (4H rows)
__global__ void permute_concat_kernel(const float* __restrict__ A, int Da, const float* __restrict__ Bm,
                                      int Db, float* __restrict__ dst, int H) {
  const int D = Da + Db;
  const long total = 4L * H * D;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int p = (int)(idx / D);
    const int c = (int)(idx - (long)p * D);
    const long o = perm_to_orig(p, H);
    dst[idx] = c < Da ? A[o * Da + c] : Bm[o * Db + (c - Da)];
  }
}

// dst[p] = a[orig(p)] + b[orig(p)]
__global__ void permute_vec_sum_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                       float* __restrict__ dst, int H) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < 4 * H) dst[p] = a[perm_to_orig(p, H)] + b[perm_to_orig(p, H)];
}

__global__ void permute_vec_kernel(const float* __restrict__ src, float* __restrict__ dst, int H) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < 4 * H) dst[p] = src[perm_to_orig(p, H)];
}

// WT[j][p] = W[orig(p)][j]  (W: [4H][H] PyTorch layout -> [H][4H] permuted, K-contiguous for
// the backward recurrent product).  32x32 LDS-tiled transpose.
__global__ void transpose_permute_kernel(const float* __restrict__ W, float* __restrict__ WT, int H) {
  __shared__ float tile[32][33];
  const int p0 = blockIdx.x * 32, j0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: ty 0..7
  for (int r = ty; r < 32; r += 8) {
    const int p = p0 + r;
    tile[r][tx] = W[(long)perm_to_orig(p, H) * H + j0 + tx];
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) WT[(long)(j0 + r) * 4 * H + p0 + tx] = tile[tx][r];
}

// W_hh [4H][H] -> W_hh^T fragment-major for the BPTT product (StepArgs::frag): row j (hidden
// unit), k = permuted gate row p; block (j>>4, p>>4), lane (j&15) + 16((p&15)>>2), element p&3.
__global__ void whhT_frag_kernel(const float* __restrict__ W, float* __restrict__ dst, int H) {
  const long total = 4L * H * H;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int e = (int)(idx & 3), lane = (int)((idx >> 2) & 63);
    const long blk = idx >> 8;
    const int nkc = H >> 2;  // 16-k chunks of 4H
    const int ct = (int)(blk / nkc), c = (int)(blk - (long)ct * nkc);
    const int j = ct * 16 + (lane & 15);
    const int p = c * 16 + 4 * (lane >> 4) + e;
    dst[idx] = W[(long)perm_to_orig(p, H) * H + j];
  }
}

// dst[orig(p)][:] (+)= src[p][:]
__global__ void unpermute_rows_kernel(const float* __restrict__ src, float* __restrict__ dst, int H,
                                      int D, int accumulate) {
  const long total = 4L * H * D;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const int p = (int)(idx / D);
    const int c = (int)(idx - (long)p * D);
    float* o = dst + (long)perm_to_orig(p, H) * D + c;
    if (accumulate) *o += src[idx]; else *o = src[idx];
  }
}

__global__ void unpermute_vec2_kernel(const float* __restrict__ src, float* __restrict__ d0,
                                      float* __restrict__ d1, int H, int accumulate) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= 4 * H) return;
  const int o = perm_to_orig(p, H);
  if (accumulate) {
    if (d0) d0[o] += src[p];
    if (d1) d1[o] += src[p];
  } else {
    if (d0) d0[o] = src[p];
    if (d1) d1[o] = src[p];
  }
}

// Per-launch arguments.  A launch may run two independent recurrences side by side (the two
// stacked layers of decoder.lstm2, layer 1 one step behind layer 0): blocks [0, nblk0) run
// layer slot 0, the rest slot 1.  The reduction operand of slot L is the concatenation of A[L]
// (columns [0, K0[L])) and A1[L] (columns [K0[L], K[L])); a NULL source contributes zero.
struct StepArgs {
  int B, H, nblk0;
  int K[2], kw[2], K0[2];
  const float* A[2]; long lda[2];
  const float* A1[2]; long lda1[2];
  const float* W[2];   // [ncols][K] K-contiguous rows (permuted gate order)
  // forward
  const float* gx[2]; long ldgx[2];   // per-row input projection (+biases); ldgx 0 = one shared row
  const float* c_prev[2]; float* c_out[2]; float* h_out[2]; long ldh_out[2]; float* gates_out[2];
  // backward (slot 0 only)
  const float* dy; long lddy; const float* gates; const float* c_cur; const float* c_prv;
  float* dc; float* dg_out;
  // BPTT operands fragment-major (frag = 1): A[0] (dG of the later step) and W[0] (W_hh^T) in
  // 1 KiB blocks of 16 rows x 16 k, lane l = r + 16q holding row r, k = 4q..4q+3; lda[0] = 16-k
  // chunks per 16-row tile.  One wave load is then one contiguous 1 KiB (full cache lines).
  int frag;
  float* dgf_out;  // the step's dG in that layout (input of the next BPTT step)
};

template <int MB, bool BWD, int CPT>
__global__ __launch_bounds__(512) void lstm_step_kernel(StepArgs a) {
  constexpr int RT = MB / 16;
  // 16-deep k-chunks loaded per batch; fewer for the 64-row tile to stay within 128 VGPRs
  constexpr int G = MB == 64 ? 2 : 4;

  extern __shared__ float part[];  // [NW][MB][16]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, NW = blockDim.x >> 6;
  const int L = (int)blockIdx.x >= a.nblk0 ? 1 : 0;  // block-uniform layer slot
  AVC_STAMP(0);
  const int cb = blockIdx.x - (L ? a.nblk0 : 0), rb = blockIdx.y;
  const int l15 = lane & 15, lq = lane >> 4;
  // K permutation of one 16*G group: lane quarter q owns k = 4Gq .. 4Gq+4G-1 (G float4, one
  // contiguous 16G-byte run per row, so a wave instruction covers whole cache lines); MFMA
  // (g, e) of the group consumes element e of float4 g on every lane — A and W alike.
  const int lk = 4 * G * lq;

  f32x4 acc0[RT], acc1[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) {
    acc0[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc1[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // Epilogue operands do not depend on the recurrence: fetch them before the MFMA phase so
  // their memory latency overlaps it.  Thread owns cells tid + NT*i (i < CPT).
  const int H = a.H;
  const int NT = blockDim.x;
  const int ncell = BWD ? MB * 16 : MB * 4;
  float pf[CPT][8];
  bool cok[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int cell = tid + NT * i;
    const int row = BWD ? (cell >> 4) : (cell >> 2);
    const int b = rb * MB + row;
    cok[i] = cell < ncell && b < a.B;
    if (!cok[i]) continue;
    if (!BWD) {
      const int u = cell & 3;
      const float* g = a.gx[L] + (long)b * a.ldgx[L] + cb * 16 + u;
      pf[i][0] = g[0];
      pf[i][1] = g[4];
      pf[i][2] = g[8];
      pf[i][3] = g[12];
      pf[i][4] = a.c_prev[L] ? a.c_prev[L][(long)b * H + cb * 4 + u] : 0.f;
    } else {
      const int j = cb * 16 + (cell & 15);
      const long pb = (long)b * 4 * H + (j >> 2) * 16 + (j & 3);
      pf[i][0] = a.gates[pb];
      pf[i][1] = a.gates[pb + 4];
      pf[i][2] = a.gates[pb + 8];
      pf[i][3] = a.gates[pb + 12];
      pf[i][4] = a.c_cur[(long)b * H + j];
      pf[i][5] = a.c_prv ? a.c_prv[(long)b * H + j] : 0.f;
      pf[i][6] = a.dc[(long)b * H + j];
      pf[i][7] = a.dy[(long)b * a.lddy + j];
    }
  }

  const int kw = a.kw[L];
  const int kbeg = w * kw;
  const bool second = kbeg >= a.K0[L];
  const float* src = second ? a.A1[L] : a.A[L];
  if (src != nullptr) {
    const long lds_ = second ? a.lda1[L] : a.lda[L];
    const int koff = second ? kbeg - a.K0[L] : kbeg;
    // element offset of group g at K offset C: base + C*sC + g*sG (row-major: 1 / 4 floats;
    // fragment-major: a 16-k chunk is 256 floats)
    const bool fr = BWD && a.frag;
    const int sC = fr ? 16 : 1, sG = fr ? 256 : 4;
    const float* wrow = fr ? a.W[L] + ((long)cb * (a.K[L] >> 4) + (kbeg >> 4)) * 256 + lane * 4
                           : a.W[L] + (long)(cb * 16 + l15) * a.K[L] + kbeg + lk;
    const float* arow[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int b = rb * MB + r * 16 + l15;
      arow[r] = fr ? src + ((long)(rb * RT + r) * lds_ + (koff >> 4)) * 256 + lane * 4
                   : src + (long)(b < a.B ? b : 0) * lds_ + koff + lk;
    }
    // Register double-buffering: the loads of group g+1 are in flight while group g's MFMAs
    // run (named buffers, unrolled by two, so no register array is indexed at run time).
    // Loads are unconditional (rows >= B read row 0 and are never stored): a per-lane
    // "load or zero" select makes hipcc branch around each load and drain vmcnt to 0,
    // which would serialise the prefetch.
    float4 wA[G], hA[G][RT], wB[G], hB[G][RT];
#define AVC_GROUP_LOAD(WV, HV, C0)                                                               \
  _Pragma("unroll") for (int g = 0; g < G; ++g) {                                               \
    WV[g] = *reinterpret_cast<const float4*>(wrow + (C0) * sC + g * sG);                        \
    _Pragma("unroll") for (int r = 0; r < RT; ++r)                                              \
      HV[g][r] = *reinterpret_cast<const float4*>(arow[r] + (C0) * sC + g * sG);               \
  }
#define AVC_GROUP_MFMA(WV, HV)                                                                   \
  _Pragma("unroll") for (int g = 0; g < G; ++g)                                                 \
    _Pragma("unroll") for (int r = 0; r < RT; ++r) {                                            \
      f32x4& acc = (g & 1) ? acc1[r] : acc0[r];                                                 \
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(HV[g][r].x, WV[g].x, acc, 0, 0, 0);           \
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(HV[g][r].y, WV[g].y, acc, 0, 0, 0);           \
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(HV[g][r].z, WV[g].z, acc, 0, 0, 0);           \
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(HV[g][r].w, WV[g].w, acc, 0, 0, 0);           \
    }
    constexpr int GK = 16 * G;
    // Every workgroup reads the same h rows; if all start at k = 0 the CUs of an XCD request the
    // same lines at the same time and queue on one L2 channel.  Rotate the starting group by
    // the workgroup's position within its XCD (block id / 8) so they stream different lines.
    const int ng = kw / GK;
    const int rot = (int)((blockIdx.x >> 3) % (unsigned)ng);
    // running K offset of the next group to load, wrapped at kw (no divisions in the loop)
    int cnext = rot * GK;
#define AVC_NEXT(C) { C = cnext; cnext += GK; cnext = cnext >= kw ? cnext - kw : cnext; }
    // sched_barrier pins the program order below: without it the scheduler sinks the next
    // group's loads under the current MFMAs' consumers and the waitcnt pass drains vmcnt to 0.
#define AVC_PIN __builtin_amdgcn_sched_barrier(0);
    int c;
    AVC_NEXT(c)
    AVC_GROUP_LOAD(wA, hA, c)
#ifdef AVC_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    AVC_STAMP(1);
#endif
    // steady state: one basic block per two groups (no conditional loads, so hipcc can count
    // vmcnt and keep the next group's loads in flight under the current MFMAs)
    int i = 0;
    for (; i + 2 < ng; i += 2) {
      AVC_NEXT(c)
      AVC_GROUP_LOAD(wB, hB, c)
      AVC_PIN
      AVC_GROUP_MFMA(wA, hA)
      AVC_PIN
      AVC_NEXT(c)
      AVC_GROUP_LOAD(wA, hA, c)
      AVC_PIN
      AVC_GROUP_MFMA(wB, hB)
      AVC_PIN
    }
    if (ng - i == 2) {
      AVC_NEXT(c)
      AVC_GROUP_LOAD(wB, hB, c)
      AVC_PIN
      AVC_GROUP_MFMA(wA, hA)
      AVC_PIN
      AVC_GROUP_MFMA(wB, hB)
    } else {
      AVC_GROUP_MFMA(wA, hA)
    }
#undef AVC_PIN
#undef AVC_NEXT
#undef AVC_GROUP_LOAD
#undef AVC_GROUP_MFMA
  }
  AVC_STAMP(2);
  // 16x16 accumulator layout: column = lane&15, rows 4*(lane>>4) + e
#pragma unroll
  for (int r = 0; r < RT; ++r)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      part[(w * MB + r * 16 + 4 * lq + e) * 16 + l15] = acc0[r][e] + acc1[r][e];
  __syncthreads();
  // cross-wave reduction, one (row, column) per thread, fixed order; result in wave-0's slab
  // (each element is read and then overwritten by the same thread only)
  if (NW > 1) {
    for (int idx = tid; idx < MB * 16; idx += blockDim.x) {
      float s = part[idx];
      for (int ww = 1; ww < NW; ++ww) s += part[ww * MB * 16 + idx];
      part[idx] = s;
    }
    __syncthreads();
  }
  AVC_STAMP(3);

  if (!BWD) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      if (!cok[i]) continue;
      const int cell = tid + NT * i;
      const int row = cell >> 2, u = cell & 3;
      const int b = rb * MB + row;
      float z[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) z[g] = pf[i][g] + part[row * 16 + g * 4 + u];
      const float ig = sigmoidf_(z[0]), fg = sigmoidf_(z[1]), gg = tanhf(z[2]), og = sigmoidf_(z[3]);
      const int j = cb * 4 + u;
      const float c = fg * pf[i][4] + ig * gg;
      const float h = og * tanhf(c);
      a.c_out[L][(long)b * H + j] = c;
      a.h_out[L][(long)b * a.ldh_out[L] + j] = h;
      if (a.gates_out[L]) {
        float* go = a.gates_out[L] + (long)b * 4 * H + cb * 16 + u;
        go[0] = ig;
        go[4] = fg;
        go[8] = gg;
        go[12] = og;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      if (!cok[i]) continue;
      const int cell = tid + NT * i;
      const int row = cell >> 4, jj = cell & 15;
      const int b = rb * MB + row;
      const int j = cb * 16 + jj;
      const float dh = pf[i][7] + part[row * 16 + jj];
      const long pb = (long)b * 4 * H + (j >> 2) * 16 + (j & 3);
      const float ig = pf[i][0], fg = pf[i][1], gg = pf[i][2], og = pf[i][3];
      const float c = pf[i][4], cp = pf[i][5];
      const float tc = tanhf(c);
      const float dct = dh * og * (1.f - tc * tc) + pf[i][6];
      a.dc[(long)b * H + j] = dct * fg;
      const float d0 = dct * gg * ig * (1.f - ig), d1 = dct * cp * fg * (1.f - fg);
      const float d2 = dct * ig * (1.f - gg * gg), d3 = dh * tc * og * (1.f - og);
      a.dg_out[pb] = d0;
      a.dg_out[pb + 4] = d1;
      a.dg_out[pb + 8] = d2;
      a.dg_out[pb + 12] = d3;
      if (a.dgf_out) {  // gate g of unit j = permuted column (j>>2)*16 + 4g + (j&3)
        float* f = a.dgf_out + ((long)(b >> 4) * (H >> 2) + (j >> 2)) * 256 + (b & 15) * 4 + (j & 3);
        f[0] = d0;
        f[64] = d1;
        f[128] = d2;
        f[192] = d3;
      }
    }
  }
  AVC_STAMP(4);
}

// ---- BPTT as split-K 3xf16 products + a per-batch-row epilogue ---------------------------
//
// lstm_step_kernel's backward step gives each workgroup 16 hidden units x 64 batch rows over the
// whole K = 4H, so every one of its 256 workgroups re-reads 1 MB of dG per step (320 MB chip-wide,
// intake-bound at ~40 GB/s per CU: 32 us per H = 1024 step at B = 256).  Here one step is
//   1. gemm_frag_partials: slab[s] = dG_{t+1} . W_hh over K-split s, 3xf16 on pre-split operands
//      (128x128 tiles, split-K to ~256 workgroups: ~256 KB of operands per CU);
//   2. bptt_row_kernel (one workgroup per batch row): dh = dy_t + sum_s slab[s] (unscaled),
//      the gate derivatives, dc, the fp32 dG_t row, and dG_t split for the next step's product.
// The split needs a power-of-two operand scale; a product's A rows may be scaled independently
// (diag(s) A W = diag(s) (A W)), so each row b of dG_t is scaled from its own max |dG_t[b, :]|,
// known inside its workgroup, and the next epilogue unscales row b by 1 / (s_b s_w).  W_hh is
// split once per call with the scale of its max |W|.
struct BpttArgs {
  int B, H, nsplit, first, last;
  const float* slab;       // [nsplit][B][H] raw partials (first: unused)
  float* rowscale;         // [B] power-of-two scale of the row's split dG (read, then replaced)
  const unsigned* amax_w;  // max |W_hh| (float bits)
  const float* dy; long lddy;
  const float* gates; const float* c_cur; const float* c_prv;
  float* dc;               // [B][H] carried cell-state gradient
  float* dg_out;           // [B][4H] fp32 dG_t (permuted gate order)
  _Float16* dgs;           // fragment-major split dG_t (rows padded to 32), for the next product
};

__device__ __forceinline__ float pow2_scale(float m) {  // max |x| -> [2^14, 2^15) (split_scale_of)
  if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, 15 - e);
}

template <int UPT, int NS>  // hidden units per thread (H / 256), K-splits of the partial slabs
__global__ __launch_bounds__(256) void bptt_row_kernel(BpttArgs a) {
  constexpr int NT = 256;
  const int H = a.H, G4 = 4 * H, b = blockIdx.x, tid = threadIdx.x;
  extern __shared__ float row[];  // [4H] the dG_t row, permuted order
  __shared__ float red[NT / 64];
  const float unscale = a.first ? 0.f : 1.f / (a.rowscale[b] * pow2_scale(__uint_as_float(*a.amax_w)));
  // every operand of the row first (UPT x NS partials and the epilogue operands in flight
  // together), then the arithmetic; partials summed in split order
  float part[UPT][NS];
#pragma unroll
  for (int m = 0; m < UPT; ++m)
#pragma unroll
    for (int sp = 0; sp < NS; ++sp)
      part[m][sp] = a.first ? 0.f : a.slab[((long)sp * a.B + b) * H + tid + NT * m];
  float mx = 0.f;
#pragma unroll
  for (int m = 0; m < UPT; ++m) {
    const int j = tid + NT * m;
    float rec = 0.f;
#pragma unroll
    for (int sp = 0; sp < NS; ++sp) rec += part[m][sp];
    rec *= unscale;
    const float dh = a.dy[(long)b * a.lddy + j] + rec;
    const long pb = (long)b * G4 + (j >> 2) * 16 + (j & 3);
    const float ig = a.gates[pb], fg = a.gates[pb + 4], gg = a.gates[pb + 8], og = a.gates[pb + 12];
    const float c = a.c_cur[(long)b * H + j], cp = a.c_prv ? a.c_prv[(long)b * H + j] : 0.f;
    const float tc = tanhf(c);
    const float dct = dh * og * (1.f - tc * tc) + a.dc[(long)b * H + j];
    a.dc[(long)b * H + j] = dct * fg;
    const float d0 = dct * gg * ig * (1.f - ig), d1 = dct * cp * fg * (1.f - fg);
    const float d2 = dct * ig * (1.f - gg * gg), d3 = dh * tc * og * (1.f - og);
    const int p = (j >> 2) * 16 + (j & 3);
    row[p] = d0;
    row[p + 4] = d1;
    row[p + 8] = d2;
    row[p + 12] = d3;
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(d0), fabsf(d1)), fmaxf(fabsf(d2), fabsf(d3))));
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  const float sb = pow2_scale(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  // the fp32 row (weight gradients, dX) and, for the next step, its split, both from LDS
  float4* out4 = reinterpret_cast<float4*>(a.dg_out + (long)b * G4);
  for (int q = tid; q < G4 / 4; q += NT) out4[q] = reinterpret_cast<const float4*>(row)[q];
  if (!a.last) {
    const int nkc = G4 / 16;
    for (int g8 = tid; g8 < G4 / 8; g8 += NT) {  // one octet of k per thread (split_frag32 layout)
      typedef _Float16 h8 __attribute__((ext_vector_type(8)));
      h8 hi, lo;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = row[8 * g8 + e] * sb;
        const _Float16 h = (_Float16)v;
        hi[e] = h;
        lo[e] = (_Float16)((v - (float)h) * 2048.0f);
      }
      const long blk = ((long)(b >> 5) * nkc + (g8 >> 1)) * 2;
      const int lane = (b & 31) + 32 * (g8 & 1);
      *reinterpret_cast<h8*>(a.dgs + blk * 512 + lane * 8) = hi;
      *reinterpret_cast<h8*>(a.dgs + (blk + 1) * 512 + lane * 8) = lo;
    }
  }
  __syncthreads();  // every thread read the old row scale before it is replaced
  if (tid == 0) a.rowscale[b] = sb;
}

int g_bptt_mode = 1;  // avc_bptt_mode(): 0 = step kernel, 1 = split-K products where faster (H = 1024), 2 = wherever eligible

struct StepCfg {
  int mb, nw;
};

int g_force_mb = 0, g_force_nw = 0;  // avc_lstm_tune() overrides (0 = automatic)

StepCfg step_cfg(int B, int ncolblocks, int K) {
  StepCfg c;
  if (B <= 16) c.mb = 16;
  else if ((long)ncolblocks * ((B + 63) / 64) >= 240) c.mb = 64;
  else if ((long)ncolblocks * ((B + 31) / 32) >= 240) c.mb = 32;
  else c.mb = 16;
  c.nw = std::max(1, std::min(8, K / 128));
  if (g_force_mb) c.mb = g_force_mb;
  if (g_force_nw) c.nw = std::min(std::min(g_force_nw, 8), std::max(1, K / 64));
  while (K % (c.nw * 64) != 0) --c.nw;
  // the epilogue gives each thread at most 4 cells (16 per row in backward, 4 in forward)
  while (c.mb * 16 > 4 * 64 * c.nw && c.mb > 16) c.mb /= 2;
  return c;
}

int cells_per_thread(const StepCfg& c, bool bwd) {
  const int cells = bwd ? c.mb * 16 : c.mb * 4;
  const int t = c.nw * 64;
  const int cpt = (cells + t - 1) / t;
  return cpt <= 1 ? 1 : (cpt <= 2 ? 2 : 4);
}

#ifdef AVC_STAMPS
void* g_stamp_buf = nullptr;
long g_stamp_target = -1, g_stamp_count = 0;
#endif

void launch_step(const StepCfg& cfg, bool bwd, dim3 grid, const StepArgs& a, hipStream_t s) {
#ifdef AVC_STAMPS
  const bool rec = g_stamp_count++ == g_stamp_target && g_stamp_buf;
  if (rec) (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_stamps), &g_stamp_buf, sizeof(void*), 0, hipMemcpyHostToDevice, s);
#endif
  const size_t lds = (size_t)cfg.nw * cfg.mb * 16 * sizeof(float);
  const int threads = cfg.nw * 64;
  const int cls = bwd ? TC_LSTM_STEP_BWD : TC_LSTM_STEP_FWD;
  hipEvent_t ev = timing_begin(cls, s);
  const int cpt = cells_per_thread(cfg, bwd);
#define AVC_STEP_LAUNCH(MBV, BW)                                                                  \
  if (cpt == 1) lstm_step_kernel<MBV, BW, 1><<<grid, threads, lds, s>>>(a);                       \
  else if (cpt == 2) lstm_step_kernel<MBV, BW, 2><<<grid, threads, lds, s>>>(a);                  \
  else lstm_step_kernel<MBV, BW, 4><<<grid, threads, lds, s>>>(a);
  if (!bwd) {
    if (cfg.mb == 64) { AVC_STEP_LAUNCH(64, false) }
    else if (cfg.mb == 32) { AVC_STEP_LAUNCH(32, false) }
    else { AVC_STEP_LAUNCH(16, false) }
  } else {
    if (cfg.mb == 64) { AVC_STEP_LAUNCH(64, true) }
    else if (cfg.mb == 32) { AVC_STEP_LAUNCH(32, true) }
    else { AVC_STEP_LAUNCH(16, true) }
  }
#undef AVC_STEP_LAUNCH
#ifdef AVC_STAMPS
  if (rec) {
    static void* null_ptr = nullptr;
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_stamps), &null_ptr, sizeof(void*), 0, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
  }
#endif
  if (ev) {
    // recurrent (+ in-step input) product per active slot; weights streamed once per step
    double flops = 0.0, bytes = 0.0;
    const int nslots = a.nblk0 < (int)grid.x ? 2 : 1;
    for (int L = (a.nblk0 == 0 ? 1 : 0); L < nslots; ++L) {
      const double kk = (a.A[L] ? a.K0[L] : 0) + (a.A1[L] ? a.K[L] - a.K0[L] : 0);
      flops += 2.0 * a.B * kk * (bwd ? a.H : 4.0 * a.H);
      bytes += 4.0 * 4.0 * (double)a.H * a.K[L];
    }
    timing_end(cls, ev, s, flops, bytes);
  }
}

// ---- H = 32 persistent single-wave kernels (encoder BiLSTM) ------------------------------

// One direction of an H = 32 layer, as seen by lstm32_fwd_kernel.
struct L32Dir {
  const float* gx;     // [T*B][ldgx] input projection (+biases), this direction's 128 columns
  const float* whh;    // [128][32]
  float* y;            // [T*B][ldy] output, this direction's 32 columns
  float* gates;        // training: [T*B][128] activated gates (or NULL)
  float* c;            // training: [T*B][32] cell states (or NULL)
  int reverse;
};

// Workgroups [0, B) run direction d0, [B, 2B) direction d1 (both directions of a bidirectional
// layer in one launch).  The step is one wave's latency chain (LDS h broadcast -> 32-deep dot
// products -> gate math -> h), so everything else is taken off it: the input projection of step
// s + PF is fetched while step s computes (a register ring of PF steps, the loop unrolled by PF
// so ring slots are static), and FAST selects hardware exp / reciprocal gate math
// (sigma(x) = rcp(1 + 2^(-x log2 e)), tanh(x) = 2 sigma(2x) - 1; within ~1e-7 of the libm forms).
// DIAG (timing experiments only, avc_lstm32_tune 2 / 3; results invalid): 1 = no output stores,
// 2 = no input loads either
template <int PF, bool FAST, int DIAG = 0>
__global__ __launch_bounds__(64) void lstm32_fwd_kernel(int T, int B, long ldgx, long ldy, L32Dir d0,
                                                        L32Dir d1) {
  const int dir = blockIdx.x >= B ? 1 : 0;
  const L32Dir& D = dir ? d1 : d0;
  const int b = blockIdx.x - dir * B, lane = threadIdx.x;
  const float* __restrict__ gx = D.gx;
  const int reverse = D.reverse;
  __shared__ __attribute__((aligned(16))) float hs[64];  // [0, 32) h; [32, 64) lanes 32..63's unused writes
  float w0[32], w1[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    w0[k] = D.whh[lane * 32 + k];
    w1[k] = D.whh[(lane + 64) * 32 + k];
  }
  hs[lane] = 0.f;
  float c = 0.f;
  auto grow = [&](int st) {
    const int sc = st < T ? st : T - 1;
    return ((long)(reverse ? T - 1 - sc : sc) * B + b) * ldgx;
  };
  auto sig = [](float x) {
    if constexpr (FAST) return __builtin_amdgcn_rcpf(1.f + __expf(-x));
    else return sigmoidf_(x);
  };
  auto th = [&](float x) {
    if constexpr (FAST) return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f;
    else return tanhf(x);
  };
  // Outputs as buffer stores, the same number of them on every path (round 5): lanes 32..63 and
  // absent outputs (no c / gates outside training: a zero-sized descriptor) store out of range,
  // which the hardware drops.  Stores under `lane < 32` / `if (D.c)` branches left the compiler's
  // counted waits unable to count them, and the loop's back edge waited for every store (a write
  // drain every PF steps).
  constexpr unsigned kOut = 0x80000000u;
  const long TB = (long)T * B;
  const auto yrs = __builtin_amdgcn_make_buffer_rsrc(D.y, 0, (int)std::min<long>(TB * ldy * 4, 0x7fffffffL), 0x00020000);
  // (launch_lstm32 refuses T * B * 512 >= 2^31; the clamps keep a descriptor from wrapping regardless)
  const auto crs = __builtin_amdgcn_make_buffer_rsrc(D.c, 0, D.c ? (int)std::min<long>(TB * 32 * 4, 0x7fffffffL) : 0, 0x00020000);
  const auto grs = __builtin_amdgcn_make_buffer_rsrc(D.gates, 0, D.gates ? (int)std::min<long>(TB * 128 * 4, 0x7fffffffL) : 0,
                                                     0x00020000);
  const bool lo = lane < 32;
  auto step = [&](int s, float z0, float z1) {
    const int t = reverse ? T - 1 - s : s;
    const long row = (long)t * B + b;
    float a0, a1, fg, og;
    if constexpr (FAST) {
      // packed FMAs (v_pk_fma_f32: two k per instruction), two chains of 8 per gate row
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 q0[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}}, q1[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
      for (int k4 = 0; k4 < 8; ++k4) {
        const float4 h4 = *reinterpret_cast<const float4*>(hs + 4 * k4);
        const f2 ha = {h4.x, h4.y}, hb = {h4.z, h4.w};
        q0[0] = __builtin_elementwise_fma(f2{w0[4 * k4], w0[4 * k4 + 1]}, ha, q0[0]);
        q0[1] = __builtin_elementwise_fma(f2{w0[4 * k4 + 2], w0[4 * k4 + 3]}, hb, q0[1]);
        q1[0] = __builtin_elementwise_fma(f2{w1[4 * k4], w1[4 * k4 + 1]}, ha, q1[0]);
        q1[1] = __builtin_elementwise_fma(f2{w1[4 * k4 + 2], w1[4 * k4 + 3]}, hb, q1[1]);
      }
      const f2 s0 = q0[0] + q0[1], s1 = q1[0] + q1[1];
      z0 += s0.x + s0.y;
      z1 += s1.x + s1.y;
      a0 = sig(z0);                      // i (lane<32) or f
      a1 = lo ? th(z1) : sig(z1);        // g (lane<32) or o
      // lanes 32..63 -> 0..31 with one VALU swap of the wave halves instead of ds_bpermute
      fg = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a0), false, false)[1]);
      og = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(a1), __float_as_uint(a1), false, false)[1]);
    } else {
      // four independent FMA chains per gate row (8 deep instead of 32)
      float p0[4] = {0.f, 0.f, 0.f, 0.f}, p1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k4 = 0; k4 < 8; ++k4) {
        const float4 h4 = *reinterpret_cast<const float4*>(hs + 4 * k4);
        p0[0] = fmaf(w0[4 * k4], h4.x, p0[0]);
        p0[1] = fmaf(w0[4 * k4 + 1], h4.y, p0[1]);
        p0[2] = fmaf(w0[4 * k4 + 2], h4.z, p0[2]);
        p0[3] = fmaf(w0[4 * k4 + 3], h4.w, p0[3]);
        p1[0] = fmaf(w1[4 * k4], h4.x, p1[0]);
        p1[1] = fmaf(w1[4 * k4 + 1], h4.y, p1[1]);
        p1[2] = fmaf(w1[4 * k4 + 2], h4.z, p1[2]);
        p1[3] = fmaf(w1[4 * k4 + 3], h4.w, p1[3]);
      }
      z0 += (p0[0] + p0[1]) + (p0[2] + p0[3]);
      z1 += (p1[0] + p1[1]) + (p1[2] + p1[3]);
      a0 = sig(z0);
      a1 = lo ? th(z1) : sig(z1);
      fg = __shfl(a0, (lane + 32) & 63);
      og = __shfl(a1, (lane + 32) & 63);
    }
    // every lane runs the cell update; only lanes 0..31's values are stored or read back.  (An
    // explicit fma, the form the compiler had chosen here through round 4: left to contraction,
    // f c + i g fused the other way round in the two-wave kernel.)
    c = fmaf(a0, a1, fg * c);
    const float h = og * th(c);
    hs[lane] = h;
    const unsigned oy = lo ? (unsigned)((row * ldy + lane) * 4) : kOut;
    const unsigned oc = lo ? (unsigned)((row * 32 + lane) * 4) : kOut;
    const unsigned og4 = lo ? (unsigned)((row * 128 + lane) * 4) : kOut;
    if constexpr (DIAG == 0) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(h), yrs, oy, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(c), crs, oc, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a0), grs, og4, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fg), grs, lo ? og4 + 128 : kOut, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a1), grs, lo ? og4 + 256 : kOut, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(og), grs, lo ? og4 + 384 : kOut, 0, 0);
    }
    // one wave: LDS operations complete in issue order, so the next step's h reads only need
    // the compiler not to move them above this write.  (__syncthreads() would also wait for
    // every outstanding global load -- the prefetch ring -- and store on every step.)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  float r0[PF], r1[PF];
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    r0[u] = gx[grow(u) + lane];
    r1[u] = gx[grow(u) + lane + 64];
  }
  __syncthreads();
  int s0 = 0;
  for (; s0 + PF <= T; s0 += PF) {
    // the next group's input rows, all requested before this group's steps (round 5): with one
    // refill per step the last refill sat behind only its own step's stores, and the back edge
    // (the ring moves into the next iteration's registers) waited for them all.  Requested first,
    // they are the oldest operations there.  (Unconditional, clamped by grow(): no joins.)
    float n0[PF], n1[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const long rn = grow(s0 + PF + u);
      n0[u] = DIAG == 2 ? 0.f : gx[rn + lane];
      n1[u] = DIAG == 2 ? 0.f : gx[rn + lane + 64];
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) step(s0 + u, r0[u], r1[u]);
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      r0[u] = n0[u];
      r1[u] = n1[u];
    }
  }
  // the last T % PF steps (their rows are the ring's first slots)
#pragma unroll
  for (int u = 0; u < PF - 1; ++u)
    if (s0 + u < T) step(s0 + u, r0[u], r1[u]);
}

// Round 5 (avc_lstm32_tune(1), the default): the same step math, with the memory operations taken
// off the chain.  Wave 0 runs the recurrence touching only LDS and registers: its input rows come
// from an LDS ring and its outputs go to an LDS ring.  Wave 1 fills the input ring one PF-step
// group ahead and stores the previous group's outputs; the two meet at one barrier per group.
// (Priced with avc_lstm32_tune 2 / 3: the one-wave kernel's loads and stores were ~100 of 383 us
// per C5 layer.)  Same expressions, same order: the same bits as lstm32_fwd_kernel<PF, true>.
template <int PF>
__global__ __launch_bounds__(128) void lstm32_fwd2_kernel(int T, int B, long ldgx, long ldy, L32Dir d0,
                                                          L32Dir d1) {
  const int dir = blockIdx.x >= B ? 1 : 0;
  const L32Dir& D = dir ? d1 : d0;
  const int b = blockIdx.x - dir * B;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int reverse = D.reverse;
  // one LDS array: hs [64] | input ring [2][PF][128] | output ring [2][PF][8][32]
  // (output rows: h, c, i, f, g, o, and two rows lanes 32..63's h / c writes land in)
  __shared__ __attribute__((aligned(16))) float lds[64 + 2 * PF * 128 + 2 * PF * 8 * 32];
  float* const hs = lds;
  float* const gxr = lds + 64;
  float* const outr = gxr + 2 * PF * 128;
  auto rowof = [&](int st) { return (long)(reverse ? T - 1 - st : st) * B + b; };
  const int ngroups = (T + PF - 1) / PF;
  // wave 1: input rows of group g into ring slot g & 1 (loads issued by load_issue, written by load_land)
  float2 lv[PF];
  auto load_issue = [&](int g) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int st = min(g * PF + u, T - 1);  // clamped: always issued
      lv[u] = *reinterpret_cast<const float2*>(D.gx + rowof(st) * ldgx + 2 * lane);
    }
  };
  auto load_land = [&](int g) {
#pragma unroll
    for (int u = 0; u < PF; ++u)
      *reinterpret_cast<float2*>(gxr + ((g & 1) * PF + u) * 128 + 2 * lane) = lv[u];
  };
  auto store_group = [&](int g) {  // wave 1: group g's outputs out of ring slot g & 1
    for (int u = 0; u < PF; ++u) {
      const int st = g * PF + u;
      if (st >= T) break;
      const long row = rowof(st);
      const float* o = outr + ((g & 1) * PF + u) * 256;
      if (lane < 32) D.y[row * ldy + lane] = o[lane];
      else if (D.c) D.c[row * 32 + lane - 32] = o[32 + lane - 32];
      if (D.gates) {
        // gate k = 2 lane + e: row 2 + k / 32 of the ring, unit k % 32 (i, f, g, o)
        const int k = 2 * lane;
        *reinterpret_cast<float2*>(D.gates + row * 128 + k) =
            make_float2(o[(2 + k / 32) * 32 + k % 32], o[(2 + k / 32) * 32 + k % 32 + 1]);
      }
    }
  };
  float w0[32], w1[32];
  if (wv == 0) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      w0[k] = D.whh[lane * 32 + k];
      w1[k] = D.whh[(lane + 64) * 32 + k];
    }
    hs[lane] = 0.f;
  } else {
    load_issue(0);
    load_land(0);
  }
  __syncthreads();
  auto sig = [](float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); };
  auto th = [](float x) { return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f; };
  const bool lo = lane < 32;
  float c = 0.f;
  for (int g = 0; g < ngroups; ++g) {
    if (wv == 0) {
      const float* gin = gxr + (g & 1) * PF * 128;
      float* gout = outr + (g & 1) * PF * 256;
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        if (g * PF + u >= T) break;
        float z0 = gin[u * 128 + lane], z1 = gin[u * 128 + 64 + lane];
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 q0[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}}, q1[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
        for (int k4 = 0; k4 < 8; ++k4) {
          const float4 h4 = *reinterpret_cast<const float4*>(hs + 4 * k4);
          const f2 ha = {h4.x, h4.y}, hb = {h4.z, h4.w};
          q0[0] = __builtin_elementwise_fma(f2{w0[4 * k4], w0[4 * k4 + 1]}, ha, q0[0]);
          q0[1] = __builtin_elementwise_fma(f2{w0[4 * k4 + 2], w0[4 * k4 + 3]}, hb, q0[1]);
          q1[0] = __builtin_elementwise_fma(f2{w1[4 * k4], w1[4 * k4 + 1]}, ha, q1[0]);
          q1[1] = __builtin_elementwise_fma(f2{w1[4 * k4 + 2], w1[4 * k4 + 3]}, hb, q1[1]);
        }
        const f2 s0 = q0[0] + q0[1], s1 = q1[0] + q1[1];
        z0 += s0.x + s0.y;
        z1 += s1.x + s1.y;
        const float a0 = sig(z0);                 // i (lane<32) or f
        const float a1 = lo ? th(z1) : sig(z1);   // g (lane<32) or o
        const float fg = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(a0), __float_as_uint(a0), false, false)[1]);
        const float og = __uint_as_float(__builtin_amdgcn_permlane32_swap(__float_as_uint(a1), __float_as_uint(a1), false, false)[1]);
        c = fmaf(a0, a1, fg * c);  // (as lstm32_fwd_kernel; lanes 32..63 carry a value nobody reads)
        const float h = og * th(c);
        hs[lane] = h;
        float* o = gout + u * 256;
        const int l = lane & 31;
        o[(lo ? 0 : 6) * 32 + l] = h;
        o[(lo ? 1 : 7) * 32 + l] = c;
        o[(lo ? 2 : 3) * 32 + l] = a0;  // i | f
        o[(lo ? 4 : 5) * 32 + l] = a1;  // g | o
        // one wave: LDS operations complete in issue order (see lstm32_fwd_kernel)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    } else {
      if (g + 1 < ngroups) load_issue(g + 1);
      if (g > 0) store_group(g - 1);
      if (g + 1 < ngroups) load_land(g + 1);
    }
    // both rings change hands: LDS operations drained, no wait for the helper's global stores
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  if (wv == 1) store_group(ngroups - 1);
}

int g_dg_dual = 1;  // avc_dg_dual_split(): one pass writes both split images of dG (dX and dW products)
int g_lstm32_mode = 1;  // avc_lstm32_tune(): 0 = libm gate math, 3-step prefetch; 1 = fast math with a
                        // memory wave (lstm32_fwd2_kernel); 4 = fast math, one wave

int launch_lstm32(int nblk, int T, int B, long ldgx, long ldy, const L32Dir& d0, const L32Dir& d1, hipStream_t s) {
  // the one-wave kernels address the saved gates / cell states through buffer descriptors with
  // 32-bit byte offsets: refuse sizes whose offsets would wrap
  AVC_CHECK_ARG((long)T * B * 512 < 0x80000000L, "encoder BiLSTM: T * B too large for 32-bit gate offsets");
  if (g_lstm32_mode == 0) lstm32_fwd_kernel<3, false><<<nblk, 64, 0, s>>>(T, B, ldgx, ldy, d0, d1);
  else if (g_lstm32_mode == 2) lstm32_fwd_kernel<8, true, 1><<<nblk, 64, 0, s>>>(T, B, ldgx, ldy, d0, d1);
  else if (g_lstm32_mode == 3) lstm32_fwd_kernel<8, true, 2><<<nblk, 64, 0, s>>>(T, B, ldgx, ldy, d0, d1);
  else if (g_lstm32_mode == 4) lstm32_fwd_kernel<8, true><<<nblk, 64, 0, s>>>(T, B, ldgx, ldy, d0, d1);
  else lstm32_fwd2_kernel<8><<<nblk, 128, 0, s>>>(T, B, ldgx, ldy, d0, d1);
  return AVC_OK;
}

// BPTT of an H = 32 direction: one single-wave workgroup per utterance walks the steps backwards.
// Lanes j and j + 32 each add one half of unit j's dh = W_hh^T dG sum and, after exchanging
// them, both run its cell math (lanes 32..63 store nothing).  The per-step operands (dy, the
// saved gates, c_t, c_{t-1}) come from a register ring whose next group is requested before a
// group's steps (loop unrolled by PF: static slots; clamped, so no join waits on them), and the dG broadcast through LDS needs
// no barrier: one wave's LDS operations complete in issue order (see lstm32_fwd_kernel).
// FAST (round 4, avc_lstm32_tune(1), the default): the 64-term dot product as two packed-FMA
// chains (v_pk_fma_f32, 16 instructions deep each, instead of one 64-deep scalar chain), and
// tanh(c_t) in the forward FAST kernel's own form, so the derivative uses the very tanh(c) value
// the forward multiplied by o_t (libm tanhf was also the longest piece of the step's chain).
template <int PF, bool FAST = false>
__global__ __launch_bounds__(64) void lstm32_bwd_kernel(int T, int B, int reverse,
                                                        const float* __restrict__ whh,
                                                        const float* __restrict__ gates,
                                                        const float* __restrict__ cs,
                                                        const float* __restrict__ dy, long lddy,
                                                        float* __restrict__ dg) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int j = lane & 31, half = lane >> 5;
  __shared__ __attribute__((aligned(16))) float dgs[128];
  float wc[64];
#pragma unroll
  for (int q = 0; q < 64; ++q) wc[q] = whh[(half * 64 + q) * 32 + j];
  dgs[lane] = 0.f;
  dgs[lane + 64] = 0.f;
  float dc = 0.f;
  __syncthreads();
  // iteration k walks s = T-1-k; time index t(s) and its predecessor in forward order
  auto tof = [&](int k) {
    const int s = T - 1 - min(k, T - 1);
    return reverse ? T - 1 - s : s;
  };
  auto tprev = [&](int k) {
    const int s = T - 1 - min(k, T - 1);
    return reverse ? T - s : s - 1;  // may be T or -1 at the ends (then unused)
  };
  float rdy[PF], rg[PF][4], rc[PF], rcp[PF];
  auto fetch = [&](int k, float& fdy, float (&fg4)[4], float& fc, float& fcp) {
    const long row = (long)tof(k) * B + b;
    const int tp = tprev(k);
    fdy = dy[row * lddy + j];
    const float* g = gates + row * 128;
    fg4[0] = g[j]; fg4[1] = g[32 + j]; fg4[2] = g[64 + j]; fg4[3] = g[96 + j];
    fc = cs[row * 32 + j];
    const int tpc = min(max(tp, 0), T - 1);
    fcp = cs[((long)tpc * B + b) * 32 + j];
  };
  // dG rows as buffer stores, the same number on every path (see lstm32_fwd_kernel): both wave
  // halves compute the same unit j (the dot product is completed across them), and lanes 32..63
  // store out of range.  Stores under `lane < 32` left the back edge waiting for all of them.
  constexpr unsigned kOut = 0x80000000u;
  const auto drs = __builtin_amdgcn_make_buffer_rsrc(dg, 0, (int)std::min<long>((long)T * B * 128 * 4, 0x7fffffffL),
                                                     0x00020000);
  auto step = [&](int k, float dyv, const float (&g4)[4], float c, float cpv) {
    const float ig = g4[0], fg = g4[1], gg = g4[2], og = g4[3];
    const int s = T - 1 - k;
    const int t = reverse ? T - 1 - s : s;
    const long row = (long)t * B + b;
    float part = 0.f;
    if constexpr (FAST) {
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 q[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
#pragma unroll
      for (int q4 = 0; q4 < 16; ++q4) {
        const float4 gq = *reinterpret_cast<const float4*>(dgs + half * 64 + 4 * q4);
        q[0] = __builtin_elementwise_fma(f2{wc[4 * q4], wc[4 * q4 + 1]}, f2{gq.x, gq.y}, q[0]);
        q[1] = __builtin_elementwise_fma(f2{wc[4 * q4 + 2], wc[4 * q4 + 3]}, f2{gq.z, gq.w}, q[1]);
      }
      const f2 sq = q[0] + q[1];
      part = sq.x + sq.y;
    } else {
#pragma unroll
      for (int q4 = 0; q4 < 16; ++q4) {
        const float4 gq = *reinterpret_cast<const float4*>(dgs + half * 64 + 4 * q4);
        part += wc[4 * q4] * gq.x + wc[4 * q4 + 1] * gq.y + wc[4 * q4 + 2] * gq.z + wc[4 * q4 + 3] * gq.w;
      }
    }
    // (lanes j and j + 32 add the same two halves: both hold the full sum)
    part += __shfl_xor(part, 32);
    const float dh = dyv + part;
    const float cp = s > 0 ? cpv : 0.f;
    // (FAST: lstm32_fwd_kernel<8, true>'s th(c))
    const float tc = FAST ? 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * c)) - 1.f : tanhf(c);
    const float dct = dh * og * (1.f - tc * tc) + dc;
    dc = dct * fg;
    const float dzi = dct * gg * ig * (1.f - ig);
    const float dzf = dct * cp * fg * (1.f - fg);
    const float dzg = dct * ig * (1.f - gg * gg);
    const float dzo = dh * tc * og * (1.f - og);
    const unsigned o = half ? kOut : (unsigned)((row * 128 + j) * 4);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dzi), drs, o, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dzf), drs, half ? kOut : o + 128, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dzg), drs, half ? kOut : o + 256, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dzo), drs, half ? kOut : o + 384, 0, 0);
    // one wave: these LDS writes land after this step's dgs reads (issue order); both halves
    // write the same values
    dgs[j] = dzi;
    dgs[32 + j] = dzf;
    dgs[64 + j] = dzg;
    dgs[96 + j] = dzo;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) fetch(u, rdy[u], rg[u], rc[u], rcp[u]);
  int k0 = 0;
  for (; k0 + PF <= T; k0 += PF) {
    // the next group's operands requested before this group's steps (see lstm32_fwd_kernel)
    float ndy[PF], ng[PF][4], nc[PF], ncp[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) fetch(k0 + PF + u, ndy[u], ng[u], nc[u], ncp[u]);  // clamped: no joins
#pragma unroll
    for (int u = 0; u < PF; ++u) step(k0 + u, rdy[u], rg[u], rc[u], rcp[u]);
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      rdy[u] = ndy[u]; rc[u] = nc[u]; rcp[u] = ncp[u];
#pragma unroll
      for (int q = 0; q < 4; ++q) rg[u][q] = ng[u][q];
    }
  }
#pragma unroll
  for (int u = 0; u < PF - 1; ++u)
    if (k0 + u < T) step(k0 + u, rdy[u], rg[u], rc[u], rcp[u]);
}

inline int ew_blocks(long n) { return (int)std::min<long>((n + 255) / 256, 8192); }

// [W_ih_f; W_ih_r] (256 x din) followed by the 256 summed biases (b_ih + b_hh per direction)
__global__ void concat_wih_kernel(const float* __restrict__ wf, const float* __restrict__ wr,
                                  const float* __restrict__ bif, const float* __restrict__ bhf,
                                  const float* __restrict__ bir, const float* __restrict__ bhr, int din,
                                  float* __restrict__ out) {
  const long n = 128L * din;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < 2 * n + 256; i += (long)gridDim.x * 256) {
    float v;
    if (i < n) v = wf[i];
    else if (i < 2 * n) v = wr[i - n];
    else {
      const int j = (int)(i - 2 * n);
      v = j < 128 ? bif[j] + bhf[j] : bir[j - 128] + bhr[j - 128];
    }
    out[i] = v;
  }
}

}  // namespace

size_t lstm_forward_scratch(int T, int B, int din, int H, bool training) {
  const size_t f = sizeof(float);
  size_t s = (size_t)T * B * 4 * H * f + 1024;
  if (H != 32) s += (size_t)4 * H * (din + H + 2) * f + (training ? 0 : (size_t)2 * B * H * f) + 2048;
  GemmDesc d;
  d.M = T * B; d.N = 4 * H; d.Kc = din; d.prec16 = 1;
  s += gemm_scratch_bytes(d);
  return lstm_split_supported(H, din) ? std::max(s, lstm_split_forward_scratch(T, B, din, H, 1)) : s;
}

int permute_rows(const float* src, float* dst, int H, int D, hipStream_t s) {
  permute_rows_kernel<<<ew_blocks(4L * H * D), 256, 0, s>>>(src, dst, H, D);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int lstm_forward_impl(avc_context* ctx, int T, int B, int din, int H, int reverse,
                      const float* x, int ldx, const float* w_ih, const float* w_hh,
                      const float* b_ih, const float* b_hh, float* y, int ldy,
                      float* saved_gates, float* saved_c, hipStream_t s, _Float16* y_frag) {
  if (y_frag) {
    // the persistent recurrence writes the split image in its epilogue; any other path splits y
    // afterwards (split_frag32_kernel's unscaled split: |h| < 1)
    if (lstm_split_supported(H, din) && !reverse && ldy == H && lstm1_persist_eligible(T, B, H))
      return lstm_split_forward_impl(ctx, T, B, din, H, reverse, x, ldx, w_ih, w_hh, b_ih, b_hh, y, ldy,
                                     saved_gates, saved_c, s, y_frag);
    AVC_TRY(lstm_forward_impl(ctx, T, B, din, H, reverse, x, ldx, w_ih, w_hh, b_ih, b_hh, y, ldy, saved_gates,
                              saved_c, s));
    return gemm_split_frag(y, ldy, T * B, H, nullptr, y_frag, s);
  }
  AVC_CHECK_ARG(T > 0 && B > 0 && din > 0, "lstm: empty problem");
  AVC_CHECK_ARG(H == 32 || (H % 64 == 0), "lstm: H must be 32 or a multiple of 64");
  AVC_CHECK_ARG(din % 4 == 0 && ldx % 4 == 0, "lstm: din/ldx must be multiples of 4");
  if (lstm_split_supported(H, din))
    return lstm_split_forward_impl(ctx, T, B, din, H, reverse, x, ldx, w_ih, w_hh, b_ih, b_hh, y, ldy,
                                   saved_gates, saved_c, s);
  Scratch sc(ctx);
  const long TB = (long)T * B;
  AVC_TAKE(gx, float, (size_t)TB * 4 * H, sc);

  GemmDesc g;
  g.M = (int)TB; g.N = 4 * H; g.Kc = din;
  g.A = x; g.lda = ldx; g.a_rows = TB;
  g.b_trans = 1; g.ldb = din;
  g.C = gx; g.ldc = 4 * H;
  g.prec16 = 1;

  if (H == 32) {
    g.B = w_ih; g.bias0 = b_ih; g.bias1 = b_hh;
    AVC_TRY(gemm_run(ctx, g, s));
    hipEvent_t ev = timing_begin(TC_LSTM32, s);
    L32Dir d{gx, w_hh, y, saved_gates, saved_c, reverse};
    AVC_TRY(launch_lstm32(B, T, B, 128, ldy, d, d, s));
    AVC_LAUNCH_CHECK();
    if (ev) timing_end(TC_LSTM32, ev, s, 2.0 * T * B * 128.0 * 32.0, 4.0 * T * B * (128.0 + 32.0));
    return AVC_OK;
  }

  AVC_TAKE(wih_p, float, (size_t)4 * H * din, sc);
  AVC_TAKE(whh_p, float, (size_t)4 * H * H, sc);
  AVC_TAKE(bih_p, float, (size_t)4 * H, sc);
  AVC_TAKE(bhh_p, float, (size_t)4 * H, sc);
  permute_rows_kernel<<<ew_blocks(4L * H * din), 256, 0, s>>>(w_ih, wih_p, H, din);
  permute_rows_kernel<<<ew_blocks(4L * H * H), 256, 0, s>>>(w_hh, whh_p, H, H);
  permute_vec_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(b_ih, bih_p, H);
  permute_vec_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(b_hh, bhh_p, H);
  AVC_LAUNCH_CHECK();
  g.B = wih_p; g.bias0 = bih_p; g.bias1 = bhh_p;
  AVC_TRY(gemm_run(ctx, g, s));

  float* cpp = nullptr;
  if (!saved_c) {
    AVC_TAKE(tmp, float, (size_t)2 * B * H, sc);
    cpp = tmp;
  }
  const StepCfg cfg = step_cfg(B, H / 4, H);
  dim3 grid(H / 4, (B + cfg.mb - 1) / cfg.mb);
  for (int st = 0; st < T; ++st) {
    const int t = reverse ? T - 1 - st : st;
    const int tp = reverse ? t + 1 : t - 1;
    StepArgs a{};
    a.B = B; a.H = H; a.nblk0 = (int)grid.x;
    a.K[0] = H; a.K0[0] = H; a.kw[0] = H / cfg.nw;
    a.A[0] = st > 0 ? y + (long)tp * B * ldy : nullptr;
    a.lda[0] = ldy;
    a.W[0] = whh_p;
    a.gx[0] = gx + (long)t * B * 4 * H;
    a.ldgx[0] = 4L * H;
    if (saved_c) {
      a.c_prev[0] = st > 0 ? saved_c + (long)tp * B * H : nullptr;
      a.c_out[0] = saved_c + (long)t * B * H;
    } else {
      a.c_prev[0] = st > 0 ? cpp + (long)((st - 1) & 1) * B * H : nullptr;
      a.c_out[0] = cpp + (long)(st & 1) * B * H;
    }
    a.h_out[0] = y + (long)t * B * ldy;
    a.ldh_out[0] = ldy;
    a.gates_out[0] = saved_gates ? saved_gates + (long)t * B * 4 * H : nullptr;
    launch_step(cfg, false, grid, a, s);
  }
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

size_t bilstm_forward_scratch(int T, int B, int din, int H, bool training) {
  if (H != 32) return lstm_forward_scratch(T, B, din, H, training);
  GemmDesc d;
  d.M = T * B; d.N = 256; d.Kc = din; d.prec16 = 1;
  return (size_t)T * B * 256 * sizeof(float) + ((size_t)256 * din + 256) * sizeof(float) + 256 +
         gemm_scratch_bytes(d) + 1024;
}

namespace {
GemmDesc bilstm_proj_desc(int T, int B, int din) {
  GemmDesc g;
  g.M = T * B; g.N = 256; g.Kc = din; g.a_rows = (long)T * B;
  g.b_trans = 1; g.ldb = din; g.prec16 = 1;
  return g;
}
}  // namespace

bool bilstm_takes_frag(int T, int B, int din) { return gemm_frag_eligible(bilstm_proj_desc(T, B, din)); }

// Bidirectional layer (encoder.py:51): y[:, 0:H] forward, y[:, H:2H] reverse.  H = 32: both input
// projections into one [T*B][256] buffer, then ONE recurrence launch for both directions.
int bilstm_forward_impl(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                        const float* const* wf, const float* const* wr, float* y, int ldy,
                        float* g_f, float* c_f, float* g_r, float* c_r, hipStream_t s, const _Float16* x_frag) {
  if (H != 32) {
    AVC_TRY(lstm_forward_impl(ctx, T, B, din, H, 0, x, ldx, wf[0], wf[1], wf[2], wf[3], y, ldy, g_f, c_f, s));
    return lstm_forward_impl(ctx, T, B, din, H, 1, x, ldx, wr[0], wr[1], wr[2], wr[3], y + H, ldy, g_r, c_r, s);
  }
  AVC_CHECK_ARG(T > 0 && B > 0 && din % 4 == 0 && ldx % 4 == 0, "bilstm: bad shape");
  Scratch sc(ctx);
  const long TB = (long)T * B;
  AVC_TAKE(gx, float, (size_t)TB * 256, sc);
  // both directions' input projections as ONE product against [W_ih_f; W_ih_r] (256 x din) with
  // the summed biases: x is split once, and gx comes out as [T*B][fwd 128 | bwd 128]
  bool fw;
  float* wcat = prep_or_scratch<float>(ctx, sc, PREP_BILSTM_WIH, wf[0], wr[0], (size_t)256 * din + 256, &fw);
  if (!wcat) return AVC_ERR_WORKSPACE;
  if (fw) {
    concat_wih_kernel<<<ew_blocks(256L * din + 256), 256, 0, s>>>(wf[0], wr[0], wf[2], wf[3], wr[2], wr[3], din,
                                                                  wcat);
    AVC_LAUNCH_CHECK();
  }
  GemmDesc g;
  g.M = (int)TB; g.N = 256; g.Kc = din;
  g.A = x; g.lda = ldx; g.a_rows = TB;
  g.b_trans = 1; g.ldb = din; g.B = wcat; g.bias0 = wcat + 256L * din;
  g.C = gx; g.ldc = 256;
  g.prec16 = 1;
  if (x_frag) {  // x handed over split by its producer (bilstm_takes_frag said yes; x itself is not read)
    AVC_CHECK_ARG(ldx == din && gemm_frag_eligible(g), "bilstm: a split input needs a fragment-streaming product");
    g.a_frag = x_frag;
  }
  if (ctx->prep_version >= 0) {
    bool fb = true;
    auto* bf = static_cast<_Float16*>(prep_buffer(ctx, PREP_GEMM_BFRAG, wcat, nullptr, gemm_bfrag_bytes(g), &fb));
    if (bf) {
      if (fb || fw) AVC_TRY(gemm_prepare_bfrag(g, bf, s));
      g.b_frag = bf;
    }
  }
  AVC_TRY(gemm_run(ctx, g, s));
  hipEvent_t ev = timing_begin(TC_LSTM32, s);
  L32Dir d0{gx, wf[1], y, g_f, c_f, 0};
  L32Dir d1{gx + 128, wr[1], y + 32, g_r, c_r, 1};
  AVC_TRY(launch_lstm32(2 * B, T, B, 256, ldy, d0, d1, s));
  AVC_LAUNCH_CHECK();
  if (ev) timing_end(TC_LSTM32, ev, s, 2.0 * 2 * T * B * 128.0 * 32.0, 2.0 * 4.0 * T * B * (128.0 + 32.0));
  return AVC_OK;
}

size_t lstm2_forward_scratch(int T, int B, int din, int H, bool training) {
  const size_t f = sizeof(float);
  size_t s = (size_t)T * B * 4 * H * f + (size_t)4 * H * (din + H + 2 * H + 3) * f + 4096;
  if (!training) s += (size_t)4 * B * H * f;
  GemmDesc d;
  d.M = T * B; d.N = 4 * H; d.Kc = din; d.prec16 = 1;
  s += gemm_scratch_bytes(d);
  return lstm_split_supported(H, din) ? std::max(s, lstm_split_forward_scratch(T, B, din, H, 2)) : s;
}

// Two stacked LSTM layers (decoder.lstm2, decoder.py:53,74) advanced as a wavefront: launch s
// runs layer 0 at t = s and layer 1 at t = s-1 side by side, so 2T recurrent steps take T+1
// launches.  Layer 1's input projection is folded into its recurrent product: its gates are
// [h0_t | h1_{t-1}] . [W_ih1 | W_hh1]^T + (b_ih1 + b_hh1) with K = 2H.
int lstm2_forward_impl(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                       const float* const* w0, const float* const* w1, float* y0, float* y1,
                       float* g0, float* c0, float* g1, float* c1, hipStream_t s, _Float16* y1_frag) {
  if (y1_frag) {  // as lstm_forward_impl's y_frag, for the second layer's output
    if (lstm_split_supported(H, din) && lstm2_persist_eligible(T, B, H))
      return lstm2_split_forward_impl(ctx, T, B, din, H, x, ldx, w0, w1, y0, y1, g0, c0, g1, c1, s, y1_frag);
    AVC_TRY(lstm2_forward_impl(ctx, T, B, din, H, x, ldx, w0, w1, y0, y1, g0, c0, g1, c1, s));
    return gemm_split_frag(y1, H, T * B, H, nullptr, y1_frag, s);
  }
  AVC_CHECK_ARG(T > 0 && B > 0 && din % 4 == 0 && ldx % 4 == 0, "lstm2: bad shape");
  AVC_CHECK_ARG(H % 64 == 0, "lstm2: H must be a multiple of 64");
  AVC_CHECK_ARG((g0 == nullptr) == (c0 == nullptr) && (g1 == nullptr) == (c1 == nullptr) &&
                    (c0 == nullptr) == (c1 == nullptr), "lstm2: saved buffers all or none");
  if (lstm_split_supported(H, din))
    return lstm2_split_forward_impl(ctx, T, B, din, H, x, ldx, w0, w1, y0, y1, g0, c0, g1, c1, s);
  Scratch sc(ctx);
  const long TB = (long)T * B;
  AVC_TAKE(gx, float, (size_t)TB * 4 * H, sc);
  AVC_TAKE(wih_p, float, (size_t)4 * H * din, sc);
  AVC_TAKE(whh_p, float, (size_t)4 * H * H, sc);
  AVC_TAKE(w1_p, float, (size_t)4 * H * 2 * H, sc);
  AVC_TAKE(bih_p, float, (size_t)4 * H, sc);
  AVC_TAKE(bhh_p, float, (size_t)4 * H, sc);
  AVC_TAKE(b1_p, float, (size_t)4 * H, sc);
  permute_rows_kernel<<<ew_blocks(4L * H * din), 256, 0, s>>>(w0[0], wih_p, H, din);
  permute_rows_kernel<<<ew_blocks(4L * H * H), 256, 0, s>>>(w0[1], whh_p, H, H);
  permute_vec_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(w0[2], bih_p, H);
  permute_vec_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(w0[3], bhh_p, H);
  permute_concat_kernel<<<ew_blocks(8L * H * H), 256, 0, s>>>(w1[0], H, w1[1], H, w1_p, H);
  permute_vec_sum_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(w1[2], w1[3], b1_p, H);
  AVC_LAUNCH_CHECK();
  GemmDesc g;
  g.M = (int)TB; g.N = 4 * H; g.Kc = din;
  g.A = x; g.lda = ldx; g.a_rows = TB;
  g.b_trans = 1; g.ldb = din; g.B = wih_p; g.bias0 = bih_p; g.bias1 = bhh_p;
  g.C = gx; g.ldc = 4 * H;
  g.prec16 = 1;
  AVC_TRY(gemm_run(ctx, g, s));

  float* cpp0 = nullptr;
  float* cpp1 = nullptr;
  if (!c0) {
    AVC_TAKE(tmp, float, (size_t)4 * B * H, sc);
    cpp0 = tmp;
    cpp1 = tmp + 2L * B * H;
  }
  StepCfg cfg = step_cfg(B, H / 4, H);
  cfg.nw = 4;  // both slots share the block shape; layer 1 waves 0-1 read h0, 2-3 read h1
  const int nb = H / 4;
  for (int st = 0; st <= T; ++st) {
    const bool l0 = st < T, l1 = st >= 1;
    StepArgs a{};
    a.B = B; a.H = H;
    const int t0 = st, t1 = st - 1;
    // slot 0: layer 0 at t0
    a.K[0] = H; a.K0[0] = H; a.kw[0] = H / cfg.nw;
    a.A[0] = (l0 && t0 > 0) ? y0 + (long)(t0 - 1) * B * H : nullptr;
    a.lda[0] = H;
    a.W[0] = whh_p;
    a.gx[0] = gx + (long)(l0 ? t0 : 0) * B * 4 * H;
    a.ldgx[0] = 4L * H;
    if (c0) {
      a.c_prev[0] = (l0 && t0 > 0) ? c0 + (long)(t0 - 1) * B * H : nullptr;
      a.c_out[0] = c0 + (long)(l0 ? t0 : 0) * B * H;
    } else {
      a.c_prev[0] = (l0 && t0 > 0) ? cpp0 + (long)((t0 - 1) & 1) * B * H : nullptr;
      a.c_out[0] = cpp0 + (long)(t0 & 1) * B * H;
    }
    a.h_out[0] = y0 + (long)(l0 ? t0 : 0) * B * H;
    a.ldh_out[0] = H;
    a.gates_out[0] = g0 ? g0 + (long)(l0 ? t0 : 0) * B * 4 * H : nullptr;
    // slot 1: layer 1 at t1 (input h0_{t1} | recurrent h1_{t1-1})
    a.K[1] = 2 * H; a.K0[1] = H; a.kw[1] = 2 * H / cfg.nw;
    a.A[1] = l1 ? y0 + (long)t1 * B * H : nullptr;
    a.lda[1] = H;
    a.A1[1] = (l1 && t1 > 0) ? y1 + (long)(t1 - 1) * B * H : nullptr;
    a.lda1[1] = H;
    a.W[1] = w1_p;
    a.gx[1] = b1_p;
    a.ldgx[1] = 0;
    const int tt1 = l1 ? t1 : 0;
    if (c1) {
      a.c_prev[1] = (l1 && t1 > 0) ? c1 + (long)(t1 - 1) * B * H : nullptr;
      a.c_out[1] = c1 + (long)tt1 * B * H;
    } else {
      a.c_prev[1] = (l1 && t1 > 0) ? cpp1 + (long)((t1 - 1) & 1) * B * H : nullptr;
      a.c_out[1] = cpp1 + (long)(tt1 & 1) * B * H;
    }
    a.h_out[1] = y1 + (long)tt1 * B * H;
    a.ldh_out[1] = H;
    a.gates_out[1] = g1 ? g1 + (long)tt1 * B * 4 * H : nullptr;
    a.nblk0 = l0 ? nb : 0;
    dim3 grid((l0 ? nb : 0) + (l1 ? nb : 0), (B + cfg.mb - 1) / cfg.mb);
    launch_step(cfg, false, grid, a, s);
  }
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

size_t lstm_backward_scratch(int T, int B, int din, int H) {
  const size_t f = sizeof(float);
  const size_t TB = (size_t)T * B;
  size_t s = TB * 4 * H * f + (size_t)B * H * f + (size_t)4 * H * (din + H) * 2 * f +
             (size_t)4 * H * f + 8192;
  s += 2 * ((size_t)B + 64) * 4 * H * f + 512;  // fragment-major dG ping-pong
  // split-K BPTT (bptt_row_kernel): split W_hh^T, split dG rows, <= 32 partial slabs, row scales
  s += gemm_afrag_bytes(H, 4 * H) + gemm_afrag_bytes(B + 31, 4 * H) + 32 * (size_t)B * H * f + (size_t)B * f + 2048;
  s += bptt_persist_scratch(B, H);  // the persistent BPTT's double-buffered slabs, split dG, dc
  s += gemm_afrag_bytes(4L * H, (int)TB) + 256;  // dG^T split once for dW_ih and dW_hh
  s += gemm_afrag_bytes((long)TB, 4 * H) + 256;  // dG split by the same pass for dX (gemm_split_dual)
  GemmDesc d1;  // dW_ih
  d1.M = 4 * H; d1.N = din; d1.Kc = (int)TB; d1.a_trans = 1; d1.b_rows = TB;
  d1.prec16 = 1; d1.split_scale = 1;
  GemmDesc d2 = d1; d2.N = H; d2.b_shift0 = B;
  GemmDesc d3; d3.M = (int)TB; d3.N = din; d3.Kc = 4 * H; d3.a_rows = TB;
  d3.prec16 = 1; d3.split_scale = 1;
  size_t gs = std::max(gemm_scratch_bytes(d1), std::max(gemm_scratch_bytes(d2), gemm_scratch_bytes(d3)));
  return s + gs + colsum_scratch((int)TB, 4 * H);
}

__device__ unsigned g_h_bound_bits = 0x3f800000u;  // 1.0f: the bound of an LSTM's |h|
// The word's address on the CURRENT device: a __device__ symbol has one instance per device, and
// the library keeps one context per device in one process (a single cached address
// made a second device's LSTM backward read the first device's global).
const unsigned* h_bound_word() {
  constexpr int kMaxDev = 64;
  static std::mutex m;
  static const unsigned* addr[kMaxDev] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  std::lock_guard<std::mutex> g(m);
  if (!addr[dev]) {
    void* q = nullptr;
    if (hipGetSymbolAddress(&q, HIP_SYMBOL(g_h_bound_bits)) == hipSuccess) addr[dev] = static_cast<const unsigned*>(q);
    else (void)hipGetLastError();
  }
  return addr[dev];  // nullptr: the product scans y itself
}

int lstm_backward_impl(avc_context* ctx, int T, int B, int din, int H, int reverse,
                       const float* x, int ldx, const float* w_ih, const float* w_hh,
                       const float* y, int ldy, const float* saved_gates, const float* saved_c,
                       const float* d_y, float* d_x, float* d_w_ih, float* d_w_hh,
                       float* d_b_ih, float* d_b_hh, int accumulate_dx, int accumulate_dw,
                       hipStream_t s, bool x_unit) {
  // x_unit: every |x| <= 1 (x is the previous stacked layer's h): dW_ih's split of x takes that
  // bound (as dW_hh's split of y does, below) instead of a max scan
  AVC_CHECK_ARG(T > 0 && B > 0 && din > 0, "lstm_backward: empty problem");
  AVC_CHECK_ARG(H == 32 || (H % 64 == 0), "lstm_backward: H must be 32 or a multiple of 64");
  AVC_CHECK_ARG(saved_gates && saved_c, "lstm_backward: saved gates/cells required");
  Scratch sc(ctx);
  const long TB = (long)T * B;
  AVC_TAKE(dg, float, (size_t)TB * 4 * H, sc);
  const bool small = H == 32;
  const float* wih_use = w_ih;
  float* dwih_dst = d_w_ih;
  float* dwhh_dst = d_w_hh;
  int acc_w = accumulate_dw;

  // the whole recurrence as one persistent launch where eligible (lstm_persist.hip), else
  // split-K products where they measured faster (scripts/bptt_ab.py, B = 256: H = 1024 7.95 vs
  // 9.44 ms per layer backward; H = 512 4.02 vs 3.40 ms, so the step kernel stays there)
  const bool persist_bptt = !small && g_bptt_mode != 0 && saved_gates && saved_c && bptt_persist_eligible(T, B, H);
  const bool gemm_bptt = persist_bptt || (!small && B >= 32 && (H == 512 || H == 1024) &&
                                          (g_bptt_mode == 2 || (g_bptt_mode == 1 && H == 1024)));
  // the persistent BPTT also produces max |dG| and the bias gradients' column partials
  AVC_TAKE(amax_dg, unsigned, 64, sc);  // one max|dG| shared by the three products below
  float* colpart = nullptr;
  if (persist_bptt) {
    AVC_TAKE(cp, float, (size_t)bptt_colpart_rows(B, H) * 4 * H, sc);
    colpart = cp;
  }
  if (small) {
    // (PF 4: a group's 28 operand loads + 16 stores stay inside the 63 counted vector-memory ops)
    if (g_lstm32_mode == 0) lstm32_bwd_kernel<4, false><<<B, 64, 0, s>>>(T, B, reverse, w_hh, saved_gates, saved_c, d_y, ldy, dg);
    else lstm32_bwd_kernel<4, true><<<B, 64, 0, s>>>(T, B, reverse, w_hh, saved_gates, saved_c, d_y, ldy, dg);
    AVC_LAUNCH_CHECK();
  } else if (gemm_bptt) {
    // W_hh^T permuted ([H][4H]: row j = hidden unit, k = permuted gate row), split once with the
    // scale of max |W_hh|; per step the split-K product and the row epilogue (see bptt_row_kernel)
    AVC_TAKE(wih_p, float, (size_t)4 * H * din, sc);
    AVC_TAKE(whhT, float, (size_t)4 * H * H, sc);
    AVC_TAKE(whhT_s, _Float16, gemm_afrag_bytes(H, 4 * H) / 2, sc);
    const long arows = (B + 31) / 32 * 32;
    AVC_TAKE(dgs, _Float16, gemm_afrag_bytes(arows, 4 * H) / 2, sc);
    AVC_TAKE(dc, float, (size_t)B * H, sc);
    AVC_TAKE(rowscale, float, (size_t)B, sc);
    AVC_TAKE(amax_w, unsigned, 64, sc);
    // 128x128 tiles, split-K toward ~256 workgroups with >= two 64-deep K-tiles each (8, 16 or
    // 32 splits).  64x64 tiles with 4-16 splits (a quarter of the slab traffic, twice the operand
    // intake per workgroup) measured 9.13 vs 7.95 ms per H = 1024 layer backward.
    const int tile = 128;
    const int tiles = (int)((B + tile - 1) / tile) * ((H + tile - 1) / tile);
    const int ktiles = 4 * H / 64;
    const int want = std::min(ktiles / 2, (256 + tiles - 1) / tiles);
    const int nsplit = want >= 32 ? 32 : want >= 16 ? 16 : 8;
    AVC_TAKE(slab, float, (size_t)nsplit * B * H, sc);
    permute_rows_kernel<<<ew_blocks(4L * H * din), 256, 0, s>>>(w_ih, wih_p, H, din);
    transpose_permute_kernel<<<dim3(4 * H / 32, H / 32), 256, 0, s>>>(w_hh, whhT, H);
    AVC_TRY(gemm_absmax(w_hh, 4L * H, H, H, amax_w, s));  // (zeroes *amax_w first)
    AVC_TRY(gemm_split_frag(whhT, 4L * H, H, 4 * H, amax_w, whhT_s, s));
    AVC_TRY(zero_async(dc, sizeof(float) * B * H, s));
    AVC_TRY(zero_async(dgs, gemm_afrag_bytes(arows, 4 * H), s));  // padding rows stay zero
    AVC_LAUNCH_CHECK();
    if (persist_bptt)
      AVC_TRY(bptt_persist_run(ctx, T, B, H, reverse, whhT_s, amax_w, d_y, ldy, saved_gates, saved_c, dg, colpart,
                               amax_dg, s));
    for (int st = persist_bptt ? -1 : T - 1; st >= 0; --st) {
      const int t = reverse ? T - 1 - st : st;
      const int tp = reverse ? t + 1 : t - 1;
      BpttArgs a{};
      a.B = B; a.H = H; a.nsplit = nsplit; a.first = st == T - 1; a.last = st == 0;
      // timing class lstm_step_bwd: the whole step (product + row epilogue)
      hipEvent_t ev = timing_begin(TC_LSTM_STEP_BWD, s);
      if (!a.first) AVC_TRY(gemm_frag_partials(B, H, 4 * H, dgs, whhT_s, tile, nsplit, slab, s));
      a.slab = slab; a.rowscale = rowscale; a.amax_w = amax_w;
      a.dy = d_y + (long)t * B * ldy; a.lddy = ldy;
      a.gates = saved_gates + (long)t * B * 4 * H;
      a.c_cur = saved_c + (long)t * B * H;
      a.c_prv = st > 0 ? saved_c + (long)tp * B * H : nullptr;
      a.dc = dc; a.dg_out = dg + (long)t * B * 4 * H; a.dgs = dgs;
#define AVC_BPTT_ROW(NSV)                                                                         \
  if (H == 1024) bptt_row_kernel<4, NSV><<<B, 256, 4 * H * sizeof(float), s>>>(a);                \
  else bptt_row_kernel<2, NSV><<<B, 256, 4 * H * sizeof(float), s>>>(a);
      if (nsplit == 32) { AVC_BPTT_ROW(32) } else if (nsplit == 16) { AVC_BPTT_ROW(16) } else { AVC_BPTT_ROW(8) }
#undef AVC_BPTT_ROW
      AVC_LAUNCH_CHECK();
      // algorithmic bytes: the split operands of the product, dy / gates / c / dc in, dG / dc out
      if (ev) timing_end(TC_LSTM_STEP_BWD, ev, s, a.first ? 0.0 : 2.0 * B * H * 4.0 * H,
                         (a.first ? 0.0 : 4.0 * (4.0 * H * H + 4.0 * B * H)) + 4.0 * B * H * 9.0);
    }
    wih_use = wih_p;
    AVC_TAKE(dwih_p, float, (size_t)4 * H * din, sc);
    AVC_TAKE(dwhh_p, float, (size_t)4 * H * H, sc);
    dwih_dst = dwih_p;
    dwhh_dst = dwhh_p;
    acc_w = 0;
  } else {
    AVC_TAKE(wih_p, float, (size_t)4 * H * din, sc);
    AVC_TAKE(whhT_p, float, (size_t)4 * H * H, sc);
    AVC_TAKE(dc, float, (size_t)B * H, sc);
    const StepCfg cfg = step_cfg(B, H / 16, 4 * H);
    dim3 grid(H / 16, (B + cfg.mb - 1) / cfg.mb);
    // the recurrent dG (and W_hh^T) travel fragment-major, padded to whole row tiles
    const long fsz = (long)grid.y * cfg.mb * 4 * H;
    AVC_TAKE(dgf, float, (size_t)2 * fsz, sc);
    permute_rows_kernel<<<ew_blocks(4L * H * din), 256, 0, s>>>(w_ih, wih_p, H, din);
    whhT_frag_kernel<<<ew_blocks(4L * H * H), 256, 0, s>>>(w_hh, whhT_p, H);
    AVC_TRY(zero_async(dc, sizeof(float) * B * H, s));
    AVC_TRY(zero_async(dgf, sizeof(float) * 2 * fsz, s));
    AVC_LAUNCH_CHECK();
    for (int st = T - 1; st >= 0; --st) {
      const int t = reverse ? T - 1 - st : st;
      const int tn = reverse ? t - 1 : t + 1;  // time index processed after t in the forward pass
      const int tp = reverse ? t + 1 : t - 1;
      StepArgs a{};
      a.B = B; a.H = H; a.nblk0 = (int)grid.x;
      a.K[0] = 4 * H; a.K0[0] = 4 * H; a.kw[0] = 4 * H / cfg.nw;
      const int it = T - 1 - st;  // iteration index: the previous launch wrote buffer (it-1)&1
      a.A[0] = st < T - 1 ? dgf + (long)((it - 1) & 1) * fsz : nullptr;
      a.lda[0] = H / 4;  // 16-k chunks per row tile
      a.frag = 1;
      a.dgf_out = st > 0 ? dgf + (long)(it & 1) * fsz : nullptr;
      a.W[0] = whhT_p;
      a.dy = d_y + (long)t * B * ldy;
      a.lddy = ldy;
      a.gates = saved_gates + (long)t * B * 4 * H;
      a.c_cur = saved_c + (long)t * B * H;
      a.c_prv = st > 0 ? saved_c + (long)tp * B * H : nullptr;
      a.dc = dc;
      a.dg_out = dg + (long)t * B * 4 * H;
      launch_step(cfg, true, grid, a, s);
    }
    AVC_LAUNCH_CHECK();
    wih_use = wih_p;
    AVC_TAKE(dwih_p, float, (size_t)4 * H * din, sc);
    AVC_TAKE(dwhh_p, float, (size_t)4 * H * H, sc);
    dwih_dst = dwih_p;
    dwhh_dst = dwhh_p;
    acc_w = 0;
  }

  // weight gradients: dW_ih = dG^T x ; dW_hh = dG^T h_prev (h_prev = y shifted one step)
  if (!persist_bptt) AVC_TRY(gemm_absmax(dg, TB, 4L * H, 4L * H, amax_dg, s));
  GemmDesc g1;
  g1.M = 4 * H; g1.N = din; g1.Kc = (int)TB;
  g1.A = dg; g1.a_trans = 1; g1.lda = 4 * H;
  g1.B = x; g1.ldb = ldx; g1.b_rows = TB;
  g1.C = dwih_dst; g1.ldc = din; g1.accumulate = acc_w;
  g1.prec16 = 1; g1.split_scale = 1; g1.amax_a = amax_dg;
  if (x_unit) g1.amax_b = h_bound_word();
  else if (x == ctx->xhint.x && ctx->xhint.amax) g1.amax_b = ctx->xhint.amax;  // max |x| from its producer
  // dG^T is split once (the larger operand of both products: TB x 4H against TB x din / H); with
  // the dX product also streaming split dG, one pass writes both images (g_dg_dual)
  const bool share = gemm_frag_eligible(g1);
  _Float16* dg_s = nullptr;  // dG as the dX product's A operand, when the dual pass wrote it
  if (share) {
    AVC_TAKE(dgT_s, _Float16, gemm_afrag_bytes(4L * H, (int)TB) / 2, sc);
    GemmDesc g3p;
    g3p.M = (int)TB; g3p.N = din; g3p.Kc = 4 * H; g3p.A = dg; g3p.lda = 4 * H; g3p.a_rows = TB;
    g3p.B = wih_use; g3p.ldb = din; g3p.b_rows = 4L * H; g3p.C = d_x; g3p.ldc = din; g3p.prec16 = 1;
    g3p.split_scale = 1;
    g3p.amax_a = amax_dg;
    if (g_dg_dual && d_x && gemm_frag_eligible(g3p) && gemm_split_dual_ok((long)TB, 4L * H, 4L * H)) {
      AVC_TAKE(dgs_a, _Float16, gemm_afrag_bytes((long)TB, 4 * H) / 2, sc);
      AVC_TRY(gemm_split_dual(dg, 4L * H, (long)TB, 4 * H, amax_dg, dgs_a, dgT_s, s));
      dg_s = dgs_a;
      g1.a_frag = dgT_s;
      g1.a_frag_scaled = 1;
    } else {
      g1.a_frag_out = dgT_s;
    }
  }
  AVC_TRY(gemm_run(ctx, g1, s));
  GemmDesc g2 = g1;
  g2.N = H;
  g2.B = y; g2.ldb = ldy; g2.b_shift0 = reverse ? B : -B;
  // y is this layer's h = o tanh(c), |h| < 1: its split takes the power of two of that bound
  // instead of a max scan of the 64-128 MB operand (round 5).  A bound above the max by 2^k moves
  // every element k binades down inside f16's range, so only elements below ~2^-28 of the bound
  // could split differently (DESIGN §9i's argument); their share of dW_hh is below 2^-28.
  g2.amax_b = h_bound_word();
  g2.C = dwhh_dst; g2.ldc = H;
  if (share && gemm_frag_eligible(g2)) {
    g2.a_frag = g1.a_frag_out ? g1.a_frag_out : g1.a_frag;
    g2.a_frag_scaled = 1;
  }
  g2.a_frag_out = nullptr;
  AVC_TRY(gemm_run(ctx, g2, s));

  if (small) {
    AVC_TRY(colsum(ctx, (int)TB, 4 * H, dg, 4 * H, d_b_ih, accumulate_dw, s, d_b_hh));  // d_b_ih = d_b_hh
  } else {
    AVC_TAKE(db_p, float, (size_t)4 * H, sc);
    if (persist_bptt)  // the BPTT's per-row-block partials
      AVC_TRY(colsum(ctx, bptt_colpart_rows(B, H), 4 * H, colpart, 4 * H, db_p, 0, s));
    else AVC_TRY(colsum(ctx, (int)TB, 4 * H, dg, 4 * H, db_p, 0, s));
    unpermute_rows_kernel<<<ew_blocks(4L * H * din), 256, 0, s>>>(dwih_dst, d_w_ih, H, din, accumulate_dw);
    unpermute_rows_kernel<<<ew_blocks(4L * H * H), 256, 0, s>>>(dwhh_dst, d_w_hh, H, H, accumulate_dw);
    unpermute_vec2_kernel<<<(4 * H + 255) / 256, 256, 0, s>>>(db_p, d_b_ih, d_b_hh, H, accumulate_dw);
    AVC_LAUNCH_CHECK();
  }

  if (d_x) {
    GemmDesc g3;
    g3.M = (int)TB; g3.N = din; g3.Kc = 4 * H;
    g3.A = dg; g3.lda = 4 * H; g3.a_rows = TB;
    g3.B = wih_use; g3.ldb = din;
    g3.b_trans = small ? 0 : 0;
    g3.C = d_x; g3.ldc = din; g3.accumulate = accumulate_dx;
    g3.prec16 = 1; g3.split_scale = 1; g3.amax_a = amax_dg;
    if (dg_s) {  // written by the dual split pass above
      g3.a_frag = dg_s;
      g3.a_frag_scaled = 1;
    }
    AVC_TRY(gemm_run(ctx, g3, s));
  }
  return AVC_OK;
}

}  // namespace avc

#ifdef AVC_STAMPS
extern "C" int avc_debug_stamps(void* buf, long target_launch) {
  avc::g_stamp_buf = buf;
  avc::g_stamp_target = target_launch;
  avc::g_stamp_count = 0;
  return AVC_OK;
}
#endif

extern "C" int avc_dg_dual_split(int on) {
  if (on != 0 && on != 1) {
    avc::set_error("avc_dg_dual_split: on must be 0 or 1");
    return AVC_ERR_INVALID;
  }
  avc::g_dg_dual = on;
  return AVC_OK;
}

extern "C" int avc_bptt_mode(int mode) {
  if (mode < 0 || mode > 2) {
    avc::set_error("avc_bptt_mode: mode must be 0 (step kernel), 1 (automatic) or 2 (split-K products wherever eligible)");
    return AVC_ERR_INVALID;
  }
  avc::g_bptt_mode = mode;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_lstm_tune(int rows_per_block, int waves) {
  if (!(rows_per_block == 0 || rows_per_block == 16 || rows_per_block == 32 || rows_per_block == 64)) {
    avc::set_error("avc_lstm_tune: rows_per_block must be 0, 16, 32 or 64");
    return AVC_ERR_INVALID;
  }
  if (waves < 0 || waves > 8) {
    avc::set_error("avc_lstm_tune: waves must be 0..8");
    return AVC_ERR_INVALID;
  }
  avc::g_force_mb = rows_per_block;
  avc::g_force_nw = waves;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_lstm32_tune(int mode) {
  if (mode < 0 || mode > 4) {
    avc::set_error("avc_lstm32_tune: mode must be 0, 1 or 4 (2, 3: timing experiments, outputs invalid)");
    return AVC_ERR_INVALID;
  }
  avc::g_lstm32_mode = mode;
  ++avc::g_config_epoch;
  return AVC_OK;
}
