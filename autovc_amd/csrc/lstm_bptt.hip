// Persistent BPTT of the stacked LSTM layers (decoder.py:37,53 under autograd): every backward
// step of a layer direction in one launch (bptt_persist_kernel), and the XCD-local form of the
// H = 512 layer (bptt_xl_kernel).  Split from lstm_persist.hip in round 6 so that the forward
// recurrences can be compiled with the max-ILP machine scheduler while these kernels keep the
// default one (under max-ILP they spill VGPRs).
#include <algorithm>
#include <vector>

#define AVC_GIVEUP_TAG 0x20000000u  // (the vocoder tags 0x40000000, the fused BN 0x80000000)
#include "kernels.h"
#include "persist_internal.h"
#include "timing.h"

namespace avc {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
inline size_t al(size_t b) { return (b + 255) & ~size_t(255); }  // (scratch rounding, as lstm_persist.hip)

__device__ unsigned g_xl_seen[2];  // (avc_debug_xl_census) XCD-local BPTT workgroups that found their group local / not
int g_xl_remote = 0;  // avc_debug_xl_force_remote(): test the not-local fallback of the XCD-local BPTT

#ifdef AVC_STAMPS
// diagnostic build only: s_memtime per (workgroup, step, phase), written by thread 0
__device__ unsigned long long* g_pstamps = nullptr;
#endif

// ---- Persistent BPTT (backward recurrence of a stacked-LSTM layer as ONE launch) ----------
//
// The launch-per-step BPTT (lstm.hip: gemm_frag_partials + bptt_row_kernel) costs ~28 us per
// H = 1024 step at B = 256: two launches, a 16-split product whose workgroups re-stream their
// W_hh^T slice every step, and a per-row epilogue.  Here all T steps run in one launch of 256
// workgroups (one per CU), each with two roles per step:
//   phase A (product):  workgroup (rt, ct, sp) owns a 128 x 128 output tile (batch rows x hidden
//     units) over K-slice sp of the gate dimension; its W_hh^T slice (128 units x K/nsplit gates,
//     split hi/lo) stays in LDS for the whole launch.  It reads the split dG_{t+1} rows of its
//     tile and K-slice, multiplies (3xf16, like gemm16f), unscales each row by the row's scale
//     for that K-slice and stores the fp32 partial to slab[sp].
//   phase B (epilogue): workgroup (rb, q) owns 32 batch rows x U = H / nsplit hidden units,
//     i.e. exactly K-slice q of dG_t: it sums the nsplit partials (fixed order) into dh, does the
//     gate derivatives, dc, writes dG_t (fp32, for the weight gradients and dX) and splits dG_t
//     for the next step's product with a power-of-two scale per (row, K-slice) -- a scale that
//     is uniform over the slice a phase-A workgroup multiplies, so it factors out of the product.
// Hand-offs use the protocol of the forward persistent kernels (write-through stores of whole
// lines, drained before an agent-scope counter add; the consumer polls, then sc1 loads; epoch-
// tagged counters that are never reset; bounded spins with a give-up word).  Dependencies:
//   phase A (rt, ct, sp) at step k waits cntB[k-1][rt][sp] = 4 (the 4 row blocks of its K-slice),
//   phase B (rb, q) at step k waits cntA[k][rt][ct] = nsplit (every K-slice of its tile).
// Write-after-read safety: slab[sp] rows of tile rt are rewritten at step k+1 only after all of
// the tile's phase-B readers of step k counted in (cntB), and a split dG block is rewritten at
// step k+1 only after every phase-A reader of step k+1's tile counted in (cntA).
// a rounded sum that is never contracted with the product that formed v (the column sums of dG
// must not depend on the compiler's contraction choices in each BPTT kernel)
__device__ __forceinline__ float add_rounded(float s, float v) {
#pragma clang fp contract(off)
  return s + v;
}

// One element of the LSTM cell's backward (decoder.py's nn.LSTM under autograd): from dh (the
// output gradient plus the recurrent product), the carried dc and the saved activated gates i, f,
// g, o, tanh(c_t) and c_{t-1}: the next carried dc and the four gate-preactivation gradients.  Every
// product and sum rounded as written (no contraction), so every BPTT kernel that uses it forms the
// same bits whatever its surrounding code lets the compiler fuse.
__device__ __forceinline__ void lstm_cell_grad(float dh, float dcv, float ig, float fg, float gg, float og, float tc,
                                               float cpv, float& dc_next, float& di, float& df, float& dgg, float& dout) {
#pragma clang fp contract(off)
  const float dct = dh * og * (1.f - tc * tc) + dcv;
  dc_next = dct * fg;
  di = dct * gg * ig * (1.f - ig);
  df = dct * cpv * fg * (1.f - fg);
  dgg = dct * ig * (1.f - gg * gg);
  dout = dh * tc * og * (1.f - og);
}

// A phase-A partial of the BPTT product: (hi.hi + (hi.lo + lo.hi) / 2048) * unscale, rounded as
// written (the same bits in every BPTT kernel)
__device__ __forceinline__ float bptt_unscale(float part, float crs, float ie) {
#pragma clang fp contract(off)
  return (part + crs * (1.f / 2048.f)) * ie;
}

__device__ __forceinline__ float pow2_scale(float m) {  // max |x| -> [2^14, 2^15) (split_scale_of)
  if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, 15 - e);
}

struct BpttPArgs {
  int B, H, T, reverse, nsplit, nrt, ntn;
  const _Float16* whhT_s;   // W_hh^T permuted, fragment-major split ([H] rows x [4H] k), scale of amax_w
  const unsigned* amax_w;
  float* slab;              // [2][nsplit][B][H] unscaled partials (step parity)
  float* rowscale;          // [2][nsplit][B] power-of-two scale of split dG row b over K-slice q
  _Float16* dgs;            // [2] x fragment-major split dG ([B/32] row blocks x [4H] k)
  float* dc;                // [B][H] carried cell-state gradient
  const float* dy; long lddy;
  const float* gates;       // [T][B][4H] saved activated gates (permuted)
  const float* c;           // [T][B][H] saved cell states
  float* dg;                // [T][B][4H] output dG (permuted)
  unsigned* cnt;            // cntA [T][nrt][ntn] then cntB [T][nrt][nsplit], one 128-B line each
  unsigned* tmo;
  unsigned long long* tickets;
  unsigned* fail_host;
  int nwg;
  unsigned spin_limit;
  int diag;                 // timing experiments (avc_debug_bptt_diag), 0 in production
  float* colpart;           // [B/RB][4H] per-row-block column sums of dG over all steps (bias grads)
  unsigned* amax_dg;        // max |dG| over all steps (float bits; zeroed before the launch)
};

// NCH: 16-deep chunks per K-slice (4H / nsplit / 16); U = H / nsplit hidden units per phase-B
// workgroup (= 4 * NCH); NS = nsplit.  slab, rowscale and dgs are double-buffered by step parity:
// a buffer written at step k is rewritten at step k + 2 only, and the counter chain in between
// (B(k+1) waits on every K-slice of a tile, A(k+2) on B(k+1)) orders every reader of step k
// before that.
// BGF (round 4, avc_bptt_coalesce(1), the default): phase B's threads take the unit group as the
// fast index (tid = row * U/4 + group) instead of the row, so one wave instruction of the partial
// reads covers 64 / (U/4) rows x U*4 contiguous bytes -- whole 128-B lines -- where row-fastest
// lanes put every 16-B piece on a line of its own (4 KB apart) and each sc1 load fetched half a
// line.  The split dG for the next step, whose fragment layout is row-fastest, is then staged in
// LDS and stored as whole 256-B / 1-KB runs, and the bias column sums are combined over the rows
// through LDS once after the last step (a fixed row order).
template <int NCH, int NS, int RB, bool BGF = false>  // RB: batch rows per phase-B workgroup (16 or 32)
__global__ __launch_bounds__(512, 1) void bptt_persist_kernel(BpttPArgs a) {
  constexpr int U = 4 * NCH;
  constexpr int UG = U / 4;                  // 4-unit groups of a phase-B workgroup's slice
  constexpr int KS = 16 * NCH;               // gate columns per K-slice
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_b[];
  unsigned char* wl = lds_b;                 // [4 col tiles][NCH][hi, lo] 1 KiB blocks
  unsigned* rmax = reinterpret_cast<unsigned*>(lds_b + 4 * NCH * 2048);  // [32] row max (float bits)
  int* flag = reinterpret_cast<int*>(rmax + 32);                         // [4]

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int B = a.B, H = a.H, T = a.T, G4 = 4 * H, nkc = G4 / 16;
  constexpr int nsplit = NS;
  const long dgs_buf = (long)(B / 32) * nkc * 1024;  // halves per dgs buffer
  const int wg = blockIdx.x;
  // phase A role
  const int sp = wg % nsplit, tile = wg / nsplit, rt = tile / a.ntn, ct = tile % a.ntn;
  const int wm = w >> 1, wn = w & 1;         // 4 x 2 waves over the 128 x 128 tile (32 x 64 each)
  // phase B role (workgroups beyond the (row block, K-slice) pairs have none)
  const int nrb = B / RB;
  const bool has_b = wg < nrb * nsplit;
  const int rb = wg / nsplit, q = wg % nsplit;
  const int brt = rb * RB / 128;  // the 128-row tile of this workgroup's rows
  unsigned* cntA = a.cnt;
  unsigned* cntB = a.cnt + (long)T * a.nrt * a.ntn * 32;
  auto ia = [&](int k, int r, int c) { return (((long)k * a.nrt + r) * a.ntn + c) * 32; };
  auto ib = [&](int k, int r, int s2) { return (((long)k * a.nrt + r) * nsplit + s2) * 32; };

  // stationary W_hh^T slice: col tiles ct*4 .. ct*4+3, chunks sp*NCH .. sp*NCH+NCH-1
  for (int blk = w; blk < 4 * NCH * 2; blk += 8) {
    const int hl = blk & 1, c = (blk >> 1) % NCH, c4 = (blk >> 1) / NCH;
    const long src = (((long)(ct * 4 + c4) * nkc + sp * NCH + c) * 2 + hl) * 512;  // halves
    const f16x8 v = *reinterpret_cast<const f16x8*>(a.whhT_s + src + lane * 8);
    *reinterpret_cast<f16x8*>(wl + ((c4 * NCH + c) * 2 + hl) * 1024 + lane * 16) = v;
  }
  if (tid == 0) {
    const unsigned long long tk = __hip_atomic_fetch_add(a.tickets, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[2] = (int)(unsigned)(tk / (unsigned long long)a.nwg + 1ull);
  }
  __syncthreads();
  const unsigned E = (unsigned)flag[2];
  const float sw_inv = 1.f / pow2_scale(__uint_as_float(*a.amax_w));
  // phase B thread task: row r (of RB), unit group g4 (4 units = one 16-deep k chunk of the slice)
  const int br = BGF ? tid / UG : tid & (RB - 1), bg = BGF ? tid % UG : tid / RB;
  const bool b_task = has_b && (BGF ? br < RB : bg < UG);
  const int b_row = rb * RB + br;
  const int fr = b_row & 31;      // the row's lane in its 32-row fragment block
  const int j0 = q * U + bg * 4;           // first hidden unit of the task
  const int kq = q * KS + bg * 16;         // first (permuted) gate column of the task

  // this task's column sums of dG over all steps (registers, or LDS where the W slice leaves room:
  // the narrower-slice instances are at the VGPR limit) and its max |dG|
  constexpr bool CS_LDS = NCH < 16;
  float* csl = reinterpret_cast<float*>(flag + 4);  // [16][512] when CS_LDS
  // BGF: the split dG staging, [UG chunks][hi, lo][2 RB slots][16 B] (slot = k-half * RB + row)
  unsigned char* stg = reinterpret_cast<unsigned char*>(csl) + (CS_LDS ? 16 * 512 * 4 : 0);
  float csum[CS_LDS ? 1 : 16], dmax = 0.f;
  if constexpr (CS_LDS) {  // [512 threads][16] as 4 x 16-B vectors per thread
#pragma unroll
    for (int g = 0; g < 4; ++g) reinterpret_cast<f32x4*>(csl)[tid * 4 + g] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) csum[e] = 0.f;
  }
  int k = 0;
  bool ok = true;
  for (; k < T && ok; ++k) {
    const int st = T - 1 - k;
    const int t = a.reverse ? T - 1 - st : st;
    const int tp = a.reverse ? t + 1 : t - 1;
    // ---------------- phase A: slab[sp] = (dG_{t+1} . W_hh)[tile, K-slice sp] ----------------
    if (k > 0) {
      if (tid == 0) flag[0] = (a.diag & 4) ? 1 : wait_ge_ctl(cntB + ib(k - 1, rt, sp), E * (unsigned)(128 / RB), a.tmo, a.fail_host, a.spin_limit, E);
      __syncthreads();
      if (!flag[0]) { ok = false; break; }
      const int rblk = rt * 4 + wm;  // this wave's 32-row block
      const int rbuf = (k - 1) & 1;  // dG_{t+1}, written by phase B of step k - 1
      const auto ars = __builtin_amdgcn_make_buffer_rsrc(a.dgs + rbuf * dgs_buf + ((long)rblk * nkc + sp * NCH) * 1024,
                                                         0, NCH * 2048, 0x00020000);
      f32x16 part[2], crs[2];
#pragma unroll
      for (int jn = 0; jn < 2; ++jn)
#pragma unroll
        for (int e = 0; e < 16; ++e) part[jn][e] = crs[jn][e] = 0.f;
      // A chunks in batches of CB, the next batch's loads issued before this batch's MFMAs
      constexpr int CB = NCH < 4 ? NCH : 4;
      constexpr int NB = NCH / CB;
      f16x8 ah[2][CB], al[2][CB];
#define AVC_BP_LOAD(BI)                                                                           \
  _Pragma("unroll") for (int c = 0; c < CB; ++c) {                                                \
    if (a.diag & 1) { ah[(BI) & 1][c] = al[(BI) & 1][c] = f16x8{}; } else {                       \
    ah[(BI) & 1][c] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(ars, lane * 16, ((BI) * CB + c) * 2048, 16)); \
    al[(BI) & 1][c] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(ars, lane * 16, ((BI) * CB + c) * 2048 + 1024, 16)); } \
  }
      AVC_BP_LOAD(0)
#pragma unroll
      for (int bi = 0; bi < NB; ++bi) {
        if (bi + 1 < NB) { AVC_BP_LOAD(bi + 1) }
#pragma unroll
        for (int c = 0; c < CB; ++c) {
#pragma unroll
          for (int jn = 0; jn < 2; ++jn) {
            const unsigned char* pb = wl + (((wn * 2 + jn) * NCH + bi * CB + c) * 2) * 1024 + lane * 16;
            const f16x8 bh = *reinterpret_cast<const f16x8*>(pb);
            const f16x8 bl = *reinterpret_cast<const f16x8*>(pb + 1024);
            part[jn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[bi & 1][c], bh, part[jn], 0, 0, 0);
            crs[jn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[bi & 1][c], bl, crs[jn], 0, 0, 0);
            crs[jn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[bi & 1][c], bh, crs[jn], 0, 0, 0);
          }
        }
      }
#undef AVC_BP_LOAD
      // unscale row by row: 1 / (scale of this row's split over K-slice sp * scale of W)
      const int row0 = rt * 128 + wm * 32;
      const float rsv = lane < 32 ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                           __builtin_amdgcn_make_buffer_rsrc(a.rowscale + ((long)rbuf * nsplit + sp) * B + row0, 0, 128, 0x00020000),
                                                           lane * 4, 0, 16))
                                  : 1.f;
      const float inv = sw_inv / rsv;
      const auto srs = __builtin_amdgcn_make_buffer_rsrc(a.slab + ((long)(k & 1) * nsplit + sp) * B * H, 0, B * H * 4,
                                                         0x00020000);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int r = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const float ie = __shfl(inv, r);
#pragma unroll
        for (int jn = 0; jn < 2; ++jn) {
          const int col = ct * 128 + wn * 64 + jn * 32 + (lane & 31);
          const float v = bptt_unscale(part[jn][e], crs[jn][e], ie);
          if (!(a.diag & 8))
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), srs, ((row0 + r) * H + col) * 4, 0,
                                                  16 /*sc1*/);
        }
      }
      if (!(a.diag & 32)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        __hip_atomic_fetch_add((gu32*)(cntA + ia(k, rt, ct)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---------------- phase B: dG_t for rows rb, K-slice q -------------------------------------
    if (has_b) {
      // this step's own operands (written before the launch, or by this workgroup) are loaded
      // before the wait for the partials
      const long tb = (long)t * B + b_row;
      f32x4 dyv = {}, ig = {}, fg = {}, gg = {}, og = {}, cc = {}, cpv = {}, dcv = {};
      if (b_task) {
        dyv = *reinterpret_cast<const f32x4*>(a.dy + (long)t * B * a.lddy + (long)b_row * a.lddy + j0);
        const float* gp = a.gates + tb * G4 + kq;
        ig = *reinterpret_cast<const f32x4*>(gp);
        fg = *reinterpret_cast<const f32x4*>(gp + 4);
        gg = *reinterpret_cast<const f32x4*>(gp + 8);
        og = *reinterpret_cast<const f32x4*>(gp + 12);
        cc = *reinterpret_cast<const f32x4*>(a.c + tb * H + j0);
        if (st > 0) cpv = *reinterpret_cast<const f32x4*>(a.c + ((long)tp * B + b_row) * H + j0);
        dcv = *reinterpret_cast<f32x4*>(a.dc + (long)b_row * H + j0);
      }
      if (k > 0) {
        if (tid == 0)
          flag[1] = (a.diag & 4) ? 1 : wait_ge_ctl(cntA + ia(k, brt, (q * U) / 128), E * (unsigned)nsplit, a.tmo, a.fail_host,
                                a.spin_limit, E);
        if (tid < 32) rmax[tid] = 0u;
        __syncthreads();
        if (!flag[1]) { ok = false; break; }
      } else {
        if (tid < 32) rmax[tid] = 0u;
        __syncthreads();
      }
      float d[16];
      float mx = 0.f;
      if (b_task) {
        f32x4 rec = {0.f, 0.f, 0.f, 0.f};
        if (k > 0) {
          const auto srs = __builtin_amdgcn_make_buffer_rsrc(a.slab + (long)(k & 1) * nsplit * B * H, 0,
                                                             nsplit * B * H * 4, 0x00020000);
          constexpr int SB = NS < 16 ? NS : 16;  // partials in flight per batch (registers)
#pragma unroll
          for (int s0 = 0; s0 < NS; s0 += SB) {
            f32x4 pv[SB];
#pragma unroll
            for (int s2 = 0; s2 < SB; ++s2)
              pv[s2] = (a.diag & 2) ? f32x4{} : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     srs, (int)((((long)(s0 + s2) * B + b_row) * H + j0) * 4), 0, 16));
#pragma unroll
            for (int s2 = 0; s2 < SB; ++s2) rec += pv[s2];  // fixed split order
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float dh = dyv[u] + rec[u];
          const float tc = gate_tanh(cc[u]);  // as the forward epilogue formed it
          float dn;
          lstm_cell_grad(dh, dcv[u], ig[u], fg[u], gg[u], og[u], tc, cpv[u], dn, d[u], d[4 + u], d[8 + u], d[12 + u]);
          dcv[u] = dn;
        }
        float* go = a.dg + tb * G4 + kq;
        if (!(a.diag & 16)) {  // (stores issued after the hand-off measured slower: 15.8 -> 16.7 us
                               // per H = 1024 step -- vmcnt is in order, so the next phase's loads
                               // wait for them anyway)
          *reinterpret_cast<f32x4*>(a.dc + (long)b_row * H + j0) = dcv;
#pragma unroll
          for (int g = 0; g < 4; ++g)
            *reinterpret_cast<f32x4*>(go + 4 * g) = f32x4{d[4 * g], d[4 * g + 1], d[4 * g + 2], d[4 * g + 3]};
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          mx = fmaxf(mx, fabsf(d[e]));
          if constexpr (!CS_LDS) csum[e] = add_rounded(csum[e], d[e]);
        }
        if constexpr (CS_LDS) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            f32x4* p4 = reinterpret_cast<f32x4*>(csl) + tid * 4 + g;
            f32x4 cs4 = *p4;
#pragma unroll
            for (int j = 0; j < 4; ++j) cs4[j] = add_rounded(cs4[j], d[4 * g + j]);
            *p4 = cs4;
          }
        }
        dmax = fmaxf(dmax, mx);
        atomicMax(rmax + br, __float_as_uint(mx));
      }
      __syncthreads();
      if (st > 0) {  // the split for the next step's product (none after the last step)
        if (b_task) {
          const float sb = pow2_scale(__uint_as_float(rmax[br]));
          // chunk kq / 16 of row block rb: lanes (row) and (row + 32) hold k 0-7 and 8-15
          typedef _Float16 h8 __attribute__((ext_vector_type(8)));
          h8 hi0, lo0, hi1, lo1;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v0 = d[e] * sb, v1 = d[8 + e] * sb;
            const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
            hi0[e] = h0; lo0[e] = (_Float16)((v0 - (float)h0) * 2048.0f);
            hi1[e] = h1; lo1[e] = (_Float16)((v1 - (float)h1) * 2048.0f);
          }
          if constexpr (BGF) {  // into the staging image; stored below as whole runs
            unsigned char* sp = stg + (long)bg * 2 * (2 * RB) * 16;
            *reinterpret_cast<h8*>(sp + (0 * RB + br) * 16) = hi0;
            *reinterpret_cast<h8*>(sp + (1 * RB + br) * 16) = hi1;
            *reinterpret_cast<h8*>(sp + (2 * RB + br) * 16) = lo0;
            *reinterpret_cast<h8*>(sp + (3 * RB + br) * 16) = lo1;
          } else {
          const auto drs = __builtin_amdgcn_make_buffer_rsrc(
              a.dgs + (k & 1) * dgs_buf + ((long)(b_row >> 5) * nkc + kq / 16) * 1024, 0, 2048, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi0), drs, fr * 16, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi1), drs, (fr + 32) * 16, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo0), drs, 1024 + fr * 16, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo1), drs, 1024 + (fr + 32) * 16, 0, 16);
          }
          if (bg == 0) {
            const auto rrs = __builtin_amdgcn_make_buffer_rsrc(a.rowscale + ((long)(k & 1) * nsplit + q) * B + rb * RB, 0,
                                                               RB * 4, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, sb), rrs, br * 4, 0, 16);
          }
        }
        if constexpr (BGF) {
          // the staged split dG as whole runs: piece p -> (chunk, hi/lo, slot); slot s = half * RB + r
          // lands at fragment lane half * 32 + ((rb * RB) & 31) + r of block (row block, chunk)
          __syncthreads();
          constexpr int PIECES = UG * 2 * 2 * RB;
          for (int p = tid; p < PIECES; p += 512) {
            const int sl = p % (2 * RB), hl = (p / (2 * RB)) & 1, c = p / (4 * RB);
            const int lane_g = (sl / RB) * 32 + ((rb * RB) & 31) + sl % RB;
            const u32x4 v = *reinterpret_cast<const u32x4*>(stg + (long)p * 16);
            const auto drs = __builtin_amdgcn_make_buffer_rsrc(
                a.dgs + (k & 1) * dgs_buf + ((long)((rb * RB) >> 5) * nkc + q * NCH + c) * 1024, 0, 2048, 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(v, drs, hl * 1024 + lane_g * 16, 0, 16);
          }
        }
        if (!(a.diag & 32)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
          __hip_atomic_fetch_add((gu32*)(cntB + ib(k, brt, q)), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // the bias gradients' column sums (32 rows of this block: lanes 0-31 / 32-63 of a wave are the
  // rows of two unit groups) and max |dG| for the weight-gradient products' operand scale
  if (ok && has_b) {
    if constexpr (BGF) {
      // rows are spread over waves: every task's 16 sums into LDS (the W slice is free now), then
      // thread (group, e) adds its column over the RB rows in row order
      __syncthreads();
      float* red = reinterpret_cast<float*>(wl);  // [512][16]
      if (b_task) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if constexpr (CS_LDS) red[tid * 16 + e] = csl[tid * 16 + e];
          else red[tid * 16 + e] = csum[e];
        }
      }
      __syncthreads();
      if (tid < UG * 16) {
        const int g = tid / 16, e = tid % 16;
        float v = 0.f;
        for (int r = 0; r < RB; ++r) v += red[(r * UG + g) * 16 + e];
        a.colpart[(long)rb * G4 + q * KS + g * 16 + e] = v;
      }
    } else {
    float cs[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if constexpr (CS_LDS) cs[e] = csl[tid * 16 + e];
      else cs[e] = csum[e];
      for (int o = RB / 2; o > 0; o >>= 1) cs[e] += __shfl_xor(cs[e], o);
    }
    if (b_task && br == 0) {
      float* cp = a.colpart + (long)rb * G4 + kq;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(cp + 4 * g) = f32x4{cs[4 * g], cs[4 * g + 1], cs[4 * g + 2], cs[4 * g + 3]};
    }
    }
    for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o));
    if (lane == 0) atomicMax(a.amax_dg, __float_as_uint(dmax));
  }
  // gave up at step k: this workgroup's dG slices of the remaining steps are NaN (never plausible)
  if (!ok && b_task) {
    for (int kk = k; kk < T; ++kk) {
      const int st = T - 1 - kk;
      const int t = a.reverse ? T - 1 - st : st;
      float* go = a.dg + ((long)t * B + b_row) * G4 + kq;
      for (int e = 0; e < 16; ++e) go[e] = __builtin_nanf("");
    }
  }
}

// ---- XCD-local BPTT of an H = 512 layer (decoder.lstm1; round 5, avc_bptt_xcd) ---------------
//
// bptt_persist_kernel's 128-row tiles make every step two all-to-all hand-offs across the chip (the
// split dG rows to the product owners, the partials back to the epilogue owners), each a
// write-through drain, a counter and a poll.  At H = 512 the split W_hh^T is 4 MB: one XCD's 32
// CUs hold all of it in LDS (128 KB each), so a group of 32 batch rows can run its whole BPTT on
// one XCD, and the batch (rows never interact) splits into up to 8 such groups.  Workgroup bid is
// (group g = bid % 8, K-slice q = bid / 8): under the round-robin deal each group lands on one XCD
// (checked at run time, as PersistArgs::xl).  Workgroup q of group g
//   phase A: (dG_{t+1} . W_hh)[32 rows, all 512 units] over K-slice q (64 permuted gate columns =
//            4 chunks of 16) -> the fp32 partial slab[q] (8 waves x 64 units);
//   phase B: rows x units 16q .. 16q + 15: sums the 32 partials (fixed order), gate derivatives,
//            dc (kept in registers), dG_t out, and splits dG_t over exactly K-slice q -- the operand
//            of its OWN next phase A, so the split goes to LDS and that hand-off disappears.
// One hand-off per step (partials, phase A -> phase B), inside one XCD: plain stores that stay in
// its L2, a per-group line of tags (one word per workgroup, written after the drain; polled by one
// wave, one load for all 32), sc1 loads.  A group that is not on one XCD uses sc1 stores and an
// agent-scope counter per (step, group) instead -- the forward kernels' protocol.  The products
// (same chunks, same MFMA order), the per-(row, K-slice) split scales, the partial order and the
// epilogue are bptt_persist_kernel<4, 32, 32, true>'s, so dG, the column sums and max |dG| are
// the same bits.
struct BpttXArgs {
  int B, T, reverse, ngrp;
  const _Float16* whhT_s;   // W_hh^T permuted, fragment-major split ([512] rows x [2048] k)
  const unsigned* amax_w;
  float* slab;              // [2][32][B][512] partials (step parity, K-slice)
  const float* dy; long lddy;
  const float* gates;       // [T][B][2048] saved activated gates (permuted)
  const float* c;           // [T][B][512] saved cell states
  float* dg;                // [T][B][2048] output dG (permuted)
  float* colpart;           // [B/32][2048] per-group column sums of dG (bias gradients)
  unsigned* amax_dg;        // max |dG| over all steps (float bits; zeroed before the launch)
  unsigned* tags;           // [8 groups][32] tag lines (local groups)
  unsigned* xl_tab;         // [256] epoch-tagged XCD of each workgroup
  unsigned* cnt;            // [T][8] counter lines (groups that are not on one XCD)
  unsigned* tmo;
  unsigned long long* tickets;
  unsigned* fail_host;
  unsigned spin_limit;
  int xl_remote;            // (avc_debug_xl_force_remote) treat every group as not local
};

constexpr int kBxNch = 4;  // 16-deep chunks per K-slice (2048 gates / 32 slices / 16)
#ifdef AVC_STAMPS
#define AVC_BXSTAMP(slot)                                                                         \
  do {                                                                                            \
    unsigned long long _t;                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (g_pstamps && tid == 0) g_pstamps[((long)blockIdx.x * T + k) * 8 + (slot)] = _t;           \
  } while (0)
#else
#define AVC_BXSTAMP(slot) do { } while (0)
#endif
size_t bptt_xl_lds() { return (size_t)16 * kBxNch * 2048 + kBxNch * 2048 + 32 * 4 + 8 * 4; }

__global__ __launch_bounds__(512, 1) void bptt_xl_kernel(BpttXArgs a) {
  constexpr int H = 512, G4 = 2048, nkc = G4 / 16, NCH = kBxNch, KS = 64, RB = 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds_x[];
  unsigned char* wl = lds_x;                                 // [16 unit tiles][NCH][hi, lo] 1 KiB blocks
  unsigned char* dgl = lds_x + 16 * NCH * 2048;              // [NCH][hi, lo] 1 KiB: this slice's split dG
  float* rsl = reinterpret_cast<float*>(dgl + NCH * 2048);   // [32] the rows' split scales
  int* flag = reinterpret_cast<int*>(rsl + 32);              // [8]

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int B = a.B, T = a.T;
  const int g = blockIdx.x & 7, q = blockIdx.x >> 3;
  if (tid == 0) {  // every workgroup takes a ticket (the epoch counts the whole grid)
    const unsigned long long tk = __hip_atomic_fetch_add(a.tickets, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[2] = (int)(unsigned)(tk / 256ull + 1ull);
  }
  __syncthreads();
  const unsigned E = (unsigned)flag[2];
  if (g >= a.ngrp) return;

  // the group's 32 workgroups record their XCD and check that they share one (bounded)
  if (tid < 64) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (tid == 0)
      __hip_atomic_store((gu32*)(a.xl_tab + blockIdx.x), (E << 4) | (xcc & 7u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool same = true, done = false;
    for (unsigned spins = 0; !done; ++spins) {
      bool all = true;
      same = true;
      if (lane < 32) {
        const unsigned v = __hip_atomic_load((gu32*)(a.xl_tab + lane * 8 + g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        all = (v >> 4) == (E & 0x0fffffffu);
        same = (v & 7u) == (xcc & 7u);
      }
      done = __builtin_amdgcn_ballot_w64(!all) == 0ull;
      if (!done && spin_give_up_ctl(spins, a.tmo, a.fail_host, a.spin_limit, E, lane)) break;
      if (!done) __builtin_amdgcn_s_sleep(2);
    }
    const bool loc = done && __builtin_amdgcn_ballot_w64(!same) == 0ull;
    if (tid == 0) {
      flag[3] = loc ? 1 : 0;
      flag[4] = done ? 1 : 0;
    }
  }
  // stationary W_hh^T slice: every unit tile, chunks q * NCH .. q * NCH + NCH - 1
  for (int blk = w; blk < 16 * NCH * 2; blk += 8) {
    const int hl = blk & 1, c = (blk >> 1) % NCH, ut = (blk >> 1) / NCH;
    const long src = (((long)ut * nkc + q * NCH + c) * 2 + hl) * 512;  // halves
    const f16x8 v = *reinterpret_cast<const f16x8*>(a.whhT_s + src + lane * 8);
    *reinterpret_cast<f16x8*>(wl + ((ut * NCH + c) * 2 + hl) * 1024 + lane * 16) = v;
  }
  __syncthreads();
  const bool loc = flag[3] != 0 && !a.xl_remote;
  bool ok = flag[4] != 0;
  if (tid == 0) atomicAdd(&g_xl_seen[loc ? 0 : 1], 1u);
  const float sw_inv = 1.f / pow2_scale(__uint_as_float(*a.amax_w));
  const auto trs = __builtin_amdgcn_make_buffer_rsrc(a.tags + g * 32, 0, 128, 0x00020000);

  // phase B task: row br of the group, hidden unit uu of the slice (every thread: 32 x 16); the
  // unit's four gate columns i, f, g, o sit at bg * 16 + {u, 4 + u, 8 + u, 12 + u} of the slice
  const int br = tid >> 4, uu = tid & 15, bg = uu >> 2, u = uu & 3;
  const int b_row = g * RB + br;
  const int j = q * 16 + uu;        // the task's hidden unit
  const int kq = q * KS + bg * 16;  // the task's 16-column chunk of (permuted) gate columns
  float csum[4] = {0.f, 0.f, 0.f, 0.f}, dmax = 0.f;
  float dcv = 0.f;  // the carried cell-state gradient of the task's unit

  int k = 0;
  for (; k < T && ok; ++k) {
    const int st = T - 1 - k;
    const int t = a.reverse ? T - 1 - st : st;
    const int tp = a.reverse ? t + 1 : t - 1;
    const int par = k & 1;
    AVC_BXSTAMP(0);
    // ---------------- phase A: slab[q] = (dG_{t+1} . W_hh)[group rows, all units] over slice q ----
    if (k > 0) {
      f32x16 part[2], crs[2];
#pragma unroll
      for (int jn = 0; jn < 2; ++jn)
#pragma unroll
        for (int e = 0; e < 16; ++e) part[jn][e] = crs[jn][e] = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const f16x8 ah = *reinterpret_cast<const f16x8*>(dgl + (c * 2 + 0) * 1024 + lane * 16);
        const f16x8 al = *reinterpret_cast<const f16x8*>(dgl + (c * 2 + 1) * 1024 + lane * 16);
#pragma unroll
        for (int jn = 0; jn < 2; ++jn) {
          const unsigned char* pb = wl + (((w * 2 + jn) * NCH + c) * 2) * 1024 + lane * 16;
          const f16x8 bh = *reinterpret_cast<const f16x8*>(pb);
          const f16x8 bl = *reinterpret_cast<const f16x8*>(pb + 1024);
          part[jn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, part[jn], 0, 0, 0);
          crs[jn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, crs[jn], 0, 0, 0);
          crs[jn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, crs[jn], 0, 0, 0);
        }
      }
      AVC_BXSTAMP(1);
      // unscale row by row: 1 / (scale of this row's split over slice q * scale of W)
      const float rsv = lane < 32 ? rsl[lane] : 1.f;
      const float inv = sw_inv / rsv;
      const auto srs = __builtin_amdgcn_make_buffer_rsrc(a.slab + ((long)par * 32 + q) * B * H + (long)g * RB * H, 0,
                                                         RB * H * 4, 0x00020000);
      // (the cache policy is an immediate: plain for a local group, sc1 otherwise)
#define AVC_BX_STORE(POL)                                                                         \
  _Pragma("unroll") for (int e = 0; e < 16; ++e) {                                                \
    const int r = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);                                       \
    const float ie = __shfl(inv, r);                                                              \
    _Pragma("unroll") for (int jn = 0; jn < 2; ++jn) {                                            \
      const int col = (w * 2 + jn) * 32 + (lane & 31);                                            \
      const float v = bptt_unscale(part[jn][e], crs[jn][e], ie);                                  \
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), srs, (r * H + col) * 4, 0, POL); \
    }                                                                                             \
  }
      if (loc) {
        AVC_BX_STORE(0)
      } else {
        AVC_BX_STORE(16)
      }
#undef AVC_BX_STORE
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      AVC_BXSTAMP(2);
      if (tid == 0) {
        if (loc)  // this workgroup's tag for step k, after every wave's drain
          __builtin_amdgcn_raw_buffer_store_b32(E * (unsigned)(T + 1) + (unsigned)k, trs, q * 4, 0, 0);
        else
          __hip_atomic_fetch_add((gu32*)(a.cnt + ((long)k * 8 + g) * 32), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // ---------------- phase B: dG_t for the group's rows, slice q ----------------------------------
    // (one element per thread: each sums its 32 partials in slice order with one round of loads)
    const long tb = (long)t * B + b_row;
    const float* gp = a.gates + tb * G4 + kq + u;
    const float dyv = a.dy[(long)t * B * a.lddy + (long)b_row * a.lddy + j];
    const float ig = gp[0], fg = gp[4], gg = gp[8], og = gp[12];
    const float cc = a.c[tb * H + j];
    const float cpv = st > 0 ? a.c[((long)tp * B + b_row) * H + j] : 0.f;
    if (k > 0) {
      if (tid < 64) {  // wave 0: every phase A of the group at step k
        bool good = true;
        if (loc) {
          const unsigned want = E * (unsigned)(T + 1) + (unsigned)k;
          auto ld = [&]() { return lane < 32 ? __builtin_amdgcn_raw_buffer_load_b32(trs, lane * 4, 0, 16 /*sc1*/) : want; };
          unsigned v = ld();
          for (unsigned spins = 0; __builtin_amdgcn_ballot_w64((int)(v - want) < 0) != 0ull; ++spins) {
            if (spin_give_up_ctl(spins, a.tmo, a.fail_host, a.spin_limit, E, lane)) {
              good = false;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
            v = ld();
          }
        } else if (lane == 0) {
          good = wait_ge_ctl(a.cnt + ((long)k * 8 + g) * 32, E * 32u, a.tmo, a.fail_host, a.spin_limit, E);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler ordering only)
        if (lane == 0) flag[1] = good ? 1 : 0;
      }
      __syncthreads();
      if (!flag[1]) { ok = false; break; }
    } else {
      __syncthreads();
    }
    AVC_BXSTAMP(3);
    float rec = 0.f;
    if (k > 0) {
      const auto srs = __builtin_amdgcn_make_buffer_rsrc(a.slab + (long)par * 32 * B * H, 0, 32 * B * H * 4, 0x00020000);
      float pv[32];
#pragma unroll
      for (int s2 = 0; s2 < 32; ++s2)
        pv[s2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                               srs, (int)((((long)s2 * B + b_row) * H + j) * 4), 0, 16 /*sc1*/));
#pragma unroll
      for (int s2 = 0; s2 < 32; ++s2) rec += pv[s2];  // fixed slice order
    }
    AVC_BXSTAMP(4);
    const float dh = dyv + rec;
    const float tc = gate_tanh(cc);  // as the forward epilogue formed it
    float d[4], dn;
    lstm_cell_grad(dh, dcv, ig, fg, gg, og, tc, cpv, dn, d[0], d[1], d[2], d[3]);
    dcv = dn;
    float* go = a.dg + tb * G4 + kq + u;
    float mx = 0.f;
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) {
      go[4 * gi] = d[gi];
      mx = fmaxf(mx, fabsf(d[gi]));
      csum[gi] = add_rounded(csum[gi], d[gi]);
    }
    dmax = fmaxf(dmax, mx);
    AVC_BXSTAMP(5);
    // the row's max over its 16 units: the 16 lanes of this row in this wave (float bits compare
    // as the magnitudes do)
    unsigned mxu = __float_as_uint(mx);
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) mxu = max(mxu, (unsigned)__shfl_xor((int)mxu, o));
    AVC_BXSTAMP(6);
    if (st > 0) {  // the split for this workgroup's next phase A (none after the last step)
      const float sb = pow2_scale(__uint_as_float(mxu));
      // chunk bg of the slice: lane (row) holds k 0-7 (i, f of the chunk's 4 units), lane (row + 32)
      // k 8-15 (g, o): this unit's i / f at elements u / 4 + u of the first, g / o of the second
#pragma unroll
      for (int gi = 0; gi < 4; ++gi) {
        const float v = d[gi] * sb;
        const _Float16 hv = (_Float16)v;
        const _Float16 lv = (_Float16)((v - (float)hv) * 2048.0f);
        const int off = (br + 32 * (gi >> 1)) * 16 + ((gi & 1) * 4 + u) * 2;
        *reinterpret_cast<_Float16*>(dgl + (bg * 2 + 0) * 1024 + off) = hv;
        *reinterpret_cast<_Float16*>(dgl + (bg * 2 + 1) * 1024 + off) = lv;
      }
      if (uu == 0) rsl[br] = sb;
      __syncthreads();
    }
    AVC_BXSTAMP(7);
  }
  // the bias gradients' column sums over the group's rows (row order, through LDS: the W slice is
  // free now) and max |dG| for the weight-gradient products' operand scale
  if (ok) {
    __syncthreads();
    float* red = reinterpret_cast<float*>(wl);  // [32 rows][64 columns of the slice]
#pragma unroll
    for (int gi = 0; gi < 4; ++gi) red[br * KS + bg * 16 + gi * 4 + u] = csum[gi];
    __syncthreads();
    if (tid < KS) {
      float v = 0.f;
      for (int r = 0; r < RB; ++r) v += red[r * KS + tid];
      a.colpart[(long)g * G4 + q * KS + tid] = v;
    }
    for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o));
    if (lane == 0) atomicMax(a.amax_dg, __float_as_uint(dmax));
  }
  // gave up at step k: this workgroup's dG columns of the remaining steps are NaN (never plausible)
  if (!ok) {
    for (int kk = k; kk < T; ++kk) {
      const int st = T - 1 - kk;
      const int t = a.reverse ? T - 1 - st : st;
      float* go = a.dg + ((long)t * B + b_row) * G4 + kq + u;
      for (int gi = 0; gi < 4; ++gi) go[4 * gi] = __builtin_nanf("");
    }
  }
}

// (+ the BGF staging of the split dG: UG x 2 x 2 RB x 16 B = 16 KB at every instance)
size_t bptt_lds(int nch) { return (size_t)4 * nch * 2048 + 32 * 4 + 16 + (nch < 16 ? 16 * 512 * 4 : 0) + 16 * 1024; }

int g_bptt_bgf = 1;  // avc_bptt_coalesce(): phase B unit-group-fastest (coalesced partial reads; C3 35.24 -> 34.92 ms)

// epilogue rows per workgroup: 16 where 32-row blocks would leave half the workgroups without an
// epilogue (nsplit = 16), else 32
int bptt_rb(int ns) { return ns == 16 ? 16 : 32; }

const void* bptt_fn(int nch, int ns) {
  if (g_bptt_bgf) {
    if (nch == 16 && ns == 16) return (const void*)bptt_persist_kernel<16, 16, 16, true>;
    if (nch == 8 && ns == 32) return (const void*)bptt_persist_kernel<8, 32, 32, true>;
    if (nch == 4 && ns == 32) return (const void*)bptt_persist_kernel<4, 32, 32, true>;
    return nullptr;
  }
  if (nch == 16 && ns == 16) return (const void*)bptt_persist_kernel<16, 16, 16>;
  if (nch == 8 && ns == 32) return (const void*)bptt_persist_kernel<8, 32, 32>;
  if (nch == 4 && ns == 32) return (const void*)bptt_persist_kernel<4, 32, 32>;
  return nullptr;
}

// the tiling of a (B, H) problem: 128 x 128 tiles x nsplit K-slices = 256 workgroups
bool bptt_plan(int B, int H, int& nrt, int& ntn, int& ns, int& nch) {
  if (B % 128 || H % 128 || B > 256) return false;
  nrt = B / 128;
  ntn = H / 128;
  if (256 % (nrt * ntn)) return false;
  ns = 256 / (nrt * ntn);
  if ((4 * H) % (16 * ns)) return false;
  nch = 4 * H / 16 / ns;
  return bptt_fn(nch, ns) != nullptr;
}

}  // namespace

unsigned bptt_giveup_count() {
  unsigned v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_persist_giveups), sizeof(unsigned), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return v;
}

#ifdef AVC_STAMPS
int bptt_set_stamps(void* buf) {
  AVC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_pstamps), &buf, sizeof(void*), 0, hipMemcpyHostToDevice));
  return AVC_OK;
}
#endif

int g_bptt_persist = 1;  // avc_bptt_persist(): the persistent BPTT where eligible
int g_bptt_diag = 0;     // avc_debug_bptt_diag(): timing experiments (results invalid when set)

bool bptt_xl_eligible(int B, int H);
int g_bptt_xl = 1;  // avc_bptt_xcd(): the XCD-local form for H = 512 (bptt_xl_kernel); 2 = also other batches

bool bptt_persist_eligible(int T, int B, int H) {
  int nrt, ntn, ns, nch;
  if (!g_bptt_persist || T < 2) return false;
  // (avc_bptt_xcd(2): any batch of whole 32-row groups, up to 8 of them; by default only the
  // batches the 128-row form takes, whose results it reproduces bit for bit)
  if (g_bptt_xl == 2 && bptt_xl_eligible(B, H)) return true;
  if (!bptt_plan(B, H, nrt, ntn, ns, nch)) return false;
  struct Entry { const void* fn; int dev; int cap; };
  static std::vector<Entry> cache;
  const void* fn = bptt_fn(nch, ns);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  int cap = -1;
  for (const auto& e : cache)
    if (e.fn == fn && e.dev == dev) cap = e.cap;
  if (cap < 0) {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bptt_lds(nch));
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 512, bptt_lds(nch)) != hipSuccess) {
      (void)hipGetLastError();
      per_cu = 0;
    }
    cap = per_cu * coresident_cus();
    cache.push_back({fn, dev, cap});
  }
  return cap >= 256;  // every workgroup co-resident
}

int bptt_colpart_rows(int B, int H) {
  int nrt, ntn, ns, nch;
  if (bptt_xl_eligible(B, H)) return B / 32;
  return bptt_plan(B, H, nrt, ntn, ns, nch) ? B / bptt_rb(ns) : 0;
}

size_t bptt_persist_scratch(int B, int H) {
  int nrt, ntn, ns, nch;
  if (bptt_xl_eligible(B, H)) return al((size_t)2 * 32 * B * H * sizeof(float)) + 4096;
  if (!bptt_plan(B, H, nrt, ntn, ns, nch)) return 0;
  return al((size_t)2 * ns * B * H * sizeof(float)) + al((size_t)2 * ns * B * sizeof(float)) +
         al((size_t)2 * (B / 32) * (4 * H / 16) * 2048) + al((size_t)B * H * sizeof(float)) + 4096;
}


// The XCD-local form takes an H = 512 layer whose batch splits into at most 8 groups of 32 rows,
// on a 256-CU device that holds the grid (one 512-thread, 136 KB-LDS workgroup per CU).
bool bptt_xl_eligible(int B, int H) {
  if (!g_bptt_xl || H != 512 || B % 32 || B > 256 || coresident_cus() != 256) return false;
  static int cap = -1;  // (one instance; the device count is checked above)
  if (cap < 0) {
    const void* fn = reinterpret_cast<const void*>(&bptt_xl_kernel);
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bptt_xl_lds());
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 512, bptt_xl_lds()) != hipSuccess) {
      (void)hipGetLastError();
      per_cu = 0;
    }
    cap = per_cu * coresident_cus();
  }
  return cap >= 256;
}

int bptt_xl_run(avc_context* ctx, int T, int B, int reverse, const _Float16* whhT_s, const unsigned* amax_w,
                const float* d_y, long ldy, const float* gates, const float* c, float* dg, float* colpart,
                unsigned* amax_dg, hipStream_t s) {
  constexpr int H = 512;
  Scratch sc(ctx);
  AVC_TAKE(slab, float, (size_t)2 * 32 * B * H, sc);
  unsigned* region = nullptr;
  // tag lines [8][32], the XCD table [256], counter lines [T][8][32]
  const size_t words = 8 * 32 + 256 + (size_t)T * 8 * 32;
  AVC_TRY(persist_region_t(ctx, 4, T, 8, 32, 256, words, s, &region));
  BpttXArgs a{};
  a.B = B; a.T = T; a.reverse = reverse; a.ngrp = B / 32;
  a.whhT_s = whhT_s; a.amax_w = amax_w; a.slab = slab;
  a.dy = d_y; a.lddy = ldy; a.gates = gates; a.c = c; a.dg = dg;
  a.colpart = colpart; a.amax_dg = amax_dg;
  AVC_TRY(zero_async(amax_dg, sizeof(unsigned), s));
  a.tickets = reinterpret_cast<unsigned long long*>(region);
  a.tmo = region + 32;
  a.tags = region + kRegionHeaderWords;
  a.xl_tab = a.tags + 8 * 32;
  a.cnt = a.xl_tab + 256;
  a.fail_host = ctx->fail_host;
  a.spin_limit = coresident_spin_limit();
  a.xl_remote = g_xl_remote;
  if (persist_inject_take()) a.spin_limit = 0;
  void* args[] = {&a};
  hipEvent_t ev = timing_begin(TC_LSTM_STEP_BWD, s);
  AVC_TRY(coresident_dispatch(ctx, reinterpret_cast<const void*>(&bptt_xl_kernel), dim3(256), dim3(512), args,
                           bptt_xl_lds(), s));
  if (ev) {
    // the recurrent products of T - 1 steps; algorithmic bytes: the partials written and read per
    // step (the split dG stays in LDS), the epilogue operands, dG written
    const double flops = (double)(T - 1) * 2.0 * B * H * 4.0 * H;
    const double bytes = (double)(T - 1) * 2.0 * 4.0 * 32 * B * H + (double)T * 4.0 * B * H * 12.0;
    timing_end(TC_LSTM_STEP_BWD, ev, s, flops, bytes);
  }
  return AVC_OK;
}

// BPTT of one LSTM layer direction over all T steps as one launch (see bptt_persist_kernel).
// whhT_s / amax_w: W_hh^T permuted and split (lstm.hip); d_y [T][B] rows (ldy), gates / c the
// forward's saved activations, dg [T][B][4H] output; colpart [bptt_colpart_rows(B, H)][4H] the
// column sums of dG per epilogue row block (the bias gradients' partials), *amax_dg = max |dG|
// (both over all steps).
int bptt_persist_run(avc_context* ctx, int T, int B, int H, int reverse, const _Float16* whhT_s,
                     const unsigned* amax_w, const float* d_y, long ldy, const float* gates, const float* c,
                     float* dg, float* colpart, unsigned* amax_dg, hipStream_t s) {
  int nrt, ntn, ns, nch;
  AVC_CHECK_ARG(bptt_persist_eligible(T, B, H), "persistent BPTT: not eligible for this shape");
  AVC_TRY(persist_guard(ctx));
  if (bptt_xl_eligible(B, H))
    return bptt_xl_run(ctx, T, B, reverse, whhT_s, amax_w, d_y, ldy, gates, c, dg, colpart, amax_dg, s);
  AVC_CHECK_ARG(bptt_plan(B, H, nrt, ntn, ns, nch), "persistent BPTT: not eligible for this shape");
  Scratch sc(ctx);
  AVC_TAKE(slab, float, (size_t)2 * ns * B * H, sc);
  AVC_TAKE(rowscale, float, (size_t)2 * ns * B, sc);
  AVC_TAKE(dgs, _Float16, (size_t)2 * (B / 32) * (4 * H / 16) * 1024, sc);
  AVC_TAKE(dc, float, (size_t)B * H, sc);
  AVC_TRY(zero_async(dc, sizeof(float) * B * H, s));
  unsigned* region = nullptr;
  const size_t words = ((size_t)T * nrt * ntn + (size_t)T * nrt * ns) * 32;
  AVC_TRY(persist_region_t(ctx, 3, T, nrt, ntn, 256, words, s, &region));
  BpttPArgs a{};
  a.B = B; a.H = H; a.T = T; a.reverse = reverse; a.nsplit = ns; a.nrt = nrt; a.ntn = ntn;
  a.whhT_s = whhT_s; a.amax_w = amax_w; a.slab = slab; a.rowscale = rowscale; a.dgs = dgs; a.dc = dc;
  a.dy = d_y; a.lddy = ldy; a.gates = gates; a.c = c; a.dg = dg;
  a.colpart = colpart; a.amax_dg = amax_dg;
  AVC_TRY(zero_async(amax_dg, sizeof(unsigned), s));
  a.tickets = reinterpret_cast<unsigned long long*>(region);
  a.tmo = region + 32;
  a.cnt = region + kRegionHeaderWords;
  a.fail_host = ctx->fail_host;
  a.nwg = 256;
  a.spin_limit = coresident_spin_limit();
  a.diag = g_bptt_diag;
  if (persist_inject_take()) a.spin_limit = 0;
  const void* fn = bptt_fn(nch, ns);
  void* args[] = {&a};
  hipEvent_t ev = timing_begin(TC_LSTM_STEP_BWD, s);
  AVC_TRY(coresident_dispatch(ctx, fn, dim3(256), dim3(512), args, bptt_lds(nch), s));
  if (ev) {
    // the recurrent products of T - 1 steps; algorithmic bytes: the split dG read and the
    // partials written and read per step, the epilogue operands, dG written
    const double flops = (double)(T - 1) * 2.0 * B * H * 4.0 * H;
    const double bytes = (double)(T - 1) * (4.0 * B * 4.0 * H * 256 / (nrt * ntn * ns) * nrt * ntn +
                                            2.0 * 4.0 * ns * B * H) + (double)T * 4.0 * B * H * 12.0;
    timing_end(TC_LSTM_STEP_BWD, ev, s, flops, bytes);
  }
  return AVC_OK;
}

}  // namespace avc

extern "C" int avc_debug_xl_census(unsigned* local_nonlocal) {
  // (test hook) copies and clears the XCD-local BPTT census: workgroups that found their group
  // local / not local since the last call
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(avc::g_xl_seen)) != hipSuccess) return AVC_ERR_HIP;
  if (hipMemcpy(local_nonlocal, p, 2 * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return AVC_ERR_HIP;
  if (hipMemset(p, 0, 2 * sizeof(unsigned)) != hipSuccess) return AVC_ERR_HIP;
  return AVC_OK;
}

extern "C" int avc_debug_bptt_diag(int bits) {
  avc::g_bptt_diag = bits;
  return AVC_OK;
}

extern "C" int avc_bptt_persist(int on) {
  avc::g_bptt_persist = on ? 1 : 0;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_bptt_xcd(int on) {
  if (on < 0 || on > 2) {
    avc::set_error("avc_bptt_xcd: 0, 1 or 2");
    return AVC_ERR_INVALID;
  }
  avc::g_bptt_xl = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_debug_xl_force_remote(int on) {
  avc::g_xl_remote = on ? 1 : 0;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_bptt_coalesce(int on) {
  if (on < 0 || on > 1) {
    avc::set_error("avc_bptt_coalesce: on must be 0 or 1");
    return AVC_ERR_INVALID;
  }
  avc::g_bptt_bgf = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}
