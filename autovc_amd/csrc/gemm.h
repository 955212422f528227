// fp32 MFMA GEMM with implicit Conv1d taps — the contraction engine behind every Conv1d,
// LSTM input projection, Linear and weight-gradient product of the Generator.
#pragma once
#include "common.h"

namespace avc {

// BatchNorm + activation fused into the split-f16 GEMM's epilogue (gemm_bnf_ok):
// y = A.B + bias stays in registers, and each workgroup normalises its own tile.  Train mode:
// every workgroup stores its column partials (write-through), counts itself in on its column
// tile's arrival counter and waits until all tilesM tiles of that column are in (the grid is
// co-resident: one launch of at most one wave of workgroups, through persist_dispatch; epoch-
// tagged counters that are never reset, bounded spins, NaN on give-up, as the persistent LSTM
// kernels); it then forms mean / invstd of its columns from the partials in bn_finalize_kernel's
// order and applies BN + act (+ residual) exactly as bn_apply / bn_apply_frag do, writing the fp32
// output and / or the split fragment image.  Eval mode uses the running statistics (no barrier).
struct BnFuse {
  int on = 0, training = 0, act = 0;
  int nkc_out = 0;                 // 16-deep chunks of the fragment image (frag)
  const float* gamma = nullptr; const float* beta = nullptr; const float* residual = nullptr;
  float* out = nullptr;            // fp32 [M][N] output (nullable)
  _Float16* frag = nullptr;        // split output image (nullable; M % 32 == 0)
  unsigned* range_flag = nullptr;  // pinned word: a finite |output| >= 65504 was produced
  float* rmean = nullptr; float* rvar = nullptr; float* mean = nullptr; float* invstd = nullptr;
  float momentum = 0.f, eps = 0.f; double count = 0.0;
  unsigned* cnt = nullptr;         // [tilesN] arrival counters, one 128-B line each
  unsigned* tmo = nullptr;         // give-up word (epoch of the last launch that gave up)
  unsigned long long* tickets = nullptr;
  unsigned* fail_host = nullptr;
  unsigned spin_limit = 0;
  int nwg = 0;
  int band = 1;                    // dispatch order: 1 = XCD-contiguous row bands per column group
};

// C(m, n) = act( sum_tap sum_k A_tap(m, k) * B_tap(k, n) + bias0[n] + bias1[n] )
//
// A (a_trans = 0): element (m, k) of tap tau at A[(m + a_shift0 + tau*a_tapshift) * lda + k];
//                  rows outside [0, a_rows) read as zero (Conv1d zero padding in time).
// A (a_trans = 1): element (m, k) at A[k * lda + m]  (operand stored K-major, e.g. dY^T).
// B (b_trans = 0): element (k, n) at B[(k + b_shift) * ldb + n] + tau*b_tapoff, storage
//                  rows outside [0, b_rows) read as zero; b_shift = b_shift0 + z*b_zshift.
// B (b_trans = 1): element (k, n) at B[n * ldb + k] + tau*b_tapoff.
// Grid z enumerates nz independent products (A += z*a_zoff, C += z*c_zoff, B shifted) times
// nsplit K-splits; with nsplit > 1 raw partial sums go to `slab` and gemm_run() reduces them.
struct GemmDesc {
  int M = 0, N = 0, Kc = 0, ntaps = 1;
  const float* A = nullptr; long lda = 0; long a_rows = 0; long a_shift0 = 0; long a_tapshift = 0;
  int a_trans = 0;
  const float* B = nullptr; long ldb = 0; long b_rows = 0; long b_shift0 = 0; long b_zshift = 0;
  long b_tapoff = 0; int b_trans = 0;
  // B straight from a PyTorch Conv1d weight W[co][ci][5] (split-f16 fragment path only, round 5):
  // 1 = the forward, element (k = ci, n = co) of tap tau at W[n][k][tau]; 2 = the data gradient,
  // element (k = co, n = ci) of tap tau at W[k][n][4 - tau].  Replaces the transposed fp32 copies.
  int b_conv = 0;
  int nz = 1; long a_zoff = 0; long c_zoff = 0;
  float* C = nullptr; long ldc = 0; long ldc_col = 1; int accumulate = 0;
  const float* bias0 = nullptr; const float* bias1 = nullptr; int act = AVC_ACT_NONE;
  int prec16 = 0;           // 1: split-fp16 ("3xf16") MFMA kernel; forward products are range-
                            // guarded: an operand whose max |x| reaches 2^15 is scaled down by a
                            // power of two before splitting (scale 1, bit-identical, otherwise)
  float a_bound = 0.f;      // forward: host-known bound on |A| (an LSTM's h: 1); < 2^15 skips the scan
  int split_scale = 0;      // with prec16: scale each operand by a power of two from its device-side
                            // max |x| before splitting (gradients: any magnitude), unscale exactly
  const unsigned* amax_a = nullptr;  // max |A| as float bits (device); preset by the caller to
                                     // share one scan between products, else filled by gemm_run
  const unsigned* amax_b = nullptr;  // max |B|: filled by gemm_run, or preset by the caller for a
                                     // scaled (gradient) product whose B's producer recorded it
  const unsigned* a_guard = nullptr; // forward products: A's range-guard word max(|A|, 2^14) from
                                     // its producer (bn_apply's amax_out + 1); skips the scan
  const _Float16* b_frag = nullptr;  // optional B already split by gemm_prepare_bfrag (prec16 only;
                                     // carries its range-guard word, see gemm_prepare_bfrag)
  const _Float16* a_frag = nullptr;  // optional A already split (row-major A, unscaled forward
                                     // products only): gemm_afrag_bytes(a_rows, Kc) bytes in the
                                     // layout split_frag32_kernel writes (e.g. by bn_apply's frag)
  _Float16* a_frag_out = nullptr;  // optional: gemm_run writes its split of A here (instead of
                                   // scratch; a_trans: gemm_afrag_bytes(M, Kc) bytes) ...
  int a_frag_scaled = 0;    // ... and a later product with the same A and amax_a passes it back as
                            // a_frag with a_frag_scaled = 1 (gradient products sharing dY^T / dG^T)
  int b_frag_scaled = 0;    // scaled (gradient) products: b_frag was split scaled by the power of two
                            // of *amax_b, as gemm_run's own split would be (a conv's x image written
                            // by its forward, gemm_split_dual2), and is streamed as is
  const unsigned* a_frag_guard = nullptr;  // forward products: a_frag was split scaled by the power of
                                           // two of this range-guard word (max(|A|, 2^14); frames_frag)
  float* stats = nullptr;   // [ceil(M/BM)][2][N] column (sum, sumsq) partials of the output
  int stats_bm = 0;         // filled by gemm_run: rows per stats partial
  BnFuse bnf;               // fused BatchNorm epilogue (bnf.on; set up by gemm_bnf_ok's caller)
};

// true when gemm_run can fuse BatchNorm (+ act) into this product's epilogue (d.bnf.on): a
// split-f16 product on streamed fragments, one K split, one co-resident wave of workgroups
bool gemm_bnf_ok(const GemmDesc& d, bool training);

// Launch (with automatic tile and split-K choice).  Uses ctx scratch for split-K slabs.
int gemm_run(avc_context* ctx, GemmDesc d, hipStream_t stream, int force_split = 0);
// Rows covered by one stats partial for a problem of M rows (so callers can size `stats`).
int gemm_stats_rows(int M, int N);
// Scratch bytes gemm_run may take for this problem.
size_t gemm_scratch_bytes(const GemmDesc& d);
// B operand of a forward (prec16) product split once into the fragment-major layout the
// split-f16 kernel streams (all taps), range-guarded (its guard word trails the fragments); pass
// it back as GemmDesc::b_frag to skip the per-call split.
size_t gemm_bfrag_bytes(const GemmDesc& d);
int gemm_prepare_bfrag(const GemmDesc& d, _Float16* dst, hipStream_t stream);
// bytes of a row-major [rows][K] operand in the fragment-major split layout (GemmDesc::a_frag)
size_t gemm_afrag_bytes(long rows, int K);
// true when gemm_run would stream this product from split fragments (so a_frag is honoured)
bool gemm_frag_eligible(const GemmDesc& d);
// slab[split][M][N] = raw split-K partials of A_frag(M x K) . B_frag(N x K)^T (both split by
// gemm_split_frag / split_frag32_kernel; tile 64 or 128); no scale, bias or epilogue
int gemm_frag_partials(int M, int N, int K, const _Float16* As, const _Float16* Bs, int tile, int nsplit,
                       float* slab, hipStream_t s);
// [R][K] fp32 (row stride rs) -> fragment-major split, scaled by the power of two of *amax
int gemm_split_frag(const float* src, long rs, int R, int K, const unsigned* amax, _Float16* dst, hipStream_t s);
// One read of row-major [R][C] src writes its scaled split as an A operand (K = C, rows R) into
// dst_a and as an A^T operand (K = R, rows C) into dst_t, the bits split_frag32_kernel gives each
// (R % 32 == 0, C % 64 == 0: gemm_split_dual_ok).  Consumers take them as a_frag + a_frag_scaled.
bool gemm_split_dual_ok(long R, long C, long ld);
int gemm_split_dual(const float* src, long ld, long R, int C, const unsigned* amax, _Float16* dst_a, _Float16* dst_t,
                    hipStream_t s);
// the A^T image of row-major [R][C] src alone (rows C, K = R): gemm_split_dual's dst_t, one pass
int gemm_split_frag_t(const float* src, long ld, long R, int C, const unsigned* amax, _Float16* dst, hipStream_t s);
// ... with its own scale for each image: dst_a scaled by *amax_a, dst_t by *amax_t (NULL: unscaled)
int gemm_split_dual2(const float* src, long ld, long R, int C, const unsigned* amax_a, const unsigned* amax_t,
                     _Float16* dst_a, _Float16* dst_t, hipStream_t s);
// max |x| of a rows x cols region (row stride ld) into *out (float bits), for GemmDesc::amax_a
int gemm_absmax(const float* src, long rows, long cols, long ld, unsigned* out, hipStream_t stream);

}  // namespace avc
