// Conv1d(k=5, pad=2) + BatchNorm1d + activation, forward and backward.
//
// Reference composition: ConvNorm (net_layers.py:39-49) -> nn.BatchNorm1d -> relu
// (encoder.py:69-70, decoder.py:69-70) or tanh (postnet.py:54-55) or nothing (postnet.py:61).
//
// Forward  : one implicit-GEMM launch (5 taps accumulated inside the K loop, bias and the
//            per-channel BN partial sums fused in the epilogue), one tiny statistics kernel,
//            one normalise+activate pass.
// Backward : BN backward (reduce + apply), dgrad as the same 5-tap implicit GEMM on the
//            tap-flipped weights, wgrad as 5 batched GEMMs over all frames (split-K).
#include <algorithm>

#include "elementwise.h"
#include "kernels.h"

namespace avc {

int g_bnb_frag = 1;  // avc_bn_bwd_frag(): the BN backward writes dY already split

namespace {

// Wt[(tau*cin + ci)*cout + co] = W[(co*cin + ci)*5 + tau]   (forward B operand, [K][N])
// Wd[(tau*cout + co)*cin + ci] = W[(co*cin + ci)*5 + 4-tau] (dgrad B operand, [K][N])
__global__ void conv_weight_fwd_kernel(const float* __restrict__ W, float* __restrict__ Wt, int cin,
                                       int cout) {
  const long total = 5L * cin * cout;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i % cout);
    const long r = i / cout;
    const int ci = (int)(r % cin), tau = (int)(r / cin);
    Wt[i] = W[((long)co * cin + ci) * 5 + tau];
  }
}

__global__ void conv_weight_dgrad_kernel(const float* __restrict__ W, float* __restrict__ Wd, int cin,
                                         int cout) {
  const long total = 5L * cin * cout;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cin);
    const long r = i / cin;
    const int co = (int)(r % cout), tau = (int)(r / cout);
    Wd[i] = W[((long)co * cin + ci) * 5 + (4 - tau)];
  }
}

inline int ew_blocks(long n) { return (int)std::max<long>(1, std::min<long>((n + 255) / 256, 8192)); }

GemmDesc conv_fwd_desc(int T, int B, int cin, int cout, const float* x, const float* Wt,
                       const float* bias, float* y) {
  GemmDesc g;
  g.M = T * B; g.N = cout; g.Kc = cin; g.ntaps = 5;
  g.A = x; g.lda = cin; g.a_rows = (long)T * B; g.a_shift0 = -2L * B; g.a_tapshift = B;
  g.B = Wt; g.ldb = cout; g.b_rows = cin; g.b_tapoff = (long)cin * cout;
  g.C = y; g.ldc = cout; g.bias0 = bias;
  g.prec16 = 1;
  return g;
}

// dW[co][ci][tau] = sum_r dY[r][co] * x[r + (tau-2)B][ci]: the weight gradient's product (its A,
// dY^T, and C are set by the caller)
GemmDesc conv_wgrad_desc(int T, int B, int cin, int cout, const float* x, const unsigned* x_amax) {
  const long TB = (long)T * B;
  GemmDesc gw;
  gw.M = cout; gw.N = cin; gw.Kc = (int)TB;
  gw.a_trans = 1; gw.lda = cout;
  gw.B = x; gw.ldb = cin; gw.b_rows = TB; gw.b_shift0 = -2L * B; gw.b_zshift = B;
  gw.nz = 5; gw.c_zoff = 1;
  gw.ldc = 5L * cin; gw.ldc_col = 5;
  gw.prec16 = 1; gw.split_scale = 1;
  gw.amax_b = x_amax;
  return gw;
}

}  // namespace

// (shape only: whether the products then stream split images depends on the process-wide GEMM
// toggles, which may change between a forward and its backward; both sides check them themselves)
bool conv_wgrad_image_ok(int T, int B, int cin, int cout) {
  const long TB = (long)T * B;
  return cout > 0 && B % 16 == 0 && TB <= 0x7fffffffL && gemm_split_dual_ok(TB, cin, cin);
}

size_t conv_wgrad_image_bytes(int T, int B, int cin) { return gemm_afrag_bytes(cin, T * B); }  // rows cin, K = T*B

bool conv_frag_chain_ok(int T, int B, int cin, int cout) {
  const GemmDesc g = conv_fwd_desc(T, B, cin, cout, nullptr, nullptr, nullptr, nullptr);
  return cin % 8 == 0 && gemm_frag_eligible(g);
}

size_t conv_bn_forward_scratch(int T, int B, int cin, int cout) {
  const int bm = gemm_stats_rows(T * B, cout);
  const size_t parts = (size_t)((T * B + bm - 1) / bm) * 2 * cout;
  const GemmDesc g = conv_fwd_desc(T, B, cin, cout, nullptr, nullptr, nullptr, nullptr);
  return (5UL * cin * cout + parts) * sizeof(float) + gemm_scratch_bytes(g) + 2048;
}

int conv_bn_act_forward_impl(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                             const float* weight, const float* bias, const float* gamma,
                             const float* beta, float* running_mean, float* running_var,
                             int training, float momentum, float eps, int act,
                             const float* residual, float* y_pre, float* out, float* mean,
                             float* invstd, hipStream_t s, const _Float16* x_frag,
                             _Float16* out_frag, const unsigned* x_amax, unsigned* out_amax,
                             const unsigned* x_frag_guard, _Float16* x_wimg) {
  // x_frag: x already split (the previous layer's bn_apply wrote it); out_frag: also emit the
  // output split for the next layer (out may then be NULL: the fp32 output is not stored).
  // x_amax: x's max words from its producer (see bn_apply's amax_out): the range scan of x is
  // skipped; out_amax: record out's max words for the next layer (with or without out_frag)
  AVC_CHECK_ARG(T > 0 && B > 0, "conv: empty input");
  AVC_CHECK_ARG(cin % 4 == 0 && cout % 4 == 0, "conv: channel counts must be multiples of 4");
  AVC_CHECK_ARG(training || (running_mean && running_var), "conv: eval mode needs running stats");
  AVC_CHECK_ARG(!training || (long)T * B > 1, "BatchNorm in training mode needs more than 1 value per channel");
  Scratch sc(ctx);
  GemmDesc g = conv_fwd_desc(T, B, cin, cout, x, weight, bias, y_pre);
  g.a_frag = x_frag;
  g.a_frag_guard = x_frag ? x_frag_guard : nullptr;  // x_frag split with that guard's scale (frames_frag)
  if (x_amax) g.a_guard = x_amax + 1;
  if (!out && !out_frag) out_amax = nullptr;
  if (gemm_frag_eligible(g)) {
    // the split-f16 taps straight from the PyTorch layout (GemmDesc::b_conv; round 5: no
    // transposed fp32 copy), cached per weight version inside the whole-Generator forward
    g.b_conv = 1;
    if (ctx->prep_version >= 0) {
      bool fb = true;
      auto* bf = static_cast<_Float16*>(prep_buffer(ctx, PREP_CONV_BFRAG, weight, nullptr, gemm_bfrag_bytes(g), &fb));
      if (bf && fb) AVC_TRY(gemm_prepare_bfrag(g, bf, s));
      if (bf) g.b_frag = bf;
    }
  } else {  // every other path reads the taps as a transposed fp32 copy
    g.b_conv = 0;
    bool fresh = true;
    float* wt = prep_or_scratch<float>(ctx, sc, PREP_CONV_WT, weight, nullptr, 5UL * cin * cout, &fresh);
    if (!wt) return AVC_ERR_WORKSPACE;
    if (fresh) {
      conv_weight_fwd_kernel<<<ew_blocks(5L * cin * cout), 256, 0, s>>>(weight, wt, cin, cout);
      AVC_LAUNCH_CHECK();
    }
    g.B = wt;
  }
  if (x_wimg) {
    // round 6: the weight gradient's split of x (its B operand, K = frames, scaled by the power of
    // two of max |x|, as that product's own split would be) written by the same pass that splits
    // x for this product (A, K = cin, guard-scaled): the backward reads x_wimg instead of
    // splitting x again (conv_bn_act_backward_impl; same bits)
    AVC_CHECK_ARG(x_amax && !x_frag && conv_wgrad_image_ok(T, B, cin, cout) && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
                  "conv forward: a weight-gradient image needs x_amax, no x_frag and avc_conv_wgrad_image_bytes > 0");
    if (g.b_conv == 1) {  // this product streams split fragments: one pass writes both images
      AVC_TAKE(ximg, _Float16, gemm_afrag_bytes((long)T * B, cin) / 2, sc);
      AVC_TRY(gemm_split_dual2(x, cin, (long)T * B, cin, x_amax + 1, x_amax, ximg, x_wimg, s));
      g.a_frag = ximg;
      g.a_frag_guard = x_amax + 1;
    } else {  // (a GEMM toggle moved this product off the split path: the image alone)
      AVC_TRY(gemm_split_frag_t(x, cin, (long)T * B, cin, x_amax, x_wimg, s));
    }
  }
  float* stats = nullptr;
  int nparts = 0, part_rows = 0;
  if (training) {
    const int bm = gemm_stats_rows(T * B, cout);
    part_rows = bm;
    nparts = (T * B + bm - 1) / bm;
    AVC_TAKE(st, float, (size_t)nparts * 2 * cout, sc);
    stats = st;
    g.stats = stats;
  }
  // inside the whole-Generator forward the output's range is checked here (its consumer then
  // skips the scan); a value the next split could not hold is reported to the host.  The layer
  // with a residual (postnet's last, model.py:131-132) produces the final mel_post, which no
  // contraction reads: nothing to check.
  const bool check = out_frag || (ctx->track_ranges && !residual);
  unsigned* flags = check ? host_flags(ctx) : nullptr;
  if (check && !flags) return AVC_ERR_HIP;
  if (!out_amax && gemm_bnf_ok(g, training != 0)) {
    // BatchNorm + act fused into the GEMM's epilogue (gemm.h BnFuse): same bits, two launches
    // fewer, and y_pre is stored only where a backward will read it (never inside the
    // whole-Generator forward, whose y_pre is the output buffer or scratch)
    if (!y_pre || y_pre == out || ctx->track_ranges) g.C = nullptr;
    BnFuse& f = g.bnf;
    f.on = 1; f.training = training != 0; f.act = act;
    f.gamma = gamma; f.beta = beta; f.residual = residual; f.out = out;
    f.frag = out_frag; f.nkc_out = (cout + 31) / 32 * 2;
    f.range_flag = flags ? flags + 1 : nullptr;
    f.rmean = running_mean; f.rvar = running_var; f.mean = mean; f.invstd = invstd;
    f.momentum = momentum; f.eps = eps; f.count = (double)T * B;
    AVC_TRY(gemm_run(ctx, g, s));
    if (check && out) mark_range_checked(ctx, out);
    return AVC_OK;
  }
  AVC_TRY(gemm_run(ctx, g, s));
  AVC_TRY(bn_finalize(cout, nparts, part_rows, stats, (double)T * B, training, momentum, eps, running_mean,
                      running_var, mean, invstd, s, out_amax));
  AVC_TRY(bn_apply((long)T * B, cout, y_pre, mean, invstd, gamma, beta, act, residual, out, s, out_frag,
                   flags ? flags + 1 : nullptr, out_amax));
  if (check && out) mark_range_checked(ctx, out);
  return AVC_OK;
}

size_t conv_bn_backward_scratch(int T, int B, int cin, int cout) {
  const size_t TB = (size_t)T * B;
  GemmDesc w;
  w.M = cout; w.N = cin; w.Kc = (int)TB; w.a_trans = 1; w.nz = 5; w.b_rows = TB; w.b_zshift = B;
  w.prec16 = 1; w.split_scale = 1;
  GemmDesc dg;
  dg.M = (int)TB; dg.N = cin; dg.Kc = cout; dg.ntaps = 5; dg.a_rows = TB;
  dg.prec16 = 1; dg.split_scale = 1;
  // (+ the dY / dY^T fragment images of the split-writing BN backward, avc_bn_bwd_frag)
  return (TB * cout + 5UL * cin * cout) * sizeof(float) + 2 * bn_backward_frag_scratch((int)TB, cout) +
         gemm_afrag_bytes(TB, cout) + gemm_afrag_bytes(cout, (int)TB) + 4096 +
         colsum_scratch((int)TB, cout) + std::max(gemm_scratch_bytes(w), gemm_scratch_bytes(dg)) + 2048;
}

int conv_bn_act_backward_impl(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                              const float* weight, const float* gamma, const float* beta,
                              const float* y_pre, const float* mean, const float* invstd,
                              int training, int act, const float* d_out, float* d_x,
                              float* d_weight, float* d_bias, float* d_gamma, float* d_beta,
                              int accumulate, hipStream_t s, const unsigned* x_amax, const _Float16* x_wimg) {
  // x_amax: max |x| recorded by x's producer (bn_apply's amax_out): the weight gradient's scan
  // of x is skipped
  AVC_CHECK_ARG(T > 0 && B > 0, "conv_backward: empty input");
  AVC_CHECK_ARG(cin % 4 == 0 && cout % 4 == 0, "conv_backward: channels must be multiples of 4");
  AVC_CHECK_ARG(accumulate >= 0 && accumulate <= 2, "conv_backward: accumulate must be 0, 1 or 2");
  const long TB = (long)T * B;
  // accumulate: 1 = every output adds into its buffer, 2 = only the parameter gradients do
  // (d_x overwritten: the caller accumulates parameter gradients in place across uses)
  const int acc_x = accumulate == 1, acc_p = accumulate != 0;
  Scratch sc(ctx);
  // the two products of dY: dgrad (dX = dY * W, taps as row shifts) and wgrad (dW = dY^T x)
  GemmDesc gd;
  gd.M = (int)TB; gd.N = cin; gd.Kc = cout; gd.ntaps = 5;
  gd.lda = cout; gd.a_rows = TB; gd.a_shift0 = -2L * B; gd.a_tapshift = B;
  gd.ldb = cin; gd.b_rows = cout; gd.b_tapoff = (long)cout * cin;
  gd.C = d_x; gd.ldc = cin; gd.accumulate = acc_x;
  gd.prec16 = 1; gd.split_scale = 1;
  GemmDesc gw = conv_wgrad_desc(T, B, cin, cout, x, x_amax);
  gw.C = d_weight; gw.accumulate = acc_p;
  if (x_wimg && gemm_frag_eligible(gw)) {  // x split by its forward (conv_bn_act_forward_impl's x_wimg)
    AVC_CHECK_ARG(x_amax && conv_wgrad_image_ok(T, B, cin, cout),
                  "conv backward: a weight-gradient image needs x_amax and avc_conv_wgrad_image_bytes > 0");
    gw.b_frag = x_wimg;
    gw.b_frag_scaled = 1;
  }
  // round 4 (avc_bn_bwd_frag): the BN backward writes dY already split for both
  // products -- dY and dY^T fragment images scaled by a proven bound on max |dY| -- so neither the
  // fp32 dY nor its max scan and two split passes exist
  const bool fb = g_bnb_frag && (d_x || d_weight) && bn_backward_frag_ok((int)TB, cout, d_out, y_pre) &&
                  (!d_x || gemm_frag_eligible(gd)) && (!d_weight || gemm_frag_eligible(gw));
  AVC_TAKE(amax_dy, unsigned, 64, sc);
  float* dy = nullptr;
  if (fb) {
    const int R = bn_backward_frag_rows((int)TB);
    AVC_TAKE(bpart, float, (size_t)R * cout, sc);
    AVC_TAKE(imgA, _Float16, gemm_afrag_bytes(TB, cout) / 2, sc);
    AVC_TAKE(imgT, _Float16, gemm_afrag_bytes(cout, (int)TB) / 2, sc);
    AVC_TRY(bn_backward_frag(ctx, (int)TB, cout, d_out, y_pre, mean, invstd, gamma, beta, act, training, d_gamma,
                             d_beta, acc_p, imgA, imgT, amax_dy, s, d_bias ? bpart : nullptr));
    if (d_bias) AVC_TRY(colsum_finish(R, cout, bpart, d_bias, acc_p, s));
    gd.a_frag = imgA; gd.a_frag_scaled = 1;
    gw.a_frag = imgT; gw.a_frag_scaled = 1;
  } else {
    // the pass that writes dY also yields the conv bias gradient's column partials and max |dY|
    // (one max shared by dgrad and wgrad)
    AVC_TAKE(dyb, float, (size_t)TB * cout, sc);
    dy = dyb;
    const int R = bn_backward_rows((int)TB, cout);
    AVC_TAKE(bpart, float, (size_t)R * cout, sc);
    AVC_TRY(bn_backward(ctx, (int)TB, cout, d_out, y_pre, mean, invstd, gamma, beta, act, training,
                        d_gamma, d_beta, acc_p, dy, s, d_bias ? bpart : nullptr, amax_dy));
    if (d_bias) AVC_TRY(colsum_finish(R, cout, bpart, d_bias, acc_p, s));
  }
  gd.A = dy; gd.amax_a = amax_dy;
  gw.A = dy; gw.amax_a = amax_dy;
  if (d_x) {
    gd.B = weight;
    gd.b_conv = 2;  // the split reads the PyTorch layout (GemmDesc::b_conv, round 5)
    if (!gemm_frag_eligible(gd)) {
      gd.b_conv = 0;
      AVC_TAKE(wd, float, 5UL * cin * cout, sc);
      conv_weight_dgrad_kernel<<<ew_blocks(5L * cin * cout), 256, 0, s>>>(weight, wd, cin, cout);
      AVC_LAUNCH_CHECK();
      gd.B = wd;
    }
    AVC_TRY(gemm_run(ctx, gd, s));
  }
  if (d_weight) AVC_TRY(gemm_run(ctx, gw, s));
  return AVC_OK;
}

}  // namespace avc

extern "C" int avc_bn_bwd_frag(int on) {
  if (on < 0 || on > 1) {
    avc::set_error("avc_bn_bwd_frag: on must be 0 or 1");
    return AVC_ERR_INVALID;
  }
  avc::g_bnb_frag = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}
