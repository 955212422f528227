// extern "C" entry points (include/autovc_hip.h), the context/arena, and the whole-Generator
// forward used by VoiceConverter.convert()-style inference (model.py:68-146).
#include <algorithm>
#include <mutex>

#include "elementwise.h"
#include "kernels.h"
#include "timing.h"

namespace avc {

namespace {
thread_local std::string g_err;
}

void set_error(const std::string& msg) { g_err = msg; }
int g_config_epoch = 0;
int g_graph_mode = 1;  // avc_graph_mode()
const char* get_error() { return g_err.c_str(); }

void* prep_buffer(avc_context* ctx, int kind, const void* key0, const void* key1, size_t bytes,
                  bool* fresh) {
  *fresh = true;
  if (ctx->prep_version < 0) return nullptr;
  for (auto& e : ctx->prep) {
    if (e.kind == kind && e.key0 == key0 && e.key1 == key1 && e.bytes == bytes) {
      *fresh = e.version != ctx->prep_version;
      e.version = ctx->prep_version;
      return e.buf;
    }
  }
  avc_prep_entry e;
  e.kind = kind; e.key0 = key0; e.key1 = key1; e.bytes = bytes; e.version = ctx->prep_version;
  if (hipMalloc(&e.buf, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;  // no room: derive into scratch this call
  }
  ctx->prep.push_back(e);
  return e.buf;
}

int ensure_arena(avc_context* ctx, size_t bytes) {
  if (ctx->cap >= bytes) return AVC_OK;
  if (ctx->top != 0) {
    set_error("arena growth requested while scratch is in use");
    return AVC_ERR_WORKSPACE;
  }
  int prev = 0;
  AVC_HIP(hipGetDevice(&prev));
  if (prev != ctx->device) AVC_HIP(hipSetDevice(ctx->device));
  size_t want = std::max(bytes, ctx->cap * 3 / 2);
  want = (want + (1u << 20) - 1) & ~size_t((1u << 20) - 1);
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, want);
  if (prev != ctx->device) (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    set_error(std::string("arena hipMalloc of ") + std::to_string(want) + " bytes: " + hipGetErrorString(e));
    return AVC_ERR_HIP;
  }
  // The old block may still be read by kernels queued earlier on the stream: retire it and
  // free it only when the context is destroyed.
  if (ctx->base) ctx->retired.push_back(ctx->base);
  ctx->base = static_cast<char*>(p);
  ctx->cap = want;
  return AVC_OK;
}

namespace {

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- whole-Generator forward --------------------------------------------------------------
enum : int {
  P_ENC_CONV = 0,    // 3 x {W, b, gamma, beta, rmean, rvar}
  P_ENC_LSTM = 18,   // l0, l0_rev, l1, l1_rev x {w_ih, w_hh, b_ih, b_hh}
  P_DEC_LSTM1 = 34,  // l0
  P_DEC_CONV = 38,   // 3 x 6
  P_DEC_LSTM2 = 56,  // l0, l1
  P_LIN = 64,        // W, b
  P_POST = 66,       // 5 x 6
  P_COUNT = 96,
};

struct GenBufs {
  size_t total = 0;
  size_t nested = 0;
};

size_t gen_scratch(int T, int B) {
  const size_t TB = (size_t)T * B, f = sizeof(float);
  size_t own = TB * (336 + 512 + 512 + 64 + 64 + 320 + 1024 + 1024 + 80 + 80) * f + 4 * 512 * f + 64 * 256 +
               2 * gemm_afrag_bytes((long)TB, 512) + gemm_afrag_bytes((long)TB, 1024) + gemm_afrag_bytes((long)TB, 336) +
               2048 + 1024;  // (+ the frames' split image and their range-guard words)
  size_t nested = 0;
  nested = std::max(nested, conv_bn_forward_scratch(T, B, 336, 512));
  nested = std::max(nested, conv_bn_forward_scratch(T, B, 512, 512));
  nested = std::max(nested, conv_bn_forward_scratch(T, B, 80, 512));
  nested = std::max(nested, bilstm_forward_scratch(T, B, 512, 32, false));
  nested = std::max(nested, lstm_forward_scratch(T, B, 320, 512, false));
  nested = std::max(nested, lstm_forward_scratch(T, B, 512, 1024, false));
  nested = std::max(nested, lstm2_forward_scratch(T, B, 512, 1024, false));
  GemmDesc lin;
  lin.M = (int)TB; lin.N = 80; lin.Kc = 1024; lin.b_trans = 1; lin.prec16 = 1;
  nested = std::max(nested, gemm_scratch_bytes(lin));
  return own + nested + (1 << 20);
}

// avc_split_handover(): the split-image hand-overs of the whole-Generator forward that do not
// come from a conv (encoder conv 3 -> BiLSTM projection, lstm1 -> decoder conv 1, lstm2 -> Linear)
int g_handover = 1;
int g_dead_y = 1;  // avc_dead_h_stores(): skip the recurrences' fp32 h stores nothing reads (avc_context::dead_y)

int generator_forward(avc_context* ctx, int T, int B, const float* const* P, const float* x,
                      const float* c_org, const float* c_trg, int training, float* mel,
                      float* mel_post, float* codes, hipStream_t s) {
  AVC_CHECK_ARG(T >= 32, "T must be >= 32 frames (model.py:99 concatenates an empty code list)");
  AVC_CHECK_ARG(B >= 1, "batch must be >= 1");
  const long TB = (long)T * B;
  Scratch sc(ctx);
  RangeScope ranges(ctx);  // producers register activations whose range they checked (gemm.hip guard)
  AVC_TAKE(x0, float, (size_t)TB * 336, sc);
  AVC_TAKE(ba, float, (size_t)TB * 512, sc);
  AVC_TAKE(bb, float, (size_t)TB * 512, sc);
  AVC_TAKE(e1, float, (size_t)TB * 64, sc);
  AVC_TAKE(e2, float, (size_t)TB * 64, sc);
  AVC_TAKE(din, float, (size_t)TB * 320, sc);
  AVC_TAKE(l1, float, (size_t)TB * 1024, sc);
  AVC_TAKE(l2, float, (size_t)TB * 1024, sc);
  AVC_TAKE(melf, float, (size_t)TB * 80, sc);
  AVC_TAKE(postf, float, (size_t)TB * 80, sc);
  AVC_TAKE(stat, float, 4 * 512, sc);
  // conv -> conv links hand the activation over already split for the next GEMM (bn_apply's
  // fragment output): no fp32 store, no separate split pass
  AVC_TAKE(fa, _Float16, gemm_afrag_bytes(TB, 512) / 2, sc);
  AVC_TAKE(fb, _Float16, gemm_afrag_bytes(TB, 512) / 2, sc);
  AVC_TAKE(fl, _Float16, gemm_afrag_bytes(TB, 1024) / 2, sc);  // lstm2's output split for the Linear
  AVC_TAKE(fx, _Float16, gemm_afrag_bytes(TB, 336) / 2, sc);   // the frames as encoder conv 1's split operand
  AVC_TAKE(xguard, unsigned, 64, sc);                           // and their range-guard words
  float* mean = stat;
  float* invstd = stat + 512;
  const float eps = 1e-5f, mom = 0.1f;
  auto M = [&](int i) { return const_cast<float*>(P[i]); };

  // in_frag: the input already split; out_frag: emit the split output instead of the fp32 one
  // (its only reader is the next conv's GEMM); off when that GEMM would not stream fragments
  const bool chain = conv_frag_chain_ok(T, B, 512, 512) && conv_frag_chain_ok(T, B, 512, 80);
  auto cba = [&](int base, int cin, int cout, const float* in, float* out, int act,
                 const float* residual, const _Float16* in_frag = nullptr, _Float16* out_frag = nullptr,
                 const unsigned* in_guard = nullptr) {
    if (!chain) in_frag = nullptr, out_frag = nullptr;
    return conv_bn_act_forward_impl(ctx, T, B, cin, cout, in, P[base], P[base + 1], P[base + 2],
                                    P[base + 3], M(base + 4), M(base + 5), training, mom, eps, act,
                                    residual, out, out_frag ? nullptr : out, mean, invstd, s, in_frag,
                                    out_frag, nullptr, nullptr, in_frag ? in_guard : nullptr);
  };

  // Encoder (encoder.py:53-97).  Round 4: the frames go straight into the first conv's split
  // operand, scaled by the range guard of the mel and embedding themselves (frames_from_mel_frag;
  // the same bits as frames -> guard scan -> split)
  if (chain && g_handover && conv_frag_chain_ok(T, B, 336, 512)) {
    AVC_TRY(frames_from_mel_frag(ctx, T, B, 80, x, 256, c_org, fx, xguard, s));
    AVC_TRY(cba(P_ENC_CONV + 0, 336, 512, x0, ba, AVC_ACT_RELU, nullptr, fx, fa, xguard + 1));
  } else {
    AVC_TRY(frames_from_mel(T, B, 80, x, 256, c_org, x0, s));
    AVC_TRY(cba(P_ENC_CONV + 0, 336, 512, x0, ba, AVC_ACT_RELU, nullptr, nullptr, fa));
  }
  AVC_TRY(cba(P_ENC_CONV + 6, 512, 512, ba, bb, AVC_ACT_RELU, nullptr, fa, fb));
  // the third conv hands its output to the BiLSTM's input projection as a split image only
  const bool to_bilstm = chain && g_handover && bilstm_takes_frag(T, B, 512);
  AVC_TRY(cba(P_ENC_CONV + 12, 512, 512, bb, ba, AVC_ACT_RELU, nullptr, fb, to_bilstm ? fa : nullptr));
  const int EL = P_ENC_LSTM;
  AVC_TRY(bilstm_forward_impl(ctx, T, B, 512, 32, ba, 512, P + EL, P + EL + 4, e1, 64, nullptr, nullptr,
                              nullptr, nullptr, s, to_bilstm ? fa : nullptr));
  mark_range_checked(ctx, e1);  // an LSTM's h: |h| < 1
  AVC_TRY(bilstm_forward_impl(ctx, T, B, 64, 32, e1, 64, P + EL + 8, P + EL + 12, e2, 64, nullptr, nullptr,
                              nullptr, nullptr, s));
  AVC_CHECK_ARG(T >= 32, "content codes need T >= 32 frames (model.py:99 cat of an empty list)");

  // Upsample + decoder (model.py:115-127, decoder.py:58-79); the content codes (model.py:94-99)
  // are written by the same pass
  {  // the decoder input's embedding part is range-checked on the way (codes are LSTM outputs)
    unsigned* flags = host_flags(ctx);
    if (!flags) return AVC_ERR_HIP;
    AVC_TRY(decoder_input(T, B, e2, 256, c_trg, din, s, flags + 1, codes));
    mark_range_checked(ctx, din);
  }
  const int D1 = P_DEC_LSTM1;
  // lstm1 also writes its h as the split image the first decoder conv streams (its epilogue, or a
  // split pass where the recurrence is not persistent)
  struct DeadY {  // the fp32 h of a recurrence is not stored where only its split image is read
    avc_context* c;
    DeadY(avc_context* c_, int bits) : c(c_) { c->dead_y = bits; }
    ~DeadY() { c->dead_y = 0; }
  };
  {
    DeadY dy(ctx, g_dead_y && chain && g_handover ? 1 : 0);  // the first decoder conv streams fb only
    AVC_TRY(lstm_forward_impl(ctx, T, B, 320, 512, 0, din, 320, P[D1], P[D1 + 1], P[D1 + 2], P[D1 + 3],
                              ba, 512, nullptr, nullptr, s, chain && g_handover ? fb : nullptr));
  }
  mark_range_checked(ctx, ba);  // lstm1's h
  AVC_TRY(cba(P_DEC_CONV + 0, 512, 512, ba, bb, AVC_ACT_RELU, nullptr, chain && g_handover ? fb : nullptr, fa));
  AVC_TRY(cba(P_DEC_CONV + 6, 512, 512, bb, ba, AVC_ACT_RELU, nullptr, fa, fb));
  AVC_TRY(cba(P_DEC_CONV + 12, 512, 512, ba, bb, AVC_ACT_RELU, nullptr, fb));
  const int D2 = P_DEC_LSTM2;
  // decoder.lstm2: both layers advanced as one wavefront (lstm.hip: lstm2_forward_impl)
  // (l2 also as the split image the Linear streams when its product takes fragments)
  GemmDesc lin;
  lin.M = (int)TB; lin.N = 80; lin.Kc = 1024;
  lin.A = l2; lin.lda = 1024;
  lin.B = P[P_LIN]; lin.b_trans = 1; lin.ldb = 1024;
  lin.bias0 = P[P_LIN + 1];
  lin.C = melf; lin.ldc = 80;
  lin.prec16 = 1;
  lin.a_bound = 1.f;  // |h| < 1 (lstm2's output): no range scan needed
  const bool lin_frag = g_handover && TB % 32 == 0 && gemm_frag_eligible(lin);
  {
    DeadY dy(ctx, g_dead_y ? (lin_frag ? 3 : 2) : 0);  // layer 0's h is read split only; l2 too with lin_frag
    AVC_TRY(lstm2_forward_impl(ctx, T, B, 512, 1024, bb, 512, P + D2, P + D2 + 4, l1, l2, nullptr,
                               nullptr, nullptr, nullptr, s, lin_frag ? fl : nullptr));
  }
  if (lin_frag) lin.a_frag = fl;
  if (ctx->prep_version >= 0) {
    bool fb = true;
    auto* bf = static_cast<_Float16*>(prep_buffer(ctx, PREP_GEMM_BFRAG, P[P_LIN], nullptr, gemm_bfrag_bytes(lin), &fb));
    if (bf) {
      if (fb) AVC_TRY(gemm_prepare_bfrag(lin, bf, s));
      lin.b_frag = bf;
    }
  }
  AVC_TRY(gemm_run(ctx, lin, s));

  // Postnet + residual (postnet.py:50-63, model.py:131-132)
  AVC_TRY(cba(P_POST + 0, 80, 512, melf, ba, AVC_ACT_TANH, nullptr, nullptr, fa));
  AVC_TRY(cba(P_POST + 6, 512, 512, ba, bb, AVC_ACT_TANH, nullptr, fa, fb));
  AVC_TRY(cba(P_POST + 12, 512, 512, bb, ba, AVC_ACT_TANH, nullptr, fb, fa));
  AVC_TRY(cba(P_POST + 18, 512, 512, ba, bb, AVC_ACT_TANH, nullptr, fa, fb));
  AVC_TRY(cba(P_POST + 24, 512, 80, bb, postf, AVC_ACT_NONE, melf, fb));
  AVC_TRY(mel_from_frames(T, B, 80, melf, mel, s, postf, mel_post));  // both outputs, one launch
  return AVC_OK;
}

void drop_graph(avc_context* ctx);  // captured Generator graphs (defined below)
}  // namespace
}  // namespace avc

using namespace avc;

extern "C" {

int avc_abi_version(void) { return 1; }
const char* avc_last_error(void) { return get_error(); }

int avc_context_create(int device, avc_context** out) {
  AVC_CHECK_ARG(out != nullptr, "out is NULL");
  int n = 0;
  AVC_HIP(hipGetDeviceCount(&n));
  AVC_CHECK_ARG(device >= 0 && device < n, "device ordinal out of range");
  auto* c = new avc_context();
  c->device = device;
  *out = c;
  return AVC_OK;
}

int avc_context_destroy(avc_context* ctx) {
  if (!ctx) return AVC_OK;
  AVC_HIP(hipDeviceSynchronize());
  persist_release(ctx);
  for (void* p : ctx->retired) (void)hipFree(p);
  for (auto& e : ctx->prep) (void)hipFree(e.buf);
  drop_graph(ctx);  // the staging graph and every direct graph
  if (ctx->gen.stage) (void)hipFree(ctx->gen.stage);
  if (ctx->zpool) (void)hipFree(ctx->zpool);
  if (ctx->capture_stream) (void)hipStreamDestroy(ctx->capture_stream);
  if (ctx->base) (void)hipFree(ctx->base);
  delete ctx;
  return AVC_OK;
}

int avc_context_reserve(avc_context* ctx, size_t bytes) {
  AVC_CHECK_ARG(ctx != nullptr, "ctx is NULL");
  return ensure_arena(ctx, bytes);
}

int avc_gemm(avc_context* ctx, int M, int N, int K, const float* A, int a_trans, const float* B,
             int b_trans, const float* bias, float* C, int accumulate, void* stream) {
  AVC_CHECK_ARG(ctx && A && B && C, "NULL pointer");
  GemmDesc d;
  d.M = M; d.N = N; d.Kc = K;
  d.A = A; d.a_trans = a_trans; d.lda = a_trans ? M : K;
  d.B = B; d.b_trans = b_trans; d.ldb = b_trans ? K : N;
  d.bias0 = bias; d.C = C; d.ldc = N; d.accumulate = accumulate;
  AVC_TRY(ensure_arena(ctx, gemm_scratch_bytes(d) + 4096));
  return gemm_run(ctx, d, S(stream));
}

int avc_conv_bn_act_forward(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                            const float* weight, const float* bias, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            int training, float momentum, float eps, int act,
                            const float* residual, float* y_pre, float* out, float* mean,
                            float* invstd, void* stream) {
  AVC_CHECK_ARG(ctx && x && weight && gamma && beta && y_pre && out && mean && invstd, "NULL pointer");
  AVC_TRY(ensure_arena(ctx, conv_bn_forward_scratch(T, B, cin, cout)));
  return conv_bn_act_forward_impl(ctx, T, B, cin, cout, x, weight, bias, gamma, beta, running_mean,
                                  running_var, training, momentum, eps, act, residual, y_pre, out,
                                  mean, invstd, S(stream));
}

int avc_conv_bn_act_forward_ex(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                               const float* weight, const float* bias, const float* gamma,
                               const float* beta, float* running_mean, float* running_var,
                               int training, float momentum, float eps, int act,
                               const float* residual, float* y_pre, float* out, float* mean,
                               float* invstd, const unsigned* x_amax, unsigned* out_amax, void* stream) {
  AVC_CHECK_ARG(ctx && x && weight && gamma && beta && y_pre && out && mean && invstd, "NULL pointer");
  AVC_CHECK_ARG(aligned16(x_amax) && aligned16(out_amax), "amax words must be 16-byte aligned");
  AVC_TRY(ensure_arena(ctx, conv_bn_forward_scratch(T, B, cin, cout)));
  return conv_bn_act_forward_impl(ctx, T, B, cin, cout, x, weight, bias, gamma, beta, running_mean,
                                  running_var, training, momentum, eps, act, residual, y_pre, out,
                                  mean, invstd, S(stream), nullptr, nullptr, x_amax, out_amax);
}

int avc_conv_bn_act_forward_frag(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                                 const void* x_frag, const float* weight, const float* bias, const float* gamma,
                                 const float* beta, float* running_mean, float* running_var, int training,
                                 float momentum, float eps, int act, const float* residual, float* y_pre,
                                 float* out, void* out_frag, float* mean, float* invstd, const unsigned* x_amax,
                                 unsigned* out_amax, void* stream) {
  AVC_CHECK_ARG(ctx && x && weight && gamma && beta && y_pre && out && mean && invstd, "NULL pointer");
  AVC_CHECK_ARG(aligned16(x_amax) && aligned16(out_amax), "amax words must be 16-byte aligned");
  AVC_CHECK_ARG(aligned16(x_frag) && aligned16(out_frag), "split images must be 16-byte aligned");
  AVC_CHECK_ARG(!x_frag || conv_frag_chain_ok(T, B, cin, cout),
                "conv forward: a split input needs B % 32 == 0 and cin % 8 == 0 (avc_conv_frag_chain_ok)");
  AVC_CHECK_ARG(!out_frag || cout % 8 == 0, "conv forward: a split output needs cout % 8 == 0");
  AVC_TRY(ensure_arena(ctx, conv_bn_forward_scratch(T, B, cin, cout)));
  return conv_bn_act_forward_impl(ctx, T, B, cin, cout, x, weight, bias, gamma, beta, running_mean,
                                  running_var, training, momentum, eps, act, residual, y_pre, out,
                                  mean, invstd, S(stream), static_cast<const _Float16*>(x_frag),
                                  static_cast<_Float16*>(out_frag), x_amax, out_amax);
}

int avc_conv_bn_act_forward_wg(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                               const void* x_frag, const float* weight, const float* bias, const float* gamma,
                               const float* beta, float* running_mean, float* running_var, int training,
                               float momentum, float eps, int act, const float* residual, float* y_pre, float* out,
                               void* out_frag, float* mean, float* invstd, const unsigned* x_amax,
                               unsigned* out_amax, void* x_wimg, void* stream) {
  AVC_CHECK_ARG(aligned16(x_wimg), "split images must be 16-byte aligned");
  AVC_CHECK_ARG(!x_wimg || (x_amax && !x_frag && T > 0 && B > 0 && cin > 0 && cout > 0 &&
                            conv_wgrad_image_ok(T, B, cin, cout)),
                "conv forward: x_wimg needs x_amax, no x_frag and avc_conv_wgrad_image_bytes(T, B, cin, cout) > 0");
  if (!x_wimg)
    return avc_conv_bn_act_forward_frag(ctx, T, B, cin, cout, x, x_frag, weight, bias, gamma, beta, running_mean,
                                        running_var, training, momentum, eps, act, residual, y_pre, out, out_frag,
                                        mean, invstd, x_amax, out_amax, stream);
  AVC_CHECK_ARG(ctx && x && weight && gamma && beta && y_pre && out && mean && invstd, "NULL pointer");
  AVC_CHECK_ARG(aligned16(x) && aligned16(x_amax) && aligned16(out_amax) && aligned16(out_frag),
                "x, amax words and split images must be 16-byte aligned");
  AVC_CHECK_ARG(!out_frag || cout % 8 == 0, "conv forward: a split output needs cout % 8 == 0");
  AVC_TRY(ensure_arena(ctx, conv_bn_forward_scratch(T, B, cin, cout)));
  return conv_bn_act_forward_impl(ctx, T, B, cin, cout, x, weight, bias, gamma, beta, running_mean,
                                  running_var, training, momentum, eps, act, residual, y_pre, out,
                                  mean, invstd, S(stream), nullptr, static_cast<_Float16*>(out_frag), x_amax,
                                  out_amax, nullptr, static_cast<_Float16*>(x_wimg));
}

size_t avc_conv_wgrad_image_bytes(int T, int B, int cin, int cout) {
  return T > 0 && B > 0 && cin > 0 && cout > 0 && conv_wgrad_image_ok(T, B, cin, cout)
             ? conv_wgrad_image_bytes(T, B, cin)
             : 0;
}

int avc_conv_frag_chain_ok(int T, int B, int cin, int cout) {
  return T > 0 && B > 0 && cin > 0 && cout > 0 && conv_frag_chain_ok(T, B, cin, cout) ? 1 : 0;
}

size_t avc_act_frag_bytes(long rows, int channels) {
  return rows > 0 && channels > 0 ? gemm_afrag_bytes(rows, channels) : 0;
}

int avc_conv_bn_act_backward_ex(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                                const float* weight, const float* gamma, const float* beta,
                                const float* y_pre, const float* mean, const float* invstd,
                                int training, int act, const float* d_out, float* d_x,
                                float* d_weight, float* d_bias, float* d_gamma, float* d_beta,
                                int accumulate, const unsigned* x_amax, void* stream) {
  AVC_CHECK_ARG(ctx && x && weight && gamma && beta && y_pre && mean && invstd && d_out, "NULL pointer");
  AVC_TRY(ensure_arena(ctx, conv_bn_backward_scratch(T, B, cin, cout)));
  return conv_bn_act_backward_impl(ctx, T, B, cin, cout, x, weight, gamma, beta, y_pre, mean, invstd,
                                   training, act, d_out, d_x, d_weight, d_bias, d_gamma, d_beta,
                                   accumulate, S(stream), x_amax);
}

int avc_conv_bn_act_backward_wg(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                                const float* weight, const float* gamma, const float* beta,
                                const float* y_pre, const float* mean, const float* invstd,
                                int training, int act, const float* d_out, float* d_x,
                                float* d_weight, float* d_bias, float* d_gamma, float* d_beta,
                                int accumulate, const unsigned* x_amax, const void* x_wimg, void* stream) {
  AVC_CHECK_ARG(ctx && x && weight && gamma && beta && y_pre && mean && invstd && d_out, "NULL pointer");
  AVC_CHECK_ARG(aligned16(x_wimg), "split images must be 16-byte aligned");
  AVC_CHECK_ARG(!x_wimg || (x_amax && T > 0 && B > 0 && cin > 0 && cout > 0 && conv_wgrad_image_ok(T, B, cin, cout)),
                "conv backward: x_wimg needs x_amax and avc_conv_wgrad_image_bytes(T, B, cin, cout) > 0");
  AVC_TRY(ensure_arena(ctx, conv_bn_backward_scratch(T, B, cin, cout)));
  return conv_bn_act_backward_impl(ctx, T, B, cin, cout, x, weight, gamma, beta, y_pre, mean, invstd,
                                   training, act, d_out, d_x, d_weight, d_bias, d_gamma, d_beta,
                                   accumulate, S(stream), x_amax, static_cast<const _Float16*>(x_wimg));
}

int avc_conv_bn_act_backward(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                             const float* weight, const float* gamma, const float* beta,
                             const float* y_pre, const float* mean, const float* invstd,
                             int training, int act, const float* d_out, float* d_x,
                             float* d_weight, float* d_bias, float* d_gamma, float* d_beta,
                             int accumulate, void* stream) {
  AVC_CHECK_ARG(ctx && x && weight && gamma && beta && y_pre && mean && invstd && d_out, "NULL pointer");
  AVC_TRY(ensure_arena(ctx, conv_bn_backward_scratch(T, B, cin, cout)));
  return conv_bn_act_backward_impl(ctx, T, B, cin, cout, x, weight, gamma, beta, y_pre, mean, invstd,
                                   training, act, d_out, d_x, d_weight, d_bias, d_gamma, d_beta,
                                   accumulate, S(stream));
}

int avc_lstm_forward(avc_context* ctx, int T, int B, int din, int H, int reverse, const float* x,
                     int ldx, const float* w_ih, const float* w_hh, const float* b_ih,
                     const float* b_hh, float* y, int ldy, float* saved_gates, float* saved_c,
                     void* stream) {
  AVC_CHECK_ARG(ctx && x && w_ih && w_hh && b_ih && b_hh && y, "NULL pointer");
  AVC_CHECK_ARG((saved_gates == nullptr) == (saved_c == nullptr), "saved_gates/saved_c must both be set or both NULL");
  AVC_TRY(ensure_arena(ctx, lstm_forward_scratch(T, B, din, H, saved_c != nullptr)));
  return lstm_forward_impl(ctx, T, B, din, H, reverse, x, ldx, w_ih, w_hh, b_ih, b_hh, y, ldy,
                           saved_gates, saved_c, S(stream));
}

int avc_lstm_forward_ex(avc_context* ctx, int T, int B, int din, int H, int reverse, const float* x,
                        int ldx, const float* w_ih, const float* w_hh, const float* b_ih,
                        const float* b_hh, float* y, int ldy, float* saved_gates, float* saved_c,
                        const unsigned* x_amax, int x_unit, void* stream) {
  AVC_CHECK_ARG(ctx, "NULL pointer");
  AVC_CHECK_ARG(x_unit == 0 || x_unit == 1, "avc_lstm_forward_ex: x_unit must be 0 or 1");
  XHintScope hint(ctx, x, x_amax, x_unit);
  return avc_lstm_forward(ctx, T, B, din, H, reverse, x, ldx, w_ih, w_hh, b_ih, b_hh, y, ldy, saved_gates,
                          saved_c, stream);
}

int avc_bilstm_forward_ex(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                          const float* const* w_f, const float* const* w_r, float* y, int ldy,
                          float* saved_gates_f, float* saved_c_f, float* saved_gates_r, float* saved_c_r,
                          const unsigned* x_amax, int x_unit, void* stream) {
  AVC_CHECK_ARG(ctx, "NULL pointer");
  AVC_CHECK_ARG(x_unit == 0 || x_unit == 1, "avc_bilstm_forward_ex: x_unit must be 0 or 1");
  XHintScope hint(ctx, x, x_amax, x_unit);
  return avc_bilstm_forward(ctx, T, B, din, H, x, ldx, w_f, w_r, y, ldy, saved_gates_f, saved_c_f, saved_gates_r,
                            saved_c_r, stream);
}

int avc_bilstm_forward(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                       const float* const* w_f, const float* const* w_r, float* y, int ldy,
                       float* saved_gates_f, float* saved_c_f, float* saved_gates_r,
                       float* saved_c_r, void* stream) {
  AVC_CHECK_ARG(ctx && x && w_f && w_r && y, "NULL pointer");
  for (int i = 0; i < 4; ++i) AVC_CHECK_ARG(w_f[i] && w_r[i], "NULL weight pointer");
  AVC_CHECK_ARG((saved_gates_f == nullptr) == (saved_c_f == nullptr) &&
                    (saved_gates_r == nullptr) == (saved_c_r == nullptr) &&
                    (saved_c_f == nullptr) == (saved_c_r == nullptr),
                "saved buffers must all be set or all NULL");
  AVC_TRY(ensure_arena(ctx, bilstm_forward_scratch(T, B, din, H, saved_c_f != nullptr)));
  return bilstm_forward_impl(ctx, T, B, din, H, x, ldx, w_f, w_r, y, ldy, saved_gates_f, saved_c_f,
                             saved_gates_r, saved_c_r, S(stream));
}

int avc_lstm_backward(avc_context* ctx, int T, int B, int din, int H, int reverse,
                      const float* x, int ldx, const float* w_ih, const float* w_hh,
                      const float* y, int ldy, const float* saved_gates, const float* saved_c,
                      const float* d_y, float* d_x, float* d_w_ih, float* d_w_hh, float* d_b_ih,
                      float* d_b_hh, int accumulate_dx, int accumulate_dw, void* stream) {
  AVC_CHECK_ARG(ctx && x && w_ih && w_hh && y && d_y && d_w_ih && d_w_hh && d_b_ih && d_b_hh, "NULL pointer");
  AVC_TRY(ensure_arena(ctx, lstm_backward_scratch(T, B, din, H)));
  return lstm_backward_impl(ctx, T, B, din, H, reverse, x, ldx, w_ih, w_hh, y, ldy, saved_gates,
                            saved_c, d_y, d_x, d_w_ih, d_w_hh, d_b_ih, d_b_hh, accumulate_dx,
                            accumulate_dw, S(stream));
}

int avc_lstm_backward_ex(avc_context* ctx, int T, int B, int din, int H, int reverse,
                         const float* x, int ldx, const float* w_ih, const float* w_hh,
                         const float* y, int ldy, const float* saved_gates, const float* saved_c,
                         const float* d_y, float* d_x, float* d_w_ih, float* d_w_hh, float* d_b_ih,
                         float* d_b_hh, int accumulate_dx, int accumulate_dw, const unsigned* x_amax, int x_unit,
                         void* stream) {
  AVC_CHECK_ARG(ctx && x && w_ih && w_hh && y && d_y && d_w_ih && d_w_hh && d_b_ih && d_b_hh, "NULL pointer");
  AVC_CHECK_ARG(x_unit == 0 || x_unit == 1, "avc_lstm_backward_ex: x_unit must be 0 or 1");
  AVC_TRY(ensure_arena(ctx, lstm_backward_scratch(T, B, din, H)));
  XHintScope hint(ctx, x, x_amax, x_unit);
  return lstm_backward_impl(ctx, T, B, din, H, reverse, x, ldx, w_ih, w_hh, y, ldy, saved_gates,
                            saved_c, d_y, d_x, d_w_ih, d_w_hh, d_b_ih, d_b_hh, accumulate_dx,
                            accumulate_dw, S(stream), x_unit != 0);
}

int avc_linear_forward(avc_context* ctx, int M, int din, int dout, const float* x,
                       const float* weight, const float* bias, float* y, void* stream) {
  AVC_CHECK_ARG(ctx && x && weight && y, "NULL pointer");
  GemmDesc d;
  d.M = M; d.N = dout; d.Kc = din;
  d.A = x; d.lda = din;
  d.B = weight; d.b_trans = 1; d.ldb = din;
  d.bias0 = bias; d.C = y; d.ldc = dout;
  d.prec16 = 1;
  AVC_TRY(ensure_arena(ctx, gemm_scratch_bytes(d) + 4096));
  return gemm_run(ctx, d, S(stream));
}

int avc_linear_backward(avc_context* ctx, int M, int din, int dout, const float* x,
                        const float* weight, const float* d_y, float* d_x, float* d_weight,
                        float* d_bias, int accumulate, void* stream) {
  AVC_CHECK_ARG(ctx && x && weight && d_y, "NULL pointer");
  GemmDesc dx;  // d_x = d_y W
  dx.M = M; dx.N = din; dx.Kc = dout;
  dx.A = d_y; dx.lda = dout;
  dx.B = weight; dx.ldb = din;
  dx.C = d_x; dx.ldc = din; dx.accumulate = accumulate == 1;
  dx.prec16 = 1; dx.split_scale = 1;
  GemmDesc dw;  // d_W = d_y^T x
  dw.M = dout; dw.N = din; dw.Kc = M;
  dw.A = d_y; dw.a_trans = 1; dw.lda = dout;
  dw.B = x; dw.ldb = din; dw.b_rows = M;
  dw.C = d_weight; dw.ldc = din; dw.accumulate = accumulate != 0;
  dw.prec16 = 1; dw.split_scale = 1;
  AVC_TRY(ensure_arena(ctx, std::max(gemm_scratch_bytes(dx), gemm_scratch_bytes(dw)) +
                                colsum_scratch(M, dout) + 8192));
  Scratch sc(ctx);
  AVC_TAKE(amax_dy, unsigned, 64, sc);  // one max|dY| scan shared by both products
  AVC_TRY(gemm_absmax(d_y, M, dout, dout, amax_dy, S(stream)));
  dx.amax_a = dw.amax_a = amax_dy;
  if (d_x) AVC_TRY(gemm_run(ctx, dx, S(stream)));
  if (d_weight) AVC_TRY(gemm_run(ctx, dw, S(stream)));
  if (d_bias) AVC_TRY(colsum(ctx, M, dout, d_y, dout, d_bias, accumulate != 0, S(stream)));
  return AVC_OK;
}

int avc_frames_from_mel(int T, int B, int cm, const float* x, int ce, const float* emb,
                        float* out, void* stream) {
  AVC_CHECK_ARG(x && out && (ce == 0 || emb), "NULL pointer");
  return frames_from_mel(T, B, cm, x, ce, emb, out, S(stream));
}

int avc_frames_from_mel_backward(int T, int B, int cm, int ce, const float* d_frames, int ld,
                                 float* d_x, float* d_emb, int accumulate, void* stream) {
  AVC_CHECK_ARG(d_frames != nullptr, "NULL pointer");
  return frames_from_mel_backward(T, B, cm, ce, d_frames, ld, d_x, d_emb, accumulate, S(stream));
}

int avc_mel_from_frames(int T, int B, int cm, const float* frames, float* mel, void* stream) {
  AVC_CHECK_ARG(frames && mel, "NULL pointer");
  return mel_from_frames(T, B, cm, frames, mel, S(stream));
}

int avc_codes_from_encoder(int T, int B, const float* enc_out, float* codes, void* stream) {
  AVC_CHECK_ARG(enc_out && codes, "NULL pointer");
  return codes_from_encoder(T, B, enc_out, codes, S(stream));
}

int avc_codes_from_encoder_backward(int T, int B, const float* d_codes, float* d_enc_out,
                                    int accumulate, void* stream) {
  AVC_CHECK_ARG(d_codes && d_enc_out, "NULL pointer");
  return codes_from_encoder_backward(T, B, d_codes, d_enc_out, accumulate, S(stream));
}

int avc_decoder_input(int T, int B, const float* enc_out, int ce, const float* c_trg,
                      float* dec_in, void* stream) {
  AVC_CHECK_ARG(enc_out && c_trg && dec_in, "NULL pointer");
  return decoder_input(T, B, enc_out, ce, c_trg, dec_in, S(stream));
}

int avc_decoder_input_backward(int T, int B, int ce, const float* d_dec_in, float* d_enc_out,
                               int accumulate, void* stream) {
  AVC_CHECK_ARG(d_dec_in && d_enc_out, "NULL pointer");
  return decoder_input_backward(T, B, ce, d_dec_in, d_enc_out, accumulate, S(stream));
}

int avc_overlap_average(int M, int C, int N, int step, const float* frames, float* out,
                        void* stream) {
  AVC_CHECK_ARG(frames && out, "NULL pointer");
  return overlap_average(M, C, N, step, frames, out, S(stream));
}

int avc_overlap_average_backward(int M, int C, int N, int step, const float* frames, const float* d_out,
                                 float* d_frames, void* stream) {
  AVC_CHECK_ARG(frames && d_out && d_frames, "NULL pointer");
  return overlap_average_backward(M, C, N, step, frames, d_out, d_frames, S(stream));
}

int avc_loss_forward(avc_context* ctx, int kind, size_t n, const float* a, const float* b,
                     float* loss_out, int accumulate, void* stream) {
  AVC_CHECK_ARG(ctx && a && b && loss_out, "NULL pointer");
  AVC_TRY(ensure_arena(ctx, loss_scratch()));
  return loss_forward(ctx, kind, n, a, b, loss_out, accumulate, S(stream));
}

int avc_loss_backward(int kind, size_t n, const float* a, const float* b, const float* dscale,
                      float* grad_a, float* grad_b, int accumulate, void* stream) {
  AVC_CHECK_ARG(a && b, "NULL pointer");
  return loss_backward(kind, n, a, b, dscale, grad_a, grad_b, accumulate, S(stream));
}

int avc_clip_adam_ema(avc_context* ctx, size_t n, float* param, float* grad, float* exp_avg,
                      float* exp_avg_sq, float* ema, float lr, float beta1, float beta2,
                      float eps, float weight_decay, int step, float max_norm, double ema_decay,
                      float* norm_out, void* stream) {
  AVC_CHECK_ARG(ctx && param && grad && exp_avg && exp_avg_sq, "NULL pointer");
  AVC_TRY(ensure_arena(ctx, optimizer_scratch()));
  return clip_adam_ema(ctx, n, param, grad, exp_avg, exp_avg_sq, ema, lr, beta1, beta2, eps,
                       weight_decay, step, max_norm, ema_decay, norm_out, S(stream));
}

int avc_clip_adam_ema_dev(avc_context* ctx, size_t n, float* param, float* grad, float* exp_avg,
                          float* exp_avg_sq, float* ema, float lr, float beta1, float beta2,
                          float eps, float weight_decay, int calls, float max_norm, double ema_decay,
                          float* norm_out, unsigned* skips, void* stream) {
  AVC_CHECK_ARG(ctx && param && grad && exp_avg && exp_avg_sq && skips, "NULL pointer");
  AVC_TRY(ensure_arena(ctx, optimizer_scratch()));
  return clip_adam_ema(ctx, n, param, grad, exp_avg, exp_avg_sq, ema, lr, beta1, beta2, eps,
                       weight_decay, calls, max_norm, ema_decay, norm_out, S(stream), skips);
}

int avc_generator_param_count(void) { return P_COUNT; }

int avc_generator_forward(avc_context* ctx, int T, int B, const float* const* params,
                          const float* x, const float* c_org, const float* c_trg, int training,
                          float* mel, float* mel_post, float* codes, void* stream) {
  AVC_CHECK_ARG(ctx && params && x && c_org && c_trg && mel && mel_post && codes, "NULL pointer");
  for (int i = 0; i < P_COUNT; ++i) AVC_CHECK_ARG(params[i] != nullptr, "NULL parameter pointer");
  AVC_TRY(ensure_arena(ctx, gen_scratch(T, B)));
  AVC_TRY(persist_guard(ctx));
  return generator_forward(ctx, T, B, params, x, c_org, c_trg, training, mel, mel_post, codes,
                           S(stream));
}

namespace avc {
namespace {

void drop_graph(avc_context* ctx) {
  avc_gen_graph& g = ctx->gen;
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g.exec = nullptr;
  g.graph = nullptr;
  for (auto& d : g.direct) {
    if (d.exec) (void)hipGraphExecDestroy(d.exec);
    if (d.graph) (void)hipGraphDestroy(d.graph);
  }
  g.direct.clear();
  g.recent.clear();
}

constexpr size_t kDirectGraphs = 4;

// Capture the forward on the caller's I/O pointers (no staging copies).
int capture_direct(avc_context* ctx, const float* const* params, const void* const* io,
                   avc_gen_graph::direct_graph& out) {
  avc_gen_graph& g = ctx->gen;
  if (!ctx->capture_stream) AVC_HIP(hipStreamCreateWithFlags(&ctx->capture_stream, hipStreamNonBlocking));
  hipStream_t cs = ctx->capture_stream;
  AVC_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed));
  const int rc = generator_forward(ctx, g.T, g.B, params, static_cast<const float*>(io[0]),
                                   static_cast<const float*>(io[1]), static_cast<const float*>(io[2]), g.training,
                                   (float*)io[3], (float*)io[4], (float*)io[5], cs);
  hipGraph_t graph = nullptr;
  const hipError_t e = hipStreamEndCapture(cs, &graph);
  if (rc != AVC_OK) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  AVC_HIP(e);
  hipGraphExec_t exec = nullptr;
  const hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  if (ie != hipSuccess) {
    (void)hipGraphDestroy(graph);
    AVC_HIP(ie);
  }
  for (int i = 0; i < 6; ++i) out.io[i] = io[i];
  out.graph = graph;
  out.exec = exec;
  return AVC_OK;
}

size_t codes_len(int T) { return (size_t)32 * (T / 32 + (T + 31) / 32); }

// Capture the forward on the context's private stream into g (staging buffers as I/O).
int capture_graph(avc_context* ctx, const float* const* params) {
  avc_gen_graph& g = ctx->gen;
  const size_t nx = (size_t)g.B * 80 * g.T, nc = (size_t)g.B * 256, ncode = (size_t)g.B * codes_len(g.T);
  const size_t need = (3 * nx + 2 * nc + ncode) * sizeof(float);
  if (g.stage_bytes < need) {
    if (g.stage) (void)hipFree(g.stage);
    g.stage = nullptr;
    g.stage_bytes = 0;
    AVC_HIP(hipMalloc(&g.stage, need));
    g.stage_bytes = need;
  }
  if (!ctx->capture_stream) AVC_HIP(hipStreamCreateWithFlags(&ctx->capture_stream, hipStreamNonBlocking));
  float* sx = g.stage;
  float* so = sx + nx;
  float* st = so + nc;
  float* sm = st + nc;
  float* sp = sm + nx;
  float* sc = sp + nx;
  hipStream_t cs = ctx->capture_stream;
  AVC_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed));
  const int rc = generator_forward(ctx, g.T, g.B, params, sx, so, st, g.training, sm, sp, sc, cs);
  hipGraph_t graph = nullptr;
  const hipError_t e = hipStreamEndCapture(cs, &graph);
  if (rc != AVC_OK) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  AVC_HIP(e);
  g.graph = graph;
  AVC_HIP(hipGraphInstantiate(&g.exec, g.graph, nullptr, nullptr, 0));
  return AVC_OK;
}

}  // namespace
}  // namespace avc

int avc_generator_forward_cached(avc_context* ctx, int T, int B, const float* const* params,
                                 long weights_version, const float* x, const float* c_org,
                                 const float* c_trg, int training, float* mel, float* mel_post,
                                 float* codes, void* stream) {
  AVC_CHECK_ARG(ctx && params && x && c_org && c_trg && mel && mel_post && codes, "NULL pointer");
  AVC_CHECK_ARG(weights_version >= 0, "weights_version must be >= 0");
  for (int i = 0; i < P_COUNT; ++i) AVC_CHECK_ARG(params[i] != nullptr, "NULL parameter pointer");
  AVC_TRY(ensure_arena(ctx, gen_scratch(T, B)));
  AVC_TRY(persist_guard(ctx));  // an earlier persistent launch timed out: report it, reset state
  hipStream_t s = S(stream);
  avc_gen_graph& g = ctx->gen;
  const bool timing = timing_on(TC_GEMM) || timing_on(TC_LSTM_STEP_FWD) || timing_on(TC_LSTM32) ||
                      timing_on(TC_LSTM2_PERSIST) || timing_on(TC_LSTM1_PERSIST);
  const bool same = g.T == T && g.B == B && g.training == training && g.version == weights_version &&
                    g.epoch == g_config_epoch &&
                    g.params.size() == (size_t)P_COUNT &&
                    std::equal(g.params.begin(), g.params.end(), params);
  ctx->prep_version = weights_version;
  // the derived-weight cache is live only inside this call: every exit (the graph replays return
  // early) drops it again, or a later per-layer call (training between conversions) would take
  // derived weights cached for an older version of the same tensors
  struct PrepScope {
    avc_context* c;
    ~PrepScope() { c->prep_version = -1; }
  } prep_scope{ctx};
  int rc = AVC_OK;
  if (same && !timing && g_graph_mode && (g.exec || g.seen >= 1)) {
    if (!g.exec) {
      rc = capture_graph(ctx, params);
      if (rc != AVC_OK) {
        drop_graph(ctx);
        g.seen = -1000000;  // capture failed: stay eager for this key
        ctx->prep_version = -1;
        (void)hipGetLastError();
        return generator_forward(ctx, T, B, params, x, c_org, c_trg, training, mel, mel_post, codes, s);
      }
    }
    // a graph on the caller's own pointers when this pointer set recurs (no staging copies)
    const void* io[6] = {x, c_org, c_trg, mel, mel_post, codes};
    ++g.clock;
    for (auto& d : g.direct) {
      if (std::equal(io, io + 6, d.io)) {
        d.last = g.clock;
        AVC_HIP(hipGraphLaunch(d.exec, s));
        return AVC_OK;
      }
    }
    const std::vector<const void*> key(io, io + 6);
    const bool again = std::find(g.recent.begin(), g.recent.end(), key) != g.recent.end();
    if (again) {
      if (g.direct.size() >= kDirectGraphs) {  // retire the least recently used one
        auto lru = std::min_element(g.direct.begin(), g.direct.end(),
                                    [](const avc_gen_graph::direct_graph& a, const avc_gen_graph::direct_graph& b) {
                                      return a.last < b.last;
                                    });
        AVC_HIP(hipStreamSynchronize(s));  // it may still be running
        if (lru->exec) (void)hipGraphExecDestroy(lru->exec);
        if (lru->graph) (void)hipGraphDestroy(lru->graph);
        g.direct.erase(lru);
      }
      avc_gen_graph::direct_graph d;
      if (capture_direct(ctx, params, io, d) == AVC_OK) {
        d.last = g.clock;
        g.direct.push_back(d);
        g.recent.erase(std::find(g.recent.begin(), g.recent.end(), key));
        AVC_HIP(hipGraphLaunch(d.exec, s));
        return AVC_OK;
      }
      (void)hipGetLastError();  // capture failed: the staging graph below serves this call
    } else {
      if (g.recent.size() >= 8) g.recent.erase(g.recent.begin());
      g.recent.push_back(key);
    }
    const size_t nx = (size_t)B * 80 * T, nc = (size_t)B * 256, ncode = (size_t)B * codes_len(T);
    float* sx = g.stage;
    float* so = sx + nx;
    float* st = so + nc;
    float* sm = st + nc;
    float* sp = sm + nx;
    float* sc = sp + nx;
    ctx->prep_version = -1;
    AVC_HIP(hipMemcpyAsync(sx, x, nx * sizeof(float), hipMemcpyDeviceToDevice, s));
    AVC_HIP(hipMemcpyAsync(so, c_org, nc * sizeof(float), hipMemcpyDeviceToDevice, s));
    AVC_HIP(hipMemcpyAsync(st, c_trg, nc * sizeof(float), hipMemcpyDeviceToDevice, s));
    AVC_HIP(hipGraphLaunch(g.exec, s));
    AVC_HIP(hipMemcpyAsync(mel, sm, nx * sizeof(float), hipMemcpyDeviceToDevice, s));
    AVC_HIP(hipMemcpyAsync(mel_post, sp, nx * sizeof(float), hipMemcpyDeviceToDevice, s));
    AVC_HIP(hipMemcpyAsync(codes, sc, ncode * sizeof(float), hipMemcpyDeviceToDevice, s));
    return AVC_OK;
  }
  // eager call; a second consecutive call with the same key captures the graph
  if (!same) {
    drop_graph(ctx);
    g.T = T; g.B = B; g.training = training; g.version = weights_version; g.epoch = g_config_epoch;
    g.params.assign(params, params + P_COUNT);
    g.seen = 0;
  }
  rc = generator_forward(ctx, T, B, params, x, c_org, c_trg, training, mel, mel_post, codes, s);
  ctx->prep_version = -1;
  if (rc == AVC_OK) ++g.seen;
  return rc;
}

int avc_graph_mode(int on) {
  g_graph_mode = on ? 1 : 0;
  ++g_config_epoch;
  return AVC_OK;
}

int avc_prepared_release(avc_context* ctx) {
  AVC_CHECK_ARG(ctx != nullptr, "ctx is NULL");
  AVC_HIP(hipDeviceSynchronize());
  drop_graph(ctx);
  ctx->gen = avc_gen_graph();
  for (auto& e : ctx->prep) (void)hipFree(e.buf);
  ctx->prep.clear();
  return AVC_OK;
}

}  // extern "C"

extern "C" int avc_dead_h_stores(int on) {
  if (on < 0 || on > 1) {
    avc::set_error("avc_dead_h_stores: on must be 0 or 1");
    return AVC_ERR_INVALID;
  }
  avc::g_dead_y = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_split_handover(int on) {
  if (on < 0 || on > 1) {
    avc::set_error("avc_split_handover: on must be 0 or 1");
    return AVC_ERR_INVALID;
  }
  avc::g_handover = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}
