// Internal (non-ABI) entry points shared between the library's translation units.
#pragma once
#include "common.h"
#include "gemm.h"

namespace avc {

// ---- reductions / elementwise (elementwise.hip) ----
// out[n] (+)= sum_m X[m*ld + n]   (fixed-order, deterministic)
int colsum(avc_context* ctx, int M, int N, const float* X, long ld, float* out, int accumulate,
           hipStream_t s, float* out2 = nullptr);
size_t colsum_scratch(int M, int N);

// ---- LSTM (lstm.hip) ----
int lstm_forward_impl(avc_context* ctx, int T, int B, int din, int H, int reverse,
                      const float* x, int ldx, const float* w_ih, const float* w_hh,
                      const float* b_ih, const float* b_hh, float* y, int ldy,
                      float* saved_gates, float* saved_c, hipStream_t s,
                      _Float16* y_frag = nullptr);  // y also as the split image a GEMM streams (a_frag)
size_t lstm_forward_scratch(int T, int B, int din, int H, bool training);
int lstm_backward_impl(avc_context* ctx, int T, int B, int din, int H, int reverse,
                       const float* x, int ldx, const float* w_ih, const float* w_hh,
                       const float* y, int ldy, const float* saved_gates, const float* saved_c,
                       const float* d_y, float* d_x, float* d_w_ih, float* d_w_hh,
                       float* d_b_ih, float* d_b_hh, int accumulate_dx, int accumulate_dw,
                       hipStream_t s, bool x_unit = false);
size_t lstm_backward_scratch(int T, int B, int din, int H);
// two stacked layers as a wavefront (w0/w1 = {w_ih, w_hh, b_ih, b_hh}); saved buffers optional
int lstm2_forward_impl(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                       const float* const* w0, const float* const* w1, float* y0, float* y1,
                       float* g0, float* c0, float* g1, float* c1, hipStream_t s,
                       _Float16* y1_frag = nullptr);  // y1 also as a split image (a_frag)
size_t lstm2_forward_scratch(int T, int B, int din, int H, bool training);

// bidirectional layer (wf/wr = {w_ih, w_hh, b_ih, b_hh}); H = 32 runs both directions in one launch
int bilstm_forward_impl(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                        const float* const* wf, const float* const* wr, float* y, int ldy,
                        float* g_f, float* c_f, float* g_r, float* c_r, hipStream_t s,
                        const _Float16* x_frag = nullptr);  // x given only as a split image (GemmDesc::a_frag)
bool bilstm_takes_frag(int T, int B, int din);  // H = 32: its input projection streams a split x
size_t bilstm_forward_scratch(int T, int B, int din, int H, bool training);

// ---- split-fp16 LSTM forward recurrence (lstm_split.hip), used by the two above when supported
bool lstm_split_supported(int H, int din);
size_t lstm_split_forward_scratch(int T, int B, int din, int H, int nlayers);
int lstm_split_forward_impl(avc_context* ctx, int T, int B, int din, int H, int reverse,
                            const float* x, int ldx, const float* w_ih, const float* w_hh,
                            const float* b_ih, const float* b_hh, float* y, int ldy,
                            float* saved_gates, float* saved_c, hipStream_t s, _Float16* y_frag = nullptr);
int lstm2_split_forward_impl(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                             const float* const* w0, const float* const* w1, float* y0, float* y1,
                             float* g0, float* c0, float* g1, float* c1, hipStream_t s,
                             _Float16* y1_frag = nullptr);
// decoder.lstm2 as one weight-stationary launch (lstm_persist.hip); gx0 = layer 0's input
// projection, w*_s = split weights (each followed by its per-row unscale), b1_p = permuted
// b_ih1 + b_hh1
// With `ip`, layer 0's input projection runs inside the launch (slot 3) and gx0 is its output
// buffer [T][B][4H]; without it gx0 is the caller's precomputed projection.
struct InProj {
  const float* x; long ldx; int din;  // layer 0's input [T*B][din], time-major rows
  const _Float16* w_s;                // split W_ih0 (split_rows_kernel layout, K = din)
  const float* winv;                  // its per-row unscale
  const float* b0;                    // permuted b_ih0 + b_hh0
};
bool lstm2_persist_eligible(int T, int B, int H);
bool lstm2_inproj_eligible(int T, int B, int H, int din);
size_t lstm2_persist_scratch(int T, int B, int H, int din);
int lstm2_persist_forward(avc_context* ctx, int T, int B, int H, float* gx0,
                          const _Float16* w0_s, const float* winv0, const _Float16* w1i_s,
                          const float* winv1i, const _Float16* w1h_s, const float* winv1h,
                          const float* b1_p, float* y0, float* y1, float* g0, float* c0, float* g1,
                          float* c1, hipStream_t s, const InProj* ip = nullptr, _Float16* y1_frag = nullptr);
// one forward layer (decoder.lstm1) as one weight-stationary launch, batch split into
// independent groups; gx = input projection + biases, whh_s = split W_hh followed by winv
bool lstm1_persist_eligible(int T, int B, int H);
bool lstm1_inproj_eligible(int T, int B, int H, int din);
size_t lstm1_persist_scratch(int T, int B, int H, int din);
int lstm1_persist_forward(avc_context* ctx, int T, int B, int H, float* gx, const _Float16* whh_s,
                          const float* winv, float* y, float* g, float* c, hipStream_t s,
                          const InProj* ip = nullptr, _Float16* y_frag = nullptr);
// K of an input slot's split operands: din padded with zeros to 128 * (3 or 4) columns
int inproj_kpad(int din);
// BPTT of one LSTM layer direction as one persistent launch (lstm_persist.hip)
bool bptt_persist_eligible(int T, int B, int H);
size_t bptt_persist_scratch(int B, int H);
int bptt_colpart_rows(int B, int H);  // rows of bptt_persist_run's colpart
int bptt_persist_run(avc_context* ctx, int T, int B, int H, int reverse, const _Float16* whhT_s,
                     const unsigned* amax_w, const float* d_y, long ldy, const float* gates, const float* c,
                     float* dg, float* colpart, unsigned* amax_dg, hipStream_t s);
// rows of a [4H][D] gate matrix into the permuted gate order p = blk*16 + gate*4 + u (lstm.hip)
int permute_rows(const float* src, float* dst, int H, int D, hipStream_t s);

// ---- conv + BN (convbn.hip) ----
int conv_bn_act_forward_impl(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                             const float* weight, const float* bias, const float* gamma,
                             const float* beta, float* running_mean, float* running_var,
                             int training, float momentum, float eps, int act,
                             const float* residual, float* y_pre, float* out, float* mean,
                             float* invstd, hipStream_t s, const _Float16* x_frag = nullptr,
                             _Float16* out_frag = nullptr, const unsigned* x_amax = nullptr,
                             unsigned* out_amax = nullptr, const unsigned* x_frag_guard = nullptr,
                             _Float16* x_wimg = nullptr);
size_t conv_bn_forward_scratch(int T, int B, int cin, int cout);
// true when a conv with cin input channels takes its input as split fragments (x_frag honoured)
bool conv_frag_chain_ok(int T, int B, int cin, int cout);
// true when a conv's forward can hand its weight gradient the split of x (x_wimg; a shape rule:
// B % 16 == 0, T*B % 32 == 0, cin % 64 == 0); conv_wgrad_image_bytes = the image's size
bool conv_wgrad_image_ok(int T, int B, int cin, int cout);
size_t conv_wgrad_image_bytes(int T, int B, int cin);
int conv_bn_act_backward_impl(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                              const float* weight, const float* gamma, const float* beta,
                              const float* y_pre, const float* mean, const float* invstd,
                              int training, int act, const float* d_out, float* d_x,
                              float* d_weight, float* d_bias, float* d_gamma, float* d_beta,
                              int accumulate, hipStream_t s, const unsigned* x_amax = nullptr,
                              const _Float16* x_wimg = nullptr);
size_t conv_bn_backward_scratch(int T, int B, int cin, int cout);

// arena growth (only legal when no scratch is outstanding)
int ensure_arena(avc_context* ctx, size_t bytes);

}  // namespace avc
