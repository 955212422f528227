// Internal declarations of the bandwidth-bound kernels (elementwise.hip).
#pragma once
#include "common.h"

namespace avc {

// amax_init != NULL: also set amax_init[0] = 0, amax_init[1] = 2^14 (bn_apply's amax_out words)
int bn_finalize(int C, int nparts, int part_rows, const float* stats, double count, int training, float momentum,
                float eps, float* rmean, float* rvar, float* mean, float* invstd, hipStream_t s,
                unsigned* amax_init = nullptr);
// frag != NULL: also write the output split into the GEMM's fragment-major A layout
// (gemm_afrag_bytes(M, C) bytes, for GemmDesc::a_frag); out may then be NULL (not stored).
// range_flag (pinned host word): set when a finite output exceeds the f16 split's range (the
// output is then range-checked: mark_range_checked lets its consumer skip the scan)
int bn_apply(long M, int C, const float* y, const float* mean, const float* invstd,
             const float* gamma, const float* beta, int act, const float* residual, float* out,
             hipStream_t s, _Float16* frag = nullptr, unsigned* range_flag = nullptr,
             unsigned* amax_out = nullptr);
// amax_out (fp32 output only; words initialised by bn_finalize's amax_init): [0] = max |out|,
// [1] = max(|out|, 2^14) -- the range-guard word a forward contraction of out would compute
size_t bn_backward_scratch(int M, int C);
int bn_backward(avc_context* ctx, int M, int C, const float* dout, const float* y,
                const float* mean, const float* invstd, const float* gamma, const float* beta,
                int act, int training, float* d_gamma, float* d_beta, int accumulate, float* dy,
                hipStream_t s, float* dy_colpart = nullptr, unsigned* dy_amax = nullptr);
// with dy_colpart ([bn_backward_rows(M, C)][C]) / dy_amax: dy's column partial sums (finish with
// colsum_finish) and max |dy| come out of the same pass that writes dy
int bn_backward_rows(int M, int C);
// bn_backward with dy written already split (round 4): imgA = dy as a row-major A
// operand (gemm_afrag_bytes(M, C)), imgT = dy^T (gemm_afrag_bytes(C, M)), both scaled by the power
// of two of *bound (zeroed by the caller; a proven upper bound on max |dy|, so GemmDesc::amax_a =
// bound with a_frag_scaled reuses the images); no fp32 dy.  dy_colpart: [bn_backward_frag_rows(M)][C].
bool bn_backward_frag_ok(int M, int C, const float* dout, const float* y);
int bn_backward_frag(avc_context* ctx, int M, int C, const float* dout, const float* y, const float* mean,
                     const float* invstd, const float* gamma, const float* beta, int act, int training,
                     float* d_gamma, float* d_beta, int accumulate, _Float16* imgA, _Float16* imgT,
                     unsigned* bound, hipStream_t s, float* dy_colpart = nullptr);
int bn_backward_frag_rows(int M);
size_t bn_backward_frag_scratch(int M, int C);
int colsum_finish(int R, int N, const float* part, float* out, int accumulate, hipStream_t s);
int frames_from_mel(int T, int B, int cm, const float* x, int ce, const float* emb, float* out,
                    hipStream_t s);
// frames_from_mel written directly as the first conv's split operand (gemm_afrag_bytes(T*B, cm+ce)),
// scaled by the range guard of x / emb it takes first: guard[0..1] = {max, max(max, 2^14)} (two
// device words; GemmDesc::a_frag_guard = guard + 1); the fp32 frames are not stored
int frames_from_mel_frag(avc_context* ctx, int T, int B, int cm, const float* x, int ce, const float* emb,
                         _Float16* frag, unsigned* guard, hipStream_t s);
int frames_from_mel_backward(int T, int B, int cm, int ce, const float* df, int ld, float* dx,
                             float* demb, int accumulate, hipStream_t s);
int mel_from_frames(int T, int B, int cm, const float* fr, float* mel, hipStream_t s,
                    const float* fr1 = nullptr, float* mel1 = nullptr);
int codes_from_encoder(int T, int B, const float* enc, float* codes, hipStream_t s);
int codes_from_encoder_backward(int T, int B, const float* dcodes, float* denc, int accumulate,
                                hipStream_t s);
// codes (optional): also the content codes (codes_from_encoder's output), in the same pass
int decoder_input(int T, int B, const float* enc, int ce, const float* ctrg, float* out,
                  hipStream_t s, unsigned* range_flag = nullptr, float* codes = nullptr);
int decoder_input_backward(int T, int B, int ce, const float* dd, float* denc, int accumulate,
                           hipStream_t s);
int overlap_average(int M, int C, int N, int step, const float* fr, float* out, hipStream_t s);
int overlap_average_backward(int M, int C, int N, int step, const float* fr, const float* dout, float* dfr,
                             hipStream_t s);
size_t loss_scratch();
int loss_forward(avc_context* ctx, int kind, size_t n, const float* a, const float* b, float* out,
                 int accumulate, hipStream_t s);
int loss_backward(int kind, size_t n, const float* a, const float* b, const float* dscale,
                  float* ga, float* gb, int accumulate, hipStream_t s);
size_t optimizer_scratch();
int clip_adam_ema(avc_context* ctx, size_t n, float* p, float* g, float* m, float* v, float* ema,
                  float lr, float b1, float b2, float eps, float wd, int step, float max_norm,
                  double ema_decay, float* norm_out, hipStream_t s, unsigned* skips = nullptr);

}  // namespace avc
