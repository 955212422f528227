/*
 * autovc_hip.h — C ABI of the MI355X-native AutoVC Generator hot path.
 *
 * The reference (Fagprojekt-Deep-voice-conversion/AutoVC) has no FFI: its replaceable unit is
 * the Python class exported at autovc/auto_encoder/__init__.py:1 (`AutoEncoder`,
 * autovc/auto_encoder/model.py:27).  This header is the native boundary that class is rebuilt
 * on: autovc_amd.auto_encoder.AutoEncoder binds exactly these symbols with ctypes.  Each entry
 * point names the reference module/lines whose arithmetic it replaces.
 *
 * Conventions
 *   - All tensors are fp32, borrowed device pointers (the caller owns every buffer).
 *   - Activations are TIME-MAJOR "frame rows": element (t, b, c) of a [T*B][C] row-major matrix
 *     at ((t*B + b)*C + c).  Mels/codes crossing the Python boundary keep the reference's
 *     channel-first (B, 80, T) / (B, n_codes) layouts; the glue kernels convert.
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream).  All work of one
 *     call is enqueued on it; nothing blocks the host.  A context must only be used with one
 *     stream at a time (its scratch arena is stream-ordered).
 *   - Return value 0 = success; otherwise an AVC_ERR_* code and avc_last_error() holds a
 *     thread-local message.  Invalid shapes are rejected before anything is launched.
 */
#ifndef AUTOVC_HIP_H_
#define AUTOVC_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVC_OK 0
#define AVC_ERR_INVALID 1
#define AVC_ERR_HIP 2
#define AVC_ERR_WORKSPACE 3
/* a device-side failure detected after the fact: a persistent recurrence launched by an
 * earlier call on this context abandoned a bounded wait (its outputs were written as NaN) */
#define AVC_ERR_DEVICE 4

/* activation codes used by the conv/BN/linear entry points */
#define AVC_ACT_NONE 0
#define AVC_ACT_RELU 1 /* encoder.py:70, decoder.py:70 */
#define AVC_ACT_TANH 2 /* postnet.py:55 */
#define AVC_ACT_DBNORM 3 /* clip((20*log10(max(1e-5,x)) + 100) / 100, 0, 1): spectrogram.py:14-31,53-55 */

typedef struct avc_context avc_context;

/* ---- library / context ------------------------------------------------------------------ */
int avc_abi_version(void);
const char* avc_last_error(void);
int avc_context_create(int device, avc_context** out);
int avc_context_destroy(avc_context* ctx);
/* grow the scratch arena to at least `bytes` (done automatically by every entry point) */
int avc_context_reserve(avc_context* ctx, size_t bytes);

/* ---- generic fp32 MFMA GEMM (building block exported for tests) ---------------------------
 * C[M][N] (+)= A[M][K] * B[K][N] (+ bias[N]) with A row-major (a_trans=0) or stored [K][M]
 * (a_trans=1), B stored [K][N] (b_trans=0) or [N][K] (b_trans=1). */
int avc_gemm(avc_context* ctx, int M, int N, int K, const float* A, int a_trans, const float* B,
             int b_trans, const float* bias, float* C, int accumulate, void* stream);

/* ---- Conv1d(k=5,p=2) + BatchNorm1d + activation -------------------------------------------
 * Replaces ConvNorm (net_layers.py:39-49) + nn.BatchNorm1d + relu/tanh as composed in
 * encoder.py:39-48,69-70, decoder.py:41-50,69-70 and postnet.py:18-63.
 *   x        [T*B][cin]            input frames (time-major)
 *   weight   [cout][cin][5]        PyTorch Conv1d layout;  bias [cout]
 *   gamma/beta/running_mean/running_var [cout]  (running stats updated in place when training)
 *   y_pre    [T*B][cout]           out: conv output before BN (kept for backward)
 *   out      [T*B][cout]           out: act(BN(y_pre)) (+ residual [T*B][cout] if non-NULL,
 *                                  added after the activation: model.py:131-132)
 *   mean/invstd [cout]             out: the statistics used (batch stats when training)
 */
int avc_conv_bn_act_forward(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                            const float* weight, const float* bias, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            int training, float momentum, float eps, int act,
                            const float* residual, float* y_pre, float* out, float* mean,
                            float* invstd, void* stream);

/* Backward of the above.  d_out [T*B][cout] is the gradient of `out`.  Gradients are written
 * (accumulate=0) or added (accumulate=1) into d_x [T*B][cin] (may be NULL), d_weight
 * [cout][cin][5], d_bias, d_gamma, d_beta [cout]. */
int avc_conv_bn_act_backward(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                             const float* weight, const float* gamma, const float* beta,
                             const float* y_pre, const float* mean, const float* invstd,
                             int training, int act, const float* d_out, float* d_x,
                             float* d_weight, float* d_bias, float* d_gamma, float* d_beta,
                             int accumulate, void* stream);
/* accumulate (conv and linear backward): 0 = every output overwritten, 1 = every output adds
 * into its buffer, 2 = only the parameter gradients add (d_x overwritten) -- parameter
 * gradients accumulated in place across the uses of a layer (the encoder runs twice per loss). */

/* The same two calls carrying the activations' max words between layers (the per-layer training
 * path's conv -> conv chains, encoder.py:69-70 and postnet.py:54-61).  out_amax (2 device words,
 * 16-byte aligned, may be NULL) receives [0] = max |out| and [1] = max(|out|, 2^14), computed
 * while `out` is written; passing them back as the next layer's x_amax (forward: skips the range
 * scan of its input; backward: skips the max scan of x in the weight gradient) gives results
 * bit-identical to the calls above.  x_amax must describe exactly the current contents of x. */
int avc_conv_bn_act_forward_ex(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                               const float* weight, const float* bias, const float* gamma,
                               const float* beta, float* running_mean, float* running_var,
                               int training, float momentum, float eps, int act,
                               const float* residual, float* y_pre, float* out, float* mean,
                               float* invstd, const unsigned* x_amax, unsigned* out_amax, void* stream);
int avc_conv_bn_act_backward_ex(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                                const float* weight, const float* gamma, const float* beta,
                                const float* y_pre, const float* mean, const float* invstd,
                                int training, int act, const float* d_out, float* d_x,
                                float* d_weight, float* d_bias, float* d_gamma, float* d_beta,
                                int accumulate, const unsigned* x_amax, void* stream);
/* The forward of _ex handing the activation over ALSO as the split-f16 fragment image the next
 * conv's product streams (the training path's conv -> conv chains: encoder.py:69-70,
 * decoder.py:69-70, postnet.py:54-61).  out_frag (avc_act_frag_bytes(T*B, cout) bytes, 16-byte
 * aligned, may be NULL) receives act(BN(y_pre)) split hi/lo while `out` is written, range-checked
 * as the fused forward's hand-over is; x_frag (NULL, or the previous layer's out_frag for exactly
 * the current contents of x) replaces the range scan and the split of x.  Requires
 * avc_conv_frag_chain_ok(T, B, cin, cout) for x_frag.  Results are bit-identical to _ex. */
int avc_conv_bn_act_forward_frag(avc_context* ctx, int T, int B, int cin, int cout, const float* x,
                                 const void* x_frag, const float* weight, const float* bias, const float* gamma,
                                 const float* beta, float* running_mean, float* running_var, int training,
                                 float momentum, float eps, int act, const float* residual, float* y_pre,
                                 float* out, void* out_frag, float* mean, float* invstd, const unsigned* x_amax,
                                 unsigned* out_amax, void* stream);
/* 1 if a conv of this shape can take its input as a split image (B % 32 == 0, cin % 8 == 0) */
int avc_conv_frag_chain_ok(int T, int B, int cin, int cout);
/* bytes of the split image of a [rows][channels] activation (0 for an empty one) */
size_t avc_act_frag_bytes(long rows, int channels);

/* ---- LSTM layer (one direction) -----------------------------------------------------------
 * Replaces one layer-direction of nn.LSTM (gates i,f,g,o; zero initial state) as used at
 * encoder.py:51,75 (H=32, bidirectional), decoder.py:37,65 (H=512) and decoder.py:53,74
 * (H=1024, 2 layers).
 *   x      [T*B][din] (row stride ldx)    w_ih [4H][din], w_hh [4H][H], b_ih, b_hh [4H]
 *   y      [T*B][H]   written at column offset inside rows of stride ldy (bidirectional concat)
 *   saved_gates [T*B][4H], saved_c [T*B][H]  (needed for backward; may be NULL when not training)
 * reverse=1 runs t = T-1 .. 0 (the `_reverse` direction). */
int avc_lstm_forward(avc_context* ctx, int T, int B, int din, int H, int reverse, const float* x,
                     int ldx, const float* w_ih, const float* w_hh, const float* b_ih,
                     const float* b_hh, float* y, int ldy, float* saved_gates, float* saved_c,
                     void* stream);

/* Bidirectional layer (encoder.py:51,75: nn.LSTM(..., bidirectional=True)): y[:, 0:H] is the
 * forward direction, y[:, H:2H] the reverse one (rows of stride ldy).  w_f / w_r are the four
 * tensors {w_ih, w_hh, b_ih, b_hh} of each direction; saved buffers per direction as in
 * avc_lstm_forward.  For H = 32 both directions run in one launch. */
int avc_bilstm_forward(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                       const float* const* w_f, const float* const* w_r, float* y, int ldy,
                       float* saved_gates_f, float* saved_c_f, float* saved_gates_r,
                       float* saved_c_r, void* stream);

/* Backward through time.  d_y [T*B] rows of stride ldy (gradient of y).  Writes
 * (accumulate_dx/accumulate_dw = 0) or adds (= 1) d_x [T*B][din] (may be NULL) and d_w_ih,
 * d_w_hh, d_b_ih, d_b_hh (PyTorch layout); the two directions of a bidirectional layer share
 * d_x, hence the separate flags. */
int avc_lstm_backward(avc_context* ctx, int T, int B, int din, int H, int reverse,
                      const float* x, int ldx, const float* w_ih, const float* w_hh,
                      const float* y, int ldy, const float* saved_gates, const float* saved_c,
                      const float* d_y, float* d_x, float* d_w_ih, float* d_w_hh, float* d_b_ih,
                      float* d_b_hh, int accumulate_dx, int accumulate_dw, void* stream);
/* Round 5: the LSTM calls with what the caller knows about x, so no product or split scans it.
 * x_amax (device, may be NULL): two words from x's producer, [0] = max |x|, [1] = max(max |x|, 2^14)
 * (avc_conv_bn_act_forward_frag's out_amax); x_unit = 1: every |x| <= 1 (x is another LSTM layer's
 * h = o tanh(c)).  The input projection's guard, the input slot's split scale and the W_ih
 * gradient's split of x take them; with x_amax every value is the one the scan would have found
 * (same bits), with x_unit the bound 1.  Otherwise as the calls without _ex. */
int avc_lstm_forward_ex(avc_context* ctx, int T, int B, int din, int H, int reverse, const float* x,
                        int ldx, const float* w_ih, const float* w_hh, const float* b_ih,
                        const float* b_hh, float* y, int ldy, float* saved_gates, float* saved_c,
                        const unsigned* x_amax, int x_unit, void* stream);
int avc_bilstm_forward_ex(avc_context* ctx, int T, int B, int din, int H, const float* x, int ldx,
                          const float* const* w_f, const float* const* w_r, float* y, int ldy,
                          float* saved_gates_f, float* saved_c_f, float* saved_gates_r, float* saved_c_r,
                          const unsigned* x_amax, int x_unit, void* stream);
int avc_lstm_backward_ex(avc_context* ctx, int T, int B, int din, int H, int reverse,
                         const float* x, int ldx, const float* w_ih, const float* w_hh,
                         const float* y, int ldy, const float* saved_gates, const float* saved_c,
                         const float* d_y, float* d_x, float* d_w_ih, float* d_w_hh, float* d_b_ih,
                         float* d_b_hh, int accumulate_dx, int accumulate_dw, const unsigned* x_amax,
                         int x_unit, void* stream);

/* ---- Linear (decoder.linear_projection, decoder.py:56,77; net_layers.py:3-20) ------------ */
int avc_linear_forward(avc_context* ctx, int M, int din, int dout, const float* x,
                       const float* weight, const float* bias, float* y, void* stream);
int avc_linear_backward(avc_context* ctx, int M, int din, int dout, const float* x,
                        const float* weight, const float* d_y, float* d_x, float* d_weight,
                        float* d_bias, int accumulate, void* stream);

/* ---- layout glue --------------------------------------------------------------------------
 * frames_from_mel: x (B,cm,T) channel-first + optional per-utterance embedding emb (B,ce)
 * broadcast over time (encoder.py:65-66, model.py:124) -> out [T*B][cm+ce].  */
int avc_frames_from_mel(int T, int B, int cm, const float* x, int ce, const float* emb,
                        float* out, void* stream);
/* backward: d_x (B,cm,T) (+)= transpose of the first cm columns of d_frames [T*B][ld];
 * d_emb (B,ce) (+)= time-sum of columns [cm, cm+ce) (d_emb may be NULL). */
int avc_frames_from_mel_backward(int T, int B, int cm, int ce, const float* d_frames, int ld,
                                 float* d_x, float* d_emb, int accumulate, void* stream);
/* mel_from_frames: frames [T*B][cm] -> mel (B,cm,T) (model.py:127 transpose) */
int avc_mel_from_frames(int T, int B, int cm, const float* frames, float* mel, void* stream);

/* Content codes (encoder.py:94-96, model.py:99/143): enc_out [T*B][64] (fwd||bwd) ->
 * codes (B, 32*(floor(T/32)+ceil(T/32))).  T must be >= 32. */
int avc_codes_from_encoder(int T, int B, const float* enc_out, float* codes, void* stream);
int avc_codes_from_encoder_backward(int T, int B, const float* d_codes, float* d_enc_out,
                                    int accumulate, void* stream);
/* Decoder input (model.py:115-124): upsampled codes ++ c_trg -> dec_in [T*B][64+ce]. */
int avc_decoder_input(int T, int B, const float* enc_out, int ce, const float* c_trg,
                      float* dec_in, void* stream);
/* d_enc_out (+)= backward of the upsampling of the first 64 columns of d_dec_in. */
int avc_decoder_input_backward(int T, int B, int ce, const float* d_dec_in, float* d_enc_out,
                               int accumulate, void* stream);

/* Long-form paste (AutoEncoder.batch_forward, model.py:428-437): M converted slices
 * frames (M, C, N), slice i shifted right by i*step frames, NaN-padded and nan-averaged:
 * out (C, (M-1)*step + N). */
int avc_overlap_average(int M, int C, int N, int step, const float* frames, float* out,
                        void* stream);
/* Its backward (torch's nanmean backward: d_out / count of non-NaN slices at the column, 0 for NaN
 * entries), so batch_forward keeps the autograd graph like the reference: d_frames (M, C, N). */
int avc_overlap_average_backward(int M, int C, int N, int step, const float* frames, const float* d_out,
                                 float* d_frames, void* stream);

/* ---- losses (model.py:184-215; criteria at model.py:286-288) -----------------------------
 * kind 0 = nn.MSELoss (mean of (a-b)^2), kind 1 = nn.L1Loss (mean of |a-b|).
 * forward : loss_out[0] (+)= loss(a, b)   (fixed-order fp64 reduction)
 * backward: grad_a (+)= dL/da * dscale[0], grad_b (+)= dL/db * dscale[0]; dscale is a DEVICE
 *           scalar (the incoming gradient of the loss, 1 when NULL); grad_a/grad_b may be NULL. */
int avc_loss_forward(avc_context* ctx, int kind, size_t n, const float* a, const float* b,
                     float* loss_out, int accumulate, void* stream);
int avc_loss_backward(int kind, size_t n, const float* a, const float* b, const float* dscale,
                      float* grad_a, float* grad_b, int accumulate, void* stream);

/* ---- optimizer (model.py:312-321) ---------------------------------------------------------
 * One fused pass over flat buffers of n parameters:
 *   total_norm = ||grad||_2 (written to norm_out[0]); coef = min(1, max_norm/(norm+1e-6))
 *   Adam(lr, beta1, beta2, eps, weight_decay, step) with the clipped gradient (torch.optim.Adam
 *   semantics, amsgrad=False), then ema = ema_decay*ema + (1-ema_decay)*param (ema may be NULL),
 *   rounded like the reference's fp32 tensor expression with Python-double scalars.
 * max_norm <= 0 disables clipping.  A non-finite total_norm (a persistent recurrence that gave
 * up writes NaN gradients) skips the update: param, exp_avg, exp_avg_sq and ema are left as they
 * were (torch would write NaN into all of them).  Needs the norm: max_norm > 0 or
 * norm_out != NULL. */
int avc_clip_adam_ema(avc_context* ctx, size_t n, float* param, float* grad, float* exp_avg,
                      float* exp_avg_sq, float* ema, float lr, float beta1, float beta2,
                      float eps, float weight_decay, int step, float max_norm, double ema_decay,
                      float* norm_out, void* stream);
/* The same update with the count of skipped updates kept on the device: `calls` counts every
 * update requested so far (this one included); *skips (device word, zero-initialised by the
 * caller) counts those skipped for a non-finite norm and is raised by this call when it skips.
 * Adam's bias correction uses calls - *skips (host-computed values for up to 7 skips), so the
 * caller never waits for the norm to know the step count.  Needs the norm (max_norm > 0 or norm_out). */
int avc_clip_adam_ema_dev(avc_context* ctx, size_t n, float* param, float* grad, float* exp_avg,
                          float* exp_avg_sq, float* ema, float lr, float beta1, float beta2,
                          float eps, float weight_decay, int calls, float max_norm, double ema_decay,
                          float* norm_out, unsigned* skips, void* stream);

/* ---- whole Generator forward (inference / convert(), model.py:68-146) ---------------------
 * One call runs the full encoder -> upsample -> decoder -> postnet chain on device, with the
 * same semantics as the layer entry points.  `params` is an array of device pointers in the
 * reference state_dict order (avc_generator_param_count() entries: every tensor of
 * AutoEncoder.state_dict() except num_batches_tracked).  training!=0 uses batch statistics
 * and updates the running buffers in place, exactly like the reference's convert() which
 * never calls .eval().  x (B,80,T), c_org/c_trg (B,256) -> mel, mel_post (B,80,T),
 * codes (B, 32*(floor(T/32)+ceil(T/32))). */
int avc_generator_param_count(void);
int avc_generator_forward(avc_context* ctx, int T, int B, const float* const* params,
                          const float* x, const float* c_org, const float* c_trg, int training,
                          float* mel, float* mel_post, float* codes, void* stream);

/* Same as avc_generator_forward, but the derived weight layouts (split-f16 fragment-major
 * copies, permuted LSTM gate rows, conv tap transposes) are kept in the context between calls
 * and rebuilt only when `weights_version` differs from the last call's (or a parameter pointer
 * changed).  The caller bumps the version whenever any weight changes (the Python drop-in
 * derives it from the parameters' in-place version counters and its optimizer's step count).
 * Replaces the reference's convert() hot loop (voice_converter.py:163-175) for repeated calls
 * on fixed weights. */
int avc_generator_forward_cached(avc_context* ctx, int T, int B, const float* const* params,
                                 long weights_version, const float* x, const float* c_org,
                                 const float* c_trg, int training, float* mel, float* mel_post,
                                 float* codes, void* stream);
/* Frees every cached derived-weight buffer of the context. */
int avc_prepared_release(avc_context* ctx);

/* ---- measurement (bench.py) ---------------------------------------------------------------
 * When bit `cls` of mask is set, every launch of that kernel class is bracketed by HIP events on
 * its stream; avc_timing_read sums the event-measured durations and the algorithmic FLOPs/bytes
 * of the recorded launches.  Classes: 0 GEMM (gemm_kernel), 1 LSTM step forward,
 * 2 LSTM step backward, 3 H=32 persistent LSTM, 4 fp64 DFT of the mel frontends,
 * 5 the weight-stationary decoder.lstm2 recurrence (one launch per forward). */
int avc_timing_enable(int mask);
/* Tuning hook for the per-step LSTM kernel: force the batch rows per workgroup (16/32/64) and the
 * number of waves splitting the reduction (1..8); 0 restores the automatic choice. */
int avc_lstm_tune(int rows_per_block, int waves);
/* BPTT recurrence of H = 512 / 1024 LSTMs with batch >= 32 (training backward): per step a
 * split-K 3xf16 product on pre-split operands + a per-batch-row epilogue, or the fp32 step
 * kernel (lstm_step_kernel).  0 = step kernel always, 1 = split-K where it measured faster
 * (H = 1024; default), 2 = split-K wherever eligible. */
int avc_bptt_mode(int mode);
/* Tuning hook for the split-fp16 forward step (lstm_split.hip): force the K range per workgroup
 * (a multiple of 32) and the 16-column gate blocks per workgroup tile (1 or 4); 0 = automatic.
 * rows64 = 1 keeps 64 batch rows per workgroup on the narrow tiles (else 32 when that fills
 * more CUs). */
int avc_lstm_split_tune(int kslice, int col_blocks, int rows64);
/* Tuning hook for split-f16 products: 0 = every product on the fp32 MFMA kernel; 1 = forward
 * products split while staged; 2 = forward products on pre-split fragments and backward products
 * scaled-split (default); 3 = as 2 but backward products on the fp32 kernel. */
int avc_gemm_tune(int prec16);
/* Tuning hook: variant of the pre-split split-f16 GEMM for 128x128 tiles (8 waves each):
 * 0 = 4x2 waves, 4-stage ring of 32-deep K-tiles; 1 = 4x2, 2 stages of 64-deep K-tiles, Kahan
 * fold of the 128-k partials; 2 = 4x2, 3 stages x 48; 3 = 2x4, 4 x 32; 4 = 2x4, 2 x 64; 5 = 4x2,
 * 3 x 32; 6 / 7 = 4x2, 2 x 32 / 2 x 64 with plain (not Kahan-compensated) 128-k partial folds,
 * 128 VGPRs (two workgroups per CU for 6); 8 (default) = 1 with the plain fold; 9 / 10 = 256 x 128 tiles,
 * 3 stages x 32, plain fold / hi.hi products in one MFMA chain over K; 11 = 8 with the hi.hi
 * products in one chain (no 128-k partials).  Default 8. */
int avc_gemm_config(int cfg);
/* Conv1d + BatchNorm1d + activation forward (the reference's ConvNorm -> BatchNorm1d -> relu /
 * tanh, encoder.py:69-70, decoder.py:69-70, postnet.py:54-61): 1 (default) = BatchNorm fused
 * into the convolution's GEMM epilogue wherever the GEMM's grid is one co-resident wave of
 * workgroups (train mode: a column-tile barrier inside the launch, whose group -- one column
 * tile's row tiles, a contiguous dispatch range -- must be resident at once; eval mode: running
 * statistics); 2 = fused wherever one such group fits the device (grids of several waves);
 * 0 = the GEMM, a statistics launch and a normalise launch.  All give the same bits. */
/* Tuning hook (round 5): 1 (default) = the fused-BN GEMM deals each XCD a contiguous band of a
 * column group's row tiles (the conv taps' neighbouring row tiles then share its L2); 0 = round 4's
 * order (row tile = dispatch index within the group).  Same products: bit-identical. */
int avc_bn_fuse_band(int on);
int avc_bn_fuse(int on);
/* Whole-Generator forward: 1 (default) = the encoder's last conv, decoder lstm1 and decoder lstm2
 * hand their outputs to the next contraction (BiLSTM projection, first decoder conv, Linear) as
 * the split image that contraction streams, written by their own epilogues; 0 = fp32 outputs and
 * a split pass in front of each consumer.  Both give the same bits. */
int avc_split_handover(int on);
/* Whole-Generator forward: 1 (default) = the persistent recurrences skip the fp32 h stores nothing
 * reads (lstm2's layer 0, handed to layer 1 as the split hand-off; lstm1's and lstm2's last layer
 * where the next contraction streams their split image); 0 = store them.  Same outputs either way. */
int avc_dead_h_stores(int on);
/* Test hook: the next `launches` train-mode fused-BatchNorm conv launches give up at their
 * barrier's first unmet poll (NaN outputs; the next call or avc_persist_check reports it, as for
 * avc_debug_persist_inject). */
int avc_debug_bnf_inject(int launches);
/* Decoder lstm2 (two stacked layers, H = 512 or 1024, batch <= 64) and decoder lstm1 (one layer,
 * batch <= 256) as ONE weight-stationary launch each (lstm_persist.hip) instead of one launch per
 * time step: 0 = never; whenever eligible with the in-launch hand-offs read 1 = after an
 * agent-scope acquire, 2 = by sc1 loads (default).
 * Every path computes the same arithmetic in the same order (bit-identical outputs). */
int avc_lstm_persist_tune(int mode);
/* Tuning hook: split-h chunks the persistent recurrence keeps in flight ahead of the chunk being
 * multiplied (1 or 2 = default; 3 or 4 select deeper instances of the batch-halves form only,
 * avc_lstm_persist_halves, whose chunks are half as large); same arithmetic either way. */
int avc_lstm_persist_depth(int chunks);
/* Tuning hook: the persistent recurrences' per-step waits.  Bit set = every wave waits for the
 * quarter of the producing slot whose h it multiplies (quarter counters, no workgroup barrier);
 * clear = one polling lane per operand and a workgroup barrier.  Bit 0: two-layer form (lstm2),
 * bit 1: one-layer form (lstm1); default 1.  Same arithmetic either way (bit-identical). */
int avc_lstm_persist_qwait(int mask);
/* Tuning hook: 1 = the one-layer persistent form at H = 512 (decoder lstm1) hands split h from
 * step to step as data-tagged 8-B granules (no counter, drain or barrier on the step's critical
 * path); 0 (default since round 4: 20 us faster at C2, equal at C5, half the h bytes) = the counter
 * hand-off.  Applies when bit 1 of the qwait mask is clear and
 * the default hand-off form and depth are set.  Same arithmetic either way (bit-identical). */
int avc_lstm_persist_granules(int on);
/* Tuning hook (round 5): sentinel hand-off of split h in the persistent recurrences, bit 0 = the
 * two-layer form (decoder.lstm2), bit 1 = the one-layer form (decoder.lstm1).  The split-h buffers
 * live in the launch's region as two sets (launch epoch parity), every byte 0xFF until written;
 * consumers re-load an h chunk until none of its dwords is 0xFFFFFFFF (a pair of f16 NaNs no
 * producer writes) instead of waiting on arrival counters, and each producer resets its bytes in the
 * other set for the next launch.  Same products in the same order: bit-identical outputs. */
int avc_lstm_persist_sentinel(int mask);
/* Tuning hook (round 5): 1 (default) = the persistent recurrences hand split h over in 16-B
 * pieces (the two pair leads sharing a fragment piece exchange halves by a lane shuffle; one
 * write-through store each); 0 = two 8-B stores per pair lead.  Same bytes. */
int avc_lstm_persist_st16(int on);
/* Tuning hook (round 5): 1 = the two-layer persistent form (decoder.lstm2, batch > 16) waits per
 * 32-deep chunk of h (a counter per chunk that its two producing workgroups count in on, polled one
 * chunk ahead of the loads) instead of for the whole K quarter a wave reads; 0 (default) = the
 * quarter counters.  Same products in the same order: bit-identical outputs. */
int avc_lstm_persist_chunkwait(int on);
/* Tuning hook (round 5): 1 = the one-layer persistent form (decoder.lstm1, H = 512, at most 8
 * recurrent + input-slot groups) deals each batch group's workgroups to one XCD and, where a
 * run-time check confirms they share one, hands h over with plain stores that stay in that XCD's L2
 * and signals each step through a line of per-workgroup tags there (the consumers' sc1 loads read
 * both); any other group keeps the write-through stores and counters.  Same arithmetic
 * (bit-identical); 0 (default: measured no faster) = the round-4 grid. */
int avc_lstm_persist_xcd(int on);
/* Test hook: recurrent workgroups of XCD-local launches that found their group on one XCD / not,
 * since the last call (two words, then cleared). */
int avc_debug_xl_census(unsigned* local_nonlocal);
/* Test hook: 1 = the XCD-local forms (avc_lstm_persist_xcd, avc_bptt_xcd) treat every group as not
 * local and run their fallback (write-through stores, counters) -- the path a box whose workgroup
 * deal differs takes.  Same bits. */
int avc_debug_xl_force_remote(int on);
/* Tuning hook (round 5): 1 (default) = long-K products (weight gradients) pick their split-K count
 * by rounds of one workgroup per CU (a grid that spills a few workgroups into an extra round pays
 * the whole round); 0 = ~4 workgroups per CU (round 4).  The sums split differently: not
 * bit-identical, same accuracy. */
int avc_gemm_plan_rounds(int on);
/* Tuning hook: 1 = the two-layer persistent form (decoder lstm2, batch > 16) walks its
 * workgroup's rows as two independent batch halves, step t of one half while the other half's
 * hand-off is in flight (counters per step and half); 0 (default, measured faster) = all rows at
 * once.  Same arithmetic either way (bit-identical). */
int avc_lstm_persist_halves(int on);
/* Tuning hook: 1 (default) = the backward of Conv1d + BatchNorm (avc_conv_bn_act_backward*) has its
 * BatchNorm backward write dY already split for both products (the dgrad operand dY and the weight
 * gradient's dY^T, fragment images scaled by a proven upper bound on max |dY|), instead of an fp32
 * dY that a max scan and two split passes re-read; 0 = the fp32 dY path.  The products agree to the
 * last bit except where an element lies 2^-27 below the operand's max. */
int avc_bn_bwd_frag(int on);
/* Tuning hook: 1 (default) = the persistent BPTT's epilogue phase maps its threads unit-group-fast,
 * so its reads of the split-K partials are whole cache lines, and stages the split dG it writes for
 * the next step in LDS (whole-run stores); 0 = the round-3 row-fast mapping.  Same dG, dc and split
 * dG bits; the bias gradients' column sums are combined in a different (fixed) order. */
int avc_bptt_coalesce(int on);
/* Tuning hook: 1 (default) = the LSTM backward splits dG for its dX product (A operand) and for its
 * two weight-gradient products (A^T operand) in ONE pass over the fp32 dG (split_frag32_dual_kernel),
 * where the shapes allow (T * B % 32 == 0, 4H % 64 == 0); 0 = two split passes.  Same bits. */
int avc_dg_dual_split(int on);
/* Tuning hook: which recurrences may take the persistent form (bit 0 = one layer, e.g. decoder
 * lstm1; bit 1 = two stacked layers, decoder lstm2; default 3 = both). */
int avc_lstm_persist_layers(int mask);
/* Synchronises the device and returns in *giveups the number of persistent-recurrence launches
 * that abandoned a bounded wait since the library was loaded (0 = every launch completed). */
int avc_lstm_persist_status(long* giveups);
/* Health check of a context (the persistent recurrences' safety net, lstm_persist.hip):
 * synchronises `stream`, then returns AVC_ERR_DEVICE if a persistent launch of this context timed
 * out since the last check (*failed = 1) and AVC_OK otherwise (*failed = 0).  Every entry point
 * that launches a persistent recurrence performs the same check (without the synchronisation)
 * before launching, so a failure is reported by the next call at the latest. */
int avc_persist_check(avc_context* ctx, void* stream, int* failed);
/* Tuning hook: launch the persistent recurrences with hipLaunchCooperativeKernel (1) instead of
 * a plain launch after an occupancy check (0, default).  Both require every workgroup to be
 * co-resident; the cooperative launch has the runtime guarantee it. */
int avc_lstm_persist_coop(int on);
/* Tuning hook: decoder lstm1's and lstm2's layer-0 input projection (decoder.py:50,53: the
 * x W_ih0^T term of nn.LSTM) computed inside the persistent launch, one time step at a time on the
 * CUs the recurrence leaves idle (1, default), or by a GEMM before the launch (0; then the
 * persistent and launch-per-step forms are bit-identical).  2 / 3: as 1 with the input slot held
 * at most 12 steps ahead of the recurrence, checked every 4th step / every step (experiments). */
int avc_lstm_persist_inproj(int on);
/* Tuning hook for the encoder BiLSTM (H = 32) recurrence: 1 (default) = hardware exp/reciprocal
 * gate math and an 8-step prefetch of the input projection; 0 = libm gate math, 3-step prefetch. */
int avc_lstm32_tune(int mode);
/* Tuning hook: the BPTT of LSTM layers with B = 128 / 256 and H a multiple of 128 as one
 * persistent launch (1, default; lstm_persist.hip: bptt_persist_kernel) or launch per step (0). */
int avc_bptt_persist(int on);
/* Tuning hook (round 5): 1 (default) = the persistent BPTT of an H = 512 layer (decoder.lstm1)
 * runs XCD-local: groups of 32 batch rows, each on one XCD's 32 CUs with all of W_hh^T in their
 * LDS, one in-XCD hand-off per step (bptt_xl_kernel), for the batches the 128-row-tile form takes
 * (B = 256; same bits); 2 = also every other batch of whole 32-row groups up to 256, which
 * otherwise run the launch-per-step BPTT (within 2e-5 of it, not the same bits); 0 = the
 * 128-row-tile form. */
int avc_bptt_xcd(int on);
/* Diagnostic hook (timing experiments only; results are NOT valid while set): bit 0 skips the
 * persistent BPTT's dG operand loads, bit 1 its partial loads, bit 2 its waits. */
int avc_debug_bptt_diag(int bits);
/* Test hook: the next `launches` persistent launches give up at their first unsatisfied wait (as
 * if a peer workgroup never became resident); eager launches only (captured graphs are dropped). */
int avc_debug_persist_inject(int launches);
/* Co-residency hooks (replaces nothing in the reference: its training step,
 * autovc/auto_encoder/model.py:312-318, has no persistent kernels).  A persistent launch needs
 * every workgroup resident; a kernel of another stream that waits on something outside the GPU
 * (an RCCL collective waiting for a peer rank) must not hold CUs while one dispatches.
 * avc_persist_notify: record `event` (a hipEvent_t; NULL = none) on the launch stream right after
 *   every later persistent launch on ctx, so a caller can start collectives behind the recurrence
 *   (autovc_amd/dp.py GradBuckets).
 * avc_persist_launches: persistent launches enqueued on ctx so far.
 * avc_bptt_persist_eligible: 1 if avc_lstm_backward at (T, B, H) runs the persistent BPTT.
 * The environment variable AVC_PERSIST_XPROC_LOCK=<file> serialises persistent launches across
 * processes that share one GPU (flock held from the launch until the kernel has finished). */
int avc_persist_notify(avc_context* ctx, void* event);
int avc_persist_launches(avc_context* ctx, long* count);
int avc_bptt_persist_eligible(int T, int B, int H);
/* Test hooks for the co-residency tests: the spin limit of the persistent kernels' bounded waits in
 * polls (0 = the default, 2^21); a load of n_wg workgroups holding lds_bytes of LDS each (a whole
 * CU at 163840) for `usec` microseconds on `stream`, and how many of them have started. */
int avc_debug_persist_spin_limit(unsigned polls);
int avc_debug_hog(avc_context* ctx, int n_wg, int lds_bytes, long usec, void* stream);
int avc_debug_hog_resident(avc_context* ctx, int* n);
/* Test hook: per_xcd[8] = how many of the current hog's started workgroups run on each XCD
 * (HW_REG_XCC_ID), so a co-residency test can state the CUs each XCD has left. */
int avc_debug_hog_xcds(avc_context* ctx, int* per_xcd);
/* Forward-graph policy of avc_generator_forward_cached: 1 = capture on the second call with the
 * same key and replay (default); 0 = always eager (tests that need eager reference outputs). */
int avc_graph_mode(int on);
int avc_timing_reset(void);
int avc_timing_read(int cls, double* total_ms, double* total_flops, double* total_bytes,
                    long* launches);

/* ---- rows either side of the Generator ----------------------------------------
 * Mel frontends of autovc/audio/spectrogram.py and the speaker encoder of
 * autovc/speaker_encoder/model.py (inference).  librosa's algorithms (stft center=True with a
 * periodic Hann window centred in n_fft; filters.mel with the Slaney scale and norm) restated.
 *
 * avc_stft_frames: frames of a centred STFT, 1 + n_samples / hop.
 * avc_mel_basis: librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) as [n_mels][ld] fp32 rows
 *   (ld >= n_fft/2 + 1, zero tail); replaces the call inside librosa.feature.melspectrogram
 *   (spectrogram.py:118, 200-205). */
int avc_stft_frames(long n_samples, int hop);
int avc_mel_basis(double sr, int n_fft, int n_mels, double fmin, double fmax, int ld, float* out,
                  void* stream);
/* avc_mel_spectrogram: wav [n_samples] -> out = mel_basis . |stft(wav)|^power, then with
 * db_normalize = 1 the dB + normalisation of spectrogram.py:121-125 (AVC_ACT_DBNORM).
 *   pad_mode 0 = zeros, 1 = reflect (librosa < 0.10); power 1 (auto-encoder
 *   frontend, spectrogram.py:112-118) or 2 (speaker encoder, spectrogram.py:200-205);
 *   mel_basis [n_mels][ld_basis] from avc_mel_basis with ld_basis = (n_fft/2 + 1) rounded up to 4;
 *   out (n_mels, F) if channels_first else (F, n_mels), F = avc_stft_frames(n_samples, hop). */
int avc_mel_spectrogram(avc_context* ctx, const float* wav, long n_samples, int n_fft, int hop,
                        int win_length, int pad_mode, int power, const float* mel_basis, int n_mels,
                        int ld_basis, int db_normalize, int channels_first, float* out, void* stream);
/* Speaker encoder forward (speaker_encoder/model.py:71-91): 3-layer LSTM (n_in -> H, zero
 * state), Linear(H -> E) + ReLU on the last layer's final hidden state, L2-normalised rows.
 *   x (B, T, n_in) batch-first; params = the 14 tensors of SpeakerEncoder.state_dict() in order
 *   (lstm.{weight_ih,weight_hh,bias_ih,bias_hh}_l{0,1,2}, linear.weight, linear.bias);
 *   embeds (B, E). */
int avc_speaker_encoder_param_count(void);
int avc_speaker_encoder_forward(avc_context* ctx, int T, int B, int n_in, int H, int E,
                                const float* const* params, const float* x, float* embeds,
                                void* stream);
/* embed_utterance's reduction (speaker_encoder/model.py:189-190): out[E] = mean_b(embeds[b]),
 * L2-normalised. */
int avc_embedding_mean_normalize(int B, int E, const float* embeds, float* out, void* stream);

/* ---- WaveRNN vocoder `generate` (autovc/wavernn/model.py:214-329) ---------
 * dims[11] = {feat_dims, compute_dims, res_out_dims, res_blocks, rnn_dims, fc_dims, n_classes,
 *             pad, upsample_factors[0..2]} (hparams.py:92-107; n_classes 30 for MOL, 2 * bits RAW).
 * params = the float tensors of WaveRNN.state_dict() in order, without `step` and the BatchNorm
 *   `num_batches_tracked` counters (avc_wavernn_param_count(res_blocks) pointers).
 * avc_wavernn_upsample: generate()'s up-sampling (model.py:249-252) of a (1, F, T) mel:
 *   m [T * hop][F] (time-major), aux [T][res_out_dims] at frame rate (replaces
 *   UpsampleNetwork.forward, model.py:80-93, eval-mode BN).
 * avc_wavernn_generate: replaces WaveRNN.generate's body (model.py:243-329).  batched folds the
 *   T * hop positions into rows of target + 2 * overlap (avc_wavernn_fold_shape gives rows x steps);
 *   mol = 1 samples the mixture of logistics (distribution.py:87-123), 0 the RAW categorical;
 *   uniforms come from a counter-based stream keyed by `seed`.  Outputs: samples [rows][steps]
 *   (optional), wave [(T - 1) * hop] float32 after cross-fade and fade-out (needs T >= 21).
 *   With x_teacher [rows][steps] != NULL the call is the reference's teacher-forced
 *   forward(x, mels) (model.py:180-211): the mel carries `pad` real context frames on each side,
 *   the previous samples come from x_teacher and logits [rows][steps][n_classes] are written.
 *   The call returns after the generated samples are complete (stream-synchronous). */
int avc_wavernn_param_count(int res_blocks);
int avc_wavernn_fold_shape(long n_positions, int batched, int target, int overlap, long* rows, long* steps);
int avc_wavernn_upsample(avc_context* ctx, const int* dims, int T, const float* const* params, const float* mel,
                         float* m, float* aux, void* stream);
int avc_wavernn_generate(avc_context* ctx, const int* dims, int T, const float* const* params, const float* mel,
                         int batched, int target, int overlap, int mol, unsigned long long seed,
                         const float* x_teacher, float* logits, float* samples, float* wave, void* stream);
/* Tuning hook: 1 (default) = avc_wavernn_generate runs the whole sample loop as ONE persistent launch of
 * rnn_dims / 2 workgroups with in-launch hand-offs where eligible
 * (avc_wavernn_persist_eligible: <= 96 fold rows, 2 * ceil(fc_dims / 8) + rows <= rnn_dims / 2,
 * every workgroup resident); 0 = five graph-captured launches per sample step.  Same arithmetic,
 * bit-identical samples, logits and waveform.  A loop launch that abandons a bounded wait (its
 * workgroups could not all be resident, e.g. CUs held by another process) is re-run by the same
 * call on the per-step graph path from a fresh state (same bits); avc_wavernn_fallbacks() counts
 * such re-runs. */
int avc_wavernn_persist(int on);
int avc_wavernn_fallbacks(void);
/* Tuning hook: 1 (default) = generate()'s input projection of every sample position (pI) as an
 * LDS-tiled kernel; 0 = one thread per output.  Same bits. */
int avc_wavernn_proj_tiled(int on);
int avc_wavernn_persist_eligible(int rows, int rnn_dims, int fc_dims);
/* Test hook: the next `launches` loop launches give up at their first unmet wait. */
int avc_debug_wavernn_inject(int launches);
/* Diagnostics: the next avc_wavernn_generate call (if its loop runs as one launch) stamps its first
 * `steps` steps (s_memrealtime, 100 MHz) into buf [rnn_dims / 2][steps][24] (u64; per op of the
 * loop: start, wait done, end).  That call consumes the request whichever path it takes. */
int avc_debug_wavernn_stamps(void* buf, int steps);

#ifdef __cplusplus
}
#endif

#endif /* AUTOVC_HIP_H_ */
