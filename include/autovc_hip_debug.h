/*
 * autovc_hip_debug.h -- tuning toggles, test hooks and diagnostics of libautovc_hip.so.
 *
 * NOT part of the drop-in product surface (include/autovc_hip.h is): these entry points select
 * kernel variants kept for same-binary A/B measurement (each default is the measured-fastest
 * form; every variant gives the documented bits), inject failures for the safety-net tests,
 * occupy CUs for the co-residency tests, or enable timing experiments whose outputs are not
 * valid.  Conventions as in autovc_hip.h: int status, avc_last_error() after a failure; toggles are
 * process-wide and take effect at the next call (captured forward graphs are re-captured).
 * Round 6 removed the hand-off variants measured and rejected in rounds 3-5 (granules, batch
 * halves, sentinel h, per-chunk waits, XCD-local lstm1 groups, 8-B h stores).
 */
#ifndef AUTOVC_HIP_DEBUG_H_
#define AUTOVC_HIP_DEBUG_H_

#include "autovc_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

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
 * multiplied (1 or 2 = default); same arithmetic either way. */
int avc_lstm_persist_depth(int chunks);
/* Tuning hook: the persistent recurrences' per-step waits.  Bit set = every wave waits for the
 * quarter of the producing slot whose h it multiplies (quarter counters, no workgroup barrier);
 * clear = one polling lane per operand and a workgroup barrier.  Bit 0: two-layer form (lstm2),
 * bit 1: one-layer form (lstm1); default 1.  Same arithmetic either way (bit-identical). */
int avc_lstm_persist_qwait(int mask);
/* Test hook: workgroups of XCD-local BPTT launches (avc_bptt_xcd) that found their group on one
 * XCD / not, since the last call (two words, then cleared). */
int avc_debug_xl_census(unsigned* local_nonlocal);
/* Test hook: 1 = the XCD-local BPTT (avc_bptt_xcd) treats every group as not
 * local and runs its fallback (write-through stores, counters) -- the path a box whose workgroup
 * deal differs takes.  Same bits. */
int avc_debug_xl_force_remote(int on);
/* Tuning hook (round 5): 1 (default) = long-K products (weight gradients) pick their split-K count
 * by rounds of one workgroup per CU (a grid that spills a few workgroups into an extra round pays
 * the whole round); 0 = ~4 workgroups per CU (round 4).  The sums split differently: not
 * bit-identical, same accuracy. */
int avc_gemm_plan_rounds(int on);
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
/* Tuning hook: 1 (default) = avc_wavernn_generate runs the whole sample loop as ONE persistent launch of
 * rnn_dims / 2 workgroups with in-launch hand-offs where eligible
 * (avc_wavernn_persist_eligible: <= 96 fold rows, 2 * ceil(fc_dims / 8) + rows <= rnn_dims / 2,
 * every workgroup resident); 0 = five graph-captured launches per sample step.  Same arithmetic,
 * bit-identical samples, logits and waveform.  A loop launch that abandons a bounded wait (its
 * workgroups could not all be resident, e.g. CUs held by another process) is re-run by the same
 * call on the per-step graph path from a fresh state (same bits); avc_wavernn_fallbacks() counts
 * such re-runs. */
int avc_wavernn_persist(int on);
/* Tuning hook: 1 (default) = generate()'s input projection of every sample position (pI) as an
 * LDS-tiled kernel; 0 = one thread per output.  Same bits. */
int avc_wavernn_proj_tiled(int on);
/* Test hook: the next `launches` loop launches give up at their first unmet wait. */
int avc_debug_wavernn_inject(int launches);
/* Diagnostics: the next avc_wavernn_generate call (if its loop runs as one launch) stamps its first
 * `steps` steps (s_memrealtime, 100 MHz) into buf [rnn_dims / 2][steps][24] (u64; per op of the
 * loop: start, wait done, end).  That call consumes the request whichever path it takes. */
int avc_debug_wavernn_stamps(void* buf, int steps);

/* (The diagnostic stamps build, `make stamps` = -DAVC_STAMPS, also exports avc_debug_persist_diag
 * -- timing experiment bits of the persistent forward recurrences: 1 skips the gx1 loads, 4 the h
 * loads, 8 the second half of each wave's h chunks -- and avc_debug_stamps_persist, the stamp
 * buffer [3 slots][ncb][T][8] u64; the shipped library has neither.) */

#ifdef __cplusplus
}
#endif

#endif /* AUTOVC_HIP_DEBUG_H_ */
