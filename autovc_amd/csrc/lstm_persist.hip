// Weight-stationary two-layer LSTM recurrence (decoder.lstm2, decoder.py:53,74) as ONE launch.
//
// Why: the launch-per-step three-slot wavefront (lstm_split.hip) streams all 48 MB of split
// weights (W_hh0, W_ih1, W_hh1 as hi/lo f16) from the Infinity Cache in EVERY time step: 192
// workgroups x (256 KB of weights + 256 KB of h) per step is both the per-CU intake limit
// (~80 GB/s per CU) and the chip's Infinity-Cache rate (~8.6 TB/s; MI355X_MICROARCH.md), which is
// why a step costs ~15 us.  Here every workgroup loads its 64 gate rows (256 KB split) ONCE into
// registers (three 16-row tiles) and LDS (the fourth), and per time step only the 256 KB split h
// operand moves — read from the XCD's L2, which all of the XCD's CUs share.
//
// Structure: grid = 3 slots x ncb workgroups, one per CU (LDS use forces one workgroup per CU;
// 3*ncb <= CUs is checked on the host, so every workgroup is resident and the waits below always
// make progress).  Slot L's workgroup cb owns permuted gate rows [64cb, 64cb+64) of
//   slot 0: W_hh0  (layer 0's recurrence, h0_t = cell(h0_{t-1} W_hh0^T + gx0_t)),
//   slot 1: W_ih1  (layer 1's input product gx1_t = h0_t W_ih1^T + b_ih1 + b_hh1),
//   slot 2: W_hh1  (layer 1's recurrence, h1_t = cell(h1_{t-1} W_hh1^T + gx1_t)),
// and walks t = 0..T-1 on its own.  Every hand-off writes a buffer of its own per time step
// (split h0_t / h1_t, gx1_t), so there is never a write-after-read hazard; the cell state c
// stays in registers (the epilogue thread of a (batch row, 4 hidden units) pair never changes).
//
// Dependencies (arrival counters per slot and time step; E = this launch's epoch, below):
//   slot 0 at t waits  cnt0[t-1] >= E*ncb         (all of h0_{t-1})  [replicated: see kRep]
//   slot 1 at t waits  cnt0[t]   >= E*ncb         (all of h0_t)
//   slot 2 at t waits  cnt1[t]   >= E*ncb and cnt2[t-1] >= E*ncb
// The counters are never reset: they live in a per-context region of their own (one per counter
// layout), every successful launch adds exactly ncb to every word, and each workgroup derives the
// launch's epoch E from a ticket it takes at start (E = ticket / grid size + 1).  A counter value
// left by an earlier launch is at most (E-1)*ncb, so it can never satisfy a wait of this launch:
// correctness does not depend on any reset being ordered before the waiters (the round-1 design
// zeroed the counters per call and was exposed to exactly that).
// Hand-off protocol (cdna_hip_programming.md Guideline 16, counter form with replicas): payload
// stored write-through (sc1; every 128-B line written whole by one wave instruction), every
// storing wave drains vmcnt, workgroup barrier, one 8-lane instruction adds to the 8 counter
// replicas (agent scope); the consumer polls one replica relaxed, workgroup barrier, then EVERY
// load of handed-off bytes is an sc1 load (default, mode 2: 9.8 us per step), or one agent-scope
// acquire followed by plain loads (mode 1: 11.4 us per step).
// Every spin is bounded: on timeout the workgroup raises the region's give-up word to E, every
// waiter of this launch sees it and leaves, the rows a workgroup did not compute are written as
// NaN (a timed-out launch can never return plausible numbers), and the first workgroup to give up
// stores the device's running failure count into the context's pinned host word.  The next call on the context that reaches a
// persistent recurrence (or avc_persist_check) sees it, drops the counter regions and the
// captured graph, and fails with AVC_ERR_DEVICE (a RuntimeError in Python).
// Co-residency of the grid (every wait assumes its producers run) is checked before launching:
// the occupancy API's resident workgroups per CU x CUs must cover the grid, else the
// launch-per-step kernels run instead; avc_lstm_persist_coop(1) launches cooperatively.
//
// One-layer form (decoder.lstm1, decoder.py:50,69): slot 0 alone, grid (ncb, ngrp).  Batch rows
// never interact in an LSTM, so the batch is split into ngrp independent groups of 16/32/64 rows
// (blockIdx.y), each with counters of its own: a workgroup then reads only its group's rows of
// split h per step (32 KB at 16 rows, H = 512) and waits on ncb peers, not ncb x ngrp.  C2 lstm1
// (B = 64, H = 512): 4 groups x 32 workgroups, 3.7 us per step against ~6.9 us per step launch.
//
// Arithmetic is identical to lstm_split_step_kernel's NC = 4 tiles: the same 3xf16 products
// (hi.lo, lo.hi, hi.hi per 32-deep chunk, in that order), the same K split over 4 waves and
// the same fixed-order LDS reduction, so the two paths agree bit for bit.
#include <fcntl.h>
#include <sys/file.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "kernels.h"
#include "persist_internal.h"
#include "timing.h"

namespace avc {

int g_persist_mode = 2;  // avc_lstm_persist_tune(): 0 = never; 1 / 2 = when eligible (hand-off form)
int g_persist_layers = 3;  // avc_lstm_persist_layers(): bit 0 = one-layer form, bit 1 = two-layer form
int g_persist_pd = 2;    // avc_lstm_persist_depth(): h chunks in flight ahead of the MFMAs (1 or 2)

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr float kHScale = 32768.0f;   // split h is stored as h * 2^15 (lstm_split.hip)
// Arrival counters are kept in kRep replicas, each on a 128-B line of its own: a producer adds to
// every replica with one 8-lane wave instruction, a consumer polls the replica of its own
// blockIdx % 8 (the XCD under round-robin placement: speed only, any replica is complete once all
// adds landed).  One shared counter had 128 pollers and 64 adders on one line.
constexpr int kRep = 8, kLine = 32;  // replicas; unsigned words per 128-B line
__host__ __device__ __forceinline__ long cnt_index(int L, int T, int t, int r) {
  return (((long)L * T + t) * kRep + r) * kLine;
}
// Quarter counters (round 3, `avc_lstm_persist_qwait`): wave w of a consumer multiplies the K
// chunks [w*NCH, (w+1)*NCH) of h, i.e. hidden units [w*H/4, (w+1)*H/4), which exactly the
// workgroups [w*ncb/4, (w+1)*ncb/4) of the producing slot write.  Every producer also counts itself
// in on the counter of its quarter (after the nslot*T full lines), so each wave waits for its own
// 16 producers instead of the whole slot behind one workgroup barrier.
constexpr int kQuarters = 4;
__host__ __device__ __forceinline__ long qcnt_index(int nslot, int L, int T, int t, int q, int r) {
  return (long)nslot * T * kRep * kLine + ((((long)L * T + t) * kQuarters + q) * kRep + r) * kLine;
}
// counter words of one group: the full lines, and with quarter counters four more per (slot, step)
__host__ __device__ __forceinline__ long cnt_words(int nslot, int T, bool quarters) {
  return (long)nslot * T * kRep * kLine * (quarters ? 1 + kQuarters : 1);
}
// gx1 hand-off: a ring of kGxRing steps of per-column-block slabs [64 rows][64 columns] fp32, so
// each (step, column block) pair exchanges one contiguous 16 KB; slot 1 re-fills a ring entry
// only after every slot-2 workgroup has finished the step that read it (back-pressure wait)
constexpr int kGxRing = 4;
constexpr int kLead = 3;  // slot 0 may run at most this many steps ahead of slot 2



#ifdef AVC_STAMPS
// diagnostic build only: s_memtime per (workgroup, step, phase), written by thread 0
__device__ unsigned long long* g_pstamps = nullptr;
#define AVC_PSTAMP(slot)                                                                          \
  do {                                                                                            \
    unsigned long long _t;                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (g_pstamps && tid == 0) g_pstamps[((long)blockIdx.x * T + t) * 8 + (slot)] = _t;           \
  } while (0)
// s_memrealtime (constant clock shared by all XCDs) for cross-workgroup comparisons
#define AVC_PRSTAMP(slot)                                                                         \
  do {                                                                                            \
    unsigned long long _t;                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (g_pstamps && tid == 0) g_pstamps[((long)blockIdx.x * T + t) * 8 + (slot)] = _t;           \
  } while (0)
#else
#define AVC_PSTAMP(slot) do { } while (0)
#define AVC_PRSTAMP(slot) do { } while (0)
#endif

struct PersistArgs {
  int B, T, H, ncb, ntile;
  int nslot;                  // 3 = two-layer wavefront (lstm2), 4 = the same + slot 3 (input projection);
                              // 1 = one layer (slot 0 only: lstm1)
  long cnt_gstride;           // counter words per batch group (blockIdx.y; one-layer form only)
  const unsigned char* W[4];  // split fragment-major weights, permuted gate rows
  const float* winv[4];       // per-row unscale
  const float* gx0;           // [T][B][4H] layer-0 input projection + biases (permuted); written
                              // by slot 3 inside the launch when nslot == 4
  // input slot (in_slot > 0: layer 0's input projection inside the launch, on CUs the recurrence
  // leaves idle): gx0_t = x_t W_ih0^T + b_ih0 + b_hh0 from the split x (split_steps16_kernel) and
  // the split W_ih0 (split_rows_kernel layout, K = din)
  const unsigned char* xs;    // [T][hszx] split x_t (fragment-major, 2 KiB per 16-row x 32-k block)
  long hszx;                  // bytes per time step of xs
  int din;                    // K of the input projection, padded to 128 * NCH3 (3 or 4) with zeros
  int in_slot;                // slot index of the input projection (3: lstm2, 1: lstm1), 0 = none
  int in_lead;                // input slot back-pressure: 1 = none (default: measured fastest),
                              // 2 = at most kLead3 steps ahead checked every 4th step, 3 = every step
  const float* b0;            // [4H] b_ih0 + b_hh0 (permuted)
  const unsigned* x_amax;     // optional max |x| (float bits): x was split scaled by its power of two
  const float* b1;            // [4H] b_ih1 + b_hh1 (permuted)
  float* gx1;                 // [kGxRing][ncb][64][64] slabs (see gx1_slab)
  unsigned char* hs0;         // [T][hsz] split h0_t (fragment-major, 2 KiB per 16-row x 32-k block)
  unsigned char* hs1;         // [2][hsz] ring (only slot 2 reads it, one step later)
  long hsz;                   // bytes per time step of a split-h buffer
  float* y0; float* y1;       // [T][B][H] fp32 h
  _Float16* yfrag;            // optional: slot yf_slot's h_t also as the split image the next
  int yf_slot, yf_nkc;        // contraction streams (GemmDesc::a_frag, rows t*B + b, nkc chunks)
  float* g0; float* g1;       // optional [T][B][4H] activated gates (training)
  float* c0; float* c1;       // optional [T][B][H] cell state (training)
  unsigned* cnt;              // [nslot][T] arrivals (never reset; see the epoch above)
  unsigned* tmo;              // give-up word: epoch of the last launch that gave up
  unsigned long long* tickets;  // one per workgroup per launch
  unsigned* fail_host;        // pinned host word (avc_context::fail_host): last failure number
  int nwg;                    // workgroups in the grid
  unsigned spin_limit;        // polls before giving up (0 = test injection: give up at once)
  int diag;                   // diagnostic build only (avc_debug_persist_diag): timing experiments
};
int g_persist_diag = 0;
// avc_lstm_persist_qwait(): per-wave waits on quarter counters, bit 0 = two-layer form (lstm2:
// 1141 -> 1073 us at C2), bit 1 = one-layer form (lstm1: 384 -> 400 us at C2, so off)
int g_persist_qwait = 1;

__device__ bool spin_give_up(unsigned spins, const PersistArgs& a, unsigned E, int lane) {
  return spin_give_up_ctl(spins, a.tmo, a.fail_host, a.spin_limit, E, lane);
}

__device__ __forceinline__ bool wait_ge(unsigned* p, unsigned target, const PersistArgs& a, unsigned E) {
  return wait_ge_ctl(p, target, a.tmo, a.fail_host, a.spin_limit, E);
}

// One lane waits until *p_i >= t_i for every enabled i (e_i): each poll loads all of them back to
// back (one round trip for the lot), then compares; bounded and giving up like wait_ge_ctl.
__device__ bool wait3(unsigned* p0, unsigned t0, bool e0, unsigned* p1, unsigned t1, bool e1, unsigned* p2,
                      unsigned t2, bool e2, const PersistArgs& a, unsigned E, unsigned* p3 = nullptr,
                      unsigned t3 = 0, bool e3 = false) {
  if (!e0 && !e1 && !e2 && !e3) return true;
  gu32* gt = (gu32*)(a.tmo);
  for (unsigned spins = 0;; ++spins) {
    const unsigned v0 = e0 ? __hip_atomic_load((gu32*)p0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const unsigned v1 = e1 ? __hip_atomic_load((gu32*)p1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const unsigned v2 = e2 ? __hip_atomic_load((gu32*)p2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    const unsigned v3 = e3 ? __hip_atomic_load((gu32*)p3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    if ((!e0 || (int)(v0 - t0) >= 0) && (!e1 || (int)(v1 - t1) >= 0) && (!e2 || (int)(v2 - t2) >= 0) &&
        (!e3 || (int)(v3 - t3) >= 0))
      return true;
    if ((spins & 63) == 63 && __hip_atomic_load(gt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == E)
      return false;
    if (spins >= a.spin_limit) {
      const unsigned old = __hip_atomic_fetch_max(gt, E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old != E) {
        const unsigned nf = atomicAdd(&g_persist_giveups, 1u) + 1u;
        if (a.fail_host)
          __hip_atomic_store(a.fail_host, nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// power of two the x split was scaled by (split_steps16_kernel): max |x| -> [2^14, 2^15)
__device__ __forceinline__ float x_split_scale(const unsigned* amax) {
  if (!amax) return 1.f;
  const float m = __uint_as_float(*amax);
  if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
  int e;
  (void)frexpf(m, &e);
  return ldexpf(1.f, 15 - e);
}

constexpr int kLead3 = 12;  // with back-pressure (in_lead 2 / 3) the input slot runs at most this many
                            // steps ahead of slot 0 (> 3: see slot 0's every-4th-step wait)

// Slot 3 of the two-layer launch: layer 0's input projection, one time step per iteration, on the
// 64 CUs the three recurrence slots leave idle (it replaces a separate 8192 x 4096 x 512 GEMM that
// ran before the recurrence).  Workgroup cb owns the same 64 permuted gate rows as slot 0's cb and
// keeps them in registers (W_ih0 rows, K = din = 512: 4 gate tiles x 4 chunks per wave); per
// step it reads the split x_t (plain loads: x was written before the launch), forms
// x_hi.W_hi + x_hi.W_lo and, in a second accumulator, x_lo.W_hi (x_lo carries 2^11, as
// bn_apply_frag's split), reduces the 4 waves' K quarters in a fixed order and stores
// gx0_t = sum * unscale + b0 with whole-line write-through stores, then counts itself in on
// cnt[3][t].  Slot 0 waits for that counter and reads gx0_t with sc1 loads (the gx1 hand-off form).
template <int RT, int NCH3>
__device__ void input_slot(const PersistArgs& a, unsigned* cnt, int grp, float* part, int* flag, unsigned E,
                           unsigned target, int cb) {
  constexpr int NW = 4, NC = 4, MB = 16 * RT, TW = 16 * NC, RP = TW + 4;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lq = lane >> 4;
  const int B = a.B, T = a.T;
  const int nck3 = 4 * NCH3;  // a.din == 128 * NCH3
  const long G4 = 4L * a.H;
  const int rep = blockIdx.x & (kRep - 1);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(a.W[a.in_slot]) + (long)cb * NC * nck3 * 2048, 0, NC * nck3 * 2048, 0x00020000);
  const int kc0 = w * NCH3;
  f16x8 wr[NC][NCH3][2];
#pragma unroll
  for (int n = 0; n < NC; ++n)
#pragma unroll
    for (int c = 0; c < NCH3; ++c)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl)
        wr[n][c][hl] = __builtin_bit_cast(
            f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, (n * nck3 + kc0 + c) * 2048 + hl * 1024, 0));
  // store lanes: 4 consecutive gate columns 4*pc.. of the block for one batch row
  const int pc = lane & 15;
  const int p0 = cb * TW;
  const float xun = 32768.f / x_split_scale(a.x_amax);  // W rows carry 2^15 more than winv undoes for h
  f32x4 wiv, b0v;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    wiv[e] = a.winv[a.in_slot][p0 + 4 * pc + e] * xun;
    b0v[e] = a.b0[p0 + 4 * pc + e];
  }
  // this workgroup's batch rows: [grp * MB, grp * MB + MB) (one-layer form: its batch group)
  const int tile0 = grp * RT;
  const int ntile = a.ntile - tile0;
  for (int t = 0; t < T; ++t) {
    // back-pressure: at most kLead3 steps ahead of slot 0
    if (tid == 0) {
      const bool check = t >= kLead3 && (a.in_lead == 3 || (a.in_lead == 2 && (t & 3) == 0));
      const bool ok = !check || wait_ge(cnt + cnt_index(0, T, t - kLead3, rep), target, a, E);
      flag[0] = ok ? 1 : 0;
    }
    __syncthreads();
    if (flag[0] == 0) return;
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(a.xs) + (long)t * a.hszx + (long)tile0 * nck3 * 2048, 0, ntile * nck3 * 2048,
        0x00020000);
    f16x8 xv[NCH3][RT][2];
#pragma unroll
    for (int c = 0; c < NCH3; ++c)
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int hl = 0; hl < 2; ++hl)
          xv[c][r][hl] = __builtin_bit_cast(
              f16x8, __builtin_amdgcn_raw_buffer_load_b128(xrs, lane * 16, (r * nck3 + kc0 + c) * 2048 + hl * 1024, 0));
    f32x4 acc[RT][NC], accl[RT][NC];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int n = 0; n < NC; ++n) acc[r][n] = accl[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH3; ++c)
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int n = 0; n < NC; ++n) {
          accl[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xv[c][r][1], wr[n][c][0], accl[r][n], 0, 0, 0);
          acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xv[c][r][0], wr[n][c][1], acc[r][n], 0, 0, 0);
          acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xv[c][r][0], wr[n][c][0], acc[r][n], 0, 0, 0);
        }
    float* mine = part + w * MB * RP;
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int n = 0; n < NC; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          mine[(r * 16 + 4 * lq + e) * RP + n * 16 + l15] = acc[r][n][e] + accl[r][n][e] * (1.f / 2048.f);
    __syncthreads();
    const auto ors = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.gx0) + (long)t * B * G4, 0,
                                                       (int)(B * G4 * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = w * 16 + i * 4 + (lane >> 4);
      if (r < MB && tile0 * 16 + r < B) {
        const int off = r * RP + 4 * pc;
        f32x4 v = *reinterpret_cast<const f32x4*>(part + off);
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) v += *reinterpret_cast<const f32x4*>(part + ww * MB * RP + off);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v * wiv + b0v), ors,
                                               (int)(((tile0 * 16 + r) * G4 + p0 + 4 * pc) * 4), 0, 16 /*sc1*/);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < kRep)
      __hip_atomic_fetch_add((gu32*)(cnt + cnt_index(a.in_slot, T, t, tid)), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
}

// HO = hand-off form on the consumer side: 0 = one agent-scope acquire (L1 invalidate) then plain
// loads; 1 = no invalidate, EVERY load of handed-off bytes (split h, gx1) an sc1 load
// (cdna_hip_programming.md Guideline 16, "Valid forms": producer stores sc1 + drained).
// PD = h chunks loaded ahead of the chunk being multiplied (register buffers PD + 1).
// QW = 1: per-wave waits on quarter counters (see qcnt_index) instead of three polling lanes and a
// workgroup barrier at the top of every step.
// (Round 6: the hand-off variants measured and rejected in rounds 3-5 -- granules, batch halves,
// sentinel h, per-chunk waits, XCD-local lstm1 groups -- are no longer compiled)
template <int NCH, int RT, int HO, int PD, int QW>
__global__ __launch_bounds__(256, 1) void lstm_persist_kernel(PersistArgs a) {
  constexpr int NW = 4, NC = 4;
  constexpr int MB = 16 * RT;        // batch rows computed (B <= MB)
  constexpr int TW = 16 * NC;        // 64 gate rows
  constexpr int RP = TW + 4;
  constexpr int NPAIR = MB * NC;     // (row, 16-column block) epilogue pairs, <= 256
  // LDS: gate tile 3's weights for every wave (NW x NCH x 2 KiB), then the reduction partials
  extern __shared__ float lds[];
  unsigned char* wl = reinterpret_cast<unsigned char*>(lds);
  float* part = lds + NW * NCH * 512;
  // [8]: polling lanes' results (0, 1, 3), epoch (2); QW: each wave's wait result (4 + w)
  int* flag = reinterpret_cast<int*>(part + NW * MB * RP);
  // [TW] per-row unscale of this block's gate rows, then [TW] b_ih1 + b_hh1 (slot 1): read from
  // LDS in the epilogue instead of living in registers through the MFMA loop
  float* cpar = reinterpret_cast<float*>(flag + 8);
  // [MB][16] the unscaled split of this workgroup's h for the y_frag image (whole fragment rows)
  unsigned* yst = reinterpret_cast<unsigned*>(cpar + 2 * 64);

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lq = lane >> 4;
  // batch group: rows [grp * MB, grp * MB + MB).  LSTM batch rows never interact, so in the
  // one-layer form every group is an independent recurrence with counters of its own.
  const int L = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - L * a.ncb;
  const int grp = blockIdx.y;
  const int B = a.B, H = a.H, T = a.T;
  unsigned* const cnt = a.cnt + (long)grp * a.cnt_gstride;
  const int nck = H >> 5;            // 32-deep chunks per row
  const long G4 = 4L * H;

  // this launch's epoch (see the header): every workgroup takes one ticket
  if (tid == 0) {
    const unsigned long long tk = __hip_atomic_fetch_add(a.tickets, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[2] = (int)(unsigned)(tk / (unsigned long long)a.nwg + 1ull);
  }
  __syncthreads();
  const unsigned E = (unsigned)flag[2];
  const unsigned target = E * (unsigned)a.ncb;

  if (a.in_slot > 0 && L == a.in_slot) {  // layer 0's input projection
    if (a.din == 512) input_slot<RT, 4>(a, cnt, grp, part, flag, E, target, cb);
    else input_slot<RT, 3>(a, cnt, grp, part, flag, E, target, cb);
    return;
  }

  // ---- stationary weights: wave w owns K chunks [w*NCH, (w+1)*NCH) of the 4 gate tiles ----
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(a.W[L]) + (long)cb * NC * nck * 2048, 0, NC * nck * 2048, 0x00020000);
  const int kc0 = w * NCH;
  f16x8 wreg[3][NCH][2];
#pragma unroll
  for (int n = 0; n < 3; ++n)
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int hl = 0; hl < 2; ++hl)
        wreg[n][c][hl] = __builtin_bit_cast(
            f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, (n * nck + kc0 + c) * 2048 + hl * 1024, 0));
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int hl = 0; hl < 2; ++hl) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, (3 * nck + kc0 + c) * 2048 + hl * 1024, 0);
      *reinterpret_cast<u32x4*>(wl + ((w * NCH + c) * 2 + hl) * 1024 + lane * 16) = v;
    }

  // ---- epilogue ownership: every thread owns UPT = RT hidden units of one (row, 16-column
  // block) pair: tid -> pair tid / SUB, units u0 .. u0 + UPT - 1 of the block's 4 (the gate
  // math of a step is spread over all 256 threads whatever the batch tile)
  constexpr int UPT = RT, SUB = 4 / UPT;
  static_assert(NPAIR * SUB == 256, "one epilogue slot per thread");
  const int pair = tid / SUB, sub = tid % SUB, u0 = sub * UPT;
  const int row = pair / NC, blk = pair % NC;
  const int b = grp * MB + row;            // this thread's batch row
  const bool live = b < B;
  const int bc = min(b, B - 1);
  const int p0 = cb * TW + blk * 16;       // first permuted gate column of the pair
  const int j0 = cb * 4 * NC + blk * 4;    // first hidden unit of the pair
  typedef float fu __attribute__((ext_vector_type(UPT)));
  if (tid < TW) {  // published to the epilogue by the first step's barriers
    cpar[tid] = a.winv[L][cb * TW + tid];
    if (L == 1) cpar[TW + tid] = a.b1[cb * TW + tid];
  }
  fu cst = fu{};  // cell state
  // slot 1 stores gx1 in whole lines: lane -> (row 4i + lane/16 of the wave's 16, columns 4*pc..)
  const int pc = lane & 15;
  float* c_save = L == 0 ? a.c0 : a.c1;
  float* g_save = L == 0 ? a.g0 : a.g1;
  float* y_out = L == 0 ? a.y0 : a.y1;
  auto gx1_slab = [&](int tt, int c) -> long { return ((long)(tt % kGxRing) * a.ncb + c) * (64 * TW); };
  const int rep = blockIdx.x & (kRep - 1);
  // outputs nobody reads inside this launch: h, and for training c and the activated gates
  _Float16* const yfrag = L == a.yf_slot ? a.yfrag : nullptr;
  // frag: also this thread's units of y_frag (the give-up NaN fill; normally yfrag_rows writes it)
  auto store_out = [&](int tt, const fu& h, const fu& c, const fu& i, const fu& f, const fu& g, const fu& o,
                       bool frag = false) {
    if (y_out) *reinterpret_cast<fu*>(y_out + ((long)tt * B + b) * H + j0 + u0) = h;
    if (yfrag && frag) {  // split_frag32_kernel's unscaled split (|h| < 1), at its fragment position
      const long r = (long)tt * B + b;
      const int k = j0 + u0;
      const long blk = ((r >> 5) * a.yf_nkc + (k >> 4)) * 2;
      const long off = blk * 512 + ((r & 31) + 32 * ((k >> 3) & 1)) * 8 + (k & 7);
      typedef _Float16 hu __attribute__((ext_vector_type(UPT)));
      hu hi, lo;
#pragma unroll
      for (int u = 0; u < UPT; ++u) {
        const _Float16 hh = (_Float16)h[u];
        hi[u] = hh;
        lo[u] = (_Float16)((h[u] - (float)hh) * 2048.0f);
      }
      *reinterpret_cast<hu*>(yfrag + off) = hi;
      *reinterpret_cast<hu*>(yfrag + off + 512) = lo;
    }
    if (c_save) *reinterpret_cast<fu*>(c_save + ((long)tt * B + b) * H + j0 + u0) = c;
    if (g_save) {
      float* go = g_save + ((long)tt * B + b) * G4 + p0 + u0;
      *reinterpret_cast<fu*>(go) = i;
      *reinterpret_cast<fu*>(go + 4) = f;
      *reinterpret_cast<fu*>(go + 8) = g;
      *reinterpret_cast<fu*>(go + 12) = o;
    }
  };
  // y_frag as whole fragment rows (round 4): the MB rows staged in yst (batch rows rb0 ..) of step
  // tt go out as 16-B pieces, 32 consecutive fragment lanes of one (hi / lo, k half) per 512 B.
  // This workgroup's 16 units are exactly the 16-k chunk cb of the image.  (Per-thread stores of
  // 2-8 B pieces left partly written lines on several XCDs; every thread takes part here.)
  auto yfrag_rows = [&](int tt, int rb0) {
    for (int p = tid; p < MB * 4; p += 256) {
      const int r = p % MB, kh = (p / MB) & 1, hl2 = p / (2 * MB);
      const int bb = rb0 + r;
      if (bb >= B) continue;
      const long rr = (long)tt * B + bb;
      const long blk2 = ((rr >> 5) * a.yf_nkc + cb) * 2 + hl2;
      const u32x4 q0 = *reinterpret_cast<const u32x4*>(yst + r * 16 + kh * 8);
      const u32x4 q1 = *reinterpret_cast<const u32x4*>(yst + r * 16 + kh * 8 + 4);
      auto half = [&](unsigned q) { return hl2 ? q >> 16 : q & 0xffffu; };
      const u32x4 v = {half(q0[0]) | (half(q0[1]) << 16), half(q0[2]) | (half(q0[3]) << 16),
                       half(q1[0]) | (half(q1[1]) << 16), half(q1[2]) | (half(q1[3]) << 16)};
      *reinterpret_cast<u32x4*>(yfrag + blk2 * 512 + ((rr & 31) + 32 * kh) * 8) = v;
    }
  };

  int t = 0;
  for (; t < T; ++t) {
    // ---- wait for this step's operands ----------------------------------------------------
    AVC_PSTAMP(0);
    if constexpr (QW) {
      // Lane 0 of every wave waits for what THIS wave reads, all in one multi-counter poll: the
      // quarter of the h source its K chunks come from; slot 2: the slot-1 quarter that wrote its
      // gx1 slab (the one of workgroup cb); slot 0 with the input slot, every 4th step: gx0 for 4
      // steps (as below).  Wave 1 also takes the back-pressure wait; it gates nothing but the
      // stores after the reduction barrier (slot 1's gx1 ring entry), which every wave passes after
      // wave 1's wait.  No workgroup barrier: each wave starts its loads as soon as its own
      // producers are in.  A failed wait is acted on after the reduction barrier (all waves leave).
      if (lane == 0) {
        const unsigned qtarget = E * (unsigned)(a.ncb / kQuarters);
        const int hsl = L == 1 ? 0 : L;      // slot whose h this slot reads (0: h0, 2: h1)
        const int ht = L == 1 ? t : t - 1;   // and its step
        // 0: the h quarter; 1: the gx operand; 2: back-pressure (wave 1)
        const bool e0 = ht >= 0;
        unsigned* p0 = cnt + qcnt_index(a.nslot, hsl, T, e0 ? ht : 0, w, rep);
        const bool e1 = L == 2 || (L == 0 && a.in_slot > 0 && (t & 3) == 0);
        unsigned* p1 = L == 2 ? cnt + qcnt_index(a.nslot, 1, T, t, cb / (a.ncb / kQuarters), rep)
                              : cnt + cnt_index(a.in_slot, T, min(t + 3, T - 1), rep);
        const unsigned t1 = L == 2 ? qtarget : target;
        const bool e2 = w == 1 && ((L == 0 && t >= kLead && a.nslot >= 3) || (L == 1 && t >= kGxRing));
        unsigned* p2 = cnt + cnt_index(2, T, e2 ? t - (L == 0 ? kLead : kGxRing) : 0, rep);
        flag[4 + w] = wait3(p0, qtarget, e0, p1, t1, e1, p2, target, e2, a, E) ? 1 : 0;
      }
      // the polled values are in (the loop compared them); nothing below moves above this point
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      AVC_PSTAMP(1);
      AVC_PRSTAMP(7);
      AVC_PSTAMP(2);
    } else {
    // Two lanes poll in parallel (lane 0 of waves 0 and 1): the data this step reads, and the
    // back-pressure that keeps slots 0 and 1 at most kLead / kGxRing steps ahead of slot 2 (a
    // slot running far ahead streams gx0 / writes h0 through the Infinity Cache and starves the
    // others: measured as a bistable 10 vs 20 us per step).  Each polling lane then acquires.
    // With slot 3 (nslot == 4) a third lane (wave 2) waits for this step's gx0.
    if (tid == 0 || tid == 64 || tid == 128) {
      const bool primary = tid == 0;
      long idx = -1;
      // the input slot runs ahead (up to kLead3 steps), so its progress is checked every 4th step
      // for 4 steps at once: its workgroups finish steps in order, so all of them counting in on
      // step t + 3 implies steps t .. t + 2 are complete (and drained) as well
      if (tid == 128) idx = L == 0 && a.in_slot > 0 && (t & 3) == 0 ? cnt_index(a.in_slot, T, min(t + 3, T - 1), rep) : -1;
      else if (L == 0) idx = primary ? (t > 0 ? cnt_index(0, T, t - 1, rep) : -1)
                                     : (t >= kLead && a.nslot >= 3 ? cnt_index(2, T, t - kLead, rep) : -1);
      else if (L == 1) idx = primary ? cnt_index(0, T, t, rep)
                                     : (t >= kGxRing ? cnt_index(2, T, t - kGxRing, rep) : -1);
      else idx = primary ? (t > 0 ? cnt_index(2, T, t - 1, rep) : -1) : cnt_index(1, T, t, rep);
      const bool ok = idx < 0 || wait_ge(cnt + idx, target, a, E);
      if (primary) {
        AVC_PSTAMP(1);
        AVC_PRSTAMP(7);
      }
      if constexpr (HO == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
      }
      flag[tid == 128 ? 3 : (primary ? 0 : 1)] = ok ? 1 : 0;
    }
    __syncthreads();
    if (flag[0] == 0 || flag[1] == 0 || flag[3] == 0) break;
    AVC_PSTAMP(2);
    }

    // ---- recurrent / input product over this wave's K quarter ----------------------------
    // The epilogue operands (gx0 / b1 / the gx1 hand-off) are loaded right after the LAST h
    // chunk's loads: vmcnt retires in issue order, so loads issued ahead of the h chunks would
    // hold every MFMA until they land.
    fu gxv[4];
    const float* gxr = L == 0 ? a.gx0 + ((long)t * B + bc) * G4 + p0 + u0 : a.b1 + p0 + u0;
    auto load_gx = [&]() {
#ifdef AVC_STAMPS
      if ((a.diag & 1) && L == 2) {  // timing experiment: skip the gx1 hand-off loads
#pragma unroll
        for (int g = 0; g < 4; ++g) gxv[g] = fu{};
        return;
      }
#endif
      if (L == 2) {
        // descriptor base uniform (the slab), lane offset in the VGPR: a per-lane base would make
        // hipcc wrap each load in a waterfall loop over the 64 distinct descriptors (~10 us/step)
        const auto grs = __builtin_amdgcn_make_buffer_rsrc(a.gx1 + gx1_slab(t, cb), 0, 64 * TW * 4, 0x00020000);
        const int vo = (bc * TW + blk * 16 + u0) * 4;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if constexpr (UPT == 4) {
            gxv[g] = __builtin_bit_cast(fu, __builtin_amdgcn_raw_buffer_load_b128(grs, vo + 16 * g, 0, HO ? 16 : 0));
          } else {  // 4-B sc1 loads (an 8-B sc1 load is not a validated hand-off form)
#pragma unroll
            for (int uu = 0; uu < UPT; ++uu)
              gxv[g][uu] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, vo + 16 * g + 4 * uu, 0, HO ? 16 : 0));
          }
        }
      } else if (L == 0 && a.in_slot > 0) {
        // gx0_t handed off by slot 3 inside this launch: the same load form as gx1's
        const auto grs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.gx0) + (long)t * B * G4, 0,
                                                           (int)(B * G4 * 4), 0x00020000);
        const int vo = (int)((bc * G4 + p0 + u0) * 4);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if constexpr (UPT == 4) {
            gxv[g] = __builtin_bit_cast(fu, __builtin_amdgcn_raw_buffer_load_b128(grs, vo + 16 * g, 0, HO ? 16 : 0));
          } else {
#pragma unroll
            for (int uu = 0; uu < UPT; ++uu)
              gxv[g][uu] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(grs, vo + 16 * g + 4 * uu, 0, HO ? 16 : 0));
          }
        }
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) gxv[g] = *reinterpret_cast<const fu*>(gxr + 4 * g);
      }
    };
    f32x4 acc[RT][NC];
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int n = 0; n < NC; ++n) acc[r][n] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned char* src =
        L == 0 ? (t > 0 ? a.hs0 + (long)(t - 1) * a.hsz : nullptr)
               : (L == 1 ? a.hs0 + (long)t * a.hsz : (t > 0 ? a.hs1 + (long)((t - 1) & 1) * a.hsz : nullptr));
    if (src == nullptr) {
      load_gx();
    } else {
      const int hrow16 = nck * 2048;
      const long hbase = (long)grp * RT * hrow16 + (long)kc0 * 2048;
      const auto hrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(src) + hbase, 0,
                                                         (int)((long)a.ntile * nck * 2048 - hbase), 0x00020000);
      // h chunk buffers: PDX chunks in flight ahead of the MFMAs.  With one 16-row tile (the
      // one-layer form's batch groups) a chunk is only 8 VGPRs, so every chunk of the wave's K
      // quarter is requested at once: one load round trip per step instead of NCH / PD
      constexpr int PDX = RT == 1 ? NCH : PD;
      constexpr int NB = PDX + 1;
      f16x8 hb[NB][RT][2], wt[2];
#ifdef AVC_STAMPS
// timing experiments: diag 4 = no h loads (zeros); diag 8 = the second half of the wave's K chunks
// not loaded (the per-CU h intake of a K split over two workgroups, priced without its fan-in hop)
#define AVC_PLD_SKIP(C) ((a.diag & 4) || ((a.diag & 8) && (C) >= NCH / 2))
#else
#define AVC_PLD_SKIP(C) false
#endif
#define AVC_PLD(HV, C)                                                                             \
  if (AVC_PLD_SKIP(C)) { _Pragma("unroll") for (int r = 0; r < RT; ++r) HV[r][0] = HV[r][1] = f16x8{}; } else \
  _Pragma("unroll") for (int r = 0; r < RT; ++r) {                                                 \
    HV[r][0] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(hrs, lane * 16, r * hrow16 + (C) * 2048, HO ? 16 : 0)); \
    HV[r][1] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(hrs, lane * 16, r * hrow16 + (C) * 2048 + 1024, HO ? 16 : 0)); \
  }
#ifdef AVC_MFMA_PASSES
// experiment: the three products of a chunk in passes over all accumulators (each accumulator
// still sees hi.lo, lo.hi, hi.hi in that order, so bit-identical); measured slower on gfx950
// (mfma loop 10.3k -> 11.7k ticks/step), hence off by default
#define AVC_PMFMA(HV, C)                                                                           \
  wt[0] = *reinterpret_cast<const f16x8*>(wl + ((w * NCH + (C)) * 2 + 0) * 1024 + lane * 16);      \
  wt[1] = *reinterpret_cast<const f16x8*>(wl + ((w * NCH + (C)) * 2 + 1) * 1024 + lane * 16);      \
  _Pragma("unroll") for (int pass = 0; pass < 3; ++pass) {                                         \
    const int ha = pass == 0 ? 1 : 0, wb = pass == 1 ? 1 : 0;                                      \
    _Pragma("unroll") for (int r = 0; r < RT; ++r) {                                               \
      _Pragma("unroll") for (int n = 0; n < 3; ++n)                                                \
        acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][ha], wreg[n][C][wb], acc[r][n], 0, 0, 0); \
      acc[r][3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][ha], wt[wb], acc[r][3], 0, 0, 0);  \
    }                                                                                              \
  }
#else
#define AVC_PMFMA(HV, C)                                                                           \
  wt[0] = *reinterpret_cast<const f16x8*>(wl + ((w * NCH + (C)) * 2 + 0) * 1024 + lane * 16);      \
  wt[1] = *reinterpret_cast<const f16x8*>(wl + ((w * NCH + (C)) * 2 + 1) * 1024 + lane * 16);      \
  _Pragma("unroll") for (int r = 0; r < RT; ++r) {                                                 \
    _Pragma("unroll") for (int n = 0; n < 3; ++n) {                                                \
      acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][1], wreg[n][C][0], acc[r][n], 0, 0, 0); \
      acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][0], wreg[n][C][1], acc[r][n], 0, 0, 0); \
      acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][0], wreg[n][C][0], acc[r][n], 0, 0, 0); \
    }                                                                                              \
    acc[r][3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][1], wt[0], acc[r][3], 0, 0, 0);      \
    acc[r][3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][0], wt[1], acc[r][3], 0, 0, 0);      \
    acc[r][3] = __builtin_amdgcn_mfma_f32_16x16x32_f16(HV[r][0], wt[0], acc[r][3], 0, 0, 0);      \
  }
#endif
#pragma unroll
      for (int c = 0; c < PDX && c < NCH; ++c) { AVC_PLD(hb[c], c) }
      if constexpr (NCH <= PDX) load_gx();
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (c + PDX < NCH) {
          AVC_PLD(hb[(c + PDX) % NB], c + PDX)
          if (c + PDX == NCH - 1) load_gx();
        }
        __builtin_amdgcn_sched_barrier(0);
        AVC_PMFMA(hb[c % NB], c)
        __builtin_amdgcn_sched_barrier(0);
      }
#undef AVC_PMFMA
#undef AVC_PLD
#undef AVC_PLD_SKIP
    }

    AVC_PSTAMP(3);
    // ---- fixed-order cross-wave reduction (as lstm_split_step_kernel) --------------------
    float* mine = part + w * MB * RP;
#pragma unroll
    for (int r = 0; r < RT; ++r)
#pragma unroll
      for (int n = 0; n < NC; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e) mine[(r * 16 + 4 * lq + e) * RP + n * 16 + l15] = acc[r][n][e];
    __syncthreads();
    if constexpr (QW) {
      if (flag[4] == 0 || flag[5] == 0 || flag[6] == 0 || flag[7] == 0) break;
    }
    fu hv, ig, fg, gg, og;
    if (L == 1) {
      // projection slot: the same fixed-order sum, scale and bias per 4 columns, stored to this
      // (step, column block)'s contiguous 16 KB slab as whole 128-B lines (a wave instruction
      // writes 4 rows x 256 B; partial-line write-through stores took ~10 us per step to drain)
      AVC_PSTAMP(4);
      const auto ors = __builtin_amdgcn_make_buffer_rsrc(a.gx1 + gx1_slab(t, cb), 0, 64 * TW * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = w * 16 + i * 4 + (lane >> 4);
        if (r < MB && r < B) {
          const int off = r * RP + 4 * pc;
          f32x4 v = *reinterpret_cast<const f32x4*>(part + off);
#pragma unroll
          for (int ww = 1; ww < NW; ++ww) v += *reinterpret_cast<const f32x4*>(part + ww * MB * RP + off);
          const f32x4 wiv1 = *reinterpret_cast<const f32x4*>(cpar + 4 * pc);
          const f32x4 b1v = *reinterpret_cast<const f32x4*>(cpar + TW + 4 * pc);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v * wiv1 + b1v), ors,
                                                 (r * TW + 4 * pc) * 4, 0, 16 /*sc1*/);
        }
      }
    } else {
      fu sum[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int off = row * RP + blk * 16 + 4 * g + u0;
        fu v = *reinterpret_cast<const fu*>(part + off);
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) v += *reinterpret_cast<const fu*>(part + ww * MB * RP + off);
        sum[g] = v;
      }
      AVC_PSTAMP(4);
      // ---- gate epilogue; only the split h (the hand-off) is stored before publishing ------
      unsigned hl[UPT] = {};  // split h of this thread's units: f16 hi | f16 lo << 16
      if (live) {
        fu wiv[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) wiv[g] = *reinterpret_cast<const fu*>(cpar + blk * 16 + 4 * g + u0);
#pragma unroll
        for (int u = 0; u < UPT; ++u) {  // explicit fmas: the launch-per-step kernel forms the same values
          ig[u] = gate_sigmoid(fmaf(sum[0][u], wiv[0][u], gxv[0][u]));
          fg[u] = gate_sigmoid(fmaf(sum[1][u], wiv[1][u], gxv[1][u]));
          gg[u] = gate_tanh(fmaf(sum[2][u], wiv[2][u], gxv[2][u]));
          og[u] = gate_sigmoid(fmaf(sum[3][u], wiv[3][u], gxv[3][u]));
          cst[u] = fmaf(fg[u], cst[u], ig[u] * gg[u]);
          hv[u] = og[u] * gate_tanh(cst[u]);
          const float v = hv[u] * kHScale;
          const _Float16 hi = (_Float16)v;
          const _Float16 lo = (_Float16)(v - (float)hi);
          hl[u] = (unsigned)__builtin_bit_cast(unsigned short, hi) |
                  ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16);
          if (yfrag) {  // the unscaled split of the y_frag image (store_out's expressions)
            const _Float16 yh = (_Float16)hv[u];
            const _Float16 yl = (_Float16)((hv[u] - (float)yh) * 2048.0f);
            yst[row * 16 + blk * 4 + u0 + u] = (unsigned)__builtin_bit_cast(unsigned short, yh) |
                                               ((unsigned)__builtin_bit_cast(unsigned short, yl) << 16);
          }
        }
      }
      if (t + 1 < T || L == 0) {
        // the pair's 4 units go out as one 8-B hi and one 8-B lo piece (whole fragment rows) from
        // its first thread; the other SUB - 1 threads hand their units over by lane shuffles
        unsigned q[4];
#pragma unroll
        for (int u = 0; u < UPT; ++u) q[u] = hl[u];
#pragma unroll
        for (int k = 1; k < SUB; ++k)
#pragma unroll
          for (int u = 0; u < UPT; ++u) q[k * UPT + u] = __shfl_down(hl[u], k);
        const u32x2 hi2 = {(q[0] & 0xffffu) | (q[1] << 16), (q[2] & 0xffffu) | (q[3] << 16)};
        const u32x2 lo2 = {(q[0] >> 16) | (q[1] & 0xffff0000u), (q[2] >> 16) | (q[3] & 0xffff0000u)};
        // 16-B pieces (round 5): the pair leads of blocks 2m and 2m + 1 (lanes tid and tid ^ SUB,
        // same row) hold the two halves of one 8-k fragment piece; the even one stores the hi
        // piece, the odd one the lo piece (half the store instructions, each 16 B)
        const bool odd = (blk & 1) != 0;
        const unsigned x0 = __shfl_xor(odd ? hi2[0] : lo2[0], SUB), x1 = __shfl_xor(odd ? hi2[1] : lo2[1], SUB);
        if (live && sub == 0) {
          const long off = ((long)(b >> 4) * nck + (j0 >> 5)) * 2048 + (((b & 15) + 16 * ((j0 & 31) >> 3)) * 8 + (j0 & 7)) * 2;
          const u32x4 pc = odd ? u32x4{x0, x1, lo2[0], lo2[1]} : u32x4{hi2[0], hi2[1], x0, x1};
          const int off16 = (int)off + (odd ? 1024 - 8 : 0);  // the piece starts at the even lead's units
          unsigned char* const hb = L == 0 ? a.hs0 + (long)t * a.hsz : a.hs1 + (long)(t & 1) * a.hsz;
          const auto ors = __builtin_amdgcn_make_buffer_rsrc(hb, 0, (int)a.hsz, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(pc, ors, off16, 0, 16 /*sc1*/);
        }
      }
    }
    // ---- publish: every storing wave drains, barrier, the workgroup counts itself in ------
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    AVC_PSTAMP(5);
    AVC_PRSTAMP(6);
    // lanes 8..15 count in on this workgroup's quarter -- in both wait forms, so every launch adds
    // ncb / 4 to every quarter word and the epoch targets hold whichever form the next launch takes
    if (tid < 2 * kRep) {
      const long ci = tid < kRep ? cnt_index(L, T, t, tid)
                                 : qcnt_index(a.nslot, L, T, t, cb / (a.ncb / kQuarters), tid - kRep);
      __hip_atomic_fetch_add((gu32*)(cnt + ci), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // outputs nobody reads inside this launch: stored after publishing (off the hand-off path);
    // the publish barrier above orders every thread's yst writes before yfrag_rows reads them
    if (L != 1 && live) store_out(t, hv, cst, ig, fg, gg, og);
    if (yfrag) yfrag_rows(t, grp * MB);
  }
  // gave up at step t: the rows this workgroup owns for steps t..T-1 are written as NaN, so a
  // timed-out launch never hands plausible numbers downstream (the host reports it, see above) --
  // through every output, the split image included
  if (t < T && L != 1 && live) {
    fu nv;
#pragma unroll
    for (int u = 0; u < UPT; ++u) nv[u] = __builtin_nanf("");
    for (int tt = t; tt < T; ++tt) store_out(tt, nv, nv, nv, nv, nv, nv, true);
  }
}

// x [T*B][K] (row stride ldx, time-major rows t*B + b) -> per time step the fragment-major split
// slot 3 reads: 16-row x 32-k blocks of 2 KiB (hi, then lo), lane (b & 15) + 16 * ((k & 31) >> 3)
// holding k & 7 = 0..7, i.e. the layout split_rows_kernel gives the weights.  hi = f16(x s),
// lo = f16((x s - hi) 2^11) with s the power of two of *amax (1 without it); rows b >= B are zero.
__global__ __launch_bounds__(256) void split_steps16_kernel(const float* __restrict__ x, long ldx, int T, int B,
                                                            int K, int Kp, int ntile, long hszx,
                                                            unsigned char* __restrict__ dst,
                                                            const unsigned* __restrict__ amax) {
  const int nck = Kp >> 5;  // columns [K, Kp) are zeros (K % 8 == 0)
  const long total = (long)T * ntile * nck * 64;
  const float sc = x_split_scale(amax);
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int l = (int)(idx & 63);
    const long blk = idx >> 6;
    const int kc = (int)(blk % nck);
    const long rest = blk / nck;
    const int rt = (int)(rest % ntile);
    const long t = rest / ntile;
    const int b = rt * 16 + (l & 15), k0 = kc * 32 + 8 * (l >> 4);
    float o[8];
    if (b < B && k0 < K) {
      const float4* q = reinterpret_cast<const float4*>(x + (t * B + b) * ldx + k0);
      const float4 u = q[0], v = q[1];
      o[0] = u.x; o[1] = u.y; o[2] = u.z; o[3] = u.w; o[4] = v.x; o[5] = v.y; o[6] = v.z; o[7] = v.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = 0.f;
    }
    f16x8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = o[e] * sc;
      const _Float16 h = (_Float16)v;
      hi[e] = h;
      lo[e] = (_Float16)((v - (float)h) * 2048.0f);
    }
    unsigned char* d = dst + t * hszx + ((long)rt * nck + kc) * 2048 + l * 16;
    *reinterpret_cast<f16x8*>(d) = hi;
    *reinterpret_cast<f16x8*>(d + 1024) = lo;
  }
}

inline size_t al(size_t b) { return (b + 255) & ~size_t(255); }


int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return cus;
}

// One-layer form: the narrowest batch groups (16, 32 or 64 rows) whose workgroups all fit the
// chip side by side.  Every group is an independent recurrence over ncb workgroups, and per step
// each workgroup reads only its own group's rows of split h.
int lstm1_rows_per_group(int B, int H) {
  const int ntile = (B + 15) / 16, ncb = 4 * H / 64, cus = device_cus();
  for (int RT = 1; RT < 4; RT *= 2)
    if ((ntile + RT - 1) / RT * ncb <= cus) return RT;
  return 4;
}

size_t persist_lds(int H, int RT) {
  const int nch = H / 32 / 4;
  return (size_t)4 * nch * 2048 + (size_t)4 * 16 * RT * 68 * sizeof(float) + 32 + 2 * 64 * sizeof(float) +
         (size_t)16 * RT * 16 * sizeof(unsigned);  // yst
}


// The template instance a launch of (H, RT) runs under the current tuning.
const void* persist_fn(int H, int RT, bool two_layer = true) {
  const bool qw = (g_persist_qwait & (two_layer ? 1 : 2)) != 0;
  const int nch = H / 32 / 4;
#define AVC_PERSIST_FN(NCHV, RTV)                                                                 \
  return g_persist_mode == 1 ? (const void*)lstm_persist_kernel<NCHV, RTV, 0, 1, 0>               \
       : g_persist_pd == 1   ? (const void*)lstm_persist_kernel<NCHV, RTV, 1, 1, 0>               \
       : qw                  ? (const void*)lstm_persist_kernel<NCHV, RTV, 1, 2, 1>               \
                             : (const void*)lstm_persist_kernel<NCHV, RTV, 1, 2, 0>;
  if (nch == 8) {
    if (RT == 1) { AVC_PERSIST_FN(8, 1) } else if (RT == 2) { AVC_PERSIST_FN(8, 2) } else { AVC_PERSIST_FN(8, 4) }
  } else {
    if (RT == 1) { AVC_PERSIST_FN(4, 1) } else if (RT == 2) { AVC_PERSIST_FN(4, 2) } else { AVC_PERSIST_FN(4, 4) }
  }
#undef AVC_PERSIST_FN
}

// Workgroups of instance (H, RT) the device can hold at once: the occupancy API's resident
// workgroups per CU (LDS, VGPRs, waves) x CUs.  Cached per instance.
int persist_capacity(int H, int RT, bool two_layer = true) {
  struct Entry { const void* fn; int dev; int cap; };
  static std::vector<Entry> cache;
  const void* fn = persist_fn(H, RT, two_layer);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  for (const auto& e : cache)
    if (e.fn == fn && e.dev == dev) return e.cap;
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, persist_lds(H, RT)) != hipSuccess) {
    (void)hipGetLastError();
    per_cu = 0;
  }
  const int cap = per_cu * device_cus();
  cache.push_back({fn, dev, cap});
  return cap;
}

int g_persist_coop = 0;          // avc_lstm_persist_coop()
int g_persist_inject = 0;        // avc_debug_persist_inject(): launches left that give up at once
unsigned g_spin_limit = kSpinLimit;  // avc_debug_persist_spin_limit()

// ---- Co-residency of persistent launches ---------------------------------------
// A persistent launch needs every workgroup resident at once; the occupancy check above only
// sees an idle device.  Two things can hold CUs while a persistent grid dispatches:
//  * kernels of this process's other streams that wait on something outside the GPU: an RCCL
//    collective waiting for a lagging peer rank.  The host layer keeps them out (dp.GradBuckets:
//    no collective is in flight while a persistent launch dispatches; the buckets that become
//    ready meanwhile are issued behind the event avc_persist_notify records right after the
//    launch, so they run beside the rest of the backward, never beside a dispatch);
//  * persistent launches of another process on the same GPU (several ranks per device: the
//    world-2 DP test on a one-GPU box).  AVC_PERSIST_XPROC_LOCK=<file> serialises them: the
//    launching thread holds an exclusive flock on the file from before the launch until a host
//    function enqueued behind it runs (the kernel has finished).  Nothing is waited on while the
//    lock is held except this process's own queued work, so the lock cannot deadlock.
struct XprocLock {
  std::mutex m;
  int fd = -2;    // -2: environment not read yet; -1: off
  int held = 0;   // launches enqueued and not yet finished
};
XprocLock g_xl;

bool xproc_lock_on() {
  std::lock_guard<std::mutex> g(g_xl.m);
  if (g_xl.fd == -2) {
    const char* path = getenv("AVC_PERSIST_XPROC_LOCK");
    g_xl.fd = (path && *path) ? open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0666) : -1;
  }
  return g_xl.fd >= 0;
}

int xproc_acquire() {
  std::lock_guard<std::mutex> g(g_xl.m);
  if (g_xl.held == 0) {
    int rc;
    do rc = flock(g_xl.fd, LOCK_EX); while (rc != 0 && errno == EINTR);
    if (rc != 0) {
      set_error(std::string("AVC_PERSIST_XPROC_LOCK: flock failed: ") + strerror(errno));
      return AVC_ERR_HIP;
    }
  }
  ++g_xl.held;
  return AVC_OK;
}

void xproc_release() {
  std::lock_guard<std::mutex> g(g_xl.m);
  if (g_xl.held > 0 && --g_xl.held == 0) (void)flock(g_xl.fd, LOCK_UN);
}

void xproc_release_cb(void*) { xproc_release(); }

// Every persistent launch goes through here: the cross-process lock, the launch itself (plain or
// cooperative), the context's notify event and launch count.
int persist_dispatch(avc_context* ctx, const void* fn, dim3 grid, dim3 block, void** args, size_t lds,
                     hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  AVC_HIP(hipStreamIsCapturing(s, &cs));
  const bool capturing = cs != hipStreamCaptureStatusNone;
  const bool xl = xproc_lock_on();
  if (xl) {
    if (capturing) {  // the lock is taken at launch time, which a graph replay does not revisit
      set_error("persistent recurrence: not captured into a graph while AVC_PERSIST_XPROC_LOCK is set");
      return AVC_ERR_WORKSPACE;  // the capturing caller falls back to eager calls
    }
    AVC_TRY(xproc_acquire());
  }
  const hipError_t e = g_persist_coop ? hipLaunchCooperativeKernel(fn, grid, block, args, (unsigned)lds, s)
                                      : hipLaunchKernel(fn, grid, block, args, lds, s);
  if (xl) {
    if (e != hipSuccess || hipLaunchHostFunc(s, xproc_release_cb, nullptr) != hipSuccess) {
      (void)hipStreamSynchronize(s);
      xproc_release();
    }
  }
  AVC_HIP(e);
  if (ctx->persist_event && !capturing)
    AVC_HIP(hipEventRecord(static_cast<hipEvent_t>(ctx->persist_event), s));
  ++ctx->persist_launches;
  return AVC_OK;
}

// Launch: grid (nslot * ncb, ngrp); co-residency was checked by the eligibility test.
int persist_launch(avc_context* ctx, PersistArgs a, int RT, int ngrp, hipStream_t s) {
  const dim3 grid(a.nslot * a.ncb, ngrp);
  a.nwg = (int)(grid.x * grid.y);
  for (int L = 0; L < a.nslot; ++L)
    AVC_CHECK_ARG(a.W[L] && a.winv[L], "persistent recurrence: a slot's split weights are missing");
  AVC_CHECK_ARG(a.in_slot == 0 || (a.in_slot == a.nslot - 1 && a.xs && a.b0 && a.gx0 && (a.din == 384 || a.din == 512)),
                "persistent recurrence: input slot operands are missing");
  a.spin_limit = g_spin_limit;
  if (g_persist_inject > 0) {
    --g_persist_inject;
    a.spin_limit = 0;
  }
  const void* fn = persist_fn(a.H, RT, a.nslot >= 3);
  void* args[] = {&a};
  return persist_dispatch(ctx, fn, grid, dim3(256), args, persist_lds(a.H, RT), s);
}

// The counter region of launch layout (kind, T, ngrp, ncb, nwg) on this context: created zeroed (stream-ordered, before
// the first launch that uses it) and kept; least recently used regions beyond kMaxRegions are
// retired (freed when the context is destroyed: a captured graph may still reference them).
constexpr int kMaxRegions = 32;
int persist_region(avc_context* ctx, int kind, int T, int ngrp, int ncb, int nwg, size_t counter_words,
                   hipStream_t s, unsigned** out) {
  const size_t bytes = (kRegionHeaderWords + counter_words) * sizeof(unsigned);
  for (auto& r : ctx->regions) {
    if (r.kind == kind && r.T == T && r.ngrp == ngrp && r.ncb == ncb && r.nwg == nwg && r.bytes == bytes) {
      r.last_use = ++ctx->region_clock;
      *out = static_cast<unsigned*>(r.mem);
      return AVC_OK;
    }
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  AVC_HIP(hipStreamIsCapturing(s, &cs));
  if (cs != hipStreamCaptureStatusNone) {
    set_error("persistent recurrence: counter region missing during graph capture");
    return AVC_ERR_WORKSPACE;  // the caller falls back to eager calls
  }
  if ((int)ctx->regions.size() >= kMaxRegions) {
    auto lru = std::min_element(ctx->regions.begin(), ctx->regions.end(),
                                [](const avc_persist_region& x, const avc_persist_region& y) { return x.last_use < y.last_use; });
    ctx->retired.push_back(lru->mem);
    ctx->regions.erase(lru);
  }
  void* mem = nullptr;
  AVC_HIP(hipMalloc(&mem, bytes));
  AVC_TRY(zero_async(mem, bytes, s));
  avc_persist_region r;
  r.kind = kind; r.T = T; r.ngrp = ngrp; r.ncb = ncb; r.nwg = nwg; r.bytes = bytes; r.mem = mem;
  r.last_use = ++ctx->region_clock;
  ctx->regions.push_back(r);
  *out = static_cast<unsigned*>(mem);
  return AVC_OK;
}

void set_region_args(PersistArgs& a, avc_context* ctx, unsigned* region) {
  a.tickets = reinterpret_cast<unsigned long long*>(region);
  a.tmo = region + 32;
  a.cnt = region + kRegionHeaderWords;
  a.fail_host = ctx->fail_host;
}


}  // namespace

// the co-resident launch machinery for other grid-synchronised kernels (gemm.hip's fused BN)
int coresident_region(avc_context* ctx, int kind, int ngrp, int ncb, int nwg, size_t counter_words, hipStream_t s,
                      unsigned** region) {
  return persist_region(ctx, kind, 0, ngrp, ncb, nwg, counter_words, s, region);
}
int coresident_dispatch(avc_context* ctx, const void* fn, dim3 grid, dim3 block, void** args, size_t lds,
                        hipStream_t s) {
  return persist_dispatch(ctx, fn, grid, block, args, lds, s);
}
unsigned coresident_spin_limit() { return g_spin_limit; }
int persist_region_t(avc_context* ctx, int kind, int T, int ngrp, int ncb, int nwg, size_t counter_words,
                     hipStream_t s, unsigned** out) {
  return persist_region(ctx, kind, T, ngrp, ncb, nwg, counter_words, s, out);
}
bool persist_inject_take() {
  if (g_persist_inject <= 0) return false;
  --g_persist_inject;
  return true;
}
int coresident_cus() { return device_cus(); }

unsigned* host_flags(avc_context* ctx) {
  if (!ctx->fail_host) {
    void* p = nullptr;
    const hipError_t e = hipHostMalloc(&p, 256, hipHostMallocDefault);
    if (e != hipSuccess) {
      set_error(std::string("hipHostMalloc of the context's health words: ") + hipGetErrorString(e));
      return nullptr;
    }
    ctx->fail_host = static_cast<unsigned*>(p);
    ctx->fail_host[0] = ctx->fail_host[1] = 0;
    ctx->fail_seen = 0;
  }
  return ctx->fail_host;
}

int persist_guard(avc_context* ctx) {
  if (!host_flags(ctx)) return AVC_ERR_HIP;
  if (__atomic_exchange_n(ctx->fail_host + 1, 0u, __ATOMIC_ACQ_REL) != 0) {
    set_error("a forward activation handed from one convolution to the next exceeded the split-f16 "
              "operand range (|x| >= 65504) in an earlier call on this context; that call's outputs are "
              "not valid (inf/NaN)");
    return AVC_ERR_DEVICE;
  }
  const unsigned v = __atomic_load_n(ctx->fail_host, __ATOMIC_ACQUIRE);
  if (v == ctx->fail_seen) return AVC_OK;
  ctx->fail_seen = v;
  // the timed-out launch left its counters part-way: start every layout from a fresh region
  for (auto& r : ctx->regions) ctx->retired.push_back(r.mem);
  ctx->regions.clear();
  ctx->gen.epoch = -2;  // the captured forward graph references the retired regions: re-capture
  set_error("a persistent launch (LSTM recurrence, vocoder sample loop, or a convolution with fused BatchNorm) made by an "
            "earlier call on this context abandoned a bounded wait (a workgroup was not resident); that "
            "call's outputs were written as NaN and "
            "the BatchNorm running statistics it updated are not valid. State has been reset.");
  return AVC_ERR_DEVICE;
}

void persist_release(avc_context* ctx) {
  for (auto& r : ctx->regions) (void)hipFree(r.mem);
  ctx->regions.clear();
  if (ctx->fail_host) (void)hipHostFree(ctx->fail_host);
  ctx->fail_host = nullptr;
}

bool lstm2_persist_eligible(int T, int B, int H) {
  if (g_persist_mode == 0 || !(g_persist_layers & 2) || T < 1 || B < 1 || B > 64 || !(H == 1024 || H == 512)) return false;
  const int ntile = (B + 15) / 16, RT = ntile <= 1 ? 1 : (ntile <= 2 ? 2 : 4);
  return 3 * (4 * H / 64) <= persist_capacity(H, RT);  // every workgroup co-resident
}

bool lstm1_persist_eligible(int T, int B, int H) {
  if (g_persist_mode == 0 || !(g_persist_layers & 1) || T < 1 || B < 1 || B > 256 || !(H == 1024 || H == 512)) return false;
  const int RT = lstm1_rows_per_group(B, H), ngrp = (B + 16 * RT - 1) / (16 * RT);
  return ngrp * (4 * H / 64) <= persist_capacity(H, RT, false);
}

int g_persist_inproj = 1;  // avc_lstm_persist_inproj(): an input slot computes layer 0's input projection

namespace {
// The input slot's operands: x split per time step (scaled by the power of two of max |x| unless
// its producer range-checked it: then unscaled, |x| < 65504, as the forward GEMM's guard would
// leave it) into scratch; the split weights come from the caller (split_rows_kernel, K padded).
int attach_inproj(avc_context* ctx, Scratch& sc, const InProj& ip, int T, int B, int slot, PersistArgs& a,
                  hipStream_t s) {
  const int Kp = inproj_kpad(ip.din);
  const int ntile = (B + 15) / 16;
  const long hszx = (long)ntile * 16 * Kp * 2 * 2;
  AVC_TAKE(xs, unsigned char, (size_t)T * hszx, sc);
  const unsigned* amax = nullptr;
  if (ip.x == ctx->xhint.x && (ctx->xhint.amax || ctx->xhint.unit)) {
    amax = ctx->xhint.amax;  // max |x| from x's producer; |x| <= 1: unscaled (XHintScope)
  } else if (!range_checked(ctx, ip.x)) {
    AVC_TAKE(am, unsigned, 2, sc);
    AVC_TRY(gemm_absmax(ip.x, (long)T * B, ip.din, ip.ldx, am, s));
    amax = am;
  }
  const long total = (long)T * ntile * (Kp / 32) * 64;
  split_steps16_kernel<<<(int)std::min<long>((total + 255) / 256, 8192), 256, 0, s>>>(
      ip.x, ip.ldx, T, B, ip.din, Kp, ntile, hszx, xs, amax);
  AVC_LAUNCH_CHECK();
  a.xs = xs; a.hszx = hszx; a.din = Kp; a.b0 = ip.b0; a.x_amax = amax; a.in_slot = slot;
  a.in_lead = g_persist_inproj;
  a.W[slot] = reinterpret_cast<const unsigned char*>(ip.w_s);
  a.winv[slot] = ip.winv;
  return AVC_OK;
}
}  // namespace

// the input slot's scratch: split x per time step, the split W_ih (when not cached), max |x|
size_t inproj_scratch(int T, int B, int H, int din) {
  const size_t ntile = (size_t)(B + 15) / 16, Kp = inproj_kpad(din);
  return al((size_t)T * ntile * 16 * Kp * 2 * 2) + al((size_t)4 * H * Kp * 2 * 2 + 4 * H * sizeof(float)) +
         al(2 * sizeof(unsigned));
}

bool lstm1_inproj_eligible(int T, int B, int H, int din) {
  if (!g_persist_inproj || din <= 256 || din > 512 || din % 8 || !lstm1_persist_eligible(T, B, H)) return false;
  const int RT = lstm1_rows_per_group(B, H), ngrp = (B + 16 * RT - 1) / (16 * RT);
  return 2 * ngrp * (4 * H / 64) <= persist_capacity(H, RT, false);
}

size_t lstm1_persist_scratch(int T, int B, int H, int din) {
  const size_t ntile = (size_t)(B + 15) / 16;
  const size_t hsz = ntile * 16 * H * 2 * 2;
  return al((size_t)T * hsz) + inproj_scratch(T, B, H, din) + 4096;
}

// One LSTM layer (decoder.lstm1, decoder.py:50,69) as one weight-stationary launch: slot 0 of the
// kernel above, with the batch split into independent groups.  gx [T][B][4H] is the input
// projection + biases (permuted columns); whh_s / winv the split W_hh (lstm_split.hip layout).
// y / c [T][B][H], g [T][B][4H] (permuted, optional: training).  Bit-identical to the
// launch-per-step form (same products, same K split, same reduction order).
int lstm1_persist_forward(avc_context* ctx, int T, int B, int H, float* gx, const _Float16* whh_s,
                          const float* winv, float* y, float* g, float* c, hipStream_t s, const InProj* ip,
                          _Float16* y_frag) {
  AVC_CHECK_ARG(lstm1_persist_eligible(T, B, H), "lstm1 persistent path: not eligible for this shape");
  AVC_CHECK_ARG(!ip || lstm1_inproj_eligible(T, B, H, ip->din), "lstm1 input-projection slot: not eligible");
  AVC_TRY(persist_guard(ctx));
  Scratch sc(ctx);
  const int ntile = (B + 15) / 16;
  const long hsz = (long)ntile * 16 * H * 2 * 2;
  const int RT = lstm1_rows_per_group(B, H), ngrp = (B + 16 * RT - 1) / (16 * RT);
  const int nslot = ip ? 2 : 1;
  const long gstride = cnt_words(nslot, T, true);  // counter words per group: full + quarter lines
  const size_t cwords = ((size_t)ngrp * gstride + 63) & ~size_t(63);
  AVC_TAKE(hs0, unsigned char, (size_t)T * hsz, sc);
  unsigned* region = nullptr;
  AVC_TRY(persist_region(ctx, 1, T, ngrp, 4 * H / 64, nslot * ngrp * (4 * H / 64), cwords, s, &region));
  PersistArgs a{};
  a.B = B; a.T = T; a.H = H; a.ncb = 4 * H / 64; a.ntile = ntile;
  a.nslot = nslot; a.cnt_gstride = gstride;
  if (ip) AVC_TRY(attach_inproj(ctx, sc, *ip, T, B, 1, a, s));
  a.W[0] = reinterpret_cast<const unsigned char*>(whh_s);
  a.winv[0] = winv;
  a.gx0 = gx;
  a.hs0 = hs0; a.hsz = hsz;
  a.y0 = y_frag && (ctx->dead_y & 1) ? nullptr : y;  // only the split image is read (avc_context::dead_y)
  a.g0 = g; a.c0 = c;
  a.yfrag = y_frag; a.yf_slot = 0; a.yf_nkc = (H + 31) / 32 * 2;
  a.diag = g_persist_diag;
  set_region_args(a, ctx, region);
  hipEvent_t ev = timing_begin(TC_LSTM1_PERSIST, s);
  AVC_TRY(persist_launch(ctx, a, RT, ngrp, s));
  if (ev) {
    // split W_hh read once; per step the split h operand of every workgroup's group, gx, h, c
    const double flops = (double)T * 2.0 * B * H * 4.0 * H + (ip ? (double)T * 2.0 * B * ip->din * 4.0 * H : 0.0);
    const double bytes = 16.0 * (double)H * H +
                         (double)T * (4.0 * B * H * a.ncb + 4.0 * B * 4.0 * H + 2.0 * 4.0 * B * H);
    timing_end(TC_LSTM1_PERSIST, ev, s, flops, bytes);
  }
  return AVC_OK;
}



// Slot 3 (layer 0's input projection inside the launch) needs K = 512 (4 chunks per wave) and a
// fourth ncb-workgroup slot that is co-resident with the other three.
int inproj_kpad(int din) { return din <= 384 ? 384 : 512; }

bool lstm2_inproj_eligible(int T, int B, int H, int din) {
  if (!g_persist_inproj || din <= 256 || din > 512 || din % 8 || !lstm2_persist_eligible(T, B, H)) return false;
  const int ntile = (B + 15) / 16, RT = ntile <= 1 ? 1 : (ntile <= 2 ? 2 : 4);
  return 4 * (4 * H / 64) <= persist_capacity(H, RT);
}

size_t lstm2_persist_scratch(int T, int B, int H, int din) {
  const size_t ntile = (size_t)(B + 15) / 16;
  const size_t hsz = ntile * 16 * H * 2 * 2;
  return al((size_t)T * hsz) + al((size_t)2 * hsz) + al((size_t)kGxRing * (4 * H / 64) * 64 * 64 * sizeof(float)) +
         inproj_scratch(T, B, H, din) + 4096;
}

// gx0 [T][B][4H] (layer 0's input projection + biases, permuted columns) is computed by the
// caller; w*_s are the split weights with their per-row unscale (lstm_split.hip layout).
int lstm2_persist_forward(avc_context* ctx, int T, int B, int H, float* gx0,
                          const _Float16* w0_s, const float* winv0, const _Float16* w1i_s,
                          const float* winv1i, const _Float16* w1h_s, const float* winv1h,
                          const float* b1_p, float* y0, float* y1, float* g0, float* c0, float* g1,
                          float* c1, hipStream_t s, const InProj* ip, _Float16* y1_frag) {
  AVC_CHECK_ARG(lstm2_persist_eligible(T, B, H), "lstm2 persistent path: not eligible for this shape");
  AVC_CHECK_ARG(!ip || lstm2_inproj_eligible(T, B, H, ip->din), "lstm2 input-projection slot: not eligible");
  AVC_TRY(persist_guard(ctx));
  Scratch sc(ctx);
  const int ntile = (B + 15) / 16;
  const long hsz = (long)ntile * 16 * H * 2 * 2;  // bytes per split-h step buffer
  AVC_TAKE(hs0, unsigned char, (size_t)T * hsz, sc);
  AVC_TAKE(hs1, unsigned char, (size_t)2 * hsz, sc);                      // ring of 2
  AVC_TAKE(gx1, float, (size_t)kGxRing * (4 * H / 64) * 64 * 64, sc);     // slab ring
  const int nslot = ip ? 4 : 3;
  const int RT = ntile <= 1 ? 1 : (ntile <= 2 ? 2 : 4);
  // counters [nslot][T][kRep] (one 128-B line each) and the quarter counters in the persistent
  // region of this layout
  const size_t cwords = ((size_t)cnt_words(nslot, T, true) + 63) & ~size_t(63);
  unsigned* region = nullptr;
  AVC_TRY(persist_region(ctx, 2, T, 1, 4 * H / 64, nslot * (4 * H / 64), cwords, s, &region));
  PersistArgs a{};
  a.B = B; a.T = T; a.H = H; a.ncb = 4 * H / 64; a.ntile = ntile;
  a.nslot = nslot; a.cnt_gstride = 0;
  if (ip) AVC_TRY(attach_inproj(ctx, sc, *ip, T, B, 3, a, s));
  a.W[0] = reinterpret_cast<const unsigned char*>(w0_s);
  a.W[1] = reinterpret_cast<const unsigned char*>(w1i_s);
  a.W[2] = reinterpret_cast<const unsigned char*>(w1h_s);
  a.winv[0] = winv0; a.winv[1] = winv1i; a.winv[2] = winv1h;
  a.gx0 = gx0; a.b1 = b1_p; a.gx1 = gx1;
  a.hs0 = hs0; a.hs1 = hs1; a.hsz = hsz;
  a.y0 = (ctx->dead_y & 2) ? nullptr : y0;             // (avc_context::dead_y)
  a.y1 = y1_frag && (ctx->dead_y & 1) ? nullptr : y1;
  a.g0 = g0; a.g1 = g1; a.c0 = c0; a.c1 = c1;
  a.yfrag = y1_frag; a.yf_slot = 2; a.yf_nkc = (H + 31) / 32 * 2;
  a.diag = g_persist_diag;
  set_region_args(a, ctx, region);
  hipEvent_t ev = timing_begin(TC_LSTM2_PERSIST, s);
  AVC_TRY(persist_launch(ctx, a, RT, 1, s));
  if (ev) {
    // one launch = the whole 2-layer recurrence: 3 products of [B x H] . [H x 4H] per time step;
    // algorithmic bytes = the split weights read once + per step the split h operands and the
    // gx / h / c traffic
    const double flops = 3.0 * T * 2.0 * B * (double)H * 4.0 * H + (ip ? (double)T * 2.0 * B * ip->din * 4.0 * H : 0.0);
    const double bytes = 3.0 * 16.0 * (double)H * H + (double)T * (3.0 * 4.0 * B * H + 3.0 * 4.0 * B * 4.0 * H +
                                                                   2.0 * 4.0 * B * H * 2.0);
    timing_end(TC_LSTM2_PERSIST, ev, s, flops, bytes);
  }
  return AVC_OK;
}

}  // namespace avc

#ifdef AVC_STAMPS
extern "C" int avc_debug_persist_diag(int bits) {
  avc::g_persist_diag = bits;
  ++avc::g_config_epoch;
  return AVC_OK;
}
extern "C" int avc_debug_stamps_persist(void* buf) {
  AVC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(avc::g_pstamps), &buf, sizeof(void*), 0, hipMemcpyHostToDevice));
  return avc::bptt_set_stamps(buf);  // (the BPTT kernels' own copy, lstm_bptt.hip)
}
#endif

extern "C" int avc_lstm_persist_tune(int mode) {
  if (mode < 0 || mode > 2) {
    avc::set_error("avc_lstm_persist_tune: mode must be 0 (off), 1 (acquire hand-off) or 2 (sc1 loads)");
    return AVC_ERR_INVALID;
  }
  avc::g_persist_mode = mode;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_lstm_persist_depth(int chunks) {
  if (chunks < 1 || chunks > 2) {
    avc::set_error("avc_lstm_persist_depth: chunks must be 1 or 2");
    return AVC_ERR_INVALID;
  }
  avc::g_persist_pd = chunks;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_lstm_persist_layers(int mask) {
  if (mask < 0 || mask > 3) {
    avc::set_error("avc_lstm_persist_layers: mask must be 0..3");
    return AVC_ERR_INVALID;
  }
  avc::g_persist_layers = mask;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_lstm_persist_qwait(int mask) {
  if (mask < 0 || mask > 3) {
    avc::set_error("avc_lstm_persist_qwait: mask must be 0..3");
    return AVC_ERR_INVALID;
  }
  avc::g_persist_qwait = mask;
  ++avc::g_config_epoch;
  return AVC_OK;
}


extern "C" int avc_lstm_persist_inproj(int on) {
  if (on < 0 || on > 3) {
    avc::set_error("avc_lstm_persist_inproj: 0 (off), 1 (on), 2 / 3 (on with back-pressure every 4th / every step)");
    return AVC_ERR_INVALID;
  }
  avc::g_persist_inproj = on;
  ++avc::g_config_epoch;
  return AVC_OK;
}





extern "C" int avc_lstm_persist_coop(int on) {
  avc::g_persist_coop = on ? 1 : 0;
  ++avc::g_config_epoch;
  return AVC_OK;
}

extern "C" int avc_debug_persist_inject(int launches) {
  if (launches < 0) {
    avc::set_error("avc_debug_persist_inject: launches must be >= 0");
    return AVC_ERR_INVALID;
  }
  avc::g_persist_inject = launches;
  ++avc::g_config_epoch;  // drop a captured graph: the injection applies to eager launches
  return AVC_OK;
}

extern "C" int avc_persist_check(avc_context* ctx, void* stream, int* failed) {
  AVC_CHECK_ARG(ctx != nullptr, "ctx is NULL");
  AVC_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
  const int rc = avc::persist_guard(ctx);
  if (failed) *failed = rc == AVC_ERR_DEVICE ? 1 : 0;
  return rc;
}

extern "C" int avc_persist_notify(avc_context* ctx, void* event) {
  AVC_CHECK_ARG(ctx != nullptr, "ctx is NULL");
  ctx->persist_event = event;
  return AVC_OK;
}

extern "C" int avc_persist_launches(avc_context* ctx, long* count) {
  AVC_CHECK_ARG(ctx != nullptr && count != nullptr, "NULL pointer");
  *count = ctx->persist_launches;
  return AVC_OK;
}

extern "C" int avc_bptt_persist_eligible(int T, int B, int H) {
  return avc::bptt_persist_eligible(T, B, H) ? 1 : 0;
}

extern "C" int avc_debug_persist_spin_limit(unsigned polls) {
  avc::g_spin_limit = polls ? polls : avc::kSpinLimit;
  ++avc::g_config_epoch;  // drop a captured graph: the limit is a launch argument
  return AVC_OK;
}

namespace avc {
namespace {
// Test load for the co-residency tests: n_wg workgroups that each hold lds_bytes of LDS (a whole
// CU at the maximum) for `ticks` of the constant 100 MHz wall clock, counting themselves resident
// in a pinned host word of its own first (1 + the XCD the workgroup runs on, HW_REG_XCC_ID, so a
// test can see how many CUs each XCD has left).  Bounded by construction (no waits on anything but
// the clock).
__global__ void __launch_bounds__(64) hog_kernel(unsigned long long ticks, unsigned* resident) {
  extern __shared__ unsigned hog_lds[];
  if (threadIdx.x == 0) {
    hog_lds[0] = 1u;
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    __hip_atomic_store(resident + blockIdx.x, 1u + (xcc & 7u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
  }
  __syncthreads();
}
}  // namespace
}  // namespace avc

static unsigned* g_hog_words = nullptr;  // pinned: one "started" word per hog workgroup
static int g_hog_n = 0;

extern "C" int avc_debug_hog(avc_context* ctx, int n_wg, int lds_bytes, long usec, void* stream) {
  AVC_CHECK_ARG(ctx != nullptr, "ctx is NULL");
  AVC_CHECK_ARG(n_wg > 0 && n_wg <= 4096, "avc_debug_hog: n_wg must be 1..4096");
  AVC_CHECK_ARG(lds_bytes >= 4 && lds_bytes <= 160 * 1024, "avc_debug_hog: lds_bytes must be 4..163840");
  AVC_CHECK_ARG(usec > 0 && usec <= 10000000L, "avc_debug_hog: usec must be 1..10^7");
  if (!g_hog_words) AVC_HIP(hipHostMalloc((void**)&g_hog_words, 4096 * sizeof(unsigned), hipHostMallocDefault));
  int dev = 0, khz = 0;
  AVC_HIP(hipGetDevice(&dev));
  AVC_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  if (khz <= 0) khz = 100000;
  AVC_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));  // an earlier hog is done
  memset(g_hog_words, 0, 4096 * sizeof(unsigned));
  g_hog_n = n_wg;
  const void* fn = (const void*)avc::hog_kernel;
  AVC_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
  unsigned long long ticks = (unsigned long long)usec * (unsigned long long)khz / 1000ull;
  unsigned* resident = g_hog_words;
  void* args[] = {&ticks, &resident};
  AVC_HIP(hipLaunchKernel(fn, dim3(n_wg), dim3(64), args, (size_t)lds_bytes, reinterpret_cast<hipStream_t>(stream)));
  return AVC_OK;
}

extern "C" int avc_debug_hog_resident(avc_context* ctx, int* n) {
  AVC_CHECK_ARG(ctx != nullptr && n != nullptr, "NULL pointer");
  int k = 0;
  for (int i = 0; g_hog_words && i < g_hog_n; ++i) k += __atomic_load_n(g_hog_words + i, __ATOMIC_ACQUIRE) != 0;
  *n = k;
  return AVC_OK;
}

extern "C" int avc_debug_hog_xcds(avc_context* ctx, int* per_xcd) {
  AVC_CHECK_ARG(ctx != nullptr && per_xcd != nullptr, "NULL pointer");
  for (int x = 0; x < 8; ++x) per_xcd[x] = 0;
  for (int i = 0; g_hog_words && i < g_hog_n; ++i) {
    const unsigned v = __atomic_load_n(g_hog_words + i, __ATOMIC_ACQUIRE);
    if (v) ++per_xcd[(v - 1) & 7];
  }
  return AVC_OK;
}

extern "C" int avc_lstm_persist_status(long* giveups) {
  if (!giveups) {
    avc::set_error("avc_lstm_persist_status: NULL pointer");
    return AVC_ERR_INVALID;
  }
  unsigned v = 0;
  AVC_HIP(hipDeviceSynchronize());
  AVC_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(avc::g_persist_giveups), sizeof(unsigned), 0, hipMemcpyDeviceToHost));
  *giveups = (long)v + (long)avc::bptt_giveup_count();  // (the BPTT's unit counts its own, lstm_bptt.hip)
  return AVC_OK;
}

