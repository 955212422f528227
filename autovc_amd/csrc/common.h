// Shared helpers for the AutoVC HIP library (gfx950 / MI355X only).
//
// Conventions used by every kernel in this library:
//   * activations live in HBM time-major: row r = t*B + b of a [T*B][C] row-major matrix
//     ("frame rows"), so a Conv1d tap shift is a row shift of +-B and BatchNorm statistics
//     are plain column reductions;
//   * every pointer is borrowed from the caller (torch owns all tensors); scratch comes from
//     the avc_context arena;
//   * errors are reported through a thread-local message and a non-zero status.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/autovc_hip.h"
#include "../../include/autovc_hip_debug.h"

namespace avc {

void set_error(const std::string& msg);
// bumped by every tuning hook (avc_*_tune / avc_gemm_config): a captured forward graph is only
// replayed under the kernel configuration it was captured with
extern int g_config_epoch;
const char* get_error();

#define AVC_CHECK_ARG(cond, msg)                         \
  do {                                                   \
    if (!(cond)) {                                       \
      ::avc::set_error(std::string("invalid argument: ") + (msg)); \
      return AVC_ERR_INVALID;                            \
    }                                                    \
  } while (0)

#define AVC_HIP(expr)                                                            \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    if (_e != hipSuccess) {                                                      \
      ::avc::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));        \
      return AVC_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

#define AVC_LAUNCH_CHECK()                                                       \
  do {                                                                           \
    hipError_t _e = hipGetLastError();                                           \
    if (_e != hipSuccess) {                                                      \
      ::avc::set_error(std::string("kernel launch: ") + hipGetErrorString(_e));   \
      return AVC_ERR_HIP;                                                        \
    }                                                                            \
  } while (0)

#define AVC_TRY(expr)                  \
  do {                                 \
    int _s = (expr);                   \
    if (_s != AVC_OK) return _s;       \
  } while (0)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace avc

// Device arena owned by a context.  Scratch is handed out stack-like inside one API call
// (mark/release); every call on a context is stream-ordered on the stream it was given, so a
// region is never reused while an earlier kernel on that stream could still read it.
// Derived weight layouts kept across calls (split / permuted / transposed copies of weights),
// keyed by what they are derived from and valid for one caller-supplied weights version.
struct avc_prep_entry {
  int kind = 0;
  const void* key0 = nullptr;
  const void* key1 = nullptr;
  size_t bytes = 0;
  long version = -1;
  void* buf = nullptr;
};

// One captured whole-Generator forward (avc_generator_forward_cached): replayed with a single
// hipGraphLaunch when the next call has the same shapes, parameters and weights version.  The
// graph reads/writes fixed staging buffers; the caller's tensors are copied in and out.
struct avc_gen_graph {
  int T = 0, B = 0, training = -1;
  int epoch = -1;               // avc::g_config_epoch at capture (tuning hooks invalidate graphs)
  long version = -1;
  std::vector<const float*> params;
  int seen = 0;                 // consecutive eager calls with this key
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  float* stage = nullptr;       // x | c_org | c_trg | mel | mel_post | codes
  size_t stage_bytes = 0;
  // graphs captured on the caller's own I/O pointers (no staging copies), for pointer sets that
  // recur (a serving loop alternates a few output buffers); least recently used dropped first
  struct direct_graph {
    const void* io[6];
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    unsigned long last = 0;
  };
  std::vector<direct_graph> direct;
  std::vector<std::vector<const void*>> recent;  // pointer sets seen once (candidates)
  unsigned long clock = 0;
};

// Counter region of a persistent recurrence (lstm_persist.hip): arrival counters that are never
// reset between launches.  Every launch takes a ticket per workgroup; ticket / grid size gives
// the launch's epoch E, and a wait for "all ncb producers of step t" is a wait for the counter to
// reach E * ncb, so a value left by an earlier launch can never satisfy it.  One region per
// launch layout (kind, T, groups, producers per step, grid size), because every word must advance
// by exactly ncb per launch and the ticket count per launch must be the grid size.
struct avc_persist_region {
  int kind = 0, T = 0, ngrp = 0, ncb = 0, nwg = 0;
  size_t bytes = 0;
  void* mem = nullptr;
  unsigned long last_use = 0;
};

struct avc_context {
  int device = 0;
  std::vector<avc_persist_region> regions;
  unsigned long region_clock = 0;
  unsigned* fail_host = nullptr;  // pinned host word: device-wide number of the last timed-out persistent launch
  unsigned* guard_ticket = nullptr;  // self-resetting ticket of the single-launch range scan (gemm.hip)
  // activations whose range a producer already checked (or bounds by construction: an LSTM's h)
  // inside the current whole-Generator forward; their contractions skip the range scan
  bool track_ranges = false;
  // What the caller of one per-layer LSTM call knows about its input x (XHintScope, round 5):
  // its producer's max words ([0] max |x|, [1] max(max |x|, 2^14): ConvBNAct's out_amax), or that
  // |x| <= 1 (x is another LSTM layer's h).  Products and splits that would scan x use them.
  struct { const void* x; const unsigned* amax; bool unit; } xhint{nullptr, nullptr, false};
  std::vector<const void*> range_ok;
  // inside the whole-Generator forward: fp32 outputs of the persistent recurrences that nothing
  // reads (bit 0: the h whose split image y_frag the next contraction streams instead -- lstm1's,
  // lstm2's layer 1; bit 1: lstm2's layer-0 h, which slot 1 takes from the split hand-off); the
  // kernels then skip those stores
  int dead_y = 0;
  unsigned fail_seen = 0;         // value of *fail_host already reported to the caller
  // co-residency hooks (lstm_persist.hip: persist_dispatch): an event recorded right after every
  // persistent launch (avc_persist_notify), and the number of persistent launches so far
  void* persist_event = nullptr;
  long persist_launches = 0;
  // pool of device words handed out already zeroed (max-scan accumulators of gradient products):
  // one zeroing launch per kZeroPool words instead of one per product (zeroed_words)
  unsigned* zpool = nullptr;
  int zpool_next = 0;
  std::vector<avc_prep_entry> prep;
  avc_gen_graph gen;
  hipStream_t capture_stream = nullptr;
  long prep_version = -1;       // >= 0 while a caching call (avc_generator_forward_cached) runs
  std::vector<void*> retired;   // grown-out blocks, freed at destroy
  char* base = nullptr;
  size_t cap = 0;
  size_t top = 0;
};

namespace avc {

// zero `bytes` at p (16-B aligned) on stream s with a kernel (elementwise.hip); used instead of
// hipMemsetAsync everywhere (see there)
int zero_async(void* p, size_t bytes, hipStream_t s);
int fill_async(void* p, size_t bytes, unsigned v, hipStream_t s);
// n (<= 64) device words that read as zero in stream order on s: taken from the context's pool,
// which is re-zeroed by one launch when it wraps (every earlier use of the pool precedes that
// launch on the stream).  While s is capturing a graph the words are zeroed by their own node
// instead (a replay must not depend on the pool's host-side position).  nullptr + error on failure.
unsigned* zeroed_words(avc_context* ctx, int n, hipStream_t s);

// Device-side failures reported through the context's pinned host words (host_flags):
//   [0] number of the last persistent-recurrence launch that abandoned a bounded wait;
//   [1] set when a conv -> conv hand-over held a finite value beyond the f16 split's range.
// persist_guard reports each (once) as AVC_ERR_DEVICE with a message; for [0] it first drops the
// counter regions and the captured forward graph so the next call starts from fresh state.
unsigned* host_flags(avc_context* ctx);  // nullptr (error set) if the pinned words cannot be allocated
inline void mark_range_checked(avc_context* ctx, const void* p) {
  if (ctx->track_ranges) ctx->range_ok.push_back(p);
}
// scope of range tracking: one whole-Generator forward
struct RangeScope {
  avc_context* ctx;
  explicit RangeScope(avc_context* c) : ctx(c) { ctx->track_ranges = true; ctx->range_ok.clear(); }
  ~RangeScope() { ctx->track_ranges = false; ctx->range_ok.clear(); }
};
struct XHintScope {
  avc_context* ctx;
  XHintScope(avc_context* c, const void* x, const unsigned* amax, int unit) : ctx(c) {
    ctx->xhint.x = x; ctx->xhint.amax = amax; ctx->xhint.unit = unit != 0;
  }
  ~XHintScope() { ctx->xhint.x = nullptr; ctx->xhint.amax = nullptr; ctx->xhint.unit = false; }
};
inline bool range_checked(const avc_context* ctx, const void* p) {
  for (const void* q : ctx->range_ok)
    if (q == p) return true;
  return false;
}
int persist_guard(avc_context* ctx);
void persist_release(avc_context* ctx);
// Co-resident launches besides the LSTM recurrences (lstm_persist.hip): the counter region of a
// launch layout (header: ticket line, give-up line; then counter_words), the dispatch (cross-
// process lock, cooperative option, notify event), the bounded spin count, the device's CUs.
// Region kinds: 1-3 the recurrences, 4 the fused-BN GEMM (gemm.hip).
int coresident_region(avc_context* ctx, int kind, int ngrp, int ncb, int nwg, size_t counter_words, hipStream_t s,
                      unsigned** region);
int coresident_dispatch(avc_context* ctx, const void* fn, dim3 grid, dim3 block, void** args, size_t lds,
                        hipStream_t s);
unsigned coresident_spin_limit();
int coresident_cus();

struct Scratch {
  avc_context* ctx;
  size_t mark;
  explicit Scratch(avc_context* c) : ctx(c), mark(c->top) {}
  ~Scratch() { ctx->top = mark; }
  // returns nullptr (and sets error) when the arena is exhausted
  template <typename T>
  T* take(size_t count) {
    size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
    if (ctx->top + bytes > ctx->cap) {
      set_error("context arena exhausted: need " + std::to_string(ctx->top + bytes) +
                " bytes, have " + std::to_string(ctx->cap) + " (call avc_context_reserve)");
      return nullptr;
    }
    T* p = reinterpret_cast<T*>(ctx->base + ctx->top);
    ctx->top += bytes;
    return p;
  }
};

#define AVC_TAKE(var, T, n, scratch)                 \
  T* var = (scratch).template take<T>(n);            \
  if (var == nullptr) return AVC_ERR_WORKSPACE

enum PrepKind : int {
  PREP_CONV_WT = 1,     // conv W [co][ci][5] -> Wt [5][ci][co] fp32
  PREP_CONV_BFRAG,      // ... and its split-f16 fragment-major copy
  PREP_GEMM_BFRAG,      // plain B operand split (key: the fp32 B)
  PREP_LSTM_WIH,        // permuted W_ih fp32
  PREP_LSTM_WIH_BFRAG,  // ... split fragment-major for the input GEMM
  PREP_LSTM_BIAS,       // permuted b_ih + b_hh
  PREP_LSTM_WHH,        // split-f16 fragment-major W_hh (+ per-row unscale after it)
  PREP_LSTM_WIH_SPLIT,  // W_ih in the same split layout (lstm2's input-projection slot)
  PREP_BILSTM_WIH,      // [W_ih_f; W_ih_r] + summed biases (encoder BiLSTM's one input product)
};

// Persistent buffer for derived weights, or nullptr when no caching call is active (the caller
// then derives into scratch as usual).  *fresh: the contents must be (re)computed now.
void* prep_buffer(avc_context* ctx, int kind, const void* key0, const void* key1, size_t bytes,
                  bool* fresh);

// Derived-weight buffer: the cached one when a caching call is active, else scratch.
template <typename T>
T* prep_or_scratch(avc_context* ctx, Scratch& sc, int kind, const void* key0, const void* key1,
                   size_t count, bool* fresh) {
  T* p = static_cast<T*>(prep_buffer(ctx, kind, key0, key1, count * sizeof(T), fresh));
  if (p) return p;
  *fresh = true;
  return sc.template take<T>(count);
}

// running max |x| as float bits (atomicMax of non-negative floats), skipped when the word
// already holds at least v: within a launch the word only grows, so a stale read costs at most
// an unneeded atomic -- thousands of blocks otherwise serialise on one L2 line
__device__ __forceinline__ void amax_update(unsigned* w, float v) {
  const unsigned u = __float_as_uint(v);
  if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < u) atomicMax(w, u);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// One BatchNorm statistics partial (S = column sum of its n rows, Q = sum of squares about its own
// mean S / n; gemm.hip bn_tile_stats) folded into fp64 accumulators about the common shift K:
// s += S, a1 += n (m - K), a2 += Q + n (m - K)^2.  Then mean = s / count and
// var = a2 / count - (a1 / count)^2 -- exact for any K, and with K = the first partial's mean the
// subtraction cancels nothing that fp32 rounding put there.  Shared by bn_finalize_kernel and the
// fused BN epilogue (contraction off: both form the same bits).
// inv_n = 1 / n (callers pass the one reciprocal of the full partial size, and divide only for the
// short last partial: an fp64 division per partial made the combine several times slower).
__device__ __forceinline__ void bn_combine(float S, float Q, long n, double inv_n, double K, double& s, double& a1,
                                           double& a2) {
#pragma clang fp contract(off)
  const double dn = (double)n;
  const double dm = (double)S * inv_n - K;
  s += (double)S;
  a1 += dn * dm;
  a2 += (double)Q + dn * dm * dm;
}
// Gate nonlinearities of the recurrences' step epilogues (the dependent chain of every time step):
// hardware exp (v_exp_f32) and reciprocal (v_rcp_f32), ~1e-7 relative of the libm forms, a few
// instructions instead of ~30 each.  tanh(x) = 2 sigmoid(2x) - 1 (saturates to +-1 correctly).
__device__ __forceinline__ float gate_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float gate_tanh(float x) {
  // |x| < 0.4: odd Taylor polynomial to x^13 (truncation < 3e-8 relative; no cancellation near 0,
  // where 1 - 2 / (e^2x + 1) would lose the small values' relative precision); else
  // sign(x) (1 - 2 / (e^2|x| + 1)) from hardware exp / reciprocal
  const float ax = fabsf(x);
  const float x2 = x * x;
  float p = -0.00359212803f;                // -21844 / 6081075
  p = fmaf(p, x2, 0.00886323552f);          // 1382 / 155925
  p = fmaf(p, x2, -0.0218694885f);          // -62 / 2835
  p = fmaf(p, x2, 0.0539682540f);           // 17 / 315
  p = fmaf(p, x2, -0.133333333f);           // -2 / 15
  p = fmaf(p, x2, 0.333333333f);            // 1 / 3
  const float small = fmaf(-x * x2, p, x);  // x - x^3 (1/3 - 2/15 x^2 + ...)
  const float big = 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * ax));
  return ax < 0.4f ? small : copysignf(big, x);
}

}  // namespace avc
