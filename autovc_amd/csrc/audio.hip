// Rows either side of the Generator: the mel frontends of
// autovc/audio/spectrogram.py and the speaker encoder of autovc/speaker_encoder/model.py.
//
// Mel spectrogram = framing -> DFT -> |.|^p -> mel projection -> (dB + normalise), as
//   frame_signal_kernel   centre-padded (reflect / zero) frames, only the win_length taps the
//                         window does not zero: frames [F][Kp]
//   dft_basis_kernel      windowed cos / -sin rows [2·nb][Kp] in fp64 (Hann folded in; angles
//                         reduced exactly in integers)
//   dft64_kernel (fp64 MFMA) spec [F][2·nb] = frames · basisᵀ, rounded to fp32 (the DFT as one
//                         product, in float64 like librosa's rfft)
//   spec_power_kernel     |X| or |X|² into [F][ld] (ld = nb rounded up to 4, zero tail)
//   gemm (fp32 MFMA)      mel = mag · melbᵀ, epilogue = 20·log10(max(1e-5,·)) -> (·+100)/100
//                         clipped to [0,1] (spectrogram.py:14-31,53-55), stored channel-first
//                         (n_mels, F) or frame-major (F, n_mels) straight from the epilogue.
// The DFT as a GEMM costs 2·2·nb·win FLOP per frame (4.5 MFLOP at n_fft 2048 / win 1100) on
// the fp64 matrix cores — far above an FFT's count, but one MFMA pass over resident operands
// replaces an FFT's log2(n) dependent passes, and fp64 keeps every bin at librosa's accuracy
// whatever the in-frame dynamic range.
#include <cmath>

#include "common.h"
#include "gemm.h"
#include "kernels.h"
#include "timing.h"

namespace avc {
namespace {

inline int ew_grid(long n) { return (int)std::min<long>((n + 255) / 256, 65536); }

__device__ __forceinline__ long reflect_index(long j, long n) {
  if (n == 1) return 0;
  const long p = 2 * (n - 1);  // numpy 'reflect' (edge not repeated), applied repeatedly
  j %= p;
  if (j < 0) j += p;
  return j >= n ? p - j : j;
}

// frames[f][k] = y[f·hop + (n_fft - win)/2 - n_fft/2 + k] for k < win (librosa.stft, center=True)
__global__ void frame_signal_kernel(const float* __restrict__ y, long n, int n_fft, int hop, int win,
                                    int Kp, int F, int reflect, float* __restrict__ frames) {
  const long total = (long)F * Kp;
  const long off = (n_fft - win) / 2 - n_fft / 2;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int f = (int)(idx / Kp), k = (int)(idx - (long)f * Kp);
    float v = 0.f;
    if (k < win) {
      long j = (long)f * hop + off + k;
      if (j >= 0 && j < n) v = y[j];
      else if (reflect) v = y[reflect_index(j, n)];
    }
    frames[idx] = v;
  }
}

// basis[r][k]: r < nb: w[k]·cos(2π r (k+o)/n_fft); r >= nb: -w[k]·sin(2π (r-nb) (k+o)/n_fft),
// w = periodic Hann of length win, o = (n_fft - win)/2 (the window centred in n_fft)
__global__ void dft_basis_kernel(int n_fft, int win, int nb, int Kp, double* __restrict__ basis) {
  const long total = 2L * nb * Kp;
  const int o = (n_fft - win) / 2;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int r = (int)(idx / Kp), k = (int)(idx - (long)r * Kp);
    double v = 0.0;
    if (k < win) {
      const double w = 0.5 - 0.5 * cospi(2.0 * k / win);
      const int bin = r < nb ? r : r - nb;
      const long ph = ((long)bin * (k + o)) % n_fft;  // exact angle reduction
      const double a = 2.0 * (double)ph / n_fft;
      v = r < nb ? w * cospi(a) : -w * sinpi(a);
    }
    basis[idx] = v;
  }
}

// spec[f][n] = sum_k frames[f][k] * basis[n][k] in fp64 (v_mfma_f64_16x16x4_f64), rounded to
// fp32 — librosa computes the STFT in float64 and stores complex64 (the fp32 MFMA product's
// error is relative to the frame's peak bin: bins > ~140 dB under it, e.g. a pure tone's
// far skirt, would be rounding noise).  64x64 output tile per 256-thread workgroup, 2x2 waves
// of 2x2 16x16 MFMA tiles, K staged through LDS 16 deep (frames widened to fp64 on the way).
__global__ __launch_bounds__(256) void dft64_kernel(int F, int N, int Kp, const float* __restrict__ frames,
                                                    const double* __restrict__ basis, float* __restrict__ spec) {
  __shared__ double As[64][17];
  __shared__ double Bs[64][17];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int f0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  typedef double d4 __attribute__((ext_vector_type(4)));
  d4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < Kp; k0 += 16) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // 64 rows x 16 k of each operand, k fastest
      const int idx = tid + 256 * e, r = idx >> 4, kk = idx & 15;
      const int k = k0 + kk;
      const int f = f0 + r, n = n0 + r;
      As[r][kk] = (f < F && k < Kp) ? (double)frames[(long)f * Kp + k] : 0.0;
      Bs[r][kk] = (n < N && k < Kp) ? basis[(long)n * Kp + k] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[wm * 32 + i * 16 + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[wn * 32 + j * 16 + (lane & 15)][kk + (lane >> 4)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // C/D: col = lane & 15, row = (lane >> 4) + 4 r
        const int f = f0 + wm * 32 + i * 16 + (lane >> 4) + 4 * r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (f < F && n < N) spec[(long)f * N + n] = (float)acc[i][j][r];
      }
}

__global__ void spec_power_kernel(int F, int nb, const float* __restrict__ spec, int power2, int ld,
                                  float* __restrict__ mag) {
  const long total = (long)F * ld;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int f = (int)(idx / ld), j = (int)(idx - (long)f * ld);
    float v = 0.f;
    if (j < nb) {
      const float re = spec[(long)f * 2 * nb + j], im = spec[(long)f * 2 * nb + nb + j];
      const float p = re * re + im * im;
      v = power2 ? p : sqrtf(p);
    }
    mag[idx] = v;
  }
}

// Slaney mel scale (librosa hz_to_mel / mel_to_hz, htk=False)
__device__ double hz_to_mel_d(double f) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = log(6.4) / 27.0;
  return f >= min_log_hz ? min_log_mel + log(f / min_log_hz) / logstep : f / f_sp;
}
__device__ double mel_to_hz_d(double m) {
  const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp;
  const double logstep = log(6.4) / 27.0;
  return m >= min_log_mel ? min_log_hz * exp(logstep * (m - min_log_mel)) : f_sp * m;
}

// librosa.filters.mel(norm='slaney'): out[m][j] (row stride ld, zero tail)
__global__ void mel_basis_kernel(double sr, int n_fft, int n_mels, double f_lo, double f_hi, int ld,
                                 float* __restrict__ out) {
  const int nb = n_fft / 2 + 1;
  const long total = (long)n_mels * ld;
  const double m0 = hz_to_mel_d(f_lo), m1 = hz_to_mel_d(f_hi);
  const double mstep = (m1 - m0) / (n_mels + 1);  // numpy.linspace(m0, m1, n_mels + 2)
  const double fstep = (sr / 2.0) / (nb - 1);     // numpy.linspace(0, sr/2, nb)
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int m = (int)(idx / ld), j = (int)(idx - (long)m * ld);
    float v = 0.f;
    if (j < nb) {
      auto pt = [&](int i) { return mel_to_hz_d(i == n_mels + 1 ? m1 : m0 + i * mstep); };
      const double f0 = pt(m), f1 = pt(m + 1), f2 = pt(m + 2);
      const double fj = j == nb - 1 ? sr / 2.0 : j * fstep;
      const double lower = (fj - f0) / (f1 - f0), upper = (f2 - fj) / (f2 - f1);
      const double w = fmax(0.0, fmin(lower, upper));
      v = (float)(w * (2.0 / (f2 - f0)));
    }
    out[idx] = v;
  }
}

// batch-first (B, T, C) -> time-major frame rows [T*B][C]
__global__ void batch_to_time_major_kernel(int B, int T, int C, const float* __restrict__ src,
                                           float* __restrict__ dst) {
  const long total = (long)B * T * C;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int c = (int)(idx % C);
    const long r = idx / C;  // destination row t*B + b
    const int t = (int)(r / B), b = (int)(r - (long)t * B);
    dst[idx] = src[((long)b * T + t) * C + c];
  }
}

// out[b] = x[b] / ||x[b]||_2 (model.py:88), one 256-thread block per row
__global__ __launch_bounds__(256) void rows_l2_normalize_kernel(int E, const float* __restrict__ x,
                                                                float* __restrict__ out) {
  __shared__ float red[4];
  const float* row = x + (long)blockIdx.x * E;
  float s = 0.f;
  for (int e = threadIdx.x; e < E; e += 256) s += row[e] * row[e];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float nrm = sqrtf(red[0] + red[1] + red[2] + red[3]);
  for (int e = threadIdx.x; e < E; e += 256) out[(long)blockIdx.x * E + e] = row[e] / nrm;
}

// embed_utterance (model.py:189-190): mean over the B partial embeddings, then L2-normalise
__global__ __launch_bounds__(256) void mean_l2_normalize_kernel(int B, int E, const float* __restrict__ x,
                                                                float* __restrict__ out) {
  extern __shared__ float mean[];
  __shared__ float red[4];
  float s = 0.f;
  for (int e = threadIdx.x; e < E; e += 256) {
    float a = 0.f;
    for (int b = 0; b < B; ++b) a += x[(long)b * E + e];
    a /= (float)B;
    mean[e] = a;
    s += a * a;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float nrm = sqrtf(red[0] + red[1] + red[2] + red[3]);
  for (int e = threadIdx.x; e < E; e += 256) out[e] = mean[e] / nrm;
}

struct MelPlan {
  int F, nb, Kp, ld;
  GemmDesc mel;
};

MelPlan mel_plan(long n, int n_fft, int hop, int win, int n_mels, int ld_basis) {
  MelPlan p;
  p.F = (int)(1 + n / hop);
  p.nb = n_fft / 2 + 1;
  p.Kp = (win + 3) & ~3;
  p.ld = (p.nb + 3) & ~3;
  (void)ld_basis;
  p.mel.M = p.F; p.mel.N = n_mels; p.mel.Kc = p.ld;
  p.mel.lda = p.ld; p.mel.b_trans = 1; p.mel.ldb = p.ld;
  return p;
}

}  // namespace
}  // namespace avc

using namespace avc;

extern "C" {

int avc_stft_frames(long n_samples, int hop) { return hop > 0 && n_samples >= 0 ? (int)(1 + n_samples / hop) : -1; }

int avc_mel_basis(double sr, int n_fft, int n_mels, double fmin, double fmax, int ld, float* out, void* stream) {
  AVC_CHECK_ARG(out && sr > 0 && n_fft >= 2 && n_mels > 0 && fmin >= 0 && fmax > fmin, "mel_basis: bad arguments");
  AVC_CHECK_ARG(ld >= n_fft / 2 + 1, "mel_basis: ld < n_fft/2 + 1");
  mel_basis_kernel<<<ew_grid((long)n_mels * ld), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      sr, n_fft, n_mels, fmin, fmax, ld, out);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int avc_mel_spectrogram(avc_context* ctx, const float* wav, long n_samples, int n_fft, int hop,
                        int win_length, int pad_mode, int power, const float* mel_basis, int n_mels,
                        int ld_basis, int db_normalize, int channels_first, float* out, void* stream) {
  AVC_CHECK_ARG(ctx && wav && mel_basis && out, "NULL pointer");
  AVC_CHECK_ARG(n_samples > 0 && n_fft >= 2 && hop > 0 && win_length > 0 && win_length <= n_fft,
                "mel_spectrogram: bad STFT geometry");
  AVC_CHECK_ARG(pad_mode == 0 || pad_mode == 1, "mel_spectrogram: pad_mode must be 0 (constant) or 1 (reflect)");
  AVC_CHECK_ARG(power == 1 || power == 2, "mel_spectrogram: power must be 1 or 2");
  AVC_CHECK_ARG(ld_basis == ((n_fft / 2 + 1 + 3) & ~3), "mel_spectrogram: ld_basis must be n_fft/2+1 rounded up to 4");
  AVC_CHECK_ARG(aligned16(mel_basis), "mel_spectrogram: mel_basis must be 16-byte aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  MelPlan p = mel_plan(n_samples, n_fft, hop, win_length, n_mels, ld_basis);
  const size_t need = 4 * ((size_t)p.F * p.Kp + 2ull * p.F * p.nb + (size_t)p.F * p.ld) + 8 * 2ull * p.nb * p.Kp +
                      gemm_scratch_bytes(p.mel) + 8 * 256;
  AVC_TRY(ensure_arena(ctx, need));
  Scratch sc(ctx);
  AVC_TAKE(frames, float, (size_t)p.F * p.Kp, sc);
  AVC_TAKE(basis, double, 2ull * p.nb * p.Kp, sc);
  AVC_TAKE(spec, float, 2ull * p.F * p.nb, sc);
  AVC_TAKE(mag, float, (size_t)p.F * p.ld, sc);
  frame_signal_kernel<<<ew_grid((long)p.F * p.Kp), 256, 0, s>>>(wav, n_samples, n_fft, hop, win_length, p.Kp,
                                                                 p.F, pad_mode, frames);
  dft_basis_kernel<<<ew_grid(2L * p.nb * p.Kp), 256, 0, s>>>(n_fft, win_length, p.nb, p.Kp, basis);
  AVC_LAUNCH_CHECK();
  hipEvent_t ev = timing_begin(TC_DFT, s);
  dft64_kernel<<<dim3((p.F + 63) / 64, (2 * p.nb + 63) / 64), 256, 0, s>>>(p.F, 2 * p.nb, p.Kp, frames, basis, spec);
  AVC_LAUNCH_CHECK();
  if (ev)
    timing_end(TC_DFT, ev, s, 2.0 * p.F * 2.0 * p.nb * p.Kp,
               4.0 * p.F * p.Kp + 8.0 * 2.0 * p.nb * p.Kp + 4.0 * p.F * 2.0 * p.nb);
  spec_power_kernel<<<ew_grid((long)p.F * p.ld), 256, 0, s>>>(p.F, p.nb, spec, power == 2, p.ld, mag);
  AVC_LAUNCH_CHECK();
  p.mel.A = mag; p.mel.B = mel_basis; p.mel.C = out;
  p.mel.act = db_normalize ? AVC_ACT_DBNORM : AVC_ACT_NONE;
  if (channels_first) { p.mel.ldc = 1; p.mel.ldc_col = p.F; }
  else { p.mel.ldc = n_mels; p.mel.ldc_col = 1; }
  return gemm_run(ctx, p.mel, s);
}

int avc_speaker_encoder_param_count(void) { return 14; }

int avc_speaker_encoder_forward(avc_context* ctx, int T, int B, int n_in, int H, int E,
                                const float* const* params, const float* x, float* embeds, void* stream) {
  AVC_CHECK_ARG(ctx && params && x && embeds, "NULL pointer");
  AVC_CHECK_ARG(T > 0 && B > 0 && n_in > 0 && n_in % 4 == 0 && H % 64 == 0 && E > 0,
                "speaker_encoder: need T, B > 0, n_in % 4 == 0, H % 64 == 0");
  for (int i = 0; i < 14; ++i) AVC_CHECK_ARG(params[i] != nullptr, "speaker_encoder: NULL parameter");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const long TB = (long)T * B;
  GemmDesc lin;
  lin.M = B; lin.N = E; lin.Kc = H;
  lin.lda = H; lin.b_trans = 1; lin.ldb = H;
  lin.B = params[12]; lin.bias0 = params[13]; lin.act = AVC_ACT_RELU; lin.ldc = E;
  lin.prec16 = 1;
  const size_t need = 4 * ((size_t)TB * n_in + 3ull * TB * H + (size_t)B * E) + 8 * 256 +
                      std::max({lstm2_forward_scratch(T, B, n_in, H, false), lstm_forward_scratch(T, B, H, H, false),
                                gemm_scratch_bytes(lin)});
  AVC_TRY(ensure_arena(ctx, need));
  Scratch sc(ctx);
  AVC_TAKE(xt, float, (size_t)TB * n_in, sc);
  AVC_TAKE(y0, float, (size_t)TB * H, sc);
  AVC_TAKE(y1, float, (size_t)TB * H, sc);
  AVC_TAKE(y2, float, (size_t)TB * H, sc);
  AVC_TAKE(raw, float, (size_t)B * E, sc);
  batch_to_time_major_kernel<<<ew_grid(TB * n_in), 256, 0, s>>>(B, T, n_in, x, xt);
  AVC_LAUNCH_CHECK();
  // layers 0 and 1 as one two-layer wavefront, layer 2 on its own (model.py:48-53, 84)
  AVC_TRY(lstm2_forward_impl(ctx, T, B, n_in, H, xt, n_in, params, params + 4, y0, y1, nullptr, nullptr,
                             nullptr, nullptr, s));
  AVC_TRY(lstm_forward_impl(ctx, T, B, H, H, 0, y1, H, params[8], params[9], params[10], params[11], y2, H,
                            nullptr, nullptr, s));
  // hidden[-1] = last layer's output at t = T-1 -> Linear -> ReLU (model.py:87) -> L2 (model.py:90)
  lin.A = y2 + (TB - B) * H; lin.C = raw;
  AVC_TRY(gemm_run(ctx, lin, s));
  rows_l2_normalize_kernel<<<B, 256, 0, s>>>(E, raw, embeds);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

int avc_embedding_mean_normalize(int B, int E, const float* embeds, float* out, void* stream) {
  AVC_CHECK_ARG(embeds && out && B > 0 && E > 0 && E <= 8192, "embedding_mean_normalize: bad arguments");
  mean_l2_normalize_kernel<<<1, 256, E * sizeof(float), reinterpret_cast<hipStream_t>(stream)>>>(B, E, embeds, out);
  AVC_LAUNCH_CHECK();
  return AVC_OK;
}

}  // extern "C"
