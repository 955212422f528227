// Host-side AddressSanitizer / UndefinedBehaviorSanitizer driver for the C ABI
// (include/autovc_hip.h).  Built by `make sanitize` from the library sources with the sanitizers
// on the HOST code only (-Xarch_host; GPU code is compiled normally), and linked statically into
// this executable, so every host path it reaches -- argument validation, error reporting, the
// arena, shape arithmetic, the tuning hooks and, when a GPU is present, real calls that allocate,
// capture graphs and launch kernels -- runs under ASan/UBSan.
//
//   ./build/sanitize/abi_driver          # exit 0 = no sanitizer report and every check held
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/autovc_hip.h"
#include "../../include/autovc_hip_debug.h"

static int failures = 0;
#define CHECK(cond)                                                             \
  do {                                                                          \
    if (!(cond)) {                                                              \
      std::fprintf(stderr, "CHECK failed at %s:%d: %s (last error: %s)\n", __FILE__, __LINE__, #cond, \
                   avc_last_error());                                           \
      ++failures;                                                               \
    }                                                                           \
  } while (0)

static void host_only() {
  CHECK(avc_abi_version() > 0);
  CHECK(avc_last_error() != nullptr);
  // argument validation returns before touching the device
  CHECK(avc_context_reserve(nullptr, 16) != AVC_OK);
  CHECK(std::strlen(avc_last_error()) > 0);
  CHECK(avc_generator_forward(nullptr, 128, 2, nullptr, nullptr, nullptr, nullptr, 1, nullptr, nullptr, nullptr,
                              nullptr) == AVC_ERR_INVALID);
  CHECK(avc_persist_check(nullptr, nullptr, nullptr) == AVC_ERR_INVALID);
  CHECK(avc_wavernn_generate(nullptr, nullptr, 8, nullptr, nullptr, 1, 100, 10, 1, 0, nullptr, nullptr, nullptr,
                             nullptr, nullptr) == AVC_ERR_INVALID);
  // shape arithmetic
  CHECK(avc_stft_frames(110000, 275) == 1 + 110000 / 275);
  CHECK(avc_generator_param_count() == 96);
  CHECK(avc_speaker_encoder_param_count() == 14);
  CHECK(avc_wavernn_param_count(10) == 126);
  long rows = 0, steps = 0;
  CHECK(avc_wavernn_fold_shape(220275, 1, 11000, 550, &rows, &steps) == AVC_OK && rows == 20 && steps == 12100);
  CHECK(avc_wavernn_fold_shape(8800, 0, 0, 0, &rows, &steps) == AVC_OK && rows == 1 && steps == 8800);
  CHECK(avc_wavernn_fold_shape(0, 1, 1, 1, &rows, &steps) == AVC_ERR_INVALID);
  // tuning hooks: valid values accepted, invalid ones rejected with a message
  CHECK(avc_gemm_config(12) == AVC_ERR_INVALID);
  CHECK(avc_gemm_config(8) == AVC_OK);
  CHECK(avc_lstm_persist_qwait(4) == AVC_ERR_INVALID);
  CHECK(avc_lstm_persist_qwait(1) == AVC_OK);
  CHECK(avc_lstm_tune(17, 0) == AVC_ERR_INVALID);
  CHECK(avc_lstm_tune(0, 0) == AVC_OK);
  CHECK(avc_lstm_persist_tune(3) == AVC_ERR_INVALID);
  CHECK(avc_lstm_persist_tune(2) == AVC_OK);
  CHECK(avc_lstm_persist_depth(0) == AVC_ERR_INVALID);
  CHECK(avc_lstm_persist_depth(3) == AVC_ERR_INVALID);
  CHECK(avc_lstm_persist_layers(4) == AVC_ERR_INVALID);
  CHECK(avc_debug_persist_inject(-1) == AVC_ERR_INVALID);
  // timing bookkeeping (host vectors)
  CHECK(avc_timing_enable(0) == AVC_OK);
  CHECK(avc_timing_reset() == AVC_OK);
  double ms = -1, fl = -1, by = -1;
  long n = -1;
  CHECK(avc_timing_read(0, &ms, &fl, &by, &n) == AVC_OK && n == 0);
  CHECK(avc_timing_read(99, &ms, &fl, &by, &n) == AVC_ERR_INVALID);
}

// splitmix-ish fill of a device buffer with U[-a, a)
static float* dev_uniform(size_t n, float a, unsigned seed) {
  std::vector<float> h(n);
  unsigned long long z = 0x9E3779B97F4A7C15ull * (seed + 1);
  for (size_t i = 0; i < n; ++i) {
    z += 0x9E3779B97F4A7C15ull;
    unsigned long long x = z;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    h[i] = a * (2.0f * (float)((x >> 40) * (1.0 / 16777216.0)) - 1.0f);
  }
  float* d = nullptr;
  if (hipMalloc(&d, n * sizeof(float)) != hipSuccess) return nullptr;
  (void)hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice);
  return d;
}

static void with_gpu() {
  avc_context* ctx = nullptr;
  CHECK(avc_context_create(0, &ctx) == AVC_OK);
  if (!ctx) return;
  // a small GEMM
  const int M = 96, N = 80, K = 64;
  float* A = dev_uniform((size_t)M * K, 1.f, 1);
  float* B = dev_uniform((size_t)K * N, 1.f, 2);
  float* C = nullptr;
  CHECK(hipMalloc(&C, (size_t)M * N * sizeof(float)) == hipSuccess);
  CHECK(avc_gemm(ctx, M, N, K, A, 0, B, 0, nullptr, C, 0, nullptr) == AVC_OK);
  CHECK(avc_gemm(ctx, M, N, K, A, 0, B, 0, nullptr, nullptr, 0, nullptr) != AVC_OK);  // NULL C rejected
  // a whole-Generator forward (eager, then cached twice: the second cached call captures a graph)
  // on small random weights; shapes of the 96 tensors do not matter to the host code beyond
  // being valid allocations of the right sizes, so the real parameter layout is used
  const int P = avc_generator_param_count();
  std::vector<const float*> params(P, nullptr);
  // sizes in state_dict order (autovc_amd/auto_encoder: 3 enc convs, enc BiLSTM, dec lstm1,
  // 3 dec convs, lstm2, linear, 5 postnet convs); each conv block = W, b, gamma, beta, rm, rv
  std::vector<size_t> sizes;
  std::vector<int> positive;  // BN gamma / running_var: drawn around 1
  auto add = [&](size_t n, int pos) { sizes.push_back(n); positive.push_back(pos); };
  auto conv = [&](int ci, int co) {
    add((size_t)co * ci * 5, 0); add(co, 0);      // conv weight, bias
    add(co, 1); add(co, 0); add(co, 0); add(co, 1);  // gamma, beta, running_mean, running_var
  };
  auto lstm = [&](int din, int H) {
    add((size_t)4 * H * din, 0); add((size_t)4 * H * H, 0); add(4 * H, 0); add(4 * H, 0);
  };
  conv(336, 512); conv(512, 512); conv(512, 512);
  lstm(512, 32); lstm(512, 32); lstm(64, 32); lstm(64, 32);
  lstm(320, 512);
  conv(512, 512); conv(512, 512); conv(512, 512);
  lstm(512, 1024); lstm(1024, 1024);
  add((size_t)80 * 1024, 0); add(80, 0);
  conv(80, 512); conv(512, 512); conv(512, 512); conv(512, 512); conv(512, 80);
  CHECK((int)sizes.size() == P);
  std::vector<float*> owned;
  for (int i = 0; i < P && i < (int)sizes.size(); ++i) {
    float* p = dev_uniform(sizes[i], positive[i] ? 0.2f : 0.05f, 100 + i);
    if (positive[i]) {  // shift U[-0.2, 0.2) to [0.8, 1.2)
      std::vector<float> h(sizes[i]);
      (void)hipMemcpy(h.data(), p, sizes[i] * 4, hipMemcpyDeviceToHost);
      for (float& v : h) v += 1.0f;
      (void)hipMemcpy(p, h.data(), sizes[i] * 4, hipMemcpyHostToDevice);
    }
    owned.push_back(p);
    params[i] = p;
  }
  const int Bt = 2, T = 64;
  float* x = dev_uniform((size_t)Bt * 80 * T, 1.f, 7);
  float* c = dev_uniform((size_t)Bt * 256, 0.1f, 8);
  float *mel = nullptr, *post = nullptr, *codes = nullptr;
  CHECK(hipMalloc(&mel, (size_t)Bt * 80 * T * 4) == hipSuccess);
  CHECK(hipMalloc(&post, (size_t)Bt * 80 * T * 4) == hipSuccess);
  CHECK(hipMalloc(&codes, (size_t)Bt * 32 * 4 * 4) == hipSuccess);
  CHECK(avc_generator_forward(ctx, T, Bt, params.data(), x, c, c, 0, mel, post, codes, nullptr) == AVC_OK);
  for (int k = 0; k < 3; ++k)
    CHECK(avc_generator_forward_cached(ctx, T, Bt, params.data(), 1, x, c, c, 0, mel, post, codes, nullptr) == AVC_OK);
  CHECK(avc_generator_forward(ctx, 16, Bt, params.data(), x, c, c, 0, mel, post, codes, nullptr) == AVC_ERR_INVALID);
  CHECK(hipDeviceSynchronize() == hipSuccess);
  int failed = -1;
  CHECK(avc_persist_check(ctx, nullptr, &failed) == AVC_OK && failed == 0);
  CHECK(avc_prepared_release(ctx) == AVC_OK);
  CHECK(avc_context_destroy(ctx) == AVC_OK);
  for (float* p : owned) (void)hipFree(p);
  (void)hipFree(A); (void)hipFree(B); (void)hipFree(C); (void)hipFree(x); (void)hipFree(c);
  (void)hipFree(mel); (void)hipFree(post); (void)hipFree(codes);
}

int main() {
  host_only();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
    with_gpu();
    std::printf("abi_driver: host checks and GPU calls done\n");
  } else {
    std::printf("abi_driver: host checks done (no GPU visible)\n");
  }
  if (failures) std::fprintf(stderr, "abi_driver: %d check(s) failed\n", failures);
  return failures ? 1 : 0;
}
