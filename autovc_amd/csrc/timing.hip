#include "timing.h"

#include <mutex>
#include <vector>

namespace avc {
namespace {
struct Rec {
  hipEvent_t a, b;
  double flops, bytes;
};
std::mutex g_mu;
int g_mask = 0;
std::vector<Rec> g_recs[TC_COUNT];
std::vector<hipEvent_t> g_pool;

hipEvent_t get_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
}  // namespace

bool timing_on(int cls) { return (g_mask >> cls) & 1; }

hipEvent_t timing_begin(int cls, hipStream_t s) {
  if (!timing_on(cls)) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e = get_event();
  if (e) (void)hipEventRecord(e, s);
  return e;
}

void timing_end(int cls, hipEvent_t start, hipStream_t s, double flops, double bytes) {
  if (!start) return;
  std::lock_guard<std::mutex> lk(g_mu);
  hipEvent_t e = get_event();
  if (!e) return;
  (void)hipEventRecord(e, s);
  g_recs[cls].push_back({start, e, flops, bytes});
}

}  // namespace avc

using namespace avc;

extern "C" {

int avc_timing_enable(int mask) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_mask = mask;
  return AVC_OK;
}

int avc_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& v : g_recs) {
    for (auto& r : v) {
      g_pool.push_back(r.a);
      g_pool.push_back(r.b);
    }
    v.clear();
  }
  return AVC_OK;
}

int avc_timing_read(int cls, double* total_ms, double* total_flops, double* total_bytes,
                    long* launches) {
  AVC_CHECK_ARG(cls >= 0 && cls < TC_COUNT, "timing class out of range");
  std::lock_guard<std::mutex> lk(g_mu);
  double ms = 0, fl = 0, by = 0;
  for (auto& r : g_recs[cls]) {
    AVC_HIP(hipEventSynchronize(r.b));
    float t = 0.f;
    AVC_HIP(hipEventElapsedTime(&t, r.a, r.b));
    ms += t;
    fl += r.flops;
    by += r.bytes;
  }
  if (total_ms) *total_ms = ms;
  if (total_flops) *total_flops = fl;
  if (total_bytes) *total_bytes = by;
  if (launches) *launches = (long)g_recs[cls].size();
  return AVC_OK;
}

}  // extern "C"
