// Optional per-kernel-class timing: when enabled, each launch of a class is bracketed by HIP
// events on its stream and its algorithmic FLOPs/bytes are recorded (bench.py roofline).
#pragma once
#include "common.h"

namespace avc {

enum TimingClass : int { TC_GEMM = 0, TC_LSTM_STEP_FWD = 1, TC_LSTM_STEP_BWD = 2, TC_LSTM32 = 3, TC_DFT = 4, TC_LSTM2_PERSIST = 5, TC_LSTM1_PERSIST = 6, TC_WAVERNN = 7, TC_COUNT = 8 };

bool timing_on(int cls);
// returns an event to record after the launch (nullptr when timing is off for cls)
hipEvent_t timing_begin(int cls, hipStream_t s);
void timing_end(int cls, hipEvent_t start, hipStream_t s, double flops, double bytes);

}  // namespace avc
