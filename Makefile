# Builds the MI355X (gfx950) HIP library behind the C ABI in include/autovc_hip.h.
#   make            -> autovc_amd/libautovc_hip.so
#   make check-abi  -> verifies every symbol declared in the header is exported
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable
SRC      := $(wildcard autovc_amd/csrc/*.hip)
HDR      := $(wildcard autovc_amd/csrc/*.h) include/autovc_hip.h include/autovc_hip_debug.h
OBJ      := $(patsubst autovc_amd/csrc/%.hip,build/%.o,$(SRC))
LIB      := autovc_amd/libautovc_hip.so

all: $(LIB)

# per-file machine-scheduler strategy (round 6, same-box A/B in DESIGN §9p): the persistent
# recurrences schedule for instruction-level parallelism
SCHED_lstm_persist := -mllvm -amdgpu-sched-strategy=max-ilp
SCHED_lstm := -mllvm -amdgpu-sched-strategy=max-ilp

build/%.o: autovc_amd/csrc/%.hip $(HDR) Makefile
	@mkdir -p build
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(SCHED_$*) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

#   (product surface: include/autovc_hip.h; tuning toggles / test hooks: include/autovc_hip_debug.h)
check-abi: $(LIB)
	python3 -c "import re,ctypes;lib=ctypes.CDLL('$(LIB)');n=[re.findall(r'^\w[\w\s\*]*?\b(avc_\w+)\(',open(f).read(),re.M) for f in ('include/autovc_hip.h','include/autovc_hip_debug.h')];[getattr(lib,x) for v in n for x in v];print(len(n[0]),'product +',len(n[1]),'debug symbols ok')"

clean:
	rm -rf build $(LIB)

.PHONY: all clean check-abi

# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the whole library linked into
# tests/host_sanitize/abi_driver.cpp (the sanitizers instrument HOST code only: every -fsanitize
# sits behind -Xarch_host; GPU code is compiled as usual).  `make sanitize` builds and runs it.
SAN_FLAGS := -O2 -g -std=c++17 -fno-omit-frame-pointer -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
             -Xarch_host -fno-sanitize-recover=undefined
SAN_OBJ   := $(patsubst autovc_amd/csrc/%.hip,build/sanitize/%.o,$(SRC))
SAN_BIN   := tests/host_sanitize/abi_driver

build/sanitize/%.o: autovc_amd/csrc/%.hip $(HDR)
	@mkdir -p build/sanitize
	$(HIPCC) --offload-arch=$(ARCH) $(SAN_FLAGS) -c $< -o $@

$(SAN_BIN): $(SAN_OBJ) tests/host_sanitize/abi_driver.cpp include/autovc_hip.h include/autovc_hip_debug.h
	$(HIPCC) --offload-arch=$(ARCH) $(SAN_FLAGS) $(SAN_OBJ) tests/host_sanitize/abi_driver.cpp -o $@

sanitize: $(SAN_BIN)
	ASAN_OPTIONS=protect_shadow_gap=0:detect_leaks=1:abort_on_error=1 LSAN_OPTIONS=suppressions=tests/host_sanitize/lsan.supp UBSAN_OPTIONS=print_stacktrace=1 ./$(SAN_BIN)

.PHONY: sanitize

# diagnostic build with in-kernel s_memtime stamps (never shipped): diag/libautovc_hip_stamps.so
stamps:
	@mkdir -p diag
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -DAVC_STAMPS -shared $(SRC) -o diag/libautovc_hip_stamps.so
.PHONY: stamps
