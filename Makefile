# Native build: host C++ (g++ -O3 -fopenmp) + HIP kernels (hipcc --offload-arch=gfx950)
# linked into one shared library loaded by the Python package via ctypes, plus the CLI.
#   make -j8            build lib + cli
#   make clean
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
BUILD := build
LIBDIR := lightgbmv1_amd/lib
LIB := $(LIBDIR)/lib_lightgbmv1_amd.so
CLI := $(LIBDIR)/lightgbm

CXXFLAGS ?= -O3 -std=c++17 -fPIC -fopenmp -Wall -Wno-unused-function -Wno-sign-compare -Iinclude -I$(ROCM)/include -D__HIP_PLATFORM_AMD__
# -amdgpu-atomic-optimizer-strategy=None: the device code's global atomics come from one lane
# (reservations, arrival counters); the optimizer's wave loop would wait for each one's return
# at once instead of when its result is used
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -munsafe-fp-atomics -mllvm -amdgpu-atomic-optimizer-strategy=None -Wno-unused-result
HIPEXTRA ?=
LDFLAGS := -shared -fopenmp -L$(ROCM)/lib -lamdhip64 -lrccl -ldl -Wl,-rpath,$(ROCM)/lib

HOST_SRCS := $(filter-out src/cli/main.cpp,$(shell find src -name '*.cpp'))
DEV_SRCS := $(shell find src -name '*.hip')
HOST_OBJS := $(patsubst src/%.cpp,$(BUILD)/%.o,$(HOST_SRCS))
DEV_OBJS := $(patsubst src/%.hip,$(BUILD)/%.hip.o,$(DEV_SRCS))
HEADERS := $(shell find include src -name '*.h' -o -name '*.hpp' -o -name '*.inc' -o -name '*.cuh')

all: $(LIB) $(CLI)

include/lgbm_amd/config_fields.inc src/config/config_auto.cpp: tools/param_spec.py tools/gen_params.py
	python3 tools/gen_params.py

$(BUILD)/%.o: src/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(BUILD)/%.hip.o: src/%.hip $(HEADERS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) $(HIPEXTRA) -c $< -o $@

$(LIB): $(HOST_OBJS) $(DEV_OBJS)
	@mkdir -p $(LIBDIR)
	$(CXX) -o $@ $^ $(LDFLAGS)

$(CLI): src/cli/main.cpp $(LIB)
	$(CXX) $(CXXFLAGS) -o $@ src/cli/main.cpp -L$(LIBDIR) -l_lightgbmv1_amd -Wl,-rpath,'$$ORIGIN' -fopenmp

# host-code sanitizer build (AddressSanitizer + UndefinedBehaviorSanitizer): the CLI linked
# from ASan/UBSan-instrumented host objects and the regular gfx950 device objects.  Device
# code is never instrumented (GPU sanitizers are not used on this platform); the CPU learner
# paths run fully instrumented:  make sanitize && build_asan/lightgbm config=...
ASAN_FLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined
ASAN_OBJS := $(patsubst src/%.cpp,build_asan/%.o,$(HOST_SRCS))

build_asan/%.o: src/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(filter-out -O3,$(CXXFLAGS)) $(ASAN_FLAGS) -c $< -o $@

build_asan/lightgbm: $(ASAN_OBJS) $(DEV_OBJS) src/cli/main.cpp
	$(CXX) $(filter-out -O3,$(CXXFLAGS)) $(ASAN_FLAGS) -o $@ src/cli/main.cpp $(ASAN_OBJS) $(DEV_OBJS) \
	  -fopenmp -L$(ROCM)/lib -lamdhip64 -lrccl -Wl,-rpath,$(ROCM)/lib

sanitize: build_asan/lightgbm

# ThreadSanitizer build of the host code: the C API driver
# tests/native/tsan_driver.cpp linked from TSan-instrumented host objects (device objects
# uninstrumented); OpenMP runs at one thread (libgomp is not instrumented)
TSAN_FLAGS := -O1 -g -fno-omit-frame-pointer -fsanitize=thread
TSAN_OBJS := $(patsubst src/%.cpp,build_tsan/%.o,$(HOST_SRCS))

build_tsan/%.o: src/%.cpp $(HEADERS)
	@mkdir -p $(dir $@)
	$(CXX) $(filter-out -O3,$(CXXFLAGS)) $(TSAN_FLAGS) -c $< -o $@

build_tsan/tsan_driver: $(TSAN_OBJS) $(DEV_OBJS) tests/native/tsan_driver.cpp
	$(CXX) $(filter-out -O3,$(CXXFLAGS)) $(TSAN_FLAGS) -o $@ tests/native/tsan_driver.cpp $(TSAN_OBJS) $(DEV_OBJS) \
	  -fopenmp -L$(ROCM)/lib -lamdhip64 -lrccl -Wl,-rpath,$(ROCM)/lib

tsan: build_tsan/tsan_driver

clean:
	rm -rf $(BUILD) build_asan build_tsan $(LIB) $(CLI)

.PHONY: all clean sanitize tsan
