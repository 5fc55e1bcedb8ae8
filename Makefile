# Builds (in-tree, so the .so files travel to the GPU box with gpurun):
#   sycl-ray-tracing_amd/lib/librt_hip.so      product: gfx950 kernel + C ABI (hipcc)
#   sycl-ray-tracing_amd/lib/librt_hostsim.so  CPU build of the same device code (tests only)
#   oracle/liboracle.so                        CPU restatement oracle (tests / cpu_baseline only)
#   build/libm_check                           libm restatement vs glibc checker
#
# Numerics: every object is built with -ffp-contract=off and without
# -ffast-math / -march, because the reference (g++ -O2, baseline x86-64) never
# fuses a*b+c and keeps IEEE division, sqrt, denormals and infinities.
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
ARCH ?= gfx950
PKG := sycl-ray-tracing_amd
SRC := $(PKG)/csrc
LIB := $(PKG)/lib
OBJ := build/obj

CXXFLAGS := -std=c++17 -O2 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function -Wno-unknown-pragmas
HIPFLAGS := -std=c++17 -O3 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math \
            -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -Wno-unknown-pragmas

HDRS := $(wildcard $(SRC)/*.h) include/rt_hip.h
# the kernel sources' hash, compiled into each library (rt_build_id) so a run reports the build it loaded
SRC_HASH := $(shell cat $(SRC)/* include/*.h 2>/dev/null | sha256sum | cut -c1-12)

all: $(LIB)/librt_hip.so $(LIB)/librt_hostsim.so oracle/liboracle.so build/libm_check build/cdf_check stamp

$(OBJ)/%.host.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -c $< -o $@

# (the two objects that compile SRC_HASH in as rt_build_id depend on every file it hashes,
# so a change to a host-only source cannot leave a stale build id in the library)
ALL_SRC := $(wildcard $(SRC)/*) $(wildcard include/*.h)

$(OBJ)/rt_hostsim.o: $(SRC)/rt_hostsim.cpp $(HDRS) $(ALL_SRC)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -fopenmp -DRT_BUILD_SRC='"$(SRC_HASH)"' -c $< -o $@

$(OBJ)/rt_render.o: $(SRC)/rt_render.hip $(HDRS) $(ALL_SRC)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DRT_BUILD_SRC='"$(SRC_HASH)"' -c $< -o $@

$(LIB)/librt_hip.so: $(OBJ)/rt_render.o $(OBJ)/rt_scene.host.o $(OBJ)/rt_imageio.host.o $(OBJ)/rt_capi_host.host.o
	@mkdir -p $(LIB)
	$(HIPCC) -shared --offload-arch=$(ARCH) -fPIC $^ -o $@

# BUILD_COMMIT: "<commit>[-dirty] src=<hash of the kernel sources>", rewritten by every `make`
# (the sources' hash names the build whatever was committed since; bench.py reports it)
stamp: $(LIB)/librt_hip.so
	@c=$$(git rev-parse --short HEAD 2>/dev/null || echo unknown); \
	  git diff --quiet HEAD -- $(SRC) include 2>/dev/null || c="$$c-dirty"; \
	  h=$$(cat $(SRC)/* include/*.h | sha256sum | cut -c1-12); echo "$$c src=$$h" > BUILD_COMMIT

$(LIB)/librt_hostsim.so: $(OBJ)/rt_hostsim.o $(OBJ)/rt_scene.host.o $(OBJ)/rt_imageio.host.o $(OBJ)/rt_capi_host.host.o
	@mkdir -p $(LIB)
	$(CXX) -shared -fopenmp $^ -o $@

oracle/liboracle.so: oracle/cpu_oracle.cpp
	$(MAKE) -C oracle liboracle.so

build/libm_check: tests/native/libm_check.cpp $(SRC)/rt_libm.h $(SRC)/rt_fp.h
	@mkdir -p build
	$(CXX) -std=c++17 -O2 -fopenmp -ffp-contract=off -I$(SRC) $< -o $@ -lm

build/cdf_check: tests/native/cdf_check.cpp $(OBJ)/rt_scene.host.o $(HDRS)
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -I$(SRC) $< $(OBJ)/rt_scene.host.o -o $@

# CPU replay of logged rays over search-BVH variants (tools/probe/walk_probe.cpp; study tool)
build/walk_probe: tools/probe/walk_probe.cpp $(OBJ)/rt_scene.host.o $(HDRS)
	@mkdir -p build
	$(CXX) -std=c++17 -O2 -fopenmp -ffp-contract=off -I$(SRC) $< $(OBJ)/rt_scene.host.o -o $@ -lpthread

# CPU trip counts of stackless occlusion walks vs the short stack (tools/probe/stackless_probe.cpp; study tool)
build/stackless_probe: tools/probe/stackless_probe.cpp $(OBJ)/rt_scene.host.o $(HDRS)
	@mkdir -p build
	$(CXX) -std=c++17 -O2 -fopenmp -ffp-contract=off -I$(SRC) $< $(OBJ)/rt_scene.host.o -o $@ -lpthread

# the reference build (container only; needs /root/reference)
ref:
	$(MAKE) -C oracle/ref OPT=-O2

clean:
	rm -rf $(OBJ) $(LIB) build/libm_check oracle/liboracle.so

.PHONY: all ref clean stamp

# experiment builds: make variant V=name DEFS="-DRT_TAIL_OCC=2" -> lib/librt_hip_name.so (RT_HIP_LIB=...)
variant: $(OBJ)/rt_scene.host.o $(OBJ)/rt_imageio.host.o $(OBJ)/rt_capi_host.host.o
	@mkdir -p $(LIB)
	$(HIPCC) $(HIPFLAGS) $(DEFS) -DRT_BUILD_SRC='"$(SRC_HASH)"' -DRT_BUILD_DEFS='"$(DEFS)"' -c $(SRC)/rt_render.hip -o $(OBJ)/rt_render_$(V).o
	$(HIPCC) -shared --offload-arch=$(ARCH) -fPIC $(OBJ)/rt_render_$(V).o $^ -o $(LIB)/librt_hip_$(V).so

# the same for the hostsim build: make hostsim-variant V=name DEFS="-DRT_SLABS=0" ->
# lib/librt_hostsim_name.so (RT_HOSTSIM_LIB=...; study probes such as tools/far_probe.py)
hostsim-variant: $(OBJ)/rt_imageio.host.o
	@mkdir -p $(LIB)
	$(CXX) $(CXXFLAGS) -fopenmp $(DEFS) -DRT_BUILD_SRC='"$(SRC_HASH)"' -DRT_BUILD_DEFS='"$(DEFS)"' -c $(SRC)/rt_hostsim.cpp -o $(OBJ)/rt_hostsim_$(V).o
	$(CXX) $(CXXFLAGS) $(DEFS) -c $(SRC)/rt_scene.cpp -o $(OBJ)/rt_scene_$(V).o
	$(CXX) $(CXXFLAGS) $(DEFS) -c $(SRC)/rt_capi_host.cpp -o $(OBJ)/rt_capi_host_$(V).o
	$(CXX) -shared -fopenmp $(OBJ)/rt_hostsim_$(V).o $(OBJ)/rt_scene_$(V).o $(OBJ)/rt_capi_host_$(V).o $(OBJ)/rt_imageio.host.o -o $(LIB)/librt_hostsim_$(V).so

# C++ drop-in check (container only): include/render_kernel_hip.h against the
# reference's headers and objects (oracle/_ref, `make ref`), linked to the hostsim
# build of the C ABI. tests/test_shim.py runs it.
REFDIR ?= /root/reference
REFOBJ := oracle/_ref/objO2
build/shim_test: tests/native/shim_test.cpp include/render_kernel_hip.h include/rt_hip.h $(LIB)/librt_hostsim.so
	@mkdir -p build
	$(CXX) -std=gnu++20 -O2 -fopenmp -Iinclude -I$(REFDIR)/include -I$(REFDIR)/rapidobj -I$(REFDIR) $< \
	  $(REFOBJ)/bvh.o $(REFOBJ)/flattened_bvh.o $(REFOBJ)/triangle.o $(REFOBJ)/vec.o $(REFOBJ)/color.o \
	  $(REFOBJ)/mat.o $(REFOBJ)/camera.o $(REFOBJ)/ray.o $(REFOBJ)/utils.o -Wl,--gc-sections \
	  -L$(LIB) -lrt_hostsim -Wl,-rpath,'$$ORIGIN/../$(LIB)' -o $@

# the same drop-in linked to the product library (gfx950): built here, run on the GPU box by
# tests/test_shim.py's gpu test (the box has no /root/reference; the binary carries what it needs)
build/shim_test_hip: tests/native/shim_test.cpp include/render_kernel_hip.h include/rt_hip.h $(LIB)/librt_hip.so
	@mkdir -p build
	$(CXX) -std=gnu++20 -O2 -fopenmp -Iinclude -I$(REFDIR)/include -I$(REFDIR)/rapidobj -I$(REFDIR) $< \
	  $(REFOBJ)/bvh.o $(REFOBJ)/flattened_bvh.o $(REFOBJ)/triangle.o $(REFOBJ)/vec.o $(REFOBJ)/color.o \
	  $(REFOBJ)/mat.o $(REFOBJ)/camera.o $(REFOBJ)/ray.o $(REFOBJ)/utils.o -Wl,--gc-sections \
	  -L$(LIB) -lrt_hip -Wl,-rpath,'$$ORIGIN/../$(LIB)' -o $@

# Host sanitizers: the hostsim build of the render path + the CPU oracle +
# tests/native/sanitize_driver.cpp in one executable per sanitizer.
#   make sanitize  -> build/sanitize_asan (ASan + UBSan) and build/sanitize_tsan (TSan), run
#                     both; logs in profiles/r04_sanitize_{asan,tsan}.log
# TSan: libgomp is not TSan-instrumented (its barriers would be reported as races), so the
# TSan run uses one OpenMP thread per region; what it checks is the std::thread layer of the
# multi-device driver (rt_for_devices, rt_render_variants) and the shared context state.
SAN_SRCS := $(SRC)/rt_hostsim.cpp $(SRC)/rt_scene.cpp $(SRC)/rt_imageio.cpp $(SRC)/rt_capi_host.cpp
SAN_NUM := -ffp-contract=off -fno-fast-math -fno-omit-frame-pointer -g -O1 -fopenmp
ASAN := -fsanitize=address,undefined -fno-sanitize-recover=undefined
TSAN := -fsanitize=thread

build/san_%/driver: tests/native/sanitize_driver.cpp oracle/cpu_oracle.cpp $(SAN_SRCS) $(HDRS)
	@mkdir -p build/san_$*
	for f in $(SAN_SRCS); do $(CXX) -std=c++17 $(SAN_NUM) $($(shell echo $* | tr a-z A-Z)) -c $$f -o build/san_$*/$$(basename $$f .cpp).o || exit 1; done
	$(CXX) -std=gnu++20 $(SAN_NUM) $($(shell echo $* | tr a-z A-Z)) -c oracle/cpu_oracle.cpp -o build/san_$*/cpu_oracle.o
	$(CXX) -std=c++17 $(SAN_NUM) $($(shell echo $* | tr a-z A-Z)) tests/native/sanitize_driver.cpp build/san_$*/*.o -o $@

sanitize: build/san_asan/driver build/san_tsan/driver
	ASAN_OPTIONS=halt_on_error=1:detect_leaks=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
	  OMP_NUM_THREADS=4 build/san_asan/driver scenes asan 2>&1 | tee profiles/r04_sanitize_asan.log
	TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 OMP_NUM_THREADS=1 \
	  build/san_tsan/driver scenes tsan 2>&1 | tee profiles/r04_sanitize_tsan.log

.PHONY: sanitize
