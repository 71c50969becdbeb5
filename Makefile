# liborbx.so (HIP, gfx950) + the CPU oracle used by the tests.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := multiagent_orb_slam2_amd
SRC := $(PKG)/csrc
HIPFLAGS := -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result \
            -mllvm -amdgpu-mfma-vgpr-form
HDRS := include/orbx.h $(SRC)/orbx_common.h $(SRC)/orbx_pattern.h $(SRC)/orbx_sincos.h
OBJS := $(SRC)/orbx_extract.o $(SRC)/orbx_match.o $(SRC)/orbx_vocab.o $(SRC)/orbx_proj.o $(SRC)/orbx_kfdb.o $(SRC)/orbx_fusion.o

all: $(PKG)/liborbx.so oracle build/host_api_bench build/concurrency

# native multi-thread check of the C-ABI (tests/test_gpu_native_concurrency.py runs it; make tsan = the TSan form)
build/concurrency: tests/native/concurrency.cpp include/orbx.h $(PKG)/liborbx.so
	mkdir -p build
	g++ -O2 -std=c++17 -pthread $< -L$(PKG) -lorbx -Wl,-rpath,'$$ORIGIN/../$(PKG)' -o $@

# native per-call latency driver (bench.py host_api.native; dlopens a liborbx.so by path)
build/host_api_bench: scripts/micro/host_api_bench.cpp include/orbx.h
	mkdir -p build
	g++ -O2 -std=c++17 -pthread $< -ldl -o $@

$(SRC)/%.o: $(SRC)/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/liborbx.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -ldl

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -f $(OBJS) $(PKG)/liborbx.so
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean

# Diagnostics build: k_quadtree stage stamps (orbx_debug_qt_prof), scripts/qt_prof.py.  Not the product library.
qtprof: $(OBJS)
	mkdir -p build/qtprof
	$(HIPCC) $(HIPFLAGS) -DORBX_QT_PROF -c $(SRC)/orbx_extract.hip -o build/qtprof/orbx_extract.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o build/qtprof/liborbx.so build/qtprof/orbx_extract.o $(filter-out $(SRC)/orbx_extract.o,$(OBJS)) -ldl
.PHONY: qtprof

# A/B builds of compile-time variants: make variant V=name D="-DORBX_X=1" [VF=orbx_proj] -> build/<name>/liborbx.so
# (ORBX_LIB=...); VF is the source file the defines apply to (default orbx_extract)
VF ?= orbx_extract
variant: $(OBJS)
	mkdir -p build/$(V)
	$(HIPCC) $(HIPFLAGS) $(D) -c $(SRC)/$(VF).hip -o build/$(V)/$(VF).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o build/$(V)/liborbx.so build/$(V)/$(VF).o $(filter-out $(SRC)/$(VF).o,$(OBJS)) -ldl
.PHONY: variant

# ThreadSanitizer on the host code of liborbx and the native concurrency driver (tests/native/concurrency.cpp):
# host-only instrumentation (-Xarch_host), device code untouched.  Run on a GPU box: scripts/tsan_gpu.sh
TSAN := build/tsan
tsan:
	mkdir -p $(TSAN)
	for f in orbx_extract orbx_match orbx_vocab orbx_proj orbx_kfdb orbx_fusion; do \
	  $(HIPCC) $(HIPFLAGS) -Xarch_host -fsanitize=thread -Xarch_host -g -c $(SRC)/$$f.hip -o $(TSAN)/$$f.o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -fsanitize=thread -fno-gpu-sanitize -o $(TSAN)/liborbx.so $(TSAN)/*.o -ldl
	$(HIPCC) -O1 -g -std=c++17 -fsanitize=thread -fno-gpu-sanitize -o $(TSAN)/concurrency tests/native/concurrency.cpp \
	  -L$(TSAN) -lorbx -Wl,-rpath,'$$ORIGIN' -lpthread
.PHONY: tsan
