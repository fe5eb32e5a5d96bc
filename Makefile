# gpu-mpi-tests-amd — native build (gfx950 / CDNA4 only).
#
#   make            -> HIP libs + host libs + every native MPI app (HIP and host builds)
#   make lib        -> gpu_mpi_tests_amd/_lib/libgmt.so (+ libgmt_ccl.so): kernels, runtime, RCCL
#   make host       -> build/lib-host/libgmt.so (+ libgmt_ccl.so): the CPU backend (same ABI)
#   make apps       -> build/bin/<app> (HIP) and build/bin-host/<app> (CPU backend)
#
# The apps are compiled ONCE (plain C++17 + MPI against gmt/rt.h, gmt/kernels.h,
# gmt/ccl.h) and linked twice; only the runtime library differs.  No CUDA, no
# SYCL, no gtensor, no #ifdef dual paths: the kernels are hand-written HIP for gfx950.

ROCM      ?= /opt/rocm
MPI_HOME  ?= /opt/conda
ARCH      ?= gfx950
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       := g++

BUILD     := build
OBJ       := $(BUILD)/obj
BIN       := $(BUILD)/bin
BINH      := $(BUILD)/bin-host
LIBDIR    := gpu_mpi_tests_amd/_lib
LIBH_DIR  := $(BUILD)/lib-host
LIB       := $(LIBDIR)/libgmt.so
LIB_CCL   := $(LIBDIR)/libgmt_ccl.so
LIBH      := $(LIBH_DIR)/libgmt.so
LIBH_CCL  := $(LIBH_DIR)/libgmt_ccl.so
LIB_ENG   := $(LIBDIR)/libgmt_engine.so
LIBH_ENG  := $(LIBH_DIR)/libgmt_engine.so

HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
             -Icsrc/include -munsafe-fp-atomics
ROCM_HOST := -O2 -std=c++17 -fPIC -Wall -Icsrc/include -I$(ROCM)/include -D__HIP_PLATFORM_AMD__=1
# SAN: host-side sanitizer flags (make asan-host); never applied to GPU code
SAN       ?=
HOSTFLAGS := -O3 -std=c++17 -fPIC -Wall -ffp-contract=off -Icsrc/include $(SAN)
APPFLAGS  := -O2 -std=c++17 -Wall -Icsrc/include -Icsrc/apps -I$(MPI_HOME)/include $(SAN)
ENGFLAGS  := -O2 -std=c++17 -Wall -fPIC -Icsrc/include $(SAN)
MPI_LIBS  := $(MPI_HOME)/lib/libmpi.so -Wl,-rpath,$(MPI_HOME)/lib -static-libstdc++ -static-libgcc -Wl,--allow-shlib-undefined

KERNEL_SRCS := $(wildcard csrc/kernels/*.hip)
KERNEL_OBJS := $(patsubst csrc/kernels/%.hip,$(OBJ)/kernels/%.o,$(KERNEL_SRCS))
KERNEL_HDRS := $(wildcard csrc/kernels/*.hpp) csrc/include/gmt/kernels.h csrc/include/gmt/tb_geom.h
RT_OBJ      := $(OBJ)/runtime/rt_hip.o
CCL_OBJ     := $(OBJ)/runtime/ccl_rccl.o
HOST_OBJS   := $(OBJ)/host/kernels_host.o $(OBJ)/host/rt_host.o
HOSTCCL_OBJ := $(OBJ)/host/ccl_host.o
COMM_OBJS   := $(OBJ)/comm/transport_mpi.o $(OBJ)/comm/transport_core.o $(OBJ)/comm/transport_ipc.o \
               $(OBJ)/comm/control_socket.o $(OBJ)/engine/jacobi.o
ENG_OBJS    := $(OBJ)/comm/transport_core.o $(OBJ)/comm/transport_ipc.o $(OBJ)/comm/control_socket.o \
               $(OBJ)/engine/jacobi.o $(OBJ)/engine/engine_capi.o $(OBJ)/engine/deriv_bench.o
APP_HDRS    := $(wildcard csrc/include/gmt/*.hpp csrc/include/gmt/*.h csrc/apps/*.hpp)

# reference binary names (Makefile:2, CMakeLists.txt:22-82) + MI355X additions
APPS := daxpy daxpy_nvtx mpi_daxpy mpi_daxpy_nvtx_managed mpi_daxpy_nvtx_unmanaged \
        mpienv mpigatherinplace mpi_daxpy_gt mpi_stencil_gt mpi_stencil2d_gt \
        mpi_stencil2d_sycl mpi_stencil2d_sycl_oo mpi_jacobi2d mpi_stencil2d mpi_halo_bench \
        gmt_kernel_bench

.PHONY: all lib host apps host-apps asan-host sweep clean
all: lib host apps sweep

lib: $(LIB) $(LIB_CCL) $(LIB_ENG)
host: $(LIBH) $(LIBH_CCL) $(LIBH_ENG)

$(OBJ)/kernels/%.o: csrc/kernels/%.hip $(KERNEL_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/runtime/%.o: csrc/runtime/%.cpp csrc/include/gmt/rt.h csrc/include/gmt/ccl.h csrc/include/gmt/numa_bind.hpp
	@mkdir -p $(dir $@)
	$(CXX) $(ROCM_HOST) -c $< -o $@

$(LIB): $(KERNEL_OBJS) $(RT_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -Wl,-soname,libgmt.so \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64 -lrocprofiler-sdk-roctx -ldl

$(LIB_CCL): $(CCL_OBJ) $(LIB)
	$(CXX) -shared -fPIC -o $@ $(CCL_OBJ) -Wl,-soname,libgmt_ccl.so \
	  -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lrccl -lamdhip64

$(OBJ)/host/%.o: csrc/host/%.cpp csrc/include/gmt/rt.h csrc/include/gmt/kernels.h csrc/include/gmt/ccl.h csrc/include/gmt/tb_geom.h csrc/include/gmt/numa_bind.hpp
	@mkdir -p $(dir $@)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIBH): $(HOST_OBJS)
	@mkdir -p $(LIBH_DIR)
	$(CXX) $(SAN) -shared -fPIC -o $@ $^ -Wl,-soname,libgmt.so

$(LIBH_CCL): $(HOSTCCL_OBJ)
	@mkdir -p $(LIBH_DIR)
	$(CXX) $(SAN) -shared -fPIC -o $@ $^ -Wl,-soname,libgmt_ccl.so

$(OBJ)/comm/%.o: csrc/comm/%.cpp $(APP_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(APPFLAGS) -fPIC -c $< -o $@

$(OBJ)/engine/%.o: csrc/engine/%.cpp $(APP_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(ENGFLAGS) -c $< -o $@

# MPI-free engine library for Python (torch.distributed bootstraps RCCL)
$(LIB_ENG): $(ENG_OBJS) $(LIB) $(LIB_CCL)
	$(CXX) -shared -fPIC -o $@ $(ENG_OBJS) -Wl,-soname,libgmt_engine.so -L$(LIBDIR) -lgmt -lgmt_ccl \
	  -Wl,-rpath,'$$ORIGIN' -static-libstdc++ -static-libgcc

$(LIBH_ENG): $(ENG_OBJS) $(LIBH) $(LIBH_CCL)
	$(CXX) -shared -fPIC -o $@ $(ENG_OBJS) -Wl,-soname,libgmt_engine.so -L$(LIBH_DIR) -lgmt -lgmt_ccl \
	  -Wl,-rpath,'$$ORIGIN' -static-libstdc++ -static-libgcc

$(OBJ)/apps/%.o: csrc/apps/%.cpp $(APP_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(APPFLAGS) -c $< -o $@

$(OBJ)/apps/mpi_daxpy_nvtx_managed.o: csrc/apps/mpi_daxpy_nvtx.cpp $(APP_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(APPFLAGS) -DGMT_MANAGED -c $< -o $@

# BASELINE.json names the stencil benchmark "mpi_stencil2d": same program as mpi_jacobi2d
$(OBJ)/apps/mpi_stencil2d.o: csrc/apps/mpi_jacobi2d.cpp $(APP_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(APPFLAGS) -c $< -o $@

$(OBJ)/apps/mpi_daxpy_nvtx_unmanaged.o: csrc/apps/mpi_daxpy_nvtx.cpp $(APP_HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(APPFLAGS) -c $< -o $@

apps: $(addprefix $(BIN)/,$(APPS)) $(addprefix $(BINH)/,$(APPS))

# CPU-only subset (no hipcc needed): host backend + build/bin-host apps
host-apps: host $(addprefix $(BINH)/,$(APPS))

$(BIN)/%: $(OBJ)/apps/%.o $(COMM_OBJS) $(LIB) $(LIB_CCL)
	@mkdir -p $(BIN)
	$(CXX) -o $@ $< $(COMM_OBJS) -L$(LIBDIR) -lgmt -lgmt_ccl \
	  -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)' -Wl,-rpath,$(ROCM)/lib $(MPI_LIBS)

$(BINH)/%: $(OBJ)/apps/%.o $(COMM_OBJS) $(LIBH) $(LIBH_CCL)
	@mkdir -p $(BINH)
	$(CXX) $(SAN) -o $@ $< $(COMM_OBJS) -L$(LIBH_DIR) -lgmt -lgmt_ccl \
	  -Wl,-rpath,'$$ORIGIN/../lib-host' $(MPI_LIBS)

# CPU backend + apps under AddressSanitizer/UBSan (host code only; the
# SURVEY §5.2 plan: sanitizers on host code for CPU-only CI).  Separate tree.
asan-host:
	$(MAKE) BUILD=$(BUILD)/asan SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -g" host-apps

# tuning harnesses (standalone, not part of the libraries): stream_sweep, and
# variant_bench — the A/B kernel variants checked and timed against libgmt
sweep: $(BUILD)/bench/stream_sweep $(BUILD)/bench/variant_bench $(BUILD)/bench/d1_walk $(BUILD)/bench/sdma_probe \
       $(BUILD)/bench/plan_model $(BUILD)/bench/wave_place
# the segment planner on the host (no GPU): plan_model [ny nx mask [resident]] ...
$(BUILD)/bench/plan_model: csrc/bench/plan_model.hip $(KERNEL_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -Icsrc/include -Icsrc/kernels --cuda-host-only -o $@ $<
$(BUILD)/bench/sdma_probe: csrc/bench/sdma_probe.hip
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<
# where the dispatcher puts a workgroup's waves: wave_place [strips_per_wg] [lds_kb_per_strip]
$(BUILD)/bench/wave_place: csrc/bench/wave_place.hip
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<
$(BUILD)/bench/stream_sweep: csrc/bench/stream_sweep.hip
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<
$(BUILD)/bench/variant_bench: csrc/bench/variant_bench.hip $(KERNEL_HDRS) $(LIB)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Icsrc/include -o $@ $< -L$(LIBDIR) -lgmt \
	  -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

$(BUILD)/bench/d1_walk: csrc/bench/d1_walk.hip csrc/kernels/stencil5_d1.hpp csrc/kernels/common.hpp
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Icsrc/include -o $@ $<

.SECONDARY:

clean:
	rm -rf $(BUILD) $(LIB) $(LIB_CCL)
