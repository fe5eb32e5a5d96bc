# gpu-mpi-tests-amd — native build (gfx950 / CDNA4 only).
#
#   make            -> libgmt.so (kernels, C ABI) + native MPI apps in build/bin
#   make lib        -> gpu_mpi_tests_amd/_lib/libgmt.so only
#   make apps       -> build/bin/{daxpy, mpi_daxpy, mpi_stencil2d_gt, ...}
#
# No CUDA, no SYCL, no gtensor: every kernel is hand-written HIP for gfx950
# and every binary is plain C++17 + HIP + MPI (+ RCCL, roctx).

ROCM      ?= /opt/rocm
MPI_HOME  ?= /opt/conda
ARCH      ?= gfx950
HIPCC     ?= $(ROCM)/bin/hipcc
CXX_HOST  ?= g++

BUILD     := build
OBJ       := $(BUILD)/obj
BIN       := $(BUILD)/bin
LIBDIR    := gpu_mpi_tests_amd/_lib
LIB       := $(LIBDIR)/libgmt.so

HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
             -Icsrc/include -munsafe-fp-atomics
HOSTFLAGS := -O2 -std=c++17 -fPIC -Wall -Icsrc/include -I$(ROCM)/include -D__HIP_PLATFORM_AMD__=1

KERNEL_SRCS := $(wildcard csrc/kernels/*.hip)
KERNEL_OBJS := $(patsubst csrc/kernels/%.hip,$(OBJ)/kernels/%.o,$(KERNEL_SRCS))
KERNEL_HDRS := $(wildcard csrc/kernels/*.hpp) csrc/include/gmt/kernels.h

.PHONY: all lib apps clean
all: lib apps

lib: $(LIB)

$(OBJ)/kernels/%.o: csrc/kernels/%.hip $(KERNEL_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(KERNEL_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -Wl,-soname,libgmt.so

-include apps.mk

clean:
	rm -rf $(BUILD) $(LIB)
