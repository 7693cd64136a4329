# Builds the C-ABI HIP library (gfx950) and the C oracle.  `make -j` is safe.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := torchmd-net_amd
LIBDIR   := $(PKG)/torchmdnet/lib
LIB      := $(LIBDIR)/libtmdnet_hip.so
SRCS     := $(wildcard $(PKG)/csrc/*.hip)
OBJS     := $(patsubst $(PKG)/csrc/%.hip,build/hip/%.o,$(SRCS))
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Iinclude -I$(PKG)/csrc -Wall -Wno-unused-function

DBGLIB   := $(LIBDIR)/libtmdnet_hip_debug.so
DBGOBJS  := $(patsubst $(PKG)/csrc/%.hip,build/hip_dbg/%.o,$(SRCS))

# the PyTorch dispatcher boundary (TORCH_LIBRARY ops over the C ABI): host C++, g++ + torch headers
TORCH_DIR := $(shell python3 -c "import os, torch; print(os.path.dirname(torch.__file__))" 2>/dev/null)
TLIB     := $(LIBDIR)/libtmdnet_torch.so
TFLAGS   := -O2 -std=c++17 -fPIC -shared -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -Iinclude \
            -I$(TORCH_DIR)/include -I$(TORCH_DIR)/include/torch/csrc/api/include -I/opt/rocm/include
TLIBS    := -L$(TORCH_DIR)/lib -L$(LIBDIR) -ltorch -ltorch_cpu -lc10 -lc10_hip -ltorch_hip -ltmdnet_hip \
            -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(TORCH_DIR)/lib

all: $(LIB) $(TLIB) oracle

$(TLIB): $(PKG)/csrc/torch_ops.cpp include/tmdnet.h $(LIB)
	g++ $(TFLAGS) $< -o $@ $(TLIBS)

# index-range checks in the CSR kernels (TMD_DCHECK); load with TMDNET_LIB=debug
debug: $(DBGLIB)

build/hip_dbg/%.o: $(PKG)/csrc/%.hip $(wildcard $(PKG)/csrc/*.h) include/tmdnet.h
	@mkdir -p build/hip_dbg
	$(HIPCC) $(HIPFLAGS) -DTMDNET_DEBUG_INDEX -c $< -o $@

$(DBGLIB): $(DBGOBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(DBGOBJS) -o $@

# the fused edge kernels: no SLP packing of f32 math (v_pk_* beside MFMAs costs issue cycles and,
# here, registers: 416 -> 213 VGPR+AGPR for the unrolled variant)
build/hip/et_fused.o build/hip_dbg/et_fused.o: HIPFLAGS += -fno-slp-vectorize

build/hip/%.o: $(PKG)/csrc/%.hip $(wildcard $(PKG)/csrc/*.h) include/tmdnet.h
	@mkdir -p build/hip
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) $(DBGLIB) $(TLIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean debug
