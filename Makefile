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

all: $(LIB) oracle

# index-range checks in the CSR kernels (TMD_DCHECK); load with TMDNET_LIB=debug
debug: $(DBGLIB)

build/hip_dbg/%.o: $(PKG)/csrc/%.hip $(wildcard $(PKG)/csrc/*.h) include/tmdnet.h
	@mkdir -p build/hip_dbg
	$(HIPCC) $(HIPFLAGS) -DTMDNET_DEBUG_INDEX -c $< -o $@

$(DBGLIB): $(DBGOBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(DBGOBJS) -o $@

build/hip/%.o: $(PKG)/csrc/%.hip $(wildcard $(PKG)/csrc/*.h) include/tmdnet.h
	@mkdir -p build/hip
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) $(DBGLIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean debug
