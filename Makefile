# Builds the gfx950 library (libiblb.so) in-tree, and the CPU oracle (test infrastructure).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
PKG      := cuda_iblb_11_amd
CSRC     := $(PKG)/csrc
BUILD    := $(PKG)/build
LIB      := $(PKG)/lib/libiblb.so
SRCS     := $(wildcard $(CSRC)/*.hip)
OBJS     := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(SRCS))
HDRS     := $(wildcard $(CSRC)/*.h) include/iblb.h

all: $(LIB) oracle

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lrccl

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(BUILD) $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
