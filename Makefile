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

MOCK     := tests/mock_rccl/libiblb_mockrccl.so
# drop-in for the reference driver (main.cu; its Makefile names the binary IBLB)
APP      := $(PKG)/bin/IBLB
CXX      ?= g++

all: $(LIB) $(APP) oracle $(MOCK)

$(APP): $(PKG)/app/iblb_main.cpp include/iblb.h $(LIB)
	@mkdir -p $(dir $(APP))
	$(CXX) -O2 -std=c++17 -Wall -o $@ $< -L$(PKG)/lib -liblb -Wl,-rpath,'$$ORIGIN/../lib'

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lrccl

oracle:
	$(MAKE) -s -C oracle

# test-only build: the product objects + an in-process RCCL stand-in (threads as ranks),
# bound with -Bsymbolic so its ncclX calls never reach a real librccl in the process
$(BUILD)/mock_rccl.o: tests/mock_rccl/mock_rccl.cpp
	@mkdir -p $(BUILD)
	$(HIPCC) -O2 -std=c++17 -fPIC -c $< -o $@

$(MOCK): $(OBJS) $(BUILD)/mock_rccl.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -Wl,-Bsymbolic -o $@ $^ -lpthread

clean:
	rm -rf $(BUILD) $(LIB) $(MOCK) $(APP)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
