# Top-level build: HIP library (gfx950), hpipm-cpp shim + its tests, CPU oracle.
# Outputs stay in-tree (git-ignored .so files travel to the GPU box with gpurun).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := srbd-nmpc-solver_amd
CSRC := $(PKG)/csrc
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value
HIP_SRCS := $(CSRC)/riccati_unconstr.hip $(CSRC)/ipm_box.hip $(CSRC)/srbd_qp_capi.hip
HIP_HDRS := $(wildcard $(CSRC)/*.h) include/srbd_qp.h
LIB := $(PKG)/libsrbd_qp.so
OBJDIR := build/obj

all: $(LIB) oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
