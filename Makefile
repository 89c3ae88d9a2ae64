# Top-level build (no cmake needed).  `make -j8` builds:
#   fqtool_amd/lib/libfqengine.so  -- C-ABI engine: HIP kernels for gfx950 (include/fqengine.h)
#   oracle/build/liboracle.so      -- CPU restatement (test infrastructure only)
HIPCC      ?= /opt/rocm/bin/hipcc
ARCH       ?= gfx950
HIPFLAGS   ?= -std=c++17 -O3 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CSRC       := fqtool_amd/csrc
LIBDIR     := fqtool_amd/lib
OBJDIR     := build/obj

ENGINE_SRCS := $(CSRC)/engine.hip $(CSRC)/pe_kernel.hip $(CSRC)/pe_fast.hip $(CSRC)/synth.hip
ENGINE_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(ENGINE_SRCS))
ENGINE_HDRS := include/fqengine.h $(CSRC)/engine_internal.h $(CSRC)/device_ops.h

all: engine oracle

engine: $(LIBDIR)/libfqengine.so

$(OBJDIR)/%.o: $(CSRC)/%.hip $(ENGINE_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/libfqengine.so: $(ENGINE_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf build $(LIBDIR) fqtool_amd/bin oracle/build

.PHONY: all engine oracle clean
