# Top-level build (no cmake needed).  `make -j8` builds:
#   fqtool_amd/lib/libfqengine.so  -- C-ABI engine: HIP kernels for gfx950 (include/fqengine.h)
#   oracle/build/liboracle.so      -- CPU restatement (test infrastructure only)
.DEFAULT_GOAL := all
HIPCC      ?= /opt/rocm/bin/hipcc
ARCH       ?= gfx950
HIPFLAGS   ?= -std=c++17 -O3 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
# make STAMPS=1: compile the per-phase cycle stamps of the fast kernel in (profiling only)
ifneq ($(STAMPS),)
HIPFLAGS   += -DFQ_PHASE_STAMPS
endif
# make AHEAD=n: staging look-ahead of the fast kernel (profiling)
ifneq ($(ABLATE_STAGE),)
HIPFLAGS   += -DFQ_ABLATE_STAGE=$(ABLATE_STAGE)
endif
ifneq ($(OPAQUE_NCH),)
HIPFLAGS   += -DFQ_OPAQUE_NCH=$(OPAQUE_NCH)
endif
ifneq ($(OPAQUE_LK),)
HIPFLAGS   += -DFQ_OPAQUE_LK=$(OPAQUE_LK)
endif
ifneq ($(SCHED_PIN),)
HIPFLAGS   += -DFQ_SCHED_PIN=$(SCHED_PIN)
endif
ifneq ($(AHEAD),)
HIPFLAGS   += -DFQ_AHEAD=$(AHEAD)
endif
CSRC       := fqtool_amd/csrc
LIBDIR     := fqtool_amd/lib
OBJDIR     := build/obj

ENGINE_SRCS := $(CSRC)/engine.hip $(CSRC)/pe_kernel.hip $(CSRC)/pe_fast.hip $(CSRC)/pe_fast_long.hip $(CSRC)/synth.hip $(CSRC)/dup.hip $(CSRC)/kmer.hip $(CSRC)/text.hip $(CSRC)/raw.hip
ENGINE_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(ENGINE_SRCS))
ENGINE_HDRS := include/fqengine.h $(CSRC)/engine_internal.h $(CSRC)/device_ops.h
$(OBJDIR)/pe_fast_long.o: $(CSRC)/pe_fast.hip

CXX        ?= g++
HOSTFLAGS  ?= -std=c++17 -O2 -fPIC -Wall -Wextra -pthread
HOSTDIR    := fqtool_amd/host
HOST_SRCS  := $(HOSTDIR)/json.cpp $(HOSTDIR)/options.cpp $(HOSTDIR)/fastq.cpp $(HOSTDIR)/evaluator.cpp \
              $(HOSTDIR)/report.cpp $(HOSTDIR)/html.cpp $(HOSTDIR)/processor.cpp $(HOSTDIR)/capi.cpp \
              $(HOSTDIR)/pargz.cpp
HOST_OBJS  := $(patsubst $(HOSTDIR)/%.cpp,$(OBJDIR)/host_%.o,$(HOST_SRCS))
HOST_HDRS  := $(wildcard $(HOSTDIR)/*.h) $(HOSTDIR)/known_adapters.inc include/fqengine.h
BINDIR     := fqtool_amd/bin

all: engine host oracle

host: $(LIBDIR)/libfqhost.so $(BINDIR)/fqtool

$(OBJDIR)/host_%.o: $(HOSTDIR)/%.cpp $(HOST_HDRS)
	@mkdir -p $(OBJDIR)
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIBDIR)/libfqhost.so: $(HOST_OBJS) $(LIBDIR)/libfqengine.so
	@mkdir -p $(LIBDIR)
	$(CXX) $(HOSTFLAGS) -shared -o $@ $(HOST_OBJS) -L$(LIBDIR) -lfqengine -Wl,-rpath,'$$ORIGIN' -lz

$(BINDIR)/fqtool: $(HOSTDIR)/main.cpp $(LIBDIR)/libfqhost.so
	@mkdir -p $(BINDIR)
	$(CXX) $(HOSTFLAGS) -o $@ $< -L$(LIBDIR) -lfqhost -lfqengine -Wl,-rpath,'$$ORIGIN/../lib' -lz

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

.PHONY: all engine host oracle clean

# ThreadSanitizer build of the host pipeline (test infrastructure, CPU only): the tool's host sources
# instrumented, linked against oracle/cpu_engine.cpp (the oracle standing in for the engine: host
# packs, text packs and raw streams restated on the CPU) instead of the GPU engine.
# tests/test_tsan_cpu.py runs it.
TSANDIR    := build/tsan
TSANFLAGS  := -std=c++17 -O1 -g -fPIC -pthread -fsanitize=thread
tsan: $(TSANDIR)/fqtool

$(TSANDIR)/host_%.o: $(HOSTDIR)/%.cpp $(HOST_HDRS)
	@mkdir -p $(TSANDIR)
	$(CXX) $(TSANFLAGS) -c $< -o $@

$(TSANDIR)/libfqengine.so: oracle/cpu_engine.cpp oracle/fq_oracle.c oracle/fq_oracle.h include/fqengine.h
	@mkdir -p $(TSANDIR)
	gcc -std=c11 -O1 -g -fPIC -fsanitize=thread -c oracle/fq_oracle.c -o $(TSANDIR)/fq_oracle.o
	$(CXX) $(TSANFLAGS) -Iinclude -Ioracle -shared -o $@ oracle/cpu_engine.cpp $(TSANDIR)/fq_oracle.o -lm

$(TSANDIR)/fqtool: $(patsubst $(HOSTDIR)/%.cpp,$(TSANDIR)/host_%.o,$(HOST_SRCS)) $(HOSTDIR)/main.cpp $(TSANDIR)/libfqengine.so
	$(CXX) $(TSANFLAGS) -o $@ $(HOSTDIR)/main.cpp $(patsubst $(HOSTDIR)/%.cpp,$(TSANDIR)/host_%.o,$(HOST_SRCS)) \
	    -L$(TSANDIR) -lfqengine -Wl,-rpath,'$$ORIGIN' -lz

.PHONY: tsan

# The same host pipeline against the CPU stand-in, uninstrumented (test infrastructure, CPU only):
# tests/test_raw_cpu.py runs the raw-stream and text-pack paths of the tool on the CPU with it.
CPUHDIR    := build/cpuhost
CPUHFLAGS  := -std=c++17 -O2 -g -fPIC -pthread
cpuhost: $(CPUHDIR)/fqtool

$(CPUHDIR)/host_%.o: $(HOSTDIR)/%.cpp $(HOST_HDRS)
	@mkdir -p $(CPUHDIR)
	$(CXX) $(CPUHFLAGS) -c $< -o $@

$(CPUHDIR)/libfqengine.so: oracle/cpu_engine.cpp oracle/fq_oracle.c oracle/fq_oracle.h include/fqengine.h
	@mkdir -p $(CPUHDIR)
	gcc -std=c11 -O2 -g -fPIC -c oracle/fq_oracle.c -o $(CPUHDIR)/fq_oracle.o
	$(CXX) $(CPUHFLAGS) -Iinclude -Ioracle -shared -o $@ oracle/cpu_engine.cpp $(CPUHDIR)/fq_oracle.o -lm

$(CPUHDIR)/fqtool: $(patsubst $(HOSTDIR)/%.cpp,$(CPUHDIR)/host_%.o,$(HOST_SRCS)) $(HOSTDIR)/main.cpp $(CPUHDIR)/libfqengine.so
	$(CXX) $(CPUHFLAGS) -o $@ $(HOSTDIR)/main.cpp $(patsubst $(HOSTDIR)/%.cpp,$(CPUHDIR)/host_%.o,$(HOST_SRCS)) \
	    -L$(CPUHDIR) -lfqengine -Wl,-rpath,'$$ORIGIN' -lz

.PHONY: cpuhost
