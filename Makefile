# Build of the MI355X-native fp64 SpMV engine (gfx950 only).
#
#   make            -> singlespmv_amd/libspmv_hip.so   (C-ABI + HIP kernels)
#                      bin/spmv                        (reference-shaped driver)
#                      oracle/liboracle.so             (test oracle, CPU)
#   make ref        -> oracle/_ref/*.so from /root/reference/src (if present)
#
# Everything is built in-tree so the .so files travel to the GPU box with the
# snapshot (they are git-ignored, not gpurun-ignored).

HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
JOBS     ?= 8
ROCM     ?= /opt/rocm
CXXFLAGS  = -O3 -std=c++17 -fPIC -fopenmp -Wall -Wno-unused-result -Iinclude -I$(ROCM)/include \
            -Isinglespmv_amd/csrc
HIPFLAGS  = $(CXXFLAGS) --offload-arch=$(ARCH) -munsafe-fp-atomics -ffp-contract=off

CSRC      = singlespmv_amd/csrc
LIB       = singlespmv_amd/libspmv_hip.so
OPTLIB    = singlespmv_amd/libopt_hip.so
OBJDIR    = build/obj
HOST_SRC  = $(CSRC)/capi.cpp $(CSRC)/formats.cpp $(CSRC)/build_bin.cpp $(CSRC)/hostutil.cpp $(CSRC)/mmio.cpp
KERN_SRC  = $(CSRC)/k_csr.hip $(CSRC)/k_ell.hip $(CSRC)/k_ss.hip $(CSRC)/k_dia.hip $(CSRC)/k_css.hip $(CSRC)/k_coo.hip $(CSRC)/k_convert.hip $(CSRC)/k_probe.hip $(CSRC)/k_bin.hip $(CSRC)/k_bin_build.hip
HOST_OBJ  = $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(HOST_SRC))
KERN_OBJ  = $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(KERN_SRC))
HDRS      = include/spmv_hip.h include/opt_hip.h include/spmv_util.h \
            $(CSRC)/internal.hpp $(CSRC)/device.hpp

all: $(LIB) $(OPTLIB) bin/spmv bin/csr5_api bin/gather_probe oracle

$(OBJDIR):
	mkdir -p $(OBJDIR)

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS) Makefile | $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) -x c++ -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS) Makefile | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HOST_OBJ) $(KERN_OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^ -Wl,-soname,libspmv_hip.so

# Reference-shaped driver (src/main.cpp counterpart) linked against the
# drop-in OptimizeProblem/SpMV of include/opt_hip.h.
bin/spmv: tools/spmv_main.cpp $(CSRC)/opt_hip.cpp $(LIB) $(HDRS)
	mkdir -p bin
	$(HIPCC) $(CXXFLAGS) -x c++ -D__HIP_PLATFORM_AMD__ -o $@ tools/spmv_main.cpp \
	    $(CSRC)/opt_hip.cpp -Lsinglespmv_amd -lspmv_hip -Wl,-rpath,'$$ORIGIN/../singlespmv_amd'

# the CSR5 benchmark's driver flow over include/csr5_hip.h (anonymouslibHandle)
bin/csr5_api: tools/csr5_api_main.cpp include/csr5_hip.h $(LIB) $(HDRS)
	mkdir -p bin
	$(HIPCC) $(CXXFLAGS) -x c++ -D__HIP_PLATFORM_AMD__ -o $@ tools/csr5_api_main.cpp \
	    -Lsinglespmv_amd -lspmv_hip -Wl,-rpath,'$$ORIGIN/../singlespmv_amd'

# the drop-in as a shared object (format from SPMV_HIP_FORMAT) for ABI tests
$(OPTLIB): $(CSRC)/opt_hip.cpp $(LIB) $(HDRS)
	$(HIPCC) $(CXXFLAGS) -x c++ -D__HIP_PLATFORM_AMD__ -shared -o $@ $(CSRC)/opt_hip.cpp \
	    -Lsinglespmv_amd -lspmv_hip -Wl,-rpath,'$$ORIGIN'

# x-gather micro-benchmark (tools/gather_probe.hip)
bin/gather_probe: tools/gather_probe.hip Makefile
	mkdir -p bin
	$(HIPCC) $(HIPFLAGS) -o $@ $<

oracle:
	$(MAKE) -s -C oracle all

ref:
	$(MAKE) -s -C oracle ref

clean:
	rm -rf build $(LIB) $(OPTLIB) bin
	$(MAKE) -s -C oracle clean

.PHONY: all oracle ref clean
