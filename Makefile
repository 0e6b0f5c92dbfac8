# Build of the MI355X-native fp64 SpMV engine (gfx950 only).
#
#   make            -> singlespmv_amd/libspmv_hip.so   (C-ABI + HIP kernels)
#                      bin/spmv                        (reference-shaped driver)
#                      oracle/liboracle.so             (test oracle, CPU)
#   make ref        -> oracle/_ref/*.so from /root/reference/src (if present)
#   make probes     -> probes_build/libspmv_hip.so: the same library with the
#                      experiment switches (SPMV_<FMT>_* env variables,
#                      ablation kernels) compiled in, for tools/ only; load it
#                      with SPMV_HIP_LIBRARY=probes_build/libspmv_hip.so
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
HOST_SRC  = $(CSRC)/capi.cpp $(CSRC)/formats.cpp $(CSRC)/build_bin.cpp $(CSRC)/hostutil.cpp $(CSRC)/mmio.cpp \
            $(CSRC)/dist.cpp
KERN_SRC  = $(CSRC)/k_csr.hip $(CSRC)/k_ell.hip $(CSRC)/k_ss.hip $(CSRC)/k_dia.hip $(CSRC)/k_css.hip $(CSRC)/k_coo.hip $(CSRC)/k_convert.hip $(CSRC)/k_probe.hip $(CSRC)/k_bin.hip $(CSRC)/k_bin_build.hip $(CSRC)/k_devbuild.hip $(CSRC)/k_css_build.hip
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
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^ -Wl,-soname,libspmv_hip.so -L$(ROCM)/lib -lrccl

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

# experiment build (tools/ only): -DSPMV_PROBES
PROBEDIR  = probes_build
PROBE_OBJ = $(patsubst $(CSRC)/%.cpp,$(PROBEDIR)/%.o,$(HOST_SRC)) $(patsubst $(CSRC)/%.hip,$(PROBEDIR)/%.o,$(KERN_SRC))

$(PROBEDIR):
	mkdir -p $(PROBEDIR)

$(PROBEDIR)/%.o: $(CSRC)/%.cpp $(HDRS) Makefile | $(PROBEDIR)
	$(HIPCC) $(CXXFLAGS) -DSPMV_PROBES -x c++ -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(PROBEDIR)/%.o: $(CSRC)/%.hip $(HDRS) Makefile | $(PROBEDIR)
	$(HIPCC) $(HIPFLAGS) -DSPMV_PROBES -c $< -o $@

$(PROBEDIR)/libspmv_hip.so: $(PROBE_OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^ -Wl,-soname,libspmv_hip.so -L$(ROCM)/lib -lrccl

# stand-alone HBM probes (tools/*.hip) used by the placement study
bin/region_probe: tools/region_probe.hip Makefile
	mkdir -p bin
	$(HIPCC) $(HIPFLAGS) -o $@ $<

bin/mulorder_probe: tools/mulorder_probe.hip Makefile
	mkdir -p bin
	$(HIPCC) $(HIPFLAGS) -o $@ $<

probes: $(PROBEDIR)/libspmv_hip.so bin/region_probe bin/mulorder_probe

# host-code sanitizer build (CPU only): build/asan/libspmv_hip.so
# with AddressSanitizer + UBSan on every host object (the device code of the
# .hip files is compiled as usual -- GPU sanitizers are not used), plus the
# BIN layout check; `make asan-check` runs the layout check and the CPU test
# suite against it (LD_PRELOAD of the ASan runtime into python).
ASANDIR   = build/asan
SAN_HOST  = -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined -g
ASAN_OBJ  = $(patsubst $(CSRC)/%.cpp,$(ASANDIR)/%.o,$(HOST_SRC)) $(patsubst $(CSRC)/%.hip,$(ASANDIR)/%.o,$(KERN_SRC))
ASAN_RT   = $(shell $(HIPCC) -print-file-name=libclang_rt.asan-x86_64.so)

$(ASANDIR):
	mkdir -p $(ASANDIR)

$(ASANDIR)/%.o: $(CSRC)/%.cpp $(HDRS) Makefile | $(ASANDIR)
	$(HIPCC) $(CXXFLAGS) -O1 $(SAN_HOST) -x c++ -D__HIP_PLATFORM_AMD__ -c $< -o $@

$(ASANDIR)/%.o: $(CSRC)/%.hip $(HDRS) Makefile | $(ASANDIR)
	$(HIPCC) $(HIPFLAGS) -O1 -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -g -c $< -o $@

$(ASANDIR)/libspmv_hip.so: $(ASAN_OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -fsanitize=address,undefined -shared-libsan -o $@ $^ \
	    -Wl,-soname,libspmv_hip.so -L$(ROCM)/lib -lrccl

$(ASANDIR)/bin_layout_check: tests/bin_layout_check.cpp $(ASANDIR)/libspmv_hip.so $(HDRS) Makefile
	$(HIPCC) $(CXXFLAGS) -O1 $(SAN_HOST) -shared-libsan -x c++ -D__HIP_PLATFORM_AMD__ -o $@ tests/bin_layout_check.cpp \
	    -L$(ASANDIR) -lspmv_hip -Wl,-rpath,'$$ORIGIN'

asan: $(ASANDIR)/libspmv_hip.so $(ASANDIR)/bin_layout_check

asan-check: asan
	ASAN_OPTIONS=detect_leaks=0 $(ASANDIR)/bin_layout_check
	ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 LD_PRELOAD=$(ASAN_RT) \
	    SPMV_HIP_LIBRARY=$(ASANDIR)/libspmv_hip.so python3 -m pytest tests -x -q -m "not gpu" -p no:cacheprovider

oracle:
	$(MAKE) -s -C oracle all

ref:
	$(MAKE) -s -C oracle ref

clean:
	rm -rf build $(LIB) $(OPTLIB) bin
	$(MAKE) -s -C oracle clean

.PHONY: all oracle ref clean probes asan asan-check
