# Top-level build: the HIP scan library, the drop-in CLI and the generator.
# Everything is built in-tree so the .so files travel to the GPU box.
HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
CXX     ?= g++
ARCH    ?= gfx950
CFLAGS  ?= -O2 -g -Wall -Wno-alloc-size-larger-than -fPIC
HIPFLAGS ?= -O3 -g --offload-arch=$(ARCH) -fPIC -std=c++17 -Wall -pthread
LIBDIR  = grom_amd/lib
BINDIR  = grom_amd/bin

HOST_SRC = grom_amd/csrc/bamio.c grom_amd/csrc/stream.c grom_amd/csrc/tables.c grom_amd/csrc/synth.c grom_amd/csrc/hostapi.c grom_amd/csrc/grom_main.c grom_amd/csrc/pdecode.c
HOST_OBJ = $(patsubst grom_amd/csrc/%.c,build/%.o,$(HOST_SRC)) build/snvfmt.o build/svcall.o build/inflate_host.o build/devmem.o
DEV_OBJ = build/scan.o build/cnv.o build/sv.o build/ddecode.o
HDRS = include/grom_amd.h grom_amd/csrc/devmem.h grom_amd/csrc/scan_common.h grom_amd/csrc/bamio.h grom_amd/csrc/stream.h grom_amd/csrc/synth.h grom_amd/csrc/pdecode.h grom_amd/csrc/ddecode.h
KHDRS = grom_amd/csrc/k_scan_tile.h grom_amd/csrc/device_common.h grom_amd/csrc/snvfmt.h

all: $(LIBDIR)/libgrom_amd.so $(BINDIR)/grom $(BINDIR)/grom_synth $(BINDIR)/gromc_binding oracle

build/%.o: grom_amd/csrc/%.c $(HDRS)
	@mkdir -p build
	$(CC) $(CFLAGS) -c $< -o $@

# the device BGZF inflater's host twin (same decoder, one lane; tests)
build/inflate_host.o: grom_amd/csrc/inflate_host.cpp grom_amd/csrc/inflate.h $(HDRS)
	@mkdir -p build
	$(CXX) -O2 -g -Wall -fPIC -std=c++17 -c $< -o $@

build/snvfmt.o: grom_amd/csrc/snvfmt.cpp grom_amd/csrc/snvfmt.h $(HDRS)
	@mkdir -p build
	$(CXX) -O2 -g -Wall -fPIC -std=c++17 -pthread -c $< -o $@

build/scan.o: grom_amd/csrc/scan.hip $(HDRS) $(KHDRS) grom_amd/csrc/cnv.h grom_amd/csrc/sv.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# BAM decode on the device (BGZF inflate, inflate.h)
build/ddecode.o: grom_amd/csrc/ddecode.hip grom_amd/csrc/ddecode.h grom_amd/csrc/inflate.h $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the CNV path reproduces the reference's double arithmetic: no fused multiply-add
build/cnv.o: grom_amd/csrc/cnv.hip grom_amd/csrc/cnv.h $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -ffp-contract=off -c $< -o $@

# the breakpoint clusters keep the reference's running-mean arithmetic: no fused multiply-add
build/sv.o: grom_amd/csrc/sv.hip grom_amd/csrc/sv.h $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -ffp-contract=off -c $< -o $@

# device allocations: accounting, reclaim / wait / retry (host code on the HIP runtime)
build/devmem.o: grom_amd/csrc/devmem.cpp $(HDRS)
	@mkdir -p build
	$(HIPCC) -O2 -g -Wall -fPIC -std=c++17 -c $< -o $@

# host list logic and SV rows (needs only the HIP runtime headers)
build/svcall.o: grom_amd/csrc/svcall.cpp grom_amd/csrc/sv.h $(HDRS)
	@mkdir -p build
	$(HIPCC) -O2 -g -Wall -fPIC -std=c++17 -ffp-contract=off -c $< -o $@

$(LIBDIR)/libgrom_amd.so: $(DEV_OBJ) $(HOST_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ -lz -lm -ldl -lpthread

$(BINDIR)/grom: grom_amd/csrc/grom_cli.c $(LIBDIR)/libgrom_amd.so $(HDRS)
	@mkdir -p $(BINDIR)
	$(CC) $(CFLAGS) -o $@ grom_amd/csrc/grom_cli.c -L$(LIBDIR) -lgrom_amd -Wl,-rpath,'$$ORIGIN/../lib' -lz -lm

# INTEGRATION.md section 2's GROM.c-side binding, compiled as written (tests/test_gpu_parity.py)
$(BINDIR)/gromc_binding: tools/gromc_binding.c $(LIBDIR)/libgrom_amd.so $(HDRS)
	@mkdir -p $(BINDIR)
	$(CC) $(CFLAGS) -Iinclude -o $@ tools/gromc_binding.c -L$(LIBDIR) -lgrom_amd -Wl,-rpath,'$$ORIGIN/../lib' -lz -lm

$(BINDIR)/grom_synth: tools/grom_synth.c build/synth.o build/bamio.o
	@mkdir -p $(BINDIR)
	$(CC) $(CFLAGS) -o $@ $^ -lz -lm -ldl -lpthread

oracle:
	$(MAKE) -C oracle

# kernel tuning variants, loaded with GROM_AMD_LIB=...:
#   make variant V=w4 VFLAGS=-DGROM_WAVES_PER_EU=4  ->  grom_amd/lib/variants/libgrom_amd_w4.so
#   make variant V=q0 VFLAGS=-DGI_QUAD=0            (the inflater's bit reader)
variant: $(HOST_OBJ) build/sv.o
	@mkdir -p build/variants $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c grom_amd/csrc/scan.hip -o build/variants/scan_$(V).o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -ffp-contract=off -c grom_amd/csrc/cnv.hip -o build/variants/cnv_$(V).o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c grom_amd/csrc/ddecode.hip -o build/variants/ddecode_$(V).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(LIBDIR)/variants/libgrom_amd_$(V).so build/variants/scan_$(V).o build/variants/cnv_$(V).o build/sv.o build/variants/ddecode_$(V).o $(HOST_OBJ) -lz -lm

clean:
	rm -rf build $(LIBDIR) $(BINDIR)
	$(MAKE) -C oracle clean

.PHONY: all clean oracle variant

# host code under sanitizers (tests/test_sanitize.py): SAN=asan (AddressSanitizer
# + UBSan) or SAN=tsan (ThreadSanitizer).  The device objects are linked
# uninstrumented and never called (tools/san_driver.c runs host paths only).
SAN ?= asan
SANDIR = build/san-$(SAN)
ifeq ($(SAN),tsan)
SANFLAGS = -fsanitize=thread
else
SANFLAGS = -fsanitize=address,undefined -fno-sanitize-recover=undefined
endif
SAN_OBJ = $(patsubst grom_amd/csrc/%.c,$(SANDIR)/%.o,$(HOST_SRC)) $(SANDIR)/snvfmt.o $(SANDIR)/inflate_host.o

$(SANDIR)/%.o: grom_amd/csrc/%.c $(HDRS)
	@mkdir -p $(SANDIR)
	$(CC) -O1 -g -fno-omit-frame-pointer -Wall -Wno-alloc-size-larger-than -fPIC $(SANFLAGS) -c $< -o $@

$(SANDIR)/inflate_host.o: grom_amd/csrc/inflate_host.cpp grom_amd/csrc/inflate.h $(HDRS)
	@mkdir -p $(SANDIR)
	$(CXX) -O1 -g -fno-omit-frame-pointer -Wall -fPIC -std=c++17 $(SANFLAGS) -c $< -o $@

$(SANDIR)/snvfmt.o: grom_amd/csrc/snvfmt.cpp grom_amd/csrc/snvfmt.h $(HDRS)
	@mkdir -p $(SANDIR)
	$(CXX) -O1 -g -fno-omit-frame-pointer -Wall -fPIC -std=c++17 -pthread $(SANFLAGS) -c $< -o $@

# the host list logic and SV rows (only the HIP runtime's API header, for hipStream_t)
$(SANDIR)/svcall.o: grom_amd/csrc/svcall.cpp grom_amd/csrc/sv.h $(HDRS)
	@mkdir -p $(SANDIR)
	$(CXX) -O1 -g -fno-omit-frame-pointer -Wall -fPIC -std=c++17 -pthread -ffp-contract=off -I/opt/rocm/include \
	    -D__HIP_PLATFORM_AMD__ $(SANFLAGS) -c $< -o $@

# the device allocations (host code on the HIP runtime API)
$(SANDIR)/devmem.o: grom_amd/csrc/devmem.cpp $(HDRS)
	@mkdir -p $(SANDIR)
	$(CXX) -O1 -g -fno-omit-frame-pointer -Wall -fPIC -std=c++17 -pthread -I/opt/rocm/include \
	    -D__HIP_PLATFORM_AMD__ $(SANFLAGS) -c $< -o $@

$(SANDIR)/san_driver: tools/san_driver.c $(SAN_OBJ) $(SANDIR)/svcall.o $(SANDIR)/devmem.o $(DEV_OBJ)
	$(CXX) -O1 -g -fno-omit-frame-pointer $(SANFLAGS) -x c tools/san_driver.c -x none $(SAN_OBJ) $(SANDIR)/svcall.o $(SANDIR)/devmem.o $(DEV_OBJ) \
	    -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lz -lm -ldl -lpthread -o $@

$(SANDIR)/grom_synth: tools/grom_synth.c $(SANDIR)/synth.o $(SANDIR)/bamio.o
	$(CC) -O1 -g -fno-omit-frame-pointer $(SANFLAGS) -o $@ $^ -lz -lm -ldl -lpthread

sanitize: $(SANDIR)/san_driver $(SANDIR)/grom_synth

.PHONY: sanitize
