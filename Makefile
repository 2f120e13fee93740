# Build of the MI355X-native AOI library (gfx950 only) and the CPU oracle.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
# strict float32: the window bounds fl(c-d), fl(c+d) must round like Go's float32
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function
LIBDIR   := goworld_amd/lib
CSRC     := goworld_amd/csrc
HDR      := $(CSRC)/prim.hpp $(CSRC)/gw_internal.hpp $(CSRC)/dev_common.hpp $(CSRC)/ctx.hpp include/gpuaoi.h
OBJ      := $(LIBDIR)/aoi.o $(LIBDIR)/sync.o $(LIBDIR)/halo.o $(LIBDIR)/capi.o $(LIBDIR)/world.o $(LIBDIR)/wire.o $(LIBDIR)/space.o $(LIBDIR)/xport.o
ROCM     ?= /opt/rocm

all: $(LIBDIR)/libgpuaoi.so $(LIBDIR)/c_harness oracle

$(LIBDIR)/%.o: $(CSRC)/%.hip $(HDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/%.o: $(CSRC)/%.cpp $(HDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/libgpuaoi.so: $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ) -L$(ROCM)/lib -lrccl -Wl,-rpath,$(ROCM)/lib

# plain-C caller of the ABI (tests/test_c_harness.py): gcc, no HIP headers
$(LIBDIR)/c_harness: tests/c_harness.c include/gpuaoi.h $(LIBDIR)/libgpuaoi.so
	gcc -O2 -std=c99 -Wall -Iinclude -o $@ tests/c_harness.c -L$(LIBDIR) -lgpuaoi -Wl,-rpath,'$$ORIGIN'

# the plain-C harness with ASan + UBSan on its host code (gcc; the library it
# calls is not instrumented): tests/test_c_harness.py runs it where no GPU is
# needed (argument, input and error paths)
$(LIBDIR)/c_harness_san: tests/c_harness.c include/gpuaoi.h $(LIBDIR)/libgpuaoi.so
	gcc -O1 -g -std=c99 -Wall -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer \
	    -Iinclude -o $@ tests/c_harness.c -L$(LIBDIR) -lgpuaoi -Wl,-rpath,'$$ORIGIN'

san: $(LIBDIR)/c_harness_san
	$(MAKE) -s -C oracle san

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(LIBDIR)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle san clean
