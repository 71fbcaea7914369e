# Top-level build (no cmake): HIP codec library for gfx950, host C++ layer,
# synthetic-data generator, and the test-only oracle.  `make -j8`.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := flare-cpp_amd
LIB      := $(PKG)/lib
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall
CSRC     := $(PKG)/csrc/capi.hip $(PKG)/csrc/snappy_decode.hip $(PKG)/csrc/snappy_encode.hip
CHDRS    := $(PKG)/csrc/snappy_device.h include/flare_snappy_gpu.h
OBJDIR   := build/obj

all: gpu datagen oracle

gpu: $(LIB)/libflare_snappy_gpu.so

$(OBJDIR)/%.o: $(PKG)/csrc/%.hip $(CHDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB)/libflare_snappy_gpu.so: $(patsubst $(PKG)/csrc/%.hip,$(OBJDIR)/%.o,$(CSRC))
	@mkdir -p $(LIB)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

datagen: $(LIB)/libflare_datagen.so

$(LIB)/libflare_datagen.so: $(PKG)/tools/datagen.c
	@mkdir -p $(LIB)
	gcc -std=c11 -O2 -fPIC -shared -pthread -o $@ $< -lm

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB)/*.so
	$(MAKE) -C oracle clean

.PHONY: all gpu datagen oracle clean
