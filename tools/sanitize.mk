# Host ASan + UBSan builds for tools/sanitize.sh (CPU only; run from the repo root with
# `make -f tools/sanitize.mk`).  Kept out of the product Makefiles so that no file a GPU run
# uses carries sanitizer flags.
#  - variants/libshockidx_san.so: the C-ABI layer with host-only sanitizers, linked with the
#    unchanged device objects of shock_amd/csrc/build (GPU sanitizers are not used)
#  - oracle/build/liboracle_san.so: the C oracle under clang (one sanitizer runtime for both)
HIPCC ?= /opt/rocm/bin/hipcc
SANCC ?= /opt/rocm/lib/llvm/bin/clang
ARCH ?= gfx950
C := shock_amd/csrc
SANFLAGS := -O1 -g -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Xarch_host -fsanitize=address \
	-Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer
ORC := oracle/shockidx_oracle.c oracle/subset_oracle.c oracle/chunk_oracle.c oracle/part_oracle.c oracle/filter_oracle.c

all: shock_amd/variants/libshockidx_san.so oracle/build/liboracle_san.so

$(C)/build/san/sidx_capi.o: $(C)/sidx_capi.cpp $(C)/sidx_common.hpp $(C)/sidx_subset.hpp $(C)/sidx_host.hpp include/shockidx.h
	@mkdir -p $(C)/build/san
	$(HIPCC) $(SANFLAGS) -c $(C)/sidx_capi.cpp -o $@

$(C)/build/san/sidx_multi.o: $(C)/sidx_multi.cpp $(C)/sidx_host.hpp include/shockidx.h
	@mkdir -p $(C)/build/san
	$(HIPCC) $(SANFLAGS) -c $(C)/sidx_multi.cpp -o $@

shock_amd/variants/libshockidx_san.so: $(C)/build/sidx_kernels.o $(C)/build/sidx_subset.o $(C)/build/sidx_chunk.o \
		$(C)/build/sidx_filter.o $(C)/build/san/sidx_capi.o $(C)/build/san/sidx_multi.o
	@mkdir -p shock_amd/variants
	$(HIPCC) -O1 -std=c++17 -fPIC --offload-arch=$(ARCH) -shared -shared-libasan -Xarch_host -fsanitize=address \
		-Xarch_host -fsanitize=undefined -o $@ $^ -L/opt/rocm/lib -lrccl

oracle/build/liboracle_san.so: $(ORC) oracle/shockidx_oracle.h
	@mkdir -p oracle/build
	$(SANCC) -O1 -g -fPIC -Wall -std=c11 -fsanitize=address,undefined -fno-sanitize-recover=undefined \
		-fno-omit-frame-pointer -shared-libasan -shared -o $@ $(ORC)

.PHONY: all
