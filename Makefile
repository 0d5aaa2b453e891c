# Builds the gfx950 HIP engine and the CPU oracle in-tree.
HIPCC ?= /opt/rocm/bin/hipcc
HIPFLAGS ?= --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wall
ENGINE := sctools_amd/libsctools_gpu.so
SRC := sctools_amd/csrc/sct_engine.hip
HDRS := $(wildcard sctools_amd/csrc/*.h) include/sctools_gpu.h

BAMDEC := sctools_amd/libsct_bam.so
CSVFMT := sctools_amd/libsct_csv.so
GBAM := sctools_amd/libsct_gbam.so

SI4 := tests/native/libsct_engine_si4.so

all: $(ENGINE) $(BAMDEC) $(CSVFMT) $(GBAM) oracle/liboracle.so tests/native/libfxcheck.so $(SI4)

$(ENGINE): $(SRC) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -o $@ $(SRC) -L/opt/rocm/lib -lrccl

# test infrastructure: the engine with 1024-item radix tiles (tests/test_gpu_tagsort.py)
$(SI4): $(SRC) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DSCT_SORT_ITEMS=4 -o $@ $(SRC) -L/opt/rocm/lib -lrccl

$(BAMDEC): sctools_amd/csrc/bamdec.cpp sctools_amd/csrc/bamsplit.cpp sctools_amd/csrc/bgzf.h include/sct_bam.h
	g++ -O3 -std=c++17 -fopenmp -fPIC -shared -Wall -o $@ sctools_amd/csrc/bamdec.cpp sctools_amd/csrc/bamsplit.cpp -lz

$(GBAM): sctools_amd/csrc/gbam.hip sctools_amd/csrc/inflate.h sctools_amd/csrc/bgzf.h include/sct_gbam.h include/sct_bam.h
	$(HIPCC) $(HIPFLAGS) -o $@ sctools_amd/csrc/gbam.hip -lz

$(CSVFMT): sctools_amd/csrc/csvfmt.cpp include/sct_csv.h
	g++ -O3 -std=c++17 -fopenmp -fPIC -shared -Wall -o $@ sctools_amd/csrc/csvfmt.cpp -lz

oracle/liboracle.so: oracle/sct_oracle.c include/sctools_gpu.h
	$(MAKE) -s -C oracle liboracle.so

tests/native/libfxcheck.so: tests/native/fxcheck.cpp sctools_amd/csrc/fixedpt.h
	g++ -O2 -std=c++17 -ffp-contract=off -fPIC -shared -o $@ tests/native/fxcheck.cpp

clean:
	rm -f $(ENGINE) $(BAMDEC) $(CSVFMT) $(GBAM) oracle/liboracle.so tests/native/libfxcheck.so $(SI4)

.PHONY: all clean
