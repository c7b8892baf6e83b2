# Builds the HIP library (gfx950) and the CPU oracle. __graft_entry__.build() runs this.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -shared --offload-arch=$(ARCH) -Wall
LIB := last_torch_amd/liblt_lattice.so

all: $(LIB) oracle

$(LIB): last_torch_amd/csrc/lt_lattice.hip include/lt_lattice.h
	$(HIPCC) $(HIPFLAGS) -o $@ $<

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -f $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
