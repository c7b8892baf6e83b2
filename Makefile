# Builds the HIP library (gfx950) and the CPU oracle. __graft_entry__.build() runs this.
# The frame-recursion kernels are instantiated once per terms-per-lane value
# (lt_inst.hip -DLT_P=..) so the objects compile in parallel (make -j).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall
CSRC := last_torch_amd/csrc
OBJ := build/obj
# kernel variants LG_P (LG = log2 lanes per group, M1 = runtime); keep in sync
# with LT_VARIANTS in lt_kernels.h
VARIANTS := 3_5 2_9 1_4 1_3 2_5 3_3 2_3 M1_4 M1_8 M1_16
INST_OBJS := $(foreach v,$(VARIANTS),$(OBJ)/lt_inst_$(v).o)
lg_of = $(subst M1,-1,$(word 1,$(subst _, ,$(1))))
lgn_of = $(word 1,$(subst _, ,$(1)))
p_of = $(word 2,$(subst _, ,$(1)))
LIB := last_torch_amd/liblt_lattice.so
DEPS := $(CSRC)/lt_kernels.h $(CSRC)/lt_joint.h include/lt_lattice.h

CPULIB := last_torch_amd/liblt_lattice_cpu.so
CXX ?= g++
CPUFLAGS ?= -O3 -std=c++17 -fPIC -march=x86-64-v3 -fno-math-errno -fopenmp-simd -Wall -pthread

all: $(LIB) $(CPULIB) oracle

# the host twin (include/lt_lattice_cpu.h): g++ only, no HIP
$(CPULIB): $(CSRC)/lt_cpu.cpp include/lt_lattice_cpu.h include/lt_lattice.h
	$(CXX) $(CPUFLAGS) -shared -o $@ $<

$(OBJ)/lt_inst_%.o: $(CSRC)/lt_inst.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_LG=$(call lg_of,$*) -DLT_LGN=$(call lgn_of,$*) -DLT_P=$(call p_of,$*) -c -o $@ $<

$(OBJ)/lt_lattice.o: $(CSRC)/lt_lattice.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJ)/lt_pipe.o: $(CSRC)/lt_pipe.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJ)/lt_table.o: $(CSRC)/lt_table.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJ)/lt_chunk.o: $(CSRC)/lt_chunk.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJ)/lt_tri.o: $(CSRC)/lt_tri.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJ)/lt_vit.o: $(CSRC)/lt_vit.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJ)/lt_producer.o: $(CSRC)/lt_producer.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJ)/lt_joint.o: $(CSRC)/lt_joint.hip $(DEPS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJ)/lt_lattice.o $(OBJ)/lt_pipe.o $(OBJ)/lt_chunk.o $(OBJ)/lt_table.o $(OBJ)/lt_producer.o $(OBJ)/lt_joint.o $(OBJ)/lt_vit.o $(OBJ)/lt_tri.o $(INST_OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(OBJ) $(LIB) $(CPULIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean

# Diagnostic build with in-kernel s_memtime stamps (never shipped / loaded by
# the package): build/stamps/liblt_lattice_stamps.so
STAMP_OBJ := build/stamps
$(STAMP_OBJ)/lt_inst_%.o: $(CSRC)/lt_inst.hip $(DEPS)
	@mkdir -p $(STAMP_OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_STAMPS -DLT_DIAG -DLT_LG=$(call lg_of,$*) -DLT_LGN=$(call lgn_of,$*) -DLT_P=$(call p_of,$*) -c -o $@ $<
$(STAMP_OBJ)/lt_lattice.o: $(CSRC)/lt_lattice.hip $(DEPS)
	@mkdir -p $(STAMP_OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_STAMPS -DLT_DIAG -c -o $@ $<
$(STAMP_OBJ)/lt_pipe.o: $(CSRC)/lt_pipe.hip $(DEPS)
	@mkdir -p $(STAMP_OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_STAMPS -DLT_DIAG -c -o $@ $<
$(STAMP_OBJ)/lt_joint.o: $(CSRC)/lt_joint.hip $(DEPS)
	@mkdir -p $(STAMP_OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_STAMPS -DLT_DIAG -c -o $@ $<
$(STAMP_OBJ)/lt_tri4.o: $(CSRC)/lt_tri4.hip $(DEPS)
	@mkdir -p $(STAMP_OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_STAMPS -DLT_DIAG -c -o $@ $<
$(STAMP_OBJ)/lt_tri.o: $(CSRC)/lt_tri.hip $(DEPS)
	@mkdir -p $(STAMP_OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_STAMPS -DLT_DIAG -c -o $@ $<
stamps: $(STAMP_OBJ)/lt_lattice.o $(STAMP_OBJ)/lt_pipe.o $(OBJ)/lt_chunk.o $(OBJ)/lt_table.o $(OBJ)/lt_producer.o $(STAMP_OBJ)/lt_joint.o $(OBJ)/lt_vit.o $(STAMP_OBJ)/lt_tri.o $(STAMP_OBJ)/lt_tri4.o $(foreach v,$(VARIANTS),$(STAMP_OBJ)/lt_inst_$(v).o)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $(STAMP_OBJ)/liblt_lattice_stamps.so $^
.PHONY: stamps

# Diagnostic build (role ablations behind LT_DIAG; never loaded unless
# LT_LIB_PATH points at it): build/diag/liblt_lattice_diag.so
DIAG_OBJ := build/diag
$(DIAG_OBJ)/lt_inst_%.o: $(CSRC)/lt_inst.hip $(DEPS)
	@mkdir -p $(DIAG_OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_DIAG -DLT_LG=$(call lg_of,$*) -DLT_LGN=$(call lgn_of,$*) -DLT_P=$(call p_of,$*) -c -o $@ $<
$(DIAG_OBJ)/%.o: $(CSRC)/%.hip $(DEPS)
	@mkdir -p $(DIAG_OBJ)
	$(HIPCC) $(HIPFLAGS) -DLT_DIAG -c -o $@ $<
diag: $(DIAG_OBJ)/lt_lattice.o $(DIAG_OBJ)/lt_pipe.o $(DIAG_OBJ)/lt_chunk.o $(DIAG_OBJ)/lt_table.o $(DIAG_OBJ)/lt_producer.o $(DIAG_OBJ)/lt_joint.o $(DIAG_OBJ)/lt_vit.o $(DIAG_OBJ)/lt_tri.o $(DIAG_OBJ)/lt_tri4.o $(foreach v,$(VARIANTS),$(DIAG_OBJ)/lt_inst_$(v).o)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $(DIAG_OBJ)/liblt_lattice_diag.so $^
.PHONY: diag

# Clock probe (dev tool, tools/clock_probe.py): build/libclock_probe.so
probe: build/libclock_probe.so
build/libclock_probe.so: tools/probe/clock_probe.hip
	@mkdir -p build
	$(HIPCC) --offload-arch=$(ARCH) -O3 -shared -fPIC -o $@ $<
.PHONY: probe
