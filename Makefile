# Top-level build: the product library (gfx950 HIP) and the test oracle.
#
#   make            -> kmldpc_amd/libkmldpc_amd.so, kmldpc_amd/bin/kmldpc_sim, oracle/*
#   make lib        -> product library + the kmldpc_sim driver executable
#   make oracle     -> oracle/liboracle.so, oracle/cpu_baseline (+ oracle/_ref when /root/reference exists)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result -Wno-unused-value
CSRC     := kmldpc_amd/csrc
OBJDIR   := build/obj
CPP_SRCS := config code modem layout capi simulate refstream comm
HIP_SRCS := bp bp_regular bp_irregular bp_coop demap kmeans framegen
OBJS     := $(addprefix $(OBJDIR)/,$(addsuffix .o,$(CPP_SRCS) $(HIP_SRCS)))
HDRS     := $(wildcard $(CSRC)/*.hpp) include/kmldpc_amd.h
LIB      := kmldpc_amd/libkmldpc_amd.so
SIM      := kmldpc_amd/bin/kmldpc_sim

all: lib oracle

lib: $(LIB) $(SIM)

$(SIM): $(CSRC)/sim_main.cpp include/kmldpc_amd.h $(LIB)
	@mkdir -p kmldpc_amd/bin
	g++ -O2 -std=c++17 -Wall -o $@ $< -Lkmldpc_amd -lkmldpc_amd -Wl,-rpath,'$$ORIGIN/..'

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -ldl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) $(SIM)
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean

# Phase-timing build of the partitioned cooperative kernel and the fused
# k-means (s_memtime stamps, kml_debug_part_stamps / kml_debug_km_stamps);
# load it with KML_LIB=kmldpc_amd/libkmldpc_amd_stamps.so
STAMPED  := bp_coop kmeans bp_regular bp_irregular
STAMPS_LIB := kmldpc_amd/libkmldpc_amd_stamps.so
STAMPS_OBJS := $(addprefix $(OBJDIR)/,$(addsuffix .o,$(CPP_SRCS) $(filter-out $(STAMPED),$(HIP_SRCS)))) \
               $(addprefix $(OBJDIR)/stamps/,$(addsuffix .o,$(STAMPED)))
$(OBJDIR)/stamps/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)/stamps
	$(HIPCC) $(HIPFLAGS) -DKML_STAMPS=1 -c -o $@ $<
$(STAMPS_LIB): $(STAMPS_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(STAMPS_OBJS) -ldl -Wl,-rpath,/opt/rocm/lib
stamps: $(STAMPS_LIB)
.PHONY: stamps

# Experiment builds of the whole library with extra defines (A/B on one box):
#   make variant V=<name> VFLAGS="-DKML_IRR_VN_PAIR_MAX=5"  -> kmldpc_amd/libkmldpc_amd_<name>.so
VAR_DIR  := $(OBJDIR)/var_$(V)
VAR_OBJS := $(addprefix $(VAR_DIR)/,$(addsuffix .o,$(CPP_SRCS) $(HIP_SRCS)))
$(VAR_DIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(VAR_DIR)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c -o $@ $<
$(VAR_DIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(VAR_DIR)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c -o $@ $<
kmldpc_amd/libkmldpc_amd_$(V).so: $(VAR_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(VAR_OBJS) -ldl -Wl,-rpath,/opt/rocm/lib
variant:
	@test -n "$(V)" || (echo "variant: set V=<name>" && false)
	$(MAKE) kmldpc_amd/libkmldpc_amd_$(V).so V=$(V) VFLAGS='$(VFLAGS)'
.PHONY: variant
