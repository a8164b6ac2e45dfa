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
CPP_SRCS := config code modem layout capi simulate refstream
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
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) $(SIM)
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean

# Phase-timing build of the partitioned cooperative kernel and the fused
# k-means (s_memtime stamps, kml_debug_part_stamps / kml_debug_km_stamps);
# load it with KML_LIB=kmldpc_amd/libkmldpc_amd_stamps.so
STAMPED  := bp_coop kmeans bp_regular
STAMPS_LIB := kmldpc_amd/libkmldpc_amd_stamps.so
STAMPS_OBJS := $(addprefix $(OBJDIR)/,$(addsuffix .o,$(CPP_SRCS) $(filter-out $(STAMPED),$(HIP_SRCS)))) \
               $(addprefix $(OBJDIR)/stamps/,$(addsuffix .o,$(STAMPED)))
$(OBJDIR)/stamps/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)/stamps
	$(HIPCC) $(HIPFLAGS) -DKML_STAMPS=1 -c -o $@ $<
$(STAMPS_LIB): $(STAMPS_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(STAMPS_OBJS) -Wl,-rpath,/opt/rocm/lib
stamps: $(STAMPS_LIB)
.PHONY: stamps
