# Build recipe for the MI355X `path` integrator (no cmake needed).
#   make            -> host scene library, GPU library (gfx950), CLI, oracle
#   make device     -> my-mitsuba_amd/libmtsg.so only (hipcc --offload-arch=gfx950)
# Outputs are in-tree .so files (git-ignored, shipped to the GPU box by gpurun).

HIPCC   ?= /opt/rocm/bin/hipcc
CXX     ?= g++
PKG     := my-mitsuba_amd
ARCH    ?= gfx950
JOBS    ?= 8

HOST_SRC := $(wildcard $(PKG)/host/*.cpp)
HOST_HDR := $(wildcard $(PKG)/host/*.h) $(PKG)/host/ior_table.inc include/mtsg.h include/mtsh.h
DEV_SRC  := $(PKG)/csrc/mtsg.hip $(PKG)/csrc/smp_kernels.hip $(PKG)/csrc/kdbuild.hip
DEV_HDR  := $(wildcard $(PKG)/csrc/*.h) include/mtsg.h

HOST_LIB := $(PKG)/libmtsg_host.so
DEV_LIB  := $(PKG)/libmtsg.so
PATH_LIB := $(PKG)/libmtsg_path.so
CLI      := $(PKG)/mtsg-render

ORACLE      := oracle/liboracle.so
ORACLE_FAST := oracle/liboracle_fast.so

.PHONY: all host device oracle clean
all: host device oracle $(PATH_LIB) $(CLI) scenes/sky512.pfm tools/math_probe tools/math_bench tools/div_probe tools/check_glibc_mathf tools/check_env_guide
host: $(HOST_LIB)
device: $(DEV_LIB)
oracle: $(ORACLE) $(ORACLE_FAST)

SOBOL_BIN := $(PKG)/data/sobol_tables.bin
$(HOST_LIB): $(HOST_SRC) $(HOST_HDR) $(SOBOL_BIN)
	$(CXX) -std=c++17 -O2 -g -fPIC -shared -Wall -DMTSH_SOBOL_BIN='"$(SOBOL_BIN)"' -o $@ $(HOST_SRC) -lz -lpthread

# gfx950 only: no dual CUDA/HIP paths, no hipify output.
# -ffp-contract=off: no FMA contraction, like Mitsuba's SSE2 build
# (build/config-linux-gcc.py:7); long specular paths otherwise diverge from
# the oracle through ulp-level differences (measured: C5 parity 2.0e-3 ->
# 1.8e-4 relative L1), at no measured cost (C3 1262 vs 1256 Msamples/s).
# The device library is six translation units built in parallel: mtsg.hip
# (host side, traversal, camera, splat) and smp_kernels.hip once per sampler
# (k_shade / k_finish of MTSG_SAMPLER_* = 0..4; unit 0 also answers the
# k_finish occupancy query).  DEV_EXTRA / DEV_OBJ: measurement variants.
# -fno-slp-vectorize: no v_pk_* float pairs; the traversal then needs fewer
# register moves and VGPRs (63 -> 60 flat, 80 -> 76 two-level): C3 +1.8%,
# two-level +1.2% (r03 variant noslp), results unchanged (same IEEE ops).
DEV_FLAGS := -O3 -std=c++17 -fPIC -Wall -ffp-contract=off -fno-slp-vectorize -munsafe-fp-atomics -Wno-unused-value -Wno-unused-result
# the flat traversal's own unit (trace_flat.hip): the memory-clause scheduler
# groups each iteration's node-pair and TriAccel loads (C3 trace -1.0%, C5
# -0.6%; the two-level kernel in mtsg.hip loses 3% under it: DESIGN §3)
DEV_FLAT_FLAGS ?= -mllvm -amdgpu-sched-strategy=max-memory-clause
DEV_OBJ   ?= build/dev
DEV_OBJS  := $(DEV_OBJ)/mtsg.o $(DEV_OBJ)/trace_flat.o $(DEV_OBJ)/kdbuild.o $(foreach k,0 1 2 3 4,$(DEV_OBJ)/smp_$(k).o)
$(DEV_OBJ)/mtsg.o: $(PKG)/csrc/mtsg.hip $(DEV_HDR)
	@mkdir -p $(DEV_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) $(DEV_FLAGS) $(DEV_EXTRA) -c -o $@ $<
$(DEV_OBJ)/trace_flat.o: $(PKG)/csrc/trace_flat.hip $(DEV_HDR)
	@mkdir -p $(DEV_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) $(DEV_FLAGS) $(DEV_FLAT_FLAGS) $(DEV_EXTRA) -c -o $@ $<
$(DEV_OBJ)/kdbuild.o: $(PKG)/csrc/kdbuild.hip include/mtsg.h
	@mkdir -p $(DEV_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) $(DEV_FLAGS) $(DEV_EXTRA) -c -o $@ $<
$(DEV_OBJ)/smp_%.o: $(PKG)/csrc/smp_kernels.hip $(DEV_HDR)
	@mkdir -p $(DEV_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) $(DEV_FLAGS) $(DEV_EXTRA) -DMTSG_TU_SAMPLER=$* $(if $(filter 0,$*),-DMTSG_TU_OCCUPANCY) -c -o $@ $<
$(DEV_LIB): $(DEV_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(DEV_OBJS)

# Host-side `path` integrator plugin mirror: tiles the film over GPUs
$(PATH_LIB): $(PKG)/host/path_integrator.cc $(HOST_LIB) $(DEV_LIB) include/mtsg.h include/mtsh.h include/mtsg_path.h
	$(CXX) -std=c++17 -O2 -fPIC -shared -Wall -o $@ $(PKG)/host/path_integrator.cc \
	    -L$(PKG) -lmtsg_host -lmtsg -Wl,-rpath,'$$ORIGIN' -lpthread

$(CLI): $(PKG)/host/mtsg_render_main.cc $(PATH_LIB)
	$(CXX) -std=c++17 -O2 -Wall -o $@ $(PKG)/host/mtsg_render_main.cc \
	    -L$(PKG) -lmtsg_path -lmtsg_host -lmtsg -Wl,-rpath,'$$ORIGIN' -lpthread

# Oracle (TEST INFRASTRUCTURE): precise build for parity ...
$(ORACLE): oracle/oracle.cpp oracle/oracle.h include/mtsg.h
	$(CXX) -std=c++17 -O2 -fPIC -shared -ffp-contract=off -o $@ oracle/oracle.cpp -lpthread
# ... and the reference's own compiler flags (build/config-linux-gcc.py:7)
# for the timed CPU baseline.
$(ORACLE_FAST): oracle/oracle.cpp oracle/oracle.h include/mtsg.h
	$(CXX) -std=c++17 -O3 -msse2 -march=nocona -funsafe-math-optimizations -fPIC -shared \
	    -o $@ oracle/oracle.cpp -lpthread

# glibc_mathf.h (the device's glibc float transcendentals) against libm: on
# the GPU (math_probe) and on the host (check_glibc_mathf)
tools/math_probe: tools/math_probe.hip $(PKG)/csrc/glibc_mathf.h
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -ffp-contract=off -o $@ $< -lpthread
# fast reciprocal / division sequences against the IEEE division, on the GPU
tools/div_probe: tools/div_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off -Wno-unused-result -o $@ $<
tools/math_bench: tools/math_bench.hip $(PKG)/csrc/glibc_mathf.h
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -ffp-contract=off -Wno-unused-result -o $@ $<
tools/check_glibc_mathf: tools/check_glibc_mathf.cpp $(PKG)/csrc/glibc_mathf.h
	$(HIPCC) -O2 -mfma -std=c++17 -ffp-contract=off -o $@ $< -lpthread

# the device's guided envmap CDF searches against std::lower_bound, on the host
tools/check_env_guide: tools/check_env_guide.cpp $(PKG)/csrc/envmap.h $(HOST_LIB)
	$(HIPCC) -O2 -std=c++17 -ffp-contract=off -Iinclude -o $@ $< -L$(PKG) -lmtsg_host -Wl,-rpath,'$$ORIGIN/../$(PKG)'

# synthetic HDR environment for the envmap scenes (tools/gen_envmap.py)
scenes/sky512.pfm: tools/gen_envmap.py
	python3 tools/gen_envmap.py $@ 512 256

clean:
	rm -f $(HOST_LIB) $(DEV_LIB) $(PATH_LIB) $(CLI) $(ORACLE) $(ORACLE_FAST)

# Measurement variants of the device library (my-mitsuba_amd/var/, loaded with
# MTSG_LIB=...; objects in build/var/, which gpurun does not ship)
VARIANTS := sg64:-DMTSG_SHADE_WG_PER_CU=64 sg128:-DMTSG_SHADE_WG_PER_CU=128 sg512:-DMTSG_SHADE_WG_PER_CU=512 sg32:-DMTSG_SHADE_WG_PER_CU=32 sb512:-DMTSG_SHADE_BLOCK=512 popsel:-DMTSG_POPSEL=1 eb0:-DMTSG_ENTER_BATCH=0 eb4:-DMTSG_ENTER_BATCH=4 eb16:-DMTSG_ENTER_BATCH=16 shocc3:-DMTSG_SHADE_LDS_PAD=2048 ii32:-DMTSG_INST_MIN_IDLE=32 ii24:-DMTSG_INST_MIN_IDLE=24 eb8x8:-DMTSG_EXIT_BATCH=8 iw7s5:-DMTSG_INST_WAVES=7@-DMTSG_INNER_STACK=5 ss7:-DMTSG_INST_REGSAVE=0@-DMTSG_INNER_STACK=5 ss8:-DMTSG_INST_REGSAVE=0@-DMTSG_INST_WAVES=8@-DMTSG_INNER_STACK=4@-DMTSG_SAVE_INV=0 occ7:-DMTSG_LDS_PAD=1024 occ6:-DMTSG_LDS_PAD=1792 powout:-DGMF_CALLS=45 fm16:-DMTSG_FETCH_MIN=16 fm64:-DMTSG_FETCH_MIN=64 gs1:-DMTSG_GUIDE_SPLIT=1 gs4:-DMTSG_GUIDE_SPLIT=4 noguide:-DMTSG_FETCH_MIN=256 wt:-DMTSG_WT_DRAIN=1 ss5:-DMTSG_SHORT_STACK=5 ldstop:-DMTSG_LDS_TOP=1 noguard:-DMTSG_RST_GUARD=0 iw7:-DMTSG_INST_WAVES=7 gs5:-DMTSG_INNER_STACK=5 noshlds:-DMTSG_SHADE_LDS=0 nosave:-DMTSG_SAVE_RAY=0 soct:-DMTSG_SORT_OCT=1 nomb:-DMTSG_MAILBOX=0 sinv:-DMTSG_SAVE_INV=1 silp:-mllvm@-amdgpu-sched-strategy=max-ilp smem:-mllvm@-amdgpu-sched-strategy=max-memory-clause ocmlmath:-DMTSG_GLIBC_MATH=0 call31:-DGMF_CALLS=31 call14:-DGMF_CALLS=14 call12:-DGMF_CALLS=12 call13:-DGMF_CALLS=13 slotsave:-DMTSG_INST_REGSAVE=0 pre0:-DMTSG_SHADE_PRELOAD=0 pre2:-DMTSG_SHADE_PRELOAD=2 rpend:-DMTSG_RECT_PEND=1 envfull:-DMTSG_ENV_GUIDE=0 fw3:-DMTSG_FINISH_WAVES=3 call0:-DGMF_CALLS=0 pre1:-DMTSG_SHADE_PRELOAD=1 pd:-DMTSG_PUSHDOWN=1 sc16:-DMTSG_SPLAT_CHUNK=16 shenv4:-DMTSG_SHADE_WAVES_MATS_ENV=4 tie1:-DMTSG_TIE_INLINE=1 shuf1:-DMTSG_SHUFFLE=1 shuf2:-DMTSG_SHUFFLE=2 sw16k:-DMTSG_SORT_WINDOW=16384 sw1k:-DMTSG_SORT_WINDOW=1024 sb3:-DMTSG_SORT_BINS_LOG=3 sb5:-DMTSG_SORT_BINS_LOG=5 ssort0:-DMTSG_SHADE_SORT=0 trow:-DMTSG_TILE_MORTON=0 nopf:-DMTSG_INST_PREFILTER=0 sg256:-DMTSG_SHADE_WG_PER_CU=256 finm0:-DMTSG_FINISH_MATS=0 finm3:-DMTSG_FINISH_WAVES_MATS=3
VAR_LIBS := $(foreach v,$(VARIANTS),$(PKG)/var/libmtsg_$(word 1,$(subst :, ,$(v))).so)
.PHONY: variants
variants: $(VAR_LIBS)
$(PKG)/var/libmtsg_%.so: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(PKG)/var
	$(MAKE) DEV_OBJ=build/var/$* DEV_LIB=$@ DEV_EXTRA="$(subst @, ,$(word 2,$(subst :, ,$(filter $*:%,$(VARIANTS)))))" $@
