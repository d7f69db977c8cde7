# Build of the MI355X BFS engine.  Everything compiles for gfx950 only.
#   libbfsx.so   : C-ABI (include/bfsx.h) + HIP kernels   -> bfs-with-mapreduce_amd/libbfsx.so
#   libbfsx_diag.so : the same with the test hooks (-DBFSX_DIAG) -> bfs-with-mapreduce_amd/libbfsx_diag.so
#   bfsx_spark   : C++ host twin of BfsSpark.main          -> bfs-with-mapreduce_amd/bfsx_spark
#   liboracle.so : CPU oracle (test infrastructure only)   -> oracle/liboracle.so
#   fetch_calib  : FETCH_SIZE / WRITE_SIZE calibration      -> tools/fetch_calib (profiling aid)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := bfs-with-mapreduce_amd
CSRC     := $(PKG)/csrc
HOSTSRC  := $(PKG)/host
OBJDIR   := $(PKG)/build
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result -I include
CXXFLAGS ?= -O2 -std=c++17 -Wall -I include

# the BFS kernel families (bfs_core.h): push, pull, persistent (K3p), the single-device loop, the partitioned loop
BFS_SRCS    := $(CSRC)/kernels_push.hip $(CSRC)/kernels_pull.hip $(CSRC)/kernels_persist.hip $(CSRC)/kernels_level.hip \
               $(CSRC)/kernels_dist.hip
KERNEL_SRCS := $(CSRC)/kernels_build.hip $(BFS_SRCS) $(CSRC)/kernels_parse.hip $(CSRC)/kernels_validate.hip
HOST_SRCS   := $(CSRC)/bfsx_api.cpp $(CSRC)/bfsx_comm.cpp
# every header a translation unit may include: an edit to any of them rebuilds the objects
HDRS := $(CSRC)/bfs_core.h $(CSRC)/bfsx_internal.h $(CSRC)/java_digits.h $(CSRC)/exchange_plan.h include/bfsx.h include/bfsx_levels.h
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(KERNEL_SRCS)) $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(HOST_SRCS))
# the diagnostic library: the same sources with the test hooks and the encoded hub domain (-DBFSX_DIAG)
DIAGDIR  := $(PKG)/build_diag
DIAGOBJS := $(patsubst $(CSRC)/%.hip,$(DIAGDIR)/%.o,$(KERNEL_SRCS)) $(patsubst $(CSRC)/%.cpp,$(DIAGDIR)/%.o,$(HOST_SRCS))

all: $(PKG)/libbfsx.so $(PKG)/libbfsx_diag.so $(PKG)/bfsx_spark tools/fetch_calib oracle

tools/fetch_calib: tools/fetch_calib.hip
	$(HIPCC) -O3 --offload-arch=$(ARCH) -o $@ $<

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/libbfsx.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

$(DIAGDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(DIAGDIR)
	$(HIPCC) $(HIPFLAGS) -DBFSX_DIAG -c $< -o $@

$(DIAGDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(DIAGDIR)
	$(HIPCC) $(HIPFLAGS) -DBFSX_DIAG -c $< -o $@

$(PKG)/libbfsx_diag.so: $(DIAGOBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(DIAGOBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

$(PKG)/bfsx_spark: $(HOSTSRC)/bfsx_spark.cpp include/bfsx.h $(PKG)/libbfsx.so
	$(CXX) $(CXXFLAGS) -o $@ $(HOSTSRC)/bfsx_spark.cpp -L$(PKG) -lbfsx -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(OBJDIR) $(DIAGDIR) $(PKG)/libbfsx.so $(PKG)/libbfsx_diag.so $(PKG)/bfsx_spark tools/fetch_calib
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
