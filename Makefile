# Build the in-tree native libraries (gfx950 only).
#   libghm_hip.so  : HIP kernels + C ABI (include/ghm_hip.h)
#   libghm_host.so : host GHM sampler (include/ghm_sampler.h)
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
LIBDIR := multimodal-ghm_amd/ghmclip/_lib
SRC := multimodal-ghm_amd/csrc
HIPOBJFLAGS := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
HIP_SRCS := $(SRC)/ghm_genc.hip $(SRC)/ghm_fwd.hip $(SRC)/ghm_bwd.hip $(SRC)/ghm_x3.hip $(SRC)/ghm_guide.hip $(SRC)/ghm_cdm.hip $(SRC)/ghm_vlm.hip $(SRC)/ghm_gemm.hip $(SRC)/ghm_vlm_x3.hip $(SRC)/ghm_wgrad.hip $(SRC)/ghm_optim.hip $(SRC)/ghm_eval.hip
HIP_HDRS := $(SRC)/ghm_common.h $(SRC)/ghm_launch.h $(SRC)/ghm_split.h $(SRC)/ghm_ln.h include/ghm_hip.h

all: $(LIBDIR)/libghm_hip.so $(LIBDIR)/libghm_host.so

# source hash baked into both libraries (ghm_build_id / ghm_sampler_build_id;
# multimodal-ghm_amd/ghmclip/_buildid.py): the generated file changes only with it
BUILD_ID_SRC := build/obj/ghm_build_id.cpp
$(BUILD_ID_SRC): FORCE
	@python3 tools/build_id.py $@ > /dev/null
FORCE:

OBJDIR := build/obj
HIP_OBJS := $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))

# one object per translation unit (parallel, incremental), linked into one library
$(OBJDIR)/%.o: $(SRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPOBJFLAGS) -c -o $@ $<

$(OBJDIR)/ghm_build_id.o: $(BUILD_ID_SRC)
	$(CXX) -O2 -fPIC -c -o $@ $<

$(LIBDIR)/libghm_hip.so: $(HIP_OBJS) $(OBJDIR)/ghm_build_id.o
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(HIP_OBJS) $(OBJDIR)/ghm_build_id.o

$(LIBDIR)/libghm_host.so: $(SRC)/ghm_sampler.cpp include/ghm_sampler.h $(BUILD_ID_SRC)
	@mkdir -p $(LIBDIR)
	$(CXX) -O3 -std=c++17 -fPIC -shared -pthread -DGHM_HOST_LIB -o $@ $(SRC)/ghm_sampler.cpp -x c++ $(BUILD_ID_SRC)

resource-usage: $(HIP_SRCS) $(HIP_HDRS)
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Rpass-analysis=kernel-resource-usage $(SRC)/ghm_fwd.hip -o /tmp/ghm_fwd.o
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Rpass-analysis=kernel-resource-usage $(SRC)/ghm_bwd.hip -o /tmp/ghm_bwd.o
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Rpass-analysis=kernel-resource-usage $(SRC)/ghm_x3.hip -o /tmp/ghm_x3.o

clean:
	rm -f $(LIBDIR)/*.so $(OBJDIR)/*.o

.PHONY: all clean resource-usage FORCE
