# Build the in-tree native libraries (gfx950 only).
#   libghm_hip.so  : HIP kernels + C ABI (include/ghm_hip.h)
#   libghm_host.so : host GHM sampler (include/ghm_sampler.h)
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
LIBDIR := multimodal-ghm_amd/ghmclip/_lib
SRC := multimodal-ghm_amd/csrc
HIPOBJFLAGS := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
HIP_SRCS := $(SRC)/ghm_fwd.hip $(SRC)/ghm_bwd.hip $(SRC)/ghm_x3.hip $(SRC)/ghm_guide.hip $(SRC)/ghm_cdm.hip $(SRC)/ghm_vlm.hip $(SRC)/ghm_gemm.hip $(SRC)/ghm_vlm_x3.hip $(SRC)/ghm_optim.hip $(SRC)/ghm_eval.hip
HIP_HDRS := $(SRC)/ghm_common.h $(SRC)/ghm_launch.h $(SRC)/ghm_split.h $(SRC)/ghm_ln.h include/ghm_hip.h

all: $(LIBDIR)/libghm_hip.so $(LIBDIR)/libghm_host.so

OBJDIR := build/obj
HIP_OBJS := $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))

# one object per translation unit (parallel, incremental), linked into one library
$(OBJDIR)/%.o: $(SRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPOBJFLAGS) -c -o $@ $<

$(LIBDIR)/libghm_hip.so: $(HIP_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(HIP_OBJS)

$(LIBDIR)/libghm_host.so: $(SRC)/ghm_sampler.cpp include/ghm_sampler.h
	@mkdir -p $(LIBDIR)
	$(CXX) -O3 -std=c++17 -fPIC -shared -pthread -o $@ $(SRC)/ghm_sampler.cpp

resource-usage: $(HIP_SRCS) $(HIP_HDRS)
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Rpass-analysis=kernel-resource-usage $(SRC)/ghm_fwd.hip -o /tmp/ghm_fwd.o
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Rpass-analysis=kernel-resource-usage $(SRC)/ghm_bwd.hip -o /tmp/ghm_bwd.o
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Rpass-analysis=kernel-resource-usage $(SRC)/ghm_x3.hip -o /tmp/ghm_x3.o

clean:
	rm -f $(LIBDIR)/*.so $(OBJDIR)/*.o

.PHONY: all clean resource-usage
