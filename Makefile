# Builds the gfx950 HIP library behind the C ABI in include/binquant_amd.h.
# The .so is written in-tree (binquant_amd/lib/) so it travels to the GPU box.
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
HIPFLAGS  ?= -O3 --offload-arch=$(ARCH) -ffp-contract=off -fPIC -std=c++17 \
             -Iinclude -Ibinquant_amd/csrc -Wall -Wno-unused-function
SRCS      := $(wildcard binquant_amd/csrc/*.hip)
CXXSRCS   := $(wildcard binquant_amd/csrc/*.cpp)
OBJS      := $(patsubst binquant_amd/csrc/%.hip,build/%.o,$(SRCS)) \
             $(patsubst binquant_amd/csrc/%.cpp,build/%.o,$(CXXSRCS))
CXX       ?= g++
CXXFLAGS  ?= -O3 -fPIC -std=c++17 -Iinclude -Wall
LIB       := binquant_amd/lib/libbinquant_amd.so

all: $(LIB)

build/%.o: binquant_amd/csrc/%.hip $(wildcard binquant_amd/csrc/*.h) include/binquant_amd.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host-only sources (wire-format ingest)
build/%.o: binquant_amd/csrc/%.cpp include/binquant_amd.h
	@mkdir -p build
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p binquant_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lhiprtc

resource-usage: $(SRCS)
	@for f in $(SRCS); do $(HIPCC) $(HIPFLAGS) -c $$f -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "remark" ; done

clean:
	rm -rf build $(LIB)

.PHONY: all clean resource-usage
