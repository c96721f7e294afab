# Builds the MI355X (gfx950) C-ABI library libensvs.so in-tree and the CPU
# oracle helper.  `make -j8` here (cross-compile, no GPU needed).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
PKG   := ensemble_svs_with_interactions_amd
SRCS  := $(wildcard $(PKG)/csrc/*.hip)
OBJS  := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(SRCS))
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
            -Wno-unused-variable -Wno-unused-but-set-variable -I$(PKG)/csrc -Iinclude

all: $(PKG)/libensvs.so

build/%.o: $(PKG)/csrc/%.hip $(wildcard $(PKG)/csrc/*.h) include/ensvs.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/libensvs.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

clean:
	rm -rf build $(PKG)/libensvs.so

.PHONY: all clean
