# Build libmaeclip.so (gfx950 only) and the C oracle helpers.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -munsafe-fp-atomics -Wall -Wno-unused-function
SRC := $(wildcard mae_clip_amd/csrc/*.hip)
OBJ := $(patsubst mae_clip_amd/csrc/%.hip,build/obj/%.o,$(SRC))
LIB := mae_clip_amd/libmaeclip.so

all: $(LIB)

build/obj/%.o: mae_clip_amd/csrc/%.hip mae_clip_amd/csrc/common.h include/maeclip.h
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean
