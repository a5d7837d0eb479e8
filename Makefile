# Builds the MI355X (gfx950) shared library behind include/sv2n.h (the
# oracle is Python and needs no build).  `python -c "import __graft_entry__ as g; g.build()"`
# runs the same recipe.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -Wall -Wno-unused-result
BUILD ?= build
# EXTRA: extra compiler flags for diagnostic A/B builds (into their own BUILD / LIB)
HIPFLAGS += $(EXTRA)
LIB ?= spotv2net_amd/libsv2n.so
ifeq ($(STAMPS),1)
HIPFLAGS += -DSV2N_STAMPS   # diagnostic phase stamps (tools/stamps.py)
endif
# diagnostic bound checks (SV2N_CHK, sv2n_check_hits): make CHECK=1 builds
# build_check/ -> spotv2net_amd/libsv2n_check.so; tests load it with
# SV2N_LIB=spotv2net_amd/libsv2n_check.so (tools/measure.sh check)
ifeq ($(CHECK),1)
HIPFLAGS += -DSV2N_CHECK
BUILD = build_check
LIB = spotv2net_amd/libsv2n_check.so
endif
SRC := $(wildcard spotv2net_amd/csrc/*.hip)
OBJ := $(patsubst spotv2net_amd/csrc/%.hip,$(BUILD)/%.o,$(SRC))

all: $(LIB)

$(BUILD)/%.o: spotv2net_amd/csrc/%.hip $(wildcard spotv2net_amd/csrc/*.h) include/sv2n.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJ)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
