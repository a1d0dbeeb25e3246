# Build of the MI355X (gfx950) Starch library + CLI.  hipcc cross-compiles
# here; the built .so/binary travel to the GPU box with the repo snapshot.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
BUILD ?= starch_amd/_build
CSRC := starch_amd/csrc
HIPSRC := $(wildcard $(CSRC)/*.hip)
CPPSRC := $(wildcard $(CSRC)/*.cpp)
OBJS := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.o,$(HIPSRC)) $(patsubst $(CSRC)/%.cpp,$(BUILD)/%.o,$(CPPSRC))
HDRS := $(wildcard $(CSRC)/*.hpp) include/starch_amd.h include/starch_bzlib.h
FLAGS := -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable --offload-arch=$(ARCH) $(EXTRA)

all: $(BUILD)/libstarch_amd.so $(BUILD)/starch3 $(BUILD)/starch3_hpp_example oracle

$(BUILD)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(FLAGS) -c $< -o $@

$(BUILD)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) -O3 -std=c++17 -fPIC -Wall -c $< -o $@

$(BUILD)/libstarch_amd.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -lpthread

$(BUILD)/starch3: tools/starch3_cli.cpp $(BUILD)/libstarch_amd.so include/starch_amd.h
	$(HIPCC) -O2 -std=c++17 -o $@ tools/starch3_cli.cpp -L$(BUILD) -lstarch_amd -Wl,-rpath,'$$ORIGIN'

$(BUILD)/starch3_hpp_example: tools/starch3_hpp_example.cpp $(BUILD)/libstarch_amd.so include/starch3_amd.hpp include/starch_amd.h
	g++ -O2 -std=c++11 -Wall -o $@ tools/starch3_hpp_example.cpp -L$(BUILD) -lstarch_amd -Wl,-rpath,'$$ORIGIN'

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD)

.PHONY: all oracle clean
