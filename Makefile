# Top-level build.  `make` builds everything that ships to the GPU box:
#   xdp-tools_amd/lib/libxdpfilter_gpu.so  the product (C ABI + HIP kernels, gfx950)
#   xdp-tools_amd/bin/xdp-filter          the CLI over the C ABI
#   tools/libxfsynth.so                    synthetic traffic (tests / bench)
#   oracle/build/liboracle.so              CPU restatement (tests / bench cpu_baseline)
# `make asan` builds the host C (restatement, runtime, I/O, CLI) under ASAN +
# UBSAN for the CPU suite's sanitizer run (tools/asan_suite.sh).
JOBS ?= 8

all: product synth oracle diag

diag: product

# (one sub-make for the product and the diagnostics library: their two
# kernel objects compile in parallel, the shared host objects once)
product:
	$(MAKE) -C xdp-tools_amd -j$(JOBS) all diag

synth: tools/libxfsynth.so

tools/libxfsynth.so: tools/xfsynth.c
	gcc -O2 -fPIC -Wall -shared -o $@ $<

oracle:
	$(MAKE) -C oracle

asan: product
	$(MAKE) -C oracle asan
	$(MAKE) -C xdp-tools_amd asan
	@mkdir -p tools/build-asan
	gcc -O1 -g -fPIC -Wall -fsanitize=address,undefined -fno-omit-frame-pointer \
		-fno-sanitize-recover=undefined -shared -o tools/build-asan/libxfsynth.so tools/xfsynth.c

clean:
	$(MAKE) -C xdp-tools_amd clean
	$(MAKE) -C oracle clean
	rm -rf tools/libxfsynth.so tools/build-asan

.PHONY: all product synth oracle diag asan clean
