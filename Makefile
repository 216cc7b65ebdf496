# Top-level build.  `make` builds everything that ships to the GPU box:
#   xdp-tools_amd/lib/libxdpfilter_gpu.so  the product (C ABI + HIP kernels, gfx950)
#   xdp-tools_amd/bin/xdp-filter          the CLI over the C ABI
#   tools/libxfsynth.so                    synthetic traffic (tests / bench)
#   oracle/build/liboracle.so              CPU restatement (tests / bench cpu_baseline)
# `make ref` additionally builds oracle/_ref/ from /root/reference (container only).
JOBS ?= 8

all: product synth oracle diag

diag:
	$(MAKE) -C xdp-tools_amd diag

product:
	$(MAKE) -C xdp-tools_amd -j$(JOBS)

synth: tools/libxfsynth.so

tools/libxfsynth.so: tools/xfsynth.c
	gcc -O2 -fPIC -Wall -shared -o $@ $<

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

clean:
	$(MAKE) -C xdp-tools_amd clean
	$(MAKE) -C oracle clean
	rm -f tools/libxfsynth.so

.PHONY: all product synth oracle ref diag clean
