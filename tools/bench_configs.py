#!/usr/bin/env python3
"""tools/bench_configs.py — the BASELINE.json configurations beside C3
(SURVEY.md §8d), one GPU, one JSON line each:

  c2  xdpfilt_dny_ip, 1k IPv4 dst rules, 64 B frames, device-resident
  c4  xdpfilt_dny_all, IMIX 64/570/1514 (7:4:1), 1M IPv4 rules: one GPU's
      shard of the 8-GPU configuration (weak scaling: per-GPU work fixed)
  c5  xdpfilt_dny_all, 1514 B frames, 15M IPv4 + 1M IPv6 dst rules + 1024
      dst-port rules: device-resident, and end to end from host memory
      (header windows H2D, verdicts D2H, xfg_classify_host)
  c3  C3 itself at SURVEY.md §8d's 2^24 batch (bench.py times 2^26)
  c3sd  C3 with every rule src|dst (`-m src,dst`): both IPv4 lookups live,
      so a packet probes two keys (the case C3's all-dst census skips)
  c3e  C3 plus C1's 8 MAC rules (4 dst, 4 src; a ruled MAC in 10 % of the
      frames): Ethernet rules beside IP rules, the generic pipelined kernel
      with the Ethernet map as its LDS key table

  c1  xdpfilt_alw_eth, the 8 MAC rules 02:00:00:00:00:0{1..8} (4 dst, 4
      src), 64 B Ethernet/IPv4/UDP frames, 25% carrying a ruled MAC (SURVEY.md
      §8d: BASELINE.json configs[0], the reference's in-kernel CPU case): the
      GPU path, and the CPU restatement timed on the same batch on 1 thread
      and on every usable host core (SURVEY §8d CPU item 2; the in-kernel
      veth run itself needs a BPF toolchain this image lacks)

Roofline bytes per packet are min(len, 128) + 1.
Usage: python3 tools/bench_configs.py [c2] [c4] [c5] [--log2-packets N]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

HBM_PEAK_GBS = 8000.0


def run_c1(args):
    import numpy as np
    import xftools as X
    import xfgpu as G
    sys.path.insert(0, ROOT)
    import bench
    n = 1 << (args.log2_packets or 24)
    rules = X.c1_rules()
    data, lens = X.gen_c1(1, n)
    f = G.Filter(X.VARIANT_FEATURES["xdpfilt_alw_eth"], devices=[0])
    assert f.prog_name == "xdpfilt_alw_eth"
    f.load_rules(rules)
    alg = int(np.minimum(lens.astype(np.int64), 128).sum() + n)
    d_data, d_lens, d_verd = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(n)
    d_data.upload(data)
    d_lens.upload(lens)
    f.classify_timed(d_data.ptr, d_lens.ptr, n, 64, d_verd.ptr, 2)
    ms = f.classify_timed(d_data.ptr, d_lens.ptr, n, 64, d_verd.ptr, args.iters)
    path = f.last_path()
    f.close()
    if args.no_cpu:
        print(json.dumps({"config": "c1", "packets": n, "kernel_path": path,
                          "kernel_ms": round(ms, 4), "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
                          "roofline": {"frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}),
              flush=True)
        return
    # the CPU restatement on the same batch: 1 thread and every usable core
    # (a bounded sample: whole passes until ~4 s each)
    feats = X.VARIANT_FEATURES["xdpfilt_alw_eth"]
    m = min(n, 1 << 22)
    prepared = rules.prepared()
    maps = X.OracleMaps(prepared, hashed=True)

    def rate(threads, secs=4.0):
        done, t0 = 0, time.perf_counter()
        while True:
            X.run_oracle(feats, data[:m * 64], lens[:m], prepared, stride=64, maps=maps,
                         nthreads=threads)
            done += m
            el = time.perf_counter() - t0
            if el >= secs:
                return done / el / 1e6
    nt = bench.host_threads()
    r1, rn = rate(1), rate(nt)
    line = {"config": "c1", "program": "xdpfilt_alw_eth", "packets": n, "stride": 64,
            "rules_eth": 8, "kernel_path": path, "kernel_ms": round(ms, 4),
            "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "roofline": {"alg_bytes_per_launch": alg,
                         "achieved_GBps": round(alg / (ms * 1e-3) / 1e9, 1),
                         "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "cpu_restatement": {"Mpps_1thread": round(r1, 2), "Mpps_all": round(rn, 2),
                                "threads": nt, "cpu_model": bench.cpu_model(),
                                "sample": f"2^{m.bit_length() - 1} packets of the same batch, "
                                          "whole passes for ~4 s each"},
            "in_kernel_xdp": "not measured: needs a BPF-capable clang, libbpf, bpffs, "
                             "iproute2 and root, absent from this image"}
    print(json.dumps(line), flush=True)


def run(name, args):
    import numpy as np
    import xftools as X
    import xfgpu as G
    if name == "c1":
        return run_c1(args)
    kind = {"c2": 2, "c3": 3, "c4": 4, "c5": 5, "c3sd": 3, "c3e": 3}[name]
    n = 1 << (args.log2_packets or {"c2": 24, "c3": 24, "c4": 23, "c5": 23, "c3sd": 24, "c3e": 24}[name])
    stride = 64 if kind in (2, 3) else 1536
    n4 = {2: 1000, 3: 1_000_000, 4: 1_000_000, 5: 15_000_000}[kind]
    flag = 3 if name == "c3sd" else 2
    n6 = 1_000_000 if kind == 5 else 0
    nports = 1024 if kind == 5 else 16
    t0 = time.time()
    v4 = X.rand_keys(kind, int(n4 * 1.02) + 16, 4)[:n4]
    v6 = X.rand_keys(kind + 100, int(n6 * 1.02) + 16, 16)[:n6] if n6 else None
    ports = (np.arange(nports, dtype=np.uint32) * 61 + 53).astype(np.uint16)
    print(f"[{name}] keys {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    data, lens = X.gen_workload(kind, kind, n, stride, v4=v4, v6=v6, ports=ports)
    print(f"[{name}] frames {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    feats = G.FEAT_IPV4 | G.FEAT_IPV6 | G.FEAT_DENY if kind == 2 else G.FEAT_ALL | G.FEAT_DENY
    f = G.Filter(feats, devices=[0], ipv4_capacity=n4, ipv6_capacity=max(n6, 1024))
    f.update_batch(G.MAP_IPV4, v4, np.full(len(v4), flag, np.uint64))
    if n6:
        f.update_batch(G.MAP_IPV6, v6, np.full(len(v6), 2, np.uint64))
    if kind != 2:
        pk = np.array([X.port_key(int(p)) for p in ports], "<u4").view(np.uint8)
        f.update_batch(G.MAP_PORTS, pk, np.full(len(ports), 2 | 4 | 8, np.uint64))
    if name == "c3e":   # C1's MAC rules, a ruled MAC where its rule looks in 10 % of the frames
        er = X.c1_rules().prepared()
        f.update_batch(G.MAP_ETHERNET, er.eth_keys, er.eth_vals)
        rng = np.random.default_rng(9)
        d = data.reshape(n, stride)
        pick = rng.choice(n, n // 10, replace=False)
        which = rng.integers(0, len(er.eth_keys), len(pick))
        dst = (er.eth_vals[which] & 2) != 0
        d[pick[dst], 0:6] = er.eth_keys[which[dst]]
        d[pick[~dst], 6:12] = er.eth_keys[which[~dst]]
    setup_s = time.time() - t0
    print(f"[{name}] rules loaded {setup_s:.1f}s", file=sys.stderr, flush=True)
    alg = int(np.minimum(lens.astype(np.int64), 128).sum() + n)
    d_data, d_lens, d_verd = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(n)
    d_data.upload(data)
    d_lens.upload(lens)
    f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_verd.ptr, 2)
    ms = f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_verd.ptr, args.iters)
    line = {"config": name, "program": f.prog_name, "packets": n, "stride": stride,
            "kernel_path": f.last_path(),
            "rules_ipv4": n4, "rules_ipv6": n6, "port_rules": nports if kind != 2 else 0,
            "kernel_ms": round(ms, 4), "Mpps": round(n / (ms * 1e-3) / 1e6, 1),
            "roofline": {"alg_bytes_per_launch": alg,
                         "achieved_GBps": round(alg / (ms * 1e-3) / 1e9, 1),
                         "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "setup_s": round(setup_s, 1)}
    if kind == 5 and not args.no_host:
        # end to end from host memory: whole frames and lengths H2D, verdicts D2H
        f.classify_host(data, lens, stride=stride)
        t1 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            f.classify_host(data, lens, stride=stride)
        hs = (time.perf_counter() - t1) / reps
        pcie = n * (128 + 4) + n   # header windows + lengths H2D, verdicts D2H
        line["host_path"] = {"Mpps": round(n / hs / 1e6, 2), "ms": round(hs * 1e3, 2),
                             "pcie_bytes": pcie, "GBps_pcie": round(pcie / hs / 1e9, 1),
                             "frame_GBps": round(data.nbytes / hs / 1e9, 1),
                             "note": "xfg_classify_host: 128 B header windows + u32 lens H2D "
                                     "(gathered by the per-device pool), verdicts D2H; frames "
                                     "whose program leaves the window go again whole (none "
                                     "in this mix)"}
        # the same frames registered once (a capture ring / UMEM kept by the
        # caller, xfg_host_register): the kernel reads the 64 B header
        # windows of the 1536 B slots in place over PCIe (zero copy), the
        # pool gathers the lengths only
        f.host_register(data)
        f.classify_host(data, lens, stride=stride)
        t1 = time.perf_counter()
        for _ in range(reps):
            f.classify_host(data, lens, stride=stride)
        hr = (time.perf_counter() - t1) / reps
        f.host_unregister(data)
        zpcie = n * (64 + 4) + n   # windows read in place, lengths H2D, verdicts D2H
        line["host_path"].update({"registered_Mpps": round(n / hr / 1e6, 2),
                                  "registered_ms": round(hr * 1e3, 2),
                                  "registered_pcie_bytes": zpcie,
                                  "registered_GBps_pcie": round(zpcie / hr / 1e9, 1),
                                  "registered_frame_GBps": round(data.nbytes / hr / 1e9, 1)})
    f.close()
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c2", "c4", "c5", "c3sd"])
    ap.add_argument("--log2-packets", type=int, default=0)
    ap.add_argument("--no-cpu", action="store_true", help="c1: the GPU leg only")
    ap.add_argument("--no-host", action="store_true",
                    help="c5: the device-resident leg only (PMC passes of its kernel)")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    for c in a.configs:
        run(c, a)


if __name__ == "__main__":
    main()
