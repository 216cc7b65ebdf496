"""Worker of tests/test_gpu_io.py::test_classify_host_registered_hybrid (a
fresh process on the diagnostics library, XFG_LIB=diag, with XFG_HYB_ZLOG2 /
XFG_HYB_ST in the environment so that a batch of a few hundred thousand
frames already takes several rounds of the hybrid host path: a zero-copy
chunk, then staged chunks of header windows): registered 1536-byte slots
of the structured fuzz corpus (IPv6 extension chains that leave the
128-byte window go again whole) -- verdicts, every rule value and the stats
equal the restatement's.  Usage: python gpu_hyb_worker.py; prints OK."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import numpy as np  # noqa: E402


def main():
    import xftools as X
    import xfgpu as G
    stride = 1536
    n = (1 << 19) + 12345
    rules, pool = X.random_rules(511, n4=600, n6=300, ne=0, nports=40)
    data, lens = X.gen_fuzz(512, n, stride, rules, pool)
    for variant in ("xdpfilt_dny_all", "xdpfilt_alw_ip"):
        feats = X.VARIANT_FEATURES[variant]
        ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=stride, nthreads=8)
        f = G.Filter(feats, devices=[0])
        f.load_rules(rules)
        f.host_register(data)
        try:
            v = f.classify_host(data, lens, stride=stride)
        finally:
            f.host_unregister(data)
        np.testing.assert_array_equal(v, ov)
        np.testing.assert_array_equal(f.stats(), ost)
        r = rules.prepared()
        np.testing.assert_array_equal(f.values_of(G.MAP_IPV4, r.v4_keys), orules.v4_vals)
        np.testing.assert_array_equal(f.values_of(G.MAP_IPV6, r.v6_keys), orules.v6_vals)
        np.testing.assert_array_equal(f.values_of(G.MAP_PORTS, np.arange(65536, dtype=np.uint32)),
                                      orules.ports)
        f.close()
    print("OK")


if __name__ == "__main__":
    main()
