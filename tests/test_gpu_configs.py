"""GPU parity at the BASELINE.json configurations themselves:
the HIP path against the CPU restatement (oracle/) on the exact rule sets,
capacities, strides and frame mixes the bench and DESIGN.md quote.
Bit-exact: verdicts, every rule's value (hits << 6 | flags) and the
per-action stats.  Contract: xdp-filter/xdpfilt_prog.h:56-64,214-310.

  C1  xdpfilt_alw_eth, the 8 MAC rules 02:00:00:00:00:0{1..8} (4 dst, 4
      src), 64 B frames, 25% carrying a ruled MAC, 2^22 packets
  C2  xdpfilt_dny_ip, 1,000 IPv4 dst rules, ipv4_capacity=1000 (the direct
      LDS counter path, kargs.dcnt), 64 B dense frames, 2^22 packets
  C3  xdpfilt_dny_all, 1M IPv4 dst rules at capacity 1M + 16 dst-port rules,
      64 B frames, 2^22 packets (the quotient-index kernel, hit log)
  C4  xdpfilt_dny_all, IMIX 64/570/1514 at a 1536 B stride, 1M IPv4 rules
  C5  xdpfilt_dny_all, 15M IPv4 + 1M IPv6 dst rules + 1024 dst-port rules,
      1514 B frames at a 1536 B stride, 2^18 packets, device-resident (the
      quotient-index kernel) and through xfg_classify_host
"""
import numpy as np
import pytest

import xftools as X
from test_gpu import assert_same, gpu_values, make_filter

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G():
    import xfgpu
    return xfgpu


def config_rules(kind, n4, n6, nports, port_rules=True):
    """The bench's rule set for configuration C<kind> (tools/bench_configs.py,
    bench.py setup): dst-flagged IPv4/IPv6 keys, dst|tcp|udp ports."""
    v4 = X.rand_keys(kind, int(n4 * 1.02) + 16, 4)[:n4]
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64)
    v6 = None
    if n6:
        v6 = X.rand_keys(kind + 100, int(n6 * 1.02) + 16, 16)[:n6]
        rules.v6_keys = v6
        rules.v6_vals = np.full(len(v6), 2, np.uint64)
    ports = (np.arange(nports, dtype=np.uint32) * 61 + 53).astype(np.uint16)
    if port_rules:
        for p in ports:
            rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    return rules, v4, v6, ports


def check(G, variant, rules, data, lens, stride, host=False, path=None, **caps):
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, rules,
                                   stride=stride, nthreads=8)
    f = make_filter(G, variant, **caps)
    f.load_rules(rules)
    v = f.run(data, lens, stride=stride)
    if path is not None:
        assert f.last_path() == path
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()
    if host:
        f = make_filter(G, variant, **caps)
        f.load_rules(rules)
        vh = f.classify_host(data, lens, stride=stride)
        assert_same(vh, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
        f.close()
    return ov


@pytest.mark.timeout(300)
def test_c1_alw_eth_8_mac_rules(G):
    rules = X.c1_rules()
    data, lens = X.gen_c1(1, 1 << 22)
    ov = check(G, "xdpfilt_alw_eth", rules, data, lens, 64, path=6)
    # a quarter of the frames carry a ruled MAC where its rule tests it: DROP
    # under allow mode (xdpfilt_prog.h:187-196)
    assert abs(int((ov == 1).sum()) - (1 << 20)) < (1 << 14)


@pytest.mark.timeout(300)
def test_c2_dny_ip_1k_rules_direct_counters(G):
    rules, v4, _, ports = config_rules(2, 1000, 0, 16, port_rules=False)
    data, lens = X.gen_workload(2, 2, 1 << 22, 64, v4=v4, ports=ports)
    ov = check(G, "xdpfilt_dny_ip", rules, data, lens, 64, ipv4_capacity=1000)
    assert (ov == 1).sum() > (1 << 20)   # half the frames carry a ruled dst


@pytest.mark.timeout(300)
def test_c3_full_1m_rule_table(G):
    rules, v4, _, _ = config_rules(3, 1_000_000, 0, 16, port_rules=False)
    # bench.py's port rules: 16 dst ports 53 + 1031k
    ports = (np.arange(16, dtype=np.uint16) * 1031 + 53).astype(np.uint16)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    data, lens = X.gen_workload(3, 3, 1 << 22, 64, v4=v4, ports=ports, dst_permille=500,
                                port_permille=250, bad_permille=10)
    check(G, "xdpfilt_dny_all", rules, data, lens, 64, ipv4_capacity=1_000_000)


@pytest.mark.timeout(300)
def test_c4_imix_1536_stride(G):
    rules, v4, _, ports = config_rules(4, 1_000_000, 0, 16)
    data, lens = X.gen_workload(4, 4, 1 << 20, 1536, v4=v4, ports=ports)
    assert len(np.unique(lens)) >= 3   # the IMIX sizes
    check(G, "xdpfilt_dny_all", rules, data, lens, 1536, ipv4_capacity=1_000_000)


@pytest.mark.timeout(600)
def test_c5_16m_rules_1514b_device_and_host(G):
    rules, v4, v6, ports = config_rules(5, 15_000_000, 1_000_000, 1024)
    data, lens = X.gen_workload(5, 5, 1 << 18, 1536, v4=v4, v6=v6, ports=ports)
    # (the quotient index of 2^21 buckets -- more slots than packets here, so
    # its hits count through the LDS cache and atomics, no hit log -- with
    # the IPv6 lookups in its loop, V6P: one line read per IPv6 frame)
    check(G, "xdpfilt_dny_all", rules, data, lens, 1536, host=True, path=5,
          ipv4_capacity=15_000_000, ipv6_capacity=1_000_000)
