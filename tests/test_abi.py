"""CPU tests of the C ABI (include/xdpfilter_gpu.h) — no GPU needed.

The library must load, export every symbol the header declares, select
programs exactly like find_prog_file() (xdp-filter/xdp-filter.c:48-60), and
implement the BPF map semantics the CLI relies on
(xdp-filter/xdp-filter.c:73-157): per-device values, -ENOENT / -E2BIG,
array vs hash maps, get_next_key iteration.  A host-only context (ndev=0)
exercises the host tables without a device.
"""
import errno
import os
import re

import numpy as np
import pytest

import xfgpu as G
import xftools as X

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("header,listed", [("xdpfilter_gpu.h", "EXPORTS"),
                                           ("xdpfilter_io.h", "IO_EXPORTS")])
def test_library_exports_every_declared_symbol(header, listed):
    hdr = open(os.path.join(ROOT, "include", header)).read()
    declared = set(re.findall(r"\b(xfg_[a-z0-9_]+)\s*\(", hdr))
    assert declared, "no declarations parsed"
    missing = [s for s in sorted(declared) if not hasattr(G.lib, s)]
    assert not missing, f"not exported: {missing}"
    assert set(getattr(G, listed)) <= declared
    assert declared <= set(G.EXPORTS) | set(G.IO_EXPORTS)


@pytest.mark.parametrize("sel", ["/nonexistent/libxdpfilter_gpu.so", "product"])
def test_a_library_selection_that_names_nothing_fails_loudly(sel):
    """XFG_LIB naming a missing file or an unknown build is an error, never the
    product library loaded in its place."""
    import subprocess
    import sys
    pydir = os.path.dirname(G.__file__)
    r = subprocess.run([sys.executable, "-c", "import xfgpu"], cwd=pydir, capture_output=True,
                       text=True, env=dict(os.environ, XFG_LIB=sel), timeout=120)
    assert r.returncode != 0 and "XFG_LIB" in r.stderr


def test_native_library_is_the_in_tree_build():
    assert os.path.realpath(G.LIB_PATH).startswith(os.path.realpath(ROOT))
    with open("/proc/self/maps") as f:
        assert any("libxdpfilter_gpu.so" in line for line in f)


def _reference_select(features):
    """find_prog_file() over the xdp-filter/Makefile:3-6 order."""
    if not features:
        return None
    for name, feats in X.VARIANTS:
        if feats & features == features:
            return name
    return None


def test_select_program_matches_find_prog_file():
    for feats in range(0, 128):
        want = _reference_select(feats)
        if want is None:
            with pytest.raises(OSError):
                G.select_program(feats)
        else:
            assert G.select_program(feats) == (want, X.VARIANT_FEATURES[want])


def test_select_program_documented_cases():
    # xdp-filter/tests/test-xdp-filter.sh:28-54
    D = G.FEAT_DENY
    assert G.select_program(G.FEAT_TCP | D)[0] == "xdpfilt_dny_tcp"
    assert G.select_program(G.FEAT_UDP | D)[0] == "xdpfilt_dny_udp"
    assert G.select_program(G.FEAT_IPV4 | D)[0] == "xdpfilt_dny_ip"
    assert G.select_program(G.FEAT_IPV6 | D)[0] == "xdpfilt_dny_ip"
    assert G.select_program(G.FEAT_ETHERNET | D)[0] == "xdpfilt_dny_eth"
    assert G.select_program(G.FEAT_ALL | D)[0] == "xdpfilt_dny_all"
    assert G.select_program(G.FEAT_TCP | G.FEAT_UDP | G.FEAT_ALLOW)[0] == "xdpfilt_alw_all"
    with pytest.raises(OSError) as e:
        G.select_program(G.FEAT_ALLOW | G.FEAT_DENY)
    assert e.value.errno == errno.ENOENT


@pytest.fixture
def host():
    f = G.Filter(G.FEAT_ALL | G.FEAT_DENY, ndev=0, ipv4_capacity=100, ipv6_capacity=50,
                 eth_capacity=20)
    yield f
    f.close()


def test_open_window_option():
    """xfg_open_opts.window: 0 (64-byte windows), 64 or 128; anything else is
    -EINVAL (include/xdpfilter_gpu.h)."""
    for w in (0, 64, 128):
        G.Filter(G.FEAT_ALL | G.FEAT_DENY, ndev=0, window=w).close()
    for w in (32, 96, 256):
        with pytest.raises(OSError) as e:
            G.Filter(G.FEAT_ALL | G.FEAT_DENY, ndev=0, window=w)
        assert e.value.errno == errno.EINVAL


def test_host_context_basics(host):
    assert host.ndev == 0 and host.prog_name == "xdpfilt_dny_all"
    with pytest.raises(OSError) as e:
        host.classify(0x1000, 0x1000, 1, 64, 0x1000)   # never dereferenced
    assert e.value.errno == errno.ENODEV


def test_hash_map_crud_semantics(host):
    k = bytes([10, 0, 0, 1])
    with pytest.raises(OSError) as e:
        host.lookup(G.MAP_IPV4, k)
    assert e.value.errno == errno.ENOENT
    host.update(G.MAP_IPV4, k, (5 << 6) | 2)
    assert host.lookup(G.MAP_IPV4, k) == [(5 << 6) | 2]
    host.update(G.MAP_IPV4, k, 0xFFFFFFFFFFFFFFC3)   # full 64-bit value round-trips
    assert host.lookup(G.MAP_IPV4, k) == [0xFFFFFFFFFFFFFFC3]
    host.delete(G.MAP_IPV4, k)
    with pytest.raises(OSError):
        host.delete(G.MAP_IPV4, k)
    # zero keys are ordinary keys
    for m, kl in ((G.MAP_IPV4, 4), (G.MAP_IPV6, 16), (G.MAP_ETHERNET, 6)):
        host.update(m, bytes(kl), 1)
        assert host.lookup(m, bytes(kl)) == [1]
        assert bytes(kl) in host.keys(m)
        host.delete(m, bytes(kl))
        assert host.count(m) == 0


def test_capacity_e2big(host):
    keys = X.rand_keys(3, 100, 4)
    host.update_batch(G.MAP_IPV4, keys, np.full(len(keys), 2, np.uint64))
    assert host.count(G.MAP_IPV4) == len(keys) == 100
    with pytest.raises(OSError) as e:
        host.update(G.MAP_IPV4, bytes([1, 2, 3, 4]) if bytes([1, 2, 3, 4]) not in
                    {bytes(k) for k in keys} else bytes([4, 3, 2, 1]), 2)
    assert e.value.errno == errno.E2BIG
    # overwriting an existing key still works when full
    host.update(G.MAP_IPV4, bytes(keys[0]), 3)
    assert host.lookup(G.MAP_IPV4, bytes(keys[0])) == [3]
    # after a delete there is room again
    host.delete(G.MAP_IPV4, bytes(keys[1]))
    host.update(G.MAP_IPV4, bytes([9, 9, 9, 9]), 2)


def test_ports_are_an_array_map(host):
    assert host.lookup(G.MAP_PORTS, X.port_key(53)) == [0]    # every key exists
    host.update(G.MAP_PORTS, X.port_key(53), 2 | 8)
    assert host.lookup(G.MAP_PORTS, X.port_key(53)) == [10]
    assert host.count(G.MAP_PORTS) == 1
    with pytest.raises(OSError) as e:
        host.delete(G.MAP_PORTS, X.port_key(53))
    assert e.value.errno == errno.EINVAL
    with pytest.raises(OSError):
        host.lookup(G.MAP_PORTS, 70000)
    keys = host.keys(G.MAP_PORTS)
    assert len(keys) == 65536 and keys[0] == bytes(4)


def test_get_next_key_iterates_all_keys_once(host):
    keys = X.rand_keys(8, 40, 16)
    for k in keys:
        host.update(G.MAP_IPV6, bytes(k), 1)
    host.update(G.MAP_IPV6, bytes(16), 2)
    got = host.keys(G.MAP_IPV6)
    assert sorted(got) == sorted([bytes(k) for k in keys] + [bytes(16)])


def test_random_crud_against_dict_model():
    """Insert/overwrite/delete at high load factor with the exact-match model
    of a BPF hash map; every lookup and the key set must agree."""
    rng = np.random.default_rng(5)
    for keylen, mid in ((4, G.MAP_IPV4), (16, G.MAP_IPV6), (6, G.MAP_ETHERNET)):
        cap = 300
        f = G.Filter(G.FEAT_ALL | G.FEAT_DENY, ndev=0, ipv4_capacity=cap, ipv6_capacity=cap,
                     eth_capacity=cap)
        pool = [bytes(k) for k in X.rand_keys(keylen, 500, keylen)] + [bytes(keylen)]
        model = {}
        for step in range(4000):
            k = pool[rng.integers(len(pool))]
            op = rng.integers(3)
            if op < 2:
                v = int(rng.integers(0, 1 << 62))
                if k not in model and len(model) >= cap:
                    with pytest.raises(OSError):
                        f.update(mid, k, v)
                    continue
                f.update(mid, k, v)
                model[k] = v
            else:
                if k in model:
                    f.delete(mid, k)
                    del model[k]
                else:
                    with pytest.raises(OSError):
                        f.delete(mid, k)
            if step % 500 == 0:
                assert sorted(f.keys(mid)) == sorted(model)
        for k in pool:
            if k in model:
                assert f.lookup(mid, k) == [model[k]]
            else:
                with pytest.raises(OSError):
                    f.lookup(mid, k)
        vals, present = f.lookup_batch(mid, np.frombuffer(b"".join(pool), np.uint8).reshape(-1, keylen))
        assert [bool(p) for p in present] == [k in model for k in pool]
        assert [int(v[0]) for v, k in zip(vals, pool) if k in model] == \
            [model[k] for k in pool if k in model]
        f.close()


def test_update_batch_equals_single_updates():
    keys = X.rand_keys(11, 2000, 4)
    vals = np.arange(len(keys), dtype=np.uint64) << np.uint64(6) | np.uint64(2)
    a = G.Filter(G.FEAT_ALL | G.FEAT_DENY, ndev=0, ipv4_capacity=5000)
    b = G.Filter(G.FEAT_ALL | G.FEAT_DENY, ndev=0, ipv4_capacity=5000)
    a.update_batch(G.MAP_IPV4, keys, vals)
    for k, v in zip(keys, vals):
        b.update(G.MAP_IPV4, bytes(k), int(v))
    np.testing.assert_array_equal(a.values_of(G.MAP_IPV4, keys), vals)
    np.testing.assert_array_equal(b.values_of(G.MAP_IPV4, keys), vals)
    assert a.keys(G.MAP_IPV4) == b.keys(G.MAP_IPV4)
