"""CPU tests of the host formats around the classifier (include/xdpfilter_io.h):
pcap / pcapng ingest, the pcapng verdict dump (xdpdump's EPB verdict option,
lib/util/xpcapng.c:392-479) and the rule store that replaces the bpffs pin
directory.  The files are written and parsed by tests/pcaputil.py, an
independent struct-based implementation.
"""
import errno
import os

import numpy as np
import pytest

import pcaputil as P
import xfgpu as G
import xftools as X


def sample_frames(n=300, seed=5):
    rules, pool = X.random_rules(seed)
    data, lens = X.gen_fuzz(seed, n, 160, rules, pool)
    return P.frames_of(data, lens, stride=160)


def check_batch(path, frames):
    data, offs, lens, olens, ts = G.read_pcap(path)
    assert len(lens) == len(frames)
    assert (offs % 16 == 0).all()
    for i, fr in enumerate(frames):
        assert lens[i] == len(fr)
        assert bytes(data[offs[i]:offs[i] + lens[i]]) == fr
        assert (data[offs[i] + lens[i]:(offs[i] + lens[i] + 15) // 16 * 16] == 0).all()
    return data, offs, lens, olens, ts


@pytest.mark.parametrize("nsec", [False, True])
@pytest.mark.parametrize("big", [False, True])
def test_pcap_classic(tmp_path, nsec, big):
    frames = sample_frames()
    p = tmp_path / "a.pcap"
    P.write_pcap(p, frames, nsec=nsec, big_endian=big)
    _, _, lens, olens, ts = check_batch(p, frames)
    np.testing.assert_array_equal(olens, lens + 4)     # orig_len kept apart from caplen
    i = np.arange(len(frames))
    # the writer stores i % 1000 microseconds, as µs or as ns fractions
    want = (1_700_000_000 + i // 1000) * 10**9 + (i % 1000) * 1000
    np.testing.assert_array_equal(ts, want)


@pytest.mark.parametrize("big", [False, True])
@pytest.mark.parametrize("spb", [False, True])
def test_pcapng(tmp_path, big, spb):
    frames = sample_frames(seed=9)
    p = tmp_path / "a.pcapng"
    P.write_pcapng(p, frames, big_endian=big, use_spb=spb, tsresol=9 if not spb else None)
    _, _, _, _, ts = check_batch(p, frames)
    if not spb:   # if_tsresol 9 = ns units
        np.testing.assert_array_equal(ts, 1_700_000_000_000_000 + np.arange(len(frames)))


def test_pcapng_default_resolution_is_microseconds(tmp_path):
    p = tmp_path / "a.pcapng"
    P.write_pcapng(p, sample_frames(10))
    _, _, _, _, ts = G.read_pcap(p)
    np.testing.assert_array_equal(ts, (1_700_000_000_000_000 + np.arange(10)) * 1000)


def test_pcap_errors(tmp_path):
    frames = sample_frames(20)
    p = tmp_path / "raw.pcap"
    P.write_pcap(p, frames, linktype=101)           # LINKTYPE_RAW: no Ethernet header
    with pytest.raises(OSError) as e:
        G.read_pcap(p)
    assert e.value.errno == errno.EPROTONOSUPPORT
    P.write_pcap(p, frames)
    b = open(p, "rb").read()
    open(p, "wb").write(b[:-3])                     # truncated last record
    with pytest.raises(OSError) as e:
        G.read_pcap(p)
    assert e.value.errno == errno.EINVAL
    open(p, "wb").write(b"not a capture file")
    with pytest.raises(OSError):
        G.read_pcap(p)
    with pytest.raises(OSError) as e:
        G.read_pcap(tmp_path / "missing.pcap")
    assert e.value.errno == errno.ENOENT


def test_empty_capture(tmp_path):
    p = tmp_path / "e.pcap"
    P.write_pcap(p, [])
    data, offs, lens, _, _ = G.read_pcap(p)
    assert len(lens) == 0


def test_verdict_dump_roundtrip(tmp_path):
    frames = sample_frames(200, seed=3)
    data, offs, lens = P.batch_from(frames)
    verdicts = np.random.default_rng(1).integers(0, 3, len(frames)).astype(np.uint8)
    p = tmp_path / "v.pcapng"
    G.write_verdicts_pcapng(p, "veth0", data, offs, lens, verdicts)
    got = P.read_verdict_pcapng(p)
    assert [g[0] for g in got] == frames
    assert all(g[1] == 2 for g in got)               # PCAPNG_EPB_VEDRICT_TYPE_EBPF_XDP
    assert [g[2] for g in got] == verdicts.tolist()
    # and the dump is itself a capture the ingest path reads back
    check_batch(p, frames)


def _host(cap=5000):
    return G.Filter(G.FEAT_ALL | G.FEAT_DENY, ndev=0, ipv4_capacity=cap, ipv6_capacity=cap,
                    eth_capacity=cap)


def test_store_roundtrip(tmp_path):
    d = str(tmp_path)
    rules, pool = X.random_rules(21, n4=400, n6=200, ne=50, nports=60)
    for m, cap in ((G.MAP_PORTS, 0), (G.MAP_IPV4, 5000), (G.MAP_IPV6, 5000), (G.MAP_ETHERNET, 5000)):
        assert G.lib.xfg_store_create_map(d.encode(), m, cap) == 0
        assert G.lib.xfg_store_has_map(d.encode(), m) == 1
    assert G.lib.xfg_store_map_capacity(d.encode(), G.MAP_IPV4) == 5000
    assert G.lib.xfg_store_map_capacity(d.encode(), G.MAP_PORTS) == 65536
    a = _host()
    a.load_rules(rules)
    a.store_save(d)
    b = _host()
    b.store_load(d)
    r = rules.prepared()
    for m, keys, vals in ((G.MAP_IPV4, r.v4_keys, r.v4_vals), (G.MAP_IPV6, r.v6_keys, r.v6_vals),
                          (G.MAP_ETHERNET, r.eth_keys, r.eth_vals)):
        np.testing.assert_array_equal(b.values_of(m, keys), vals)
        assert sorted(b.keys(m)) == sorted(a.keys(m))
    np.testing.assert_array_equal(b.values_of(G.MAP_PORTS, np.arange(65536, dtype=np.uint32)),
                                  r.ports)
    # a map that is not "pinned" is neither saved nor loaded
    assert G.lib.xfg_store_remove_map(d.encode(), G.MAP_ETHERNET) == 0
    assert G.lib.xfg_store_has_map(d.encode(), G.MAP_ETHERNET) == 0
    a.store_save(d)
    c = _host()
    c.store_load(d)
    assert c.count(G.MAP_ETHERNET) == 0 and c.count(G.MAP_IPV4) == len(r.v4_keys)


def test_store_load_respects_capacity(tmp_path):
    d = str(tmp_path)
    G.lib.xfg_store_create_map(d.encode(), G.MAP_IPV4, 1000)
    a = _host(1000)
    keys = X.rand_keys(4, 1000, 4)
    a.update_batch(G.MAP_IPV4, keys, np.full(len(keys), 2, np.uint64))
    a.store_save(d)
    small = _host(999)
    with pytest.raises(OSError) as e:
        small.store_load(d)
    assert e.value.errno == errno.E2BIG


def test_stats_file(tmp_path):
    d = str(tmp_path)
    recs = (G.StatsRecord * 5)(*[G.StatsRecord(i, 100 * i) for i in range(5)])
    assert G.lib.xfg_store_stats_write(d.encode(), recs) == 0
    np.testing.assert_array_equal(G.store_stats(d), [[i, 100 * i] for i in range(5)])
    assert G.lib.xfg_store_stats_remove(d.encode()) == 0
    with pytest.raises(OSError) as e:
        G.store_stats(d)
    assert e.value.errno == errno.ENOENT


def test_update_batch_percpu_host_context():
    keys = X.rand_keys(12, 500, 16)
    vals = (np.arange(len(keys), dtype=np.uint64) << np.uint64(6)) | np.uint64(1)
    a, b = _host(), _host()
    a.update_batch_percpu(G.MAP_IPV6, keys, vals.reshape(-1, 1))
    b.update_batch(G.MAP_IPV6, keys, vals)
    np.testing.assert_array_equal(a.values_of(G.MAP_IPV6, keys), b.values_of(G.MAP_IPV6, keys))
