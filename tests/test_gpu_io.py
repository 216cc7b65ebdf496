"""GPU tests of the paths either side of the kernel:

  * AF_XDP descriptor batches (xfg_classify_descs): a UMEM with 4 KiB frames,
    aligned and unaligned-chunk addresses, an RX ring view that wraps;
  * the CLI end to end: rules added with `xdp-filter ip/port/ether`, a pcap
    classified with `xdp-filter run`, the pcapng verdict dump, and the hit
    counters / stats that `status` then prints; the traffic checks of
    xdp-filter/tests/test-xdp-filter.sh (ports allow/deny, :95-130) restated
    as frames;
  * the rule store's per-device reload.
All bit-exact against the CPU restatement (oracle/) on the same frames.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import pcaputil as P
import xftools as X

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XF = os.path.join(ROOT, "xdp-tools_amd",
                  "bin-asan" if os.environ.get("XFG_LIB") == "asan" else "bin", "xdp-filter")


@pytest.fixture(scope="module")
def G():
    import xfgpu
    return xfgpu


def test_classify_descs_umem_ring(G):
    rules, pool = X.random_rules(61, n4=120, n6=60, ne=20, nports=30)
    n = 20000
    data, lens = X.gen_fuzz(23, n, 160, rules, pool)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=160)
    # UMEM: 4 KiB chunks; frame i in chunk perm[i] at headroom 256 (aligned
    # mode) or, for every third frame, chunk base + offset in bits 48..63
    # (unaligned-chunk mode)
    rng = np.random.default_rng(4)
    nchunks = n + 100
    perm = rng.permutation(nchunks)[:n]
    umem = np.zeros(nchunks * 4096, np.uint8)
    addr = np.zeros(n, np.uint64)
    for i in range(n):
        base, head = int(perm[i]) * 4096, 256 + 16 * (i % 3)
        umem[base + head:base + head + lens[i]] = data[i * 160:i * 160 + lens[i]]
        addr[i] = (base | (head << 48)) if i % 3 == 2 else base + head
    # RX ring of 32768 entries; the batch starts near the end so it wraps
    ring, first = 32768, 32768 - 777
    descs = np.zeros((ring, 2), np.uint64)
    idx = (first + np.arange(n)) & (ring - 1)
    descs[idx, 0] = addr
    descs[idx, 1] = lens.astype(np.uint64)                  # len | options 0 << 32
    f = G.Filter(feats, ndev=1)
    f.load_rules(rules)
    d_umem, d_descs, d_v = f.alloc(umem.nbytes), f.alloc(descs.nbytes), f.alloc(n)
    d_umem.upload(umem)
    d_descs.upload(descs)
    f.classify_descs(d_umem.ptr, d_descs.ptr, n, d_v.ptr, first=first, mask=ring - 1)
    f.sync()
    v = d_v.download(np.zeros(n, np.uint8))
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(f.stats(), ost)
    r = rules.prepared()
    np.testing.assert_array_equal(f.values_of(G.MAP_IPV4, r.v4_keys), orules.v4_vals)
    np.testing.assert_array_equal(f.values_of(G.MAP_PORTS, np.arange(65536, dtype=np.uint32)),
                                  orules.ports)
    with pytest.raises(OSError):      # a ring mask must be 2^k - 1
        f.classify_descs(d_umem.ptr, d_descs.ptr, n, d_v.ptr, mask=1000)
    f.close()


def test_store_reload_keeps_counters(G, tmp_path):
    d = str(tmp_path)
    rules, pool = X.random_rules(71, n4=100, n6=40, ne=10, nports=20)
    data, lens = X.gen_fuzz(3, 30000, 160, rules, pool)
    feats = X.VARIANT_FEATURES["xdpfilt_alw_all"]
    for m in range(4):
        G.lib.xfg_store_create_map(d.encode(), m, 10000)
    f = G.Filter(feats, ndev=1)
    f.load_rules(rules)
    f.run(data, lens, stride=160)
    f.store_save(d)
    f.close()
    f = G.Filter(feats, ndev=1)
    f.store_load(d)
    f.run(data, lens, stride=160)
    _, once, _ = X.run_oracle(feats, data, lens, rules, stride=160)
    _, twice, _ = X.run_oracle(feats, data, lens, once, stride=160)
    r = rules.prepared()
    np.testing.assert_array_equal(f.values_of(G.MAP_IPV6, r.v6_keys), twice.v6_vals)
    np.testing.assert_array_equal(f.values_of(G.MAP_PORTS, np.arange(65536, dtype=np.uint32)),
                                  twice.ports)
    f.close()


@pytest.fixture
def cli(tmp_path):
    env = dict(os.environ, XDP_FILTER_STATE_DIR=str(tmp_path / "state"))

    def run(*args, ok=True):
        p = subprocess.run([XF, *map(str, args)], env=env, capture_output=True, text=True,
                           timeout=120)
        if ok:
            assert p.returncode == 0, (args, p.stdout, p.stderr)
        return p
    return run


def _parse_status(out):
    """{key: (flags, hits)} of every Filtered ... section, and the stats."""
    rules, stats = {}, {}
    for line in out.splitlines():
        m = re.fullmatch(r"  (XDP_\w+)\s+(\d+) pkts\s+(\d+) KiB", line)
        if m:
            stats[m.group(1)] = int(m.group(2))
            continue
        m = re.fullmatch(r"  (\S+)\s+([a-z,]+)\s+(\d+)", line)
        if m and m.group(1) != "Mode":
            rules[m.group(1)] = (m.group(2), int(m.group(3)))
    return rules, stats


def test_cli_run_end_to_end(G, cli, tmp_path):
    # rules through the CLI, traffic from a pcap, verdicts through the dump
    import ipaddress
    rs, pool = X.random_rules(81, n4=40, n6=20, ne=8, nports=12, flag_mode="dst")
    cli("load", "veth0", "-p", "deny")
    for k in rs.v4_keys:
        cli("ip", str(ipaddress.IPv4Address(bytes(k))))
    for k in rs.v6_keys:
        cli("ip", str(ipaddress.IPv6Address(bytes(k))))
    for k in rs.eth_keys:
        cli("ether", ":".join(f"{b:02x}" for b in k))
    for p in pool:
        cli("port", int(p))
    # what the CLI stored, as oracle rules: ip/ether dst, ports dst,tcp,udp
    rules = X.RuleSet()
    rules.v4_keys, rules.v6_keys, rules.eth_keys = rs.v4_keys, rs.v6_keys, rs.eth_keys
    rules.v4_vals = np.full(len(rs.v4_keys), 2, np.uint64)
    rules.v6_vals = np.full(len(rs.v6_keys), 2, np.uint64)
    rules.eth_vals = np.full(len(rs.eth_keys), 2, np.uint64)
    for p in pool:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    data, lens = X.gen_fuzz(17, 5000, 160, rules, pool)
    frames = P.frames_of(data, lens, stride=160)
    pcap = tmp_path / "in.pcap"
    P.write_pcap(pcap, frames)
    bdata, boffs, blens = P.batch_from(frames)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, orules, ost = X.run_oracle(feats, bdata, blens, rules, offsets=boffs)
    dump = tmp_path / "out.pcapng"
    out = cli("run", "veth0", pcap, "--dump", dump).stdout
    assert "Classified 5000 packets on veth0 with xdpfilt_dny_all" in out
    got = P.read_verdict_pcapng(dump)
    assert [g[0] for g in got] == frames
    np.testing.assert_array_equal([g[2] for g in got], ov)
    st_rules, stats = _parse_status(cli("status").stdout)
    assert stats == {"XDP_ABORTED": int(ost[0, 0]), "XDP_DROP": int(ost[1, 0]),
                     "XDP_PASS": int(ost[2, 0])}
    for k, v in zip(rs.v4_keys, orules.v4_vals):
        assert st_rules[str(ipaddress.IPv4Address(bytes(k)))] == ("dst", int(v) >> 6)
    for p in pool:
        assert st_rules[str(int(p))] == ("dst,tcp,udp", int(orules.ports[X.port_key(int(p))]) >> 6)
    # a second run accumulates, like packets arriving later
    cli("run", "veth0", pcap, "-q")
    st2, stats2 = _parse_status(cli("status").stdout)
    assert stats2["XDP_PASS"] == 2 * stats["XDP_PASS"]
    cli("unload", "veth0")


@pytest.mark.parametrize("policy", ["allow", "deny"])
def test_cli_ports_traffic(G, cli, tmp_path, policy):
    # test-xdp-filter.sh:95-130: TCP/UDP to port 10000 vs 10001 before, while
    # and after port 10000 is filtered
    def frame(proto, dport):
        eth = bytes.fromhex("02000000000102000000000286dd")
        l4 = (bytes.fromhex("c0de") + dport.to_bytes(2, "big") +
              (bytes(8) + bytes([0x50, 0x02]) + bytes(6) if proto == 6 else bytes([0, 13, 0, 0])))
        ip6 = bytes([0x60, 0, 0, 0]) + len(l4 + b"x").to_bytes(2, "big") + bytes([proto, 64]) + \
            bytes(15) + b"\x01" + bytes(15) + b"\x02"
        return eth + ip6 + l4 + b"x"
    frames = [frame(6, 10000), frame(17, 10000), frame(6, 10001), frame(17, 10001)]
    pcap = tmp_path / "p.pcap"
    P.write_pcap(pcap, frames)
    PASS, DROP = 2, 1
    ok, blocked = (PASS, DROP) if policy == "allow" else (DROP, PASS)
    cli("load", "veth0", "-p", policy, "-f", "udp,tcp")

    def verdicts():
        cli("run", "veth0", pcap, "-d", tmp_path / "v.pcapng", "-q")
        return [g[2] for g in P.read_verdict_pcapng(tmp_path / "v.pcapng")]
    assert verdicts() == [ok] * 4
    cli("port", 10000)
    assert verdicts() == [blocked, blocked, ok, ok]
    cli("port", 10000, "-r")
    assert verdicts() == [ok] * 4
    cli("unload", "veth0")


REMOVALS = [("-m src", "dst,tcp,udp"), ("-m dst", "src,tcp,udp"), ("-p udp", "src,dst,tcp"),
            ("-p tcp", "src,dst,udp"), ("-m src -p udp", "dst,tcp"), ("-m src -p tcp", "dst,udp"),
            ("-m dst -p udp", "src,tcp"), ("-m dst -p tcp", "src,udp"), ("", ""),
            ("-m src,dst", ""), ("-p tcp,udp", ""), ("-m src,dst -p tcp,udp", "")]


@pytest.mark.parametrize("opts,left", REMOVALS)
def test_cli_removal_algebra_traffic(G, cli, tmp_path, opts, left):
    """test-xdp-filter.sh:309-351 (check_port_removal_from_all,
    test_output_remove): port 54321 with src,dst,tcp,udp, then one removal;
    the flags `status` prints must be what the HIP path then matches: tcp and
    udp frames with 54321 as source and as destination port, the verdicts,
    and the hit count beside the flags."""
    port = 54321

    def frame(proto, sport, dport):
        eth = bytes.fromhex("020000000001020000000002" "0800")
        l4 = sport.to_bytes(2, "big") + dport.to_bytes(2, "big") + (
            bytes(8) + bytes([0x50, 0x02]) + bytes(6) if proto == 6 else bytes([0, 9, 0, 0]) + b"x")
        ip = bytes([0x45, 0]) + (20 + len(l4)).to_bytes(2, "big") + bytes(4) + \
            bytes([64, proto, 0, 0]) + bytes([192, 0, 2, 1, 192, 0, 2, 2])
        return eth + ip + l4
    cases = [(6, port, 9), (6, 9, port), (17, port, 9), (17, 9, port)]
    frames = [frame(*c) for c in cases]
    pcap = tmp_path / "r.pcap"
    P.write_pcap(pcap, frames)
    cli("load", "veth0", "-p", "deny", "-f", "udp,tcp")
    cli("port", port, "-p", "tcp,udp", "-m", "src,dst")
    cli("port", port, *opts.split(), "-r")
    st, _ = _parse_status(cli("status").stdout)
    if left:
        assert st[str(port)] == (left, 0)
    else:
        assert str(port) not in st
    fl = set(left.split(",")) if left else set()
    want = []
    for proto, sport, dport in cases:
        pr = "tcp" if proto == 6 else "udp"
        hit = pr in fl and (("dst" in fl and dport == port) or ("src" in fl and sport == port))
        want.append(2 if hit else 1)   # deny policy: a hit passes
    cli("run", "veth0", pcap, "-d", tmp_path / "v.pcapng", "-q")
    assert [g[2] for g in P.read_verdict_pcapng(tmp_path / "v.pcapng")] == want
    st, stats = _parse_status(cli("status").stdout)
    if left:
        assert st[str(port)] == (left, want.count(2))
    assert stats["XDP_PASS"] == want.count(2) and stats["XDP_DROP"] == want.count(1)
    cli("unload", "veth0")


@pytest.mark.parametrize("n", [0, 1, 15, 4095, 4096, 4097, 65536 * 3 + 7, (1 << 22) + 13])
def test_compact_matches_nonzero(G, n):
    """Ordered verdict compaction (xfg_compact) equals np.nonzero for every
    action, on tile-boundary and ragged sizes."""
    rng = np.random.default_rng(n)
    v = rng.choice(np.array([0, 1, 2], np.uint8), n, p=[0.05, 0.45, 0.5]).astype(np.uint8)
    f = G.Filter(X.VARIANT_FEATURES["xdpfilt_dny_all"], ndev=1)
    d_v, d_i, d_c = f.alloc(max(n, 16)), f.alloc(max(4 * n, 16)), f.alloc(16)
    if n:
        d_v.upload(v)
    for action in (0, 1, 2, 3):
        f.compact(d_v.ptr, n, action, d_i.ptr, d_c.ptr)
        f.sync()
        cnt = int(d_c.download(np.zeros(1, np.uint64))[0])
        want = np.nonzero(v == action)[0].astype(np.uint32)
        assert cnt == len(want)
        if cnt:
            np.testing.assert_array_equal(d_i.download(np.zeros(cnt, np.uint32)), want)
    f.close()


def test_compact_pass_list_after_classify(G):
    """The PASS list of a classified C3 batch, as a forwarding stage uses it."""
    n = 1 << 20
    v4 = X.rand_keys(3, 50000, 4)
    data, lens = X.gen_workload(3, 3, n, 64, v4=v4)
    rules = X.RuleSet()
    rules.v4_keys, rules.v4_vals = v4, np.full(len(v4), 2, np.uint64)
    ov, _, _ = X.run_oracle(X.VARIANT_FEATURES["xdpfilt_dny_all"], data, lens, rules, stride=64,
                            nthreads=8)
    f = G.Filter(X.VARIANT_FEATURES["xdpfilt_dny_all"], ndev=1, ipv4_capacity=len(v4))
    f.load_rules(rules)
    d_data, d_lens, d_v = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(n)
    d_i, d_c = f.alloc(4 * n), f.alloc(16)
    d_data.upload(data)
    d_lens.upload(lens)
    f.classify(d_data.ptr, d_lens.ptr, n, 64, d_v.ptr)
    f.compact(d_v.ptr, n, 2, d_i.ptr, d_c.ptr)
    f.sync()
    cnt = int(d_c.download(np.zeros(1, np.uint64))[0])
    np.testing.assert_array_equal(d_i.download(np.zeros(cnt, np.uint32)),
                                  np.nonzero(ov == 2)[0].astype(np.uint32))
    f.close()


def _long_header_frames(rules, n, seed):
    """IPv6 frames whose L4 header lies past the 128-byte header window
    (hop-by-hop chains of 16-40 bytes per header before UDP/TCP to a ruled
    or unruled port), padded to 200-1400 bytes: the host path's fallback."""
    import pktbuild as PB
    rng = np.random.default_rng(seed)
    ruled = [k for k in np.nonzero(rules.prepared().ports)[0]]
    out = []
    for i in range(n):
        chain = b""
        nx = int(rng.integers(2, 6))
        for j in range(nx):
            chain += PB.ext(0 if j + 1 < nx else (17 if i % 2 else 6), int(rng.integers(1, 5)))
        port = int(ruled[i % len(ruled)]) if ruled and i % 3 else 4242
        port = ((port & 0xff) << 8) | (port >> 8) if ruled and i % 3 else port
        l4 = PB.udp(1000 + i, port) if i % 2 else PB.tcp(1000 + i, port)
        fr = PB.eth(ethertype=0x86DD) + PB.ipv6(nh=0, payload=chain + l4)
        out.append(fr + bytes(int(rng.integers(0, 1200))))
    return out


@pytest.mark.parametrize("layout", ["stride", "offsets_u16"])
def test_classify_host_header_windows_exact(G, layout):
    """xfg_classify_host sends 128-byte header windows; frames whose program
    reads past the window are classified again whole.  Verdicts, counters and
    stats equal a whole-frame oracle run, with fallbacks actually taken."""
    rules, pool = X.random_rules(101, n4=200, n6=100, ne=30, nports=40)
    fuzz_d, fuzz_l = X.gen_fuzz(31, 30000, 160, rules, pool)
    frames = P.frames_of(fuzz_d, fuzz_l, stride=160) + _long_header_frames(rules, 3000, 5)
    rng = np.random.default_rng(8)
    frames = [frames[i] for i in rng.permutation(len(frames))]
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    if layout == "stride":
        stride = 1536
        data = np.zeros(len(frames) * stride, np.uint8)
        lens = np.array([len(f) for f in frames], np.uint32)
        for i, fr in enumerate(frames):
            data[i * stride:i * stride + len(fr)] = np.frombuffer(fr, np.uint8)
        ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=stride)
        offs = None
    else:
        data, offs, lens = P.batch_from(frames)
        lens = lens.astype(np.uint16)
        stride = 0
        ov, orules, ost = X.run_oracle(feats, data, lens.astype(np.uint32), rules, offsets=offs)
    f = G.Filter(feats, ndev=1)
    f.load_rules(rules)
    v = f.classify_host(data, lens, stride=stride, offsets=offs)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(f.stats(), ost)
    r = rules.prepared()
    np.testing.assert_array_equal(f.values_of(G.MAP_IPV6, r.v6_keys), orules.v6_vals)
    np.testing.assert_array_equal(f.values_of(G.MAP_PORTS, np.arange(65536, dtype=np.uint32)),
                                  orules.ports)
    f.close()


@pytest.mark.parametrize("registered", [False, True])
def test_classify_xsk_host_ring_wrap_unaligned(G, registered):
    """The host-memory AF_XDP consumer (xfg_classify_xsk_host): a UMEM of
    4 KiB chunks in host memory, frames at aligned and unaligned-chunk
    addresses (offset in bits 48..63, headers/xdp/xsk.h:173-186), an RX ring
    view that wraps; long-header frames take the whole-frame fallback, or,
    with the UMEM registered, every frame is read in place (zero copy)."""
    rules, pool = X.random_rules(111, n4=120, n6=60, ne=20, nports=30)
    fd, fl = X.gen_fuzz(29, 20000, 160, rules, pool)
    frames = P.frames_of(fd, fl, stride=160) + _long_header_frames(rules, 1500, 9)
    n = len(frames)
    data, offs, lens = P.batch_from(frames)
    feats = X.VARIANT_FEATURES["xdpfilt_alw_all"]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, offsets=offs)
    rng = np.random.default_rng(12)
    nchunks = n + 64
    perm = rng.permutation(nchunks)[:n]
    umem = np.zeros(nchunks * 4096, np.uint8)
    addr = np.zeros(n, np.uint64)
    for i, fr in enumerate(frames):
        base, head = int(perm[i]) * 4096, 256 + 16 * (i % 3)
        umem[base + head:base + head + len(fr)] = np.frombuffer(fr, np.uint8)
        addr[i] = (base | (head << 48)) if i % 3 == 2 else base + head
    ring, first = 32768, 32768 - 1001
    descs = np.zeros((ring, 2), np.uint64)
    idx = (first + np.arange(n)) & (ring - 1)
    descs[idx, 0] = addr
    descs[idx, 1] = lens.astype(np.uint64)
    f = G.Filter(feats, ndev=1)
    f.load_rules(rules)
    if registered:
        f.host_register(umem)
    v = f.classify_xsk_host(umem, descs, n, first=first, mask=ring - 1)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(f.stats(), ost)
    r = rules.prepared()
    np.testing.assert_array_equal(f.values_of(G.MAP_IPV4, r.v4_keys), orules.v4_vals)
    np.testing.assert_array_equal(f.values_of(G.MAP_PORTS, np.arange(65536, dtype=np.uint32)),
                                  orules.ports)
    with pytest.raises(OSError):      # a frame outside the UMEM
        bad = descs.copy()
        bad[idx[0], 0] = umem.nbytes - 8
        f.classify_xsk_host(umem, bad, n, first=first, mask=ring - 1)
    with pytest.raises(OSError):      # a ring mask must be 2^k - 1
        f.classify_xsk_host(umem, descs, n, first=first, mask=1000)
    if registered:
        f.host_unregister(umem)
    f.close()


def test_compact_two_streams_concurrently(G):
    """Two compactions in flight at once on two streams of one device
    (the per-device scratch is ordered through the library's
    stream, so neither resets the other's tile status)."""
    import torch
    n = (1 << 22) + 77
    rng = np.random.default_rng(21)
    va = rng.integers(0, 3, n, dtype=np.uint8)
    vb = rng.integers(0, 3, n, dtype=np.uint8)
    f = G.Filter(X.VARIANT_FEATURES["xdpfilt_dny_all"], ndev=1)
    bufs = [(f.alloc(n), f.alloc(4 * n), f.alloc(16)) for _ in range(2)]
    bufs[0][0].upload(va)
    bufs[1][0].upload(vb)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        f.compact(bufs[0][0].ptr, n, 2, bufs[0][1].ptr, bufs[0][2].ptr, stream=s1.cuda_stream)
        f.compact(bufs[1][0].ptr, n, 1, bufs[1][1].ptr, bufs[1][2].ptr, stream=s2.cuda_stream)
    s1.synchronize()
    s2.synchronize()
    f.sync()
    for (dv, di, dc), v, act in ((bufs[0], va, 2), (bufs[1], vb, 1)):
        cnt = int(dc.download(np.zeros(1, np.uint64))[0])
        np.testing.assert_array_equal(di.download(np.zeros(cnt, np.uint32)),
                                      np.nonzero(v == act)[0].astype(np.uint32))
    f.close()


@pytest.mark.parametrize("stride", [64, 160])
def test_length_past_stride_is_clamped_to_slot(G, stride):
    """A fixed-stride batch whose lengths exceed the stride: the
    kernel reads no byte past a slot (the last packet's included) and
    classifies each frame as its slot-long prefix."""
    rules, pool = X.random_rules(131, n4=100, n6=40, ne=10, nports=20)
    n = 50000
    data, lens = X.gen_fuzz(41, n, stride, rules, pool) if stride == 160 else \
        X.gen_workload(3, 3, n, stride, v4=rules.v4_keys, ports=np.array([53], np.uint16))
    big = lens.copy()
    big[::7] = stride + 1000
    big[-1] = 65000
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, orules, ost = X.run_oracle(feats, data, np.minimum(big, stride).astype(np.uint32), rules,
                                   stride=stride)
    f = G.Filter(feats, ndev=1)
    f.load_rules(rules)
    d_data, d_lens, d_v = f.alloc(data.nbytes), f.alloc(big.nbytes), f.alloc(n)
    d_data.upload(data)
    d_lens.upload(big)
    f.classify(d_data.ptr, d_lens.ptr, n, stride, d_v.ptr)
    f.sync()
    np.testing.assert_array_equal(d_v.download(np.zeros(n, np.uint8)), ov)
    np.testing.assert_array_equal(f.stats(), ost)
    f.close()


def test_cli_run_capture_with_one_huge_frame(G, cli, tmp_path):
    """`xdp-filter run` over a capture holding one 64 KB (GRO-sized) frame
    among ordinary ones (staging is fixed-size, not stride-sized):
    it runs, and the verdicts match the restatement."""
    import pktbuild as PB
    rules, pool = X.random_rules(141, n4=30, n6=10, ne=5, nports=10, flag_mode="dst")
    d, l = X.gen_fuzz(43, 3000, 160, rules, pool)
    frames = P.frames_of(d, l, stride=160)
    huge = PB.eth() + PB.ipv4("10.1.2.3", "10.4.5.6", 17, payload=PB.udp(7, 53, payload=bytes(65000)))
    frames.insert(1234, huge)
    pcap = tmp_path / "huge.pcap"
    P.write_pcap(pcap, frames)
    bdata, boffs, blens = P.batch_from(frames)
    cli("load", "veth0", "-p", "deny")
    for p in pool:
        cli("port", int(p))
    prules = X.RuleSet()
    for p in pool:
        prules.ports[X.port_key(int(p))] = 2 | 4 | 8
    ov, _, _ = X.run_oracle(X.VARIANT_FEATURES["xdpfilt_dny_all"], bdata, blens, prules,
                            offsets=boffs)
    cli("run", "veth0", pcap, "-d", tmp_path / "v.pcapng", "-q")
    got = P.read_verdict_pcapng(tmp_path / "v.pcapng")
    assert len(got[1234][0]) == len(huge)
    np.testing.assert_array_equal([g[2] for g in got], ov)
    cli("unload", "veth0")


def test_classify_host_registered_buffer(G):
    """xfg_host_register: a registered 64-byte-stride batch is read by the
    kernels where it lies (zero copy, no staging); same verdicts, counters
    and stats; overlapping registration and unknown unregister are refused."""
    n = (1 << 19) + 5
    v4 = X.rand_keys(3, 20000, 4)
    ports = np.array([53, 80], np.uint16)
    data, lens = X.gen_workload(3, 3, n, 64, v4=v4, ports=ports)
    rules = X.RuleSet()
    rules.v4_keys, rules.v4_vals = v4, np.full(len(v4), 2, np.uint64)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=64, nthreads=8)
    f = G.Filter(feats, ndev=1, ipv4_capacity=len(v4))
    f.load_rules(rules)
    f.host_register(data)
    with pytest.raises(OSError):
        f.host_register(data[64:])            # overlaps
    v = f.classify_host(data, lens.astype(np.uint16), stride=64)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(f.stats(), ost)
    r = rules.prepared()
    np.testing.assert_array_equal(f.values_of(G.MAP_IPV4, r.v4_keys), orules.v4_vals)
    f.host_unregister(data)
    with pytest.raises(OSError):
        f.host_unregister(data)
    f.close()


@pytest.mark.parametrize("stride,first", [(1536, 0), (1536, 777), (128, 4099), (168, 0)])
def test_classify_host_registered_slices(G, stride, first):
    """Registered batches the zero-copy path reads in place: large slots
    (whole 1514-byte frames, walked past the window by the IPv6 extension
    headers), a batch starting inside the registered buffer (the device
    address offset), and a stride the kernels' 16-byte loads cannot take in
    place (168: the staging path) -- all equal to the restatement."""
    n = 40000 if stride > 128 else 300000
    rules, pool = X.random_rules(71 + stride, n4=300, n6=100, ne=20, nports=40)
    data, lens = X.gen_fuzz(5 + first, n + first, stride, rules, pool)
    feats = X.VARIANT_FEATURES["xdpfilt_alw_all"]
    sub = data[first * stride:]
    slens = lens[first:].astype(np.uint32)
    slens[-1] = 65000                     # past its slot: capped at the stride
    ov, _, ost = X.run_oracle(feats, sub, np.minimum(slens, stride), rules, stride=stride,
                              nthreads=8)
    f = G.Filter(feats, ndev=1)
    f.load_rules(rules)
    f.host_register(data)
    try:
        v = f.classify_host(sub, slens, stride=stride)
    finally:
        f.host_unregister(data)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(f.stats(), ost)
    f.close()


@pytest.mark.parametrize("shift", [8, 4])
def test_classify_host_registered_unaligned(G, shift):
    """A registered buffer whose batch does not start 16-byte aligned: the
    zero-copy path (16-byte loads in place) needs aligned slots, so the
    batch takes the staged path -- results equal to the restatement."""
    n, stride = 200000, 160
    rules, pool = X.random_rules(91 + shift, n4=300, n6=100, ne=20, nports=40)
    data, lens = X.gen_fuzz(17 + shift, n, stride, rules, pool)
    buf = np.zeros(n * stride + 64, np.uint8)
    assert buf.ctypes.data % 16 == 0
    sub = buf[shift:shift + n * stride]
    sub[:] = data[:n * stride]
    assert sub.ctypes.data % 16 != 0
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, _, ost = X.run_oracle(feats, data, lens, rules, stride=stride, nthreads=8)
    f = G.Filter(feats, ndev=1)
    f.load_rules(rules)
    f.host_register(buf)
    try:
        v = f.classify_host(sub, lens, stride=stride)
    finally:
        f.host_unregister(buf)
    np.testing.assert_array_equal(v, ov)
    np.testing.assert_array_equal(f.stats(), ost)
    f.close()


@pytest.mark.timeout(300)
def test_classify_host_registered_hybrid():
    """Registered 1536-byte slots through the hybrid host path -- each round
    a zero-copy chunk and staged chunks of header windows, side by side
    (xfg_ctx.c host_run_hyb) -- equal to the restatement; run in a fresh
    process on the diagnostics library with the rounds made small enough
    (XFG_HYB_ZLOG2=16) for a test-sized batch (tests/gpu_hyb_worker.py)."""
    import subprocess
    import sys
    env = dict(os.environ, XFG_LIB="diag", XFG_HYB_ZLOG2="16", XFG_HYB_ST="2")
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "gpu_hyb_worker.py")],
                       capture_output=True, text=True, timeout=280, env=env)
    assert p.returncode == 0 and "OK" in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]


def test_classify_host_registered_large_slots_many_frames(G):
    """Registered 1536-byte slots, 798k frames read in place (zero copy)
    (500 rules: the generic pipelined kernel) and IPv6 frames whose
    program walks past the 64-byte window (the kernels' deferred walk reads
    the mapped frame) -- every frame's verdict, every counter and the
    stats equal the restatement's."""
    stride = 1536
    n = (1 << 19) + (1 << 18) + 12345
    rules, pool = X.random_rules(404, n4=500, n6=200, ne=30, nports=40)
    data, lens = X.gen_fuzz(405, n, stride, rules, pool)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=stride, nthreads=8)
    f = G.Filter(feats, ndev=1)
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
