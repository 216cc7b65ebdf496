"""GPU parity of the quotient-index path (xfg_pipeq_kernel, XFG_PATH_QT):
the IPv4-key pipelined classify that answers each lookup with one read of a
32-byte bucket of a derived index (xfg_layout.h), against the CPU
restatement (oracle/), bit-exact: verdicts, every rule's value, stats.
Contract: xdp-filter/xdpfilt_prog.h:56-64 (CHECK_MAP), :121-134
(lookup_verdict_ipv4), :214-310.

The index applies when exactly one IPv4 lookup direction can hit; these
tests open the context with qt_min_keys=1 so that small rule sets take it,
and assert that the launch did (last_path).  Covered: dst-only and src-only
rule sets with keys whose flags lack the live mask, the zero key, both
window sizes and a non-dense stride, ports beside the index, buckets that
overflow (their misses and their spilled keys decided by the canonical
table), rebuilds after inserts / deletes / flag changes between batches,
both IPv4 directions live (one image for src|dst rule sets, two
otherwise), single edits patched into the index between batches, IPv6
rules beside the index (their lookups in the kernel's loop, beside one or
both IPv4 directions), and the hit log in one and in two count passes.  The kernel logs its hits only for batches of at least
as many packets as the index has slots (xfg_ctx.c launch_batch); the
smaller batches here count through its LDS counter cache and atomics.
"""
import os

import numpy as np
import pytest

import xftools as X
from test_gpu import assert_same, gpu_values, make_filter

pytestmark = pytest.mark.gpu
M32 = 0xffffffff


@pytest.fixture(scope="module")
def G():
    import xfgpu
    return xfgpu


def fmix32(h):
    h = h.astype(np.uint64)
    h ^= h >> 16
    h = (h * 0x85ebca6b) & M32
    h ^= h >> 13
    h = (h * 0xc2b2ae35) & M32
    h ^= h >> 16
    return h.astype(np.uint32)


# the index's hash for the default table seed (xfg_ctx.c xfg_open, qt_refresh)
QT_SEED = 0x5eed1234 ^ 0x51ed2701


QT_BITS, QT_SLOTS = 17, 16    # xfg_layout.h: 2^17 buckets of 16 entries (small maps)


def qt_bucket(keys_u8, bits=QT_BITS):
    k = np.ascontiguousarray(keys_u8, np.uint8).reshape(-1, 4).view("<u4").reshape(-1)
    return fmix32(k ^ np.uint32(QT_SEED)) >> np.uint32(32 - bits)


def one_direction_rules(seed, n4, live, nports=16):
    """IPv4 rules whose only live lookup is `live` (2 dst / 1 src): most keys
    carry it, some carry only proto bits (present, never matching)."""
    rng = np.random.default_rng(seed)
    rules = X.RuleSet()
    v4 = X.rand_keys(seed, n4, 4)        # (distinct: possibly a few fewer than n4)
    n4 = len(v4)
    f = np.full(n4, live, np.uint64)
    f[rng.random(n4) < 0.1] = 4          # TCP bit only: the key exists, CHECK_MAP misses
    f |= rng.integers(0, 50, n4).astype(np.uint64) << 6   # pre-existing hits
    rules.v4_keys, rules.v4_vals = v4, f
    ports = rng.choice(65536, nports, replace=False).astype(np.uint16)
    for p in ports:
        rules.ports[X.port_key(int(p))] = int(rng.integers(1, 16))
    return rules, v4, ports


def fuzz_at(seed, n, stride, rules, ports):
    """The structured fuzz corpus (generated at a 160-byte stride) laid out at
    `stride`: longer frames cut to the slot (lengths capped with them)."""
    d, l = X.gen_fuzz(seed, n, 160, rules, ports)
    out = np.zeros((n, stride), np.uint8)
    w = min(stride, 160)
    out[:, :w] = d.reshape(n, 160)[:, :w]
    return out.reshape(-1), np.minimum(l, stride).astype(np.uint32)


def run_both(G, variant, rules, data, lens, stride, path=5, **kw):
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, rules,
                                   stride=stride, nthreads=8)
    f = make_filter(G, variant, qt_min_keys=1, ipv4_capacity=1 << 16, **kw)
    f.load_rules(rules)
    v = f.run(data, lens, stride=stride)
    assert f.last_path() == path
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()
    return ov


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_all", "xdpfilt_dny_ip",
                                     "xdpfilt_alw_ip"])
@pytest.mark.parametrize("live", [2, 1])
@pytest.mark.parametrize("stride", [64, 128, 256])
def test_qt_one_direction(G, variant, live, stride):
    rules, v4, ports = one_direction_rules(7 + live, 20000, live)
    # C3-shaped traffic (hits on the live side: the generator puts ruled
    # addresses in the destination; src-live rule sets get src hits by the
    # fuzz corpus below) + the structured fuzz corpus
    d1, l1 = X.gen_workload(11 + live, 3, 1 << 16, stride, v4=v4, ports=ports)
    d2, l2 = fuzz_at(13 + live, 1 << 15, stride, rules, ports)
    data = np.concatenate([d1, d2])
    lens = np.concatenate([l1, l2])
    ov = run_both(G, variant, rules, data, lens, stride)
    assert len(np.unique(ov)) == 3


def test_qt_zero_key_and_ports(G):
    rules, v4, ports = one_direction_rules(21, 5000, 2)
    v4[0] = 0                                       # the all-zero key, as a dst rule
    rules.v4_keys = v4
    rules.v4_vals[0] = 2
    data, lens = X.gen_workload(22, 3, 1 << 16, 64, v4=v4, ports=ports, dst_permille=600)
    d = data.reshape(-1, 64)
    d[::97, 30:34] = 0                              # frames to 0.0.0.0
    run_both(G, "xdpfilt_dny_all", rules, data, lens, 64)


def test_qt_overflowing_bucket(G):
    """20 rules homed in one index bucket (15 fit beside the overflow
    marker): the 5 spilled keys and every miss homed there are decided by
    the canonical table (deferred)."""
    rng = np.random.default_rng(5)
    cand = rng.integers(0, 2**32, 1 << 23, dtype=np.uint64).astype(np.uint32)
    cu8 = cand.view(np.uint8).reshape(-1, 4)
    b = qt_bucket(cu8)
    tgt = np.argmax(np.bincount(b))
    same = cu8[b == tgt]
    assert len(same) >= 40
    base, _, ports = one_direction_rules(31, 3000, 2)
    keys = np.concatenate([same[:20], base.v4_keys])
    rules = X.RuleSet()
    rules.v4_keys = keys
    rules.v4_vals = np.full(len(keys), 2, np.uint64)
    rules.ports = base.ports
    # traffic: the 20 crowded keys, 20 absent keys homed in the same bucket,
    # and C3-shaped traffic over the rest
    data, lens = X.gen_workload(32, 3, 1 << 16, 64, v4=keys, ports=ports, dst_permille=500)
    d = data.reshape(-1, 64)
    probe = np.concatenate([same[:20], same[20:40]])
    ip4 = np.nonzero((d[:, 12] == 8) & (d[:, 13] == 0) & (lens >= 62))[0][:4000]
    d[ip4, 30:34] = probe[np.arange(len(ip4)) % len(probe)]
    ov = run_both(G, "xdpfilt_dny_all", rules, data, lens, 64)
    assert (ov[ip4] == 2).sum() > 1000 and (ov[ip4] == 1).sum() > 1000


def test_qt_rebuilt_after_rule_changes(G):
    variant = "xdpfilt_dny_all"
    rules, v4, ports = one_direction_rules(41, 20000, 2)
    data, lens = X.gen_workload(42, 3, 1 << 16, 64, v4=v4, ports=ports)
    f = make_filter(G, variant, qt_min_keys=1, ipv4_capacity=1 << 16)
    f.load_rules(rules)
    cur = rules.prepared().copy()
    for step in range(3):
        v = f.run(data, lens, stride=64)
        assert f.last_path() == 5
        ov, cur, ost = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, cur, stride=64)
        got = gpu_values(f, G, cur)
        np.testing.assert_array_equal(v, ov)
        for fld in ("ports", "v4_vals"):
            np.testing.assert_array_equal(getattr(got, fld), getattr(cur, fld), err_msg=fld)
        f.stats_reset()
        # delete 1000 rules, drop the live bit from 1000, add 1000 new ones
        keep = np.ones(len(cur.v4_keys), bool)
        keep[step * 1000:(step + 1) * 1000] = False
        for k in cur.v4_keys[~keep]:
            f.delete(G.MAP_IPV4, bytes(k))
        nk = X.rand_keys(100 + step, 1200, 4)
        nk32 = nk.view("<u4").reshape(-1)
        nk = nk[~np.isin(nk32, cur.v4_keys.view("<u4").reshape(-1))][:1000]
        vals = cur.v4_vals[keep].copy()
        vals[:1000] = (vals[:1000] & ~np.uint64(3)) | np.uint64(4)
        for k, val in zip(cur.v4_keys[keep][:1000], vals[:1000]):
            f.update(G.MAP_IPV4, bytes(k), int(val))
        f.update_batch(G.MAP_IPV4, nk, np.full(len(nk), 2, np.uint64))
        nxt = X.RuleSet()
        nxt.ports = cur.ports
        nxt.v4_keys = np.concatenate([cur.v4_keys[keep], nk])
        nxt.v4_vals = np.concatenate([vals, np.full(len(nk), 2, np.uint64)])
        cur = nxt.prepared()
        data, lens = X.gen_workload(43 + step, 3, 1 << 16, 64, v4=cur.v4_keys, ports=ports)
    f.close()


def both_direction_traffic(seed, n, v4, ports, stride=64):
    """C3-shaped traffic with ruled destinations, a ruled source in a
    quarter of the IPv4 frames (some with a ruled destination too: the dst
    lookup decides those), and the structured fuzz corpus."""
    d1, l1 = X.gen_workload(seed, 3, n, stride, v4=v4, ports=ports)
    d = d1.reshape(-1, stride)
    ip4 = np.nonzero((d[:, 12] == 8) & (d[:, 13] == 0))[0][::4]
    d[ip4, 26:30] = v4[(np.arange(len(ip4)) * 7919) % len(v4)]
    return d1, l1


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_ip"])
@pytest.mark.parametrize("shape", ["sym", "asym"])
@pytest.mark.parametrize("stride", [64, 128])
def test_qt_both_directions(G, variant, shape, stride):
    """Both IPv4 lookups through the index (lookup_verdict_ipv4,
    xdpfilt_prog.h:121-134: dst first, then src; only the first hit
    counts).  sym: every ruled key carries src|dst (`xdp-filter ip -m
    src,dst`), one image serves both lookups; asym: keys with dst only, src
    only, both, and proto bits only -- two images."""
    rules, v4, ports = one_direction_rules(51, 20000, 3)
    if shape == "asym":
        rng = np.random.default_rng(52)
        f = rules.v4_vals & ~np.uint64(3)
        pick = rng.integers(0, 4, len(v4)).astype(np.uint64)   # 0: proto only
        rules.v4_vals = f | pick
    d1, l1 = both_direction_traffic(53, 1 << 16, v4, ports, stride)
    d2, l2 = fuzz_at(54, 1 << 15, stride, rules, ports)
    data, lens = np.concatenate([d1, d2]), np.concatenate([l1, l2])
    run_both(G, variant, rules, data, lens, stride)


def test_qt_both_directions_single_edits(G):
    """Single edits on a both-direction index: patched in place within one
    shape, rebuilt when a key with one direction first appears in a
    one-image index."""
    variant = "xdpfilt_dny_all"
    feat = X.VARIANT_FEATURES[variant]
    rules, v4, ports = one_direction_rules(61, 20000, 3)
    f = make_filter(G, variant, qt_min_keys=1, ipv4_capacity=1 << 16)
    f.load_rules(rules)
    cur = rules.prepared().copy()
    rng = np.random.default_rng(62)
    for step, newflag in enumerate([3, 0, 2, 1, 3]):
        d, l = both_direction_traffic(63 + step, 1 << 15, cur.v4_keys, ports)
        v = f.run(d, l, stride=64)
        assert f.last_path() == 5
        ov, cur, ost = X.run_oracle(feat, d, l, cur, stride=64)
        got = gpu_values(f, G, cur)
        assert_same(v, got, f.stats(), ov, cur, ost)
        f.stats_reset()
        idx = rng.choice(len(cur.v4_keys), 30, replace=False)
        for i in idx:   # 30 single edits: flags to newflag (counts kept)
            val = (int(cur.v4_vals[i]) & ~3) | newflag
            f.update(G.MAP_IPV4, bytes(cur.v4_keys[i]), val)
            cur.v4_vals[i] = val
    f.close()


def test_qt_counts_folded_across_batches_and_writes(G):
    """The count kernel adds to QT-order counts that the runtime folds into
    the canonical counters before any read, write or re-index: two batches
    with no readout between them, then deletes + inserts (each folds first,
    through the index being replaced), a third batch, one readout."""
    variant = "xdpfilt_dny_all"
    rules, v4, ports = one_direction_rules(61, 20000, 2)
    data, lens = X.gen_workload(62, 3, 1 << 16, 64, v4=v4, ports=ports)
    f = make_filter(G, variant, qt_min_keys=1, ipv4_capacity=1 << 16)
    f.load_rules(rules)
    cur = rules.prepared().copy()
    feat = X.VARIANT_FEATURES[variant]
    for _ in range(2):
        v = f.run(data, lens, stride=64)
        assert f.last_path() == 5
        ov, cur, _ = X.run_oracle(feat, data, lens, cur, stride=64)
        np.testing.assert_array_equal(v, ov)
    gone = cur.v4_keys[:500]
    for k in gone:
        f.delete(G.MAP_IPV4, bytes(k))
    nk = X.rand_keys(163, 700, 4)
    nk = nk[~np.isin(nk.view("<u4").reshape(-1), cur.v4_keys.view("<u4").reshape(-1))][:500]
    f.update_batch(G.MAP_IPV4, nk, np.full(len(nk), 2, np.uint64))
    nxt = X.RuleSet()
    nxt.ports = cur.ports
    nxt.v4_keys = np.concatenate([cur.v4_keys[500:], nk])
    nxt.v4_vals = np.concatenate([cur.v4_vals[500:], np.full(len(nk), 2, np.uint64)])
    cur = nxt.prepared()
    data, lens = X.gen_workload(64, 3, 1 << 16, 64, v4=cur.v4_keys, ports=ports)
    v = f.run(data, lens, stride=64)
    assert f.last_path() == 5
    ov, cur, _ = X.run_oracle(feat, data, lens, cur, stride=64)
    np.testing.assert_array_equal(v, ov)
    got = gpu_values(f, G, cur)
    for fld in ("ports", "v4_vals"):
        np.testing.assert_array_equal(getattr(got, fld), getattr(cur, fld), err_msg=fld)
    assert (cur.v4_vals >> np.uint64(6)).sum() > 0
    f.close()


def crowd(seed, bits=QT_BITS, need=40):
    """Random keys that all home in one index bucket (the fullest of 2^23)."""
    rng = np.random.default_rng(seed)
    cand = rng.integers(0, 2**32, 1 << 23, dtype=np.uint64).astype(np.uint32)
    cu8 = cand.view(np.uint8).reshape(-1, 4)
    b = qt_bucket(cu8, bits)
    same = cu8[b == np.argmax(np.bincount(b))]
    assert len(same) >= need
    return same


def test_qt_single_edits_between_batches(G):
    """Single-rule edits (xfg_map_update / xfg_map_delete, one key each, as the
    CLI makes them) patch the index in place between batches: a bucket filled
    to 16, the 17th key that turns entry 15 into the overflow marker, deletes
    that leave holes, inserts into those holes, flag changes that take keys
    out of and back into the index, and single inserts / deletes spread over
    the map -- each group followed by a batch aimed at the edited keys,
    checked bit-exactly (verdicts, every rule value, stats) against the
    restatement with the same edits.  Contract: map_set_flags / bpf_map_*_elem
    edits between packets, xdp-filter/xdp-filter.c:111-157."""
    variant = "xdpfilt_dny_all"
    feat = X.VARIANT_FEATURES[variant]
    rules, v4, ports = one_direction_rules(71, 20000, 2)
    same = crowd(72)
    rules.v4_keys = np.concatenate([same[:16], v4])      # one bucket exactly full
    rules.v4_vals = np.concatenate([np.full(16, 2, np.uint64), rules.v4_vals])
    f = make_filter(G, variant, qt_min_keys=1, ipv4_capacity=1 << 16)
    f.load_rules(rules)
    cur = {bytes(k): int(v) for k, v in zip(rules.v4_keys, rules.v4_vals)}
    cur_ports = rules.ports.copy()
    rng = np.random.default_rng(73)

    def batch(seed, aim):
        nonlocal cur, cur_ports
        rs = X.RuleSet()
        rs.ports = cur_ports
        ks = list(cur)
        rs.v4_keys = np.frombuffer(b"".join(ks), np.uint8).reshape(-1, 4).copy()
        rs.v4_vals = np.array([cur[k] for k in ks], np.uint64)
        data, lens = X.gen_workload(seed, 3, 1 << 15, 64, v4=rs.v4_keys, ports=ports)
        d = data.reshape(-1, 64)
        ip4 = np.nonzero((d[:, 12] == 8) & (d[:, 13] == 0) & (lens >= 62))[0][:6000]
        aim = np.asarray(aim, np.uint8).reshape(-1, 4)
        d[ip4, 30:34] = aim[np.arange(len(ip4)) % len(aim)]
        v = f.run(data, lens, stride=64)
        assert f.last_path() == 5
        ov, orules, ost = X.run_oracle(feat, data, lens, rs, stride=64)
        assert_same(v, gpu_values(f, G, rs), f.stats(), ov, orules, ost)
        f.stats_reset()
        cur = {bytes(k): int(x) for k, x in zip(orules.v4_keys, orules.v4_vals)}
        cur_ports = orules.ports.copy()

    batch(74, same[:24])
    # the 17th key homed in the full bucket: entry 15 becomes the marker
    for k in same[16:18]:
        f.update(G.MAP_IPV4, bytes(k), 2)
        cur[bytes(k)] = 2
    batch(75, same[:24])
    # holes: delete 3 of the bucket's keys (one of them maybe the spilled
    # one), then insert 2 new keys homed there
    for k in same[[1, 5, 16]]:
        f.delete(G.MAP_IPV4, bytes(k))
        del cur[bytes(k)]
    batch(76, same[:24])
    for k in same[18:20]:
        f.update(G.MAP_IPV4, bytes(k), 2 | (3 << 6))
        cur[bytes(k)] = 2 | (3 << 6)
    batch(77, same[:24])
    # flags: the live bit off for 40 keys, back on for 20 of them
    ks = [bytes(k) for k in v4[rng.choice(len(v4), 40, replace=False)] if bytes(k) in cur]
    for k in ks:
        nv = (cur[k] & ~3) | 4
        f.update(G.MAP_IPV4, k, nv)
        cur[k] = nv
    batch(78, np.frombuffer(b"".join(ks), np.uint8))
    for k in ks[:20]:
        nv = (cur[k] & ~7) | 2
        f.update(G.MAP_IPV4, k, nv)
        cur[k] = nv
    batch(79, np.frombuffer(b"".join(ks), np.uint8))
    # 50 single deletes and 50 single inserts over the map
    gone = [bytes(k) for k in v4[rng.choice(len(v4), 50, replace=False)] if bytes(k) in cur]
    for k in gone:
        f.delete(G.MAP_IPV4, k)
        del cur[k]
    nk = X.rand_keys(80, 80, 4)
    nk = [bytes(k) for k in nk if bytes(k) not in cur][:50]
    for k in nk:
        f.update(G.MAP_IPV4, k, 2)
        cur[k] = 2
    batch(81, np.frombuffer(b"".join(gone + nk), np.uint8))
    f.close()


def test_qt_single_edits_concurrent_with_classify(G):
    """single inserts on one thread while another thread
    launches classifies.  Each insert is the 17th key homed in an exactly full
    index bucket, so entry 15 becomes the overflow marker and the key that
    was there -- still live, still hit by the traffic -- moves to the
    canonical table.  Hits a classify counted through the old bucket must be
    folded before the bucket and its trans[] entries are replaced (qt_edit
    folds in the same device-lock section), so every live key's count equals
    the packets that hit it: M identical batches = M x one pass of the
    restatement.  Contract: per-CPU counters edited between packets,
    xdp-filter/xdp-filter.c:93-157; CHECK_MAP, xdpfilt_prog.h:56-64."""
    import threading
    feat = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    base, v4, ports = one_direction_rules(171, 20000, 2)
    busy = set(qt_bucket(base.v4_keys).tolist())
    rng = np.random.default_rng(172)
    cand = np.unique(rng.integers(0, 2**32, 1 << 22, dtype=np.uint64).astype(np.uint32))
    cu8 = cand.view(np.uint8).reshape(-1, 4)
    b = qt_bucket(cu8)
    order = np.argsort(b, kind="stable")
    b, cu8 = b[order], cu8[order]
    starts = np.searchsorted(b, np.arange(1 << QT_BITS))
    counts = np.bincount(b, minlength=1 << QT_BITS)
    pick_b = [bb for bb in np.nonzero(counts >= 17)[0] if bb not in busy][:256]
    full = np.concatenate([cu8[starts[bb]:starts[bb] + 16] for bb in pick_b])   # 16 per bucket
    extra = np.stack([cu8[starts[bb] + 16] for bb in pick_b])                  # each one's 17th
    rules = X.RuleSet()
    rules.v4_keys = np.concatenate([full, base.v4_keys])
    rules.v4_vals = np.concatenate([np.full(len(full), 2, np.uint64), base.v4_vals])
    rules.ports = base.ports
    data, lens = X.gen_workload(173, 3, 1 << 16, 64, v4=rules.v4_keys, ports=ports)
    d = data.reshape(-1, 64)
    ip4 = np.nonzero((d[:, 12] == 8) & (d[:, 13] == 0) & (lens >= 62))[0][:40000]
    d[ip4, 30:34] = full[np.arange(len(ip4)) % len(full)]
    ov, orules, ost = X.run_oracle(feat, data, lens, rules, stride=64, nthreads=8)

    f = make_filter(G, "xdpfilt_dny_all", qt_min_keys=1, ipv4_capacity=1 << 16)
    f.load_rules(rules)
    d_data, d_lens, d_v = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(len(lens))
    d_data.upload(data)
    d_lens.upload(lens)
    M = 48
    errs = []

    def classify_loop():
        try:
            for _ in range(M):
                f.classify(d_data.ptr, d_lens.ptr, len(lens), 64, d_v.ptr)
        except Exception as e:  # reported below
            errs.append(e)

    th = threading.Thread(target=classify_loop)
    th.start()
    for k in extra:
        f.update(G.MAP_IPV4, bytes(k), 2)
    th.join()
    f.sync()
    assert not errs, errs
    assert f.last_path() == 5
    v = np.zeros(len(lens), np.uint8)
    d_v.download(v)
    np.testing.assert_array_equal(v, ov)
    # live keys: M passes' hits on top of their loaded values; the inserted keys: untouched
    one = (orules.v4_vals >> np.uint64(6)) - (rules.prepared().v4_vals >> np.uint64(6))
    exp = X.RuleSet()
    exp.v4_keys = np.concatenate([rules.prepared().v4_keys, extra])
    pv = rules.prepared().v4_vals
    exp.v4_vals = np.concatenate([pv + ((one * np.uint64(M)) << np.uint64(6)),
                                  np.full(len(extra), 2, np.uint64)])
    got = f.values_of(G.MAP_IPV4, exp.v4_keys)
    np.testing.assert_array_equal(got, exp.v4_vals)
    np.testing.assert_array_equal(f.stats(), ost * np.uint64(M))
    for x in (d_data, d_lens, d_v):
        x.free()
    f.close()


def test_qt_falls_back_when_the_log_cannot_run(G):
    """qt_min_keys=1 with maps small enough that every counter has a direct
    LDS counter: the index is not used -- the IPv4-key kernel's direct LDS
    counters serve such maps -- and the launch is a result, not -EIO (ADVICE
    r3: launch_batch decides the kernel from the log's conditions)."""
    rules, v4, ports = one_direction_rules(91, 300, 2)
    data, lens = X.gen_workload(92, 3, 1 << 15, 64, v4=v4, ports=ports)
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES["xdpfilt_dny_all"], data, lens, rules,
                                   stride=64)
    f = make_filter(G, "xdpfilt_dny_all", qt_min_keys=1, ipv4_capacity=512,
                    ipv6_capacity=16, eth_capacity=16)
    f.load_rules(rules)
    v = f.run(data, lens, stride=64)
    assert f.last_path() == 2
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()


@pytest.mark.parametrize("stride", [64, 128])
def test_qt_hits_concentrated_in_few_log_partitions(G, stride):
    """Every ruled key's index bucket is 7 or 200 mod 256, so all hits fall
    into two hit-log partitions: the kernel's LDS rings for them fill, flush
    in chunks, overflow into the counter cache, and end with more than a
    wave's worth of entries each -- every count checked against the
    restatement (xdpfilt_prog.h:56-64: one bump per hit)."""
    rng = np.random.default_rng(81)
    cand = rng.integers(0, 2**32, 1 << 22, dtype=np.uint64).astype(np.uint32)
    cu8 = cand.view(np.uint8).reshape(-1, 4)
    b = qt_bucket(cu8)
    keys = cu8[((b & 255) == 7) | ((b & 255) == 200)][:3000]
    keys = np.unique(keys.view("<u4").reshape(-1)).view(np.uint8).reshape(-1, 4)
    rules = X.RuleSet()
    rules.v4_keys = keys
    rules.v4_vals = np.full(len(keys), 2, np.uint64)
    # (2^22 packets: twice as many as the index has slots, so the log runs)
    data, lens = X.gen_workload(82, 3, 1 << 22, stride, v4=keys, dst_permille=700)
    run_both(G, "xdpfilt_dny_all", rules, data, lens, stride)


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_all", "xdpfilt_dny_ip"])
@pytest.mark.parametrize("stride", [64, 128, 1536])
@pytest.mark.parametrize("dirs6", ["dst", "src", "both"])
def test_qt_with_ipv6_rules(G, variant, stride, dirs6):
    """IPv6 rules beside the IPv4 map (C5's shape, no Ethernet rule): the
    index kernel still takes the batch and the IPv4 lookups stay on the
    index.  The kernel looks the IPv6 keys up in its loop -- up to 16
    frames a tile through their home bucket lines, the rest and the misses
    in overflowed buckets deferred -- with one direction live (dst or src
    rules: one line a frame) or both (src,dst rule sets, V6B: the src line
    beside the dst one, matched only where the dst key decided nothing,
    dst then src, xdpfilt_prog.h:152-165).  For both, frames carry ruled
    sources, and destinations ruled for the source direction only (found,
    CHECK_MAP's mask fails, the src key decides)."""
    rng = np.random.default_rng(101)
    rules, v4, ports = one_direction_rules(102, 20000, 2)
    v6 = X.rand_keys(103, 4000, 16)
    rules.v6_keys = v6
    if dirs6 == "both":
        f6 = rng.choice(np.array([1, 2, 3], np.uint64), len(v6))
    else:
        f6 = np.full(len(v6), 2 if dirs6 == "dst" else 1, np.uint64)
    f6[rng.random(len(v6)) < 0.1] |= 4
    rules.v6_vals = f6 | (rng.integers(0, 50, len(v6)).astype(np.uint64) << 6)
    kind = 5 if stride == 1536 else 3
    d1, l1 = X.gen_workload(104, kind, 1 << 15, stride, v4=v4, v6=v6, ports=ports)
    d2, l2 = fuzz_at(105, 1 << 14, stride, rules, ports)
    # a run of IPv6 frames only: whole tiles with more than 16 IPv6 lookups
    fr = d1.reshape(-1, stride)
    six = np.nonzero((fr[:, 12] == 0x86) & (fr[:, 13] == 0xdd))[0]
    if dirs6 == "both":
        # ruled sources on a third of the IPv6 frames; on a sixth, a
        # destination ruled for the source direction only
        srcs = six[::3]
        fr[srcs, 22:38] = v6[rng.integers(0, len(v6), len(srcs))]
        only_src = v6[(f6 & 3) == 1]
        dsts = six[1::6]
        fr[dsts, 38:54] = only_src[rng.integers(0, len(only_src), len(dsts))]
    pick = six[np.arange(1 << 13) % len(six)]
    d3, l3 = fr[pick].reshape(-1), l1[pick]
    data = np.concatenate([d1, d2, d3])
    lens = np.concatenate([l1, l2, l3])
    ov = run_both(G, variant, rules, data, lens, stride, ipv6_capacity=1 << 13)
    assert len(np.unique(ov)) == 3


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_ip"])
@pytest.mark.parametrize("shape", ["sym", "asym"])
@pytest.mark.parametrize("dirs6", ["dst", "src", "both"])
def test_qt_both_ipv4_directions_with_ipv6_rules(G, variant, shape, dirs6):
    """IPv4 rules on both lookup directions (`xdp-filter ip -m src,dst`:
    lookup_verdict_ipv4, dst then src, xdpfilt_prog.h:121-134) beside IPv6
    dst, src or src,dst rules (lookup_verdict_ipv6, :152-165): the index
    kernel's two-stage IPv4 lookup and its in-loop IPv6 lookups together.
    A third of the IPv6 frames carry a ruled source, a quarter of the IPv4
    frames a ruled source; tiles of IPv6 frames only (more than 16 a tile)."""
    rng = np.random.default_rng(141)
    rules, v4, ports = one_direction_rules(142, 20000, 3)
    if shape == "asym":
        f = rules.v4_vals & ~np.uint64(3)
        rules.v4_vals = f | rng.integers(0, 4, len(v4)).astype(np.uint64)
    v6 = X.rand_keys(143, 4000, 16)
    rules.v6_keys = v6
    if dirs6 == "both":
        f6 = rng.choice(np.array([1, 2, 3], np.uint64), len(v6))
    else:
        f6 = np.full(len(v6), 2 if dirs6 == "dst" else 1, np.uint64)
    f6[rng.random(len(v6)) < 0.1] |= 4
    rules.v6_vals = f6 | (rng.integers(0, 50, len(v6)).astype(np.uint64) << 6)
    d1, l1 = X.gen_workload(144, 3, 1 << 16, 64, v4=v4, v6=v6, ports=ports)
    fr = d1.reshape(-1, 64)
    ip4 = np.nonzero((fr[:, 12] == 8) & (fr[:, 13] == 0))[0][::4]
    fr[ip4, 26:30] = v4[(np.arange(len(ip4)) * 7919) % len(v4)]
    six = np.nonzero((fr[:, 12] == 0x86) & (fr[:, 13] == 0xdd))[0]
    srcs = six[::3]
    fr[srcs, 22:38] = v6[rng.integers(0, len(v6), len(srcs))]
    d2, l2 = fuzz_at(145, 1 << 14, 64, rules, ports)
    pick = six[np.arange(1 << 13) % len(six)]
    d3, l3 = fr[pick].reshape(-1), l1[pick]
    data, lens = np.concatenate([d1, d2, d3]), np.concatenate([l1, l2, l3])
    ov = run_both(G, variant, rules, data, lens, 64, ipv6_capacity=1 << 13)
    assert len(np.unique(ov)) == 3


@pytest.mark.timeout(300)
@pytest.mark.parametrize("dirs6", ["dst", "both"])
def test_qt_both_ipv4_directions_ipv6_in_loop(dirs6):
    """With both IPv4 directions live the IPv6 frames are looked up in the
    index kernel's loop, not deferred to the whole-frame walk: a fresh
    process on the diagnostics library leaves deferred packets unclassified
    (XFG_DIAG_MASK=2048) and every IPv6 frame still carries the oracle's
    verdict (tests/gpu_defer_worker.py)."""
    import subprocess
    import sys
    env = dict(os.environ, XFG_LIB="diag")
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "gpu_defer_worker.py"), dirs6],
                       capture_output=True, text=True, timeout=280, env=env)
    assert p.returncode == 0 and "OK" in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_all"])
@pytest.mark.parametrize("neth,path", [(1, 5), (12, 5), (511, 5), (600, 1)])
def test_qt_with_ethernet_rules_live(G, variant, neth, path):
    """Ethernet rules are tested on every frame before its IP keys
    (lookup_verdict_ethernet, xdpfilt_prog.h:187-196,224-227; a hit ends
    the program, even for a frame whose IP header would abort).  With the
    Ethernet map small enough for its LDS key table (at most 512 keys) the
    index kernel takes the batch and answers both Ethernet lookups from the
    table ahead of its IPv4 lookups (path 5); a larger map keeps the generic
    pipelined kernel (path 1).  A fifth of the frames carry a ruled MAC in
    the direction its rule tests, some in the other direction."""
    rng = np.random.default_rng(111 + neth)
    rules, v4, ports = one_direction_rules(111, 20000, 2)
    ek = X.rand_keys(113 + neth, neth, 6)
    rules.eth_keys = ek
    rules.eth_vals = rng.choice(np.array([1, 2, 3], np.uint64), len(ek)) | \
        (rng.integers(0, 30, len(ek)).astype(np.uint64) << 6)
    d1, l1 = X.gen_workload(112, 3, 1 << 15, 64, v4=v4, ports=ports)
    d2, l2 = fuzz_at(114, 1 << 14, 64, rules, ports)
    data, lens = np.concatenate([d1, d2]), np.concatenate([l1, l2])
    d = data.reshape(-1, 64)
    n = len(d)
    pick = rng.choice(n, n // 5, replace=False)
    which = rng.integers(0, len(ek), len(pick))
    half = len(pick) // 2
    d[pick[:half], 0:6] = ek[which[:half]]
    d[pick[half:], 6:12] = ek[which[half:]]
    ov = run_both(G, variant, rules, data, lens, 64, path=path, eth_capacity=1024)
    assert len(np.unique(ov)) == 3


@pytest.mark.timeout(300)
def test_qt_index_past_one_count_pass(G):
    """2.2M IPv4 rules: an index of 2^19 buckets, whose hit log the count
    kernel takes in two passes of its LDS histogram (u16 local indices), at
    a batch of as many packets as the index has slots (the log's bound)."""
    n4 = 2_200_000
    v4 = X.rand_keys(121, int(n4 * 1.02) + 16, 4)[:n4]
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64)
    data, lens = X.gen_workload(122, 3, 1 << 23, 64, v4=v4, dst_permille=600)
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES["xdpfilt_dny_all"], data, lens, rules,
                                   stride=64, nthreads=8)
    f = make_filter(G, "xdpfilt_dny_all", ipv4_capacity=n4)
    f.load_rules(rules)
    v = f.run(data, lens, stride=64)
    assert f.last_path() == 5
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()


@pytest.mark.parametrize("stride", [128, 256, 1536])
def test_qt_window_128_option(G, stride):
    """xfg_open_opts.window = 128: the 128-byte-window kernels (IPv6/TCP's
    doff at byte 66 inside the window, not deferred), with IPv6 rules of one
    direction beside the index, on the fuzz corpus and C3/C5 traffic."""
    rules, v4, ports = one_direction_rules(131, 20000, 2)
    v6 = X.rand_keys(132, 3000, 16)
    rules.v6_keys = v6
    rules.v6_vals = np.full(len(v6), 2, np.uint64)
    kind = 5 if stride == 1536 else 3
    d1, l1 = X.gen_workload(133, kind, 1 << 15, stride, v4=v4, v6=v6, ports=ports)
    d2, l2 = fuzz_at(134, 1 << 14, stride, rules, ports)
    data = np.concatenate([d1, d2])
    lens = np.concatenate([l1, l2])
    run_both(G, "xdpfilt_dny_all", rules, data, lens, stride, ipv6_capacity=1 << 13, window=128)


@pytest.mark.timeout(300)
def test_qt_counts_folded_before_32_bits():
    """The QT-order hit counts are 32-bit (xfg_kargs.qt_hits): the runtime
    folds them into the canonical 64-bit counters before the packets
    classified since the last fold could overflow one. Run in a fresh
    process on the diagnostics library with the fold threshold lowered to
    100,000 packets, so that folds are queued between the launches of one
    timed classify, with and without the hit log: every rule's value and the
    stats equal the oracle's figures for the same number of passes."""
    import subprocess
    import sys
    env = dict(os.environ, XFG_LIB="diag", XFG_QT_FOLD_AT="100000")
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "gpu_fold_worker.py"), "5"],
                       capture_output=True, text=True, timeout=280, env=env)
    assert p.returncode == 0 and "OK" in p.stdout, p.stdout[-2000:] + p.stderr[-4000:]
