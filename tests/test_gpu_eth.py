"""The Ethernet-key kernel (xdp-tools_amd/csrc/xfg_pipee.hip, kernel path 6):
the Ethernet-only programs xdpfilt_alw_eth and xdpfilt_dny_eth over
fixed-stride batches, their map as an LDS key table, against the CPU
restatement (oracle/) -- verdicts, every rule's value (hits << 6 | flags) and
the per-action stats bit-exact.  Contract: xdp-filter/xdpfilt_prog.h:187-196
(lookup_verdict_ethernet: dst, then src), :224-226 (parse_ethhdr, then the
Ethernet check, nothing else), headers/xdp/parsing_helpers.h:100-134
(parse_ethhdr fails only below 14 bytes)."""
import numpy as np
import pytest

import xftools as X
from test_gpu import assert_same, gpu_values, make_filter

pytestmark = pytest.mark.gpu

ETH_VARIANTS = ["xdpfilt_alw_eth", "xdpfilt_dny_eth"]


@pytest.fixture(scope="module")
def G():
    import xfgpu
    return xfgpu


def eth_rules(seed, ne, zero=True):
    """ne random MAC rules (dst, src or both), plus the all-zero MAC."""
    rules, _ = X.random_rules(seed, n4=0, n6=0, ne=ne, nports=0)
    if zero:
        rules.eth_keys = np.vstack([rules.eth_keys, np.zeros((1, 6), np.uint8)])
        rules.eth_vals = np.append(rules.eth_vals, np.uint64(3))
    return rules


def eth_frames(seed, n, stride, rules):
    """Fuzz frames carrying the rule MACs, plus runts (0-13 bytes: ABORTED),
    frames of exactly 14 bytes, all-zero destination or source MACs, and
    lengths past the slot (capped at the stride)."""
    gs = max(stride, 128)   # (the fuzz generator's smallest slot)
    data, lens = X.gen_fuzz(seed, n, gs, rules, np.zeros(0, np.uint16))
    if gs != stride:        # the first `stride` bytes of each (lengths past it capped)
        data = np.ascontiguousarray(data.reshape(n, gs)[:, :stride]).reshape(-1)
    rng = np.random.default_rng(seed)
    d = data.reshape(n, stride)
    runt = rng.choice(n, n // 50, replace=False)
    lens[runt] = rng.integers(0, 14, len(runt))
    lens[rng.choice(n, n // 100, replace=False)] = 14
    zd = rng.choice(n, n // 40, replace=False)
    d[zd, 0:6] = 0
    zs = rng.choice(n, n // 40, replace=False)
    d[zs, 6:12] = 0
    lens[rng.choice(n, 3, replace=False)] = 65000
    return data, lens


def run_check(G, variant, rules, data, lens, stride, path, **caps):
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES[variant], data,
                                   np.minimum(lens, stride).astype(lens.dtype), rules,
                                   stride=stride, nthreads=8)
    f = make_filter(G, variant, **caps)
    f.load_rules(rules)
    v = f.run(data, lens, stride=stride)
    assert f.last_path() == path
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()
    return ov


@pytest.mark.parametrize("variant", ETH_VARIANTS)
@pytest.mark.parametrize("stride,l16", [(64, True), (64, False), (128, True), (1536, False)])
def test_eth_kernel_parity(G, variant, stride, l16):
    rules = eth_rules(7 + stride, 40)
    n = 150011 if stride <= 128 else 20011   # (not a multiple of a tile)
    data, lens = eth_frames(3 + stride, n, stride, rules)
    lens = lens.astype(np.uint16 if l16 else np.uint32)
    ov = run_check(G, variant, rules, data, lens, stride, path=6)
    assert (ov == 0).sum() >= n // 120   # the runts
    assert len(np.unique(ov)) == 3


def test_eth_kernel_c1_rules_many_hits(G):
    """C1's eight hot keys: a quarter of the frames hit, every hit counted
    through the LDS counter cache."""
    rules = X.c1_rules()
    data, lens = X.gen_c1(5, 1 << 20)
    run_check(G, "xdpfilt_alw_eth", rules, data, lens, 64, path=6)


def test_eth_kernel_dst_only_and_src_only_census(G):
    """One lookup direction live (flag census): the other is skipped, as a
    lookup whose mask no key carries cannot hit."""
    for fl in (1, 2):
        rules = eth_rules(31 + fl, 20, zero=False)
        rules.eth_vals = np.full(len(rules.eth_vals), fl, np.uint64)
        data, lens = eth_frames(41 + fl, 70001, 64, rules)
        run_check(G, "xdpfilt_dny_eth", rules, data, lens, 64, path=6)


def test_eth_kernel_empty_map(G):
    rules = X.RuleSet()
    data, lens = eth_frames(9, 30000, 64, eth_rules(9, 4))
    ov = run_check(G, "xdpfilt_alw_eth", rules, data, lens, 64, path=6)
    assert set(np.unique(ov)) <= {0, 2}


def test_eth_kernel_full_table(G):
    """XFG_EK_MAX_KEYS keys: the largest LDS table (1024 entries)."""
    rules = eth_rules(77, 511)
    data, lens = eth_frames(78, 100000, 64, rules)
    run_check(G, "xdpfilt_alw_eth", rules, data, lens, 64, path=6)


def test_eth_map_past_the_table_takes_the_generic_kernel(G):
    rules = eth_rules(91, 700)
    data, lens = eth_frames(92, 60000, 64, rules)
    run_check(G, "xdpfilt_dny_eth", rules, data, lens, 64, path=1)


def test_eth_table_follows_map_edits(G):
    """Keys added, deleted and re-flagged between classifies: each batch is
    classified against the map as it stands (the LDS table rebuilt)."""
    feats = X.VARIANT_FEATURES["xdpfilt_dny_eth"]
    rules = eth_rules(55, 30)
    data, lens = eth_frames(56, 50000, 64, rules)
    f = make_filter(G, "xdpfilt_dny_eth")
    f.load_rules(rules)
    for step in range(4):
        v = f.run(data, lens, stride=64)
        assert f.last_path() == 6
        ov, _, _ = X.run_oracle(feats, data, np.minimum(lens, 64), rules, stride=64)
        np.testing.assert_array_equal(v, ov, err_msg=f"step {step}")
        k = rules.eth_keys
        if step == 0:     # delete a third of the keys
            for key in k[::3]:
                f.delete(G.MAP_ETHERNET, bytes(key))
            keep = np.ones(len(k), bool)
            keep[::3] = False
            rules.eth_keys, rules.eth_vals = k[keep], rules.eth_vals[keep]
        elif step == 1:   # flip every key's direction
            for i, key in enumerate(k):
                nf = int(rules.eth_vals[i]) ^ 3 or 3
                f.update(G.MAP_ETHERNET, bytes(key), nf)
                rules.eth_vals[i] = nf
        elif step == 2:   # new keys
            extra = X.rand_keys(57, 12, 6)
            for key in extra:
                f.update(G.MAP_ETHERNET, bytes(key), 2)
            rules.eth_keys = np.vstack([k, extra])
            rules.eth_vals = np.append(rules.eth_vals, np.full(len(extra), 2, np.uint64))
    f.close()


M32 = 0xffffffff
ETH_SEED = 0x5eed1234 ^ 0xbb67ae85     # xfg_open's default seed ^ the Ethernet map's


def eth_home(keys, slots):
    """The LDS key table's home entry of each MAC (xfg_ek_home, xfg_layout.h:
    multiply-shift over the MAC's two 24-bit halves, the top bits)."""
    k = np.ascontiguousarray(keys, np.uint8).reshape(-1, 6).astype(np.uint64)
    lo = k[:, 0] | (k[:, 1] << 8) | (k[:, 2] << 16) | (k[:, 3] << 24)
    hi = k[:, 4] | (k[:, 5] << 8)
    a = (lo ^ np.uint64(ETH_SEED)) & np.uint64(0xffffff)
    b = ((lo >> np.uint64(24)) | (hi << np.uint64(8))) ^ np.uint64(ETH_SEED >> 8)
    h = (a * np.uint64(0x9e3779) + (b & np.uint64(0xffffff)) * np.uint64(0x7f4a7b)) & np.uint64(M32)
    lg = int(slots).bit_length() - 1
    return (h >> np.uint64(32 - lg)).astype(np.int64)


def test_eth_table_long_probe_chains_and_the_513th_key(G):
    """A full table (512 keys, 1024 entries) with 40 keys sharing one home
    entry, so every lookup reads 40+ entries (ek_disp), then a 513th insert
    (the map past the table: the generic pipelined kernel) and a delete
    back to 512 (the table again): verdicts, every rule value and the stats
    equal the restatement's at each step."""
    feats = X.VARIANT_FEATURES["xdpfilt_alw_eth"]
    cand = X.rand_keys(301, 200000, 6)
    home = eth_home(cand, 1024)
    h0 = np.bincount(home).argmax()
    same = cand[home == h0][:40]
    assert len(same) == 40
    rest = cand[home != h0][:472]
    rng = np.random.default_rng(302)
    rules = X.RuleSet()
    rules.eth_keys = np.vstack([same, rest])
    rules.eth_vals = rng.choice(np.array([1, 2, 3], np.uint64), 512) | \
        (rng.integers(0, 30, 512).astype(np.uint64) << 6)
    data, lens = eth_frames(303, 120000, 64, rules)
    d = data.reshape(-1, 64)
    pick = rng.choice(len(d), len(d) // 5, replace=False)       # the colliding keys, often
    d[pick, 0:6] = same[rng.integers(0, 40, len(pick))]
    f = make_filter(G, "xdpfilt_alw_eth")
    f.load_rules(rules)
    cur = rules.prepared().copy()
    extra = X.rand_keys(304, 1, 6)
    for step, path in enumerate([6, 1, 6]):
        if step == 1:          # the 513th key
            f.update(G.MAP_ETHERNET, bytes(extra[0]), 3)
            cur.eth_keys = np.vstack([cur.eth_keys, extra])
            cur.eth_vals = np.append(cur.eth_vals, np.uint64(3))
        elif step == 2:        # one colliding key deleted: 512 again
            f.delete(G.MAP_ETHERNET, bytes(cur.eth_keys[3]))
            keep = np.ones(len(cur.eth_keys), bool)
            keep[3] = False
            cur.eth_keys, cur.eth_vals = cur.eth_keys[keep], cur.eth_vals[keep]
        v = f.run(data, lens, stride=64)
        assert f.last_path() == path, (step, f.last_path())
        ov, cur, ost = X.run_oracle(feats, data, np.minimum(lens, 64), cur, stride=64)
        assert_same(v, gpu_values(f, G, cur), f.stats(), ov, cur, ost)
        f.stats_reset()
    f.close()


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_all"])
@pytest.mark.parametrize("stride", [64, 1536])
def test_eth_table_beside_ip_rules(G, variant, stride):
    """A few MAC rules beside IPv4, IPv6 and port rules (dny_all / alw_all):
    the generic pipelined kernel answers both Ethernet lookups from the LDS
    key table (a hit ends the program before any IP lookup,
    xdpfilt_prog.h:224-227) and the IP keys by its Bloom and bucket stages:
    verdicts, every rule value and the stats equal the restatement's."""
    rules, pool = X.random_rules(311 + stride, n4=20000, n6=2000, ne=12, nports=30)
    n = 200000 if stride == 64 else 30000
    gs = max(stride, 160)   # (the fuzz generator's slot; a 64-byte slot takes each frame's head)
    g, gl = X.gen_fuzz(312 + stride, n, gs, rules, pool)
    d = np.ascontiguousarray(g.reshape(n, gs)[:, :stride])
    data, lens = d.reshape(-1), np.minimum(gl, stride).astype(np.uint32)
    rng = np.random.default_rng(313)
    k = rules.eth_keys
    dst = rng.choice(n, n // 8, replace=False)
    d[dst, 0:6] = k[rng.integers(0, len(k), len(dst))]
    src = rng.choice(n, n // 8, replace=False)
    d[src, 6:12] = k[rng.integers(0, len(k), len(src))]
    ov = run_check(G, variant, rules, data, lens, stride, path=1,
                   ipv4_capacity=1 << 15, ipv6_capacity=1 << 12, eth_capacity=64)
    assert len(np.unique(ov)) == 3
