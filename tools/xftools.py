"""tools/xftools.py — test / bench tooling (NOT the product).

ctypes bindings for:
  * tools/libxfsynth.so        seeded synthetic traffic (workloads C2..C5, fuzz)
  * oracle/build/liboracle.so  our CPU restatement of the xdpfilt_* program

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use the
oracle binding, and only as the checker / the CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# XFG_LIB=asan: the sanitizer builds (make asan; tools/asan_suite.sh)
_ASAN = os.environ.get("XFG_LIB") == "asan"

FEAT_TCP, FEAT_UDP, FEAT_IPV6, FEAT_IPV4, FEAT_ETHERNET = 1, 2, 4, 8, 16
FEAT_ALL = 31
FEAT_ALLOW, FEAT_DENY = 32, 64
FLAG_SRC, FLAG_DST, FLAG_TCP, FLAG_UDP = 1, 2, 4, 8
COUNTER_SHIFT = 6

# xdp-filter/Makefile:3-6 order, with each program's _features word
# (xdp-filter/xdpfilt_prog.h:313-315 evaluated for each xdpfilt_*.c).
VARIANTS = [
    ("xdpfilt_dny_udp", FEAT_UDP | FEAT_DENY),
    ("xdpfilt_dny_tcp", FEAT_TCP | FEAT_DENY),
    ("xdpfilt_dny_ip", FEAT_IPV4 | FEAT_IPV6 | FEAT_DENY),
    ("xdpfilt_dny_eth", FEAT_ETHERNET | FEAT_DENY),
    ("xdpfilt_dny_all", FEAT_ALL | FEAT_DENY),
    ("xdpfilt_alw_udp", FEAT_UDP | FEAT_ALLOW),
    ("xdpfilt_alw_tcp", FEAT_TCP | FEAT_ALLOW),
    ("xdpfilt_alw_ip", FEAT_IPV4 | FEAT_IPV6 | FEAT_ALLOW),
    ("xdpfilt_alw_eth", FEAT_ETHERNET | FEAT_ALLOW),
    ("xdpfilt_alw_all", FEAT_ALL | FEAT_ALLOW),
]
VARIANT_FEATURES = dict(VARIANTS)

_u8p = C.POINTER(C.c_uint8)
_u16p = C.POINTER(C.c_uint16)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


def ptr(a, t=_u8p):
    if a is None:
        return None
    return a.ctypes.data_as(t)


@dataclass
class RuleSet:
    """Rule maps in the reference's value encoding (hits << 6 | flags)."""
    ports: np.ndarray = field(default_factory=lambda: np.zeros(65536, np.uint64))
    v4_keys: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), np.uint8))
    v4_vals: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    v6_keys: np.ndarray = field(default_factory=lambda: np.zeros((0, 16), np.uint8))
    v6_vals: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    eth_keys: np.ndarray = field(default_factory=lambda: np.zeros((0, 6), np.uint8))
    eth_vals: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))

    def copy(self) -> "RuleSet":
        return RuleSet(*(np.array(getattr(self, f), copy=True) for f in
                         ("ports", "v4_keys", "v4_vals", "v6_keys", "v6_vals",
                          "eth_keys", "eth_vals")))

    def prepared(self):
        """Contiguous arrays of the right dtypes (for ctypes)."""
        r = RuleSet(np.ascontiguousarray(self.ports, np.uint64),
                    np.ascontiguousarray(self.v4_keys, np.uint8).reshape(-1, 4),
                    np.ascontiguousarray(self.v4_vals, np.uint64),
                    np.ascontiguousarray(self.v6_keys, np.uint8).reshape(-1, 16),
                    np.ascontiguousarray(self.v6_vals, np.uint64),
                    np.ascontiguousarray(self.eth_keys, np.uint8).reshape(-1, 6),
                    np.ascontiguousarray(self.eth_vals, np.uint64))
        return r


def port_key(port: int) -> int:
    """Key of filter_ports for a host-order port: htons(port) as u32
    (xdp-filter/xdp-filter.c:634)."""
    return ((port & 0xff) << 8) | (port >> 8)


# ----------------------------------------------------------------- synth
_synth = None


def synth():
    global _synth
    if _synth is None:
        lib = C.CDLL(os.path.join(ROOT, "tools", "build-asan" if _ASAN else "", "libxfsynth.so"))
        lib.xfs_gen_workload.argtypes = [C.c_uint64, C.c_int, C.c_uint64, C.c_uint32,
                                         _u8p, _u32p, _u8p, C.c_uint32, _u8p, C.c_uint32,
                                         _u16p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        lib.xfs_gen_fuzz.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, _u8p, _u32p,
                                     _u8p, C.c_uint32, _u8p, C.c_uint32, _u8p, C.c_uint32,
                                     _u16p, C.c_uint32]
        lib.xfs_rand_keys.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, _u8p]
        _synth = lib
    return _synth


def rand_keys(seed: int, n: int, keylen: int, distinct: bool = True) -> np.ndarray:
    out = np.zeros((n, keylen), np.uint8)
    if n:
        synth().xfs_rand_keys(seed, n, keylen, ptr(out))
    if distinct and n:
        # first occurrence of each key (a flat view sorts far faster than axis=0)
        flat = (out.view("<u4").ravel() if keylen == 4 else
                out.view(np.dtype((np.void, keylen))).ravel())
        _, idx = np.unique(flat, return_index=True)
        out = out[np.sort(idx)]
    return out


def gen_workload(seed, kind, n, stride, v4=None, v6=None, ports=None,
                 dst_permille=500, port_permille=250, bad_permille=10,
                 data=None, lens=None):
    """Synthetic batch for configuration C<kind>; returns (data u8[n*stride], lens u32[n])."""
    if data is None:
        data = np.zeros(n * stride, np.uint8)
    if lens is None:
        lens = np.zeros(n, np.uint32)
    v4 = np.ascontiguousarray(v4 if v4 is not None else np.zeros((0, 4), np.uint8), np.uint8)
    v6 = np.ascontiguousarray(v6 if v6 is not None else np.zeros((0, 16), np.uint8), np.uint8)
    ports = np.ascontiguousarray(ports if ports is not None else np.zeros(0, np.uint16), np.uint16)
    rc = synth().xfs_gen_workload(seed, kind, n, stride, ptr(data), ptr(lens, _u32p),
                                  ptr(v4), len(v4), ptr(v6), len(v6), ptr(ports, _u16p),
                                  len(ports), dst_permille, port_permille, bad_permille)
    if rc:
        raise ValueError("xfs_gen_workload failed (stride too small?)")
    return data, lens


C1_MACS = np.array([[2, 0, 0, 0, 0, i] for i in range(1, 9)], np.uint8)   # 02:00:00:00:00:0{1..8}


def c1_rules():
    """C1's rule set: the 8 MACs 02:00:00:00:00:0{1..8}, the
    first 4 dst rules, the last 4 src rules (`xdp-filter ether -m dst|src`)."""
    rules = RuleSet()
    rules.eth_keys = C1_MACS.copy()
    rules.eth_vals = np.array([2] * 4 + [1] * 4, np.uint64)
    return rules


def gen_c1(seed, n, stride=64, hit_permille=250, bad_permille=10, data=None, lens=None):
    """C1's traffic: 64 B Ethernet/IPv4/UDP frames with random MACs, a ruled
    MAC (where its rule tests it) in `hit_permille` of them, and the
    Appendix A malformed classes in `bad_permille`."""
    return gen_workload(seed, 1, n, stride, v6=C1_MACS, dst_permille=hit_permille,
                        port_permille=0, bad_permille=bad_permille, data=data, lens=lens)


def gen_fuzz(seed, n, stride=160, rules: RuleSet | None = None, port_pool=None):
    data = np.zeros(n * stride, np.uint8)
    lens = np.zeros(n, np.uint32)
    r = (rules or RuleSet()).prepared()
    ports = np.ascontiguousarray(port_pool if port_pool is not None else
                                 np.zeros(0, np.uint16), np.uint16)
    rc = synth().xfs_gen_fuzz(seed, n, stride, ptr(data), ptr(lens, _u32p),
                              ptr(r.v4_keys), len(r.v4_keys), ptr(r.v6_keys), len(r.v6_keys),
                              ptr(r.eth_keys), len(r.eth_keys), ptr(ports, _u16p), len(ports))
    if rc:
        raise ValueError("xfs_gen_fuzz failed")
    return data, lens


def random_rules(seed, n4=64, n6=32, ne=16, nports=24, flag_mode="any"):
    """Random rule set with random flag combinations (incl. src-only/dst-only
    and proto-restricted port rules).  Returns (RuleSet, port_pool)."""
    rng = np.random.default_rng(seed)

    def flags(n, ip=True):
        if flag_mode == "dst":
            return np.full(n, FLAG_DST, np.uint64)
        f = rng.integers(1, 16, n).astype(np.uint64)
        if ip:   # ip/ether rules carry src/dst only (xdp-filter.c:784-786)
            f = rng.integers(1, 4, n).astype(np.uint64)
        return f

    rs = RuleSet()
    rs.v4_keys = rand_keys(seed * 11 + 1, n4, 4)
    rs.v4_vals = flags(len(rs.v4_keys)) | (rng.integers(0, 1000, len(rs.v4_keys)).astype(np.uint64) << 6)
    rs.v6_keys = rand_keys(seed * 11 + 2, n6, 16)
    rs.v6_vals = flags(len(rs.v6_keys)) | (rng.integers(0, 1000, len(rs.v6_keys)).astype(np.uint64) << 6)
    rs.eth_keys = rand_keys(seed * 11 + 3, ne, 6)
    rs.eth_vals = flags(len(rs.eth_keys))
    pool = rng.choice(65536, nports, replace=False).astype(np.uint16)
    for p in pool:
        rs.ports[port_key(int(p))] = np.uint64(int(rng.integers(1, 16)) | (int(rng.integers(0, 50)) << 6))
    return rs, pool


# ----------------------------------------------------------------- oracle
_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        lib = C.CDLL(os.path.join(ROOT, "oracle", "build-asan" if _ASAN else "build", "liboracle.so"))
        lib.xfo_map_new.restype = C.c_void_p
        lib.xfo_map_new.argtypes = [C.c_uint32, C.c_uint32, _u8p]
        lib.xfo_map_new_hashed.restype = C.c_void_p
        lib.xfo_map_new_hashed.argtypes = [C.c_uint32, C.c_uint32, _u8p, _u64p]
        lib.xfo_map_free.argtypes = [C.c_void_p]
        common = [C.c_uint32, _u8p, _u64p, C.c_uint32, C.c_void_p, C.c_int, C.c_uint64, _u64p]
        lib.xfo_run.argtypes = common + [C.c_void_p, _u64p, C.c_void_p, _u64p, C.c_void_p,
                                         _u64p, _u8p, _u64p]
        lib.xfo_run_mt.argtypes = common + [C.c_void_p, _u64p, C.c_uint32, C.c_void_p, _u64p,
                                            C.c_uint32, C.c_void_p, _u64p, C.c_uint32,
                                            _u8p, _u64p, C.c_int]
        _oracle = lib
    return _oracle


class OracleMaps:
    """Prebuilt exact-match indexes for a RuleSet (reusable across runs)."""

    def __init__(self, rules: RuleSet, hashed: bool = False):
        """hashed: add the hash index (one probe per lookup, the reference's
        BPF hash-map cost model: the CPU baseline); results are identical."""
        lib = oracle()
        self.rules = rules.prepared()
        r = self.rules
        if hashed:   # (the slots carry the rules' flags as they are now)
            self.m4 = lib.xfo_map_new_hashed(len(r.v4_keys), 4, ptr(r.v4_keys), ptr(r.v4_vals, _u64p))
            self.m6 = lib.xfo_map_new_hashed(len(r.v6_keys), 16, ptr(r.v6_keys), ptr(r.v6_vals, _u64p))
            self.me = lib.xfo_map_new_hashed(len(r.eth_keys), 6, ptr(r.eth_keys),
                                             ptr(r.eth_vals, _u64p))
        else:
            self.m4 = lib.xfo_map_new(len(r.v4_keys), 4, ptr(r.v4_keys))
            self.m6 = lib.xfo_map_new(len(r.v6_keys), 16, ptr(r.v6_keys))
            self.me = lib.xfo_map_new(len(r.eth_keys), 6, ptr(r.eth_keys))

    def __del__(self):
        try:
            lib = oracle()
            for m in (self.m4, self.m6, self.me):
                lib.xfo_map_free(m)
        except Exception:
            pass


def run_oracle(features, data, lens, rules: RuleSet, stride=0, offsets=None,
               nthreads=1, maps: OracleMaps | None = None, stats=None):
    """Run the CPU restatement; returns (verdicts, rules_after, stats[5,2])."""
    lib = oracle()
    maps = maps or OracleMaps(rules)
    r = rules.prepared().copy()
    n = len(lens)
    verdicts = np.zeros(n, np.uint8)
    st = np.zeros(10, np.uint64) if stats is None else stats.reshape(10)
    lens_u16 = lens.dtype == np.uint16
    lens = np.ascontiguousarray(lens)
    offs = None if offsets is None else np.ascontiguousarray(offsets, np.uint64)
    if nthreads <= 1:
        rc = lib.xfo_run(features, ptr(data), ptr(offs, _u64p), stride, lens.ctypes.data,
                         int(lens_u16), n, ptr(r.ports, _u64p), maps.m4, ptr(r.v4_vals, _u64p),
                         maps.m6, ptr(r.v6_vals, _u64p), maps.me, ptr(r.eth_vals, _u64p),
                         ptr(verdicts), ptr(st, _u64p))
    else:
        rc = lib.xfo_run_mt(features, ptr(data), ptr(offs, _u64p), stride, lens.ctypes.data,
                            int(lens_u16), n, ptr(r.ports, _u64p),
                            maps.m4, ptr(r.v4_vals, _u64p), len(r.v4_vals),
                            maps.m6, ptr(r.v6_vals, _u64p), len(r.v6_vals),
                            maps.me, ptr(r.eth_vals, _u64p), len(r.eth_vals),
                            ptr(verdicts), ptr(st, _u64p), nthreads)
    if rc:
        raise RuntimeError("oracle run failed")
    return verdicts, r, st.reshape(5, 2)


