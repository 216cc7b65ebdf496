"""Known-answer frames and rules for the xdpfilt_* programs.

Two sources, both restated as frame + rule + expected verdict:
  * SURVEY.md Appendix A — edge semantics observed by running the unmodified
    reference (host-compiled) on hand-built frames;
  * the reference's behavioural tests: xdp-filter/tests/test-xdp-filter.sh
    (ports/ipv4/ipv6/ether allow+deny, ARP request/reply/gratuitous, NDISC
    NS/NA, src vs dst, TCP and UDP on one port) and
    xdp-filter/tests/test_basic.py:156-232 (IPv6 extension headers before
    UDP dport 55555; IPv4-mapped IPv6 addresses are distinct keys).
Expected actions: 0 ABORTED, 1 DROP, 2 PASS.

Each row may also carry
  * SOURCE[name]: the reference file:line it restates (rows without one
    restate SURVEY.md Appendix A);
  * HIT[name]: the rule whose counter a HIT verdict bumps -- ("port", p),
    ("v4", addr), ("v6", addr) or ("eth", mac).  CHECK_MAP adds
    1 << COUNTER_SHIFT to the matched rule's value and nothing else
    (xdp-filter/xdpfilt_prog.h:56-64), so for a variant whose expected verdict
    is its VERDICT_HIT (PASS under deny, DROP under allow) that rule's hits
    grow by one; a MISS or an ABORTED frame changes no counter.
"""
from __future__ import annotations

import struct

import numpy as np

import pktbuild as P

ABORTED, DROP, PASS = 0, 1, 2
SRC, DST, TCPF, UDPF = 1, 2, 4, 8

# Addresses with no rules unless stated.
A_SRC, A_DST = "192.0.2.1", "192.0.2.2"
A6_SRC, A6_DST = "2001:db8::1", "2001:db8::2"

# The reference test bed (lib/testing/test_runner.sh:361-397): the program
# runs on the OUTSIDE end of a veth pair and sees what the namespace's INSIDE
# end sends; OUTSIDE = <prefix>1, INSIDE = <prefix>2 in 10.11.<n>.0/24 and
# fc42:dead:cafe:<n>::/64.  Each test function loads its own rules; here the
# rows share one rule set, so each phase gets its own <n>: 2 = a dst rule on
# OUTSIDE (`xdp-filter ip $OUTSIDE_IP*`), 4 = a src rule on INSIDE (`ip -m src
# $INSIDE_IP*`), 3 = no address rule (the port tests).
OUT4, IN4 = "10.11.2.1", "10.11.2.2"
OUT4_S, IN4_SRC = "10.11.4.1", "10.11.4.2"
OUT6, IN6 = "fc42:dead:cafe:2::1", "fc42:dead:cafe:2::2"
OUT6_S, IN6_SRC = "fc42:dead:cafe:4::1", "fc42:dead:cafe:4::2"
OUT6_N, IN6_N = "fc42:dead:cafe:3::1", "fc42:dead:cafe:3::2"
OUT4_N, IN4_N = "10.11.3.1", "10.11.3.2"
OUT_MAC, IN_MAC = "02:00:00:00:02:01", "02:00:00:00:02:02"
OUT_MAC_S, IN_MAC_SRC = "02:00:00:00:04:01", "02:00:00:00:04:02"


def port_key(p):
    return ((p & 0xff) << 8) | (p >> 8)


def kat_rules():
    import xftools as X
    rs = X.RuleSet()
    rs.ports[port_key(53)] = DST | TCPF | UDPF
    rs.ports[port_key(55555)] = DST | UDPF
    rs.ports[port_key(2000)] = SRC | TCPF         # tcp source-port rule
    rs.ports[port_key(3000)] = DST | UDPF         # udp only: TCP to 3000 misses
    rs.ports[port_key(4000)] = SRC | DST | UDPF | TCPF
    # the reference tests' `xdp-filter port N` (default mode dst, tcp|udp,
    # xdp-filter/xdp-filter.c:647-651) and test_basic.py's default-packet ports
    rs.ports[port_key(10000)] = DST | TCPF | UDPF
    rs.ports[port_key(60002)] = DST | TCPF | UDPF
    rs.ports[port_key(60001)] = SRC | TCPF | UDPF
    v4 = [("10.0.0.1", SRC), ("10.11.1.2", DST), ("10.11.1.9", SRC | DST),
          ("10.22.0.1", SRC), ("10.33.0.1", DST), ("0.0.0.0", DST),
          (OUT4, DST), (IN4_SRC, SRC)]
    rs.v4_keys = np.array([list(P.ip4(a)) for a, _ in v4], np.uint8)
    rs.v4_vals = np.array([f | (7 << 6) for _, f in v4], np.uint64)   # pre-existing hits
    v6 = [("fc00:dead:cafe:1::2", DST), ("fc00:dead:cafe:1::1", SRC),
          ("fc00::99", SRC | DST), ("::ffff:10.11.1.1", SRC), ("fe80::1", DST),
          ("fe80::2", SRC), ("::", SRC), (OUT6, DST), (IN6_SRC, SRC)]
    rs.v6_keys = np.array([list(P.ip6(a)) for a, _ in v6], np.uint8)
    rs.v6_vals = np.array([f for _, f in v6], np.uint64)
    macs = [("aa:00:00:00:00:01", DST), ("aa:00:00:00:00:02", SRC),
            ("aa:00:00:00:00:03", SRC | DST), ("00:00:00:00:00:00", SRC),
            (OUT_MAC, DST), (IN_MAC_SRC, SRC)]
    rs.eth_keys = np.array([list(P.mac(m)) for m, _ in macs], np.uint8)
    rs.eth_vals = np.array([f for _, f in macs], np.uint64)
    return rs


def _v4udp(dport=53, sport=12345, src=A_SRC, dst=A_DST, e=None, **kw):
    return (e or P.eth()) + P.ipv4(src, dst, 17, payload=P.udp(sport, dport), **kw)


def _v4tcp(dport=53, sport=12345, doff=5, src=A_SRC, dst=A_DST):
    return P.eth() + P.ipv4(src, dst, 6, payload=P.tcp(sport, dport, doff))


def _v6(nh, payload, src=A6_SRC, dst=A6_DST):
    return P.eth(ethertype=0x86DD) + P.ipv6(src, dst, nh, payload)


def _hbh_chain(n, final=17):
    b = b""
    for i in range(n):
        b += P.ext(0 if i + 1 < n else final, 0)
    return b


class Ann:
    """A row's annotation: the rule a HIT bumps, the reference source."""

    def __init__(self, hit=None, src=None):
        self.hit, self.src = hit, src


SOURCE: dict[str, str] = {}
HIT: dict[str, tuple] = {}

SH = "xdp-filter/tests/test-xdp-filter.sh"
PORTS_SH = SH + ":83-130"        # check_port, test_ports_allow/deny
IPV6_SH = SH + ":132-174"        # check_ping6/ndisc6, test_ipv6_allow/deny
IPV4_SH = SH + ":176-229"        # check_ping4/arp/arp_src, test_ipv4_allow/deny
ETHER_SH = SH + ":231-259"       # test_ether_allow/deny


def kat_frames():
    """List of (name, frame, {variant: expected}) — expectations only where
    the source states them; the golden fixture pins every variant.  Fills
    SOURCE and HIT (module level) as a side effect."""
    F = []
    SOURCE.clear()
    HIT.clear()

    def add(name, *args, **exp):
        ann, frame = (args[0], args[1]) if isinstance(args[0], Ann) else (Ann(), args[0])
        F.append((name, bytes(frame), {("xdpfilt_" + k): v for k, v in exp.items()}))
        if ann.hit is not None:
            HIT[name] = ann.hit
        SOURCE[name] = ann.src or "SURVEY.md Appendix A"

    # ---- SURVEY.md Appendix A ------------------------------------------------
    add("A1 ipv4/udp dst 53, port rule dst|udp", Ann(hit=("port", 53)), _v4udp(53), dny_all=PASS)
    add("A2 ipv4 dst 10.0.0.1 with src-only rule", _v4udp(9, dst="10.0.0.1"), dny_all=DROP)
    add("A3 udp len 7", P.eth() + P.ipv4(A_SRC, A_DST, 17, payload=P.udp(1, 2, length=7)),
        dny_all=ABORTED)
    add("A4 ipv4/udp truncated to 41B", _v4udp(53)[:41], dny_all=ABORTED)
    # ihl = 0: the UDP header is parsed at the IP header itself; bytes o+2..3
    # (total length) act as the dest port and o+4..5 (id) as the UDP length.
    ip0 = struct.pack("!BBHHHBBH4s4s", 0x40, 0, 53, 0x0100, 0, 64, 17, 0,
                      P.ip4(A_SRC), P.ip4(A_DST))
    add("A5 ipv4 ihl=0, 'dport' = total length 53", Ann(hit=("port", 53)), P.eth() + ip0 + b"\0" * 8, dny_all=PASS)
    add("A6 ipv6/udp 54B, no L4 bytes", _v6(17, b""), dny_all=ABORTED)
    add("A7 ipv6 + 4 HBH + udp 53", Ann(hit=("port", 53)), _v6(0, _hbh_chain(4) + P.udp(1, 53)),
        dny_all=PASS, alw_tcp=PASS, dny_ip=DROP)
    add("A8 ipv6 + 5 HBH + udp 53", Ann(hit=("port", 53)), _v6(0, _hbh_chain(5) + P.udp(1, 53)),
        dny_all=PASS, alw_tcp=PASS, dny_ip=DROP)
    add("A9 ipv6 + 6 HBH + udp", _v6(0, _hbh_chain(6) + P.udp(1, 53)),
        dny_all=ABORTED, alw_tcp=ABORTED, dny_ip=ABORTED)
    add("A10 ndisc NS truncated target", _v6(58, P.ndisc_ns("fe80::5")[:16]),
        dny_all=ABORTED, alw_tcp=ABORTED, dny_ip=ABORTED)
    add("A11 ndisc NS full target, no rule", _v6(58, P.ndisc_ns("fe80::5")),
        dny_all=DROP, alw_tcp=PASS, dny_ip=DROP)
    add("A12 all-zero ARP", P.eth(ethertype=0x0806) + b"\0" * 28,
        dny_all=ABORTED, alw_tcp=PASS, dny_ip=ABORTED)
    add("A13 ARP request sip 10.0.0.1 (src rule)", Ann(hit=("v4", "10.0.0.1")), P.eth(ethertype=0x0806) +
        P.arp(1, sip="10.0.0.1", tip=A_DST), dny_all=PASS)
    add("A14 ARP bad hln", P.eth(ethertype=0x0806) + P.arp(1, hln=5), dny_all=ABORTED)
    add("A15 ipv4/tcp dst 53 doff 5", Ann(hit=("port", 53)), _v4tcp(53), dny_all=PASS, alw_tcp=DROP, dny_ip=DROP)
    add("A16 ipv4/tcp doff 15 > frame", _v4tcp(53, doff=15)[:54],
        dny_all=ABORTED, alw_tcp=ABORTED, dny_ip=DROP)
    tcp0 = bytearray(_v4tcp(53))
    tcp0[14 + 20 + 12] = 0
    add("A17 ipv4/tcp doff 0", Ann(hit=("port", 53)), tcp0, dny_all=PASS, alw_tcp=DROP, dny_ip=DROP)
    add("A18 truncated VLAN tag (16B)", P.eth(ethertype=0x8100) + b"\x00\x05", dny_all=DROP)
    add("A19 VLAN + ipv4/udp 53", Ann(hit=("port", 53)), P.eth(vlans=[(0x8100, 5)]) +
        P.ipv4(A_SRC, A_DST, 17, payload=P.udp(1, 53)), dny_all=PASS)
    add("A20 LLDP", P.eth(ethertype=0x88CC) + b"\x02\x07" + b"\0" * 40, dny_all=DROP)
    add("A21 13B runt", P.eth()[:13], dny_all=ABORTED)

    # ---- test-xdp-filter.sh: ports (src/dst, tcp+udp on one port) -----------
    add("P1 udp dport 53", Ann(hit=("port", 53), src=PORTS_SH), _v4udp(53), dny_udp=PASS, alw_udp=DROP, dny_tcp=DROP)
    add("P2 tcp dport 53", Ann(hit=("port", 53), src=PORTS_SH), _v4tcp(53), dny_tcp=PASS, alw_tcp=DROP, dny_udp=DROP)
    add("P3 udp sport 53 (dst-only rule)", Ann(src=PORTS_SH), _v4udp(9, sport=53), dny_udp=DROP, alw_udp=PASS)
    add("P4 tcp sport 2000 (src|tcp)", Ann(hit=("port", 2000), src=PORTS_SH), _v4tcp(9, sport=2000), dny_tcp=PASS, alw_tcp=DROP)
    add("P5 udp sport 2000 (rule is tcp-only)", Ann(src=PORTS_SH), _v4udp(9, sport=2000), dny_udp=DROP, alw_udp=PASS)
    add("P6 tcp dport 3000 (rule is udp-only)", Ann(src=PORTS_SH), _v4tcp(3000), dny_tcp=DROP, alw_all=PASS)
    add("P7 udp dport 3000", Ann(hit=("port", 3000), src=PORTS_SH), _v4udp(3000), dny_udp=PASS)
    add("P8 udp src+dst 4000", Ann(hit=("port", 4000), src=PORTS_SH), _v4udp(4000, sport=4000), dny_all=PASS)
    add("P9 ipv6/udp dport 53", Ann(hit=("port", 53), src=PORTS_SH), _v6(17, P.udp(7, 53)), dny_udp=PASS, dny_ip=DROP)
    add("P10 ipv6/tcp dport 53", Ann(hit=("port", 53), src=PORTS_SH), _v6(6, P.tcp(7, 53)), dny_tcp=PASS)
    # ---- ipv4 src/dst (ping) ----------------------------------------------
    add("I1 icmp to 10.11.1.2 (dst rule)", Ann(hit=("v4", "10.11.1.2"), src=IPV4_SH), P.eth() + P.ipv4(A_SRC, "10.11.1.2", 1,
                                                           payload=P.icmp4_echo()),
        dny_ip=PASS, alw_ip=DROP, dny_udp=DROP)
    add("I2 icmp from 10.11.1.2 (dst-only rule)", Ann(src=IPV4_SH), P.eth() + P.ipv4("10.11.1.2", A_SRC, 1,
                                                                   payload=P.icmp4_echo()),
        dny_ip=DROP, alw_ip=PASS)
    add("I3 icmp from 10.22.0.1 (src rule)", Ann(hit=("v4", "10.22.0.1"), src=IPV4_SH), P.eth() + P.ipv4("10.22.0.1", A_DST, 1,
                                                              payload=P.icmp4_echo()),
        dny_ip=PASS)
    add("I4 icmp 10.11.1.9 both ways", Ann(hit=("v4", "10.11.1.9"), src=IPV4_SH), P.eth() + P.ipv4("10.11.1.9", "10.11.1.9", 1,
                                                        payload=P.icmp4_echo()), dny_ip=PASS)
    add("I5 dst 0.0.0.0 (zero key rule)", Ann(hit=("v4", "0.0.0.0")), P.eth() + P.ipv4(A_SRC, "0.0.0.0", 1,
                                                           payload=P.icmp4_echo()), dny_ip=PASS)
    add("I6 ipv4 options ihl 7 + udp 53", Ann(hit=("port", 53)), P.eth() + P.ipv4(A_SRC, A_DST, 17, ihl=7,
                                                           payload=P.udp(1, 53)), dny_all=PASS)
    add("I7 ipv4 fragment (MF) udp 53", Ann(hit=("port", 53)), P.eth() + P.ipv4(A_SRC, A_DST, 17, frag=0x2000,
                                                         payload=P.udp(1, 53)), dny_all=PASS)
    # ---- ipv6 src/dst --------------------------------------------------------
    add("S1 ping6 to fc00:dead:cafe:1::2", Ann(hit=("v6", "fc00:dead:cafe:1::2"), src=IPV6_SH), _v6(58, P.icmp6(128, 0, b"abcd"),
                                             dst="fc00:dead:cafe:1::2"), dny_ip=PASS)
    add("S2 ping6 from fc00:dead:cafe:1::1", Ann(hit=("v6", "fc00:dead:cafe:1::1"), src=IPV6_SH), _v6(58, P.icmp6(128, 0, b"abcd"),
                                               src="fc00:dead:cafe:1::1"), dny_ip=PASS)
    add("S3 ping6 from fc00:dead:cafe:1::2 (dst-only)", Ann(src=IPV6_SH), _v6(58, P.icmp6(128, 0, b"abcd"),
                                                          src="fc00:dead:cafe:1::2"), dny_ip=DROP)
    add("S4 ping6 src :: (zero key, src rule)", Ann(hit=("v6", "::")), _v6(58, P.icmp6(128, 0, b"abcd"), src="::"),
        dny_ip=PASS)
    # ---- ARP ------------------------------------------------------------------
    add("R1 ARP request tip 10.11.1.2 (dst)", Ann(hit=("v4", "10.11.1.2"), src=IPV4_SH), P.eth(ethertype=0x0806) +
        P.arp(1, sip=A_SRC, tip="10.11.1.2"), dny_ip=PASS, alw_ip=DROP)
    add("R2 ARP reply tip 10.11.1.2 (tip as SRC: dst rule misses)", Ann(src=IPV4_SH), P.eth(ethertype=0x0806) +
        P.arp(2, sip=A_SRC, tip="10.11.1.2"), dny_ip=DROP)
    add("R3 ARP reply tip 10.22.0.1 (src rule)", Ann(hit=("v4", "10.22.0.1"), src=IPV4_SH), P.eth(ethertype=0x0806) +
        P.arp(2, sip=A_SRC, tip="10.22.0.1"), dny_ip=PASS)
    add("R4 gratuitous ARP sip=tip=10.22.0.1", Ann(hit=("v4", "10.22.0.1"), src=IPV4_SH), P.eth(ethertype=0x0806) +
        P.arp(1, sip="10.22.0.1", tip="10.22.0.1"), dny_ip=PASS)
    add("R5 ARP op 3 with tip 10.11.1.2", P.eth(ethertype=0x0806) +
        P.arp(3, sip=A_SRC, tip="10.11.1.2"), dny_ip=DROP)
    add("R6 ARP pro 0x86dd", P.eth(ethertype=0x0806) + P.arp(1, pro=0x86DD), dny_ip=ABORTED)
    add("R7 ARP under dny_udp (no ipv4 feature) => miss", P.eth(ethertype=0x0806) + b"\0" * 28,
        dny_udp=DROP, alw_eth=PASS)
    # ---- NDISC ---------------------------------------------------------------
    add("N1 NS target fe80::1 (dst)", Ann(hit=("v6", "fe80::1"), src=IPV6_SH), _v6(58, P.ndisc_ns("fe80::1")), dny_ip=PASS)
    add("N2 NA target fe80::1 (as SRC: miss)", Ann(src=IPV6_SH), _v6(58, P.ndisc_na("fe80::1")), dny_ip=DROP)
    add("N3 NA target fe80::2 (src)", Ann(hit=("v6", "fe80::2"), src=IPV6_SH), _v6(58, P.ndisc_na("fe80::2")), dny_ip=PASS)
    add("N4 NS target fe80::2 (as DST: miss)", Ann(src=IPV6_SH), _v6(58, P.ndisc_ns("fe80::2")), dny_ip=DROP)
    add("N5 icmp6 truncated header", _v6(58, P.icmp6(128)[:6]), dny_udp=ABORTED, dny_eth=DROP)
    # ---- ether src/dst --------------------------------------------------------
    add("E1 dst aa:..:01", Ann(hit=("eth", "aa:00:00:00:00:01"), src=ETHER_SH), _v4udp(9, e=P.eth(dst=P.mac("aa:00:00:00:00:01"))),
        dny_eth=PASS, alw_eth=DROP, dny_ip=DROP)
    add("E2 src aa:..:01 (dst-only)", Ann(src=ETHER_SH), _v4udp(9, e=P.eth(src=P.mac("aa:00:00:00:00:01"))),
        dny_eth=DROP)
    add("E3 src aa:..:02", Ann(hit=("eth", "aa:00:00:00:00:02"), src=ETHER_SH), _v4udp(9, e=P.eth(src=P.mac("aa:00:00:00:00:02"))), dny_eth=PASS)
    add("E4 src 00:..:00 (zero key)", Ann(hit=("eth", "00:00:00:00:00:00")), _v4udp(9, e=P.eth(src=b"\0" * 6)), dny_eth=PASS)
    add("E5 mac rule + runt 13B", P.eth(dst=P.mac("aa:00:00:00:00:01"))[:13], dny_eth=ABORTED)
    # ---- test_basic.py:156-185 — IPv6 extension headers then UDP 55555 --------
    for kind, nh, e in (("routing", 43, P.ext(17, 2)), ("hbh", 0, P.ext(17, 0)),
                        ("dstopt", 60, P.ext(17, 1)), ("frag", 44, P.ext(17, kind="frag")),
                        ("ah", 51, P.ext(17, 1, kind="ah")), ("mh", 135, P.ext(17, 0))):
        add(f"X {kind} + udp 55555", Ann(hit=("port", 55555), src="xdp-filter/tests/test_basic.py:156-185"), _v6(nh, e + P.udp(1, 55555)), dny_udp=PASS, alw_udp=DROP)
    # ---- test_basic.py:188-232 — IPv4-mapped IPv6 is a distinct key -----------
    add("M1 ipv4 from 10.11.1.1 vs rule ::ffff:10.11.1.1", Ann(src="xdp-filter/tests/test_basic.py:188-232"), P.eth() +
        P.ipv4("10.11.1.1", A_DST, 1, payload=P.icmp4_echo()), dny_ip=DROP)
    add("M2 ipv6 from ::ffff:10.11.1.1", Ann(hit=("v6", "::ffff:10.11.1.1"), src="xdp-filter/tests/test_basic.py:188-232"), _v6(58, P.icmp6(128), src="::ffff:10.11.1.1"),
        dny_ip=PASS)
    # ---- more edges ------------------------------------------------------------
    add("V1 5 VLAN tags (beyond depth)", P.eth(vlans=[(0x8100, 1)] * 5, ethertype=0x0800) +
        P.ipv4(A_SRC, A_DST, payload=P.udp(1, 53)), dny_all=DROP)
    add("V2 4 QinQ tags + udp 53", Ann(hit=("port", 53)), P.eth(vlans=[(0x88A8, 1)] * 4) +
        P.ipv4(A_SRC, A_DST, payload=P.udp(1, 53)), dny_all=PASS)
    add("L1 empty frame", b"", dny_all=ABORTED)
    add("L2 exactly eth header", P.eth(), dny_all=ABORTED, dny_eth=DROP)
    add("L3 ipv4 exactly 20B hdr, proto 17, no udp", P.eth() + P.ipv4(A_SRC, A_DST, 17),
        dny_all=ABORTED, dny_ip=DROP)

    # ---- the reference tests' traffic, as their tools put it on the wire ----
    # (test-xdp-filter.sh: socat TCP6/UDP6 :89-90, ping6 :134, ndisc6 :139,
    # ping :178, arping :183, arping -A :188; test_basic.py's default packets)
    e6 = P.eth(ethertype=0x86DD)
    add("Q1 socat TCP6 SYN (doff 10) to port 10000", Ann(hit=("port", 10000), src=SH + ":89"),
        e6 + P.ipv6(IN6_N, OUT6_N, 6, P.tcp_syn_linux(40000, 10000)),
        dny_tcp=PASS, alw_tcp=DROP, dny_all=PASS, alw_all=DROP, dny_udp=DROP, dny_ip=DROP)
    add("Q2 socat TCP6 SYN (doff 10) to port 10001", Ann(src=SH + ":89"),
        e6 + P.ipv6(IN6_N, OUT6_N, 6, P.tcp_syn_linux(40000, 10001)),
        dny_tcp=DROP, alw_tcp=PASS, dny_all=DROP, alw_all=PASS)
    add("Q3 socat UDP6 'test' to port 10000", Ann(hit=("port", 10000), src=SH + ":90"),
        e6 + P.ipv6(IN6_N, OUT6_N, 17, P.udp(40001, 10000, b"test\n")),
        dny_udp=PASS, alw_udp=DROP, dny_all=PASS, alw_all=DROP, dny_tcp=DROP, dny_ip=DROP)
    add("Q4 socat UDP6 'test' to port 10001", Ann(src=SH + ":90"),
        e6 + P.ipv6(IN6_N, OUT6_N, 17, P.udp(40001, 10001, b"test\n")),
        dny_udp=DROP, alw_udp=PASS, dny_all=DROP)
    add("Q5 socat TCP4-style SYN (doff 10) to port 10000", Ann(hit=("port", 10000), src=SH + ":89"),
        P.eth() + P.ipv4(IN4_N, OUT4_N, 6, payload=P.tcp_syn_linux(40000, 10000)),
        dny_tcp=PASS, alw_tcp=DROP, dny_all=PASS)
    add("Q6 ping to OUTSIDE (dst rule)", Ann(hit=("v4", OUT4), src=IPV4_SH.split(":")[0] + ":178"),
        P.ping4(IN4, OUT4), dny_ip=PASS, alw_ip=DROP, dny_all=PASS, alw_all=DROP, dny_udp=DROP,
        alw_tcp=PASS, alw_eth=PASS)
    add("Q7 ping from INSIDE (src rule)", Ann(hit=("v4", IN4_SRC), src=IPV4_SH.split(":")[0] + ":178"),
        P.ping4(IN4_SRC, OUT4_S), dny_ip=PASS, alw_ip=DROP, dny_all=PASS)
    add("Q8 arping request for OUTSIDE (tip as DST)", Ann(hit=("v4", OUT4), src=SH + ":183"),
        P.arping(1, P.mac(IN_MAC), IN4, OUT4), dny_ip=PASS, alw_ip=DROP, dny_all=PASS,
        dny_udp=DROP, alw_eth=PASS)
    add("Q9 arping -A from INSIDE (reply, sip = tip, src rule)", Ann(hit=("v4", IN4_SRC), src=SH + ":188"),
        P.arping(2, P.mac(IN_MAC), IN4_SRC, IN4_SRC), dny_ip=PASS, alw_ip=DROP, dny_all=PASS)
    add("Q10 arping -A with no src rule", Ann(src=SH + ":188"),
        P.arping(2, P.mac(IN_MAC), IN4, IN4), dny_ip=DROP, alw_ip=PASS)
    add("Q11 ping6 to OUTSIDE (dst rule)", Ann(hit=("v6", OUT6), src=SH + ":134"),
        P.ping6(IN6, OUT6), dny_ip=PASS, alw_ip=DROP, dny_all=PASS, dny_udp=DROP)
    add("Q12 ping6 from INSIDE (src rule)", Ann(hit=("v6", IN6_SRC), src=SH + ":134"),
        P.ping6(IN6_SRC, OUT6_S), dny_ip=PASS, alw_ip=DROP)
    add("Q13 ndisc6 NS for OUTSIDE, SLLA option (target as DST)", Ann(hit=("v6", OUT6), src=SH + ":139"),
        P.ndisc6_ns(IN6, OUT6, P.mac(IN_MAC)), dny_ip=PASS, alw_ip=DROP, dny_all=PASS,
        dny_udp=DROP, dny_tcp=DROP)
    add("Q14 ndisc6 NS for an unruled target", Ann(src=SH + ":139"),
        P.ndisc6_ns(IN6_N, OUT6_N, P.mac(IN_MAC)), dny_ip=DROP, alw_ip=PASS)
    add("Q15 ping6 to OUTSIDE_MAC (ether dst rule)", Ann(hit=("eth", OUT_MAC), src=ETHER_SH),
        P.ping6(IN6_N, OUT6_N, P.eth(dst=P.mac(OUT_MAC), src=P.mac(IN_MAC), ethertype=0x86DD)),
        dny_eth=PASS, alw_eth=DROP, dny_all=PASS, dny_ip=DROP)
    add("Q16 ping6 from INSIDE_MAC (ether src rule)", Ann(hit=("eth", IN_MAC_SRC), src=ETHER_SH),
        P.ping6(IN6_N, OUT6_N, P.eth(dst=P.mac(OUT_MAC_S), src=P.mac(IN_MAC_SRC), ethertype=0x86DD)),
        dny_eth=PASS, alw_eth=DROP, dny_all=PASS)
    TB = "xdp-filter/tests/test_basic.py:88-92 (common.py:25-31 packets)"
    add("Q17 default udp 60001->60002, `port 60002` (dst)", Ann(hit=("port", 60002), src=TB),
        P.eth() + P.ipv4(IN4_N, OUT4_N, 17, payload=P.udp(60001, 60002)),
        dny_udp=PASS, alw_udp=DROP, dny_all=PASS, alw_all=DROP, dny_ip=DROP)
    add("Q18 default udp6 60001->60002, `port 60002` (dst)", Ann(hit=("port", 60002), src=TB),
        e6 + P.ipv6(IN6_N, OUT6_N, 17, P.udp(60001, 60002)),
        dny_udp=PASS, alw_udp=DROP, dny_all=PASS)
    add("Q19 udp 60001->60005, `port 60001 --mode src`", Ann(hit=("port", 60001), src=TB),
        P.eth() + P.ipv4(IN4_N, OUT4_N, 17, payload=P.udp(60001, 60005)),
        dny_udp=PASS, alw_udp=DROP, dny_all=PASS)
    add("Q20 tcp 60001->60005, `port 60001 --mode src`", Ann(hit=("port", 60001), src=TB),
        P.eth() + P.ipv4(IN4_N, OUT4_N, 6, payload=P.tcp(60001, 60005)),
        dny_tcp=PASS, alw_tcp=DROP, dny_udp=DROP)
    return F
