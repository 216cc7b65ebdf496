"""Minimal packet builders for the known-answer tests (scapy is not
available here).  Each helper returns raw frame bytes."""
from __future__ import annotations

import ipaddress
import struct

MAC_A = bytes.fromhex("02000000000a")   # "local" end of the reference's veth fixture
MAC_B = bytes.fromhex("02000000000b")


def mac(s: str) -> bytes:
    return bytes(int(x, 16) for x in s.split(":"))


def ip4(s: str) -> bytes:
    return ipaddress.IPv4Address(s).packed


def ip6(s: str) -> bytes:
    return ipaddress.IPv6Address(s).packed


def eth(dst=MAC_B, src=MAC_A, ethertype=0x0800, vlans=()) -> bytes:
    b = dst + src
    for tpid, vid in vlans:
        b += struct.pack("!HH", tpid, vid)
    return b + struct.pack("!H", ethertype)


def ipv4(src="10.11.1.1", dst="10.11.1.2", proto=17, ihl=5, payload=b"", frag=0x4000,
         total_len=None) -> bytes:
    opts = b"\x01" * max(0, ihl * 4 - 20)
    tl = total_len if total_len is not None else 20 + len(opts) + len(payload)
    h = struct.pack("!BBHHHBBH4s4s", 0x40 | ihl, 0, tl, 0, frag, 64, proto, 0,
                    ip4(src), ip4(dst))
    return h + opts + payload


def ipv6(src="fc00:dead:cafe:1::1", dst="fc00:dead:cafe:1::2", nh=17, payload=b"") -> bytes:
    return struct.pack("!IHBB16s16s", 0x60000000, len(payload), nh, 64, ip6(src), ip6(dst)) + payload


def ext(nh: int, hdrlen: int = 0, kind: str = "opt") -> bytes:
    """IPv6 extension header with next-header nh.  kind: opt (HBH/DST/ROUTING/MH:
    (hdrlen+1)*8 bytes), ah ((hdrlen+2)*4), frag (8)."""
    if kind == "frag":
        return bytes([nh, 0]) + b"\x00" * 6
    size = (hdrlen + 2) * 4 if kind == "ah" else (hdrlen + 1) * 8
    return bytes([nh, hdrlen]) + b"\x00" * (size - 2)


def udp(sport=12345, dport=53, payload=b"x" * 8, length=None) -> bytes:
    ln = length if length is not None else 8 + len(payload)
    return struct.pack("!HHHH", sport, dport, ln, 0) + payload


def tcp(sport=12345, dport=53, doff=5, payload=b"") -> bytes:
    h = struct.pack("!HHIIBBHHH", sport, dport, 0, 0, doff << 4, 0x02, 1024, 0, 0)
    opts = b"\x01" * max(0, doff * 4 - 20)
    return h + opts + payload


def icmp6(typ=128, code=0, body=b"") -> bytes:
    return struct.pack("!BBH", typ, code, 0) + b"\x00" * 4 + body


def ndisc_ns(target: str) -> bytes:
    return icmp6(135, 0, ip6(target))


def ndisc_na(target: str) -> bytes:
    return icmp6(136, 0, ip6(target))


def arp(op=1, sha=MAC_A, sip="10.11.1.1", tha=b"\x00" * 6, tip="10.11.1.2",
        hrd=1, pro=0x0800, hln=6, pln=4) -> bytes:
    return struct.pack("!HHBBH6s4s6s4s", hrd, pro, hln, pln, op, sha, ip4(sip), tha, ip4(tip))


def icmp4_echo() -> bytes:
    return struct.pack("!BBHHH", 8, 0, 0, 1, 1) + b"ping" * 4


# ---- the shapes the reference's own test traffic has (iputils ping/ping6/
# arping, socat, ndisc6), used by tests/kat.py's reference-traffic rows

def ping_data() -> bytes:
    """ping's default 56 data bytes: a 16-byte timestamp, then 0x10, 0x11, ..."""
    return b"\x11" * 16 + bytes(range(0x10, 0x10 + 40))


def ping4(src, dst, eth_hdr=None) -> bytes:
    """`ping -c 1`: ICMP echo request, 64 ICMP bytes, DF, TTL 64 (98-byte frame)."""
    icmp = struct.pack("!BBHHH", 8, 0, 0, 0x1234, 1) + ping_data()
    return (eth_hdr or eth()) + ipv4(src, dst, 1, payload=icmp, frag=0x4000)


def ping6(src, dst, eth_hdr=None) -> bytes:
    """`ping6 -c 1`: ICMPv6 echo request, 64 ICMPv6 bytes (118-byte frame)."""
    icmp = struct.pack("!BBHHH", 128, 0, 0, 0x1234, 1) + ping_data()
    return (eth_hdr or eth(ethertype=0x86DD)) + ipv6(src, dst, 58, icmp)


def tcp_syn_linux(sport, dport) -> bytes:
    """A Linux connect() SYN (socat TCP6:...): doff 10, options MSS, SACK-permitted,
    timestamps, NOP, window scale."""
    opts = bytes.fromhex("020405a0" "0402" "080a") + struct.pack("!II", 0x01020304, 0) + \
        bytes.fromhex("01" "030307")
    return struct.pack("!HHIIBBHHH", sport, dport, 0x11223344, 0, 10 << 4, 0x02, 64800, 0, 0) + opts


def arping(op, sha, sip, tip, tha=b"\xff" * 6) -> bytes:
    """iputils arping: a 42-byte ARP frame to the broadcast address (`-A`: an ARP
    reply with sip == tip)."""
    return eth(dst=b"\xff" * 6, src=sha, ethertype=0x0806) + arp(op, sha=sha, sip=sip, tha=tha, tip=tip)


def ndisc6_ns(src, target, sll) -> bytes:
    """`ndisc6 -r 1 <target> -s <src> <if>`: a neighbour solicitation to the
    target's solicited-node group, hop limit 255, with a source link-layer
    address option (type 1, length 1)."""
    t = ipaddress.IPv6Address(target).packed
    group = ipaddress.IPv6Address("ff02::1:ff00:0").packed[:13] + t[13:]
    body = struct.pack("!BBHI", 135, 0, 0, 0) + t + bytes([1, 1]) + sll
    e = eth(dst=b"\x33\x33" + group[12:], src=sll, ethertype=0x86DD)
    h = struct.pack("!IHBB16s16s", 0x60000000, len(body), 58, 255, ip6(src), group)
    return e + h + body
