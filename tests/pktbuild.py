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
