"""Test tooling: write pcap / pcapng files with Python's struct module and
read back the pcapng verdict dump, independently of the C implementation
(xdp-tools_amd/csrc/xfg_io.c) under test.

Formats: libpcap classic (https://www.tcpdump.org/manpages/pcap-savefile.5.txt)
and pcapng (SHB / IDB / EPB / SPB; epb_verdict option code 7, the option
lib/util/xpcapng.c:150-161,392-479 writes for xdpdump).
"""
import struct

import numpy as np


def frames_of(data, lens, stride=0, offsets=None):
    out = []
    for i, l in enumerate(lens):
        o = int(offsets[i]) if offsets is not None else i * stride
        out.append(bytes(data[o:o + int(l)]))
    return out


def write_pcap(path, frames, nsec=False, big_endian=False, linktype=1, ts0=1_700_000_000):
    e = ">" if big_endian else "<"
    magic = 0xa1b23c4d if nsec else 0xa1b2c3d4
    with open(path, "wb") as f:
        f.write(struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, 262144, linktype))
        for i, fr in enumerate(frames):
            sec, frac = ts0 + i // 1000, (i % 1000) * (1000 if nsec else 1)
            f.write(struct.pack(e + "IIII", sec, frac, len(fr), len(fr) + 4))
            f.write(fr)


def _opt(code, payload, e):
    pad = (-len(payload)) % 4
    return struct.pack(e + "HH", code, len(payload)) + payload + b"\0" * pad


def _block(btype, body, e):
    total = 12 + len(body)
    return struct.pack(e + "II", btype, total) + body + struct.pack(e + "I", total)


def write_pcapng(path, frames, big_endian=False, tsresol=None, use_spb=False, linktype=1,
                 extra_blocks=True):
    e = ">" if big_endian else "<"
    shb = struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1) + _opt(4, b"pytest", e) + \
        struct.pack(e + "I", 0)
    idb_opts = _opt(2, b"veth0", e)
    if tsresol is not None:
        idb_opts += _opt(9, bytes([tsresol]), e)
    idb = struct.pack(e + "HHI", linktype, 0, 0) + idb_opts + struct.pack(e + "I", 0)
    with open(path, "wb") as f:
        f.write(struct.pack(e + "I", 0x0A0D0D0A) + struct.pack(e + "I", 12 + len(shb)) + shb +
                struct.pack(e + "I", 12 + len(shb)))
        f.write(_block(1, idb, e))
        if extra_blocks:   # a name-resolution block: no packets, must be skipped
            f.write(_block(4, struct.pack(e + "HH", 0, 0), e))
        for i, fr in enumerate(frames):
            pad = b"\0" * ((-len(fr)) % 4)
            if use_spb:
                f.write(_block(3, struct.pack(e + "I", len(fr)) + fr + pad, e))
            else:
                ts = 1_700_000_000_000_000 + i
                body = struct.pack(e + "IIIII", 0, ts >> 32, ts & 0xffffffff, len(fr), len(fr))
                f.write(_block(6, body + fr + pad + struct.pack(e + "I", 0), e))


def read_verdict_pcapng(path):
    """Return [(frame bytes, verdict type, verdict value)] from an EPB dump."""
    out = []
    b = open(path, "rb").read()
    o = 0
    e = "<"
    while o < len(b):
        btype, blen = struct.unpack_from(e + "II", b, o)
        if btype == 0x0A0D0D0A:
            bom = struct.unpack_from("<I", b, o + 8)[0]
            e = "<" if bom == 0x1A2B3C4D else ">"
            btype, blen = struct.unpack_from(e + "II", b, o)
        assert struct.unpack_from(e + "I", b, o + blen - 4)[0] == blen
        if btype == 6:
            _, _, _, cap, orig = struct.unpack_from(e + "IIIII", b, o + 8)
            fr = b[o + 28:o + 28 + cap]
            p = o + 28 + cap + ((-cap) % 4)
            vtype = vval = None
            while p < o + blen - 4:
                code, ln = struct.unpack_from(e + "HH", b, p)
                if code == 0:
                    break
                if code == 7:
                    vtype = b[p + 4]
                    vval = struct.unpack_from(e + "q", b, p + 5)[0]
                p += 4 + ln + ((-ln) % 4)
            out.append((fr, vtype, vval))
        o += blen
    return out


def batch_from(frames):
    """Frames -> (data, offsets, lens) at 16-byte aligned offsets, for the oracle."""
    offs, lens, o = [], [], 0
    for fr in frames:
        offs.append(o)
        lens.append(len(fr))
        o += (len(fr) + 15) // 16 * 16
    data = np.zeros(o + 64, np.uint8)
    for fr, off in zip(frames, offs):
        data[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
    return data, np.array(offs, np.uint64), np.array(lens, np.uint32)
