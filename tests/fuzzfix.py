"""Checksum repair for the mutation fuzzers (test infrastructure).

A mutated frame almost always fails the IPv4 header or L4 checksum
(parser.rs:205-210, 316-361), so plain byte flips stop the reference's
checks there. `repair` rewrites the checksum fields of a mutated frame the
way the reference builder fills them (ipv4.rs:119-126 header checksum;
tcp.rs:123-129, udp.rs:65-71, icmpv4.rs:74-80, icmpv6.rs:71-77 over the
whole remaining segment with the pseudo-header of the innermost IP,
checksum.rs:38-69), following the frame's own (possibly mutated) header
chain. Repaired frames get past the checksums into the field checks that
follow them in the reference order, and into the accept path with unusual
field values (TCP flags/offsets, UDP lengths, ICMP types and codes, IHL,
tags). The repair is best effort: where it cannot follow the chain it
leaves the bytes alone, and the frame is still a valid fuzz input.
"""
from pybuilder import internet_checksum, pseudo_header

EXT = (0, 43, 44, 51, 60)


def _be16(f, i):
    return (f[i] << 8) | f[i + 1]


def _put16(f, i, v):
    f[i] = (v >> 8) & 0xFF
    f[i + 1] = v & 0xFF


def _ext_end(f, p, nh):
    """End of an IPv6 extension chain from p (headers.rs:51-213, simplified:
    at most 6 headers, stops where a header would not fit)."""
    n = len(f)
    for _ in range(6):
        if nh not in EXT or p + 8 > n:
            break
        hl = 8 if nh == 44 else ((f[p + 1] + 2) * 4 if nh == 51 else (f[p + 1] + 1) * 8)
        if p + hl > n:
            break
        nh = f[p]
        p += hl
    return p, nh


def repair(frame):
    f = bytearray(frame)
    n = len(f)
    if n < 18:
        return bytes(f)
    t = _be16(f, 12)
    hl = 18 if t == 0x8100 else (22 if t == 0x88A8 else 14)
    if n < hl:
        return bytes(f)
    et = _be16(f, hl - 2)
    if et not in (0x0800, 0x86DD):
        return bytes(f)
    pos, v4 = hl, et == 0x0800
    proto = src = dst = None
    l4 = None
    for _ in range(3):                     # outer IP, at most two encapsulations
        if v4:
            if n - pos < 20:
                return bytes(f)
            ihl = (f[pos] & 15) * 4
            if ihl < 20 or pos + ihl > n:
                return bytes(f)
            _put16(f, pos + 10, 0)
            _put16(f, pos + 10, internet_checksum(f[pos:pos + ihl]))
            proto, src, dst, l4 = f[pos + 9], f[pos + 12:pos + 16], f[pos + 16:pos + 20], pos + ihl
        else:
            if n - pos < 40:
                return bytes(f)
            l4, proto = _ext_end(f, pos + 40, f[pos + 6])
            src, dst = f[pos + 8:pos + 24], f[pos + 24:pos + 40]
        if proto not in (4, 41):
            break
        pos, v4 = l4, proto == 4
    at = {6: 16, 17: 6, 1: 2, 58: 2}.get(proto)
    if at is None or l4 + at + 2 > n:
        return bytes(f)
    _put16(f, l4 + at, 0)
    acc = 0 if (v4 and proto == 1) else pseudo_header(bytes(src), bytes(dst), proto, n - l4)
    _put16(f, l4 + at, internet_checksum(f[l4:], acc))
    return bytes(f)
