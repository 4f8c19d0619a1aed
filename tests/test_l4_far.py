"""The 8-B record's one escape (ABI v4, include/zero_packet.h): an L4 header
that starts at or past ZP_L4_FAR (262,143) does not fit the record's 18-bit
l4_off and is reported as ZP_L4_FAR. Only an IPv6 jumbogram with thousands of
nested IPv6-in-IPv6 headers reaches it (parser.rs:134-135 recurses without a
limit; IPv6 payload_length is never checked, ipv6.rs:147-167). The oracle's
packed record and the GPU's agree on it, and the facades refuse the record
instead of building an L4 reader at a wrong offset."""
import contextlib

import numpy as np
import pytest

import oracle as orc


def deep_ipv6_frame(levels, tail=64, seed=3):
    """Ethernet + `levels` nested IPv6 headers (next header 41, the last 58)
    + an ICMPv6 echo request with a valid checksum over the innermost IPv6
    pseudo-header (ICMPv6 has no length field, so any length is accepted)."""
    from pybuilder import internet_checksum, pseudo_header
    rng = np.random.default_rng(seed)
    l4 = 14 + 40 * levels
    f = bytearray(rng.integers(0, 256, l4 + tail, dtype=np.uint8).tobytes())
    f[12:14] = b"\x86\xdd"
    for k in range(levels):
        h = 14 + 40 * k
        f[h] = 0x60
        f[h + 6] = 41 if k + 1 < levels else 58
    f[l4] = 128                                            # echo request (misc.rs:164-204)
    f[l4 + 2:l4 + 4] = b"\0\0"
    ip = l4 - 40
    c = internet_checksum(f[l4:], pseudo_header(f[ip + 8:ip + 24], f[ip + 24:ip + 40], 58, tail))
    f[l4 + 2:l4 + 4] = c.to_bytes(2, "big")
    return bytes(f), l4


def test_l4_far_escape_in_the_oracle_and_the_facade(zp):
    for levels, far in ((6550, False), (6600, True)):      # L4 at 262,014 / 264,014
        frame, l4 = deep_ipv6_frame(levels)
        err, rec, ext = orc.parse_one(frame)
        assert err == 0 and rec["l4_off"] == l4 and rec["inner_off"] == 54
        packed = orc.pack(rec)[0]
        u = zp.records.unpack(np.array([packed], zp.records.RECORD_DTYPE))[0]
        assert u["l4_off"] == (zp.records.L4_FAR if far else l4) and u["inner_off"] == 54
        if far:
            with pytest.raises(ValueError):
                zp.PacketParser.from_record(frame, packed, ext)
        else:
            p = zp.PacketParser.from_record(frame, packed, ext)
            assert p.icmpv6 is not None and len(p.icmpv6.bytes) == 64
            assert p.ip_in_ip.kind == "ipv6"


@pytest.mark.gpu
def test_l4_far_escape_on_the_gpu(zp):
    """Both frames through the device batch path and zp_parse_one (frames
    over 64 KiB take its batch host path): records byte-identical to the
    oracle's packed ones."""
    import torch
    frames = [deep_ipv6_frame(lv)[0] for lv in (6550, 6600)]
    offs = np.array([0, len(frames[0])], np.int64)
    arena = np.frombuffer(b"".join(frames) + bytes(64), np.uint8).copy()
    lens = np.array([len(f) for f in frames], np.int32)
    d = torch.device("cuda:0")
    r, e = zp.batch.parse_batch(torch.from_numpy(arena).to(d), torch.from_numpy(offs).to(d),
                                torch.from_numpy(lens).to(d))
    got, gext = zp.batch.records_to_numpy(r, e)
    want, wext = orc.parse_batch(arena, offs.astype(np.uint64), lens.astype(np.uint32))
    assert (want["err"] == 0).all()
    assert got.tobytes() == orc.pack(want).tobytes()
    assert zp.records.ext_match(gext, wext, want)
    for f, w in zip(frames, want):
        far = w["l4_off"] >= zp.records.L4_FAR
        with pytest.raises(ValueError) if far else contextlib.nullcontext():
            p = zp.PacketParser.parse(f)
            assert p.icmpv6 is not None

