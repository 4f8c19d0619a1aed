"""Frames whose L4 header starts past byte 262,143 (ZP_L4_NEAR_MAX): the
record's far-L4 form (ABI v5, include/zero_packet.h). Only an IPv6 jumbogram
with thousands of nested IPv6 headers reaches such an offset
(parser.rs:134-135 recurses without a limit; IPv6 payload_length is never
checked, ipv6.rs:147-167), and the reference returns Ok with the L4 reader
there. ABI v4 saturated the offset and the facades refused the record; v5
keeps the whole offset in `offs` (Ethernet code 3) and reads the Ethernet
header length and the ip_in_ip offset from the frame, so every result equals
the oracle's unpacked record: the GPU records, zp_rec_decode, both facades,
the column views and PacketParser.parse."""
import ctypes

import numpy as np
import pytest

import oracle as orc


def deep_frame(levels, l4="icmpv6", inner="ipv6", vlan=False, outer_chain=False, tail=64,
               seed=3):
    """Ethernet (+ an 802.1Q tag) + `levels` nested IPv6 headers (the outer
    one optionally with a Hop-by-Hop header) + optionally an IPv4 header,
    then an L4 header (`l4`: icmpv6 / tcp / udp) with a valid checksum over
    the innermost IP's pseudo-header. Returns (frame, l4 offset)."""
    from pybuilder import internet_checksum, pseudo_header
    rng = np.random.default_rng(seed)
    eth = 18 if vlan else 14
    hbh = 16 if outer_chain else 0
    v4 = 20 if inner == "ipv4" else 0
    off = eth + 40 * levels + hbh + v4
    f = bytearray(rng.integers(0, 256, off + tail, dtype=np.uint8).tobytes())
    if vlan:
        f[12:16] = b"\x81\x00\x00\x64"
    f[eth - 2:eth] = b"\x86\xdd"
    proto = {"icmpv6": 58, "tcp": 6, "udp": 17}[l4]
    pos = eth
    for k in range(levels):
        f[pos] = 0x60
        nxt = 41 if k + 1 < levels else (4 if v4 else proto)
        if k == 0 and outer_chain:
            f[pos + 6] = 0                                  # Hop-by-Hop (headers.rs:90-113)
            f[pos + 40] = nxt
            f[pos + 41] = 1                                 # (1 + 1) * 8 = 16 B
            pos += 40 + hbh
        else:
            f[pos + 6] = nxt
            pos += 40
    ip = pos - 40
    if v4:                                                  # parser.rs:188-212
        f[pos:pos + 2] = b"\x45\x00"
        f[pos + 2:pos + 4] = (20 + tail).to_bytes(2, "big")
        f[pos + 6:pos + 8] = b"\0\0"
        f[pos + 9] = proto
        f[pos + 10:pos + 12] = b"\0\0"
        f[pos + 10:pos + 12] = internet_checksum(f[pos:pos + 20]).to_bytes(2, "big")
        src, dst, ip = f[pos + 12:pos + 16], f[pos + 16:pos + 20], pos
        pos += 20
    else:
        src, dst = f[ip + 8:ip + 24], f[ip + 24:ip + 40]
    assert pos == off
    if l4 == "icmpv6":
        f[off] = 128                                        # echo request (misc.rs:164-204)
        ck = off + 2
    elif l4 == "tcp":
        f[off + 12] = 0x50                                  # data offset 5
        f[off + 13] = 0x18                                  # flags != 0
        ck = off + 16
    else:
        f[off + 4:off + 6] = tail.to_bytes(2, "big")        # length == slice (parser.rs:262)
        ck = off + 6
    f[ck:ck + 2] = b"\0\0"
    c = internet_checksum(f[off:], pseudo_header(src, dst, proto, tail))
    f[ck:ck + 2] = c.to_bytes(2, "big")
    return bytes(f), off


# (levels, kwargs): near and far, ICMPv6 / TCP / UDP, an IPv4 innermost level,
# VLAN, an outer extension chain
CASES = [(6550, {}), (6600, {}), (6600, dict(l4="tcp", inner="ipv4")),
         (6601, dict(l4="udp", vlan=True, outer_chain=True)),
         (6700, dict(l4="tcp", vlan=True, outer_chain=True))]


def _cases():
    return [deep_frame(lv, **kw) for lv, kw in CASES]


def _zp_decode(zp, frame, packed, ext):
    """zp_rec_decode (libzp_hip.so host code) through ctypes."""
    lib = zp._lib.hip()
    fields = np.zeros(1, np.dtype([("flags", "<u4"), ("err", "u1"), ("eth_len", "u1"),
                                   ("final_nh", "u1"), ("inner_final_nh", "u1"),
                                   ("inner_off", "<u4"), ("l4_off", "<u4")]))
    buf = ctypes.create_string_buffer(frame, len(frame))
    rec = np.array([packed], zp.records.RECORD_DTYPE)
    e = None if ext is None else np.ascontiguousarray(ext)
    rc = lib.zp_rec_decode(rec.ctypes.data, buf, len(frame),
                           None if e is None else e.ctypes.data, fields.ctypes.data)
    return rc, fields[0]


FIELDS = ("flags", "err", "eth_len", "final_nh", "inner_final_nh", "inner_off", "l4_off")


def _reader_offsets(frame, p):
    """Start offset of every reader of a PacketParser (views run to the frame end)."""
    n = len(frame)
    out = {}
    for name in ("ethernet", "ipv4", "ipv6", "tcp", "udp", "icmpv4", "icmpv6"):
        r = getattr(p, name)
        out[name] = None if r is None else n - len(r.bytes)
    out["ip_in_ip"] = None if p.ip_in_ip is None else n - len(p.ip_in_ip.reader.bytes)
    return out


def test_far_records_decode_exactly(zp):
    """Oracle record -> packed (far form past 262,143) -> zp_rec_decode,
    records.decode and PacketParser.from_record: every field equals the
    oracle's unpacked record, the L4 reader starts where the reference's
    does."""
    R = zp.records
    for (lv, kw), (frame, l4) in zip(CASES, _cases()):
        err, rec, ext = orc.parse_one(frame)
        assert err == 0 and rec["l4_off"] == l4, (lv, kw, err)
        packed = orc.pack(rec, ext)[0]
        far = l4 > R.L4_NEAR_MAX
        assert bool(R.is_far(np.array([packed], R.RECORD_DTYPE))[0]) == far
        if far:
            assert int(packed["offs"]) == l4 and (int(packed["flags"]) >> 24) & 3 == 3
        for e in (ext, None if not (int(rec["flags"]) & (R.F_EXT | R.F_INNER_EXT)) else ext):
            rc, d = _zp_decode(zp, frame, packed, e)
            assert rc == 0
            assert all(int(d[k]) == int(rec[k]) for k in FIELDS), (lv, kw, d, rec)
        rc, d = _zp_decode(zp, frame, packed, None)          # chains re-walked over the frame
        assert rc == 0 and all(int(d[k]) == int(rec[k]) for k in FIELDS)
        pd = R.decode(frame, packed, ext)
        assert all(pd[k] == int(rec[k]) for k in FIELDS), (pd, rec)
        # without entries records.decode walks the chains again, as zp_rec_decode
        pd = R.decode(frame, packed, None)
        assert all(pd[k] == int(rec[k]) for k in FIELDS), ("no ext", pd, rec)
        p = zp.PacketParser.from_record(frame, packed, ext)
        offs = _reader_offsets(frame, p)
        assert offs["ethernet"] == 0 and offs["ip_in_ip"] == rec["inner_off"]
        l4r = {"icmpv6": "icmpv6", "tcp": "tcp", "udp": "udp"}[kw.get("l4", "icmpv6")]
        assert offs[l4r] == l4 and offs["ipv6"] == rec["eth_len"]
        assert p.ip_in_ip.kind == "ipv6"
        if kw.get("outer_chain"):
            assert p.ipv6.extension_headers.hop_by_hop is not None


def test_far_record_mismatch_is_refused(zp):
    """zp_rec_decode refuses a far record that cannot belong to the frame."""
    frame, l4 = deep_frame(6600)
    _, rec, ext = orc.parse_one(frame)
    packed = orc.pack(rec, ext)[0].copy()
    rc, _ = _zp_decode(zp, frame[:l4], packed, ext)        # L4 past the end
    assert rc == -1
    packed["flags"] = int(packed["flags"]) & ~zp.records.F_IP_IN_IP
    assert _zp_decode(zp, frame, packed, ext)[0] == -1     # far without ip_in_ip


@pytest.mark.gpu
def test_l4_far_on_the_gpu(zp):
    """The deep frames through the device batch path, zp_parse_one
    (PacketParser.parse; frames over 64 KiB take its batch host path) and the
    column views: records byte-identical to the oracle's packed ones, and
    every field decoded from them equal to the oracle's unpacked record."""
    import torch
    cases = _cases()
    frames = [f for f, _ in cases]
    offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.int64)
    arena = np.frombuffer(b"".join(frames) + bytes(64), np.uint8).copy()
    lens = np.array([len(f) for f in frames], np.int32)
    d = torch.device("cuda:0")
    da, do, dl = (torch.from_numpy(x).to(d) for x in (arena, offs, lens))
    r, e = zp.batch.parse_batch(da, do, dl)
    got, gext = zp.batch.records_to_numpy(r, e)
    want, wext = orc.parse_batch(arena, offs.astype(np.uint64), lens.astype(np.uint32))
    assert (want["err"] == 0).all()
    assert zp.records.is_far(got).sum() == sum(l4 > zp.records.L4_NEAR_MAX for _, l4 in cases)
    assert got.tobytes() == orc.pack(want, wext).tobytes()
    assert zp.records.ext_match(gext, wext, want)
    for k, (f, l4) in enumerate(cases):
        pd = zp.records.decode(f, got[k], gext[:, k])
        assert all(pd[x] == int(want[k][x]) for x in FIELDS)
        p = zp.PacketParser.parse(f)                          # the reference's Ok result
        offs_k = _reader_offsets(f, p)
        l4r = [n for n in ("tcp", "udp", "icmpv6") if offs_k[n] is not None]
        assert len(l4r) == 1 and offs_k[l4r[0]] == l4 == want[k]["l4_off"]
        assert offs_k["ip_in_ip"] == want[k]["inner_off"]
    # the column views of the far records: the L4 getters at the true offset
    cols = zp.columns.extract(da, do, dl, r)
    torch.cuda.synchronize()
    wc = orc.columns(arena, offs, lens, want)
    for name, t in cols.items():
        assert np.array_equal(t.cpu().numpy(), wc[name]), name
    assert (wc["l4_proto"] != 0).all() and (wc["inner_version"] == 6).all()
