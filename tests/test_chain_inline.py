"""The inline outer chain (ABI v6, include/zero_packet.h ZP_CHAIN_INLINE): a
short RFC-ordered IPv6 extension chain of a frame without ip_in_ip and with
an L4 reader lives in the record's free inner_off bits, and its 16-B ext
entry is not written (c4-shaped traffic writes 8 B per frame instead of 24).
CPU: the oracle's packing rule (zpo_pack) against the chains themselves; the
rebuilt entries (Python records.inline_chains, C zp_rec_chain through
zp_rec_decode and the C++ facade) equal the oracle's ExtensionHeaders
(headers.rs:19-28) offset for offset."""
import ctypes

import numpy as np

import oracle as orc


def _rfc_chain(ext, flags, R):
    """True when the chain's headers lie back to back from offset 0 in RFC
    order with lengths the inline code holds (the rule, restated)."""
    at = 0
    seq = [k for k in (0, 4, 1, 2, 3, 5) if flags & R.F_EXT_SLOT(k)]
    for q, k in enumerate(seq):
        if int(ext["off"][k]) != at:
            return False
        end = int(ext["off"][seq[q + 1]]) if q + 1 < len(seq) else int(ext["len"])
        hl = end - at
        if k == 2:
            ok = hl == 8
        elif k == 3:
            ok = hl % 4 == 0 and 0 <= hl // 4 - 2 <= 3
        else:
            ok = hl % 8 == 0 and 0 <= hl // 8 - 1 <= (7 if k in (0, 1) else 3)
        if not ok:
            return False
        at = end
    return bool(seq)


def _corpus(zp, golden):
    from test_gpu_parity import fuzz_frames
    frames = [bytes.fromhex(f["bytes"]) for f in golden["fixtures"]]
    for cfg in ("c4", "c5", "c6"):
        a, o, l = zp.batch.generate_host(cfg, 3000, first=31)
        frames += [a[int(o[i]):int(o[i]) + int(l[i])].tobytes() for i in range(len(o))]
    return frames + fuzz_frames(zp, golden, 3000, 17, repair_p=0.5)


def test_inline_rule_and_rebuild(zp, golden):
    R = zp.records
    frames = _corpus(zp, golden)
    n_inline = n_wide = 0
    lib = zp._lib.hip()
    fields = np.zeros(1, np.dtype([("flags", "<u4"), ("err", "u1"), ("eth_len", "u1"),
                                   ("final_nh", "u1"), ("inner_final_nh", "u1"),
                                   ("inner_off", "<u4"), ("l4_off", "<u4")]))
    for f in frames:
        err, rec, ext = orc.parse_one(f)
        packed = orc.pack(rec, ext)
        inl = bool(R.chain_inline(packed)[0])
        fl = int(rec["flags"])
        l4 = fl & (R.F_TCP | R.F_UDP | R.F_ICMPV4 | R.F_ICMPV6)
        want_inl = (not err and fl & R.F_EXT and not fl & R.F_IP_IN_IP and bool(l4)
                    and _rfc_chain(ext[0], fl, R))
        assert inl == bool(want_inl), (f.hex()[:80], fl)
        if not inl:
            n_wide += bool(not err and fl & R.F_EXT)
            continue
        n_inline += 1
        # Python rebuild == the oracle's chain entry
        x = R.inline_chains(packed)[0]
        assert x.tobytes() == ext[0].tobytes(), (x, ext[0])
        # decoded without any ext entry: records.decode, zp_rec_decode, from_record
        d = R.decode(f, packed[0], None)
        for k in ("flags", "eth_len", "final_nh", "inner_off", "l4_off"):
            assert d[k] == int(rec[k]), k
        buf = ctypes.create_string_buffer(f, len(f))
        assert lib.zp_rec_decode(packed.ctypes.data, buf, len(f), None, fields.ctypes.data) == 0
        assert all(int(fields[0][k]) == int(rec[k]) for k in ("flags", "eth_len", "final_nh",
                                                               "inner_off", "l4_off"))
        p = zp.PacketParser.from_record(f, packed[0], None)
        eh = p.ipv6.extension_headers
        assert eh.total_headers_len == int(ext[0]["len"]) and p.ipv6.extension_headers_len == int(ext[0]["len"])
        assert eh.final_next_header == int(ext[0]["final_nh"])
        # the decoded view of the record never shows the chain as an inner offset
        assert R.unpack(packed)["inner_off"][0] == 0
    assert n_inline > 2000 and n_wide > 5


def test_c4_chains_all_inline(zp):
    """Every chain of BASELINE config 4 goes inline (RFC-ordered subsets of
    Hop-by-Hop (8-24 B) / Routing (8-40 B) / Fragment under TCP / UDP /
    ICMPv6): c4 writes no ext entries."""
    a, o, l = zp.batch.generate_host("c4", 20000, first=5)
    rec, ext = orc.parse_batch(a, o, l)
    packed = orc.pack(rec, ext)
    chained = (rec["flags"] & zp.records.F_EXT) != 0
    assert chained.sum() > 15000
    assert (zp.records.chain_inline(packed) == chained).all()
    x = zp.records.expand_ext(packed, np.zeros((2, len(rec)), zp.records.EXT_DTYPE))
    assert zp.records.ext_match(x, ext, rec)
