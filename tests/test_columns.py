"""Column views.

CPU: the oracle's column restatement (oracle/zp_oracle.c zpo_columns) agrees
with the reader getters of the PacketParser facade (zero-packet_amd/parser.py,
which mirrors ethernet.rs / ipv4.rs / ipv6.rs / tcp.rs / udp.rs / icmp*.rs) on
the golden packets, generated configs and fuzz mutations; the column table of
the C ABI matches the Python one.
GPU: zp_extract_columns_device is byte-exact against the oracle.
"""
import random

import numpy as np
import pytest

import oracle as orc
from test_oracle_fuzz import mutate


def getter_columns(zp, frame, rec, ext):
    """Expected column entries of one frame from the facade's getters."""
    want = {name: (np.zeros(w, dt) if w > 1 else dt(0)) for name, dt, w in orc.COLUMN_SPEC}
    if int(rec["err"]):
        return want
    p = zp.PacketParser.from_record(frame, orc.pack(rec, ext)[0], ext)   # the ABI record
    e = p.ethernet
    if e is None:
        return want

    def arr(b, w):
        a = np.zeros(w, np.uint8)
        a[:len(b)] = np.frombuffer(bytes(b), np.uint8)
        return a
    want["dest_mac"] = arr(e.dest_mac(), 6)
    want["src_mac"] = arr(e.src_mac(), 6)
    want["ethertype"] = np.uint16(e.ethertype())
    if e.vlan_tag() is not None:
        want["vlan_tci"] = np.uint16(e.vlan_tag()[1])
    if e.double_vlan_tag() is not None:
        want["vlan_tci"] = np.uint16(e.double_vlan_tag()[0][1])
        want["vlan_inner_tci"] = np.uint16(e.double_vlan_tag()[1][1])
    if p.arp is not None:
        want["arp_oper"] = np.uint16(p.arp.oper())

    def ip(r, v6, inner):
        pre = "inner_" if inner else ""
        want["inner_version" if inner else "ip_version"] = np.uint8(r.version())
        want[pre + "src_addr"] = arr(r.src_addr() if v6 else r.src_ip(), 16)
        want[pre + "dest_addr"] = arr(r.dest_addr() if v6 else r.dest_ip(), 16)
        want["inner_protocol" if inner else "protocol"] = np.uint8(
            r.final_next_header() if v6 else r.protocol())
        if inner:
            return
        if v6:
            want["ttl"] = np.uint8(r.hop_limit())
            want["tos"] = np.uint8(r.traffic_class())
            want["ip_id"] = np.uint32(r.flow_label())
            want["ip_len"] = np.uint16(r.payload_length())
        else:
            want["ttl"] = np.uint8(r.ttl())
            want["tos"] = np.uint8((r.dscp() << 2) | r.ecn())
            want["ip_id"] = np.uint32(r.id())
            want["ip_len"] = np.uint16(r.total_length())
    if p.ipv4 is not None:
        ip(p.ipv4, False, False)
    if p.ipv6 is not None:
        ip(p.ipv6, True, False)
    if p.ip_in_ip is not None:
        ip(p.ip_in_ip.reader, p.ip_in_ip.kind == "ipv6", True)
    l4 = p.tcp or p.udp or p.icmpv4 or p.icmpv6
    if l4 is not None:
        base = len(frame) - len(l4.bytes)
        want["l4_checksum"] = np.uint16(l4.checksum())
        if p.tcp is not None:
            t = p.tcp
            want["l4_proto"] = np.uint8(6)
            want["src_port"], want["dest_port"] = np.uint16(t.src_port()), np.uint16(t.dest_port())
            want["tcp_seq"], want["tcp_ack"] = np.uint32(t.sequence_number()), np.uint32(t.ack_number())
            want["tcp_flags"] = np.uint8(t.flags())
            want["tcp_window"] = np.uint16(t.window_size())
        elif p.udp is not None:
            want["l4_proto"] = np.uint8(17)
            want["src_port"] = np.uint16(p.udp.src_port())
            want["dest_port"] = np.uint16(p.udp.dest_port())
        else:
            want["l4_proto"] = np.uint8(1 if p.icmpv4 is not None else 58)
            want["icmp_type"] = np.uint8(l4.icmp_type())
            want["icmp_code"] = np.uint8(l4.icmp_code())
        try:
            pay = l4.payload()
            want["payload_off"] = np.uint32(len(frame) - len(pay))
        except zp.ZeroPacketError:
            pass
        assert base == int(rec["l4_off"])
    return want


def frames_corpus(zp, golden, n_fuzz, seed=99):
    """Golden and generated frames plus n_fuzz mutations of them; two thirds of
    the mutations get their checksums refilled (tests/fuzzfix.py), so most are
    accepted and their columns carry mutated field values."""
    from fuzzfix import repair
    rng = random.Random(seed)
    seeds = [bytes.fromhex(fx["bytes"]) for fx in golden["fixtures"]]
    for cfg in ("c3", "c4", "c5", "c6"):
        arena, offs, lens = zp.batch.generate_host(cfg, 60, first=4242)
        seeds += [arena[o:o + l].tobytes() for o, l in zip(offs, lens)]
    frames = list(seeds)
    for _ in range(n_fuzz):
        f = mutate(rng, rng.choice(seeds))
        frames.append(repair(f) if rng.random() < 2 / 3 else f)
    return frames


def pack(frames):
    offs, pos = [], 3
    for f in frames:
        offs.append(pos)
        pos += len(f) + 5
    arena = np.zeros(pos + 64, np.uint8)
    for o, f in zip(offs, frames):
        arena[o:o + len(f)] = np.frombuffer(f, np.uint8)
    return arena, np.array(offs, np.uint64), np.array([len(f) for f in frames], np.uint32)


def test_column_table_matches_abi(zp):
    lib = zp._lib.hip()
    assert [c[0] for c in orc.COLUMN_SPEC] == zp.columns.NAMES
    for k, (name, dt, w) in enumerate(orc.COLUMN_SPEC):
        assert lib.zp_col_width(k) == w * np.dtype(dt).itemsize == zp.columns.width(name), name
    assert lib.zp_col_width(len(orc.COLUMN_SPEC)) == 0 and lib.zp_col_width(-1) == 0


def test_oracle_columns_vs_getters(zp, golden):
    frames = frames_corpus(zp, golden, 1500)
    arena, offs, lens = pack(frames)
    recs, ext = orc.parse_batch(arena, offs, lens)
    cols = orc.columns(arena, offs, lens, recs)
    nok = 0
    for i, f in enumerate(frames):
        want = getter_columns(zp, f, recs[i], ext[:, i])
        nok += int(recs[i]["err"]) == 0
        for name, _, _ in orc.COLUMN_SPEC:
            assert np.array_equal(cols[name][i], want[name]), (i, name, f.hex())
    assert nok > 300


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["corpus", "c3", "c4", "c5", "c6"])
def test_gpu_columns_vs_oracle(zp, golden, case):
    import torch
    d = torch.device("cuda:0")
    if case == "corpus":
        arena, offs, lens = pack(frames_corpus(zp, golden, 6000, seed=7))
        a = torch.from_numpy(arena).to(d)
        o = torch.from_numpy(offs.astype(np.int64)).to(d)
        l_ = torch.from_numpy(lens.astype(np.int32)).to(d)
    else:
        a, o, l_ = zp.batch.generate(case, 50000, first=31337, device=d)
        arena, offs, lens = a.cpu().numpy(), o.cpu().numpy(), l_.cpu().numpy()
    recs, _ = zp.batch.parse_batch(a, o, l_)
    got = zp.columns.extract(a, o, l_, recs)
    # a subset request leaves the others untouched and fills the same values
    sub = zp.columns.extract(a, o, l_, recs, names=["src_port", "dest_addr"])
    torch.cuda.synchronize()
    want = orc.columns(arena, offs, lens, orc.parse_batch(arena, offs, lens)[0])
    for name in zp.columns.NAMES:
        g = got[name].cpu().numpy()
        assert np.array_equal(g, want[name]), (case, name, np.nonzero(
            (g != want[name]).reshape(len(g), -1).any(1))[0][:5])
    for name in ("src_port", "dest_addr"):
        assert np.array_equal(sub[name].cpu().numpy(), want[name])
    # parse_with_columns gives the same records and columns on every path:
    # the fused pass, parse + extract, and "auto" while it alternates and
    # times both (the first calls of a workload) and after it has chosen
    zp.columns.reset_auto()                             # this traffic: a fresh workload
    for mode in ["fused", "split"] + ["auto"] * 7:
        frecs, _, fcols = zp.columns.parse_with_columns(a, o, l_, mode=mode)
        fsub = zp.columns.parse_with_columns(a, o, l_, names=["tcp_seq", "vlan_tci"],
                                             mode=mode)[2]
        torch.cuda.synchronize()
        assert torch.equal(frecs, recs), mode
        for name in zp.columns.NAMES:
            assert np.array_equal(fcols[name].cpu().numpy(), want[name]), (mode, case, name)
        for name in ("tcp_seq", "vlan_tci"):
            assert np.array_equal(fsub[name].cpu().numpy(), want[name]), mode
    assert zp.columns.auto_choice(a, o.numel(), zp.columns.NAMES) in ("fused", "split")


@pytest.mark.gpu
def test_parse_with_columns_fresh_arenas(zp):
    """A caller that hands parse_with_columns(mode="auto") a fresh arena per
    batch: the workload is keyed by shape and stack mix, not by the buffer,
    so the choice made on the first arenas holds for the later ones (no
    re-timing per batch); the remembered workloads stay bounded. Results
    equal the fused path's on every call."""
    import torch
    d = torch.device("cuda:0")
    C = zp.columns
    C.reset_auto()
    a0, o, l_ = zp.batch.generate("c5", 1 << 16, first=5, device=d)
    names = ["src_addr", "dest_addr", "src_port", "dest_port", "protocol"]
    want_r, _, want_c = C.parse_with_columns(a0, o, l_, names=names, mode="fused")
    keep = []
    t0 = C.auto_timings
    for k in range(12):
        a = a0.clone()                                  # a fresh buffer each batch
        keep.append(a)
        r, _, c = C.parse_with_columns(a, o, l_, names=names)
        torch.cuda.synchronize()
        assert torch.equal(r, want_r) and all(torch.equal(c[x], want_c[x]) for x in names), k
    # call 1 (mix unknown) timed once; from call 2 the mix is known: 4 timed
    # calls, the choice on call 6, none timed after
    assert C.auto_timings - t0 == 5, C.auto_timings - t0
    assert C.auto_choice(keep[-1], o.numel(), names) in ("fused", "split")
    assert C.auto_choice(a0, o.numel(), names) == C.auto_choice(keep[0], o.numel(), names)
    assert len(C._auto) <= C._AUTO_MAX
    C.reset_auto()


@pytest.mark.gpu
def test_parse_with_columns_reused_arena_changed_traffic(zp, monkeypatch):
    """One arena buffer reused while its traffic changes from c3 (plain IPv4)
    to c4 (IPv6 chains behind VLAN tags): the sampled stack mix changes, so
    the c4 traffic becomes a workload of its own and is timed and decided
    afresh instead of inheriting c3's choice. No call waits for the device
    (synchronize is refused while the calls run). Results equal the oracle
    path's on every call."""
    import torch
    d = torch.device("cuda:0")
    C = zp.columns
    C.reset_auto()
    monkeypatch.setattr(C, "_SAMPLE_EVERY", 2)
    n = 1 << 15
    a3, o3, l3 = zp.batch.generate("c3", n, first=3, device=d)
    a4, o4, l4 = zp.batch.generate("c4", n, first=4, device=d)
    buf = torch.zeros(max(a3.numel(), a4.numel()), dtype=torch.uint8, device=d)
    names = ["src_addr", "dest_addr", "src_port", "dest_port", "l4_proto"]
    want = {}
    for tag, a, o, l_ in (("c3", a3, o3, l3), ("c4", a4, o4, l4)):
        buf[:a.numel()] = a
        want[tag] = C.parse_with_columns(buf, o, l_, names=names, mode="fused")
    torch.cuda.synchronize()

    def refuse(*a, **k):
        raise AssertionError("parse_with_columns(mode='auto') waited for the device")
    keys = []
    for tag, a, o, l_ in (("c3", a3, o3, l3), ("c4", a4, o4, l4)):
        buf[:a.numel()] = a
        for k in range(10):
            with monkeypatch.context() as m:
                m.setattr(torch.cuda, "synchronize", refuse)
                m.setattr(torch.cuda.Event, "synchronize", refuse)
                m.setattr(torch.cuda.Stream, "synchronize", refuse)
                r, _, c = C.parse_with_columns(buf, o, l_, names=names)
            torch.cuda.synchronize()                    # the test's own check only
            wr, _, wc = want[tag]
            assert torch.equal(r, wr) and all(torch.equal(c[x], wc[x]) for x in names), (tag, k)
        st = C._shapes[C._shape_key(buf, n, names)]
        keys.append(st.mix)
        assert C.auto_choice(buf, n, names) in ("fused", "split"), tag
    assert keys[0] != keys[1], keys                      # c4 is another workload
    assert keys[0] == (4, 0, 0), keys                    # c3: all plain IPv4
    C.reset_auto()


@pytest.mark.gpu
def test_parse_with_columns_auto_under_graph_capture(zp):
    """parse_with_columns(mode="auto") inside a HIP graph capture (ADVICE
    r05): no timing events, no sampling, no synchronisation; the captured
    launch replays to the fused path's results."""
    import torch
    d = torch.device("cuda:0")
    C = zp.columns
    C.reset_auto()
    a, o, l_ = zp.batch.generate("c5", 1 << 14, first=8, device=d)
    names = ["src_addr", "dest_port", "l4_proto"]
    want_r, _, want_c = C.parse_with_columns(a, o, l_, names=names, mode="fused")
    torch.cuda.synchronize()
    t0 = C.auto_timings
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        r, _, c = C.parse_with_columns(a, o, l_, names=names, check=False)
    for _ in range(2):
        r.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(r, want_r) and all(torch.equal(c[x], want_c[x]) for x in names)
    assert C.auto_timings == t0 and not C._shapes
    C.reset_auto()
