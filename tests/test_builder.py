"""Batched PacketBuilder.

CPU: the oracle's builder restatement (oracle/zp_oracle.c zpo_build) emits
the reference's exact builder vectors (builder.rs:1052-1296), agrees with the
independent Python restatement (tests/pybuilder.py) on random valid chains,
reaches every builder error, and its frames parse back through the parse
oracle. GPU: zp_build_batch_device is byte-exact against the oracle (frame
bytes, partial writes on error, header_len, error codes) on random valid and
invalid chains, truncated buffers, random prior buffer contents, unaligned
frames and frames past the LDS staging size.
"""
import random

import numpy as np
import pytest

import oracle as orc
from pybuilder import Builder

M1 = [0x34, 0x97, 0xf6, 0x94, 0x02, 0x0f]
M2 = [0x04, 0xb4, 0xfe, 0x9a, 0x81, 0xc7]
IP1, IP2 = [192, 168, 1, 1], [192, 168, 1, 2]
S6 = [0x20, 0x01, 0x0d, 0xb8, 0x85, 0xa3, 0, 0, 0, 0, 0x8a, 0x2e, 0x03, 0x70, 0x73, 0x34]
D6 = [0xfe, 0x80, 0, 0, 0, 0, 0, 0, 0x02, 0x02, 0xb3, 0xff, 0xfe, 0x1e, 0x83, 0x29]


def run_oracle(zp, chains, lens, fill=None, align=0, gap=0):
    """Packs buffers (initial content `fill` per frame or zeros), runs the
    oracle; returns (arena, offs, lens, results, packed batch)."""
    batch = zp.builder.BuildBatch()
    for c in chains:
        batch.add(c)
    ops, op_start, data = batch.pack()
    offs, pos = [], align
    for l_ in lens:
        offs.append(pos)
        pos += l_ + gap
    arena = np.zeros(pos + 64, np.uint8)
    if fill is not None:
        for o, l_, f in zip(offs, lens, fill):
            arena[o:o + l_] = f[:l_]
    before = arena.copy()
    offs = np.array(offs, np.uint64)
    lens = np.array(lens, np.uint32)
    res = orc.build_batch(arena, offs, lens, ops, op_start, data)
    return before, arena, offs, lens, res.view(zp.builder.RESULT_DTYPE).reshape(-1), (ops, op_start, data)


def reference_chains(zp):
    C = zp.builder.Chain
    return [
        ("arp_in_ethernet", 42, C().ethernet(M1, [0xff] * 6, 2054)
         .arp(1, 2048, 6, 4, 1, M1, IP1, [0] * 6, IP2)),
        ("tcp_in_ipv4_in_ethernet", 54, C().ethernet(M1, M2, 2048)
         .ipv4(99, 5, 99, 123, 12345, 54321, 99, 12345, 123, 6, IP1, IP2)
         .tcp(IP1, 99, IP2, 11, 123, 321, 11, 99, 99, 4321, 1234)),
        ("udp_in_ipv4_in_ethernet", 54, C().ethernet(M1, M2, 2048)
         .ipv4(99, 5, 99, 123, 12345, 54321, 99, 12345, 123, 6, IP1, IP2)
         .udp(IP1, 99, IP2, 11, 4321)),
        ("icmpv4_in_ipv4_in_ethernet", 64, C().ethernet(M1, M2, 2048)
         .ipv4(4, 5, 99, 123, 12345, 54321, 99, 12345, 123, 1, IP1, IP2).icmpv4(8, 0)),
        ("build_parse_ipv6", 64, C().ethernet(M1, M2, 34525).ipv6(6, 5, 4, 31, 17, 10, S6, D6)
         .udp(S6, 99, D6, 80, 10)),
    ]


def test_oracle_builder_reference_vectors(zp, golden):
    vec = {v["name"]: bytes.fromhex(v["bytes"]) for v in golden["builder_vectors"]}
    cases = reference_chains(zp)
    _, arena, offs, lens, res, _ = run_oracle(zp, [c for _, _, c in cases], [l for _, l, _ in cases])
    for (name, l_, _), o, r in zip(cases, offs, res):
        assert r["err"] == 0 and arena[o:o + l_].tobytes() == vec[name], name


def test_oracle_builder_very_complex_packet(zp):
    """builder.rs:1450-1556: the full extension chain + IPv4-in-IPv6 + TCP,
    built by the oracle, parses back with the reference's offsets."""
    pay = list(range(1, 11))
    c = (zp.builder.Chain().ethernet_qinq(M1, M2, 34525, 200, 100)
         .ipv6(6, 5, 4, 3, 0, 255, [0] * 16, [0] * 16)
         .hop_by_hop(60, 1, [1] * 8).destination_options1(43, 1, [1] * 8)
         .routing_header(44, 1, 2, 3, [2] * 8).fragment_header(51, 255, True, 0x04050607)
         .authentication_header(60, 2, 305419896, 2271560481, [1] * 8)
         .destination_options2(4, 1, [1] * 8)
         .ipv4(4, 5, 0, 0, 150, 0, 0, 0, 64, 6, IP1, IP2)
         .tcp(IP1, 99, IP2, 11, 123, 321, 11, 99, 99, 4321, 1234, pay))
    _, arena, offs, lens, res, _ = run_oracle(zp, [c], [300])
    assert res[0]["err"] == 0 and res[0]["ops_done"] == 10
    f = arena[:300].tobytes()
    want = (Builder(300).ethernet_qinq(M1, M2, 34525, 200, 100)
            .ipv6(6, 5, 4, 3, 0, 255, [0] * 16, [0] * 16)
            .hop_by_hop(60, 1, [1] * 8).destination_options1(43, 1, [1] * 8)
            .routing_header(44, 1, 2, 3, [2] * 8).fragment_header(51, 255, True, 0x04050607)
            .authentication_header(60, 2, 305419896, 2271560481, [1] * 8)
            .destination_options2(4, 1, [1] * 8)
            .ipv4(4, 5, 0, 0, 150, 0, 0, 0, 64, 6, IP1, IP2)
            .tcp(IP1, 99, IP2, 11, 123, 321, 11, 99, 99, 4321, 1234, pay).build())
    assert f == want
    err, rec, ext = orc.parse_one(f)
    assert err == 0 and rec["eth_len"] == 22 and rec["inner_off"] == 150 and rec["l4_off"] == 170
    # slot order hop_by_hop, routing, fragment, auth, dest1, dest2 (headers.rs:20-25)
    assert list(ext[0]["off"]) == [0, 32, 48, 56, 16, 72]
    assert res[0]["header_len"] == 170 + 44


# ---- random chains ---------------------------------------------------------

def rb(rng, k):
    return [rng.randrange(256) for _ in range(k)]


def random_chain(zp, rng, valid=True, pay_max=120):
    """A chain walking the typestate graph with random arguments, plus the
    same chain on tests/pybuilder.py (valid chains only) and a buffer length
    large enough for it (valid) or anything (invalid). Payloads are up to
    pay_max - 1 bytes (past 128 B the GPU copies them as a wave)."""
    C = zp.builder.Chain()
    P = []                                    # pybuilder calls, replayed later
    need = 0

    def both(name, *a):
        getattr(C, name)(*a)
        P.append((name, a))

    et = rng.choice([0x0800, 0x86DD, 0x0806])
    tag = rng.randrange(3)
    if tag == 0:
        both("ethernet", rb(rng, 6), rb(rng, 6), et); need = 14
    elif tag == 1:
        both("ethernet_vlan", rb(rng, 6), rb(rng, 6), et, rng.randrange(65536)); need = 18
    else:
        both("ethernet_qinq", rb(rng, 6), rb(rng, 6), et, rng.randrange(65536), rng.randrange(65536)); need = 22
    l3 = rng.choice(["arp", "v4", "v6"]) if valid else rng.choice(["arp", "v4", "v6", "tcp"])
    if l3 == "arp":
        both("arp", rng.randrange(65536), rng.randrange(65536), rng.randrange(256), rng.randrange(256),
             rng.randrange(65536), rb(rng, 6), rb(rng, 4), rb(rng, 6), rb(rng, 4))
        return C, P, need + 28
    if l3 == "tcp":                            # not allowed after ethernet: TRANSITION
        C.tcp(rb(rng, 4), 1, rb(rng, 4), 2, 3, 4, 5, 0, 2, 9, 0)
        return C, None, need + 64
    addr = 4
    ihl = 5 if valid else rng.choice([5, 5, 6, 15, 0])
    if l3 == "v4":
        both("ipv4", rng.choice([4, 4, 15]), ihl, rng.randrange(64), rng.randrange(4),
             rng.randrange(65536), rng.randrange(65536), rng.randrange(8), rng.randrange(8192),
             rng.randrange(256), rng.randrange(256), rb(rng, 4), rb(rng, 4))
        need += ihl * 4
        st = "v4"
    else:
        both("ipv6", 6, rng.randrange(256), rng.randrange(1 << 20), rng.randrange(65536),
             rng.randrange(256), rng.randrange(256), rb(rng, 16), rb(rng, 16))
        need += 40
        addr = 16
        st = "v6"
        # extension chain in builder order, random subset
        after_d1 = False
        for kind in ("hbh", "d1", "rt", "fr", "ah", "d2"):
            if after_d1 and kind != "rt":
                break                            # destination_options1 -> routing only
            if rng.random() < 0.35 or (after_d1 and rng.random() < 0.5):
                after_d1 = kind == "d1"
                if kind in ("hbh", "d1", "d2"):
                    el = rng.randrange(1, 4)
                    opt = rb(rng, el * 8 if valid else rng.choice([el * 8, 4, el * 8 + 1]))
                    both({"hbh": "hop_by_hop", "d1": "destination_options1",
                          "d2": "destination_options2"}[kind], rng.randrange(256), el, opt)
                    need += (el + 1) * 8
                elif kind == "rt":
                    el = rng.randrange(1, 4)
                    both("routing_header", rng.randrange(256), el, rng.randrange(256),
                         rng.randrange(256), rb(rng, el * 8 if valid else rng.choice([el * 8, 2])))
                    need += (el + 1) * 8
                elif kind == "fr":
                    both("fragment_header", rng.randrange(256), rng.randrange(65536),
                         rng.random() < 0.5, rng.randrange(1 << 32))
                    need += 8
                else:
                    pl = rng.randrange(1, 5)
                    both("authentication_header", rng.randrange(256), pl, rng.randrange(1 << 32),
                         rng.randrange(1 << 32), rb(rng, (pl - 1) * 4 if valid else rng.randrange(40)))
                    need += (pl + 2) * 4
        if not valid and rng.random() < 0.2:
            C.hop_by_hop(0, 1, [0] * 8)          # HBH after others: TRANSITION (or first)
    if rng.random() < 0.3:                       # IP-in-IP
        if rng.random() < 0.5:
            both("ipv4", 4, 5, 0, 0, rng.randrange(65536), 0, 0, 0, 64, rng.randrange(256),
                 rb(rng, 4), rb(rng, 4))
            need += 20
            addr, st = 4, "v4e"
        else:
            both("ipv6", 6, 0, 0, 0, rng.randrange(256), 64, rb(rng, 16), rb(rng, 16))
            need += 40
            addr, st = 16, "v6e"
    l4 = rng.choice(["tcp", "udp", "icmp"])
    pay = None
    if rng.random() < 0.6:
        pay = rb(rng, rng.randrange(0, pay_max))
    if l4 == "tcp":
        doff = rng.choice([5, 6, 8]) if valid else rng.choice([5, 15, 0, 2])
        both("tcp", rb(rng, addr), rng.randrange(65536), rb(rng, addr), rng.randrange(65536),
             rng.randrange(1 << 32), rng.randrange(1 << 32), doff, rng.randrange(16),
             rng.randrange(256), rng.randrange(65536), rng.randrange(65536), pay)
        need += max(doff * 4, 20) + (len(pay) if pay else 0)
    elif l4 == "udp":
        both("udp", rb(rng, addr), rng.randrange(65536), rb(rng, addr), rng.randrange(65536),
             rng.randrange(65536), pay)
        need += 8 + (len(pay) if pay else 0)
    elif st in ("v4", "v4e"):
        both("icmpv4", rng.randrange(256), rng.randrange(256), pay)
        need += 8 + (len(pay) if pay else 0)
    else:
        both("icmpv6", rb(rng, 16), rb(rng, 16), rng.randrange(256), rng.randrange(256), pay)
        need += 8 + (len(pay) if pay else 0)
    return C, P, need


def replay_pybuilder(P, size, fill):
    b = Builder(size)
    b.b[:] = bytes(fill[:size])
    for name, a in P:
        getattr(b, name)(*a)
    return b.build()


@pytest.mark.parametrize("pay_max", [120, 1500])
def test_oracle_builder_vs_pybuilder(zp, pay_max):
    rng = random.Random(2024 + pay_max)
    chains, pys, lens, fills = [], [], [], []
    for _ in range(600):
        c, p, need = random_chain(zp, rng, valid=True, pay_max=pay_max)
        size = need + rng.randrange(0, 200)
        chains.append(c); pys.append(p); lens.append(size)
        fills.append(np.array(rb(rng, size), np.uint8))
    _, arena, offs, lens_, res, _ = run_oracle(zp, chains, lens, fill=fills, align=5, gap=3)
    for i, (p, o, l_) in enumerate(zip(pys, offs, lens)):
        assert res[i]["err"] == 0, (i, res[i])
        assert arena[o:o + l_].tobytes() == replay_pybuilder(p, l_, fills[i]), i


def test_oracle_builder_errors(zp):
    """Every builder error is reachable with the reference's message."""
    C = zp.builder.Chain
    v4 = lambda c: c.ethernet(M1, M2, 2048).ipv4(4, 5, 0, 0, 0, 0, 0, 0, 64, 6, IP1, IP2)
    v6 = lambda c: c.ethernet(M1, M2, 34525).ipv6(6, 0, 0, 0, 0, 64, S6, D6)
    cases = [
        (C().ethernet(M1, M2, 1), 10, "ETH_SLICE"),
        (C().ethernet_vlan(M1, M2, 1, 2), 16, "ETH_VLAN"),
        (C().ethernet_qinq(M1, M2, 1, 2, 3), 20, "ETH_QINQ"),
        (C().ethernet(M1, M2, 2054).arp(1, 2, 3, 4, 5, M1, IP1, M2, IP2), 30, "ARP_SLICE"),
        (v4(C()), 30, "IPV4_SLICE"),
        (C().ethernet(M1, M2, 2048).ipv4(4, 15, 0, 0, 0, 0, 0, 0, 64, 6, IP1, IP2), 50, "PANIC"),
        (C().ethernet(M1, M2, 2048).ipv4(4, 15, 0, 0, 0, 0, 0, 0, 64, 6, IP1, IP2)
         .udp(IP1, 1, IP2, 2, 3), 80, "UDP_SLICE"),
        (v6(C()).hop_by_hop(17, 1, [1] * 8).udp(S6, 1, D6, 2, 3), 64, "UDP_DATA"),
        (v6(C()), 40, "IPV6_SLICE"),
        (v4(C()).tcp(IP1, 1, IP2, 2, 3, 4, 5, 0, 2, 9, 0), 40, "TCP_SLICE"),
        (v4(C()).tcp(IP1, 1, IP2, 2, 3, 4, 5, 0, 2, 9, 0, [1] * 30), 64, "TCP_PAYLOAD"),
        (v4(C()).tcp(IP1, 1, IP2, 2, 3, 4, 15, 0, 2, 9, 0, [1]), 64, "PANIC"),
        (v4(C()).tcp(IP1, 1, IP2, 2, 3, 4, 15, 0, 2, 9, 0), 64, "OK"),
        (v4(C()).udp(IP1, 1, IP2, 2, 3, [1] * 40), 64, "TCP_PAYLOAD"),
        (v4(C()).icmpv4(8, 0, [1] * 40), 64, "ICMPV4_PAYLOAD"),
        (v4(C()).icmpv4(8, 0), 38, "ICMP_SLICE"),
        (v6(C()).icmpv6(S6, D6, 1, 2, [3] * 20), 64, "ICMPV6_PAYLOAD"),
        (v6(C()).hop_by_hop(6, 1, [1] * 4), 100, "OPTIONS_MIN"),
        (v6(C()).hop_by_hop(6, 1, [1] * 16), 100, "OPTIONS_MATCH"),
        (v6(C()).hop_by_hop(6, 2, [1] * 16), 64, "OPTIONS_EXCEED"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8), 58, "OPTIONS_SLICE"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8).tcp(S6, 1, D6, 2, 3, 4, 5, 0, 2, 9, 0), 66, "TCP_DATA"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8).tcp(S6, 1, D6, 2, 3, 4, 5, 0, 2, 9, 0), 70, "TCP_SLICE"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8).udp(S6, 1, D6, 2, 3), 69, "UDP_DATA"),
        (v6(C()).hop_by_hop(58, 1, [1] * 8).icmpv6(S6, D6, 1, 2), 69, "ICMPV6_DATA"),
        (v6(C()).hop_by_hop(0, 1, [1] * 8).destination_options1(6, 1, [1] * 8), 69, "DEST_DATA"),
        (v6(C()).destination_options1(6, 1, [1] * 8).routing_header(6, 1, 0, 0, [1] * 8), 69, "ROUTING_DATA"),
        (v6(C()).routing_header(6, 1, 0, 0, [1] * 2), 100, "ROUTING_MIN"),
        (v6(C()).routing_header(6, 1, 0, 0, [1] * 16), 100, "ROUTING_MATCH"),
        (v6(C()).routing_header(6, 2, 0, 0, [1] * 16), 70, "ROUTING_EXCEED"),
        (v6(C()).routing_header(6, 2, 0, 0, [1] * 16), 60, "ROUTING_SLICE"),
        (v6(C()).fragment_header(6, 1, True, 7), 60, "PANIC"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8).fragment_header(6, 1, True, 7), 66, "ROUTING_DATA"),
        (v6(C()).authentication_header(6, 1, 2, 3, [1] * 40), 80, "AUTH_EXCEED"),
        (v6(C()).authentication_header(6, 1, 2, 3, []), 60, "AUTH_SLICE"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8).authentication_header(6, 1, 2, 3, []), 66, "AUTH_DATA"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8).destination_options2(6, 1, [1] * 8), 66, "DEST_DATA"),
        (v6(C()).authentication_header(6, 4, 2, 3, []), 66, "OK"),      # header_len past the end
        (v6(C()).authentication_header(6, 4, 2, 3, []).destination_options2(6, 1, [1] * 8), 66,
         "DEST_DATA"),
        (v6(C()).hop_by_hop(0, 3, [1] * 24).hop_by_hop(0, 3, [1] * 24), 200, "TRANSITION"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8).ipv4(4, 5, 0, 0, 0, 0, 0, 0, 1, 1, IP1, IP2), 66, "IPV4_DATA"),
        (v6(C()).hop_by_hop(6, 1, [1] * 8).ipv6(6, 0, 0, 0, 0, 1, S6, D6), 66, "IPV6_DATA"),
        # ARP_DATA and ICMPV4_DATA cannot occur: no step before them can move
        # header_len past the buffer (ethernet and IPv4 bound it, ipv4.rs:123)
        (C().ethernet(M1, M2, 2054).arp(1, 2, 3, 4, 5, M1, IP1, M2, IP2).icmpv4(1, 2), 90, "TRANSITION"),
        (C().ipv4(4, 5, 0, 0, 0, 0, 0, 0, 64, 6, IP1, IP2), 90, "TRANSITION"),
    ]
    names = {"OK": 0, "ETH_SLICE": 1, "ETH_VLAN": 2, "ETH_QINQ": 3, "ARP_DATA": 4, "ARP_SLICE": 5,
             "IPV4_DATA": 6, "IPV4_SLICE": 7, "IPV6_DATA": 8, "IPV6_SLICE": 9, "TCP_DATA": 10,
             "TCP_SLICE": 11, "TCP_PAYLOAD": 12, "UDP_DATA": 13, "UDP_SLICE": 14,
             "ICMPV4_DATA": 15, "ICMP_SLICE": 16, "ICMPV4_PAYLOAD": 17, "ICMPV6_DATA": 18,
             "ICMPV6_PAYLOAD": 19, "HBH_DATA": 20, "DEST_DATA": 21, "OPTIONS_SLICE": 22,
             "OPTIONS_MIN": 23, "OPTIONS_MATCH": 24, "OPTIONS_EXCEED": 25, "ROUTING_DATA": 26,
             "ROUTING_SLICE": 27, "ROUTING_MIN": 28, "ROUTING_MATCH": 29, "ROUTING_EXCEED": 30,
             "AUTH_DATA": 31, "AUTH_SLICE": 32, "AUTH_EXCEED": 33, "PANIC": 34, "TRANSITION": 35}
    before, arena, offs, lens, res, _ = run_oracle(zp, [c for c, _, _ in cases],
                                                   [l_ for _, l_, _ in cases])
    got = [int(r["err"]) for r in res]
    assert got == [names[w] for _, _, w in cases], [
        (i, w, g) for i, ((_, _, w), g) in enumerate(zip(cases, got)) if names[w] != g]
    # a refused chain (TRANSITION) writes nothing; a failing step keeps earlier writes
    for (c, l_, w), o, r in zip(cases, offs, res):
        if w == "TRANSITION":
            assert not arena[o:o + l_].any()
        elif w == "IPV4_SLICE":
            assert arena[o:o + 6].tolist() == M2
    lib = zp._lib.hip()
    assert zp.builder.error_string(12) == "Payload is too large to fit in the TCP packet."
    assert zp.builder.error_string(26) == "Data too short to contain an IPv6 Routing header."
    assert zp.builder.error_string(0) == "" and zp.builder.error_string(36) is None
    assert lib.zp_build_err_str(35) is not None


# ---- GPU ---------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("seed,big,gap,pay_max", [(1, False, 5, 120), (2, True, 5, 120),
                                                  (3, False, 0, 120), (4, True, 0, 120),
                                                  (5, True, 3, 1500), (6, False, 0, 1500)])
def test_gpu_builder_vs_oracle(zp, seed, big, gap, pay_max):
    """gap 0 packs the frames back to back: the lane path then also writes the
    previous frame's unchanged tail bytes of each header's first 64-B sector
    (when that frame's lane writes nothing there), next to pending, failing
    and truncated neighbours. pay_max 1500 sends payloads past the window
    through the wave copy behind every chain shape (extension headers,
    IP-in-IP, invalid chains)."""
    import torch
    rng = random.Random(seed)
    chains, lens, fills = [], [], []
    for k in range(3000):
        valid = rng.random() < 0.6
        c, _, need = random_chain(zp, rng, valid=valid, pay_max=pay_max)
        r = rng.random()
        if r < 0.15:
            size = rng.randrange(0, need + 1)                  # truncated: error paths
        elif big and r < 0.3:
            size = rng.randrange(2000, 9000)                    # past the LDS staging size
        else:
            size = need + rng.randrange(0, 300)
        chains.append(c); lens.append(size)
        fills.append(np.array(rb(rng, size), np.uint8) if rng.random() < 0.5
                     else np.zeros(size, np.uint8))
    before, want, offs, lens_, wres, _ = run_oracle(zp, chains, lens, fill=fills, align=7, gap=gap)
    d = torch.device("cuda:0")
    arena = torch.from_numpy(before).to(d)
    batch = zp.builder.BuildBatch()
    for c in chains:
        batch.add(c)
    got = batch.run(arena, torch.from_numpy(offs.astype(np.int64)).to(d),
                    torch.from_numpy(lens_.astype(np.int32)).to(d))
    torch.cuda.synchronize()
    ga = arena.cpu().numpy()
    bad = [i for i, (o, l_) in enumerate(zip(offs, lens_))
           if ga[o:o + l_].tobytes() != want[o:o + l_].tobytes()]
    assert not bad, (len(bad), bad[:5], [int(wres[i]["err"]) for i in bad[:5]])
    assert ga.tobytes() == want.tobytes()                   # gaps untouched too
    assert got.tobytes() == wres.tobytes()
    errs = set(int(e) for e in wres["err"])
    assert len(errs) >= 12, sorted(errs)


@pytest.mark.gpu
def test_gpu_builder_reference_vectors(zp, golden):
    import torch
    vec = {v["name"]: bytes.fromhex(v["bytes"]) for v in golden["builder_vectors"]}
    cases = reference_chains(zp)
    d = torch.device("cuda:0")
    offs = np.cumsum([0] + [l_ + 3 for _, l_, _ in cases[:-1]]).astype(np.int64) + 1
    arena = torch.zeros(int(offs[-1]) + 128, dtype=torch.uint8, device=d)
    batch = zp.builder.BuildBatch()
    for _, _, c in cases:
        batch.add(c)
    res = batch.run(arena, torch.from_numpy(offs).to(d),
                    torch.tensor([l_ for _, l_, _ in cases], dtype=torch.int32, device=d))
    a = arena.cpu().numpy()
    for (name, l_, _), o, r in zip(cases, offs, res):
        assert r["err"] == 0 and a[o:o + l_].tobytes() == vec[name], name


@pytest.mark.gpu
def test_gpu_builder_lane_path_edges(zp):
    """The lane-per-frame path at its edges: every frame alignment (0-15),
    payload copies ending exactly at / one byte past the 128-B window, frames
    of exactly 64 B, all-zero ICMPv4 segments (S == 0 -> checksum 0xFFFF) and
    segments whose sum folds to 0xFFFF; byte-exact vs the oracle."""
    import torch
    C = zp.builder.Chain
    chains, lens, fills = [], [], []
    for shift in range(16):
        wlen = 128 - shift
        for extra in (-1, 0, 1):
            pay = bytes(range(1, wlen - 42 + extra + 1)) if wlen - 42 + extra > 0 else b""
            chains.append(C().ethernet(M1, M2, 2048).ipv4(4, 5, 0, 0, 186, 7, 0, 0, 64, 17, IP1, IP2)
                          .udp(IP1, 5, IP2, 6, 166, pay))
            lens.append(200)
            fills.append(np.full(200, 0xAB, np.uint8))
        chains.append(C().ethernet([0] * 6, [0] * 6, 2048).ipv4(4, 5, 0, 0, 50, 0, 0, 0, 0, 1,
                                                                [0] * 4, [0] * 4).icmpv4(0, 0))
        lens.append(64)
        fills.append(np.zeros(64, np.uint8))
        chains.append(C().ethernet(M1, M2, 34525).ipv6(6, 0, 0, 0, 58, 1, S6, D6)
                      .icmpv6(S6, D6, 128, 0, b"\xff\xff" * 3))
        lens.append(64 + shift)
        fills.append(np.full(64 + shift, 0xFF, np.uint8))
    # every frame starts at a different offset mod 16
    offs, pos = [], 0
    for k, l_ in enumerate(lens):
        pos += (k % 16 - pos % 16) % 16
        offs.append(pos)
        pos += l_
    batch = zp.builder.BuildBatch()
    for c in chains:
        batch.add(c)
    ops, op_start, data = batch.pack()
    arena = np.zeros(pos + 64, np.uint8)
    for o, l_, f in zip(offs, lens, fills):
        arena[o:o + l_] = f
    want = arena.copy()
    wres = orc.build_batch(want, np.array(offs, np.uint64), np.array(lens, np.uint32), ops,
                           op_start, data).view(zp.builder.RESULT_DTYPE).reshape(-1)
    d = torch.device("cuda:0")
    ta = torch.from_numpy(arena).to(d)
    got = batch.run(ta, torch.tensor(offs, dtype=torch.int64, device=d),
                    torch.tensor(lens, dtype=torch.int32, device=d))
    torch.cuda.synchronize()
    assert ta.cpu().numpy().tobytes() == want.tobytes()
    assert got.tobytes() == wres.tobytes()


@pytest.mark.gpu
def test_gpu_builder_descriptor_bounds_refused(zp):
    """The builder writes into the arena: a frame past its end, a negative
    length or wrong descriptor dtypes are refused before the kernel runs."""
    import torch
    d = torch.device("cuda:0")
    C = zp.builder.Chain
    chain = C().ethernet([0] * 6, [1] * 6, 0x0806)
    arena = torch.zeros(100, dtype=torch.uint8, device=d)
    for offs, lens in (([40], [64]), ([0], [-1]), ([-8], [64])):
        with pytest.raises(ValueError):
            zp.builder.BuildBatch().add(chain).run(
                arena, torch.tensor(offs, dtype=torch.int64, device=d),
                torch.tensor(lens, dtype=torch.int32, device=d))
    with pytest.raises(ValueError):
        zp.builder.BuildBatch().add(chain).run(
            arena, torch.tensor([0], dtype=torch.int32, device=d),
            torch.tensor([64], dtype=torch.int32, device=d))
    # overlapping (and duplicated) frames are refused: the kernel writes them
    two = zp.builder.BuildBatch().add(chain).add(chain)
    for offs in ([0, 10], [20, 20], [25, 0]):
        with pytest.raises(ValueError, match="overlap"):
            two.run(arena, torch.tensor(offs, dtype=torch.int64, device=d),
                    torch.tensor([30, 30], dtype=torch.int32, device=d))
    assert int(arena.sum().item()) == 0                  # nothing written
    res = zp.builder.BuildBatch().add(chain).run(
        arena, torch.tensor([36], dtype=torch.int64, device=d),
        torch.tensor([64], dtype=torch.int32, device=d))
    assert int(res[0]["err"]) == 0 and int(arena[36 + 12].item()) == 0x08


@pytest.mark.gpu
@pytest.mark.parametrize("P,gap", [(200, 0), (200, 3), (1000, 0), (1000, 5)])
def test_gpu_builder_payload_copies(zp, P, gap):
    """set_payload(Some(..)) copies of P = 200 / 1000 bytes, each frame from
    its own range of the data blob (the lane path copies past its window
    straight from the blob; tcp.rs:108-114, udp.rs:82-88, builder.rs:473-474),
    over IPv4 and IPv6 with every tagging, frames 0-300 B longer than the
    chain, some too short (TCP_PAYLOAD / ICMPV4_PAYLOAD errors), random prior
    contents; every arena byte, header_len and error identical to the oracle."""
    import torch
    rng = random.Random(P * 7 + gap)
    C = zp.builder.Chain
    chains, lens, fills = [], [], []
    for k in range(2500):
        tag = rng.randrange(3)
        v6 = rng.random() < 0.3
        et = 0x86DD if v6 else 0x0800
        c = C()
        if tag == 0:
            c.ethernet(rb(rng, 6), rb(rng, 6), et); hl = 14
        elif tag == 1:
            c.ethernet_vlan(rb(rng, 6), rb(rng, 6), et, rng.randrange(65536)); hl = 18
        else:
            c.ethernet_qinq(rb(rng, 6), rb(rng, 6), et, rng.randrange(65536), rng.randrange(65536)); hl = 22
        if v6:
            c.ipv6(6, rng.randrange(256), rng.randrange(1 << 20), rng.randrange(65536), 17, 64,
                   rb(rng, 16), rb(rng, 16))
            hl += 40
            addr = 16
        else:
            c.ipv4(4, 5, 0, 0, rng.randrange(65536), rng.randrange(65536), 0, 0, 64,
                   rng.choice([6, 17, 1]), rb(rng, 4), rb(rng, 4))
            hl += 20
            addr = 4
        pay = bytes(rb(rng, P - rng.randrange(0, 9)))        # ragged copy lengths
        l4 = rng.choice(["tcp", "udp", "icmp"])
        if l4 == "tcp":
            c.tcp(rb(rng, addr), rng.randrange(65536), rb(rng, addr), rng.randrange(65536),
                  rng.randrange(1 << 32), rng.randrange(1 << 32), 5, 0, 0x18, 65535, 0, pay)
            hl += 20
        elif l4 == "udp":
            c.udp(rb(rng, addr), rng.randrange(65536), rb(rng, addr), rng.randrange(65536),
                  rng.randrange(65536), pay)
            hl += 8
        elif v6:
            c.icmpv6(rb(rng, 16), rb(rng, 16), 128, 0, pay)
            hl += 8
        else:
            c.icmpv4(8, 0, pay)
            hl += 8
        size = hl + len(pay) + rng.randrange(0, 300) if rng.random() < 0.9 else \
            hl + rng.randrange(0, len(pay))                  # payload does not fit
        chains.append(c); lens.append(size)
        fills.append(np.array(rb(rng, size), np.uint8))
    before, want, offs, lens_, wres, packed = run_oracle(zp, chains, lens, fill=fills, align=3,
                                                         gap=gap)
    ops, op_start, data = packed
    assert len(data) > 2000 * (P - 8)                         # one blob range per frame
    d = torch.device("cuda:0")
    arena = torch.from_numpy(before).to(d)
    batch = zp.builder.BuildBatch()
    for c in chains:
        batch.add(c)
    got = batch.run(arena, torch.from_numpy(offs.astype(np.int64)).to(d),
                    torch.from_numpy(lens_.astype(np.int32)).to(d))
    torch.cuda.synchronize()
    ga = arena.cpu().numpy()
    bad = [i for i, (o, l_) in enumerate(zip(offs, lens_))
           if ga[o:o + l_].tobytes() != want[o:o + l_].tobytes()]
    assert not bad, (len(bad), bad[:5], [int(wres[i]["err"]) for i in bad[:5]])
    assert ga.tobytes() == want.tobytes()
    assert got.tobytes() == wres.tobytes()
    errs = {int(e) for e in wres["err"]}
    assert 0 in errs and len(errs) >= 2, sorted(errs)


@pytest.mark.gpu
def test_gpu_builder_payload_overlaps(zp):
    """Payloads past the window behind chains whose writes overlap (the wave
    copy moves the whole payload, zp_build.hip ZB_PAY_HDR): a TCP data offset
    below 5 (the payload overwrites its own header, then the checksum the
    payload; tcp.rs:108-114, builder.rs:473-474), an IPv4 IHL of 0 (the L4
    header and payload overwrite the IPv4 header), authentication data longer
    than its header (authentication.rs:84-92) under a payload that fits and
    one that does not (ICMPV6_PAYLOAD); every frame start offset mod 16, every
    byte, header_len and error identical to the oracle."""
    import torch
    rng = random.Random(99)
    C = zp.builder.Chain
    chains, lens, fills = [], [], []
    for k in range(16 * 24):
        kind = k % 4
        c = C().ethernet(rb(rng, 6), rb(rng, 6), 0x86DD if kind >= 2 else 0x0800)
        pay = bytes(rb(rng, rng.randrange(90, 400)))
        if kind == 0:                                   # TCP data offset 0 or 2
            c.ipv4(4, 5, 0, 0, 60, 1, 0, 0, 64, 6, rb(rng, 4), rb(rng, 4))
            c.tcp(rb(rng, 4), 1, rb(rng, 4), 2, 3, 4, rng.choice([0, 2]), 0, 0x18, 9, 0, pay)
            need = 14 + 20 + 20 + len(pay)
        elif kind == 1:                                 # IPv4 IHL 0
            c.ipv4(4, 0, 0, 0, 60, 1, 0, 0, 64, 17, rb(rng, 4), rb(rng, 4))
            c.udp(rb(rng, 4), 1, rb(rng, 4), 2, 8 + len(pay), pay)
            need = 14 + 20 + len(pay)
        else:                                           # AH data past its header length
            c.ipv6(6, 0, 0, 0, 51, 64, rb(rng, 16), rb(rng, 16))
            c.authentication_header(58, 1, rng.randrange(1 << 32), rng.randrange(1 << 32),
                                    rb(rng, rng.randrange(8, 40)))
            c.icmpv6(rb(rng, 16), rb(rng, 16), 128, 0, pay)
            need = 14 + 40 + 12 + 8 + len(pay)
        size = need + rng.randrange(0, 200) if kind != 3 else need - rng.randrange(1, 60)
        chains.append(c); lens.append(max(size, 64))
        fills.append(np.array(rb(rng, max(size, 64)), np.uint8))
    before, want, offs, lens_, wres, _ = run_oracle(zp, chains, lens, fill=fills, align=1, gap=1)
    assert len({int(o) % 16 for o in offs}) == 16
    d = torch.device("cuda:0")
    arena = torch.from_numpy(before).to(d)
    batch = zp.builder.BuildBatch()
    for c in chains:
        batch.add(c)
    got = batch.run(arena, torch.from_numpy(offs.astype(np.int64)).to(d),
                    torch.from_numpy(lens_.astype(np.int32)).to(d))
    torch.cuda.synchronize()
    ga = arena.cpu().numpy()
    bad = [i for i, (o, l_) in enumerate(zip(offs, lens_))
           if ga[o:o + l_].tobytes() != want[o:o + l_].tobytes()]
    assert not bad, (len(bad), bad[:5], [int(wres[i]["err"]) for i in bad[:5]])
    assert ga.tobytes() == want.tobytes()
    assert got.tobytes() == wres.tobytes()
    errs = {int(e) for e in wres["err"]}
    assert 0 in errs and len(errs) >= 2, sorted(errs)
