"""Standalone readers: the reference's direct use (README.md:110-115),
`TcpReader::new(&packet[off..])?` and the getters, for the twelve readers,
plus the checksum primitives (checksum.rs:5,33,67).

The checked constructors (zp_reader_new, host code of libzp_hip.so) are
compared with the oracle's restatement (oracle/zp_oracle.c zpo_reader_new)
at every header offset of a fuzz corpus: the same Err code or the same
Ethernet header length / IPv6 extension chain. The Python facade
(XReader.new) and the C++ facade (XReader::create / try_create, with the
fallible accessors) are compared with each other line by line. CPU only: no
device is involved."""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KINDS = 12
READERS = ["EthernetReader", "ArpReader", "IPv4Reader", "IPv6Reader", "OptionsHeaderReader",
           "RoutingHeaderReader", "FragmentHeaderReader", "AuthenticationHeaderReader",
           "TcpReader", "UdpReader", "Icmpv4Reader", "Icmpv6Reader"]


@pytest.fixture(scope="module")
def frames(zp, golden):
    from test_gpu_parity import fuzz_frames
    fr = [bytes.fromhex(fx["bytes"]) for fx in golden["fixtures"]]
    # truncated prefixes (the tagged ones included): slices that end inside
    # the VLAN tags, the IP headers and the extension chain
    pre = [f[:k] for f in fr for k in range(0, min(len(f), 96))]
    return fr + pre + fuzz_frames(zp, golden, 360, 3, repair_p=0.3)


def offsets(f):
    """Every offset a header can start at (all lie in the first 160 bytes),
    and the last 48 (short slices)."""
    return sorted(set(range(0, min(len(f), 160) + 1)) | set(range(max(0, len(f) - 48), len(f) + 1)))


def test_reader_kinds_match_header(zp):
    h = open(os.path.join(ROOT, "include", "zero_packet.h")).read()
    for k, name in enumerate(["ETHERNET", "ARP", "IPV4", "IPV6", "OPTIONS", "ROUTING", "FRAGMENT",
                              "AUTH", "TCP", "UDP", "ICMPV4", "ICMPV6"]):
        assert f"ZP_READER_{name} = {k}," in h
        assert getattr(zp.records, f"READER_{name}") == k
        assert getattr(zp, READERS[k]).KIND == k


def test_library_constructors_match_oracle_every_offset(zp, frames):
    lib = zp._lib.hip()
    info = np.zeros(1, zp.records.READER_INFO_DTYPE)
    seen = set()
    chains = 0
    for f in frames:
        buf = ctypes.create_string_buffer(f, max(len(f), 1))
        base = ctypes.addressof(buf)
        for o in offsets(f):
            n = len(f) - o
            for k in range(KINDS):
                err, hl, fl, fnh, x = orc.reader_new_at(base + o, n, k)
                rc = lib.zp_reader_new(k, base + o, n, info.ctypes.data)
                assert rc == err, (f.hex(), o, k, rc, err)
                seen.add((k, rc))
                if rc:
                    continue
                i = info[0]
                assert (int(i["header_len"]), int(i["flags"]), int(i["final_nh"])) == (hl, fl, fnh), \
                    (f.hex(), o, k)
                if fl:
                    chains += 1
                    assert i["ext"].tobytes() == x.tobytes(), (f.hex(), o, k)
    errs = {rc for _, rc in seen if rc}
    # every constructor Err the readers have: too-short slices of each kind,
    # the VLAN checks, the extension walk's errors
    for name in ("ETH_SLICE_TOO_SHORT", "ETH_VLAN_TOO_SHORT", "ETH_QINQ_TOO_SHORT",
                 "ETH_INVALID_QINQ", "ARP_TOO_SHORT", "IPV4_TOO_SHORT", "IPV6_TOO_SHORT",
                 "EXT_HBH_NOT_FIRST", "EXT_OPTIONS_TOO_SHORT", "EXT_OPTIONS_EXCEEDS",
                 "EXT_ROUTING_TOO_SHORT", "EXT_ROUTING_EXCEEDS", "EXT_FRAGMENT_TOO_SHORT",
                 "EXT_AUTH_TOO_SHORT", "TCP_TOO_SHORT", "UDP_TOO_SHORT", "ICMP_TOO_SHORT"):
        assert zp.records.ERR[name] in errs, name
    assert chains > 1000


def test_library_rejects_bad_arguments(zp):
    lib = zp._lib.hip()
    assert lib.zp_reader_new(12, b"x" * 64, 64, None) == -1
    assert lib.zp_reader_new(-1, b"x" * 64, 64, None) == -1
    assert lib.zp_reader_new(8, None, 20, None) == -1
    assert lib.zp_reader_new(8, None, 0, None) == zp.records.ERR["TCP_TOO_SHORT"]


def _len_of(fn):
    try:
        return str(len(fn()))
    except IndexError:
        return "panic"
    except Exception as e:                     # ZeroPacketError
        return f"e{e.code}"


def _ext_summary(r):
    s = f" fnh={r.final_next_header()} ulp={len(r.upper_layer_payload())}"
    eh = r.extension_headers
    if eh is None:
        return s + " ext=-"
    s += f" ext={eh.total_headers_len},{eh.final_next_header}"
    for name, short in (("hop_by_hop", "hbh"), ("routing", "rt"), ("fragment", "frag"),
                        ("auth_header", "ah"), ("destination_1st", "d1"),
                        ("destination_2nd", "d2")):
        x = getattr(eh, name)
        if x is not None:
            s += f",{short}@{len(r.bytes) - len(x.bytes)}"
    return s


def py_line(zp, k, b):
    """The line tests/cpp/readers_main.cpp prints, from the Python facade."""
    try:
        r = getattr(zp, READERS[k]).new(b)
    except zp.ZeroPacketError as e:
        return f"err={e.code}|{e}"
    if k == 0:
        v = r.vlan_tag()
        return f"ok hl={r.header_len()} et={r.ethertype()} vlan={v[1] if v else '-'}"
    if k == 1:
        return f"ok oper={r.oper()}"
    if k == 2:
        try:
            vc = str(int(r.valid_checksum()))
        except zp.ZeroPacketError as e:
            vc = f"e{e.code}"
        return f"ok hl={r.header_len()} vc={vc} p={_len_of(r.payload)}"
    if k == 3:
        return "ok" + _ext_summary(r)
    if k == 4:
        return f"ok hl={r.header_len()} opt={_len_of(r.options)} p={_len_of(r.payload)}"
    if k == 5:
        return f"ok hl={r.header_len()} data={_len_of(r.data)} p={_len_of(r.payload)}"
    if k == 6:
        return f"ok fo={r.fragment_offset()} m={int(r.m_flag())} id={r.identification()}"
    if k == 7:
        return f"ok hl={r.header_len()} ad={_len_of(r.authentication_data)} p={_len_of(r.payload)}"
    if k == 8:
        return f"ok hl={r.header_len()} h={_len_of(r.header)} p={_len_of(r.payload)}"
    if k == 9:
        return f"ok len={r.length()} p={len(r.payload())}"
    return f"ok t={r.icmp_type()} c={r.icmp_code()}"


def _slices(frames, step):
    rng = random.Random(11)
    out = []
    for f in frames:
        for o in offsets(f)[rng.randrange(step)::step]:
            out.append(f[o:])
    return out


def test_python_constructors_match_oracle(zp, frames):
    """XReader.new raises the oracle's Err (exact reference string) or builds
    the reader; IPv6 readers carry the oracle's extension chain."""
    lib = zp._lib.hip()
    for b in _slices(frames, 5):
        for k in range(KINDS):
            err, hl, fl, fnh, x = orc.reader_new(k, b)
            cls = getattr(zp, READERS[k])
            if err:
                with pytest.raises(zp.ZeroPacketError) as ei:
                    cls.new(b)
                assert ei.value.code == err and str(ei.value) == lib.zp_err_str(err).decode()
                continue
            r = cls.new(b)
            assert r.bytes == b
            if k == 0:
                assert r.header_len() == hl
            if k == 3:
                assert r.final_next_header() == fnh
                assert (r.extension_headers is not None) == bool(fl)
                if fl:
                    assert r.extension_headers_len == int(x["len"])


def _build_readers_exe():
    out = os.path.join(ROOT, "tests", "cpp", "_build")
    os.makedirs(out, exist_ok=True)
    exe = os.path.join(out, "readers")
    src = os.path.join(ROOT, "tests", "cpp", "readers_main.cpp")
    lib = os.path.join(ROOT, "zero-packet_amd")
    deps = [src, os.path.join(ROOT, "include", "zero_packet.hpp"),
            os.path.join(ROOT, "include", "zero_packet.h"), os.path.join(lib, "libzp_hip.so")]
    if not (os.path.exists(exe) and all(os.path.getmtime(exe) > os.path.getmtime(d) for d in deps)):
        subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I",
                        os.path.join(ROOT, "include"), "-o", exe, src, "-L" + lib, "-lzp_hip",
                        "-Wl,-rpath," + lib], check=True)
    return exe


def test_cpp_constructors_match_python(zp, frames, built):
    """zp::XReader::create / try_create and the fallible accessors (header,
    payload, options, data, authentication_data, valid_checksum) print the
    same line as the Python facade."""
    exe = _build_readers_exe()
    cases = [(k, b) for b in _slices(frames, 9) for k in range(KINDS)]
    inp = "".join(f"r {k} {b.hex()}\n" for k, b in cases)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True,
                         timeout=300).stdout.splitlines()
    assert len(out) == len(cases)
    bad = [(k, b.hex()[:80], got, py_line(zp, k, b)) for (k, b), got in zip(cases, out)
           if got != py_line(zp, k, b)]
    assert not bad, bad[:5]
    kinds = {l.split("|")[0] for l in out if l.startswith("err")}
    assert len(kinds) >= 12
    assert any(" h=e36" in l for l in out) and any(" opt=e37" in l for l in out)
    assert any(" vc=1" in l for l in out) and any("ext=-" not in l and "fnh=" in l for l in out)


def test_tcp_reader_19_bytes(zp, built):
    """tcp.rs:141-145: TcpReader::new on a 19-byte slice is Err with the
    reference's string, in Python and C++; 20 bytes is Ok."""
    msg = "Slice is too short to contain a TCP header."
    with pytest.raises(zp.ZeroPacketError, match=msg) as ei:
        zp.TcpReader.new(bytes(19))
    assert ei.value.code == zp.records.ERR["TCP_TOO_SHORT"]
    assert zp.TcpReader.new(bytes(20)).header_len() == 0
    out = subprocess.run([_build_readers_exe()], input=f"r 8 {bytes(19).hex()}\n",
                         capture_output=True, text=True, check=True).stdout
    assert out.strip() == f"err=25|{msg}"


def test_checksum_primitives(zp, golden, built):
    """checksum.rs:75-133 known answers through the C ABI (Python and C++),
    and random data / accumulators (u32 wrap-around included) against the
    oracle's byte loop."""
    lines, want = [], []
    for kat in golden["checksum_kats"]:
        d = bytes(kat["data"])
        assert zp.internet_checksum(d, kat["acc"]) == kat["checksum"], kat["source"]
        if kat.get("verify"):
            assert zp.verify_internet_checksum(d, kat["acc"])
        lines.append(f"cs {kat['acc']} {d.hex()}")
        want.append(f"{kat['checksum']} {int(kat['checksum'] == 0)}")
    p = golden["pseudo_header_kat"]
    assert zp.pseudo_header(p["src"], p["dst"], p["protocol"], p["length"]) == p["sum"]
    lines.append(f"ph {p['protocol']} {p['length']} {bytes(p['src']).hex()} {bytes(p['dst']).hex()}")
    want.append(str(p["sum"]))
    rng = random.Random(5)
    for _ in range(300):
        d = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 300)))
        acc = rng.choice([0, rng.randrange(1 << 16), rng.randrange(1 << 32), 0xFFFFFFFF - rng.randrange(64)])
        c = orc.internet_checksum(d, acc)
        assert zp.internet_checksum(d, acc) == c
        lines.append(f"cs {acc} {d.hex()}")
        want.append(f"{c} {int(c == 0)}")
        for w in (4, 16):
            s, t = bytes(rng.randrange(256) for _ in range(w)), bytes(rng.randrange(256) for _ in range(w))
            proto, ln = rng.randrange(256), rng.randrange(1 << 40)
            ph = orc.pseudo_header(s, t, proto, ln)
            assert zp.pseudo_header(s, t, proto, ln) == ph
            lines.append(f"ph {proto} {ln} {s.hex()} {t.hex()}")
            want.append(str(ph))
    # a large buffer whose word sum wraps u32 (the reference's release semantics)
    big = b"\xff" * (1 << 17) + b"\x01\x02\x03"
    assert zp.internet_checksum(big, 0xFFFF0000) == orc.internet_checksum(big, 0xFFFF0000)
    out = subprocess.run([_build_readers_exe()], input="\n".join(lines) + "\n",
                         capture_output=True, text=True, check=True).stdout.splitlines()
    assert out == want
    with pytest.raises(ValueError):
        zp.pseudo_header(bytes(4), bytes(16), 6, 20)


def test_host_helpers_without_the_library(zp, golden, monkeypatch):
    """internet_checksum and the EthernetReader view keep working when
    libzp_hip.so cannot be loaded: the Python restatements give
    the checksum.rs:75-133 answers and the oracle's values."""
    import importlib
    parser = importlib.import_module("zero-packet_amd.parser")
    monkeypatch.setattr(parser, "_lib_available", lambda: False)
    for kat in golden["checksum_kats"]:
        d = bytes(kat["data"])
        assert parser.internet_checksum(d, kat["acc"]) == kat["checksum"], kat["source"]
    rng = random.Random(9)
    for _ in range(200):
        d = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 200)))
        acc = rng.choice([0, rng.randrange(1 << 32), 0xFFFFFFFF - rng.randrange(64)])
        assert parser.internet_checksum(d, acc) == orc.internet_checksum(d, acc)
    big = b"\xff" * (1 << 17) + b"\x01\x02\x03"
    assert parser.internet_checksum(big, 0xFFFF0000) == orc.internet_checksum(big, 0xFFFF0000)
    for fx in golden["fixtures"]:
        f = bytes.fromhex(fx["bytes"])
        want = orc.reader_new(0, f)
        if want[0] == 0:
            assert parser.EthernetReader(f).header_len() == want[1]
        else:
            with pytest.raises(parser.ZeroPacketError):
                parser.EthernetReader(f)
    with pytest.raises(parser.ZeroPacketError):
        parser.EthernetReader(bytes(13))
