"""The C++ facade (include/zero_packet.hpp) against the Python facade and the
oracle: tests/cpp/facade_main.cpp prints one summary line per frame built
from zp::PacketParser; the same line is built here from the Python
PacketParser over the oracle's record. CPU: from_record (header-only, no
GPU). GPU: zp::PacketParser::parse through zp_parse_one (libzp_hip.so)."""
import importlib
import os
import subprocess

import numpy as np
import pytest

import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "facade_main.cpp")
OUT = os.path.join(ROOT, "tests", "cpp", "_build")


def _build(gpu):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "facade_gpu" if gpu else "facade_cpu")
    deps = [SRC, os.path.join(ROOT, "include", "zero_packet.hpp"),
            os.path.join(ROOT, "include", "zero_packet.h")]
    if os.path.exists(exe) and all(os.path.getmtime(exe) > os.path.getmtime(d) for d in deps):
        return exe
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I",
           os.path.join(ROOT, "include"), "-o", exe, SRC]
    if gpu:
        lib = os.path.join(ROOT, "zero-packet_amd")
        cmd += ["-DZP_FACADE_GPU", "-L" + lib, "-lzp_hip", "-Wl,-rpath," + lib]
    subprocess.run(cmd, check=True)
    return exe


def _ext_summary(eh):
    if eh is None:
        return ";ext=-"
    s = f";ext={eh.total_headers_len},{eh.final_next_header}"
    for name, short in (("hop_by_hop", "hbh"), ("routing", "rt"), ("fragment", "frag"),
                        ("auth_header", "ah"), ("destination_1st", "d1"),
                        ("destination_2nd", "d2")):
        r = getattr(eh, name)
        if r is not None:
            s += f",{short}@{len(r.bytes)}"
    return s


def _v6(r):
    return (f"{len(r.bytes)},{r.next_header()},{r.final_next_header()},"
            f"{r.extension_headers_len},{len(r.upper_layer_payload())},{r.flow_label()}"
            + _ext_summary(r.extension_headers))


def py_summary(zp, frame, rec, ext):
    try:
        p = zp.PacketParser.from_record(frame, rec, ext)
    except zp.ZeroPacketError as e:
        return f"err={e.code}|{e}"
    out = ["ok"]
    if p.ethernet is not None:
        e = p.ethernet
        v = e.vlan_tag()
        d = e.double_vlan_tag()
        out.append(f"eth:{e.header_len()},{e.ethertype()},"
                   f"{f'{v[0]}/{v[1]}' if v else '-'},{f'{d[0][1]}/{d[1][1]}' if d else '-'}")
    if p.arp is not None:
        out.append(f"arp:{p.arp.oper()},{p.arp.htype()},{p.arp.spa()[3]}")
    if p.ipv4 is not None:
        r = p.ipv4
        out.append(f"ipv4:{len(r.bytes)},{r.ihl()},{r.total_length()},{r.protocol()},"
                   f"{r.checksum()},{r.src_ip()[0]}")
    if p.ipv6 is not None:
        out.append("ipv6:" + _v6(p.ipv6))
    if p.ip_in_ip is not None:
        if p.ip_in_ip.kind == "ipv4":
            out.append(f"iip4:{len(p.ip_in_ip.reader.bytes)},{p.ip_in_ip.reader.protocol()}")
        else:
            out.append("iip6:" + _v6(p.ip_in_ip.reader))
    if p.tcp is not None:
        t = p.tcp
        out.append(f"tcp:{len(t.bytes)},{t.src_port()},{t.dest_port()},{t.data_offset()},"
                   f"{t.flags()}")
    if p.udp is not None:
        u = p.udp
        out.append(f"udp:{len(u.bytes)},{u.src_port()},{u.dest_port()},{u.length()}")
    if p.icmpv4 is not None:
        out.append(f"icmp4:{len(p.icmpv4.bytes)},{p.icmpv4.icmp_type()},{p.icmpv4.icmp_code()}")
    if p.icmpv6 is not None:
        out.append(f"icmp6:{len(p.icmpv6.bytes)},{p.icmpv6.icmp_type()}")
    return " ".join(out)


def _frames(zp, golden):
    """Golden fixtures + samples of every config + mutated copies (errors)."""
    frames = [bytes.fromhex(f["bytes"]) for f in golden["fixtures"]]
    rng = np.random.default_rng(7)
    for cfg in ("c2", "c3", "c4", "c5"):
        a, o, l = zp.batch.generate_host(cfg, 120)
        for i in range(len(o)):
            f = bytearray(a[int(o[i]):int(o[i]) + int(l[i])].tobytes())
            frames.append(bytes(f))
            if i % 3 == 0:
                f[int(rng.integers(0, len(f)))] ^= int(rng.integers(1, 256))
                frames.append(bytes(f))
    # L4 readers past byte 262,143: the record's far-L4 form (ABI v5)
    from test_l4_far import CASES, deep_frame
    frames += [deep_frame(lv, **kw)[0] for lv, kw in CASES]
    return frames


def _expected(zp, frames):
    lines = []
    for f in frames:
        _, rec, ext = orc.parse_one_abi(f)
        lines.append((f, rec, ext, py_summary(zp, f, rec, ext)))
    return lines


def test_cpp_facade_from_record_matches_python_facade(zp, golden):
    exe = _build(gpu=False)
    exp = _expected(zp, _frames(zp, golden))
    inp = "".join(f"{f.hex()} {rec.tobytes().hex()} {ext.tobytes().hex()}\n"
                  for f, rec, ext, _ in exp)
    out = subprocess.run([exe, "cpu"], input=inp, capture_output=True, text=True,
                         check=True).stdout.splitlines()
    assert len(out) == len(exp)
    for got, (f, rec, _, want) in zip(out, exp):
        assert got == want, (f.hex()[:64], got, want)
    assert sum(1 for _, r, _, _ in exp if int(r["flags"]) >> 26) > 10
    assert any("iip6:" in s for *_, s in exp) and any(";ext=-" not in s and "ipv6" in s
                                                      for *_, s in exp)
    assert sum(1 for _, r, _, _ in exp if (int(r["flags"]) >> 24) & 3 == 3) == 4   # far-L4


@pytest.mark.gpu
def test_cpp_facade_parse_on_gpu(zp, golden):
    exe = _build(gpu=True)
    exp = _expected(zp, _frames(zp, golden))
    inp = "".join(f"{f.hex()}\n" for f, *_ in exp)
    out = subprocess.run([exe, "gpu"], input=inp, capture_output=True, text=True,
                         check=True, timeout=300).stdout.splitlines()
    assert len(out) == len(exp)
    for got, (f, _, _, want) in zip(out, exp):
        assert got == want, (f.hex()[:64], got, want)


# ---- §8(f) rows through the C++ facade: zp::PacketBuilder, zp::Ring -------

BUILDER_SRC = os.path.join(ROOT, "tests", "cpp", "builder_main.cpp")


def _compile_snippet(body, tmp_path):
    src = tmp_path / "snippet.cpp"
    src.write_text('#include "zero_packet.hpp"\nint main() {\n  uint8_t buf[128] = {0};\n'
                   '  std::array<uint8_t, 6> m{};\n  std::array<uint8_t, 4> a{};\n'
                   '  std::array<uint8_t, 16> a6{};\n  (void)a; (void)a6;\n'
                   f"  auto b = zp::PacketBuilder<>(buf, 128){body};\n  (void)b;\n}}\n")
    return subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                           str(src)], capture_output=True, text=True)


@pytest.mark.parametrize("body,ok", [
    (".ethernet(m, m, 2048).ipv4(4, 5, 0, 0, 50, 0, 0, 0, 64, 17, a, a).udp(a, 1, a, 2, 30)", True),
    (".ethernet(m, m, 34525).ipv6(6, 0, 0, 0, 0, 64, a6, a6).hop_by_hop(0, 1, zp::Bytes{})"
     ".routing_header(0, 1, 0, 0, zp::Bytes{}).ipv4(4, 5, 0, 0, 0, 0, 0, 0, 1, 6, a, a)"
     ".tcp(a, 1, a, 2, 3, 4, 5, 0, 2, 9, 0)", True),
    (".ethernet(m, m, 2048).tcp(a, 1, a, 2, 3, 4, 5, 0, 2, 9, 0)", False),          # no L3
    (".ethernet(m, m, 34525).ipv6(6, 0, 0, 0, 0, 64, a6, a6)"
     ".destination_options1(0, 1, zp::Bytes{}).fragment_header(0, 0, false, 0)", False),
    (".ethernet(m, m, 2048).ipv4(4, 5, 0, 0, 0, 0, 0, 0, 1, 58, a, a).icmpv6(a6, a6, 1, 0)", False),
    (".ethernet(m, m, 2048).ipv4(4, 5, 0, 0, 0, 0, 0, 0, 1, 6, a, a).tcp(a6, 1, a6, 2, 3, 4, 5, 0, 2, 9, 0)",
     False),                                                                         # &[u8; 4] state
])
def test_cpp_builder_typestate(body, ok, tmp_path):
    """The typestate graph of builder.rs:817-909 is enforced at compile time,
    as in the Rust builder (CPU: g++ -fsyntax-only)."""
    r = _compile_snippet(body, tmp_path)
    assert (r.returncode == 0) == ok, r.stderr[-2000:]
    if not ok and "static assertion" in r.stderr:
        assert "builder.rs:817-909" in r.stderr


@pytest.mark.gpu
def test_cpp_builder_and_ring(zp, golden):
    """builder.rs's own tests through zp::PacketBuilder (GPU build, GPU parse
    back) and a zp::Ring round trip."""
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "builder_gpu")
    lib = os.path.join(ROOT, "zero-packet_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I",
                    os.path.join(ROOT, "include"), "-o", exe, BUILDER_SRC, "-L" + lib, "-lzp_hip",
                    "-Wl,-rpath," + lib], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "ALL OK" in out.stdout, out.stdout[-3000:] + out.stderr[-2000:]
    got = dict(l.split(" ", 1) for l in out.stdout.splitlines() if not l.startswith(("OK", "ALL")))
    for v in golden["builder_vectors"]:
        assert got[v["name"]] == v["bytes"], v["name"]
    fx = {f["name"]: f["bytes"] for f in golden["fixtures"]}
    assert got["build_parse_very_complex_packet"] == fx["build_parse_very_complex_packet"]
