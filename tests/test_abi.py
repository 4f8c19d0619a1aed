"""CPU: the C-ABI libraries load and export every symbol their headers
declare (no GPU compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"static inline[^{]*\{[^}]*\}", "", text)    # header-only accessors
    return sorted(set(re.findall(r"\b(zp_\w+)\s*\(", text)) - {"zp_err", "zp_record"})


@pytest.mark.parametrize("header,lib", [("zero_packet.h", "libzp_hip.so"),
                                        ("zero_packet_host.h", "libzp_host.so")])
def test_exports(built, header, lib):
    names = declared(header)
    assert len(names) >= 2
    so = ctypes.CDLL(os.path.join(ROOT, "zero-packet_amd", lib))
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing


def test_hip_exports_complete(built):
    names = declared("zero_packet.h")
    for n in ["zp_parse_batch_device", "zp_parse_batch_host", "zp_parse_one", "zp_ctx_create",
              "zp_ctx_destroy", "zp_err_str", "zp_abi_version", "zp_last_error",
              "zp_gen_lengths_device", "zp_gen_frames_device"]:
        assert n in names


def test_err_strings(zp):
    """zp_err_str returns the exact reference strings (transcribed from the
    cited lines; see include/zero_packet.h)."""
    want = {
        1: "Slice needs to be least 64 bytes long to be a valid Ethernet frame.",
        5: "Invalid double VLAN tag.",
        7: "ARP operation field is invalid, expected request (1) or reply (2).",
        12: "IPv4 total length field is invalid. Does not match actual length.",
        13: "IPv4 checksum is invalid.",
        17: "If Hop-by-Hop Options is present, then it must be the first extension header.",
        19: "Indicated IPv6 options header length exceeds the allocated buffer.",
        26: "TCP data offset field is invalid. Indicated header length is too short.",
        30: "Slice is too short to contain an ICMP header.",
        34: "IPv4 encapsulated checksum is invalid.",
        35: "IPv6 encapsulated checksum is invalid.",
    }
    lib = zp._lib.hip()
    assert lib.zp_abi_version() == 6
    assert lib.zp_err_str(0) == b""
    for code, s in want.items():
        assert lib.zp_err_str(code).decode() == s
    assert lib.zp_err_str(38) is None and lib.zp_err_str(-1) is None
    for code in range(38):
        assert lib.zp_err_str(code) is not None


def test_record_layout(zp):
    """zp_record / zp_ext_offsets (ABI v5) as the numpy dtypes see them, and
    unpack() decoding the packed fields."""
    r, e = zp.records.RECORD_DTYPE, zp.records.EXT_DTYPE
    assert r.itemsize == 8 and e.itemsize == 16
    assert r.fields["flags"][1] == 0 and r.fields["offs"][1] == 4
    assert e.fields["len"][1] == 0 and e.fields["off"][1] == 2 and e.fields["final_nh"][1] == 14
    rec = np.zeros(3, r)
    rec[0] = (zp.records.F_ETHERNET | zp.records.F_IPV6 | zp.records.F_IP_IN_IP | zp.records.F_TCP |
              2 << 24, 170 | 150 << 18)
    rec[1] = (29 << 26, 0)                                   # Err(UDP_LENGTH)
    rec[2] = (zp.records.F_ETHERNET | zp.records.F_IPV6 | zp.records.F_IP_IN_IP |
              zp.records.F_UDP | 3 << 24, 264014)              # far-L4 form (ABI v5)
    u = zp.records.unpack(rec)
    assert list(u["err"]) == [0, 29, 0] and list(u["eth_len"]) == [22, 0, 0]
    assert list(u["l4_off"]) == [170, 0, 264014] and list(u["inner_off"]) == [150, 0, 0]
    assert list(zp.records.is_far(rec)) == [False, False, True]
    assert u["flags"][0] == (zp.records.F_ETHERNET | zp.records.F_IPV6 | zp.records.F_IP_IN_IP |
                             zp.records.F_TCP)
    assert list(zp.records.rec_err(rec)) == [0, 29, 0]


def test_no_cpu_fallback(zp):
    """The batch API refuses host tensors instead of parsing on the CPU."""
    import torch
    a = torch.zeros(64, dtype=torch.uint8)
    o = torch.zeros(1, dtype=torch.int64)
    l = torch.full((1,), 64, dtype=torch.int32)
    with pytest.raises(RuntimeError):
        zp.batch.parse_batch(a, o, l)
