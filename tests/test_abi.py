"""CPU: the C-ABI libraries load and export every symbol their headers
declare (no GPU compute calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
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
    assert lib.zp_abi_version() == 3
    assert lib.zp_err_str(0) == b""
    for code, s in want.items():
        assert lib.zp_err_str(code).decode() == s
    assert lib.zp_err_str(38) is None and lib.zp_err_str(-1) is None
    for code in range(38):
        assert lib.zp_err_str(code) is not None


def test_record_layout(zp):
    """zp_record / zp_ext_offsets (ABI v2) as the numpy dtypes see them."""
    r, e = zp.records.RECORD_DTYPE, zp.records.EXT_DTYPE
    assert r.itemsize == 16 and e.itemsize == 16
    assert r.fields["err"][1] == 4 and r.fields["eth_len"][1] == 5
    assert r.fields["inner_off"][1] == 8
    assert r.fields["l4_off"][1] == 12
    assert e.fields["len"][1] == 0 and e.fields["off"][1] == 2


def test_no_cpu_fallback(zp):
    """The batch API refuses host tensors instead of parsing on the CPU."""
    import torch
    a = torch.zeros(64, dtype=torch.uint8)
    o = torch.zeros(1, dtype=torch.int64)
    l = torch.full((1,), 64, dtype=torch.int32)
    with pytest.raises(RuntimeError):
        zp.batch.parse_batch(a, o, l)
