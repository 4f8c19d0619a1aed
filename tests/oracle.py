"""ctypes wrapper of the CPU oracle (oracle/libzp_oracle.so) — the checker.

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it. Built by `make -C oracle` (also by build()).
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "libzp_oracle.so")
_lib = None

# The oracle's per-frame result, every field unpacked (zpo_record); pack()
# encodes it as the ABI's 8-B zp_record for byte comparisons with the GPU.
RECORD_DTYPE = np.dtype([
    ("flags", "<u4"), ("err", "u1"), ("eth_len", "u1"), ("final_nh", "u1"),
    ("inner_final_nh", "u1"), ("inner_off", "<u4"), ("l4_off", "<u4"),
])
PACKED_DTYPE = np.dtype([("flags", "<u4"), ("offs", "<u4")])
EXT_DTYPE = np.dtype([("len", "<u2"), ("off", "<u2", (6,)), ("final_nh", "u1"),
                      ("reserved", "u1")])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
        l = ctypes.CDLL(LIB)
        vp, u64, i32, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t
        l.zpo_parse.restype = i32
        l.zpo_parse.argtypes = [vp, sz, vp, vp, vp]
        l.zpo_parse_batch.restype = i32
        l.zpo_parse_batch.argtypes = [vp, vp, vp, u64, vp, vp, i32]
        l.zpo_internet_checksum.restype = ctypes.c_uint16
        l.zpo_internet_checksum.argtypes = [vp, sz, ctypes.c_uint32]
        l.zpo_pseudo_header.restype = ctypes.c_uint32
        l.zpo_pseudo_header.argtypes = [vp, vp, sz, ctypes.c_uint8, sz]
        l.zpo_pack.restype = None
        l.zpo_pack.argtypes = [vp, vp, u64, vp]
        _lib = l
    return _lib


def parse_one(frame):
    """-> (err, record[RECORD_DTYPE], ext[EXT_DTYPE] (2,): outer, ip_in_ip chain)"""
    frame = bytes(frame)
    buf = ctypes.create_string_buffer(frame, max(len(frame), 1))
    rec = np.zeros(1, RECORD_DTYPE)
    ext = np.zeros(2, EXT_DTYPE)
    err = lib().zpo_parse(ctypes.addressof(buf), len(frame), rec.ctypes.data, ext[0:].ctypes.data,
                          ext[1:].ctypes.data)
    return err, rec[0], ext


def pack(rec, ext):
    """oracle records (RECORD_DTYPE) + their chains (EXT_DTYPE (2, n), or (2,)
    for one record) -> the ABI's 8-B records (PACKED_DTYPE); an outer chain
    goes inline where the ABI v6 rule says so (zpo_pack)."""
    rec = np.ascontiguousarray(np.atleast_1d(rec), dtype=RECORD_DTYPE)
    ext = np.asarray(ext, dtype=EXT_DTYPE)
    outer = np.ascontiguousarray(ext.reshape(2, -1)[0])
    assert len(outer) == len(rec), "pack: one outer-chain entry per record"
    out = np.zeros(len(rec), PACKED_DTYPE)
    if len(rec):
        lib().zpo_pack(rec.ctypes.data, outer.ctypes.data, len(rec), out.ctypes.data)
    return out


def parse_one_abi(frame):
    """parse_one with the record packed as the ABI's zp_record (what the GPU
    path returns and the facades' from_record takes)."""
    err, rec, ext = parse_one(frame)
    return err, pack(rec, ext)[0], ext


def record_tuple(rec, ext):
    """(err, flags, eth_len, final_nh, inner_final_nh, inner_off, l4_off,
    ext_len, ext_off tuple, inner_ext_len, inner ext_off tuple) of one frame
    (ext: its two zp_ext_offsets entries; zero where there is no chain)."""
    return (int(rec["err"]), int(rec["flags"]), int(rec["eth_len"]), int(rec["final_nh"]),
            int(rec["inner_final_nh"]), int(rec["inner_off"]), int(rec["l4_off"]),
            int(ext[0]["len"]), tuple(int(x) for x in ext[0]["off"]),
            int(ext[1]["len"]), tuple(int(x) for x in ext[1]["off"]))


def reader_new(kind, data):
    """zpo_reader_new: XReader::new of reader `kind` (zp_reader_kind) ->
    (err, header_len, ext flags, final_nh, ext EXT_DTYPE entry)."""
    data = bytes(data)
    buf = ctypes.create_string_buffer(data, max(len(data), 1))
    return reader_new_at(ctypes.addressof(buf), len(data), kind)


def reader_new_at(ptr, n, kind):
    l = lib()
    if not hasattr(l, "_rn_sig"):
        l.zpo_reader_new.restype = ctypes.c_int
        l.zpo_reader_new.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p]
        l._rn_sig = True
    hl, fl, fnh = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint8()
    x = np.zeros(1, EXT_DTYPE)
    err = l.zpo_reader_new(kind, ptr, n, ctypes.byref(hl), ctypes.byref(fl), ctypes.byref(fnh),
                           x.ctypes.data)
    return err, hl.value, fl.value, fnh.value, x[0]


def parse_batch(arena, offs, lens, nthreads=0):
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offs = np.ascontiguousarray(offs).astype(np.uint64, copy=False)
    lens = np.ascontiguousarray(lens).astype(np.uint32, copy=False)
    n = len(offs)
    rec = np.zeros(n, RECORD_DTYPE)
    ext = np.zeros((2, n), EXT_DTYPE)
    if n:
        lib().zpo_parse_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                              rec.ctypes.data, ext.ctypes.data, nthreads)
    return rec, ext


def internet_checksum(data, acc=0):
    data = bytes(data)
    buf = ctypes.create_string_buffer(data, max(len(data), 1))
    return lib().zpo_internet_checksum(ctypes.addressof(buf), len(data), acc)


def pseudo_header(src, dst, protocol, length):
    s = ctypes.create_string_buffer(bytes(src))
    d = ctypes.create_string_buffer(bytes(dst))
    return lib().zpo_pseudo_header(ctypes.addressof(s), ctypes.addressof(d), len(src),
                                   protocol, length)


# zp_col order and element layout (include/zero_packet.h), numpy side.
COLUMN_SPEC = [
    ("dest_mac", np.uint8, 6), ("src_mac", np.uint8, 6), ("ethertype", np.uint16, 1),
    ("vlan_tci", np.uint16, 1), ("vlan_inner_tci", np.uint16, 1), ("arp_oper", np.uint16, 1),
    ("ip_version", np.uint8, 1), ("src_addr", np.uint8, 16), ("dest_addr", np.uint8, 16),
    ("protocol", np.uint8, 1), ("ttl", np.uint8, 1), ("tos", np.uint8, 1),
    ("ip_id", np.uint32, 1), ("ip_len", np.uint16, 1), ("inner_version", np.uint8, 1),
    ("inner_src_addr", np.uint8, 16), ("inner_dest_addr", np.uint8, 16),
    ("inner_protocol", np.uint8, 1), ("l4_proto", np.uint8, 1), ("src_port", np.uint16, 1),
    ("dest_port", np.uint16, 1), ("tcp_seq", np.uint32, 1), ("tcp_ack", np.uint32, 1),
    ("tcp_flags", np.uint8, 1), ("tcp_window", np.uint16, 1), ("icmp_type", np.uint8, 1),
    ("icmp_code", np.uint8, 1), ("l4_checksum", np.uint16, 1), ("payload_off", np.uint32, 1),
]


def columns(arena, offs, lens, recs):
    """zpo_columns: the reader getters restated in C -> {name: numpy array}."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offs = np.ascontiguousarray(offs).astype(np.uint64, copy=False)
    lens = np.ascontiguousarray(lens).astype(np.uint32, copy=False)
    recs = np.ascontiguousarray(recs)
    n = len(offs)
    out = {}
    ptrs = (ctypes.c_void_p * len(COLUMN_SPEC))()
    for k, (name, dt, w) in enumerate(COLUMN_SPEC):
        out[name] = np.zeros((n, w) if w > 1 else (n,), dt)
        ptrs[k] = out[name].ctypes.data
    l = lib()
    l.zpo_columns.restype = ctypes.c_int
    l.zpo_columns.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p]
    if n:
        l.zpo_columns(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, recs.ctypes.data,
                      n, ptrs)
    return out


def build_batch(arena, offs, lens, ops, op_start, data):
    """zpo_build_batch: the PacketBuilder restatement, in place on `arena`
    (numpy uint8, modified); returns results as uint8 [n, 8]."""
    n = len(offs)
    res = np.zeros((n, 8), np.uint8)
    l = lib()
    l.zpo_build_batch.restype = ctypes.c_int
    l.zpo_build_batch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + [ctypes.c_void_p] * 4
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    if n:
        l.zpo_build_batch(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                          ops.ctypes.data, op_start.ctypes.data, data.ctypes.data,
                          res.ctypes.data)
    return res
