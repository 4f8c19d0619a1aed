"""ctypes binding of the C ABI (include/zero_packet.h, include/zero_packet_host.h).

The HIP library libzp_hip.so is the product path; there is no CPU fallback:
if it is missing or fails to load, every parse entry point raises.
Build it with `python -c "import __graft_entry__ as g; g.build()"`.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
HIP_LIB = os.path.join(HERE, "libzp_hip.so")
HOST_LIB = os.path.join(HERE, "libzp_host.so")

_hip = None
_pyhip = None
_host = None

c_u8p = ctypes.c_void_p


def _sig(lib, name, res, args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args
    return f


def hip():
    """The loaded libzp_hip.so (raises if it is not built)."""
    global _hip
    if _hip is None:
        if not os.path.exists(HIP_LIB):
            raise RuntimeError(f"zero-packet_amd: HIP library missing ({HIP_LIB}); "
                               "run __graft_entry__.build() - there is no CPU fallback")
        lib = ctypes.CDLL(HIP_LIB)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        _sig(lib, "zp_abi_version", i32, [])
        _sig(lib, "zp_err_str", ctypes.c_char_p, [i32])
        _sig(lib, "zp_last_error", ctypes.c_char_p, [])
        _sig(lib, "zp_parse_batch_device", i32, [vp, vp, vp, u64, vp, vp, vp])
        _sig(lib, "zp_set_record_slots", i32, [i32])
        _sig(lib, "zp_record_slots_state", i32, [])
        _sig(lib, "zp_ctx_create", vp, [i32, u64])
        _sig(lib, "zp_ctx_destroy", None, [vp])
        _sig(lib, "zp_parse_batch_host", i32, [vp, vp, u64, vp, vp, u64, vp, vp])
        _sig(lib, "zp_parse_batch_host_multi", i32, [vp, i32, vp, u64, vp, vp, u64, vp, vp])
        _sig(lib, "zp_parse_one", i32, [vp, vp, u64, vp, vp])
        _sig(lib, "zp_parse_one_config", i32, [vp, u32])
        _sig(lib, "zp_device_current", i32, [])
        _sig(lib, "zp__one_test_hooks", i32, [vp, u32, u64, u32])   # test hook
        _sig(lib, "zp__one_stats", i32, [vp, vp])                     # test hook
        _sig(lib, "zp_col_width", i32, [i32])
        _sig(lib, "zp_build_err_str", ctypes.c_char_p, [i32])
        _sig(lib, "zp_build_batch_device", i32, [vp, vp, vp, u64, vp, vp, vp, vp, vp])
        _sig(lib, "zp_extract_columns_device", i32, [vp, vp, vp, vp, u64, vp, vp])
        _sig(lib, "zp_parse_batch_columns_device", i32, [vp, vp, vp, u64, vp, vp, vp, vp])
        _sig(lib, "zp_stats_device", i32, [vp, u64, vp, vp])
        _sig(lib, "zp_probe_read_device", i32, [vp, u64, vp, vp])
        _sig(lib, "zp_probe_tiles_device", i32, [vp, u64, u64, vp, vp, vp, vp, vp])
        _sig(lib, "zp_probe_tiles_codes_device", i32, [vp, u64, u64, vp, vp, vp, vp, vp])
        _sig(lib, "zp_gen_lengths_device", i32, [i32, u64, u64, u64, vp, vp])
        _sig(lib, "zp_gen_frames_device", i32, [i32, u64, u64, u64, vp, vp, vp, vp])
        _sig(lib, "zp_reader_new", i32, [i32, vp, u64, vp])
        _sig(lib, "zp_internet_checksum", ctypes.c_uint16, [vp, u64, u32])
        _sig(lib, "zp_verify_internet_checksum", i32, [vp, u64, u32])
        _sig(lib, "zp_pseudo_header", u32, [vp, vp, u32, ctypes.c_uint8, u64])
        _sig(lib, "zp_rec_decode", i32, [vp, vp, u64, vp, vp])
        _hip = lib
    return _hip


def pyhip():
    """libzp_hip.so through ctypes.PyDLL: calls that keep the GIL. For
    zp_parse_one on a frame the resident server answers (~4.5 us), holding
    the GIL is cheaper than handing it over: a hand-off costs the waiting
    thread's wake-up (several us), and with several Python threads parsing
    at once the hand-offs convoy (8 threads: 47k calls/s and an 81 us p50
    against 118k / 8.6 us on one thread, profiles/r06_parse_one_latency.log)."""
    global _pyhip
    if _pyhip is None:
        hip()
        lib = ctypes.PyDLL(HIP_LIB)
        _sig(lib, "zp_device_current", ctypes.c_int, [])
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        _sig(lib, "zp_parse_one", ctypes.c_int, [vp, vp, u64, vp, vp])
        _pyhip = lib
    return _pyhip


def host():
    """The loaded libzp_host.so (CPU generator)."""
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB):
            raise RuntimeError(f"zero-packet_amd: host library missing ({HOST_LIB})")
        lib = ctypes.CDLL(HOST_LIB)
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        _sig(lib, "zp_host_gen_lengths", i32, [i32, u64, u64, u64, vp])
        _sig(lib, "zp_host_gen_frames", i32, [i32, u64, u64, u64, vp, vp, i32])
        _host = lib
    return _host


def check(rc, what):
    if rc < 0:
        msg = hip().zp_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")
    return rc
