"""Batched PacketBuilder (zp_build_batch_device, include/zero_packet.h).

The reference builds one frame with a typestate chain over a caller-sized
buffer (builder.rs:55-909):

    PacketBuilder::new(&mut buf).ethernet(src, dst, 0x0800)?.ipv4(...)?.tcp(...)?.build()

Here a chain is recorded with the same method names and arguments:

    chain = Chain().ethernet(src, dst, 0x0800).ipv4(...).tcp(...)
    batch = BuildBatch(); batch.add(chain) ...
    results = batch.run(arena, offs, lens)          # all chains, in place, on the GPU

Every frame's buffer is arena[offs[i] : offs[i] + lens[i]] (the `&mut [u8]`).
Errors do not raise per frame: results["err"] holds the zp_build_err code
(error_string() gives the reference's message) and, as in the reference, the
bytes written before the failing step stay in the buffer.
"""
import contextlib
import ctypes

import numpy as np
import torch

from . import _lib
from .batch import check_batch

OP_DTYPE = np.dtype([("kind", "u1"), ("b", "u1", (7,)), ("h", "<u2", (4,)), ("w", "<u4", (2,)),
                     ("data_off", "<u4"), ("data_len", "<u4"), ("src", "u1", (16,)),
                     ("dst", "u1", (16,))])
assert OP_DTYPE.itemsize == 64
RESULT_DTYPE = np.dtype([("header_len", "<u4"), ("err", "u1"), ("ops_done", "u1"),
                         ("reserved", "<u2")])
NO_DATA = 0xFFFFFFFF
(ETHERNET, ETHERNET_VLAN, ETHERNET_QINQ, ARP, IPV4, IPV6, HOP_BY_HOP, DEST_OPTS1, ROUTING,
 FRAGMENT, AUTH, DEST_OPTS2, TCP, UDP, ICMPV4, ICMPV6) = range(1, 17)
ERR_PANIC, ERR_TRANSITION = 34, 35


def error_string(code):
    s = _lib.hip().zp_build_err_str(int(code))
    return None if s is None else s.decode()


class Chain:
    """One frame's builder chain: the PacketBuilder methods, recorded."""

    def __init__(self):
        self.ops = []          # (fields dict, data bytes or None)

    def _op(self, kind, data=None, **f):
        self.ops.append((kind, f, data))
        return self

    # datalink (builder.rs:113-236)
    def ethernet(self, src_mac, dest_mac, ethertype):
        return self._op(ETHERNET, src=src_mac, dst=dest_mac, h={0: ethertype})

    def ethernet_vlan(self, src_mac, dest_mac, ethertype, tci):
        return self._op(ETHERNET_VLAN, src=src_mac, dst=dest_mac, h={0: ethertype, 1: tci})

    def ethernet_qinq(self, src_mac, dest_mac, ethertype, tci1, tci2):
        return self._op(ETHERNET_QINQ, src=src_mac, dst=dest_mac,
                        h={0: ethertype, 1: tci1, 2: tci2})

    def arp(self, hardware_type, protocol_type, hardware_address_length,
            protocol_address_length, operation, src_mac, src_ip, dest_mac, dest_ip):
        return self._op(ARP, h={0: hardware_type, 1: protocol_type, 2: operation},
                        b={0: hardware_address_length, 1: protocol_address_length},
                        src=list(src_mac) + list(src_ip), dst=list(dest_mac) + list(dest_ip))

    # network (builder.rs:248-430)
    def ipv4(self, version, ihl, dscp, ecn, total_length, identification, flags,
             fragment_offset, ttl, protocol, src_ip, dest_ip):
        return self._op(IPV4, b={0: version, 1: ihl, 2: dscp, 3: ecn, 4: flags, 5: ttl,
                                 6: protocol},
                        h={0: total_length, 1: identification, 2: fragment_offset},
                        src=src_ip, dst=dest_ip)

    def ipv6(self, version, traffic_class, flow_label, payload_length, next_header, hop_limit,
             src_addr, dest_addr):
        return self._op(IPV6, b={0: version, 1: traffic_class, 2: next_header, 3: hop_limit},
                        w={0: flow_label}, h={0: payload_length}, src=src_addr, dst=dest_addr)

    # IPv6 extension headers (builder.rs:611-806)
    def hop_by_hop(self, next_header, extension_len, options):
        return self._op(HOP_BY_HOP, bytes(options), b={0: next_header, 1: extension_len})

    def destination_options1(self, next_header, extension_len, options):
        return self._op(DEST_OPTS1, bytes(options), b={0: next_header, 1: extension_len})

    def destination_options2(self, next_header, extension_len, options):
        return self._op(DEST_OPTS2, bytes(options), b={0: next_header, 1: extension_len})

    def routing_header(self, next_header, header_ext_len, routing_type, segments_left, data):
        return self._op(ROUTING, bytes(data), b={0: next_header, 1: header_ext_len,
                                                 2: routing_type, 3: segments_left})

    def fragment_header(self, next_header, fragment_offset, m_flag, identification):
        return self._op(FRAGMENT, b={0: next_header, 1: int(bool(m_flag))},
                        h={0: fragment_offset}, w={0: identification})

    def authentication_header(self, next_header, payload_len, spi, seq_num, auth_data):
        return self._op(AUTH, bytes(auth_data), b={0: next_header, 1: payload_len},
                        w={0: spi, 1: seq_num})

    # transport (builder.rs:438-604); payload None = Option::None
    def tcp(self, src_ip, src_port, dest_ip, dest_port, sequence_number, acknowledgment_number,
            data_offset, reserved, flags, window_size, urgent_pointer, payload=None):
        return self._op(TCP, None if payload is None else bytes(payload), src=src_ip,
                        dst=dest_ip, h={0: src_port, 1: dest_port, 2: window_size,
                                        3: urgent_pointer},
                        w={0: sequence_number, 1: acknowledgment_number},
                        b={0: data_offset, 1: reserved, 2: flags})

    def udp(self, src_addr, src_port, dest_addr, dest_port, length, payload=None):
        return self._op(UDP, None if payload is None else bytes(payload), src=src_addr,
                        dst=dest_addr, h={0: src_port, 1: dest_port, 2: length})

    def icmpv4(self, icmp_type, icmp_code, payload=None):
        return self._op(ICMPV4, None if payload is None else bytes(payload),
                        b={0: icmp_type, 1: icmp_code})

    def icmpv6(self, src_addr, dest_addr, icmp_type, icmp_code, payload=None):
        return self._op(ICMPV6, None if payload is None else bytes(payload), src=src_addr,
                        dst=dest_addr, b={0: icmp_type, 1: icmp_code})


def check_disjoint(offs, lens, stream=None):
    """Raises ValueError unless the non-empty frames [offs[i], offs[i] +
    lens[i]) are pairwise disjoint (an empty frame holds no byte, and its
    chain fails at its first step without writing). One device sort and
    reduction on `stream`, then a sync."""
    if offs.numel() < 2:
        return
    dev = offs.device
    on = (torch.cuda.stream(torch.cuda.ExternalStream(int(stream), device=dev))
          if stream is not None else contextlib.nullcontext())
    with on:
        live = lens > 0
        o, ln = offs[live], lens[live].to(torch.int64)
        so, order = torch.sort(o)
        ends = so + ln[order]
        bad = int((ends[:-1] > so[1:]).sum().item())
    if bad:
        raise ValueError(f"{bad} frame(s) overlap the next frame in address order: "
                         "zp_build_batch_device needs disjoint frames")


class BuildBatch:
    """Chains for many frames, packed into the C-ABI arrays."""

    def __init__(self):
        self.chains = []

    def add(self, chain):
        self.chains.append(chain)
        return self

    def pack(self):
        """-> (ops OP_DTYPE[m], op_start uint32[n+1], data uint8[k])"""
        nops = sum(len(c.ops) for c in self.chains)
        ops = np.zeros(nops, OP_DTYPE)
        op_start = np.zeros(len(self.chains) + 1, np.uint32)
        blobs, pos, q = [], 0, 0
        for i, c in enumerate(self.chains):
            op_start[i] = q
            for kind, f, data in c.ops:
                o = ops[q]
                o["kind"] = kind
                for k, v in f.get("b", {}).items():
                    o["b"][k] = v & 0xFF
                for k, v in f.get("h", {}).items():
                    o["h"][k] = v & 0xFFFF
                for k, v in f.get("w", {}).items():
                    o["w"][k] = v & 0xFFFFFFFF
                for key in ("src", "dst"):
                    if key in f:
                        a = bytes(f[key])
                        o[key][:len(a)] = np.frombuffer(a, np.uint8)
                if data is None:
                    o["data_off"], o["data_len"] = 0, NO_DATA
                else:
                    o["data_off"], o["data_len"] = pos, len(data)
                    blobs.append(data)
                    pos += len(data)
                q += 1
        op_start[len(self.chains)] = q
        data = np.frombuffer(b"".join(blobs) or b"\0", np.uint8).copy()
        return ops, op_start, data

    def run(self, arena, offs, lens, stream=None):
        """Executes every chain in place on the device tensors; returns the
        results (numpy RESULT_DTYPE [n])."""
        # the kernel writes into [offs[i], offs[i] + lens[i]) of the arena:
        # dtypes, devices and bounds are checked before it runs (check_batch),
        # and so is the header's precondition that frames do not overlap (a
        # lane also completes the 64-B sector it shares with the frame before
        # its own, so overlapping frames would race on bytes of both)
        check_batch(arena, offs, lens, stream=stream)
        check_disjoint(offs, lens, stream)
        n = offs.numel()
        if n != len(self.chains):
            raise ValueError(f"{len(self.chains)} chains for {n} frames")
        ops, op_start, data = self.pack()
        d = arena.device
        t_ops = torch.from_numpy(ops.view(np.uint8)).to(d)
        t_start = torch.from_numpy(op_start.view(np.int32)).to(d)
        t_data = torch.from_numpy(data).to(d)
        res = torch.zeros((n, 8), dtype=torch.uint8, device=d)
        s = ctypes.c_void_p(stream) if stream is not None else \
            ctypes.c_void_p(torch.cuda.current_stream(d).cuda_stream)
        rc = _lib.hip().zp_build_batch_device(arena.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                              n, t_ops.data_ptr(), t_start.data_ptr(),
                                              t_data.data_ptr(), res.data_ptr(), s)
        _lib.check(rc, "zp_build_batch_device")
        return res.cpu().numpy().view(RESULT_DTYPE).reshape(-1)
