"""zero-packet_amd — MI355X-native batched PacketParser::parse.

Import with importlib (the directory name has a hyphen):
    zp = importlib.import_module("zero-packet_amd")

  zp.batch.parse_batch(arena, offs, lens)   device-resident batch parse (HIP)
  zp.batch.generate(cfg, n)                  synthetic BASELINE configs on the GPU
  zp.columns.extract(arena, offs, lens, recs) reader getters as SoA device columns
  zp.stats.count(recs)                       per-protocol / per-error counters (device)
  zp.ring.Ring(device, slots, slot_bytes)    host-ring ingestion (H2D/parse/D2H in flight)
  zp.builder.Chain / BuildBatch              batched PacketBuilder chains on the GPU
  zp.PacketParser.parse(frame)               one frame through the GPU path
  zp.PacketParser.from_record(frame, rec)    reference-shaped views over a record
  zp.TcpReader.new(slice) ...                the readers' checked constructors (host)
  zp.internet_checksum / pseudo_header       checksum.rs primitives (host)
"""
from . import _lib, debugfmt, records, ring, shard  # noqa: F401
from .parser import (ArpReader, AuthenticationHeaderReader, EthernetReader,  # noqa: F401
                     ExtensionHeaders, FragmentHeaderReader, Icmpv4Reader, Icmpv6Reader,
                     IpInIp, IPv4Reader, IPv6Reader, OptionsHeaderReader, PacketParser,
                     RoutingHeaderReader, TcpReader, UdpReader, ZeroPacketError,
                     internet_checksum, pseudo_header, verify_internet_checksum)

try:  # torch-dependent batch API
    from . import batch, builder, columns, stats  # noqa: F401
except ImportError:  # pragma: no cover
    batch = builder = columns = stats = None

__all__ = ["PacketParser", "ZeroPacketError", "batch", "records"]
