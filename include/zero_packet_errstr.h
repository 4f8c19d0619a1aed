/*
 * zero_packet_errstr.h — exact reference error strings for each zp_err code.
 * Each string is the `&'static str` the reference returns (file:line given
 * in include/zero_packet.h next to the code).
 */
#ifndef ZERO_PACKET_ERRSTR_H
#define ZERO_PACKET_ERRSTR_H

#include "zero_packet.h"

static const char* const zp_err_strings[ZP_ERR_COUNT] = {
    "",
    "Slice needs to be least 64 bytes long to be a valid Ethernet frame.",
    "Slice is too short to contain an Ethernet frame.",
    "Slice is too short to contain VLAN tagging.",
    "Slice is too short to contain double VLAN tagging.",
    "Invalid double VLAN tag.",
    "Slice is too short to contain an ARP header.",
    "ARP operation field is invalid, expected request (1) or reply (2).",
    "Slice is too short to contain an IPv4 header.",
    "IPv4 version field is invalid. Expected version 4.",
    "IPv4 IHL field is invalid. Indicated header length is too short.",
    "IPv4 header length is invalid. Indicated header length is too long.",
    "IPv4 total length field is invalid. Does not match actual length.",
    "IPv4 checksum is invalid.",
    "Indicated IPv4 header length exceeds the allocated buffer.",
    "Slice is too short to contain an IPv6 header.",
    "IPv6 version field is invalid. Expected version 6.",
    "If Hop-by-Hop Options is present, then it must be the first extension header.",
    "Slice is too short to contain an Options extension header.",
    "Indicated IPv6 options header length exceeds the allocated buffer.",
    "Slice is too short to contain a Routing extension header.",
    "Indicated IPv6 routing header length exceeds the allocated buffer.",
    "Slice is too short to contain a Fragment header.",
    "Slice is too short to contain an Authentication extension header.",
    "Indicated Authentication header length exceeds the allocated buffer.",
    "Slice is too short to contain a TCP header.",
    "TCP data offset field is invalid. Indicated header length is too short.",
    "TCP flags field is invalid.",
    "Slice is too short to contain a UDP header.",
    "UDP length field is invalid. Does not match actual length.",
    "Slice is too short to contain an ICMP header.",
    "ICMPv4 type field is invalid.",
    "ICMPv4 code field is invalid.",
    "ICMPv6 type field is invalid.",
    "IPv4 encapsulated checksum is invalid.",
    "IPv6 encapsulated checksum is invalid.",
    "Indicated TCP header length exceeds the allocated buffer.",
    "Indicated header length exceeds the allocated buffer.",
};

static inline const char* zp_err_string(int code) {
    if (code < 0 || code >= ZP_ERR_COUNT) return 0;
    return zp_err_strings[code];
}

#endif /* ZERO_PACKET_ERRSTR_H */
