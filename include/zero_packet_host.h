/*
 * zero_packet_host.h — host-side companion library (libzp_host.so).
 *
 * CPU build of the synthetic batch generator (zero-packet_amd/csrc/zp_gen.h),
 * byte-identical to zp_gen_*_device in libzp_hip.so. It produces test inputs
 * and the host-memory batches of the PCIe-inclusive measurement; it contains
 * no parse code (the parse path is GPU-only, see zero_packet.h).
 */
#ifndef ZERO_PACKET_HOST_H
#define ZERO_PACKET_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Frame length of packet first + i for i in [0, n). */
int zp_host_gen_lengths(int config, uint64_t seed, uint64_t first, uint64_t n,
                        uint32_t* lens);
/* Writes frame first + i at arena + offs[i]; nthreads <= 0 uses all cores. */
int zp_host_gen_frames(int config, uint64_t seed, uint64_t first, uint64_t n,
                       uint8_t* arena, const uint64_t* offs, int nthreads);

#ifdef __cplusplus
}
#endif

#endif /* ZERO_PACKET_HOST_H */
