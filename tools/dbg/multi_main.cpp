// Host-side check of zp_parse_batch_host_multi (built with host-only ASan).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../include/zero_packet.h"

int main() {
    const uint64_t n = 20000;
    std::vector<uint32_t> lens(n);
    std::vector<uint64_t> offs(n);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) { lens[i] = 64 + (i * 37) % 1400; offs[i] = pos; pos += lens[i]; }
    std::vector<uint8_t> arena(pos + 64, 0x5a);
    std::vector<zp_record> rec(n);
    std::vector<zp_ext_offsets> ext(2 * n);   // outer chains, then ip_in_ip chains
    zp_ctx* ctx[3];
    for (int d = 0; d < 3; ++d) { ctx[d] = zp_ctx_create(0, 1 << 20); if (!ctx[d]) { printf("ctx fail %s\n", zp_last_error()); return 1; } }
    int rc = zp_parse_batch_host(ctx[0], arena.data(), arena.size(), offs.data(), lens.data(), n, rec.data(), ext.data());
    printf("single rc=%d err0=%d\n", rc, rec[0].err);
    rc = zp_parse_batch_host_multi(ctx, 3, arena.data(), arena.size(), offs.data(), lens.data(), n, rec.data(), ext.data());
    fflush(stdout); printf("multi rc=%d err0=%d %s\n", rc, rec[0].err, rc ? zp_last_error() : "");
    for (int d = 0; d < 3; ++d) zp_ctx_destroy(ctx[d]);
    return 0;
}
