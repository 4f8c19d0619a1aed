/*
 * zp_host.c — libzp_host.so: CPU build of the synthetic generator
 * (zp_gen.h). Same bytes as zp_gen.hip; used for CPU-side test inputs and
 * host-resident batches (PCIe-inclusive path). Not a parse path.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>

#include "../../include/zero_packet_host.h"
#include "zp_gen.h"

int zp_host_gen_lengths(int config, uint64_t seed, uint64_t first, uint64_t n,
                        uint32_t* lens) {
    if (config < 1 || config > 6) return -1;
    for (uint64_t i = 0; i < n; ++i) {
        zp_plan p;
        zp_plan_packet(config, seed, first + i, &p);
        lens[i] = p.len;
    }
    return 0;
}

static void gen_one(int config, uint64_t seed, uint64_t idx, uint8_t* f) {
    zp_plan p;
    zp_plan_packet(config, seed, idx, &p);
    zp_plan_ip_csums(&p);
    p.csum_l4 = zp_plan_l4_csum(&p, zp_gen_sum(&p, p.l4_off, p.len));
    uint32_t x = 0;
    for (; x < p.pay_off && x < p.len; ++x) f[x] = zp_gen_byte(&p, x);
    for (uint32_t q = 0; x < p.len; q += 8) {
        uint64_t w = zp_h(p.key, ZP_S_PAY + 64u * (uint64_t)(q >> 3));
        for (int j = 0; j < 8 && x < p.len; ++j, ++x) f[x] = (uint8_t)(w >> (8 * j));
    }
}

typedef struct {
    int config;
    uint64_t seed, first, lo, hi;
    uint8_t* arena;
    const uint64_t* offs;
} job_t;

static void* worker(void* a) {
    job_t* j = (job_t*)a;
    for (uint64_t i = j->lo; i < j->hi; ++i)
        gen_one(j->config, j->seed, j->first + i, j->arena + j->offs[i]);
    return 0;
}

int zp_host_gen_frames(int config, uint64_t seed, uint64_t first, uint64_t n,
                       uint8_t* arena, const uint64_t* offs, int nthreads) {
    if (config < 1 || config > 6) return -1;
    if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nthreads > 64) nthreads = 64;
    if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
    pthread_t th[64];
    job_t jobs[64];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (job_t){config, seed, first, n * t / nthreads, n * (t + 1) / nthreads, arena, offs};
        if (pthread_create(&th[t], 0, worker, &jobs[t])) { worker(&jobs[t]); th[t] = 0; }
    }
    for (int t = 0; t < nthreads; ++t) if (th[t]) pthread_join(th[t], 0);
    return 0;
}
