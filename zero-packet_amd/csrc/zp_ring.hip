// zp_ring.hip — host-ring ingestion pipeline.
//
// Frames start in host memory: a NIC ring or raw-socket buffer
// (README.md:85-115 of the reference, whose loop calls PacketParser::parse
// once per received frame, parser.rs:53). A zp_ring is a fixed set of slots,
// each with pinned host buffers (arena + descriptors + records) mirrored by
// device buffers and its own HIP stream. The producer fills a slot in place
// (a NIC would DMA straight into the pinned arena), submits it, and the slot
// runs H2D copy -> zp_parse_kernel -> D2H copy of the records on its stream
// while the producer fills the next one. With k slots in flight, slot i's
// H2D copy overlaps slot i-1's parse and slot i-2's D2H copy, so the ring is
// bound by the host link, not by the kernel.
//
// Slot life cycle (FIFO, completion in submission order):
//     FREE --acquire--> FILLING --submit--> IN_FLIGHT --wait--> DONE
//     DONE --release--> FREE
// acquire / wait block on a condition variable / the slot's HIP event, up to
// a timeout; the ring is safe for one producer and one consumer thread.

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/zero_packet.h"

extern "C" char* zp__errbuf(void);
#define RING_ERR(...) snprintf(zp__errbuf(), 256, __VA_ARGS__)

enum { S_FREE = 0, S_FILLING, S_IN_FLIGHT, S_DONE };

struct RingSlot {
    int state;
    uint64_t n, bytes, seq;
    hipStream_t s;
    hipEvent_t done;
    uint8_t* h_arena;
    uint64_t* h_offs;
    uint32_t* h_lens;
    zp_record* h_rec;
    zp_ext_offsets* h_ext;
    uint8_t* d_arena;
    uint64_t* d_offs;
    uint32_t* d_lens;
    zp_record* d_rec;
    zp_ext_offsets* d_ext;
};

struct zp_ring {
    int device;
    uint32_t nslots;
    uint64_t slot_bytes, slot_frames;
    uint64_t next_seq;
    uint32_t fill_head;     // next slot to hand to the producer (slots cycle in order)
    uint32_t done_head;     // oldest submitted slot not yet returned to the consumer
    pthread_mutex_t mu;
    pthread_cond_t cv;
    RingSlot* slot;
};

// Absolute CLOCK_REALTIME deadline `ms` from now (for pthread_cond_timedwait).
static timespec deadline_in(int64_t ms) {
    timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    t.tv_sec += ms / 1000;
    t.tv_nsec += (long)(ms % 1000) * 1000000L;
    if (t.tv_nsec >= 1000000000L) { t.tv_sec += 1; t.tv_nsec -= 1000000000L; }
    return t;
}

static int64_t now_ms() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (int64_t)t.tv_sec * 1000 + t.tv_nsec / 1000000;
}

static void fill_view(const zp_ring* r, uint32_t k, zp_ring_slot* out) {
    const RingSlot& s = r->slot[k];
    out->id = (int32_t)k;
    out->arena = s.h_arena;
    out->offs = s.h_offs;
    out->lens = s.h_lens;
    out->arena_cap = r->slot_bytes;
    out->frames_cap = r->slot_frames;
    out->records = s.h_rec;
    out->ext = s.h_ext;
    out->n = s.n;
    out->seq = s.seq;
}

extern "C" void zp_ring_destroy(zp_ring* r) {
    if (!r) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(r->device);
    for (uint32_t k = 0; r->slot && k < r->nslots; ++k) {
        RingSlot& s = r->slot[k];
        if (s.s) (void)hipStreamSynchronize(s.s);
        (void)hipHostFree(s.h_arena); (void)hipHostFree(s.h_offs); (void)hipHostFree(s.h_lens);
        (void)hipHostFree(s.h_rec); (void)hipHostFree(s.h_ext);
        (void)hipFree(s.d_arena); (void)hipFree(s.d_offs); (void)hipFree(s.d_lens);
        (void)hipFree(s.d_rec); (void)hipFree(s.d_ext);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.s) (void)hipStreamDestroy(s.s);
    }
    (void)hipSetDevice(prev);
    pthread_mutex_destroy(&r->mu);
    pthread_cond_destroy(&r->cv);
    free(r->slot);
    free(r);
}

#define RTRY(x)                                                                   \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            RING_ERR("%s: %s", #x, hipGetErrorString(e_));                        \
            goto fail;                                                            \
        }                                                                         \
    } while (0)

extern "C" zp_ring* zp_ring_create(int device, uint32_t nslots, uint64_t slot_bytes,
                                   uint64_t slot_frames) {
    if (nslots < 1 || nslots > 64 || slot_bytes < 64 || slot_frames < 1) {
        RING_ERR("zp_ring_create: bad geometry (slots %u, bytes %llu, frames %llu)", nslots,
                 (unsigned long long)slot_bytes, (unsigned long long)slot_frames);
        return NULL;
    }
    zp_ring* r = (zp_ring*)calloc(1, sizeof(zp_ring));
    if (!r) return NULL;
    r->slot = (RingSlot*)calloc(nslots, sizeof(RingSlot));
    pthread_mutex_init(&r->mu, NULL);
    pthread_cond_init(&r->cv, NULL);
    r->device = device;
    r->nslots = nslots;
    r->slot_bytes = slot_bytes;
    r->slot_frames = slot_frames;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (!r->slot) goto fail;
    RTRY(hipSetDevice(device));
    for (uint32_t k = 0; k < nslots; ++k) {
        RingSlot& s = r->slot[k];
        RTRY(hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking));
        RTRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        // +64: the parse kernel reads whole 16-B chunks around frame edges
        RTRY(hipHostMalloc(&s.h_arena, slot_bytes + 64, hipHostMallocDefault));
        RTRY(hipHostMalloc(&s.h_offs, slot_frames * sizeof(uint64_t), hipHostMallocDefault));
        RTRY(hipHostMalloc(&s.h_lens, slot_frames * sizeof(uint32_t), hipHostMallocDefault));
        RTRY(hipHostMalloc(&s.h_rec, slot_frames * sizeof(zp_record), hipHostMallocDefault));
        RTRY(hipHostMalloc(&s.h_ext, 2 * slot_frames * sizeof(zp_ext_offsets), hipHostMallocDefault));
        RTRY(hipMalloc(&s.d_arena, slot_bytes + 64));
        RTRY(hipMalloc(&s.d_offs, slot_frames * sizeof(uint64_t)));
        RTRY(hipMalloc(&s.d_lens, slot_frames * sizeof(uint32_t)));
        RTRY(hipMalloc(&s.d_rec, slot_frames * sizeof(zp_record)));
        RTRY(hipMalloc(&s.d_ext, 2 * slot_frames * sizeof(zp_ext_offsets)));
    }
    (void)hipSetDevice(prev);
    return r;
fail:
    (void)hipSetDevice(prev);
    zp_ring_destroy(r);
    return NULL;
}

extern "C" int zp_ring_acquire(zp_ring* r, zp_ring_slot* out, int64_t timeout_ms) {
    if (!r || !out) return -1;
    const timespec dl = deadline_in(timeout_ms > 0 ? timeout_ms : 0);
    pthread_mutex_lock(&r->mu);
    const uint32_t k = r->fill_head;
    while (r->slot[k].state != S_FREE) {
        if (timeout_ms < 0) {
            pthread_cond_wait(&r->cv, &r->mu);
        } else if (timeout_ms == 0 || pthread_cond_timedwait(&r->cv, &r->mu, &dl) != 0) {
            pthread_mutex_unlock(&r->mu);
            RING_ERR("zp_ring_acquire: timed out (slot %u not released)", k);
            return ZP_RING_TIMEOUT;
        }
    }
    r->slot[k].state = S_FILLING;
    r->slot[k].n = 0;
    r->fill_head = (k + 1) % r->nslots;
    fill_view(r, k, out);
    pthread_mutex_unlock(&r->mu);
    return 0;
}

extern "C" int zp_ring_submit(zp_ring* r, int32_t id, uint64_t n) {
    if (!r || id < 0 || (uint32_t)id >= r->nslots) return -1;
    RingSlot& s = r->slot[id];
    if (s.state != S_FILLING) {
        RING_ERR("zp_ring_submit: slot %d was not acquired", id);
        return -1;
    }
    if (n > r->slot_frames) {
        RING_ERR("zp_ring_submit: %llu frames exceed the slot capacity %llu",
                 (unsigned long long)n, (unsigned long long)r->slot_frames);
        return -1;
    }
    // Bytes to move: up to the furthest frame end. A frame outside the slot
    // arena is refused here (the device copy holds only slot_bytes).
    uint64_t end = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t e = s.h_offs[i] + s.h_lens[i];
        if (e > r->slot_bytes || e < s.h_offs[i]) {
            RING_ERR("zp_ring_submit: frame %llu lies outside the slot arena",
                     (unsigned long long)i);
            return -1;
        }
        end = e > end ? e : end;
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(r->device) != hipSuccess) return -2;
    hipError_t e = hipSuccess;
    int rc = 0;
    if (n) {
        e = hipMemcpyAsync(s.d_arena, s.h_arena, end, hipMemcpyHostToDevice, s.s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(s.d_offs, s.h_offs, n * sizeof(uint64_t), hipMemcpyHostToDevice, s.s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(s.d_lens, s.h_lens, n * sizeof(uint32_t), hipMemcpyHostToDevice, s.s);
        if (e == hipSuccess)
            rc = zp_parse_batch_device(s.d_arena, s.d_offs, s.d_lens, n, s.d_rec, s.d_ext, s.s);
        if (e == hipSuccess && rc == 0)
            e = hipMemcpyAsync(s.h_rec, s.d_rec, n * sizeof(zp_record), hipMemcpyDeviceToHost, s.s);
        if (e == hipSuccess && rc == 0)
            e = hipMemcpyAsync(s.h_ext, s.d_ext, 2 * n * sizeof(zp_ext_offsets),
                               hipMemcpyDeviceToHost, s.s);
    }
    if (e == hipSuccess && rc == 0) e = hipEventRecord(s.done, s.s);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) {
        RING_ERR("zp_ring_submit: %s", hipGetErrorString(e));
        return -2;
    }
    if (rc) return rc;
    pthread_mutex_lock(&r->mu);
    s.n = n;
    s.bytes = end;
    s.seq = r->next_seq++;
    s.state = S_IN_FLIGHT;
    pthread_cond_broadcast(&r->cv);
    pthread_mutex_unlock(&r->mu);
    return 0;
}

// Hands the oldest in-flight slot to the consumer once its results are in
// host memory. timeout_ms < 0 blocks; 0 only checks.
extern "C" int zp_ring_wait(zp_ring* r, zp_ring_slot* out, int64_t timeout_ms) {
    if (!r || !out) return -1;
    const int64_t t_end = now_ms() + (timeout_ms > 0 ? timeout_ms : 0);
    const timespec dl = deadline_in(timeout_ms > 0 ? timeout_ms : 0);
    pthread_mutex_lock(&r->mu);
    const uint32_t k = r->done_head;
    while (r->slot[k].state != S_IN_FLIGHT) {
        if (timeout_ms < 0) {
            pthread_cond_wait(&r->cv, &r->mu);
        } else if (timeout_ms == 0 || pthread_cond_timedwait(&r->cv, &r->mu, &dl) != 0) {
            pthread_mutex_unlock(&r->mu);
            RING_ERR("zp_ring_wait: timed out (nothing submitted)");
            return ZP_RING_TIMEOUT;
        }
    }
    pthread_mutex_unlock(&r->mu);
    RingSlot& s = r->slot[k];
    hipError_t e;
    if (timeout_ms < 0) {
        e = hipEventSynchronize(s.done);
    } else {
        while ((e = hipEventQuery(s.done)) == hipErrorNotReady) {
            if (now_ms() >= t_end) {
                RING_ERR("zp_ring_wait: timed out (slot %u still in flight)", k);
                return ZP_RING_TIMEOUT;
            }
            usleep(20);
        }
    }
    if (e != hipSuccess) {
        RING_ERR("zp_ring_wait: %s", hipGetErrorString(e));
        return -2;
    }
    // inline outer chains (ABI v6) get their entry rebuilt, so every entry a
    // record flags is valid for the consumer
    for (uint64_t i = 0; i < s.n; ++i)
        if (zp_rec_chain_inline(s.h_rec[i])) zp_rec_chain(s.h_rec[i], &s.h_ext[i]);
    pthread_mutex_lock(&r->mu);
    s.state = S_DONE;
    r->done_head = (k + 1) % r->nslots;
    fill_view(r, k, out);
    pthread_mutex_unlock(&r->mu);
    return 0;
}

extern "C" int zp_ring_release(zp_ring* r, int32_t id) {
    if (!r || id < 0 || (uint32_t)id >= r->nslots) return -1;
    pthread_mutex_lock(&r->mu);
    RingSlot& s = r->slot[id];
    if (s.state != S_DONE) {
        pthread_mutex_unlock(&r->mu);
        RING_ERR("zp_ring_release: slot %d is not held by the consumer", id);
        return -1;
    }
    s.state = S_FREE;
    pthread_cond_broadcast(&r->cv);
    pthread_mutex_unlock(&r->mu);
    return 0;
}
