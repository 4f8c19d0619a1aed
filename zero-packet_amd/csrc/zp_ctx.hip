// zp_ctx.hip — host-memory entry points of the C ABI (zero_packet.h):
// zp_ctx_create / zp_ctx_destroy / zp_parse_batch_host / zp_parse_one.
//
// Frames arrive in host memory (a NIC ring / raw socket buffer,
// README.md:85-115 of the reference). The batch is cut into chunks whose byte
// span fits the device staging buffer; two slots on two streams overlap
// chunk k's H2D copy and parse with chunk k-1's D2H copy. Pinned user
// buffers are DMA'd directly; pageable ones are staged through pinned
// memory. The parse itself is the device kernel (zp_parse.hip); there is no
// host-side parse.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <immintrin.h>
#include <pthread.h>
#include <time.h>

#include "../../include/zero_packet.h"

// Thread-local error text shared with zp_parse.hip (read via zp_last_error()).
extern "C" char* zp__errbuf(void);
#define g_ctx_error (zp__errbuf())
#define ERRBUF_LEN 256

#define SLOTS 2

struct zp_ctx {
    int device;
    uint64_t chunk_bytes, chunk_pkts;
    hipStream_t s[SLOTS];
    hipEvent_t ev[SLOTS];
    uint8_t* d_arena[SLOTS];
    uint64_t* d_offs[SLOTS];
    uint32_t* d_lens[SLOTS];
    zp_record* d_rec[SLOTS];
    zp_ext_offsets* d_ext[SLOTS];
    uint8_t* h_arena[SLOTS];      // pinned staging
    uint64_t* h_offs[SLOTS];
    uint32_t* h_lens[SLOTS];
    zp_record* h_rec[SLOTS];
    zp_ext_offsets* h_ext[SLOTS];
    // zp_build_batch_host scratch, allocated on first use and grown as needed
    zp_build_op* d_bops;
    uint64_t bops_cap;
    uint8_t* d_bdata;
    uint64_t bdata_cap;
    uint32_t* d_bstart;
    zp_build_result* d_bres;
    uint32_t* h_bstart;
    // zp_parse_one: one mapped, coherent pinned block (doorbell, descriptors,
    // record, ext entries, frame) the kernel reads and writes in place
    uint8_t* one_h;
    uint8_t* one_d;
    bool one_failed;              // the mapped block could not be allocated: batch path
    // ... served by a wave of the device's shared server (SharedServer below)
    uint32_t one_idle_us;         // 0: one batch launch per call; > 0: the shared server
    uint32_t one_seq;             // last request answered (or retired by a give-up)
    int slot;                     // this context's slot in the device's server (-1: none)
    int64_t one_giveup_ns;        // no answer for this long: the request fails (-2)
};

// zp_parse_one's block: the frame at ONE_FRAME, the doorbell and the batch
// kernel's descriptor in front, the outputs between them (the server's
// offsets are ZP_ONE_* in zp_parse.hip). Frames longer than ONE_MAX take the
// batch path.
#define ONE_BELL 0       // uint64_t: seq << 32 | length (server mode)
#define ONE_OFFS 8       // uint64_t: ONE_FRAME (launch mode)
#define ONE_LENS 16      // uint32_t (launch mode)
#define ONE_REC 64       // zp_record (8 B)
#define ONE_ACK 72       // uint32_t: seq of the last finished request (server mode), written
                         // with the record by one 16-B store ...
#define ONE_TAG 76       // ... and the tag rec.x ^ rec.y ^ seq ^ ONE_TAG_KEY
#define ONE_EXT 96       // zp_ext_offsets[2]
#define ONE_FRAME 128
#define ONE_MAX (64u << 10)
#define ONE_IDLE_US_DEFAULT 5000u     // zp_parse_one_config's default (> 0: the server)
#define ONE_LIFE_US_DEFAULT 1000u     // a server kernel leaves after this long resident
#define ONE_LIFE_MARGIN_NS 100000     // the host replaces it this long before its life ends
#define ONE_GIVEUP_NS 10000000000ll   // 10 s without an answer: the request fails
#define ONE_TAG_KEY 0x9E3779B9u       // ZP_ONE_TAG (zp_parse.hip)

static_assert(ONE_FRAME + ONE_MAX + 64 == 128u + (64u << 10) + 64u,
              "the server's buffer range (ZP_SYS_BYTES, zp_stream.h) is the mapped block");

extern "C" int zp__one_server_launch(const uint8_t* ctl_d, uint32_t nslots, uint64_t life_ticks,
                                     uint32_t gen, void* stream);
extern "C" int zp__one_stall_launch(uint64_t ticks, void* stream);

static int64_t mono_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec;
}

// Grows a device buffer to at least `need` elements (contents not kept).
template <typename T>
static hipError_t grow(T** p, uint64_t* cap, uint64_t need) {
    if (*p && *cap >= need) return hipSuccess;
    (void)hipFree(*p);
    *p = NULL;
    *cap = 0;
    const uint64_t n = need < 64 ? 64 : need + need / 4;
    const hipError_t e = hipMalloc((void**)p, n * sizeof(T));
    if (e == hipSuccess) *cap = n;
    return e;
}

#define TRY(x)                                                                     \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            snprintf(g_ctx_error, ERRBUF_LEN, "%s: %s", #x,                \
                     hipGetErrorString(e_));                                       \
            fprintf(stderr, "zero-packet: %s\n", g_ctx_error);                     \
            goto fail;                                                             \
        }                                                                          \
    } while (0)

// --------------------------------------------------------------------------
// The device's shared zp_parse_one server. One kernel per device (process
// wide) serves every context of that device: wave w of its grid polls slot
// w's doorbell (the context's mapped block, registered in a table in the
// control block) and answers its requests. One kernel rather than one per
// context: a resident kernel holds its hardware queue, and the process has
// few (GPU_MAX_HW_QUEUES, 4 here), so per-context servers past the fourth
// waited behind the others (profiles/r06_parse_one_latency.log). The kernel
// leaves after `life` (1 ms) whatever the traffic; shortly before, the next
// caller queues a new generation behind it and writes the retire word, so
// the old one leaves at its next poll and the new one starts from each
// slot's acknowledgement word (nothing is answered twice). A device-wide
// synchronisation therefore waits for about one life at most.
// --------------------------------------------------------------------------
#define SRV_SLOTS 64                  // contexts per device with a server slot
#define CTL_RETIRE 0                  // uint32_t: kernels of generation <= this leave
#define CTL_TABLE 64                  // uint64_t[SRV_SLOTS]: each slot's block (device VA, 0: none)
#define CTL_BYTES (CTL_TABLE + 8 * SRV_SLOTS)
#define SRV_DEVICES 64

struct SharedServer {
    pthread_mutex_t m;            // launches, rotations, slots (not the request path)
    bool ready, failed;
    hipStream_t stream;
    uint8_t* ctl_h;               // mapped, coherent control block
    uint8_t* ctl_d;
    uint64_t clock_khz;           // the device's constant clock (s_memrealtime)
    uint64_t used;                // slot bitmap
    uint32_t nslots;              // slots in use span [0, nslots)
    uint32_t gen;                 // newest generation launched
    int64_t born_ns;              // atomic: host clock of the newest launch (0: none runs)
    uint32_t life_us;             // atomic (test hook zp__one_test_hooks)
    uint32_t stall_us;            // test hook: a stall kernel before each launch
    uint64_t launches, rotations, relaunches;
};
static SharedServer g_srv[SRV_DEVICES];
static pthread_mutex_t g_srv_init = PTHREAD_MUTEX_INITIALIZER;
static bool g_srv_mutex[SRV_DEVICES];

// The device's server (its stream and control block on first use; the
// caller has set the device). NULL: none (the batch path serves).
static SharedServer* srv_get(int device) {
    if (device < 0 || device >= SRV_DEVICES) return NULL;
    SharedServer* S = &g_srv[device];
    pthread_mutex_lock(&g_srv_init);
    if (!g_srv_mutex[device]) {
        pthread_mutex_init(&S->m, NULL);
        g_srv_mutex[device] = true;
    }
    pthread_mutex_unlock(&g_srv_init);
    pthread_mutex_lock(&S->m);
    if (!S->ready && !S->failed) {
        int khz = 0;
        hipError_t e = hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking);
        if (e == hipSuccess)
            e = hipHostMalloc((void**)&S->ctl_h, CTL_BYTES, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&S->ctl_d, S->ctl_h, 0);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
        if (e == hipSuccess) {
            memset(S->ctl_h, 0, CTL_BYTES);
            S->clock_khz = (uint64_t)(khz > 0 ? khz : 100000);
            __atomic_store_n(&S->life_us, ONE_LIFE_US_DEFAULT, __ATOMIC_RELAXED);
            S->ready = true;
        } else {
            (void)hipGetLastError();
            S->failed = true;                       // the batch path serves (not retried)
        }
    }
    const bool ok = S->ready;
    pthread_mutex_unlock(&S->m);
    return ok ? S : NULL;
}

// True when a server kernel surely still runs: launched less than its life
// ago (host clock; the device counts from a later instant).
static bool srv_sure(SharedServer* S, int64_t now) {
    const int64_t born = __atomic_load_n(&S->born_ns, __ATOMIC_ACQUIRE);
    const int64_t life = (int64_t)__atomic_load_n(&S->life_us, __ATOMIC_RELAXED) * 1000;
    return born != 0 && now - born < life - ONE_LIFE_MARGIN_NS;
}

// Launches generation gen + 1 behind whatever runs on the server stream
// (S->m held).
static int srv_launch_locked(SharedServer* S) {
    const uint64_t life = (uint64_t)__atomic_load_n(&S->life_us, __ATOMIC_RELAXED) * S->clock_khz / 1000u;
    if (S->stall_us) {
        const int rc = zp__one_stall_launch((uint64_t)S->stall_us * S->clock_khz / 1000u, S->stream);
        if (rc) return rc;
    }
    const int rc = zp__one_server_launch(S->ctl_d, S->nslots, life, S->gen + 1u, S->stream);
    if (rc) return rc;
    ++S->gen;
    ++S->launches;
    __atomic_store_n(&S->born_ns, mono_ns(), __ATOMIC_RELEASE);
    return 0;
}

// Replaces the running kernel (if any) by a new generation: the new one is
// queued, then the old one retired (S->m held).
static int srv_rotate_locked(SharedServer* S) {
    const bool live = __atomic_load_n(&S->born_ns, __ATOMIC_ACQUIRE) != 0;
    const int rc = srv_launch_locked(S);
    if (rc) return rc;
    if (live) {
        __atomic_store_n((uint32_t*)(S->ctl_h + CTL_RETIRE), S->gen - 1u, __ATOMIC_RELEASE);
        ++S->rotations;
    }
    return 0;
}

// A server runs that includes every registered slot, or is launched (the
// caller has set the device). Called when srv_sure said no.
static int srv_ensure(SharedServer* S) {
    pthread_mutex_lock(&S->m);
    int rc = 0;
    if (!srv_sure(S, mono_ns())) {                    // another thread may have done it
        if (__atomic_load_n(&S->born_ns, __ATOMIC_ACQUIRE) != 0) {
            const hipError_t q = hipStreamQuery(S->stream);
            if (q == hipSuccess) {
                __atomic_store_n(&S->born_ns, (int64_t)0, __ATOMIC_RELEASE);
            } else if (q != hipErrorNotReady) {
                snprintf(g_ctx_error, ERRBUF_LEN, "zp_parse_one server: %s", hipGetErrorString(q));
                __atomic_store_n(&S->born_ns, (int64_t)0, __ATOMIC_RELEASE);
                rc = -2;
            }
        }
        if (!rc) rc = srv_rotate_locked(S);          // a launch when none runs
    }
    pthread_mutex_unlock(&S->m);
    return rc;
}

// Retires every generation and waits for the server stream (S->m held).
static void srv_stop_locked(SharedServer* S) {
    if (__atomic_load_n(&S->born_ns, __ATOMIC_ACQUIRE) == 0 && hipStreamQuery(S->stream) == hipSuccess)
        return;
    __atomic_store_n((uint32_t*)(S->ctl_h + CTL_RETIRE), S->gen, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(S->stream);
    __atomic_store_n(&S->born_ns, (int64_t)0, __ATOMIC_RELEASE);
}

// The context's slot (registered on first use; a running kernel is replaced
// so that the new slot is served). False: no free slot (the launch mode
// serves this context).
static bool srv_register(SharedServer* S, zp_ctx* c) {
    if (c->slot >= 0) return true;
    pthread_mutex_lock(&S->m);
    int k = 0;
    while (k < SRV_SLOTS && (S->used >> k) & 1u) ++k;
    if (k < SRV_SLOTS) {
        S->used |= 1ull << k;
        if ((uint32_t)k + 1u > S->nslots) S->nslots = (uint32_t)k + 1u;
        __atomic_store_n((uint64_t*)(S->ctl_h + CTL_TABLE + 8 * k), (uint64_t)(uintptr_t)c->one_d,
                         __ATOMIC_RELEASE);
        c->slot = k;
        if (__atomic_load_n(&S->born_ns, __ATOMIC_ACQUIRE) != 0 &&
            hipStreamQuery(S->stream) == hipErrorNotReady)
            (void)srv_rotate_locked(S);
        else
            __atomic_store_n(&S->born_ns, (int64_t)0, __ATOMIC_RELEASE);
    }
    pthread_mutex_unlock(&S->m);
    return c->slot >= 0;
}

// Stops the device's server (every context's next call relaunches it).
static void one_server_stop(zp_ctx* c) {
    if (c->slot < 0) return;
    SharedServer* S = &g_srv[c->device];
    pthread_mutex_lock(&S->m);
    srv_stop_locked(S);
    pthread_mutex_unlock(&S->m);
}

// Takes the context's slot out of the table; the server is stopped first,
// so no wave reads the block afterwards.
static void srv_unregister(zp_ctx* c) {
    if (c->slot < 0) return;
    SharedServer* S = &g_srv[c->device];
    pthread_mutex_lock(&S->m);
    srv_stop_locked(S);
    __atomic_store_n((uint64_t*)(S->ctl_h + CTL_TABLE + 8 * c->slot), (uint64_t)0, __ATOMIC_RELEASE);
    S->used &= ~(1ull << c->slot);
    while (S->nslots && !((S->used >> (S->nslots - 1)) & 1u)) --S->nslots;
    c->slot = -1;
    pthread_mutex_unlock(&S->m);
}

extern "C" void zp_ctx_destroy(zp_ctx* c) {
    if (!c) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(c->device);
    srv_unregister(c);
    for (int k = 0; k < SLOTS; ++k) {
        if (c->s[k]) (void)hipStreamSynchronize(c->s[k]);
        (void)hipFree(c->d_arena[k]); (void)hipFree(c->d_offs[k]); (void)hipFree(c->d_lens[k]);
        (void)hipFree(c->d_rec[k]); (void)hipFree(c->d_ext[k]);
        (void)hipHostFree(c->h_arena[k]); (void)hipHostFree(c->h_offs[k]); (void)hipHostFree(c->h_lens[k]);
        (void)hipHostFree(c->h_rec[k]); (void)hipHostFree(c->h_ext[k]);
        if (c->ev[k]) (void)hipEventDestroy(c->ev[k]);
        if (c->s[k]) (void)hipStreamDestroy(c->s[k]);
    }
    (void)hipFree(c->d_bops); (void)hipFree(c->d_bdata); (void)hipFree(c->d_bstart);
    (void)hipFree(c->d_bres); (void)hipHostFree(c->h_bstart); (void)hipHostFree(c->one_h);
    (void)hipSetDevice(prev);
    free(c);
}

extern "C" zp_ctx* zp_ctx_create(int device, uint64_t chunk_bytes) {
    zp_ctx* c = (zp_ctx*)calloc(1, sizeof(zp_ctx));
    int prev = 0;
    if (!c) return NULL;
    if (chunk_bytes == 0) chunk_bytes = 256ull << 20;
    if (chunk_bytes < 65536) chunk_bytes = 65536;
    c->device = device;
    c->chunk_bytes = chunk_bytes;
    c->one_idle_us = ONE_IDLE_US_DEFAULT;
    c->one_giveup_ns = ONE_GIVEUP_NS;
    c->slot = -1;
    c->chunk_pkts = chunk_bytes / 64 + 1;
    (void)hipGetDevice(&prev);
    TRY(hipSetDevice(device));
    for (int k = 0; k < SLOTS; ++k) {
        TRY(hipStreamCreateWithFlags(&c->s[k], hipStreamNonBlocking));
        TRY(hipEventCreateWithFlags(&c->ev[k], hipEventDisableTiming));
        TRY(hipMalloc(&c->d_arena[k], chunk_bytes + 64));
        TRY(hipMalloc(&c->d_offs[k], c->chunk_pkts * sizeof(uint64_t)));
        TRY(hipMalloc(&c->d_lens[k], c->chunk_pkts * sizeof(uint32_t)));
        TRY(hipMalloc(&c->d_rec[k], c->chunk_pkts * sizeof(zp_record)));
        TRY(hipMalloc(&c->d_ext[k], 2 * c->chunk_pkts * sizeof(zp_ext_offsets)));
        TRY(hipHostMalloc(&c->h_arena[k], chunk_bytes + 64, hipHostMallocDefault));
        TRY(hipHostMalloc(&c->h_offs[k], c->chunk_pkts * sizeof(uint64_t), hipHostMallocDefault));
        TRY(hipHostMalloc(&c->h_lens[k], c->chunk_pkts * sizeof(uint32_t), hipHostMallocDefault));
        TRY(hipHostMalloc(&c->h_rec[k], c->chunk_pkts * sizeof(zp_record), hipHostMallocDefault));
        TRY(hipHostMalloc(&c->h_ext[k], 2 * c->chunk_pkts * sizeof(zp_ext_offsets), hipHostMallocDefault));
    }
    (void)hipSetDevice(prev);
    return c;
fail:
    (void)hipSetDevice(prev);
    zp_ctx_destroy(c);
    return NULL;
}

static bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) { (void)hipGetLastError(); return false; }
    return a.type == hipMemoryTypeHost;
}

struct Pending { uint64_t i, j; bool live; };

// Copies a finished slot's results to the user arrays: the outer and the
// ip_in_ip chains go to xo[i] / xi[i] (the two halves of the caller's 2n-entry
// ext array); the slot's device buffer holds the chunk's m frames as one
// 2m-entry ext array ([0, m) outer, [m, 2m) ip_in_ip).
static int drain(zp_ctx* c, int k, Pending& pd, zp_record* recs, zp_ext_offsets* xo,
                 zp_ext_offsets* xi, bool rec_direct) {
    if (!pd.live) return 0;
    hipError_t e = hipEventSynchronize(c->ev[k]);
    if (e != hipSuccess) {
        snprintf(g_ctx_error, ERRBUF_LEN, "hipEventSynchronize: %s", hipGetErrorString(e));
        return -2;
    }
    uint64_t m = pd.j - pd.i;
    if (!rec_direct) memcpy(recs + pd.i, c->h_rec[k], m * sizeof(zp_record));
    if (xo) {
        for (uint64_t q = 0; q < m; ++q) {
            const zp_record r = recs[pd.i + q];
            if (zp_rec_chain_inline(r)) zp_rec_chain(r, &xo[pd.i + q]);   // ABI v6
            else if (r.flags & ZP_F_EXT) xo[pd.i + q] = c->h_ext[k][q];
            if (r.flags & ZP_F_INNER_EXT) xi[pd.i + q] = c->h_ext[k][m + q];
        }
    }
    pd.live = false;
    return 0;
}

extern "C" int zp_parse_batch_device(const uint8_t*, const uint64_t*, const uint32_t*, uint64_t,
                                     zp_record*, zp_ext_offsets*, void*);

// The host path over frames [0, n) with the chains going to xo / xi (both
// NULL: chains dropped).
static int parse_host(zp_ctx* c, const uint8_t* arena, uint64_t arena_bytes,
                      const uint64_t* offs, const uint32_t* lens, uint64_t n,
                      zp_record* recs, zp_ext_offsets* xo, zp_ext_offsets* xi) {
    zp_ext_offsets* ext = xo;
    if (!c || (n && (!arena || !offs || !lens || !recs))) return -1;
    if (n == 0) return 0;
    int prev = 0;
    int rc = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(c->device) != hipSuccess) return -2;
    const bool arena_direct = is_pinned(arena);
    const bool rec_direct = is_pinned(recs);
    Pending pd[SLOTS] = {{0, 0, false}, {0, 0, false}};
    uint64_t i = 0;
    int k = 0;
    while (i < n) {
        // Chunk [i, j) with byte span [lo, hi) <= chunk_bytes.
        uint64_t lo = offs[i], hi = offs[i] + lens[i];
        if (hi - lo > c->chunk_bytes) {
            snprintf(g_ctx_error, ERRBUF_LEN,
                     "frame %llu (%u B) exceeds the context chunk size",
                     (unsigned long long)i, lens[i]);
            rc = -3;
            break;
        }
        if (arena_bytes && hi > arena_bytes) {
            snprintf(g_ctx_error, ERRBUF_LEN, "frame %llu lies outside the arena",
                     (unsigned long long)i);
            rc = -1;
            break;
        }
        uint64_t j = i + 1;
        while (j < n && j - i < c->chunk_pkts) {
            uint64_t l2 = offs[j] < lo ? offs[j] : lo;
            uint64_t h2 = offs[j] + lens[j] > hi ? offs[j] + lens[j] : hi;
            if (h2 - l2 > c->chunk_bytes || (arena_bytes && h2 > arena_bytes)) break;
            lo = l2; hi = h2; ++j;
        }
        if ((rc = drain(c, k, pd[k], recs, xo, xi, rec_direct)) != 0) break;
        uint64_t m = j - i;
        for (uint64_t q = 0; q < m; ++q) {
            c->h_offs[k][q] = offs[i + q] - lo;
            c->h_lens[k][q] = lens[i + q];
        }
        const uint8_t* src = arena + lo;
        if (!arena_direct) { memcpy(c->h_arena[k], src, hi - lo); src = c->h_arena[k]; }
        hipStream_t s = c->s[k];
        hipError_t e = hipMemcpyAsync(c->d_arena[k], src, hi - lo, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->d_offs[k], c->h_offs[k], m * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->d_lens[k], c->h_lens[k], m * 4, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) {
            snprintf(g_ctx_error, ERRBUF_LEN, "H2D copy: %s", hipGetErrorString(e));
            rc = -2;
            break;
        }
        rc = zp_parse_batch_device(c->d_arena[k], c->d_offs[k], c->d_lens[k], m, c->d_rec[k],
                                   ext ? c->d_ext[k] : NULL, s);
        if (rc) break;
        e = hipMemcpyAsync(rec_direct ? (void*)(recs + i) : (void*)c->h_rec[k], c->d_rec[k],
                           m * sizeof(zp_record), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && ext)
            e = hipMemcpyAsync(c->h_ext[k], c->d_ext[k], 2 * m * sizeof(zp_ext_offsets),
                               hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipEventRecord(c->ev[k], s);
        if (e != hipSuccess) {
            snprintf(g_ctx_error, ERRBUF_LEN, "D2H copy / event: %s", hipGetErrorString(e));
            rc = -2;
            break;
        }
        pd[k] = Pending{i, j, true};
        i = j;
        k = (k + 1) % SLOTS;
    }
    for (int q = 0; q < SLOTS; ++q) {
        int r2 = drain(c, (k + q) % SLOTS, pd[(k + q) % SLOTS], recs, xo, xi, rec_direct);
        if (!rc) rc = r2;
    }
    (void)hipSetDevice(prev);
    return rc;
}

extern "C" int zp_parse_batch_host(zp_ctx* c, const uint8_t* arena, uint64_t arena_bytes,
                                   const uint64_t* offs, const uint32_t* lens, uint64_t n,
                                   zp_record* recs, zp_ext_offsets* ext) {
    return parse_host(c, arena, arena_bytes, offs, lens, n, recs, ext, ext ? ext + n : NULL);
}

// The mapped block of zp_parse_one (allocated on first use). False: none.
static bool one_block(zp_ctx* c) {
    if (!c->one_h && !c->one_failed) {
        hipError_t a = hipHostMalloc((void**)&c->one_h, ONE_FRAME + ONE_MAX + 64,
                                     hipHostMallocMapped | hipHostMallocCoherent);
        if (a == hipSuccess) a = hipHostGetDevicePointer((void**)&c->one_d, c->one_h, 0);
        if (a != hipSuccess) {                      // no mapped block: the batch path
            (void)hipGetLastError();
            (void)hipHostFree(c->one_h);
            c->one_h = c->one_d = NULL;
            c->one_failed = true;                   // not retried on every call
        } else {
            memset(c->one_h, 0, ONE_FRAME);
        }
    }
    return c->one_h != NULL;
}

// One request through the device's server: doorbell, then spin on the
// acknowledgement. The answer is the 16-B {record, ack, tag} read as one
// load; an ack whose tag does not match the record read with it is waited
// out (a host-link write seen in pieces). On giving up, the request is
// retired (the acknowledgement word takes its seq) only after the server has
// been stopped, so a late wave never answers it from a frame being
// rewritten. `sure`: a kernel surely runs (else the caller has set the
// device and one is ensured first).
static int one_via_server(zp_ctx* c, SharedServer* S, uint32_t len, zp_record* out, bool sure) {
    if (!sure) {
        const int rc = srv_ensure(S);
        if (rc) return rc;
    }
    const uint32_t seq = c->one_seq + 1u;
    const volatile __m128i* ans = (const volatile __m128i*)(c->one_h + ONE_REC);
    __atomic_store_n((uint64_t*)(c->one_h + ONE_BELL), ((uint64_t)seq << 32) | len,
                     __ATOMIC_RELEASE);
    const int64_t t0 = mono_ns();
    int64_t next_check = t0 + 200000;                        // 200 us
    uint32_t w[4];
    for (uint32_t spin = 1;; ++spin) {
        const __m128i v = _mm_load_si128((const __m128i*)ans);
        _mm_storeu_si128((__m128i*)w, v);
        if (w[2] == seq && w[3] == (w[0] ^ w[1] ^ seq ^ ONE_TAG_KEY)) break;
        _mm_pause();
        if ((spin & 1023u) == 0) {
            const int64_t now = mono_ns();
            if (now < next_check) continue;
            // The kernel may have left before the doorbell (its life, or
            // quiesced by another thread): then its stream is done and the
            // request still open.
            const hipError_t q = hipStreamQuery(S->stream);
            if (q == hipSuccess) {
                int prev = 0;
                (void)hipGetDevice(&prev);
                (void)hipSetDevice(c->device);
                pthread_mutex_lock(&S->m);
                int rc = 0;
                if (hipStreamQuery(S->stream) == hipSuccess) {
                    __atomic_store_n(&S->born_ns, (int64_t)0, __ATOMIC_RELEASE);
                    rc = srv_launch_locked(S);
                    ++S->relaunches;
                }
                pthread_mutex_unlock(&S->m);
                (void)hipSetDevice(prev);
                if (rc) return rc;
            } else if (q != hipErrorNotReady) {
                snprintf(g_ctx_error, ERRBUF_LEN, "zp_parse_one server: %s", hipGetErrorString(q));
                __atomic_store_n(&S->born_ns, (int64_t)0, __ATOMIC_RELEASE);
                return -2;
            }
            if (now - t0 > c->one_giveup_ns) {
                int prev = 0;
                (void)hipGetDevice(&prev);
                (void)hipSetDevice(c->device);
                one_server_stop(c);                         // no wave runs after this
                c->one_seq = seq;                           // retired: never answered later
                __atomic_store_n((uint32_t*)(c->one_h + ONE_ACK), seq, __ATOMIC_RELEASE);
                (void)hipSetDevice(prev);
                snprintf(g_ctx_error, ERRBUF_LEN, "zp_parse_one: no answer from the server");
                return -2;
            }
            next_check = now + 200000;
        }
    }
    c->one_seq = seq;
    memcpy(out, w, sizeof(zp_record));
    return 0;
}

// One frame, latency first: the frame is copied into the context's mapped
// pinned block, where the GPU reads it and writes the record and chains
// back over the host link. By default a resident server wave does the parse
// (no launch per call); with zp_parse_one_config(ctx, 0) each call launches
// the batch kernel on the block and waits on the stream. Frames past ONE_MAX
// take the chunked batch path.
extern "C" int zp_parse_one(zp_ctx* c, const uint8_t* frame, uint64_t len,
                            zp_record* record, zp_ext_offsets* ext) {
    if (!c || !record || len > 0xFFFFFFFFull || (!frame && len)) return -1;
    int rc;
    uint8_t* h = c->one_h;
    SharedServer* S = c->slot >= 0 ? &g_srv[c->device] : NULL;
    if (S && len <= ONE_MAX && c->one_idle_us && srv_sure(S, mono_ns())) {
        // The fast path: a server kernel surely runs, so no HIP call at all:
        // copy, doorbell, spin.
        if (len) memcpy(h + ONE_FRAME, frame, len);
        rc = one_via_server(c, S, (uint32_t)len, record, true);
    } else {
        int prev = 0;
        (void)hipGetDevice(&prev);
        if (hipSetDevice(c->device) != hipSuccess) return -2;
        if (len > ONE_MAX || !one_block(c)) {
            (void)hipSetDevice(prev);
            uint64_t off = 0;
            uint32_t l = (uint32_t)len;
            static const uint8_t empty[16] = {0};
            if (ext) memset(ext, 0, 2 * sizeof(zp_ext_offsets));   // unflagged entries: zero
            const int r2 = zp_parse_batch_host(c, frame ? frame : empty, len, &off, &l, 1, record, ext);
            return r2 ? r2 : (int)zp_rec_err(*record);
        }
        h = c->one_h;
        if (len) memcpy(h + ONE_FRAME, frame, len);
        if (c->one_idle_us && !S) {
            S = srv_get(c->device);
            if (S && !srv_register(S, c)) S = NULL;
        }
        if (c->one_idle_us && S) {
            rc = one_via_server(c, S, (uint32_t)len, record, false);
        } else {
            const uint64_t at = ONE_FRAME;
            const uint32_t l = (uint32_t)len;
            memcpy(h + ONE_OFFS, &at, 8);
            memcpy(h + ONE_LENS, &l, 4);
            rc = zp_parse_batch_device(c->one_d, (const uint64_t*)(c->one_d + ONE_OFFS),
                                       (const uint32_t*)(c->one_d + ONE_LENS), 1,
                                       (zp_record*)(c->one_d + ONE_REC),
                                       (zp_ext_offsets*)(c->one_d + ONE_EXT), c->s[0]);
            if (!rc) {
                const hipError_t e = hipStreamSynchronize(c->s[0]);
                if (e != hipSuccess) {
                    snprintf(g_ctx_error, ERRBUF_LEN, "zp_parse_one: %s", hipGetErrorString(e));
                    rc = -2;
                }
            }
            if (!rc) memcpy(record, h + ONE_REC, sizeof(zp_record));
        }
        (void)hipSetDevice(prev);
    }
    if (rc) return rc;
    if (ext) {
        // entries are defined only where the record flags them (zero_packet.h)
        const zp_ext_offsets* x = (const zp_ext_offsets*)(h + ONE_EXT);
        memset(ext, 0, 2 * sizeof(zp_ext_offsets));
        if (zp_rec_chain_inline(*record)) zp_rec_chain(*record, &ext[0]);   // ABI v6
        else if (record->flags & ZP_F_EXT) ext[0] = x[0];
        if (record->flags & ZP_F_INNER_EXT) ext[1] = x[1];
    }
    return (int)zp_rec_err(*record);
}


// zp_parse_one's mode: idle_us = 0 launches the batch kernel per call;
// otherwise the device's shared server answers (it leaves after its 1 ms
// life, so the value is not a timeout any more). Stops the device's server
// either way (so this also quiesces it before a device-wide synchronisation;
// every context's next call relaunches it).
extern "C" int zp_parse_one_config(zp_ctx* c, uint32_t idle_us) {
    if (!c) return -1;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(c->device) != hipSuccess) return -2;
    one_server_stop(c);
    c->one_idle_us = idle_us;
    (void)hipSetDevice(prev);
    return 0;
}

extern "C" int zp_device_current(void) {
    int d = -1;
    const hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess) {
        snprintf(g_ctx_error, ERRBUF_LEN, "hipGetDevice: %s", hipGetErrorString(e));
        return -1;
    }
    return d;
}

// Test hook: the device server's counters (launches, rotations, relaunches
// by the answer wait's stream check).
extern "C" int zp__one_stats(const zp_ctx* c, uint64_t* out) {
    if (!c || !out || c->device < 0 || c->device >= SRV_DEVICES) return -1;
    const SharedServer* S = &g_srv[c->device];
    out[0] = S->launches;
    out[1] = S->rotations;
    out[2] = S->relaunches;
    return 0;
}

// Test hook (tests/test_gpu_parity.py, not in zero_packet.h): the device
// server's life (us, 0: keep) and a stall of stall_us queued in front of
// each of its launches (0: none), and this context's give-up time (us, 0:
// keep). Stops the device's server.
extern "C" int zp__one_test_hooks(zp_ctx* c, uint32_t life_us, uint64_t giveup_us,
                                  uint32_t stall_us) {
    if (!c) return -1;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(c->device) != hipSuccess) return -2;
    SharedServer* S = srv_get(c->device);
    (void)hipSetDevice(prev);
    if (!S) return -2;
    const int rc = zp_parse_one_config(c, c->one_idle_us);
    if (rc) return rc;
    pthread_mutex_lock(&S->m);
    srv_stop_locked(S);
    if (life_us) __atomic_store_n(&S->life_us, life_us, __ATOMIC_RELAXED);
    S->stall_us = stall_us;
    pthread_mutex_unlock(&S->m);
    if (giveup_us) c->one_giveup_ns = (int64_t)giveup_us * 1000;
    return 0;
}

// Several devices at once (one context each): the batch is cut into
// contiguous frame ranges with balanced byte totals, one per context, and the
// contexts run concurrently on their own host threads (the
// frames are independent, there is no exchange step). Results land in the
// caller's arrays at the frames' own indices. Plain pthreads: no C++ runtime
// objects cross the library boundary (the host process may carry another
// libstdc++).
struct MultiJob {
    zp_ctx* ctx;
    const uint8_t* arena;
    uint64_t arena_bytes;
    const uint64_t* offs;
    const uint32_t* lens;
    uint64_t n;
    zp_record* recs;
    zp_ext_offsets* xo;
    zp_ext_offsets* xi;
    int rc;
    char err[ERRBUF_LEN];
};

static void* multi_worker(void* p) {
    MultiJob* j = (MultiJob*)p;
    j->rc = parse_host(j->ctx, j->arena, j->arena_bytes, j->offs, j->lens, j->n, j->recs,
                       j->xo, j->xi);
    if (j->rc) snprintf(j->err, ERRBUF_LEN, "%s", g_ctx_error);
    return NULL;
}

extern "C" int zp_parse_batch_host_multi(zp_ctx* const* ctxs, int nctx, const uint8_t* arena,
                                         uint64_t arena_bytes, const uint64_t* offs,
                                         const uint32_t* lens, uint64_t n, zp_record* recs,
                                         zp_ext_offsets* ext) {
    if (!ctxs || nctx < 1 || nctx > 256) return -1;
    for (int d = 0; d < nctx; ++d)
        if (!ctxs[d]) return -1;
    if (n == 0) return 0;
    if (!arena || !offs || !lens || !recs) return -1;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += lens[i];
    MultiJob* jobs = (MultiJob*)calloc((size_t)nctx, sizeof(MultiJob));
    pthread_t* th = (pthread_t*)calloc((size_t)nctx, sizeof(pthread_t));
    char* started = (char*)calloc((size_t)nctx, 1);
    if (!jobs || !th || !started) {
        free(jobs); free(th); free(started);
        snprintf(g_ctx_error, ERRBUF_LEN, "zp_parse_batch_host_multi: out of memory");
        return -1;
    }
    // range d = frames whose exclusive byte prefix lies in [total*d/nctx, total*(d+1)/nctx)
    uint64_t acc = 0, i = 0;
    for (int d = 0; d < nctx; ++d) {
        const uint64_t lo = i;
        const uint64_t target = d + 1 == nctx ? ~0ull
                              : (uint64_t)((unsigned __int128)total * (unsigned)(d + 1) / (unsigned)nctx);
        while (i < n && acc < target) acc += lens[i++];
        jobs[d] = MultiJob{ctxs[d], arena, arena_bytes, offs + lo, lens + lo, i - lo, recs + lo,
                           ext ? ext + lo : NULL, ext ? ext + n + lo : NULL, 0, {0}};
    }
    int rc = 0;
    for (int d = 0; d < nctx; ++d) {
        if (jobs[d].n == 0) continue;
        if (pthread_create(&th[d], NULL, multi_worker, &jobs[d]) == 0) {
            started[d] = 1;
        } else {
            multi_worker(&jobs[d]);               // no thread: run it here
        }
    }
    for (int d = 0; d < nctx; ++d)
        if (started[d]) pthread_join(th[d], NULL);
    for (int d = 0; d < nctx; ++d) {
        if (jobs[d].rc) {
            snprintf(g_ctx_error, ERRBUF_LEN, "device context %d: %s", d, jobs[d].err);
            rc = jobs[d].rc;
            break;
        }
    }
    free(jobs); free(th); free(started);
    return rc;
}

// Batched PacketBuilder over host buffers (the builder's `&mut [u8]` in host
// memory, e.g. a transmit ring): frames are cut into chunks whose byte span
// fits the context's device arena; per chunk the frames' current bytes go
// H2D (the writers read-modify-write them), the chains run
// (zp_build_batch_device), and the span comes back D2H. The ops and the data
// blob go H2D once. Synchronous.
extern "C" int zp_build_batch_device(uint8_t*, const uint64_t*, const uint32_t*, uint64_t,
                                     const zp_build_op*, const uint32_t*, const uint8_t*,
                                     zp_build_result*, void*);

extern "C" int zp_build_batch_host(zp_ctx* c, uint8_t* arena, uint64_t arena_bytes,
                                   const uint64_t* offs, const uint32_t* lens, uint64_t n,
                                   const zp_build_op* ops, const uint32_t* op_start,
                                   const uint8_t* data, uint64_t data_bytes,
                                   zp_build_result* results) {
    if (!c || (n && (!arena || !offs || !lens || !ops || !op_start))) return -1;
    if (n == 0) return 0;
    // host-side checks of what the kernel would read out of bounds
    if (op_start[n] < op_start[0]) {
        snprintf(g_ctx_error, ERRBUF_LEN, "zp_build_batch_host: op_start not ascending");
        return -1;
    }
    for (uint64_t k = op_start[0]; k < op_start[n]; ++k) {
        const zp_build_op& o = ops[k];
        if (o.data_len != ZP_BUILD_NO_DATA && (uint64_t)o.data_off + o.data_len > data_bytes) {
            snprintf(g_ctx_error, ERRBUF_LEN,
                     "zp_build_batch_host: op %llu data range past data_bytes",
                     (unsigned long long)k);
            return -1;
        }
    }
    for (uint64_t k = 0; k < n; ++k) {
        if (op_start[k + 1] < op_start[k]) {
            snprintf(g_ctx_error, ERRBUF_LEN, "zp_build_batch_host: op_start not ascending");
            return -1;
        }
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(c->device) != hipSuccess) return -2;
    int rc = 0;
    const uint64_t nops = op_start[n] - op_start[0];
    hipStream_t s = c->s[0];
    hipError_t e = grow(&c->d_bops, &c->bops_cap, nops ? nops : 1);
    if (e == hipSuccess) e = grow(&c->d_bdata, &c->bdata_cap, data_bytes ? data_bytes : 16);
    if (e == hipSuccess && !c->d_bstart) e = hipMalloc(&c->d_bstart, (c->chunk_pkts + 1) * 4);
    if (e == hipSuccess && !c->d_bres)
        e = hipMalloc(&c->d_bres, c->chunk_pkts * sizeof(zp_build_result));
    if (e == hipSuccess && !c->h_bstart)
        e = hipHostMalloc(&c->h_bstart, (c->chunk_pkts + 1) * 4, hipHostMallocDefault);
    zp_build_op* d_ops = c->d_bops;
    uint32_t* d_start = c->d_bstart;
    uint8_t* d_data = c->d_bdata;
    zp_build_result* d_res = c->d_bres;
    uint32_t* h_start = c->h_bstart;
    if (e == hipSuccess && nops)
        e = hipMemcpyAsync(d_ops, ops + op_start[0], nops * sizeof(zp_build_op),
                           hipMemcpyHostToDevice, s);
    if (e == hipSuccess && data_bytes)
        e = hipMemcpyAsync(d_data, data, data_bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) {
        snprintf(g_ctx_error, ERRBUF_LEN, "zp_build_batch_host setup: %s", hipGetErrorString(e));
        rc = -2;
    }
    uint64_t i = 0;
    while (rc == 0 && i < n) {
        uint64_t lo = offs[i], hi = offs[i] + lens[i];
        if (hi - lo > c->chunk_bytes || (arena_bytes && hi > arena_bytes)) {
            snprintf(g_ctx_error, ERRBUF_LEN, "frame %llu does not fit the context chunk / arena",
                     (unsigned long long)i);
            rc = -3;
            break;
        }
        uint64_t j = i + 1;
        while (j < n && j - i < c->chunk_pkts) {
            const uint64_t l2 = offs[j] < lo ? offs[j] : lo;
            const uint64_t h2 = offs[j] + lens[j] > hi ? offs[j] + lens[j] : hi;
            if (h2 - l2 > c->chunk_bytes || (arena_bytes && h2 > arena_bytes)) break;
            lo = l2; hi = h2; ++j;
        }
        const uint64_t m = j - i;
        for (uint64_t q = 0; q < m; ++q) {
            c->h_offs[0][q] = offs[i + q] - lo;
            c->h_lens[0][q] = lens[i + q];
        }
        for (uint64_t q = 0; q <= m; ++q) h_start[q] = op_start[i + q] - op_start[i];
        memcpy(c->h_arena[0], arena + lo, hi - lo);
        e = hipMemcpyAsync(c->d_arena[0], c->h_arena[0], hi - lo, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->d_offs[0], c->h_offs[0], m * 8, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->d_lens[0], c->h_lens[0], m * 4, hipMemcpyHostToDevice, s);
        if (e == hipSuccess)
            e = hipMemcpyAsync(d_start, h_start, (m + 1) * 4, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) { rc = -2; break; }
        rc = zp_build_batch_device(c->d_arena[0], c->d_offs[0], c->d_lens[0], m,
                                   d_ops + (op_start[i] - op_start[0]), d_start, d_data, d_res, s);
        if (rc) break;
        e = hipMemcpyAsync(c->h_arena[0], c->d_arena[0], hi - lo, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && results)
            e = hipMemcpyAsync(results + i, d_res, m * sizeof(zp_build_result),
                               hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { rc = -2; break; }
        // frame bytes only: the chunk span may also cover bytes between frames
        for (uint64_t q = 0; q < m; ++q)
            memcpy(arena + offs[i + q], c->h_arena[0] + (offs[i + q] - lo), lens[i + q]);
        i = j;
    }
    if (rc == -2 && e != hipSuccess)
        snprintf(g_ctx_error, ERRBUF_LEN, "zp_build_batch_host: %s", hipGetErrorString(e));
    (void)hipStreamSynchronize(s);
    (void)hipSetDevice(prev);
    return rc;
}
