/*
 * host_stub.c — test-only: a CPU stand-in for the GPU frame builder behind the
 * host driver (pb_builder_t, host/sequence_gpu.h), and a threaded stress test
 * of the TX ring protocol (host/xsk_ring.c).  Built by the host tests into
 * tests/_build/libpbhost_stub.so; never part of the product.
 *
 * Stub frames: frame (k, i) of iteration k, payload i is
 *   len = 42 + min_len + (k * 7 + i) % (max_len - min_len + 1)
 * bytes whose first 16 bytes are {seq_idx, k (u64), i (u16), len (u16)} and the
 * rest zero — enough for the tests to see which frames were sent, how often
 * and in which order.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../pb-af-xdp_amd/host/sequence_gpu.h"
#include "../pb-af-xdp_amd/host/xsk_ring.h"

typedef struct stub_ctx
{
    uint16_t min_len[PB_MAX_SEQUENCES], span[PB_MAX_SEQUENCES], fpi[PB_MAX_SEQUENCES];
    int gpu;
} stub_ctx_t;

typedef struct stub_frames
{
    uint16_t seq_idx;
    uint64_t first_iter, n_frames, cap;
    uint32_t fpi;
    uint16_t *lens;
} stub_frames_t;

static uint64_t g_builds, g_lands, g_opens;

static int s_open(int gpu, void **h)
{
    stub_ctx_t *c = (stub_ctx_t *)calloc(1, sizeof *c);
    if (!c)
        return -12;
    c->gpu = gpu;
    __atomic_add_fetch(&g_opens, 1, __ATOMIC_RELAXED);
    *h = c;
    return 0;
}

static int s_load(void *h, uint16_t i, const pb_sequence_t *s, const uint8_t *sm, const uint8_t *dm,
                  const pb_rules_t *r, uint64_t seed)
{
    (void)sm, (void)dm, (void)r, (void)seed;
    stub_ctx_t *c = (stub_ctx_t *)h;
    c->fpi[i] = s->pl_cnt ? s->pl_cnt : 1;
    c->min_len[i] = s->pl_cnt ? s->pls[0].min_len : 0;
    c->span[i] = s->pl_cnt && s->pls[0].max_len >= s->pls[0].min_len ? s->pls[0].max_len - s->pls[0].min_len + 1 : 1;
    return 0;
}

static int s_alloc(void *h, uint16_t i, uint64_t n_iter, void **frames)
{
    stub_ctx_t *c = (stub_ctx_t *)h;
    stub_frames_t *f = (stub_frames_t *)calloc(1, sizeof *f);
    if (!f)
        return -12;
    f->cap = n_iter * c->fpi[i];
    f->lens = (uint16_t *)calloc(f->cap ? f->cap : 1, sizeof(uint16_t));
    if (!f->lens)
    {
        free(f);
        return -12;
    }
    *frames = f;
    return 0;
}

static int s_build(void *h, uint16_t i, uint64_t k, uint64_t n, void *frames)
{
    stub_ctx_t *c = (stub_ctx_t *)h;
    stub_frames_t *f = (stub_frames_t *)frames;
    if (n * c->fpi[i] > f->cap)
        return -28;
    f->seq_idx = i;
    f->first_iter = k;
    f->fpi = c->fpi[i];
    f->n_frames = n * c->fpi[i];
    for (uint64_t j = 0; j < f->n_frames; ++j)
    {
        const uint64_t kk = k + j / f->fpi, ii = j % f->fpi;
        f->lens[j] = (uint16_t)(42 + c->min_len[i] + (kk * 7 + ii) % c->span[i]);
    }
    __atomic_add_fetch(&g_builds, 1, __ATOMIC_RELAXED);
    return 0;
}

static uint64_t s_n_frames(void *frames)
{
    return ((stub_frames_t *)frames)->n_frames;
}

static int s_land(void *h, void *frames, uint8_t *umem, uint32_t stride, uint32_t slot, uint64_t first, uint32_t n,
                  uint16_t *lens)
{
    (void)h;
    stub_frames_t *f = (stub_frames_t *)frames;
    if (first + n > f->n_frames)
        return -22;
    for (uint32_t j = 0; j < n; ++j)
    {
        const uint64_t fi = first + j;
        const uint16_t len = f->lens[fi];
        if (len > stride)
            return -22;
        uint8_t *p = umem + (uint64_t)(slot + j) * stride;
        memset(p, 0, len);
        const uint64_t kk = f->first_iter + fi / f->fpi;
        const uint16_t ii = (uint16_t)(fi % f->fpi);
        memcpy(p, &f->seq_idx, 2);
        memcpy(p + 2, &kk, 8);
        memcpy(p + 10, &ii, 2);
        memcpy(p + 12, &len, 2);
        lens[j] = len;
    }
    __atomic_add_fetch(&g_lands, 1, __ATOMIC_RELAXED);
    return 0;
}

static int s_land_wait(void *h, uint32_t keep)
{
    (void)h, (void)keep; /* s_land is synchronous */
    return 0;
}

static int s_reg(void *h, void *p, size_t n)
{
    (void)h, (void)p, (void)n;
    return 0;
}
static int s_unreg(void *h, void *p)
{
    (void)h, (void)p;
    return 0;
}
static void s_free(void *h, void *frames)
{
    (void)h;
    stub_frames_t *f = (stub_frames_t *)frames;
    free(f->lens);
    free(f);
}
static void s_close(void *h)
{
    free(h);
}

static const pb_builder_t stub = {s_open,  s_load,   s_alloc, s_build, s_n_frames, s_land,
                                  s_land_wait, s_reg, s_unreg, s_free, s_close};

void stub_install(void)
{
    g_builds = g_lands = g_opens = 0;
    pb_set_builder(&stub);
}

/* the stub with a device count (seq_send's up-front --gpu / --gpus check) */
static int g_devices;
static pb_builder_t stub_dev;
static int s_devcount(int *n)
{
    *n = g_devices;
    return 0;
}
void stub_set_devices(int n)
{
    g_devices = n;
    stub_dev = stub;
    stub_dev.device_count = s_devcount;
    pb_set_builder(&stub_dev);
}

void stub_uninstall(void)
{
    pb_set_builder(NULL);
}

void stub_counts(uint64_t *builds, uint64_t *lands, uint64_t *opens)
{
    *builds = g_builds;
    *lands = g_lands;
    *opens = g_opens;
}

/* ---- TX ring stress: the application side on this thread, the loopback's
 * kernel side on another, as a NIC driver would run it ---- */

typedef struct kern
{
    pb_xsk_t *x;
    volatile int stop;
    uint64_t seen, bad;
    uint64_t next_tag;
} kern_t;

static void check_sink(void *ctx, const uint8_t *frame, uint32_t len, uint64_t addr)
{
    kern_t *k = (kern_t *)ctx;
    uint64_t tag;
    uint16_t l;
    memcpy(&tag, frame, 8);
    memcpy(&l, frame + 8, 2);
    /* frames arrive in submission order, with the length the descriptor says */
    if (tag != k->next_tag || l != len || addr % k->x->frame_size != 0 || frame[len - 1] != (uint8_t)tag)
        ++k->bad;
    ++k->next_tag;
    ++k->seen;
}

static void *kern_main(void *p)
{
    kern_t *k = (kern_t *)p;
    while (!k->stop)
    {
        /* take a few descriptors at a time, as a driver's TX poll would */
        if (pb_xsk_loop_consume(k->x, 1 + (uint32_t)(k->seen % 37), check_sink, k) == 0)
            sched_yield();
    }
    while (pb_xsk_loop_consume(k->x, 4096, check_sink, k))
        ;
    return NULL;
}

/* Send `total` frames of varying length through a loopback queue of n_frames
 * slots with the kernel side on its own thread; returns 0 if every frame came
 * through once, in order, intact, and every descriptor completed. */
int ring_stress(uint32_t n_frames, uint64_t total, uint64_t *wakeups_out)
{
    const uint32_t fs = 2048;
    uint8_t *umem = NULL;
    if (posix_memalign((void **)&umem, 4096, (size_t)n_frames * fs))
        return -12;
    pb_xsk_t x;
    int rc = pb_xsk_loopback(&x, umem, n_frames, fs);
    if (rc)
    {
        free(umem);
        return rc;
    }
    x.loop_auto = 0;
    kern_t k;
    memset(&k, 0, sizeof k);
    k.x = &x;
    pthread_t th;
    pthread_create(&th, NULL, kern_main, &k);
    uint64_t sent = 0;
    uint16_t lens[64];
    while (sent < total)
    {
        uint32_t want = 1 + (uint32_t)((sent * 2654435761u) % 64);
        if (want > total - sent)
            want = (uint32_t)(total - sent);
        if (want > n_frames)
            want = n_frames;
        while (pb_xsk_free_slots(&x) < want)
            if (pb_xsk_complete(&x, n_frames) == 0)
                sched_yield();
        for (uint32_t i = 0; i < want; ++i)
        {
            const uint64_t tag = sent + i;
            const uint16_t len = (uint16_t)(60 + (tag * 13) % 1400);
            uint8_t *p = umem + (size_t)((x.next_slot + i) & (n_frames - 1)) * fs;
            memcpy(p, &tag, 8);
            memcpy(p + 8, &len, 2);
            p[len - 1] = (uint8_t)tag;
            lens[i] = len;
        }
        if ((rc = pb_xsk_send(&x, lens, want)) != 0)
            break;
        sent += want;
    }
    while (rc == 0 && x.outstanding_tx)
        if (pb_xsk_complete(&x, n_frames) == 0)
            sched_yield();
    k.stop = 1;
    pthread_join(th, NULL);
    if (wakeups_out)
        *wakeups_out = x.wakeups;
    if (rc == 0 && (k.seen != total || k.bad || x.completed != total))
        rc = -EIO;
    pb_xsk_close(&x);
    free(umem);
    return rc;
}

/* ---- a recording TX hook: every frame the TX side consumes, in order ---- */
typedef struct rec
{
    uint64_t k;
    uint16_t seq_idx, i, len, thread;
    double t; /* CLOCK_MONOTONIC seconds when the TX side took the frame */
} rec_t;

static rec_t *g_rec;
static uint64_t g_rec_cap, g_rec_n;
static pthread_mutex_t g_rec_mu = PTHREAD_MUTEX_INITIALIZER;

static int rec_hook(void *ctx, int thread_id, const uint8_t *frame, uint16_t len)
{
    (void)ctx;
    rec_t r;
    memcpy(&r.seq_idx, frame, 2);
    memcpy(&r.k, frame + 2, 8);
    memcpy(&r.i, frame + 10, 2);
    memcpy(&r.len, frame + 12, 2);
    r.thread = (uint16_t)thread_id;
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    r.t = ts.tv_sec + ts.tv_nsec * 1e-9;
    if (r.len != len)
        r.len = 0xFFFF; /* the descriptor's length disagrees with the frame */
    pthread_mutex_lock(&g_rec_mu);
    if (g_rec_n < g_rec_cap)
        g_rec[g_rec_n] = r;
    ++g_rec_n;
    pthread_mutex_unlock(&g_rec_mu);
    return 0;
}

int stub_record(uint64_t cap)
{
    free(g_rec);
    g_rec = (rec_t *)calloc(cap ? cap : 1, sizeof *g_rec);
    g_rec_cap = g_rec ? cap : 0;
    g_rec_n = 0;
    pb_set_tx_hook(g_rec ? rec_hook : NULL, NULL);
    return g_rec ? 0 : -12;
}

/* the recorded frames' times (up to n) */
void stub_times(double *t, uint64_t n)
{
    const uint64_t m = g_rec_n < g_rec_cap ? g_rec_n : g_rec_cap;
    for (uint64_t j = 0; j < m && j < n; ++j)
        t[j] = g_rec[j].t;
}

/* recorded frames -> k[], i[], len[], thread[] (up to n); returns the count seen */
uint64_t stub_recorded(uint64_t *k, uint16_t *i, uint16_t *len, uint16_t *thread, uint64_t n)
{
    const uint64_t m = g_rec_n < g_rec_cap ? g_rec_n : g_rec_cap;
    for (uint64_t j = 0; j < m && j < n; ++j)
    {
        k[j] = g_rec[j].k;
        i[j] = g_rec[j].i;
        len[j] = g_rec[j].len;
        thread[j] = g_rec[j].thread;
    }
    return g_rec_n;
}
