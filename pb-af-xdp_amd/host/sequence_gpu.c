/*
 * sequence_gpu.c — seq_send() / shutdown_prog() over libpbgpu (see .h).
 *
 * One worker pthread per TX thread of a sequence (the reference's thread_hdl,
 * sequence.c:33-700, with the per-packet build moved to the GPU):
 *   setup      MACs (sequence.c:111-136), pbgpu_load_sequence (the template,
 *              sequence.c:138-374), a page-aligned UMEM registered with HIP
 *              (af_xdp.c:374-389), the TX queue (AF_XDP socket or loopback);
 *   loop       claim a batch of iterations (the max_pckts quota, exact across
 *              threads), build it on the GPU while the previous batch is
 *              landed in UMEM slots and submitted on the TX ring
 *              (send_packet/complete_tx, af_xdp.c:25-53, 178-241), count
 *              (sequence.c:633-653), pace (pps / bps / delay, sequence.c:389-431,
 *              655-659) and check the stop conditions (sequence.c:662-684).
 */
#define _GNU_SOURCE
#include "sequence_gpu.h"
#include "mac.h"
#include "xsk_ring.h"

#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#define PB_MAX_WORKERS 1024
#define PB_LAND_INFLIGHT_MAX 16 /* landings queued per thread (PB_LAND_INFLIGHT, default 2) */
/* frames per landing: half of the UMEM (PB_LAND_CHUNK overrides) */

static uint32_t env_u32(const char *name, uint32_t dflt, uint32_t lo, uint32_t hi)
{
    const char *e = getenv(name);
    long v = e ? atol(e) : (long)dflt;
    return v < (long)lo ? lo : (v > (long)hi ? hi : (uint32_t)v);
}
#define PB_BATCH_BYTES_MAX (256ull << 20) /* device bytes per frame buffer (two per worker) */
#define PB_PACE_GRAIN_US 50.0 /* a paced submit group spans about this much of the rate (one frame at least) */

static uint64_t total_pckts[PB_MAX_SEQUENCES];
static uint64_t total_bytes[PB_MAX_SEQUENCES];
static uint64_t claimed_frames[PB_MAX_SEQUENCES]; /* max_pckts quota handed to workers */
static uint64_t tx_descs[PB_MAX_SEQUENCES], tx_comps[PB_MAX_SEQUENCES], tx_wakeups[PB_MAX_SEQUENCES];
static uint64_t umem_allocs[PB_MAX_SEQUENCES]; /* UMEMs allocated per sequence (--sharedumem: one) */
static time_t start_time[PB_MAX_SEQUENCES];
static time_t end_time[PB_MAX_SEQUENCES];
static uint16_t seq_cnt;
static pthread_t workers[PB_MAX_WORKERS];
static uint8_t joined[PB_MAX_WORKERS];
static int worker_cnt;
static int last_error;
static int verbose;
static pb_tx_fn tx_hook;
static void *tx_ctx;
static volatile int stop_requested;

void pb_request_stop(void)
{
    stop_requested = 1;
}

int pb_stop_requested(void)
{
    return stop_requested;
}

void pb_set_tx_hook(pb_tx_fn fn, void *ctx)
{
    tx_hook = fn;
    tx_ctx = ctx;
}

void pb_set_verbose(int v)
{
    verbose = v;
}

int pb_last_error(void)
{
    return last_error;
}

int pb_sequence_totals(uint16_t seq, uint64_t *pckts, uint64_t *bytes)
{
    if (seq >= PB_MAX_SEQUENCES)
        return PBGPU_EINVAL;
    if (pckts)
        *pckts = __atomic_load_n(&total_pckts[seq], __ATOMIC_RELAXED);
    if (bytes)
        *bytes = __atomic_load_n(&total_bytes[seq], __ATOMIC_RELAXED);
    return PBGPU_OK;
}

int pb_sequence_umems(uint16_t seq, uint64_t *umems)
{
    if (seq >= PB_MAX_SEQUENCES)
        return PBGPU_EINVAL;
    if (umems)
        *umems = __atomic_load_n(&umem_allocs[seq], __ATOMIC_RELAXED);
    return PBGPU_OK;
}

int pb_sequence_tx_stats(uint16_t seq, uint64_t *descs, uint64_t *completions, uint64_t *wakeups)
{
    if (seq >= PB_MAX_SEQUENCES)
        return PBGPU_EINVAL;
    if (descs)
        *descs = __atomic_load_n(&tx_descs[seq], __ATOMIC_RELAXED);
    if (completions)
        *completions = __atomic_load_n(&tx_comps[seq], __ATOMIC_RELAXED);
    if (wakeups)
        *wakeups = __atomic_load_n(&tx_wakeups[seq], __ATOMIC_RELAXED);
    return PBGPU_OK;
}

/* ---------------- the builder: libpbgpu ---------------- */

static int gb_open(int gpu, void **h)
{
    pbgpu_ctx *c = NULL;
    const int rc = pbgpu_open(gpu, &c);
    if (rc == 0)
        (void)pbgpu_set_timing(c, PBGPU_TIMING_SPAN); /* a sender never reads per-launch timings */
    *h = c;
    return rc;
}
static int gb_load(void *h, uint16_t i, const pb_sequence_t *s, const uint8_t *sm, const uint8_t *dm,
                   const pb_rules_t *r, uint64_t seed)
{
    return pbgpu_load_sequence((pbgpu_ctx *)h, i, s, sm, dm, r, seed);
}
static int gb_alloc(void *h, uint16_t i, uint64_t n_iter, void **frames)
{
    uint64_t mf = 0, mb = 0;
    int rc = pbgpu_build_size((pbgpu_ctx *)h, i, n_iter, &mf, &mb);
    if (rc == 0)
        rc = pbgpu_frames_alloc((pbgpu_ctx *)h, mf, mb, (pbgpu_frames **)frames);
    return rc;
}
static int gb_build(void *h, uint16_t i, uint64_t k, uint64_t n, void *frames)
{
    return pbgpu_build((pbgpu_ctx *)h, i, k, n, (pbgpu_frames *)frames);
}
static uint64_t gb_n_frames(void *frames)
{
    return ((pbgpu_frames *)frames)->n_frames;
}
static int gb_land(void *h, void *frames, uint8_t *umem, uint32_t stride, uint32_t slot, uint64_t first, uint32_t n,
                   uint16_t *lens)
{
    return pbgpu_copy_to_umem_async((pbgpu_ctx *)h, (pbgpu_frames *)frames, umem, stride, slot, first, n, lens);
}
static int gb_land_wait(void *h, uint32_t keep)
{
    return pbgpu_land_wait((pbgpu_ctx *)h, keep);
}
static int gb_reg(void *h, void *p, size_t n)
{
    return pbgpu_host_register((pbgpu_ctx *)h, p, n);
}
static int gb_unreg(void *h, void *p)
{
    return pbgpu_host_unregister((pbgpu_ctx *)h, p);
}
static void gb_free(void *h, void *frames)
{
    pbgpu_frames_free((pbgpu_ctx *)h, (pbgpu_frames *)frames);
}
static void gb_close(void *h)
{
    pbgpu_close((pbgpu_ctx *)h);
}

static const pb_builder_t gpu_builder = {gb_open, gb_load,  gb_alloc, gb_build, gb_n_frames, gb_land,
                                         gb_land_wait, gb_reg, gb_unreg, gb_free, gb_close, pbgpu_device_count};
static const pb_builder_t *builder = &gpu_builder;

void pb_set_builder(const pb_builder_t *b)
{
    builder = b ? b : &gpu_builder;
}

/* ---------------- worker ---------------- */

/* --sharedumem (af_xdp.c:412-428): one UMEM of NUM_FRAMES slots per sequence, shared by its
 * threads; thread t owns the slot range [t * slots, (t + 1) * slots) (the reference's threads
 * all write the same frame indices, B10).  With AF_XDP sockets thread 0's socket registers it
 * and the others bind with XDP_SHARED_UMEM to that socket's fd. */
typedef struct shared_umem
{
    uint8_t *base;
    uint32_t slots; /* per thread, a power of two */
    int refs;       /* workers still using it; the last one frees it */
    int fd;         /* thread 0's socket, once open (-1 before; -2 if it failed) */
    pthread_mutex_t mu;
    pthread_cond_t cv;
    /* --queue with several threads: every socket on the owner's queue, reaping the owner's
     * completion ring (pb_xsk_shared_cq_t); the owner's socket stays open until the last
     * thread is done with the ring */
    int one_queue;
    pb_xsk_shared_cq_t scq;
    pb_xsk_t owner;
    int owner_open;
} shared_umem_t;

typedef struct worker_arg
{
    pb_sequence_t seq;
    const char *device; /* the interface seq_send() was given (MAC discovery, AF_XDP socket) */
    uint16_t seq_idx;
    int gpu;
    int shard;   /* TX thread index = queue id (af_xdp.c:443) */
    int n_shards;
    struct cmd_line_af_xdp cmd;
    shared_umem_t *shared; /* --sharedumem, else NULL */
} worker_arg_t;

static void shared_release(shared_umem_t *u)
{
    pthread_mutex_lock(&u->mu);
    const int last = --u->refs == 0;
    pthread_mutex_unlock(&u->mu);
    if (last)
    {
        if (u->owner_open)
            pb_xsk_close(&u->owner);
        if (u->one_queue)
            pb_xsk_scq_free(&u->scq);
        pthread_mutex_destroy(&u->mu);
        pthread_cond_destroy(&u->cv);
        free(u->base);
        free(u);
    }
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* sleep until monotonic time t, in slices that notice a stop request */
static void sleep_until(double t)
{
    for (;;)
    {
        const double d = t - now_s();
        if (d <= 0 || stop_requested)
            return;
        const double s = d < 0.01 ? d : 0.01;
        struct timespec ts = {(time_t)s, (long)((s - (double)(time_t)s) * 1e9)};
        nanosleep(&ts, NULL);
    }
}

/* Claim up to `want` frames of the max_pckts quota (whole iterations of fpi
 * frames): returns the iterations granted, 0 when the quota is spent.  Claims
 * are exact across threads and GPUs: the sequence sends max_pckts frames
 * (rounded up to a whole iteration), where the reference's threads overshoot
 * by up to one iteration each (sequence.c:662-666). */
static uint64_t claim_iters(uint16_t idx, uint64_t max_pckts, uint64_t want_iters, uint32_t fpi)
{
    if (max_pckts == 0)
        return want_iters;
    uint64_t cur = __atomic_load_n(&claimed_frames[idx], __ATOMIC_RELAXED);
    for (;;)
    {
        if (cur >= max_pckts)
            return 0;
        uint64_t iters = (max_pckts - cur + fpi - 1) / fpi;
        if (iters > want_iters)
            iters = want_iters;
        if (__atomic_compare_exchange_n(&claimed_frames[idx], &cur, cur + iters * fpi, 0, __ATOMIC_RELAXED,
                                        __ATOMIC_RELAXED))
            return iters;
    }
}

typedef struct sink_arg
{
    int shard;
    int seq_num;
} sink_arg_t;

static void tx_sink(void *ctx, const uint8_t *frame, uint32_t len, uint64_t addr)
{
    (void)addr;
    const sink_arg_t *a = (const sink_arg_t *)ctx;
    if (tx_hook && tx_hook(tx_ctx, a->shard, frame, (uint16_t)len) != 0)
        fprintf(stderr, "[%d][%d] ERROR - Could not send packet (%d) :: %s.\n", a->seq_num, 1, a->shard,
                strerror(errno));
}

/* The reference's per-packet verbose line (sequence.c:612-631), from a frame as it sits in its
 * UMEM slot: "[seq][payload] Sent <len> bytes of data from <src>:<sport> to <dst>:<dport>."
 * The source is the configured src_ip string, else the frame's drawn source address (rand_ip's
 * dotted string); the ports are the UDP / TCP header's (0 for ICMP), the destination the
 * configured dst_ip string. */
static void print_sent(int seq_num, uint32_t pl_idx, const pb_sequence_t *seq, const uint8_t *fr, uint16_t len)
{
    char sip[16];
    const char *src = seq->ip.src_ip;
    uint32_t sport = 0, dport = 0;
    if (len >= 34)
    {
        if (src == NULL)
        {
            snprintf(sip, sizeof sip, "%u.%u.%u.%u", fr[26], fr[27], fr[28], fr[29]);
            src = sip;
        }
        const uint32_t l4 = 14u + 4u * (fr[14] & 0xFu);
        if ((fr[23] == 17 || fr[23] == 6) && l4 + 4u <= len)
        {
            sport = ((uint32_t)fr[l4] << 8) | fr[l4 + 1];
            dport = ((uint32_t)fr[l4 + 2] << 8) | fr[l4 + 3];
        }
    }
    fprintf(stdout, "[%d][%u] Sent %u bytes of data from %s:%u to %s:%u.\n", seq_num, pl_idx + 1, (unsigned)len,
            src ? src : "", sport, seq->ip.dst_ip ? seq->ip.dst_ip : "", dport);
}

static void *gpu_worker(void *p)
{
    worker_arg_t *w = (worker_arg_t *)p;
    const pb_sequence_t *seq = &w->seq;
    const int seq_num = w->seq_idx + 1;
    const pb_builder_t *B = builder;
    void *ctx = NULL;
    void *fr[2] = {NULL, NULL};
    uint8_t *umem = NULL;
    int registered = 0;
    pb_xsk_t xsk;
    memset(&xsk, 0, sizeof xsk);
    xsk.fd = -1;
    sink_arg_t sink = {w->shard, seq_num};
    /* this thread's UMEM slots: its own NUM_FRAMES chunks of FRAME_SIZE (--umemframes) cut into
     * slots of --umemslot bytes (one per chunk by default), or its range of the sequence's
     * shared UMEM */
    const uint32_t umem_frames = w->cmd.umem_frames ? w->cmd.umem_frames : PB_NUM_FRAMES;
    const uint32_t slot_sz = w->cmd.umem_slot ? w->cmd.umem_slot : PB_FRAME_SIZE;
    const uint32_t umem_slots = umem_frames * (PB_FRAME_SIZE / slot_sz);
    const uint32_t nslots = w->shared ? w->shared->slots : umem_slots;
    const uint32_t slot_base = w->shared ? (uint32_t)w->shard * nslots : 0;
    const size_t umem_bytes = (size_t)nslots * slot_sz;
    uint16_t *lens = (uint16_t *)calloc(nslots, sizeof(uint16_t));
    int rc;
    if (lens == NULL)
    {
        last_error = PBGPU_ENOMEM;
        goto out;
    }

    if ((rc = B->open(w->gpu, &ctx)) != 0)
    {
        fprintf(stderr, "[%d] Error opening GPU %d :: %s.\n", seq_num, w->gpu, pbgpu_strerror(rc));
        last_error = rc;
        goto out;
    }
    pb_rules_t rules = {w->cmd.literal_payload ? PB_PAYLOAD_LITERAL : PB_PAYLOAD_STREAM,
                        w->cmd.single_fold ? PB_FOLD_SINGLE : PB_FOLD_FULL};
    /* MACs: a zero source MAC is the device's, a zero destination MAC the default
     * gateway's (sequence.c:111-136) */
    uint8_t smac[6] = {0}, dmac[6] = {0};
    if (seq->eth.src_mac)
        sscanf(seq->eth.src_mac, "%hhx:%hhx:%hhx:%hhx:%hhx:%hhx", &smac[0], &smac[1], &smac[2], &smac[3], &smac[4],
               &smac[5]);
    if (seq->eth.dst_mac)
        sscanf(seq->eth.dst_mac, "%hhx:%hhx:%hhx:%hhx:%hhx:%hhx", &dmac[0], &dmac[1], &dmac[2], &dmac[3], &dmac[4],
               &dmac[5]);
    static const uint8_t zero[6] = {0};
    if (memcmp(smac, zero, 6) == 0)
    {
        if (pb_get_src_mac_address(w->device, smac) != 0)
            fprintf(stdout, "[%d] WARNING - Failed to retrieve MAC address for %s.\n", seq_num, w->device);
        if (memcmp(smac, zero, 6) == 0)
            fprintf(stdout, "[%d] WARNING - Source MAC address retrieved is 00:00:00:00:00:00.\n", seq_num);
    }
    if (memcmp(dmac, zero, 6) == 0)
        (void)pb_get_gw_mac(dmac);
    if (verbose)
    {
        printf("[%d] Source MAC address => %hhx:%hhx:%hhx:%hhx:%hhx:%hhx.\n", seq_num, smac[0], smac[1], smac[2],
               smac[3], smac[4], smac[5]);
        printf("[%d] Destination MAC address => %hhx:%hhx:%hhx:%hhx:%hhx:%hhx.\n", seq_num, dmac[0], dmac[1], dmac[2],
               dmac[3], dmac[4], dmac[5]);
    }
    if ((rc = B->load(ctx, w->seq_idx, seq, smac, dmac, &rules, w->cmd.seed_base)) != 0)
    {
        fprintf(stderr, "[%d] Error loading sequence on GPU %d :: %s.\n", seq_num, w->gpu, pbgpu_strerror(rc));
        last_error = rc;
        goto out;
    }
    const uint32_t fpi = seq->pl_cnt < 1 ? 1u : seq->pl_cnt;
    uint32_t max_flen = 42 + 12; /* headers */
    for (uint16_t i = 0; i < seq->pl_cnt; ++i)
        max_flen += seq->pls[i].max_len > 0 ? seq->pls[i].max_len : 1024; /* static lengths are bounded by the parser */
    uint64_t batch = w->cmd.gpu_batch ? w->cmd.gpu_batch : (1u << 20);
    while (batch > 1 && batch * fpi * max_flen > PB_BATCH_BYTES_MAX)
        batch >>= 1;
    /* launch-level pacing: one launch covers at most ~1/10 s of the configured rate
     * (pps and bps are global over the sequence's threads; delay is per thread
     * and per packet, sequence.c:655-659) */
    if (seq->pps > 0)
    {
        const uint64_t cap = seq->pps / (10ull * (uint64_t)w->n_shards * fpi);
        batch = batch < (cap ? cap : 1) ? batch : (cap ? cap : 1);
    }
    if (seq->bps > 0)
    {
        const uint64_t cap = seq->bps / (10ull * (uint64_t)w->n_shards * fpi * max_flen);
        batch = batch < (cap ? cap : 1) ? batch : (cap ? cap : 1);
    }
    if (seq->delay > 0)
    {
        const uint64_t cap = 100000ull / ((uint64_t)seq->delay * fpi);
        batch = batch < (cap ? cap : 1) ? batch : (cap ? cap : 1);
    }
    /* submit pacing inside a landed chunk: groups of pace_g frames, each at its due time, a group
     * spanning ~PB_PACE_GRAIN_US of this thread's share of the rate (one frame when frames are
     * further apart: the reference's per-packet delay, sequence.c:655-659); 0 = unpaced */
    uint32_t pace_g = 0;
    if (seq->pps > 0 || seq->bps > 0 || seq->delay > 0)
    {
        double tf = seq->delay > 0 ? (double)seq->delay * 1e-6 : 0.0; /* seconds per frame, this thread */
        if (seq->pps > 0 && (double)w->n_shards / (double)seq->pps > tf)
            tf = (double)w->n_shards / (double)seq->pps;
        if (seq->bps > 0 && (double)w->n_shards * max_flen / (double)seq->bps > tf)
            tf = (double)w->n_shards * max_flen / (double)seq->bps;
        const double g = PB_PACE_GRAIN_US * 1e-6 / tf;
        pace_g = g < 1.0 ? 1u : g > 65536.0 ? 65536u : (uint32_t)g;
    }
    if ((rc = B->alloc(ctx, w->seq_idx, batch, &fr[0])) != 0 || (rc = B->alloc(ctx, w->seq_idx, batch, &fr[1])) != 0)
    {
        last_error = rc;
        goto out;
    }
    uint8_t *umem_base = NULL; /* the UMEM the TX ring addresses (shared: the sequence's) */
    if (w->shared)
    {
        umem_base = w->shared->base;
        umem = umem_base + (size_t)slot_base * slot_sz;
    }
    else
    {
        if (posix_memalign((void **)&umem, (size_t)sysconf(_SC_PAGESIZE), umem_bytes) != 0)
        {
            umem = NULL;
            last_error = PBGPU_ENOMEM;
            goto out;
        }
        memset(umem, 0, umem_bytes);
        umem_base = umem;
        __atomic_add_fetch(&umem_allocs[w->seq_idx], 1, __ATOMIC_RELAXED);
    }
    registered = B->host_register(ctx, umem, umem_bytes) == 0;

    /* the TX queue: an AF_XDP socket on queue `shard` (or --queue, af_xdp.c:443),
     * or the in-memory loopback whose consumer hands frames to the TX hook */
    if (w->cmd.tx && strcmp(w->cmd.tx, "xsk") == 0)
    {
        const uint16_t bf = pb_bind_flags(&w->cmd);
        const uint32_t q = w->cmd.queue_set ? (uint32_t)w->cmd.queue : (uint32_t)w->shard;
        int shared_fd = -1;
        if (w->shared && w->shard > 0)
        {
            /* thread 0's socket owns the shared UMEM registration: wait for it */
            pthread_mutex_lock(&w->shared->mu);
            while (w->shared->fd == -1 && !stop_requested)
                pthread_cond_wait(&w->shared->cv, &w->shared->mu);
            shared_fd = w->shared->fd;
            pthread_mutex_unlock(&w->shared->mu);
            if (shared_fd < 0)
            {
                last_error = PBGPU_EIO;
                goto out;
            }
        }
        pb_xsk_shared_cq_t *scq = w->shared && w->shared->one_queue ? &w->shared->scq : NULL;
        rc = pb_xsk_open(&xsk, w->device, q, umem_base, nslots, slot_sz, PB_FRAME_SIZE, bf, shared_fd, slot_base,
                         w->shared ? umem_slots : nslots, w->cmd.queue_set ? (uint32_t)w->cmd.queue : 0u, scq,
                         (uint32_t)w->shard);
        if (w->shared && w->shard == 0)
        {
            pthread_mutex_lock(&w->shared->mu);
            w->shared->fd = rc == 0 ? xsk.fd : -2;
            pthread_cond_broadcast(&w->shared->cv);
            pthread_mutex_unlock(&w->shared->mu);
        }
        if (rc != 0)
        {
            fprintf(stderr, "Could not setup AF_XDP socket at index %d :: %s (%d).\n", w->shard, strerror(-rc), -rc);
            last_error = rc;
            goto out;
        }
    }
    else if ((rc = w->shared && w->shared->one_queue
                       ? pb_xsk_loopback_shared(&xsk, umem_base, slot_sz, &w->shared->scq, (uint32_t)w->shard)
                       : pb_xsk_loopback(&xsk, umem_base, nslots, slot_sz)) != 0)
    {
        last_error = rc;
        goto out;
    }
    else
    {
        xsk.slot_base = slot_base;
        xsk.loop_sink = tx_hook ? tx_sink : NULL;
        xsk.loop_ctx = &sink;
        const char *hold = getenv("PB_LOOP_HOLD"); /* tests: frames the loopback keeps in flight */
        xsk.loop_hold = hold ? (uint32_t)atoi(hold) : 0u;
    }
    /* --batchsize: descriptors per reserve / submit / complete (send_packet, af_xdp.c:184-233);
     * without it one landed chunk is one submit */
    xsk.batch = w->cmd.batch_set ? w->cmd.batch_size : 0u;

    /* landing granularity: frames per landing and landings in flight (their launch and
     * completion latencies overlap); tunable for the host-rate probe (scripts/e2e_probe.py) */
    const uint32_t land_chunk = env_u32("PB_LAND_CHUNK", nslots / 2 > 0 ? nslots / 2 : 1, 1, nslots);
    /* 64-B UDP, one TX thread (profiles/r03/e2e): 2048 x 2 129-137 Mpps, 1024 x 3 73, 512 x 6 34-43,
     * 256 x 12 20-28 — each landing is a kernel launch and a host wait, so few large ones win */
    const uint32_t land_inflight = env_u32("PB_LAND_INFLIGHT", 2, 1, PB_LAND_INFLIGHT_MAX);
    const double t0 = now_s();
    uint64_t my_frames = 0; /* this thread's frames: the delay pacing (per thread) */
    uint64_t step = 0;
    int cur = 0;
    /* batch `step` covers iterations [(step * n_shards + shard) * batch, + n_iter) */
    uint64_t n_cur = claim_iters(w->seq_idx, seq->max_pckts, batch, fpi);
    if (n_cur && (rc = B->build(ctx, w->seq_idx, ((uint64_t)w->shard) * batch, n_cur, fr[cur])) != 0)
    {
        fprintf(stderr, "[%d] Error building frames on GPU %d :: %s.\n", seq_num, w->gpu, pbgpu_strerror(rc));
        last_error = rc;
        goto out;
    }
    int done = n_cur == 0 ? 4 : 0; /* 1 max bytes, 2 time, 3 error, 4 quota spent */
    while (!done && !stop_requested)
    {
        /* double buffering: the next batch builds on the GPU while this one lands */
        const uint64_t n_next = claim_iters(w->seq_idx, seq->max_pckts, batch, fpi);
        if (n_next &&
            (rc = B->build(ctx, w->seq_idx, ((step + 1) * (uint64_t)w->n_shards + (uint64_t)w->shard) * batch, n_next,
                           fr[cur ^ 1])) != 0)
        {
            fprintf(stderr, "[%d] Error building frames on GPU %d :: %s.\n", seq_num, w->gpu, pbgpu_strerror(rc));
            last_error = rc;
            break;
        }
        const uint64_t nf = B->n_frames(fr[cur]);
        /* land in slot-ring order with up to PB_LAND_INFLIGHT landings queued: chunk
         * c + 1 lands while chunk c is submitted (their latencies overlap) */
        uint64_t f0 = 0, f_issue = 0;
        uint32_t land_slot = xsk.next_slot, in_land = 0;
        uint32_t qn_[PB_LAND_INFLIGHT_MAX];
        int qh = 0, qn = 0;
        while (f0 < nf && !done && !stop_requested)
        {
            while (qn < (int)land_inflight && f_issue < nf)
            {
                uint32_t free_slots = pb_xsk_free_slots(&xsk) - in_land;
                if (free_slots == 0)
                {
                    if (qn)
                        break;
                    if (pb_xsk_complete(&xsk, nslots) == 0)
                        sched_yield();
                    if (stop_requested)
                        break;
                    continue;
                }
                uint32_t n = free_slots < land_chunk ? free_slots : land_chunk;
                if ((uint64_t)n > nf - f_issue)
                    n = (uint32_t)(nf - f_issue);
                if (n > nslots - land_slot) /* the slot ring wraps: a chunk never does */
                    n = nslots - land_slot;
                if ((rc = B->land(ctx, fr[cur], umem, slot_sz, land_slot, f_issue, n, lens + land_slot)) != 0)
                {
                    fprintf(stderr, "[%d] Error landing frames from GPU %d :: %s%s.\n", seq_num, w->gpu,
                            pbgpu_strerror(rc),
                            rc == PBGPU_EINVAL && slot_sz < PB_FRAME_SIZE ? " (frames longer than --umemslot?)" : "");
                    last_error = rc;
                    done = 3;
                    break;
                }
                qn_[(qh + qn) % land_inflight] = n;
                ++qn;
                in_land += n;
                land_slot = (land_slot + n) & (nslots - 1);
                f_issue += n;
            }
            if (done || qn == 0)
                break;
            /* the oldest landing is in its slots: submit it */
            if ((rc = B->land_wait(ctx, (uint32_t)qn - 1)) != 0)
            {
                last_error = rc;
                done = 3;
                break;
            }
            uint32_t n = qn_[qh];
            qh = (qh + 1) % land_inflight;
            --qn;
            in_land -= n;
            const uint16_t *ln = lens + xsk.next_slot;
            uint64_t bytes = 0;
            for (uint32_t i = 0; i < n; ++i)
                bytes += ln[i];
            if (seq->max_bytes > 0) /* send until the total reaches max_bytes (sequence.c:668-674) */
            {
                uint64_t tot = __atomic_load_n(&total_bytes[w->seq_idx], __ATOMIC_RELAXED);
                for (;;)
                {
                    if (tot >= seq->max_bytes)
                    {
                        n = 0, bytes = 0;
                        break;
                    }
                    uint32_t m = 0;
                    uint64_t b = 0;
                    while (m < n && tot + b < seq->max_bytes)
                        b += ln[m++];
                    if (__atomic_compare_exchange_n(&total_bytes[w->seq_idx], &tot, tot + b, 0, __ATOMIC_RELAXED,
                                                    __ATOMIC_RELAXED))
                    {
                        /* the budget ends inside this chunk: its remaining frames are never sent, so
                         * no further landing may be queued — the slot accounting above (in_land,
                         * land_slot) assumed the whole chunk would go out */
                        if (m < n)
                            done = 1;
                        n = m, bytes = b;
                        break;
                    }
                }
                if (n == 0)
                {
                    done = 1;
                    break;
                }
            }
            else
                __atomic_add_fetch(&total_bytes[w->seq_idx], bytes, __ATOMIC_RELAXED);
            const uint32_t sent_slot = xsk.next_slot;
            /* the chunk in pace_g groups (all at once unpaced), each group when it is due: pps
             * against the sequence's packets so far, bps against its bytes (this chunk's already
             * counted: less those not yet submitted), delay per thread */
            uint64_t left_b = bytes;
            for (uint32_t sub = 0; sub < n;)
            {
                const uint32_t m = pace_g && n - sub > pace_g ? pace_g : n - sub;
                if (pace_g && sub)
                {
                    double due = 0;
                    if (seq->pps > 0)
                        due = (double)__atomic_load_n(&total_pckts[w->seq_idx], __ATOMIC_RELAXED) / (double)seq->pps;
                    if (seq->bps > 0)
                    {
                        const double db =
                            (double)(__atomic_load_n(&total_bytes[w->seq_idx], __ATOMIC_RELAXED) - left_b) /
                            (double)seq->bps;
                        due = db > due ? db : due;
                    }
                    if (seq->delay > 0)
                    {
                        const double dd = (double)my_frames * (double)seq->delay * 1e-6;
                        due = dd > due ? dd : due;
                    }
                    sleep_until(t0 + due);
                }
                if ((rc = pb_xsk_send(&xsk, ln + sub, m)) != 0)
                    break;
                for (uint32_t i = sub; i < sub + m; ++i)
                    left_b -= ln[i];
                __atomic_add_fetch(&total_pckts[w->seq_idx], m, __ATOMIC_RELAXED);
                my_frames += m;
                sub += m;
            }
            if (rc != 0)
            {
                fprintf(stderr, "[%d][%d] ERROR - Could not send packet on AF_XDP socket (%d) :: %s.\n", seq_num, 1,
                        w->shard, strerror(-rc));
                last_error = rc;
                done = 3;
                break;
            }
            if (verbose) /* the slots keep these frames until this thread lands into them again */
                for (uint32_t i = 0; i < n; ++i)
                    print_sent(seq_num, (uint32_t)((f0 + i) % fpi), seq, umem + (size_t)(sent_slot + i) * slot_sz,
                               ln[i]);
            f0 += n;

            /* pacing (sequence.c:389-431, 655-659) at landing-chunk granularity: pps and
             * bps against the sequence's global totals, delay per thread and packet */
            double want = 0;
            if (seq->pps > 0)
                want = (double)__atomic_load_n(&total_pckts[w->seq_idx], __ATOMIC_RELAXED) / (double)seq->pps;
            if (seq->bps > 0)
            {
                const double wb = (double)__atomic_load_n(&total_bytes[w->seq_idx], __ATOMIC_RELAXED) /
                                  (double)seq->bps; /* bytes per second (README.md:113, sequence.c:650-652) */
                want = wb > want ? wb : want;
            }
            if (seq->delay > 0)
            {
                const double wd = (double)my_frames * (double)seq->delay * 1e-6;
                want = wd > want ? wd : want;
            }
            if (want > 0)
                sleep_until(t0 + want);
            if (seq->time > 0 && now_s() - t0 >= (double)seq->time)
                done = 2;
        }
        /* a stop leaves landings queued: let them finish before the buffers are reused */
        (void)B->land_wait(ctx, 0);
        if (verbose)
            fprintf(stdout, "[%d] Thread %d (GPU %d) sent %llu frames of iteration batch %llu.\n", seq_num, w->shard,
                    w->gpu, (unsigned long long)f0, (unsigned long long)step);
        if (seq->max_pckts > 0 && n_next == 0 &&
            __atomic_load_n(&claimed_frames[w->seq_idx], __ATOMIC_RELAXED) >= seq->max_pckts)
        {
            fprintf(stdout, "[%d] Max packets exceeded for sequence. Stopping...\n", seq_num);
            break;
        }
        if (done == 1 && seq->max_bytes > 0)
        {
            fprintf(stdout, "[%d] Max bytes exceeded for sequence. Stopping...\n", seq_num);
            break;
        }
        if (done == 2 || (seq->time > 0 && now_s() - t0 >= (double)seq->time))
        {
            fprintf(stdout, "[%d] Time exceeded for sequence. Stopping...\n", seq_num);
            break;
        }
        if (done || n_next == 0)
            break;
        cur ^= 1;
        ++step;
    }
    /* drain: every submitted frame completes before the UMEM goes away */
    xsk.loop_hold = 0;
    for (int spin = 0; xsk.outstanding_tx && spin < 100000; ++spin)
        if (pb_xsk_complete(&xsk, nslots) == 0)
            sched_yield();
out:
    end_time[w->seq_idx] = time(NULL);
    __atomic_add_fetch(&tx_descs[w->seq_idx], xsk.completed + xsk.outstanding_tx, __ATOMIC_RELAXED);
    __atomic_add_fetch(&tx_comps[w->seq_idx], xsk.completed, __ATOMIC_RELAXED);
    __atomic_add_fetch(&tx_wakeups[w->seq_idx], xsk.wakeups, __ATOMIC_RELAXED);
    if (w->shared && w->shard == 0 && xsk.fd < 0 && w->cmd.tx && strcmp(w->cmd.tx, "xsk") == 0)
    {
        /* thread 0 failed before publishing its socket: release the waiting threads */
        pthread_mutex_lock(&w->shared->mu);
        if (w->shared->fd == -1)
            w->shared->fd = -2;
        pthread_cond_broadcast(&w->shared->cv);
        pthread_mutex_unlock(&w->shared->mu);
    }
    if (w->shared && w->shared->one_queue && w->shard == 0 && xsk.fd >= 0)
    {
        /* the owner's completion ring serves the other sockets until they are done */
        pthread_mutex_lock(&w->shared->mu);
        w->shared->owner = xsk;
        w->shared->owner_open = 1;
        pthread_mutex_unlock(&w->shared->mu);
    }
    else
        pb_xsk_close(&xsk);
    if (umem)
    {
        if (registered)
            B->host_unregister(ctx, umem);
        if (!w->shared)
            free(umem);
    }
    if (w->shared)
        shared_release(w->shared);
    for (int i = 0; i < 2; ++i)
        if (fr[i])
            B->free_frames(ctx, fr[i]);
    if (ctx)
        B->close(ctx);
    free(lens);
    free(w);
    return NULL;
}

void seq_send(const char *interface, pb_sequence_t seq, uint16_t seqc, struct cmd_line_af_xdp cmd)
{
    if (interface == NULL) /* sequence.c:715-720 */
    {
        fprintf(stderr, "Interface not set on sequence #%d. Not moving forward with this sequence.\n", seqc);
        return;
    }
    if (seq.ip.dst_ip == NULL) /* sequence.c:723-728 */
    {
        fprintf(stderr, "Destination IP not set on sequence #%d. Not moving forward with this sequence.\n", seqc);
        return;
    }
    if (seq_cnt >= PB_MAX_SEQUENCES)
        return;
    const int gpus = cmd.gpus > 0 ? cmd.gpus : 1;
    /* TX threads (sequence.c:741): the sequence's `threads`, else one per GPU */
    int t_cnt = seq.threads > 0 ? seq.threads : gpus;
    if (t_cnt > PB_MAX_WORKERS - worker_cnt)
        t_cnt = PB_MAX_WORKERS - worker_cnt;
    /* refusals come before the sequence takes a slot (its counters and totals line) */
    if (builder->device_count)
    {
        int n_dev = 0;
        if (builder->device_count(&n_dev) != 0)
            n_dev = 0;
        if (cmd.gpu_first < 0 || cmd.gpu_first + gpus > n_dev)
        {
            fprintf(stderr, "[%d] --gpus %d from --gpu %d needs GPUs %d..%d; %d present: %s.\n", seq_cnt + 1, gpus,
                    cmd.gpu_first, cmd.gpu_first, cmd.gpu_first + gpus - 1, n_dev, pbgpu_strerror(PBGPU_ENODEV));
            last_error = PBGPU_ENODEV;
            return;
        }
    }
    if (cmd.umem_slot && (cmd.umem_slot < 64 || cmd.umem_slot > PB_FRAME_SIZE || (cmd.umem_slot & (cmd.umem_slot - 1)) ||
                          (uint64_t)(cmd.umem_frames ? cmd.umem_frames : PB_NUM_FRAMES) * (PB_FRAME_SIZE / cmd.umem_slot) >
                              (1u << 22)))
    {
        fprintf(stderr, "[%d] --umemslot %u is not a power of two from 64 to %u giving at most 2^22 slots.\n",
                seq_cnt + 1, cmd.umem_slot, PB_FRAME_SIZE);
        last_error = PBGPU_EINVAL;
        return;
    }
    const uint16_t idx = seq_cnt++;
    start_time[idx] = time(NULL);
    shared_umem_t *shared = NULL;
    if (cmd.shared_umem && t_cnt > 0)
    {
        /* one UMEM for the sequence's threads (af_xdp.c:412-428), each its own power-of-two
         * slot range */
        const uint32_t umem_frames = cmd.umem_frames ? cmd.umem_frames : PB_NUM_FRAMES;
        const uint32_t slot_sz = cmd.umem_slot ? cmd.umem_slot : PB_FRAME_SIZE;
        const uint32_t umem_slots = umem_frames * (PB_FRAME_SIZE / slot_sz);
        uint32_t slots = umem_slots;
        while (slots > 1 && slots * (uint32_t)t_cnt > umem_slots)
            slots >>= 1;
        if (slots * (uint32_t)t_cnt > umem_slots)
        {
            fprintf(stderr, "[%d] Too many threads (%d) for one shared UMEM of %u slots.\n", idx + 1, t_cnt,
                    umem_slots);
            last_error = PBGPU_EINVAL;
            return;
        }
        shared = (shared_umem_t *)calloc(1, sizeof *shared);
        if (shared == NULL ||
            posix_memalign((void **)&shared->base, (size_t)sysconf(_SC_PAGESIZE),
                           (size_t)umem_frames * PB_FRAME_SIZE) != 0)
        {
            free(shared);
            last_error = PBGPU_ENOMEM;
            return;
        }
        memset(shared->base, 0, (size_t)umem_frames * PB_FRAME_SIZE);
        shared->slots = slots;
        /* --queue with several threads: every socket binds the owner's queue (af_xdp.c:443) and
         * they share its completion ring */
        if (cmd.queue_set && t_cnt > 1)
        {
            const int loop = !(cmd.tx && strcmp(cmd.tx, "xsk") == 0);
            const int src = pb_xsk_scq_init(&shared->scq, (uint32_t)t_cnt, slots, slot_sz, loop);
            if (src != 0)
            {
                free(shared->base);
                free(shared);
                last_error = src;
                return;
            }
            shared->one_queue = 1;
        }
        shared->fd = -1;
        shared->refs = 1; /* seq_send's own reference, dropped after the threads are started */
        pthread_mutex_init(&shared->mu, NULL);
        pthread_cond_init(&shared->cv, NULL);
        __atomic_add_fetch(&umem_allocs[idx], 1, __ATOMIC_RELAXED);
    }
    const int old = worker_cnt;
    for (int t = 0; t < t_cnt; ++t)
    {
        worker_arg_t *w = (worker_arg_t *)calloc(1, sizeof *w);
        if (w == NULL)
            break;
        w->seq = seq;
        w->device = interface;
        w->seq_idx = idx;
        w->gpu = cmd.gpu_first + t % gpus;
        w->shard = t;
        w->n_shards = t_cnt;
        w->cmd = cmd;
        w->shared = shared;
        if (shared)
        {
            pthread_mutex_lock(&shared->mu);
            ++shared->refs;
            pthread_mutex_unlock(&shared->mu);
        }
        if (pthread_create(&workers[worker_cnt], NULL, gpu_worker, w) != 0)
        {
            if (shared)
                shared_release(shared);
            free(w);
            break;
        }
        joined[worker_cnt] = 0;
        ++worker_cnt;
    }
    if (shared)
    {
        pthread_mutex_lock(&shared->mu);
        if (worker_cnt == old) /* no thread started: nobody will publish a socket */
            shared->fd = -2;
        pthread_cond_broadcast(&shared->cv);
        pthread_mutex_unlock(&shared->mu);
        shared_release(shared);
    }
    if (seq.block || seq_cnt >= seqc - 1) /* sequence.c:765, including its off-by-one (B10) */
        for (int i = old; i < worker_cnt; ++i)
        {
            pthread_join(workers[i], NULL);
            joined[i] = 1;
        }
}

int pb_shutdown_stats(pb_config_t *cfg)
{
    /* the reference cancels its threads (sequence.c:781-784); these stop after their
     * current batch, and each is joined exactly once */
    pb_request_stop();
    for (int i = 0; i < worker_cnt; ++i)
        if (!joined[i])
        {
            pthread_join(workers[i], NULL);
            joined[i] = 1;
        }
    fprintf(stdout, "Completed %d sequences!\n", seq_cnt);
    for (int i = 0; i < seq_cnt && cfg; ++i)
    {
        if (!cfg->seq[i].track)
            continue;
        if (end_time[i] < 1)
            end_time[i] = time(NULL);
        time_t secs = end_time[i] - start_time[i];
        if (secs < 1)
            secs = 1;
        const uint64_t p = total_pckts[i], b = total_bytes[i];
        fprintf(stdout,
                "[%d] Completed sequence with a total of %llu packets and %llu bytes. Average PPS => %llu. "
                "Average BPS => %llu. Total seconds => %ld.\n",
                i + 1, (unsigned long long)p, (unsigned long long)b, (unsigned long long)(p / secs),
                (unsigned long long)(b / secs), (long)secs);
    }
    fflush(stdout);
    return last_error;
}

void shutdown_prog(pb_config_t *cfg)
{
    const int err = pb_shutdown_stats(cfg);
    free(cfg);
    exit(err ? EXIT_FAILURE : EXIT_SUCCESS);
}

void pb_reset(void)
{
    pb_request_stop();
    for (int i = 0; i < worker_cnt; ++i)
        if (!joined[i])
            pthread_join(workers[i], NULL);
    worker_cnt = 0;
    seq_cnt = 0;
    last_error = 0;
    memset(total_pckts, 0, sizeof total_pckts);
    memset(total_bytes, 0, sizeof total_bytes);
    memset(claimed_frames, 0, sizeof claimed_frames);
    memset(tx_descs, 0, sizeof tx_descs);
    memset(tx_comps, 0, sizeof tx_comps);
    memset(tx_wakeups, 0, sizeof tx_wakeups);
    memset(umem_allocs, 0, sizeof umem_allocs);
    memset(start_time, 0, sizeof start_time);
    memset(end_time, 0, sizeof end_time);
    stop_requested = 0;
}

/* ---- pcap TX hook ---- */
struct pb_pcap
{
    FILE *fp;
    pthread_mutex_t mu;
};

pb_pcap_t *pb_pcap_open(const char *path)
{
    FILE *fp = fopen(path, "wb");
    if (fp == NULL)
        return NULL;
    const uint32_t hdr[6] = {0xA1B2C3D4u, 0x00040002u, 0, 0, 65535, 1}; /* v2.4, snaplen, LINKTYPE_ETHERNET */
    fwrite(hdr, sizeof hdr, 1, fp);
    pb_pcap_t *p = (pb_pcap_t *)calloc(1, sizeof *p);
    if (p == NULL)
    {
        fclose(fp);
        return NULL;
    }
    p->fp = fp;
    pthread_mutex_init(&p->mu, NULL);
    return p;
}

int pb_pcap_tx(void *vp, int thread_id, const uint8_t *frame, uint16_t len)
{
    (void)thread_id;
    pb_pcap_t *p = (pb_pcap_t *)vp;
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    const uint32_t rec[4] = {(uint32_t)ts.tv_sec, (uint32_t)(ts.tv_nsec / 1000), len, len};
    pthread_mutex_lock(&p->mu);
    const int ok = fwrite(rec, sizeof rec, 1, p->fp) == 1 && fwrite(frame, 1, len, p->fp) == len;
    pthread_mutex_unlock(&p->mu);
    return ok ? 0 : -1;
}

void pb_pcap_close(pb_pcap_t *p)
{
    if (p == NULL)
        return;
    fclose(p->fp);
    pthread_mutex_destroy(&p->mu);
    free(p);
}
