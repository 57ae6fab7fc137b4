/*
 * sequence_gpu.c — seq_send() / shutdown_prog() over libpbgpu (see .h).
 *
 * Per sequence: one worker pthread per GPU.  GPU g of n builds iterations
 * [k, k + batch) with k = (step * n + g) * batch, lands the frames in its own
 * UMEM (NUM_FRAMES x FRAME_SIZE, page-aligned and HIP-registered like the
 * reference's posix_memalign'd UMEM, af_xdp.c:374-389) and calls the TX hook
 * per frame.  Counters follow sequence.c:633-653; the stop conditions
 * (max_pckts, max_bytes, time, sequence.c:662-684) and pacing (pps, bps,
 * delay, sequence.c:389-431, 655-659) are applied per launch.
 */
#define _GNU_SOURCE
#include "sequence_gpu.h"
#include "mac.h"

#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#define PB_MAX_WORKERS 64

static uint64_t total_pckts[PB_MAX_SEQUENCES];
static uint64_t total_bytes[PB_MAX_SEQUENCES];
static time_t start_time[PB_MAX_SEQUENCES];
static time_t end_time[PB_MAX_SEQUENCES];
static uint16_t seq_cnt;
static pthread_t workers[PB_MAX_SEQUENCES * 8];
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

typedef struct worker_arg
{
    pb_sequence_t seq;
    const char *device; /* the interface seq_send() was given (MAC discovery) */
    uint16_t seq_idx;
    int gpu;
    int shard;
    int n_shards;
    struct cmd_line_af_xdp cmd;
} worker_arg_t;

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

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *gpu_worker(void *p)
{
    worker_arg_t *w = (worker_arg_t *)p;
    const pb_sequence_t *seq = &w->seq;
    const int seq_num = w->seq_idx + 1;
    pbgpu_ctx *ctx = NULL;
    pbgpu_frames *fr = NULL;
    uint8_t *umem = NULL;
    uint16_t lens[PB_NUM_FRAMES];
    int rc;

    if ((rc = pbgpu_open(w->gpu, &ctx)) != 0)
    {
        fprintf(stderr, "[%d] Error opening GPU %d :: %s.\n", seq_num, w->gpu, pbgpu_strerror(rc));
        last_error = rc;
        goto out;
    }
    /* a continuous sender never reads per-launch timings: no event pair per batch */
    (void)pbgpu_set_timing(ctx, PBGPU_TIMING_SPAN);
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
    if ((rc = pbgpu_load_sequence(ctx, w->seq_idx, seq, smac, dmac, &rules, w->cmd.seed_base)) != 0)
    {
        fprintf(stderr, "[%d] Error loading sequence on GPU %d :: %s.\n", seq_num, w->gpu, pbgpu_strerror(rc));
        last_error = rc;
        goto out;
    }
    const uint64_t batch = w->cmd.gpu_batch ? w->cmd.gpu_batch : (1u << 20);
    uint64_t mf = 0, mb = 0;
    if ((rc = pbgpu_build_size(ctx, w->seq_idx, batch, &mf, &mb)) != 0 ||
        (rc = pbgpu_frames_alloc(ctx, mf, mb, &fr)) != 0)
    {
        last_error = rc;
        goto out;
    }
    if (posix_memalign((void **)&umem, (size_t)sysconf(_SC_PAGESIZE), (size_t)PB_NUM_FRAMES * PB_FRAME_SIZE) != 0)
    {
        last_error = PBGPU_ENOMEM;
        goto out;
    }
    memset(umem, 0, (size_t)PB_NUM_FRAMES * PB_FRAME_SIZE);
    pbgpu_host_register(ctx, umem, (size_t)PB_NUM_FRAMES * PB_FRAME_SIZE);

    const double t0 = now_s();
    const int fpi = seq->pl_cnt < 1 ? 1 : seq->pl_cnt;
    for (uint64_t step = 0; !stop_requested; ++step)
    {
        uint64_t n_iter = batch;
        if (seq->max_pckts > 0) /* launch-level quota of the global counter */
        {
            uint64_t done = __atomic_load_n(&total_pckts[w->seq_idx], __ATOMIC_RELAXED);
            if (done >= seq->max_pckts)
                break;
            uint64_t left = (seq->max_pckts - done + fpi - 1) / fpi;
            left = (left + w->n_shards - 1) / w->n_shards;
            if (left < n_iter)
                n_iter = left;
        }
        const uint64_t k = (step * (uint64_t)w->n_shards + (uint64_t)w->shard) * batch;
        if ((rc = pbgpu_build(ctx, w->seq_idx, k, n_iter, fr)) != 0)
        {
            fprintf(stderr, "[%d] Error building frames on GPU %d :: %s.\n", seq_num, w->gpu, pbgpu_strerror(rc));
            last_error = rc;
            break;
        }
        uint64_t bytes = 0;
        for (uint64_t f0 = 0; f0 < fr->n_frames; f0 += PB_NUM_FRAMES)
        {
            const uint32_t n = (uint32_t)(fr->n_frames - f0 < PB_NUM_FRAMES ? fr->n_frames - f0 : PB_NUM_FRAMES);
            if ((rc = pbgpu_copy_to_umem(ctx, fr, umem, PB_FRAME_SIZE, 0, f0, n, lens)) != 0)
            {
                last_error = rc;
                goto out;
            }
            for (uint32_t i = 0; i < n; ++i)
            {
                bytes += lens[i];
                if (tx_hook && tx_hook(tx_ctx, w->shard, umem + (size_t)i * PB_FRAME_SIZE, lens[i]) != 0)
                    fprintf(stderr, "[%d][%d] ERROR - Could not send packet (%d) :: %s.\n", seq_num, i + 1, w->shard,
                            strerror(errno));
            }
        }
        __atomic_add_fetch(&total_pckts[w->seq_idx], fr->n_frames, __ATOMIC_RELAXED);
        __atomic_add_fetch(&total_bytes[w->seq_idx], bytes, __ATOMIC_RELAXED);
        if (verbose)
            fprintf(stdout, "[%d] GPU %d built %llu frames (%llu bytes) from iteration %llu.\n", seq_num, w->gpu,
                    (unsigned long long)fr->n_frames, (unsigned long long)bytes, (unsigned long long)k);

        /* pacing at launch granularity (sequence.c:389-431, 655-659) */
        const double el = now_s() - t0;
        double want = 0;
        const double frames = (double)__atomic_load_n(&total_pckts[w->seq_idx], __ATOMIC_RELAXED) / w->n_shards;
        if (seq->pps > 0)
            want = frames / (double)seq->pps;
        if (seq->bps > 0)
        {
            const double b = (double)__atomic_load_n(&total_bytes[w->seq_idx], __ATOMIC_RELAXED) / w->n_shards;
            const double wb = b / (double)seq->bps;
            want = wb > want ? wb : want;
        }
        if (seq->delay > 0)
        {
            const double wd = frames * (double)seq->delay * 1e-6;
            want = wd > want ? wd : want;
        }
        if (want > el)
            usleep((useconds_t)((want - el) * 1e6));

        if (seq->max_pckts > 0 && __atomic_load_n(&total_pckts[w->seq_idx], __ATOMIC_RELAXED) >= seq->max_pckts)
        {
            fprintf(stdout, "[%d] Max packets exceeded for sequence. Stopping...\n", seq_num);
            break;
        }
        if (seq->max_bytes > 0 && __atomic_load_n(&total_bytes[w->seq_idx], __ATOMIC_RELAXED) >= seq->max_bytes)
        {
            fprintf(stdout, "[%d] Max bytes exceeded for sequence. Stopping...\n", seq_num);
            break;
        }
        if (seq->time > 0 && now_s() - t0 >= (double)seq->time)
        {
            fprintf(stdout, "[%d] Time exceeded for sequence. Stopping...\n", seq_num);
            break;
        }
    }
out:
    end_time[w->seq_idx] = time(NULL);
    if (umem)
    {
        if (ctx)
            pbgpu_host_unregister(ctx, umem);
        free(umem);
    }
    if (fr)
        pbgpu_frames_free(ctx, fr);
    pbgpu_close(ctx);
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
    const uint16_t idx = seq_cnt++;
    int n = cmd.gpus > 0 ? cmd.gpus : 1;
    if (n > PB_MAX_WORKERS)
        n = PB_MAX_WORKERS;
    start_time[idx] = time(NULL);
    const int old = worker_cnt;
    for (int g = 0; g < n; ++g)
    {
        worker_arg_t *w = (worker_arg_t *)calloc(1, sizeof *w);
        if (w == NULL)
            break;
        w->seq = seq;
        w->device = interface;
        w->seq_idx = idx;
        w->gpu = cmd.gpu_first + g;
        w->shard = g;
        w->n_shards = n;
        w->cmd = cmd;
        if (pthread_create(&workers[worker_cnt], NULL, gpu_worker, w) != 0)
        {
            free(w);
            break;
        }
        ++worker_cnt;
    }
    if (seq.block || seq_cnt >= seqc - 1) /* sequence.c:765, including its off-by-one (B10) */
        for (int i = old; i < worker_cnt; ++i)
            pthread_join(workers[i], NULL);
}

void shutdown_prog(pb_config_t *cfg, int exit_prog)
{
    for (int i = 0; i < worker_cnt; ++i)
        pthread_join(workers[i], NULL);
    worker_cnt = 0;
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
    if (exit_prog)
        exit(last_error ? EXIT_FAILURE : EXIT_SUCCESS);
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
