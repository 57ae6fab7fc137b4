/*
 * cmd_line.c — AF_XDP + GPU command-line parsing (see cmd_line.h).
 * Reference behaviour kept: getopt_long with no short options, codes 1-7 for
 * queue / nowakeup / sharedumem / batchsize / skb / zerocopy / copy, values
 * through atoi (src/cmd_line.c:24-69); unknown options are skipped silently
 * (main.c sets opterr = 0 before the passes).
 */
#define _GNU_SOURCE
#include "cmd_line.h"

#include <errno.h>
#include <getopt.h>
#include <linux/if_xdp.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/random.h>
#include <time.h>

enum
{
    OPT_QUEUE = 1,
    OPT_NOWAKEUP,
    OPT_SHAREDUMEM,
    OPT_BATCHSIZE,
    OPT_SKB,
    OPT_ZEROCOPY,
    OPT_COPY,
    OPT_GPUS = 32,
    OPT_GPU,
    OPT_GPUBATCH,
    OPT_SEED,
    OPT_LITERAL,
    OPT_SINGLEFOLD,
    OPT_PCAP,
    OPT_TX,
    OPT_VERYRANDOM,
    OPT_UMEMFRAMES,
    OPT_UMEMSLOT,
};

static const struct option af_xdp_opts[] = {
    {"queue", required_argument, NULL, OPT_QUEUE},
    {"nowakeup", no_argument, NULL, OPT_NOWAKEUP},
    {"sharedumem", no_argument, NULL, OPT_SHAREDUMEM},
    {"batchsize", required_argument, NULL, OPT_BATCHSIZE},
    {"skb", no_argument, NULL, OPT_SKB},
    {"zerocopy", no_argument, NULL, OPT_ZEROCOPY},
    {"copy", no_argument, NULL, OPT_COPY},
    {"gpus", required_argument, NULL, OPT_GPUS},
    {"gpu", required_argument, NULL, OPT_GPU},
    {"gpubatch", required_argument, NULL, OPT_GPUBATCH},
    {"seed", required_argument, NULL, OPT_SEED},
    {"literal", no_argument, NULL, OPT_LITERAL},
    {"singlefold", no_argument, NULL, OPT_SINGLEFOLD},
    {"pcap", required_argument, NULL, OPT_PCAP},
    {"tx", required_argument, NULL, OPT_TX},
    {"veryrandom", no_argument, NULL, OPT_VERYRANDOM},
    {"umemframes", required_argument, NULL, OPT_UMEMFRAMES},
    {"umemslot", required_argument, NULL, OPT_UMEMSLOT},
    {NULL, 0, NULL, 0},
};

void cmd_line_af_xdp_defaults(struct cmd_line_af_xdp *c)
{
    c->batch_size = 1; /* main.c:45-46 */
    c->gpus = 1;
    c->gpu_first = 0;
    c->gpu_batch = 1u << 20;
    c->seed_base = 0x5EEDBA5Eull;
    c->umem_frames = 4096; /* NUM_FRAMES, af_xdp.h:23 */
}

void parse_cmd_line_af_xdp(struct cmd_line_af_xdp *c, int argc, char **argv)
{
    int opt;
    while ((opt = getopt_long(argc, argv, "", af_xdp_opts, NULL)) != -1)
    {
        switch (opt)
        {
        case OPT_QUEUE:
            c->queue_set = 1;
            c->queue = atoi(optarg);
            break;
        case OPT_NOWAKEUP:
            c->no_wake_up = 1;
            break;
        case OPT_SHAREDUMEM:
            c->shared_umem = 1;
            break;
        case OPT_BATCHSIZE:
            c->batch_size = (unsigned short)atoi(optarg);
            c->batch_set = 1;
            break;
        case OPT_SKB:
            c->skb_mode = 1;
            break;
        case OPT_ZEROCOPY:
            c->zero_copy = 1;
            break;
        case OPT_COPY:
            c->copy = 1;
            break;
        case OPT_GPUS:
            c->gpus = atoi(optarg);
            break;
        case OPT_GPU:
            c->gpu_first = atoi(optarg);
            break;
        case OPT_GPUBATCH:
            c->gpu_batch = strtoull(optarg, NULL, 0);
            break;
        case OPT_SEED:
            c->seed_base = strtoull(optarg, NULL, 0);
            c->seed_set = 1;
            break;
        case OPT_LITERAL:
            c->literal_payload = 1;
            break;
        case OPT_SINGLEFOLD:
            c->single_fold = 1;
            break;
        case OPT_PCAP:
            c->pcap = optarg;
            break;
        case OPT_TX:
            c->tx = optarg;
            break;
        case OPT_VERYRANDOM:
            c->very_random = 1;
            break;
        case OPT_UMEMFRAMES:
            c->umem_frames = (uint32_t)strtoul(optarg, NULL, 0);
            break;
        case OPT_UMEMSLOT:
            c->umem_slot = (uint32_t)strtoul(optarg, NULL, 0);
            break;
        default:
            break;
        }
    }
}

int pb_af_xdp_setup(const struct cmd_line_af_xdp *c, int verbose)
{
    if (c->skb_mode && c->zero_copy)
    {
        fprintf(stderr, "--skb and --zerocopy cannot be combined: SKB (generic XDP) mode sends in copy mode.\n");
        return -EINVAL;
    }
    if (c->umem_frames < 64 || c->umem_frames > (1u << 20) || (c->umem_frames & (c->umem_frames - 1)))
    {
        fprintf(stderr, "--umemframes must be a power of two from 64 to 1048576.\n");
        return -EINVAL;
    }
    if (c->umem_slot &&
        (c->umem_slot < 64 || c->umem_slot > 4096 || (c->umem_slot & (c->umem_slot - 1)) ||
         (uint64_t)c->umem_frames * (4096u / c->umem_slot) > (1u << 22)))
    {
        fprintf(stderr, "--umemslot must be a power of two from 64 to 4096, at most 2^22 slots per UMEM.\n");
        return -EINVAL;
    }
    if (c->batch_set && c->batch_size == 0)
    {
        fprintf(stderr, "--batchsize must be at least 1.\n");
        return -EINVAL;
    }
    if (!verbose)
        return 0;
    /* af_xdp.c:291-364, line for line */
    if (c->zero_copy)
        fprintf(stdout, "Running AF_XDP sockets in zero-copy mode.\n");
    else if (c->copy)
        fprintf(stdout, "Running AF_XDP sockets in copy mode.\n");
    if (c->no_wake_up)
        fprintf(stdout, "Running AF_XDP sockets in no wake-up mode.\n");
    if (c->queue_set)
        fprintf(stdout, "Running AF_XDP sockets with one queue ID => %d.\n", c->queue);
    if (c->shared_umem)
        fprintf(stdout, "Running AF_XDP sockets with shared UMEM mode.\n");
    if (c->skb_mode)
        fprintf(stdout, "Running AF_XDP sockets in SKB mode.\n");
    fprintf(stdout, "Running AF_XDP sockets with batch size => %d.\n", c->batch_size);
    return 0;
}

uint16_t pb_bind_flags(const struct cmd_line_af_xdp *c)
{
    uint16_t bf = c->no_wake_up ? 0 : XDP_USE_NEED_WAKEUP;
    if (c->zero_copy)
        bf |= XDP_ZEROCOPY;
    else if (c->copy || c->skb_mode) /* generic (SKB) XDP has no zero-copy path */
        bf |= XDP_COPY;
    return bf;
}

uint64_t pb_resolve_seed(struct cmd_line_af_xdp *c)
{
    if (c->seed_set)
        return c->seed_base;
    uint64_t s = 0;
    if (c->very_random && getrandom(&s, sizeof s, 0) == (ssize_t)sizeof s)
    {
        c->seed_base = s;
        return s;
    }
    struct timespec ts;
    clock_gettime(CLOCK_BOOTTIME, &ts);
    s = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
    c->seed_base = s;
    return s;
}
