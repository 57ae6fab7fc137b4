/*
 * cmd_line.h — AF_XDP command-line surface of pcktbatch, extended with the
 * GPU options of this build.
 *
 * The first fields mirror the reference's struct cmd_line_af_xdp
 * (src/cmd_line.h:7-18) member for member, and parse_cmd_line_af_xdp() keeps
 * its getopt_long table (codes 1-7, src/cmd_line.c:3-13) and behaviour, so a
 * reference command line parses identically.  GPU options use codes >= 32.
 */
#pragma once

#include <stdint.h>

typedef struct cmd_line_af_xdp
{
    unsigned int queue_set : 1;
    int queue;

    unsigned int no_wake_up : 1;
    unsigned int shared_umem;
    unsigned short batch_size;
    unsigned int skb_mode : 1;
    unsigned int zero_copy : 1;
    unsigned int copy : 1;

    /* GPU options (this build) */
    int gpus;            /* --gpus N: GPUs per sequence (default 1) */
    int gpu_first;       /* --gpu I: first GPU index (default 0) */
    uint64_t gpu_batch;  /* --gpubatch K: iterations per GPU launch (default 1 << 20) */
    uint64_t seed_base;  /* --seed S: seed stream base (default 0x5EEDBA5E) */
    int literal_payload; /* --literal: reference's as-compiled payload loop (quirk B1) */
    int single_fold;     /* --singlefold: one-fold IPv4 checksum (quirk B6) */
    const char *pcap;    /* --pcap FILE: write built frames to a pcap file */
    const char *tx;      /* --tx xsk: AF_XDP sockets; otherwise the in-memory TX ring (xsk_ring.h) */
    int seed_set;        /* --seed given; otherwise pb_resolve_seed() draws seed_base per run */
    int very_random;     /* --veryrandom: draw it with getrandom() (VERY_RANDOM, sequence.h:36) */
    int batch_set;       /* --batchsize given: TX descriptors per reserve / submit (else one landed chunk) */
    uint32_t umem_frames; /* --umemframes N: UMEM slots per socket (NUM_FRAMES = 4096, af_xdp.h:23; a power of two) */
    uint32_t umem_slot;   /* --umemslot S: bytes per frame slot (FRAME_SIZE = 4096, af_xdp.h:24, when 0): the UMEM of
                             umem_frames 4-KiB chunks is cut into slots of S bytes (a power of two, 64..4096), so
                             S = 64 lands 64 frames per chunk, contiguously */
} cmd_line_af_xdp_t;

void parse_cmd_line_af_xdp(struct cmd_line_af_xdp *cmd_af_xdp, int argc, char **argv);
void cmd_line_af_xdp_defaults(struct cmd_line_af_xdp *cmd_af_xdp);

/* setup_af_xdp_variables() (af_xdp.c:289-365): the reference's verbose lines, and the
 * checks this build adds: --skb (SKB / generic XDP mode, xdp_flags = XDP_FLAGS_SKB_MODE)
 * runs the socket in copy mode, so --skb with --zerocopy is refused; --batchsize 0 is
 * refused; --umemframes must be a power of two in [64, 2^20], --umemslot 0 or a power of two in
 * [64, 4096] giving at most 2^22 slots.  Returns 0, or -EINVAL after
 * a message on stderr. */
int pb_af_xdp_setup(const struct cmd_line_af_xdp *cmd_af_xdp, int verbose);
/* bind flags of a socket (af_xdp.c:291-320): need-wakeup unless --nowakeup;
 * --zerocopy, else --copy or --skb -> XDP_COPY */
uint16_t pb_bind_flags(const struct cmd_line_af_xdp *cmd_af_xdp);
/* The seed stream's base: --seed S as given; otherwise drawn once per run, as the
 * reference draws each iteration's seed (sequence.c:434-441): CLOCK_BOOTTIME
 * nanoseconds, or getrandom() with --veryrandom.  Stores it in seed_base. */
uint64_t pb_resolve_seed(struct cmd_line_af_xdp *cmd_af_xdp);
