/*
 * sequence_gpu.h — the reference's sequence surface (src/sequence.h:52-53)
 * driven by the MI355X build.
 *
 * seq_send() starts the sequence's TX threads — `threads` of them as in the
 * reference (sequence.c:741; 0 = one per GPU here, where the reference takes
 * get_nprocs()), spread round robin over --gpus GPUs.  Thread t owns a UMEM of
 * NUM_FRAMES x FRAME_SIZE slots (af_xdp.h:23-24; with --sharedumem its own
 * power-of-two slot range of one UMEM per sequence), a TX ring + completion ring
 * (an AF_XDP socket on queue t, or the in-memory loopback), and shard t of the
 * iteration space.  It builds batches of iterations with pbgpu_build() into two
 * device buffers alternately — batch n + 1 builds on the GPU while batch n is
 * landed in the UMEM slots and its TX descriptors are filled and submitted,
 * completions reaped as send_packet()/complete_tx() do (af_xdp.c:25-53,
 * 178-241).
 *
 * Differences from the reference prototypes (sequence.h:52-53), kept because
 * PB-Common's headers are not in the reference snapshot: the sequence and
 * config types are this build's mirrors (include/pb_config.h), and seq_send's
 * last argument is the AF_XDP + GPU command line (struct cmd_line_af_xdp)
 * where the reference passes PB-Common's struct cmd_line.
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "../../include/pb_config.h"
#include "../../include/pbgpu.h"
#include "cmd_line.h"

#define PB_NUM_FRAMES 4096 /* af_xdp.h:23 */
#define PB_FRAME_SIZE 4096 /* af_xdp.h:24, XSK_UMEM__DEFAULT_FRAME_SIZE */

/* Called for every frame the TX side consumes (loopback / pcap backends), in
 * send order; a nonzero return is reported on stderr and the loop continues
 * (sequence.c:607-610). */
typedef int (*pb_tx_fn)(void *tx_ctx, int thread_id, const uint8_t *frame, uint16_t len);

void pb_set_tx_hook(pb_tx_fn fn, void *tx_ctx);
void pb_request_stop(void); /* async-signal-safe: workers stop after their current batch */
int pb_stop_requested(void);
void pb_set_verbose(int verbose);

void seq_send(const char *interface, pb_sequence_t seq, uint16_t seqc, struct cmd_line_af_xdp cmd);
/* sequence.c:779-824: stop and join the workers, print the end-of-run lines,
 * free cfg, exit(). */
void shutdown_prog(pb_config_t *cfg);
/* The same without freeing cfg or exiting (library / test use); returns the
 * last worker error (0 = none). */
int pb_shutdown_stats(pb_config_t *cfg);

int pb_sequence_totals(uint16_t seq, uint64_t *pckts, uint64_t *bytes);
int pb_last_error(void);
/* Forget all sequences, totals and errors (tests run several programs' worth
 * of sequences in one process). */
void pb_reset(void);

/* TX descriptor / wakeup / completion counts summed over the finished workers
 * of a sequence (the ring protocol's own accounting). */
int pb_sequence_tx_stats(uint16_t seq, uint64_t *descs, uint64_t *completions, uint64_t *wakeups);
/* UMEMs allocated for a sequence: one per thread, or one in all with --sharedumem. */
int pb_sequence_umems(uint16_t seq, uint64_t *umems);

/* ---- the frame builder behind the workers ----
 * Default: libpbgpu (pbgpu_open / _load_sequence / _build / _copy_to_umem).
 * The table exists so host-side tests can run the worker loop (quotas, pacing,
 * stop conditions, rings) on a CPU without a GPU by installing their own. */
typedef struct pb_builder
{
    int (*open)(int gpu, void **h);
    int (*load)(void *h, uint16_t seq_idx, const pb_sequence_t *seq, const uint8_t *smac, const uint8_t *dmac,
                const pb_rules_t *rules, uint64_t seed_base);
    int (*alloc)(void *h, uint16_t seq_idx, uint64_t n_iter, void **frames);
    /* asynchronous; the frames are ready for land() */
    int (*build)(void *h, uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter, void *frames);
    uint64_t (*n_frames)(void *frames);
    /* queue frames [first, first + n) -> slots first_slot.. of `umem` (stride bytes apart),
     * lengths to lens once land_wait(keep) has left at most `keep` landings queued */
    int (*land)(void *h, void *frames, uint8_t *umem, uint32_t stride, uint32_t first_slot, uint64_t first,
                uint32_t n, uint16_t *lens);
    int (*land_wait)(void *h, uint32_t keep);
    int (*host_register)(void *h, void *p, size_t n);
    int (*host_unregister)(void *h, void *p);
    void (*free_frames)(void *h, void *frames);
    void (*close)(void *h);
    /* GPUs present (pbgpu_device_count); NULL: not checked.  seq_send refuses a --gpu / --gpus
     * range past it before starting any thread. */
    int (*device_count)(int *n);
} pb_builder_t;

void pb_set_builder(const pb_builder_t *b); /* NULL: libpbgpu */

/* pcap (LINKTYPE_ETHERNET) TX hook */
typedef struct pb_pcap pb_pcap_t;
pb_pcap_t *pb_pcap_open(const char *path);
int pb_pcap_tx(void *pcap, int thread_id, const uint8_t *frame, uint16_t len);
void pb_pcap_close(pb_pcap_t *p);
