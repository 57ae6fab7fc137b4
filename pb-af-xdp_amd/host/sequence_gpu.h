/*
 * sequence_gpu.h — the reference's sequence surface (src/sequence.h:52-53)
 * driven by the MI355X build: seq_send() fans a sequence out over GPUs (the
 * reference fans out over pthreads / AF_XDP queues, sequence.c:741-762), each
 * GPU builds batches of iterations with pbgpu_build(), lands them in a UMEM of
 * NUM_FRAMES x FRAME_SIZE slots (af_xdp.h:23-24) and hands every frame to the
 * TX hook — the place of send_packet() (af_xdp.h:59, sequence.c:607).
 */
#pragma once

#include <stdint.h>

#include "../../include/pb_config.h"
#include "../../include/pbgpu.h"
#include "cmd_line.h"

#define PB_NUM_FRAMES 4096 /* af_xdp.h:23 */
#define PB_FRAME_SIZE 4096 /* af_xdp.h:24, XSK_UMEM__DEFAULT_FRAME_SIZE */

/* Called for every frame once it sits in its UMEM slot; return 0 on success
 * (a failure is reported on stderr and the loop continues, sequence.c:607-610). */
typedef int (*pb_tx_fn)(void *tx_ctx, int thread_id, const uint8_t *frame, uint16_t len);

void pb_set_tx_hook(pb_tx_fn fn, void *tx_ctx);
void pb_request_stop(void); /* async-signal-safe: workers stop after their current launch */
void pb_set_verbose(int verbose);

void seq_send(const char *interface, pb_sequence_t seq, uint16_t seqc, struct cmd_line_af_xdp cmd);
/* Prints the reference's end-of-run lines (sequence.c:786-815); exit_prog != 0
 * exits like the reference does, 0 returns (library / test use). */
void shutdown_prog(pb_config_t *cfg, int exit_prog);

int pb_sequence_totals(uint16_t seq, uint64_t *pckts, uint64_t *bytes);
int pb_last_error(void);

/* pcap (LINKTYPE_ETHERNET) TX hook */
typedef struct pb_pcap pb_pcap_t;
pb_pcap_t *pb_pcap_open(const char *path);
int pb_pcap_tx(void *pcap, int thread_id, const uint8_t *frame, uint16_t len);
void pb_pcap_close(pb_pcap_t *p);
