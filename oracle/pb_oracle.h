/*
 * pb_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the PB-AF-XDP per-packet build path, used as the parity
 * checker for the HIP kernels (tests/, __graft_entry__.smoke(), and the
 * cpu_baseline leg of bench.py).  Nothing in the product links or calls it.
 *
 * Parity status:
 *   pinned  : glibc rand_r (tests compare against the host libc); the UDP
 *             checksum composition and the IPv4 header checksum (the two
 *             known-answer frames of images/test1.gif, README.md:23 —
 *             transcribed in SURVEY.md Appendix C, fixtures under tests/golden);
 *             rand_num's form min + rand_r % (max - min + 1), which sets TTL,
 *             ID, range index, ports and payload length (the consecutive-second
 *             source ports of images/test1.gif and test2.gif,
 *             tests/golden/kat_gif_ports.json).
 *   UNPINNED: rand_ip's host-bit rule, the TCP/ICMP
 *             checksum composition, the IPv4 single- vs full-fold edge case,
 *             UDP 0-checksum mapping.  These live in the un-vendored PB-Common
 *             submodule (modules/common is empty in /root/reference); the
 *             oracle follows the declared rules of SURVEY.md Appendix A/B.
 */
#pragma once

#include <stdint.h>

#include "../include/pb_config.h"

#ifdef __cplusplus
extern "C" {
#endif

/* glibc rand_r restated (3-step LCG, 31-bit output). */
int pbo_rand_r(unsigned int *seed);
/* PB-Common rand_num(min, max, seed) with the seed by value (pinned, see .c). */
int pbo_rand_num(int min, int max, unsigned int seed);

/* Per-iteration seed stream (pb_config.h). */
uint32_t pbo_seed(uint64_t seed_base, uint16_t seq_idx, uint64_t k);

/* Number of frames one iteration emits (= max(pl_cnt, 1)). */
int pbo_frames_per_iter(const pb_sequence_t *seq);

/* Build frames for iterations [first_iter, first_iter + n_iter) of one
 * sequence.
 *   smac/dmac  resolved MACs, or NULL to parse seq->eth strings
 *   faithful   1: per-iteration clock_gettime + rand_ip dotted-string
 *              round trip as in sequence.c:434-497; 0: integer-only
 *   slot_stride 0: frames packed back-to-back in `out`, offsets[] filled
 *              (n_frames + 1 entries, may be NULL);  >0: frame f lands at
 *              out + f * slot_stride (the AF_XDP UMEM geometry, af_xdp.c:211-214)
 * Returns 0 or a negative error. */
int pbo_build(const pb_sequence_t *seq, const uint8_t *smac, const uint8_t *dmac,
              uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter, uint64_t seed_base,
              const pb_rules_t *rules, int faithful,
              uint8_t *out, uint64_t out_cap, uint32_t slot_stride,
              uint64_t *offsets, uint64_t *n_frames, uint64_t *total_bytes);

/* Same, split over `nthreads` pthreads (contiguous iteration ranges, one
 * private frame buffer per thread — the reference's thread fan-out,
 * sequence.c:741-762).  Slot mode only (slot_stride > 0).  ring_slots > 0:
 * thread t owns its own UMEM of ring_slots slots at out + t * ring_slots *
 * slot_stride and reuses them round-robin (NUM_FRAMES per socket,
 * af_xdp.h:23, af_xdp.c:200-214); 0: frame f lands in slot f. */
int pbo_build_mt(const pb_sequence_t *seq, const uint8_t *smac, const uint8_t *dmac,
                 uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter, uint64_t seed_base,
                 const pb_rules_t *rules, int faithful, int nthreads,
                 uint8_t *out, uint64_t out_cap, uint32_t slot_stride, uint32_t ring_slots,
                 uint64_t *total_bytes);

/* Checksum helpers restated from the expected PB-Common csum.h semantics;
 * exported so tests can pin them against the known-answer frames. */
uint16_t pbo_iph_csum(const uint8_t *iph20, int single_fold);
uint16_t pbo_l4_csum(const uint8_t *l4, uint32_t len, uint32_t saddr_be, uint32_t daddr_be, uint8_t proto);

/* Checker: the number of frames whose IPv4 checksum, tot_len or L4 checksum does not
 * verify.  Frame i is data[offsets[i] - offsets[0], offsets[i + 1] - offsets[0]), or
 * fixed_len bytes at i * fixed_len when offsets is NULL. */
uint64_t pbo_verify_frames(const uint8_t *data, const uint64_t *offsets, uint32_t fixed_len, uint64_t n,
                           int nthreads);

#ifdef __cplusplus
}
#endif
