/*
 * pbgpu.h — C ABI of the MI355X packet-build library (libpbgpu.so).
 *
 * Drop-in seam: the reference builds one frame per loop iteration inside
 * thread_hdl() (src/sequence.c:433-602) and hands each one to
 * send_packet(xsk, thread_id, buffer, len, verbose) (src/af_xdp.h:59,
 * src/sequence.c:607).  This library replaces the build side of that seam:
 * a batch of iterations is built on the GPU into device-resident frames, then
 * landed in the (pinned) AF_XDP UMEM, after which the host fills TX
 * descriptors exactly as af_xdp.c:217-227 does.
 *
 * Conventions follow the reference's C code: plain C, int
 * returns (0 = ok, negative errno-style codes), pointer out-params for setup,
 * no exit(), diagnostics on stderr only when PBGPU_VERBOSE is set.
 *
 *   reference interface                         replaced / mirrored by
 *   ------------------------------------------  ----------------------------
 *   thread_hdl() prologue: MAC/proto parse,     pbgpu_load_sequence()
 *     template + payload prep (sequence.c:66-374)
 *   thread_hdl() hot loop body                  pbgpu_build()
 *     (sequence.c:433-602), one call per batch
 *   send_packet() memcpy into UMEM slot          pbgpu_copy_to_umem()
 *     (af_xdp.c:200-214)
 *   total_pckts/total_bytes __sync counters     pbgpu_counters()
 *     (sequence.c:12-14, 633-642)
 *   pthread fan-out, one socket per thread      one pbgpu_ctx per GPU
 *     (sequence.c:741-762)                        (packets sharded by index)
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "pb_config.h"

#ifdef __cplusplus
extern "C" {
#endif

/* error codes (negative errno values, as the reference reports errno) */
#define PBGPU_OK 0
#define PBGPU_ENOENT (-2)     /* sequence slot not loaded */
#define PBGPU_EIO (-5)        /* HIP runtime error */
#define PBGPU_ENOMEM (-12)
#define PBGPU_EINVAL (-22)    /* bad config (e.g. min > max, no dst_ip) */
#define PBGPU_ENOSPC (-28)    /* frames buffer too small */
#define PBGPU_ENODEV (-19)    /* no such GPU */
#define PBGPU_ENOTSUP (-95)   /* reserved: a valid config this build would not run on the GPU (none since round 2) */

typedef struct pbgpu_ctx pbgpu_ctx;

/* Device-resident output of one pbgpu_build() call.
 * Frame f (0 <= f < n_frames) occupies bytes
 *   [offset(f), offset(f) + len(f)) of `data`, packed back to back, where
 *   fixed_len > 0 : offset(f) = f * fixed_len, len(f) = fixed_len
 *   fixed_len == 0: offset(f) = offsets[f], len(f) = offsets[f+1] - offsets[f]
 * Frames are numbered iteration-major: f = (k - first_iter) * pl_cnt + i for
 * payload i of iteration k (the reference's inner loop, sequence.c:530).
 * Variable length: offsets[n_frames] (the total) is written by every build; the
 * packed-frame kernel writes the other offsets as 4-B low words plus one 8-B start
 * per workgroup region, and offsets[] is filled from them on first use —
 * pbgpu_copy_offsets(), pbgpu_copy_to_umem[_async]() — or by pbgpu_frames_offsets()
 * for a caller that reads offsets[] on the device itself. */
typedef struct pbgpu_frames
{
    uint8_t *data;          /* device pointer, capacity_bytes (16-B padded) */
    uint64_t *offsets;      /* device pointer, capacity_frames + 1 entries */
    void *reserved;         /* library-internal: the buffer's build-completion event */
    uint64_t *scan_tmp;     /* device scratch (length scan) */
    uint64_t capacity_frames;
    uint64_t capacity_bytes;

    /* filled by pbgpu_build() */
    uint16_t seq_idx;
    uint64_t first_iter;
    uint64_t n_frames;
    uint32_t fixed_len;     /* 0 -> variable length, see offsets */
    uint64_t total_bytes;   /* exact for fixed length; UINT64_MAX until
                               pbgpu_frames_total() for variable length */
} pbgpu_frames;

/* ---- context (one per GPU; not thread-safe within one ctx) ---- */
int pbgpu_open(int device, pbgpu_ctx **out);
void pbgpu_close(pbgpu_ctx *ctx);
const char *pbgpu_strerror(int err);
int pbgpu_device_count(int *n);

/* ---- setup: compile one sequence into its GPU template ----
 * src_mac / dst_mac: resolved MACs (the reference resolves missing ones with
 * get_src_mac_address / get_gw_mac, sequence.c:111-130); NULL -> parse
 * seq->eth strings, unset -> 00:00:00:00:00:00.
 * rules: NULL -> { PB_PAYLOAD_STREAM, PB_FOLD_FULL }. */
int pbgpu_load_sequence(pbgpu_ctx *ctx, uint16_t seq_idx, const pb_sequence_t *seq,
                        const uint8_t *src_mac, const uint8_t *dst_mac, const pb_rules_t *rules,
                        uint64_t seed_base);

/* Upper bounds of frames / bytes produced by n_iter iterations. */
int pbgpu_build_size(pbgpu_ctx *ctx, uint16_t seq_idx, uint64_t n_iter,
                     uint64_t *max_frames, uint64_t *max_bytes);

int pbgpu_frames_alloc(pbgpu_ctx *ctx, uint64_t capacity_frames, uint64_t capacity_bytes,
                       pbgpu_frames **out);
void pbgpu_frames_free(pbgpu_ctx *ctx, pbgpu_frames *frames);

/* ---- hot path: build iterations [first_iter, first_iter + n_iter) ----
 * Asynchronous on the context's stream.  Seeds: pb_config.h seed stream with
 * the seed_base given to pbgpu_load_sequence(). */
int pbgpu_build(pbgpu_ctx *ctx, uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter,
                pbgpu_frames *out);

/* Several sequences' builds at once: part i builds iterations [first_iter[i],
 * first_iter[i] + n_iter[i]) of sequence seq_idx[i] into outs[i], exactly as
 * pbgpu_build() would (same frames, offsets and counters).  The reference runs
 * its sequences side by side (sequence.c:741-762, one thread group per
 * sequence); configs[4]'s three (64-B UDP, 60-B TCP SYN, 98-B ICMP echo, each
 * into its own 4-KiB-aligned buffer) are built by one fused launch
 * (pb_batch_kernel), any other set by one launch per part (also when a part's
 * sequence was loaded with PBGPU_BATCH=0).  Every part's arguments are checked
 * first: on an error no part is built and the counters are unchanged. */
int pbgpu_build_batch(pbgpu_ctx *ctx, uint32_t n, const uint16_t *seq_idx, const uint64_t *first_iter,
                      const uint64_t *n_iter, pbgpu_frames *const *outs);

int pbgpu_sync(pbgpu_ctx *ctx);
int pbgpu_frames_total(pbgpu_ctx *ctx, pbgpu_frames *frames, uint64_t *total_bytes);
/* Fills offsets[0 .. n_frames) of a variable-length build (ordered on the context's
 * stream; a no-op when they are already there). */
int pbgpu_frames_offsets(pbgpu_ctx *ctx, pbgpu_frames *frames);

/* ---- landing: device -> host ---- */
int pbgpu_copy_packed(pbgpu_ctx *ctx, const pbgpu_frames *frames, void *host_dst,
                      uint64_t byte_offset, uint64_t nbytes);
int pbgpu_copy_offsets(pbgpu_ctx *ctx, const pbgpu_frames *frames, uint64_t *host_dst);
/* UMEM landing (af_xdp.c:200-214 geometry): frame first_frame + j lands at
 * umem + (first_slot + j) * slot_stride; lens_out[j] = its length.  `umem`
 * may be any host pointer; pbgpu_host_register() it first for full speed.
 * Nothing past a frame in its slot is written, except in a tight slot (fixed
 * length, slot_stride no longer than the frame rounded up to 64 B: 64-B slots
 * for 60- or 64-B frames), which registered UMEM receives whole, the bytes past
 * the frame unspecified: back-to-back slots then cross the host link as
 * contiguous writes.
 * Runs on the context's landing stream after the build of `frames` only, so a
 * build of another buffer queued meanwhile overlaps it (double buffering);
 * returns when the frames are in place.  A frame longer than slot_stride is
 * refused (-EINVAL). */
int pbgpu_copy_to_umem(pbgpu_ctx *ctx, const pbgpu_frames *frames, void *umem, uint32_t slot_stride,
                       uint32_t first_slot, uint64_t first_frame, uint32_t n, uint16_t *lens_out);
/* The same, asynchronous: returns once the landing is queued (registered UMEM;
 * unregistered memory lands synchronously).  lens_out must stay valid until
 * pbgpu_land_wait() returns for it: that call waits until at most `keep`
 * landings are still queued, oldest first, and fills their lens_out.
 * A later pbgpu_build() into the same frames buffer is ordered after the
 * landings queued from it (the build stream waits on the last one), so a
 * caller may rebuild a buffer without waiting; builds into other buffers
 * overlap the landing. */
int pbgpu_copy_to_umem_async(pbgpu_ctx *ctx, const pbgpu_frames *frames, void *umem, uint32_t slot_stride,
                             uint32_t first_slot, uint64_t first_frame, uint32_t n, uint16_t *lens_out);
int pbgpu_land_wait(pbgpu_ctx *ctx, uint32_t keep);
int pbgpu_host_register(pbgpu_ctx *ctx, void *ptr, size_t bytes);
int pbgpu_host_unregister(pbgpu_ctx *ctx, void *ptr);

/* ---- counters (sequence.c:12-14, 633-642): frames built / bytes stored per
 * sequence since open, recorded by the build kernels' workgroups as they finish
 * their share (a skipped or short build shows here) and folded into the totals
 * here, when a sequence's record ring fills and when its slot is reloaded;
 * multi-GPU callers all-reduce these over RCCL. ---- */
int pbgpu_counters(pbgpu_ctx *ctx, uint64_t *pckts, uint64_t *bytes, int n_seq);

/* ---- measurement ---- */
/* Device time of the frame-build kernels launched since the last call, from
 * HIP events on the ctx stream, and the launch count.  PBGPU_TIMING_LAUNCH
 * (default): an event pair around every launch, ms_total = the sum of the
 * kernels' durations.  PBGPU_TIMING_SPAN: one event before the first launch
 * after the last call and one at this call, ms_total = the span on the device
 * (launch gaps included).  Each timing event is a release to system scope that
 * writes back the L2's dirty lines: the per-launch pair costs ~9 us between
 * back-to-back 2-GiB launches, so a continuously sending caller
 * runs in span mode. */
#define PBGPU_TIMING_LAUNCH 0
#define PBGPU_TIMING_SPAN 1
int pbgpu_set_timing(pbgpu_ctx *ctx, int mode);
int pbgpu_kernel_time(pbgpu_ctx *ctx, double *ms_total, uint32_t *n_launches);
/* PBGPU_TIMING_LAUNCH only: each launch's own device time since the last call
 * (the first `cap` of them into ms_each, oldest first) and the launch count. */
int pbgpu_kernel_times(pbgpu_ctx *ctx, double *ms_each, uint32_t cap, uint32_t *n_launches);
/* Write-only roofline probe: `reps` launches (best of two trials) of each of
 * PBGPU_FILL_SHAPES fill shapes over `bytes` — 16-B stores per lane at 16 / 4 /
 * 8 KiB per workgroup, plain and non-temporal, workgroups per CU capped by LDS, linear or
 * XCD-contiguous workgroup regions,
 * and the runtime's hipMemsetD32Async (probes/wbench.hip found the fastest plain
 * fills).  pbgpu_fill_probe returns the fastest shape's mean
 * device time per launch; _ex returns every shape's and the fastest's index,
 * pbgpu_fill_shape_name names a shape. */
#define PBGPU_FILL_SHAPES 15
int pbgpu_fill_probe(pbgpu_ctx *ctx, uint64_t bytes, uint32_t reps, double *ms_per_launch);
int pbgpu_fill_probe_ex(pbgpu_ctx *ctx, uint64_t bytes, uint32_t reps, double *ms_per_shape, int *best_shape);
/* The same shapes over the caller's device buffer `dst` (e.g. a pbgpu_frames data buffer): the
 * write rate of each shape at that buffer's physical placement. */
int pbgpu_fill_probe_at(pbgpu_ctx *ctx, void *dst, uint64_t bytes, uint32_t reps, double *ms_per_shape);
const char *pbgpu_fill_shape_name(int shape);

/* Name of the frame-build kernel variant a loaded sequence launches
 * (as rocprofv3 reports it). */
int pbgpu_kernel_name(pbgpu_ctx *ctx, uint16_t seq_idx, char *buf, size_t n);

/* ABI self-description for FFI bindings: sizes / offsets of the structs above.
 * which: 0 sizeof(pb_sequence_t), 1 sizeof(pb_payload_opt_t), 2 sizeof(pbgpu_frames),
 *        3 offsetof(pb_sequence_t, ip.ranges), 4 offsetof(pb_sequence_t, pls),
 *        5 offsetof(pb_sequence_t, pl_cnt), 6 offsetof(pbgpu_frames, total_bytes);
 * returns 0 for an unknown index. */
size_t pbgpu_abi_size(int which);

#ifdef __cplusplus
}
#endif
