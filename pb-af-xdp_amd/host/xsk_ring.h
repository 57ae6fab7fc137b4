/*
 * xsk_ring.h — AF_XDP TX side without libbpf: the single-producer TX ring and
 * single-consumer completion ring of linux/if_xdp.h, the UMEM slot ring, and
 * the socket setup, in this build's own C.
 *
 * Replaces what the reference gets from libbpf's xsk.h (un-vendored,
 * modules/libbpf) and does in src/af_xdp.c:
 *   xsk_ring_prod__reserve / __tx_desc / __submit    af_xdp.c:184-230 (send_packet)
 *   xsk_ring_cons__peek / __release, sendto wakeup   af_xdp.c:25-53   (complete_tx)
 *   posix_memalign UMEM, xsk_umem__create            af_xdp.c:374-389, 63-92
 *   xsk_socket__create (TX ring only), bind flags    af_xdp.c:103-165, 289-365
 * Ring protocol (the kernel's, as libbpf implements it): the producer owns
 * `producer`, the consumer owns `consumer`; entries are indices masked by
 * size - 1; a producer publishes entries with a release store of the
 * producer index after writing them, a consumer reads them after an acquire
 * load of it, and vice versa for the consumer index.
 *
 * Two backends share the ring code:
 *   - an AF_XDP socket (pb_xsk_open) when the kernel and privileges allow it;
 *   - a loopback pair in ordinary memory (pb_xsk_loopback), whose "kernel"
 *     side (pb_xsk_loop_consume) moves TX descriptors to the completion ring —
 *     the in-memory ring the unit tests drive and `--tx null` sends into.
 */
#pragma once

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

#include <linux/if_xdp.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pb_xsk_ring
{
    uint32_t cached_prod;
    uint32_t cached_cons;
    uint32_t mask;
    uint32_t size;
    uint32_t *producer;
    uint32_t *consumer;
    uint32_t *flags;
    void *ring; /* struct xdp_desc[] (TX) or uint64_t[] (completion) */
} pb_xsk_ring_t;

/* ---- producer (TX ring) ---- */
/* Reserve nb entries; returns nb and the first index, or 0 if the ring has fewer free. */
uint32_t pb_ring_prod_reserve(pb_xsk_ring_t *r, uint32_t nb, uint32_t *idx);
struct xdp_desc *pb_ring_tx_desc(pb_xsk_ring_t *r, uint32_t idx);
void pb_ring_prod_submit(pb_xsk_ring_t *r, uint32_t nb);
int pb_ring_needs_wakeup(const pb_xsk_ring_t *r);
uint32_t pb_ring_prod_free(pb_xsk_ring_t *r);

/* ---- consumer (completion ring) ---- */
uint32_t pb_ring_cons_peek(pb_xsk_ring_t *r, uint32_t nb, uint32_t *idx);
uint64_t pb_ring_comp_addr(const pb_xsk_ring_t *r, uint32_t idx);
void pb_ring_cons_release(pb_xsk_ring_t *r, uint32_t nb);

/* ---- --sharedumem with every socket on one queue (af_xdp.c:412-443) ----
 * The kernel binds a second socket of a UMEM to the owner's (device, queue) only on the owner's
 * fill and completion rings (libbpf's xsk_socket__create_shared on the same queue): every
 * socket's TX completions arrive on the owner's one completion ring.  Whichever thread reaps it
 * does so under `mu` and credits each completion to the thread whose slot range holds its
 * address; a thread takes its credits when it reaps. */
#define PB_XSK_MAX_SHARERS 256
typedef struct pb_xsk_shared_cq
{
    pthread_mutex_t mu;
    pb_xsk_ring_t cq;      /* the owner's completion ring (socket: its mapping; loopback: `mem`) */
    uint32_t slots;        /* UMEM slots per thread (thread t: [t * slots, (t + 1) * slots)) */
    uint32_t frame_size;
    uint32_t n_threads;
    uint32_t credit[PB_XSK_MAX_SHARERS]; /* per thread: completions reaped for it, not yet taken */
    void *mem;             /* loopback: the ring's backing memory */
    uint64_t reaped;       /* completions taken off the ring, all threads */
} pb_xsk_shared_cq_t;

/* Set up q for n_threads threads of `slots` slots of frame_size bytes; loopback != 0: the ring
 * lives in ordinary memory (a power of two >= n_threads * slots entries), else pb_xsk_open of
 * the owner (thread 0) maps it.  Returns 0 or -errno. */
int pb_xsk_scq_init(pb_xsk_shared_cq_t *q, uint32_t n_threads, uint32_t slots, uint32_t frame_size, int loopback);
void pb_xsk_scq_free(pb_xsk_shared_cq_t *q);

/* ---- one TX queue: UMEM + TX ring + completion ring ---- */
typedef struct pb_xsk
{
    int fd;           /* AF_XDP socket, -1 for the loopback */
    uint8_t *umem;    /* n_frames * frame_size, page aligned */
    uint32_t n_frames;
    uint32_t frame_size; /* bytes per slot: the descriptors' address stride (--umemslot; FRAME_SIZE by default) */
    pb_xsk_ring_t tx;
    pb_xsk_ring_t cq;
    pb_xsk_ring_t fq;  /* fill ring (the kernel requires one per UMEM; unused for TX) */
    uint32_t next_slot;      /* UMEM slots are used as a ring: next slot to fill */
    uint32_t outstanding_tx; /* submitted, not yet completed (af_xdp.c:227-230) */
    uint32_t need_wakeup;    /* bind flag XDP_USE_NEED_WAKEUP in effect */
    uint64_t wakeups;        /* sendto() calls made */
    uint64_t completed;      /* completions reaped */
    void *maps[3];           /* socket: mmapped ring regions (tx, cq, fq) */
    size_t map_len[3];
    void *loop_mem;          /* loopback: the rings' backing memory */
    int loop_auto;           /* loopback: pb_xsk_complete runs the kernel side inline (the wakeup) */
    void (*loop_sink)(void *ctx, const uint8_t *frame, uint32_t len, uint64_t addr);
    void *loop_ctx;
    uint32_t batch;          /* TX descriptors per reserve / submit / complete (--batchsize); 0: all of a send */
    uint32_t loop_hold;      /* loopback (tests): the kernel side leaves the newest loop_hold descriptors
                                unconsumed, as a slow NIC would keep frames in flight */
    uint32_t slot_base;      /* first UMEM slot of this queue's ring (--sharedumem: queues share one UMEM) */
    pb_xsk_shared_cq_t *scq; /* --sharedumem on one queue: the completion ring every socket shares */
    uint32_t thread;         /* this queue's thread index in scq */
} pb_xsk_t;

/* Loopback TX queue of n_frames (a power of two) slots of frame_size bytes over
 * the given UMEM (page aligned, n_frames * frame_size bytes).  loop_auto = 1:
 * every pb_xsk_complete() first runs the kernel side over all pending
 * descriptors, as a wakeup would (set loop_sink to see the frames); tests that
 * run the kernel side on a thread of their own clear it. */
int pb_xsk_loopback(pb_xsk_t *x, uint8_t *umem, uint32_t n_frames, uint32_t frame_size);
/* The same, one of several queues on one UMEM sharing scq's completion ring (its kernel side
 * posts there; scq->mu held): thread t's ring covers UMEM slots [t * scq->slots, ...), n_frames
 * = scq->slots. */
int pb_xsk_loopback_shared(pb_xsk_t *x, uint8_t *umem, uint32_t frame_size, pb_xsk_shared_cq_t *scq,
                           uint32_t thread);
/* The loopback's kernel side: take up to max TX descriptors, hand each to
 * `sink` (may be NULL), post their addresses to the completion ring.  Returns
 * the number moved. */
typedef void (*pb_xsk_sink_fn)(void *ctx, const uint8_t *frame, uint32_t len, uint64_t addr);
uint32_t pb_xsk_loop_consume(pb_xsk_t *x, uint32_t max, pb_xsk_sink_fn sink, void *ctx);

/* AF_XDP socket on (ifname, queue) over the UMEM, TX ring and completion ring
 * of n_frames entries, slots of frame_size bytes.  The UMEM is registered in
 * chunks of chunk_size bytes (0: frame_size; FRAME_SIZE = 4096 for the
 * reference's geometry): a slot smaller than its chunk (--umemslot) puts
 * chunk_size / frame_size frames in each chunk, which the kernel's aligned mode
 * accepts for TX (a descriptor may start anywhere in its chunk and must not
 * cross its end); chunk_size must be a multiple of frame_size and divide the
 * UMEM's bytes.  bind_flags: XDP_COPY / XDP_ZEROCOPY / XDP_USE_NEED_WAKEUP
 * (af_xdp.c:289-330).  shared_fd >= 0: the UMEM is already registered on that
 * socket (--sharedumem, af_xdp.c:412-428): this socket binds with
 * XDP_SHARED_UMEM and its own fill / completion rings, and uses the n_frames
 * slots from slot_base on.  shared_queue: the queue the owner socket is bound
 * to.  The kernel lets a shared-UMEM socket keep rings of its own only on
 * another queue (or device); on the owner's queue it must use the owner's
 * fill / completion rings: that needs scq (pb_xsk_shared_cq_t), which the
 * owner (shared_fd < 0, scq set) publishes its completion ring into and the
 * others reap through; without scq that case is refused with -EINVAL before
 * any socket is made.  Returns 0, or -errno (EPERM without CAP_NET_RAW,
 * EAFNOSUPPORT without AF_XDP). */
int pb_xsk_open(pb_xsk_t *x, const char *ifname, uint32_t queue, uint8_t *umem, uint32_t n_frames,
                uint32_t frame_size, uint32_t chunk_size, uint16_t bind_flags, int shared_fd, uint32_t slot_base, uint32_t umem_frames,
                uint32_t shared_queue, pb_xsk_shared_cq_t *scq, uint32_t thread);
void pb_xsk_close(pb_xsk_t *x);

/* complete_tx() (af_xdp.c:25-53): wake the kernel if it asks (or always without
 * need-wakeup), reap up to max completions; returns the number reaped. */
uint32_t pb_xsk_complete(pb_xsk_t *x, uint32_t max);

/* Slots the next batch may use without overwriting a frame still in flight. */
uint32_t pb_xsk_free_slots(const pb_xsk_t *x);

/* send: `n` frames sit in UMEM slots next_slot, next_slot + 1, ... (mod n_frames)
 * with lengths lens[]; in groups of `batch` descriptors (all n if 0): reserve them
 * (reaping completions while the ring is full, as send_packet does), fill
 * {addr = (slot_base + slot) * frame_size, len}, submit, complete once
 * (af_xdp.c:184-233).  n <= pb_xsk_free_slots(); returns 0. */
int pb_xsk_send(pb_xsk_t *x, const uint16_t *lens, uint32_t n);

#ifdef __cplusplus
}
#endif
