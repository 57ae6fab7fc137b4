/*
 * xsk_ring.c — AF_XDP TX rings, UMEM slot ring and socket setup without
 * libbpf (see xsk_ring.h for the reference code each part replaces).
 */
#define _GNU_SOURCE
#include "xsk_ring.h"

#include <errno.h>
#include <net/if.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#ifndef AF_XDP
#define AF_XDP 44
#endif
#ifndef SOL_XDP
#define SOL_XDP 283
#endif

static inline uint32_t load_acquire(const uint32_t *p)
{
    return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}

static inline void store_release(uint32_t *p, uint32_t v)
{
    __atomic_store_n(p, v, __ATOMIC_RELEASE);
}

/* ---------------- producer: the TX ring ---------------- */

uint32_t pb_ring_prod_free(pb_xsk_ring_t *r)
{
    uint32_t free_entries = r->cached_cons - r->cached_prod;
    if (free_entries == 0)
    {
        /* cached_cons is kept `size` ahead of the consumer index, so the
         * subtraction above is the free count (libbpf xsk_prod_nb_free) */
        r->cached_cons = load_acquire(r->consumer) + r->size;
        free_entries = r->cached_cons - r->cached_prod;
    }
    return free_entries;
}

uint32_t pb_ring_prod_reserve(pb_xsk_ring_t *r, uint32_t nb, uint32_t *idx)
{
    uint32_t free_entries = r->cached_cons - r->cached_prod;
    if (free_entries < nb)
    {
        r->cached_cons = load_acquire(r->consumer) + r->size;
        free_entries = r->cached_cons - r->cached_prod;
    }
    if (free_entries < nb)
        return 0;
    *idx = r->cached_prod;
    r->cached_prod += nb;
    return nb;
}

struct xdp_desc *pb_ring_tx_desc(pb_xsk_ring_t *r, uint32_t idx)
{
    return &((struct xdp_desc *)r->ring)[idx & r->mask];
}

void pb_ring_prod_submit(pb_xsk_ring_t *r, uint32_t nb)
{
    /* the descriptors written before this store are visible to the consumer
     * that acquires the new producer index */
    store_release(r->producer, *r->producer + nb);
}

int pb_ring_needs_wakeup(const pb_xsk_ring_t *r)
{
    return (__atomic_load_n(r->flags, __ATOMIC_RELAXED) & XDP_RING_NEED_WAKEUP) != 0;
}

/* ---------------- consumer: the completion ring ---------------- */

uint32_t pb_ring_cons_peek(pb_xsk_ring_t *r, uint32_t nb, uint32_t *idx)
{
    uint32_t entries = r->cached_prod - r->cached_cons;
    if (entries == 0)
    {
        r->cached_prod = load_acquire(r->producer);
        entries = r->cached_prod - r->cached_cons;
    }
    if (entries > nb)
        entries = nb;
    if (entries)
    {
        *idx = r->cached_cons;
        r->cached_cons += entries;
    }
    return entries;
}

uint64_t pb_ring_comp_addr(const pb_xsk_ring_t *r, uint32_t idx)
{
    return ((const uint64_t *)r->ring)[idx & r->mask];
}

void pb_ring_cons_release(pb_xsk_ring_t *r, uint32_t nb)
{
    /* the entries were read before this store: the producer may reuse them */
    store_release(r->consumer, *r->consumer + nb);
}

/* ---------------- loopback pair ---------------- */

/* one ring in ordinary memory: producer, consumer, flags words, then entries */
static void loop_ring(pb_xsk_ring_t *r, uint8_t *mem, uint32_t n, int producer_side)
{
    memset(r, 0, sizeof *r);
    r->producer = (uint32_t *)mem;
    r->consumer = (uint32_t *)(mem + 64);
    r->flags = (uint32_t *)(mem + 128);
    r->ring = mem + 192;
    r->size = n;
    r->mask = n - 1;
    r->cached_cons = producer_side ? n : 0; /* a producer starts with `size` free entries */
}

int pb_xsk_loopback(pb_xsk_t *x, uint8_t *umem, uint32_t n_frames, uint32_t frame_size)
{
    if (x == NULL || umem == NULL || n_frames == 0 || (n_frames & (n_frames - 1)) || frame_size == 0)
        return -EINVAL;
    memset(x, 0, sizeof *x);
    const size_t tx_bytes = 192 + (size_t)n_frames * sizeof(struct xdp_desc);
    const size_t cq_bytes = 192 + (size_t)n_frames * sizeof(uint64_t);
    uint8_t *mem = (uint8_t *)calloc(1, tx_bytes + cq_bytes);
    if (mem == NULL)
        return -ENOMEM;
    x->fd = -1;
    x->loop_mem = mem;
    x->loop_auto = 1;
    x->umem = umem;
    x->n_frames = n_frames;
    x->frame_size = frame_size;
    x->need_wakeup = 1;
    loop_ring(&x->tx, mem, n_frames, 1);
    loop_ring(&x->cq, mem + tx_bytes, n_frames, 0);
    *x->tx.flags = XDP_RING_NEED_WAKEUP; /* the loopback's kernel side runs only when woken */
    return 0;
}

int pb_xsk_scq_init(pb_xsk_shared_cq_t *q, uint32_t n_threads, uint32_t slots, uint32_t frame_size, int loopback)
{
    if (q == NULL || n_threads == 0 || n_threads > PB_XSK_MAX_SHARERS || slots == 0 || (slots & (slots - 1)) ||
        frame_size == 0)
        return -EINVAL;
    memset(q, 0, sizeof *q);
    q->slots = slots;
    q->frame_size = frame_size;
    q->n_threads = n_threads;
    if (loopback)
    {
        uint32_t n = 1;
        while (n < n_threads * slots)
            n <<= 1;
        q->mem = calloc(1, 192 + (size_t)n * sizeof(uint64_t));
        if (q->mem == NULL)
            return -ENOMEM;
        loop_ring(&q->cq, (uint8_t *)q->mem, n, 0);
    }
    pthread_mutex_init(&q->mu, NULL);
    return 0;
}

void pb_xsk_scq_free(pb_xsk_shared_cq_t *q)
{
    if (q == NULL)
        return;
    pthread_mutex_destroy(&q->mu);
    free(q->mem);
    q->mem = NULL;
}

int pb_xsk_loopback_shared(pb_xsk_t *x, uint8_t *umem, uint32_t frame_size, pb_xsk_shared_cq_t *scq,
                           uint32_t thread)
{
    if (scq == NULL || scq->mem == NULL || thread >= scq->n_threads)
        return -EINVAL;
    const int rc = pb_xsk_loopback(x, umem, scq->slots, frame_size);
    if (rc)
        return rc;
    x->scq = scq;
    x->thread = thread;
    x->slot_base = thread * scq->slots;
    return 0;
}

uint32_t pb_xsk_loop_consume(pb_xsk_t *x, uint32_t max, pb_xsk_sink_fn sink, void *ctx)
{
    /* the kernel's side of both rings: consumer of TX, producer of completions.
     * It keeps no cached indices of its own: it reads TX's producer and the
     * completion ring's consumer (both written by the application) each call. */
    /* (a queue sharing a UMEM posts to the shared completion ring: the caller holds scq->mu) */
    pb_xsk_ring_t *const cq = x->scq ? &x->scq->cq : &x->cq;
    const uint32_t tx_prod = load_acquire(x->tx.producer);
    const uint32_t tx_cons = *x->tx.consumer;
    const uint32_t cq_prod = *cq->producer;
    const uint32_t cq_free = cq->size - (cq_prod - load_acquire(cq->consumer));
    uint32_t n = tx_prod - tx_cons;
    if (n > max)
        n = max;
    if (n > cq_free)
        n = cq_free;
    for (uint32_t i = 0; i < n; ++i)
    {
        const struct xdp_desc *d = &((const struct xdp_desc *)x->tx.ring)[(tx_cons + i) & x->tx.mask];
        if (sink)
            sink(ctx, x->umem + d->addr, d->len, d->addr);
        ((uint64_t *)cq->ring)[(cq_prod + i) & cq->mask] = d->addr;
    }
    if (n)
    {
        store_release(x->tx.consumer, tx_cons + n); /* TX entries read: free for the producer */
        store_release(cq->producer, cq_prod + n);   /* completions written: visible to the reaper */
    }
    return n;
}

/* ---------------- AF_XDP socket ---------------- */

static int map_ring(int fd, pb_xsk_ring_t *r, const struct xdp_ring_offset *off, uint32_t n, size_t entry,
                    uint64_t pgoff, int producer_side, void **map, size_t *len)
{
    *len = off->desc + (size_t)n * entry;
    void *m = mmap(NULL, *len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, (off_t)pgoff);
    if (m == MAP_FAILED)
        return -errno;
    *map = m;
    memset(r, 0, sizeof *r);
    r->producer = (uint32_t *)((uint8_t *)m + off->producer);
    r->consumer = (uint32_t *)((uint8_t *)m + off->consumer);
    r->flags = (uint32_t *)((uint8_t *)m + off->flags);
    r->ring = (uint8_t *)m + off->desc;
    r->size = n;
    r->mask = n - 1;
    r->cached_prod = *r->producer;
    r->cached_cons = producer_side ? *r->consumer + n : *r->consumer;
    return 0;
}

int pb_xsk_open(pb_xsk_t *x, const char *ifname, uint32_t queue, uint8_t *umem, uint32_t n_frames,
                uint32_t frame_size, uint32_t chunk_size, uint16_t bind_flags, int shared_fd, uint32_t slot_base,
                uint32_t umem_frames, uint32_t shared_queue, pb_xsk_shared_cq_t *scq, uint32_t thread)
{
    const uint64_t umem_bytes = (uint64_t)(umem_frames ? umem_frames : n_frames) * frame_size;
    if (chunk_size == 0)
        chunk_size = frame_size;
    if (x == NULL || ifname == NULL || umem == NULL || n_frames == 0 || (n_frames & (n_frames - 1)) ||
        slot_base + n_frames > (umem_frames ? umem_frames : n_frames) || frame_size == 0 ||
        chunk_size % frame_size || umem_bytes % chunk_size)
        return -EINVAL;
    /* xsk_bind: XDP_SHARED_UMEM on the owner's (device, queue) shares its buffer pool and
     * rejects a socket with fill / completion rings of its own: such a socket takes none and
     * reaps the owner's completion ring through scq (xsk_socket__create_shared's model) */
    const int on_owner_queue = shared_fd >= 0 && shared_queue == queue;
    if (on_owner_queue && scq == NULL)
        return -EINVAL;
    memset(x, 0, sizeof *x);
    x->fd = -1;
    x->slot_base = slot_base;
    x->scq = scq;
    x->thread = thread;
    const unsigned ifindex = if_nametoindex(ifname);
    if (ifindex == 0)
        return -ENODEV;
    const int fd = socket(AF_XDP, SOCK_RAW, 0);
    if (fd < 0)
        return -errno;
    x->fd = fd;
    x->umem = umem;
    x->n_frames = n_frames;
    x->frame_size = frame_size;
    /* xsk_umem__create: register the UMEM (once: a shared UMEM stays registered on the
     * first socket), size this socket's fill and completion rings */
    struct xdp_umem_reg mr;
    memset(&mr, 0, sizeof mr);
    mr.addr = (uint64_t)(uintptr_t)umem;
    mr.len = umem_bytes;
    mr.chunk_size = chunk_size;
    int rc = 0;
    const int ring_n = (int)n_frames;
    /* the owner's fill and completion rings cover the whole UMEM when queues share it */
    const int cq_n = (int)(scq && shared_fd < 0 ? (umem_frames ? umem_frames : n_frames) : n_frames);
    if ((shared_fd < 0 && setsockopt(fd, SOL_XDP, XDP_UMEM_REG, &mr, sizeof mr)) ||
        (!on_owner_queue && (setsockopt(fd, SOL_XDP, XDP_UMEM_FILL_RING, &cq_n, sizeof cq_n) ||
                             setsockopt(fd, SOL_XDP, XDP_UMEM_COMPLETION_RING, &cq_n, sizeof cq_n))) ||
        /* xsk_socket__create with a TX ring only (af_xdp.c:103-165) */
        setsockopt(fd, SOL_XDP, XDP_TX_RING, &ring_n, sizeof ring_n))
    {
        rc = -errno;
        goto fail;
    }
    struct xdp_mmap_offsets off;
    socklen_t optlen = sizeof off;
    if (getsockopt(fd, SOL_XDP, XDP_MMAP_OFFSETS, &off, &optlen))
    {
        rc = -errno;
        goto fail;
    }
    if ((rc = map_ring(fd, &x->tx, &off.tx, n_frames, sizeof(struct xdp_desc), XDP_PGOFF_TX_RING, 1, &x->maps[0],
                       &x->map_len[0])))
        goto fail;
    if (!on_owner_queue &&
        ((rc = map_ring(fd, &x->cq, &off.cr, (uint32_t)cq_n, sizeof(uint64_t), XDP_UMEM_PGOFF_COMPLETION_RING, 0,
                        &x->maps[1], &x->map_len[1])) ||
         (rc = map_ring(fd, &x->fq, &off.fr, (uint32_t)cq_n, sizeof(uint64_t), XDP_UMEM_PGOFF_FILL_RING, 1,
                        &x->maps[2], &x->map_len[2]))))
        goto fail;
    struct sockaddr_xdp sxdp;
    memset(&sxdp, 0, sizeof sxdp);
    sxdp.sxdp_family = AF_XDP;
    sxdp.sxdp_ifindex = ifindex;
    sxdp.sxdp_queue_id = queue;
    sxdp.sxdp_flags = bind_flags;
    if (shared_fd >= 0)
    {
        sxdp.sxdp_flags = XDP_SHARED_UMEM; /* the kernel takes the copy / wakeup mode of the UMEM's owner */
        sxdp.sxdp_shared_umem_fd = (uint32_t)shared_fd;
    }
    if (bind(fd, (struct sockaddr *)&sxdp, sizeof sxdp))
    {
        rc = -errno;
        goto fail;
    }
    x->need_wakeup = (bind_flags & XDP_USE_NEED_WAKEUP) != 0;
    if (scq && shared_fd < 0)
    {
        /* the owner: its completion ring is the one every socket of the queue reaps */
        pthread_mutex_lock(&scq->mu);
        scq->cq = x->cq;
        pthread_mutex_unlock(&scq->mu);
    }
    return 0;
fail:
    pb_xsk_close(x);
    return rc;
}

void pb_xsk_close(pb_xsk_t *x)
{
    if (x == NULL)
        return;
    for (int i = 0; i < 3; ++i)
        if (x->maps[i])
            munmap(x->maps[i], x->map_len[i]);
    if (x->fd >= 0)
        close(x->fd);
    free(x->loop_mem);
    memset(x, 0, sizeof *x);
    x->fd = -1;
}

/* ---------------- send / complete ---------------- */

uint32_t pb_xsk_complete(pb_xsk_t *x, uint32_t max)
{
    if (!x->outstanding_tx)
        return 0;
    /* wake the kernel: always without need-wakeup, else only when it asks (af_xdp.c:38-41) */
    const int wake = !x->need_wakeup || pb_ring_needs_wakeup(&x->tx);
    if (wake)
    {
        ++x->wakeups;
        if (x->fd >= 0)
            (void)sendto(x->fd, NULL, 0, MSG_DONTWAIT, NULL, 0);
        else if (x->loop_auto && !x->scq) /* (a shared ring's kernel side runs under its lock, below) */
        {
            const uint32_t pending = __atomic_load_n(x->tx.producer, __ATOMIC_ACQUIRE) - *x->tx.consumer;
            if (pending > x->loop_hold)
                (void)pb_xsk_loop_consume(x, pending - x->loop_hold, x->loop_sink, x->loop_ctx);
        }
    }
    uint32_t idx = 0;
    if (x->scq)
    {
        /* the shared completion ring: reap every entry, credit each to its slot range's thread,
         * take this thread's credits (at most its outstanding frames, which bounds them) */
        pb_xsk_shared_cq_t *q = x->scq;
        pthread_mutex_lock(&q->mu);
        if (x->fd < 0 && x->loop_auto && wake)
        {
            const uint32_t pending = __atomic_load_n(x->tx.producer, __ATOMIC_ACQUIRE) - *x->tx.consumer;
            if (pending > x->loop_hold)
                (void)pb_xsk_loop_consume(x, pending - x->loop_hold, x->loop_sink, x->loop_ctx);
        }
        uint32_t got;
        while ((got = pb_ring_cons_peek(&q->cq, q->cq.size, &idx)) != 0)
        {
            for (uint32_t i = 0; i < got; ++i)
            {
                const uint64_t t = pb_ring_comp_addr(&q->cq, idx + i) / q->frame_size / q->slots;
                if (t < q->n_threads)
                    ++q->credit[t];
            }
            pb_ring_cons_release(&q->cq, got);
            q->reaped += got;
        }
        const uint32_t n = q->credit[x->thread];
        q->credit[x->thread] = 0;
        pthread_mutex_unlock(&q->mu);
        x->outstanding_tx -= n;
        x->completed += n;
        return n;
    }
    const uint32_t n = pb_ring_cons_peek(&x->cq, max, &idx);
    if (n)
    {
        pb_ring_cons_release(&x->cq, n);
        x->outstanding_tx -= n;
        x->completed += n;
    }
    return n;
}

uint32_t pb_xsk_free_slots(const pb_xsk_t *x)
{
    return x->n_frames - x->outstanding_tx;
}

int pb_xsk_send(pb_xsk_t *x, const uint16_t *lens, uint32_t n)
{
    if (n == 0)
        return 0;
    if (n > pb_xsk_free_slots(x))
        return -ENOSPC;
    const uint32_t bs = x->batch ? x->batch : n;
    for (uint32_t sent = 0; sent < n;)
    {
        const uint32_t k = n - sent < bs ? n - sent : bs;
        uint32_t idx = 0;
        /* af_xdp.c:184-190: reap completions until the TX ring has room */
        for (uint64_t spin = 0; pb_ring_prod_reserve(&x->tx, k, &idx) < k; ++spin)
        {
            if (pb_xsk_complete(x, x->n_frames) == 0 && spin > 1000)
                sched_yield();
            if (spin > (1ull << 26))
                return -EAGAIN;
        }
        for (uint32_t i = 0; i < k; ++i)
        {
            /* af_xdp.c:217-223: the slot's UMEM address and the frame length */
            struct xdp_desc *d = pb_ring_tx_desc(&x->tx, idx + i);
            const uint32_t slot = (x->next_slot + i) & (x->n_frames - 1);
            d->addr = (uint64_t)(x->slot_base + slot) * x->frame_size;
            d->len = lens[sent + i];
            d->options = 0;
        }
        pb_ring_prod_submit(&x->tx, k);
        x->next_slot = (x->next_slot + k) & (x->n_frames - 1);
        x->outstanding_tx += k;
        (void)pb_xsk_complete(x, x->n_frames); /* af_xdp.c:233 */
        sent += k;
    }
    return 0;
}
