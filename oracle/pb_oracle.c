/*
 * pb_oracle.c — TEST INFRASTRUCTURE ONLY (see pb_oracle.h for parity status).
 *
 * CPU restatement of PB-AF-XDP's per-thread packet build, src/sequence.c:
 *   - MAC / protocol parsing           sequence.c:66-86
 *   - header template                  sequence.c:150-258
 *   - payload preparation              sequence.c:260-374
 *   - per-iteration randomisation      sequence.c:433-527
 *   - payload fill + L4/L3 checksums   sequence.c:529-602
 *   - hand-off of each frame           sequence.c:604-607 -> af_xdp.c:211-214
 * The per-iteration seed comes from the explicit stream of pb_config.h
 * instead of CLOCK_BOOTTIME (sequence.c:434-441); in "faithful" mode the
 * clock is still read once per iteration and the value discarded.
 *
 * Written for clarity, not speed; it is the checker, never the product.
 */
#define _GNU_SOURCE
#include "pb_oracle.h"

#include <arpa/inet.h>
#include <ctype.h>
#include <errno.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define PBO_OK 0
#define PBO_EINVAL (-22)
#define PBO_ENOMEM (-12)
#define PBO_ENOSPC (-28)

#define ETH_LEN 14
#define IP_LEN 20
#define PROTO_UDP 17
#define PROTO_TCP 6
#define PROTO_ICMP 1

/* ---------------------------------------------------------------- PRNG -- */

/* glibc rand_r (stdlib/rand_r.c semantics): three LCG steps, 11+10+10 bits. */
int pbo_rand_r(unsigned int *seed)
{
    unsigned int x = *seed;
    unsigned int out;

    x = x * 1103515245u + 12345u;
    out = (x >> 16) & 0x7FFu;
    x = x * 1103515245u + 12345u;
    out = (out << 10) ^ ((x >> 16) & 0x3FFu);
    x = x * 1103515245u + 12345u;
    out = (out << 10) ^ ((x >> 16) & 0x3FFu);

    *seed = x;
    return (int)out;
}

static uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint32_t pbo_seed(uint64_t seed_base, uint16_t seq_idx, uint64_t k)
{
    return (uint32_t)splitmix64(seed_base ^ (((uint64_t)seq_idx << 48) + k));
}

/* PB-Common rand_num(min, max, seed): min + rand_r(&copy) % (max - min + 1).
 * The seed is taken by value, so every call in one iteration sees the same
 * first draw.  PINNED by the reference's own captures: images/test1.gif's
 * five and images/test2.gif's eight consecutive-second source ports (README.md
 * :23-27; the demo build seeded with time(NULL)) are 1 + rand_r(t) % 65535 at
 * consecutive t, and no other modulus / offset reproduces them
 * (tests/golden/kat_gif_ports.json, tests/test_rand_num_pin.py). */
static int rand_num(int min, int max, unsigned int seed)
{
    return (pbo_rand_r(&seed) % (max - min + 1)) + min;
}

int pbo_rand_num(int min, int max, unsigned int seed)
{
    return rand_num(min, max, seed);
}

/* --------------------------------------------------------- checksums -- */

/* Sum of 16-bit words read in host (little-endian) order, odd tail byte as
 * the low byte — the generic csum_partial / in_cksum accumulation. */
static uint64_t sum16_le(const uint8_t *p, uint32_t len)
{
    uint64_t s = 0;
    uint32_t i = 0;
    for (; i + 1 < len; i += 2)
        s += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
    if (len & 1)
        s += p[len - 1];
    return s;
}

static uint16_t fold_full(uint64_t s)
{
    while (s >> 16)
        s = (s & 0xFFFF) + (s >> 16);
    return (uint16_t)s;
}

/* update_iph_checksum (csum.h, un-vendored): sum the 10 header words with
 * check = 0; full RFC 1071 fold by default, or the single-fold variant
 * (SURVEY.md B6).  Returns the value to store as a host-order u16 field. */
uint16_t pbo_iph_csum(const uint8_t *iph20, int single_fold)
{
    uint8_t h[IP_LEN];
    memcpy(h, iph20, IP_LEN);
    h[10] = h[11] = 0;
    uint32_t s = (uint32_t)sum16_le(h, IP_LEN);
    if (single_fold)
        return (uint16_t)~((s & 0xFFFF) + (s >> 16));
    return (uint16_t)~fold_full(s);
}

/* csum_tcpudp_magic(saddr, daddr, len, proto, csum_partial(l4, len, 0)) on a
 * little-endian host; for proto 1 (ICMP) icmp_csum(l4, len) — no pseudo
 * header.  The caller zeroes the check field first (sequence.c:571,580,589). */
uint16_t pbo_l4_csum(const uint8_t *l4, uint32_t len, uint32_t saddr_be, uint32_t daddr_be, uint8_t proto)
{
    uint64_t s = sum16_le(l4, len);
    if (proto != PROTO_ICMP)
    {
        s += saddr_be;
        s += daddr_be;
        s += (uint64_t)(proto + len) << 8;
    }
    return (uint16_t)~fold_full(s);
}

/* ------------------------------------------------------------ setup -- */

typedef struct pbo_payload
{
    uint8_t is_static;
    uint16_t min_len, max_len;
    uint8_t *bytes; /* static payload bytes (exact / file / static random) */
} pbo_payload_t;

typedef struct pbo_state
{
    const pb_sequence_t *seq;
    pb_rules_t rules;
    int faithful;

    uint8_t proto;
    uint8_t l4_len;
    uint8_t hl;
    uint8_t tmpl[64];

    int src_static;
    int rnd_ttl, rnd_id;
    int n_ranges;
    uint32_t rng_net[PB_MAX_RANGES]; /* host order, host bits cleared */
    uint32_t rng_hm[PB_MAX_RANGES];
    uint8_t rng_ok[PB_MAX_RANGES];

    int pl_cnt;
    pbo_payload_t pl[PB_MAX_PAYLOADS];
    uint16_t data_len0[PB_MAX_PAYLOADS]; /* data_len[] as left by setup */
} pbo_state_t;

static int parse_mac(const char *s, uint8_t mac[6])
{
    memset(mac, 0, 6);
    if (s == NULL)
        return 0;
    sscanf(s, "%hhx:%hhx:%hhx:%hhx:%hhx:%hhx", &mac[0], &mac[1], &mac[2], &mac[3], &mac[4], &mac[5]);
    return 0;
}

static int str_ieq(const char *a, const char *b)
{
    for (; *a && *b; a++, b++)
        if (tolower((unsigned char)*a) != tolower((unsigned char)*b))
            return 0;
    return *a == *b;
}

/* rand_ip host-bit rule (UNPINNED): "<ip>/<cidr>", cidr in
 * [0,32]; anything else is the `goto fail` path -> 127.0.0.1. */
static int parse_range(const char *r, uint32_t *net, uint32_t *hm)
{
    if (r == NULL)
        return 0;
    char *cpy = strdup(r);
    if (cpy == NULL)
        return 0;
    char *save = NULL;
    char *ip = strtok_r(cpy, "/", &save);
    char *cs = strtok_r(NULL, "/", &save);
    int ok = 0;
    struct in_addr a;
    if (ip != NULL && cs != NULL && inet_aton(ip, &a))
    {
        int cidr = atoi(cs);
        if (cidr >= 0 && cidr <= 32)
        {
            uint32_t m = (cidr == 0) ? 0xFFFFFFFFu : (cidr == 32 ? 0u : ((1u << (32 - cidr)) - 1u));
            *hm = m;
            *net = ntohl(a.s_addr) & ~m;
            ok = 1;
        }
    }
    free(cpy);
    return ok;
}

/* Faithful rand_ip: dotted string out, as PB-Common returns it
 * (sequence.c:465-469 then inet_aton at 493-496). */
static int rand_ip_str(const char *range, unsigned int seed, char out[32])
{
    char *cpy = strdup(range);
    if (cpy == NULL)
        return 0;
    char *save = NULL;
    char *ip = strtok_r(cpy, "/", &save);
    char *cs = strtok_r(NULL, "/", &save);
    int ok = 0;
    struct in_addr a;
    if (ip != NULL && cs != NULL && inet_aton(ip, &a))
    {
        int cidr = atoi(cs);
        if (cidr >= 0 && cidr <= 32)
        {
            uint32_t m = (cidr == 0) ? 0xFFFFFFFFu : (cidr == 32 ? 0u : ((1u << (32 - cidr)) - 1u));
            uint32_t r = (uint32_t)pbo_rand_r(&seed);
            struct in_addr o;
            o.s_addr = htonl((ntohl(a.s_addr) & ~m) | (r & m));
            inet_ntop(AF_INET, &o, out, 32);
            ok = 1;
        }
    }
    free(cpy);
    return ok;
}

/* Static payload text -> bytes (sequence.c:269-337). */
static int load_exact(const pb_payload_opt_t *po, uint8_t *buf, uint16_t *len)
{
    char *text = NULL;
    size_t tlen = 0;
    if (po->is_file)
    {
        FILE *fp = fopen(po->exact, "rb");
        if (fp == NULL)
        {
            text = strdup("");
        }
        else
        {
            fseek(fp, 0, SEEK_END);
            long fl = ftell(fp);
            fseek(fp, 0, SEEK_SET);
            if (fl < 0)
                fl = 0;
            text = (char *)calloc(1, (size_t)fl + 1); /* declared: NUL-terminated at EOF */
            if (text != NULL && fl > 0)
                tlen = fread(text, 1, (size_t)fl, fp);
            (void)tlen;
            fclose(fp);
        }
    }
    else
    {
        text = strdup(po->exact);
    }
    if (text == NULL)
        return PBO_ENOMEM;

    uint32_t n = 0;
    if (po->is_string)
    {
        n = (uint32_t)strlen(text);
        if (n > PB_MAX_PCKT_LEN)
        {
            free(text);
            return PBO_EINVAL;
        }
        memcpy(buf, text, n);
    }
    else
    {
        char *rest = text, *tok;
        while ((tok = strtok_r(rest, " ", &rest)) != NULL)
        {
            if (n >= PB_MAX_PCKT_LEN)
            {
                free(text);
                return PBO_EINVAL;
            }
            unsigned char b = 0; /* declared: an unparsable token is a 0x00 byte */
            sscanf(tok, "%2hhx", &b);
            buf[n++] = b;
        }
    }
    free(text);
    *len = (uint16_t)n;
    return PBO_OK;
}

static void state_free(pbo_state_t *st)
{
    for (int i = 0; i < PB_MAX_PAYLOADS; i++)
    {
        free(st->pl[i].bytes);
        st->pl[i].bytes = NULL;
    }
}

static int state_init(pbo_state_t *st, const pb_sequence_t *seq, const uint8_t *smac, const uint8_t *dmac,
                      uint16_t seq_idx, uint64_t seed_base, const pb_rules_t *rules, int faithful)
{
    memset(st, 0, sizeof *st);
    st->seq = seq;
    st->faithful = faithful;
    if (rules)
        st->rules = *rules;
    if (seq->ip.dst_ip == NULL) /* seq_send refuses the sequence, sequence.c:723-728 */
        return PBO_EINVAL;
    if (seq->pl_cnt > PB_MAX_PAYLOADS || seq->ip.range_count > PB_MAX_RANGES)
        return PBO_EINVAL;

    uint8_t sm[6], dm[6];
    if (smac)
        memcpy(sm, smac, 6);
    else
        parse_mac(seq->eth.src_mac, sm);
    if (dmac)
        memcpy(dm, dmac, 6);
    else
        parse_mac(seq->eth.dst_mac, dm);

    st->proto = PROTO_UDP;
    if (seq->ip.protocol && str_ieq(seq->ip.protocol, "tcp"))
        st->proto = PROTO_TCP;
    else if (seq->ip.protocol && str_ieq(seq->ip.protocol, "icmp"))
        st->proto = PROTO_ICMP;
    st->l4_len = (st->proto == PROTO_TCP) ? 20 : 8;
    st->hl = (uint8_t)(ETH_LEN + IP_LEN + st->l4_len);

    if (seq->ip.min_ttl > seq->ip.max_ttl || seq->ip.min_id > seq->ip.max_id)
        return PBO_EINVAL; /* rand_num modulus <= 0: undefined in the reference */

    /* ---- template, sequence.c:150-258 (buffer defined as zero, B3) ---- */
    uint8_t *t = st->tmpl;
    memcpy(t + 0, dm, 6);
    memcpy(t + 6, sm, 6);
    t[12] = 0x08;
    t[13] = 0x00;
    t[14] = 0x45;
    t[15] = seq->ip.tos;
    t[23] = st->proto;
    st->rnd_ttl = seq->ip.min_ttl != seq->ip.max_ttl;
    st->rnd_id = seq->ip.min_id != seq->ip.max_id;
    if (!st->rnd_ttl)
        t[22] = seq->ip.max_ttl;
    if (!st->rnd_id)
    {
        t[18] = (uint8_t)(seq->ip.max_id >> 8);
        t[19] = (uint8_t)seq->ip.max_id;
    }
    if (seq->ip.src_ip != NULL)
    {
        struct in_addr a = {0};
        inet_aton(seq->ip.src_ip, &a);
        memcpy(t + 26, &a.s_addr, 4);
        st->src_static = 1;
    }
    {
        struct in_addr a = {0};
        inet_aton(seq->ip.dst_ip, &a);
        memcpy(t + 30, &a.s_addr, 4);
    }
    if (st->proto == PROTO_UDP)
    {
        if (seq->udp.src_port > 0)
        {
            t[34] = (uint8_t)(seq->udp.src_port >> 8);
            t[35] = (uint8_t)seq->udp.src_port;
        }
        if (seq->udp.dst_port > 0)
        {
            t[36] = (uint8_t)(seq->udp.dst_port >> 8);
            t[37] = (uint8_t)seq->udp.dst_port;
        }
    }
    else if (st->proto == PROTO_TCP)
    {
        if (seq->tcp.src_port > 0)
        {
            t[34] = (uint8_t)(seq->tcp.src_port >> 8);
            t[35] = (uint8_t)seq->tcp.src_port;
        }
        if (seq->tcp.dst_port > 0)
        {
            t[36] = (uint8_t)(seq->tcp.dst_port >> 8);
            t[37] = (uint8_t)seq->tcp.dst_port;
        }
        t[46] = 5 << 4; /* doff = 5, res1 = 0 */
        t[47] = (uint8_t)((seq->tcp.fin & 1) | (seq->tcp.syn & 1) << 1 | (seq->tcp.rst & 1) << 2 |
                          (seq->tcp.psh & 1) << 3 | (seq->tcp.ack & 1) << 4 | (seq->tcp.urg & 1) << 5 |
                          (seq->tcp.ece & 1) << 6 | (seq->tcp.cwr & 1) << 7);
    }
    else
    {
        t[34] = seq->icmp.type;
        t[35] = seq->icmp.code;
    }

    st->n_ranges = seq->ip.range_count;
    for (int r = 0; r < st->n_ranges; r++)
        st->rng_ok[r] = (uint8_t)parse_range(seq->ip.ranges[r], &st->rng_net[r], &st->rng_hm[r]);

    /* ---- payloads, sequence.c:264-374 ---- */
    unsigned int sseed = pbo_seed(seed_base, seq_idx, PB_STATIC_SEED_K); /* B2 */
    st->pl_cnt = seq->pl_cnt;
    for (int i = 0; i < seq->pl_cnt; i++)
    {
        const pb_payload_opt_t *po = &seq->pls[i];
        pbo_payload_t *pl = &st->pl[i];
        pl->min_len = po->min_len;
        pl->max_len = po->max_len;
        pl->is_static = po->is_static;
        if (po->exact != NULL)
        {
            pl->is_static = 1;
            pl->bytes = (uint8_t *)calloc(1, PB_MAX_PCKT_LEN + 1);
            if (pl->bytes == NULL)
                return PBO_ENOMEM;
            int rc = load_exact(po, pl->bytes, &st->data_len0[i]);
            if (rc)
                return rc;
        }
        else if (po->is_static && po->max_len > 0)
        {
            if (po->min_len > po->max_len)
                return PBO_EINVAL;
            pl->bytes = (uint8_t *)calloc(1, PB_MAX_PCKT_LEN + 1);
            if (pl->bytes == NULL)
                return PBO_ENOMEM;
            st->data_len0[i] = (uint16_t)rand_num(po->min_len, po->max_len, sseed);
            if (st->rules.payload_rule == PB_PAYLOAD_LITERAL)
            {
                /* sequence.c:349: the inner `u16 i` shadows the payload index */
                for (uint32_t j = 0; j < PB_MAX_PAYLOADS && j < st->data_len0[j]; j++)
                    pl->bytes[j] = (uint8_t)pbo_rand_r(&sseed);
            }
            else
            {
                for (uint32_t j = 0; j < st->data_len0[i]; j++)
                    pl->bytes[j] = (uint8_t)pbo_rand_r(&sseed);
            }
        }
        else if (!po->is_static && po->max_len > 0 && po->min_len > po->max_len)
        {
            return PBO_EINVAL;
        }
        if ((uint32_t)st->hl + st->data_len0[i] > PB_MAX_PCKT_LEN)
            return PBO_EINVAL;
    }
    if (st->pl_cnt < 1) /* sequence.c:364-374: one empty static payload */
    {
        st->pl_cnt = 1;
        st->pl[0].is_static = 1;
        st->data_len0[0] = 0;
    }
    for (int i = 0; i < st->pl_cnt; i++)
        if (!st->pl[i].is_static && st->pl[i].max_len > 0 && (uint32_t)st->hl + st->pl[i].max_len > PB_MAX_PCKT_LEN)
            return PBO_EINVAL;
    return PBO_OK;
}

int pbo_frames_per_iter(const pb_sequence_t *seq)
{
    return seq->pl_cnt < 1 ? 1 : seq->pl_cnt;
}

/* ------------------------------------------------------- hot loop ---- */

typedef void (*emit_fn)(void *ctx, const uint8_t *frame, uint16_t len);

/* One iteration (sequence.c:433-602) into `buf` (>= 64 KiB, zeroed once). */
static void run_iteration(const pbo_state_t *st, uint8_t *buf, unsigned int seed, emit_fn emit, void *ectx)
{
    const pb_sequence_t *seq = st->seq;
    uint8_t *iph = buf + ETH_LEN;
    uint8_t *l4 = iph + IP_LEN;
    uint8_t *data = l4 + st->l4_len;

    if (st->faithful)
    {
        struct timespec ts; /* the reference's seed source; value discarded */
        clock_gettime(CLOCK_BOOTTIME, &ts);
        __asm__ __volatile__("" ::"r"(ts.tv_nsec));
    }

    if (st->rnd_ttl)
        iph[8] = (uint8_t)rand_num(seq->ip.min_ttl, seq->ip.max_ttl, seed);
    if (st->rnd_id)
    {
        uint16_t id = (uint16_t)rand_num(seq->ip.min_id, seq->ip.max_id, seed);
        iph[4] = (uint8_t)(id >> 8);
        iph[5] = (uint8_t)id;
    }
    if (!st->src_static)
    {
        uint32_t saddr_be;
        if (st->n_ranges > 0)
        {
            int ri = rand_num(0, st->n_ranges - 1, seed);
            if (st->faithful)
            {
                char sip[32];
                if (seq->ip.ranges[ri] == NULL || !rand_ip_str(seq->ip.ranges[ri], seed, sip))
                    strcpy(sip, "127.0.0.1");
                struct in_addr a;
                inet_aton(sip, &a);
                saddr_be = a.s_addr;
            }
            else if (st->rng_ok[ri])
            {
                unsigned int s2 = seed;
                uint32_t r = (uint32_t)pbo_rand_r(&s2);
                saddr_be = htonl(st->rng_net[ri] | (r & st->rng_hm[ri]));
            }
            else
            {
                saddr_be = htonl(0x7F000001u);
            }
        }
        else
        {
            saddr_be = htonl(0x7F000001u); /* sequence.c:484-490 */
        }
        memcpy(iph + 12, &saddr_be, 4);
    }
    if (st->proto == PROTO_UDP || st->proto == PROTO_TCP)
    {
        uint16_t sp = st->proto == PROTO_UDP ? seq->udp.src_port : seq->tcp.src_port;
        uint16_t dp = st->proto == PROTO_UDP ? seq->udp.dst_port : seq->tcp.dst_port;
        if (sp == 0)
        {
            uint16_t v = (uint16_t)rand_num(1, 65535, seed);
            l4[0] = (uint8_t)(v >> 8);
            l4[1] = (uint8_t)v;
        }
        if (dp == 0)
        {
            uint16_t v = (uint16_t)rand_num(1, 65535, seed);
            l4[2] = (uint8_t)(v >> 8);
            l4[3] = (uint8_t)v;
        }
    }

    /* data_len[] as the reference sees it this iteration (declared rule:
     * entries of later payloads hold their setup-time values, B8). */
    uint16_t data_len[PB_MAX_PAYLOADS];
    memcpy(data_len, st->data_len0, sizeof data_len);

    uint32_t saddr_be, daddr_be;
    memcpy(&saddr_be, iph + 12, 4);
    memcpy(&daddr_be, iph + 16, 4);

    for (int i = 0; i < st->pl_cnt; i++)
    {
        const pbo_payload_t *pl = &st->pl[i];
        if (pl->is_static)
        {
            if (data_len[i] > 0)
                memcpy(data, pl->bytes, data_len[i]);
        }
        else if (pl->max_len > 0)
        {
            data_len[i] = (uint16_t)rand_num(pl->min_len, pl->max_len, seed);
            if (st->rules.payload_rule == PB_PAYLOAD_LITERAL)
            {
                memset(data, 0, data_len[i]); /* declared: unwritten bytes are 0 */
                for (uint32_t j = 0; j < PB_MAX_PAYLOADS && j < data_len[j]; j++)
                    data[j] = (uint8_t)pbo_rand_r(&seed);
            }
            else
            {
                for (uint32_t j = 0; j < data_len[i]; j++)
                    data[j] = (uint8_t)pbo_rand_r(&seed);
            }
        }
        uint32_t plen = data_len[i];
        uint32_t l4tot = st->l4_len + plen;

        if (st->proto == PROTO_UDP)
        {
            l4[4] = (uint8_t)(l4tot >> 8);
            l4[5] = (uint8_t)l4tot;
            if (seq->l4_csum)
            {
                l4[6] = l4[7] = 0;
                uint16_t c = pbo_l4_csum(l4, l4tot, saddr_be, daddr_be, PROTO_UDP);
                memcpy(l4 + 6, &c, 2);
            }
        }
        else if (st->proto == PROTO_TCP)
        {
            if (seq->l4_csum)
            {
                l4[16] = l4[17] = 0;
                uint16_t c = pbo_l4_csum(l4, l4tot, saddr_be, daddr_be, PROTO_TCP);
                memcpy(l4 + 16, &c, 2);
            }
        }
        else
        {
            if (seq->l4_csum)
            {
                l4[2] = l4[3] = 0;
                uint16_t c = pbo_l4_csum(l4, l4tot, 0, 0, PROTO_ICMP);
                memcpy(l4 + 2, &c, 2);
            }
        }

        uint32_t tot = IP_LEN + l4tot;
        iph[2] = (uint8_t)(tot >> 8);
        iph[3] = (uint8_t)tot;
        if (seq->ip.csum)
        {
            uint16_t c = pbo_iph_csum(iph, st->rules.iph_fold == PB_FOLD_SINGLE);
            memcpy(iph + 10, &c, 2);
        }
        emit(ectx, buf, (uint16_t)(ETH_LEN + tot));
    }
}

typedef struct emit_ctx
{
    uint8_t *out;
    uint64_t cap;
    uint32_t slot;
    uint32_t ring; /* slot mode: wrap after `ring` slots (0 = never) */
    uint64_t pos;
    uint64_t n;
    uint64_t *offsets;
    int err;
} emit_ctx_t;

static void emit_out(void *vctx, const uint8_t *frame, uint16_t len)
{
    emit_ctx_t *e = (emit_ctx_t *)vctx;
    if (e->slot)
    {
        uint64_t at = (e->ring ? e->n % e->ring : e->n) * e->slot;
        if (len > e->slot || at + e->slot > e->cap)
        {
            e->err = PBO_ENOSPC;
            return;
        }
        memcpy(e->out + at, frame, len);
        e->pos += len;
    }
    else
    {
        if (e->pos + len > e->cap)
        {
            e->err = PBO_ENOSPC;
            return;
        }
        if (e->offsets)
            e->offsets[e->n] = e->pos;
        memcpy(e->out + e->pos, frame, len);
        e->pos += len;
    }
    e->n++;
}

int pbo_build(const pb_sequence_t *seq, const uint8_t *smac, const uint8_t *dmac,
              uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter, uint64_t seed_base,
              const pb_rules_t *rules, int faithful,
              uint8_t *out, uint64_t out_cap, uint32_t slot_stride,
              uint64_t *offsets, uint64_t *n_frames, uint64_t *total_bytes)
{
    pbo_state_t *st = (pbo_state_t *)malloc(sizeof *st);
    uint8_t *buf = (uint8_t *)calloc(1, PB_MAX_PCKT_LEN + 64);
    if (st == NULL || buf == NULL)
    {
        free(st);
        free(buf);
        return PBO_ENOMEM;
    }
    int rc = state_init(st, seq, smac, dmac, seq_idx, seed_base, rules, faithful);
    if (rc == PBO_OK)
    {
        memcpy(buf, st->tmpl, sizeof st->tmpl);
        emit_ctx_t e = {out, out_cap, slot_stride, 0, 0, 0, offsets, 0};
        for (uint64_t k = 0; k < n_iter && !e.err; k++)
            run_iteration(st, buf, pbo_seed(seed_base, seq_idx, first_iter + k), emit_out, &e);
        if (e.err)
            rc = e.err;
        if (offsets && !slot_stride)
            offsets[e.n] = e.pos;
        if (n_frames)
            *n_frames = e.n;
        if (total_bytes)
            *total_bytes = e.pos;
    }
    state_free(st);
    free(st);
    free(buf);
    return rc;
}

typedef struct mt_job
{
    const pbo_state_t *st;
    uint16_t seq_idx;
    uint64_t seed_base;
    uint64_t k0, k1;
    emit_ctx_t e;
} mt_job_t;

static void *mt_worker(void *arg)
{
    mt_job_t *j = (mt_job_t *)arg;
    uint8_t *buf = (uint8_t *)calloc(1, PB_MAX_PCKT_LEN + 64);
    if (buf == NULL)
    {
        j->e.err = PBO_ENOMEM;
        return NULL;
    }
    memcpy(buf, j->st->tmpl, sizeof j->st->tmpl);
    for (uint64_t k = j->k0; k < j->k1 && !j->e.err; k++)
        run_iteration(j->st, buf, pbo_seed(j->seed_base, j->seq_idx, k), emit_out, &j->e);
    free(buf);
    return NULL;
}

int pbo_build_mt(const pb_sequence_t *seq, const uint8_t *smac, const uint8_t *dmac,
                 uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter, uint64_t seed_base,
                 const pb_rules_t *rules, int faithful, int nthreads,
                 uint8_t *out, uint64_t out_cap, uint32_t slot_stride, uint32_t ring_slots,
                 uint64_t *total_bytes)
{
    if (slot_stride == 0 || nthreads < 1 || nthreads > 1024)
        return PBO_EINVAL;
    pbo_state_t *st = (pbo_state_t *)malloc(sizeof *st);
    if (st == NULL)
        return PBO_ENOMEM;
    int rc = state_init(st, seq, smac, dmac, seq_idx, seed_base, rules, faithful);
    if (rc)
    {
        state_free(st);
        free(st);
        return rc;
    }
    int fpi = st->pl_cnt;
    mt_job_t *jobs = (mt_job_t *)calloc((size_t)nthreads, sizeof *jobs);
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof *th);
    if (!jobs || !th)
    {
        free(jobs);
        free(th);
        state_free(st);
        free(st);
        return PBO_ENOMEM;
    }
    for (int t = 0; t < nthreads; t++)
    {
        uint64_t a = first_iter + n_iter * (uint64_t)t / (uint64_t)nthreads;
        uint64_t b = first_iter + n_iter * (uint64_t)(t + 1) / (uint64_t)nthreads;
        uint64_t fa = ring_slots ? (uint64_t)t * ring_slots : (a - first_iter) * (uint64_t)fpi;
        jobs[t].st = st;
        jobs[t].seq_idx = seq_idx;
        jobs[t].seed_base = seed_base;
        jobs[t].k0 = a;
        jobs[t].k1 = b;
        jobs[t].e.out = out + fa * slot_stride;
        jobs[t].e.cap = out_cap > fa * slot_stride ? out_cap - fa * slot_stride : 0;
        jobs[t].e.slot = slot_stride;
        jobs[t].e.ring = ring_slots;
        pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
    }
    uint64_t tot = 0;
    for (int t = 0; t < nthreads; t++)
    {
        pthread_join(th[t], NULL);
        tot += jobs[t].e.pos;
        if (jobs[t].e.err)
            rc = jobs[t].e.err;
    }
    if (total_bytes)
        *total_bytes = tot;
    free(jobs);
    free(th);
    state_free(st);
    free(st);
    return rc;
}

/* ---------------- checker: every frame's checksums (test infrastructure) ----------------
 * RFC 1071 verification of packed frames (Ethernet + IPv4 without options + UDP / TCP /
 * ICMP), independent of how they were built: the IPv4 header words and the L4 segment
 * words (plus the pseudo header for UDP / TCP, sequence.c:585-602) each fold to 0xFFFF,
 * and tot_len equals the frame length - 14.  Used by the full-size GPU tests, whose
 * frames are too many to compare one by one with the oracle. */
static uint32_t sum16_be(const uint8_t *p, uint32_t len)
{
    uint32_t s = 0;
    uint32_t i = 0;
    for (; i + 1 < len; i += 2)
        s += (uint32_t)p[i] << 8 | p[i + 1];
    if (i < len)
        s += (uint32_t)p[i] << 8;
    return s;
}

static uint32_t fold16(uint64_t s)
{
    while (s >> 16)
        s = (s & 0xFFFF) + (s >> 16);
    return (uint32_t)s;
}

static int verify_one(const uint8_t *f, uint32_t len)
{
    if (len < 34)
        return 1;
    if (fold16(sum16_be(f + 14, 20)) != 0xFFFF)
        return 1;
    if (((uint32_t)f[16] << 8 | f[17]) != len - 14)
        return 1;
    const uint8_t proto = f[23];
    uint64_t s = sum16_be(f + 34, len - 34);
    if (proto == 6 || proto == 17)
        s += sum16_be(f + 26, 8) + proto + (len - 34);
    return fold16(s) != 0xFFFF;
}

typedef struct verify_job
{
    const uint8_t *data;
    const uint64_t *off;
    uint32_t flen;
    uint64_t a, b, bad;
} verify_job_t;

static void *verify_worker(void *arg)
{
    verify_job_t *j = (verify_job_t *)arg;
    for (uint64_t i = j->a; i < j->b; i++)
    {
        const uint64_t s = j->off ? j->off[i] - j->off[0] : i * (uint64_t)j->flen;
        const uint32_t len = j->off ? (uint32_t)(j->off[i + 1] - j->off[i]) : j->flen;
        j->bad += (uint64_t)verify_one(j->data + s, len);
    }
    return NULL;
}

uint64_t pbo_verify_frames(const uint8_t *data, const uint64_t *offsets, uint32_t fixed_len, uint64_t n,
                           int nthreads)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    verify_job_t jobs[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++)
    {
        jobs[t] = (verify_job_t){data, offsets, fixed_len, n * (uint64_t)t / (uint64_t)nthreads,
                                 n * (uint64_t)(t + 1) / (uint64_t)nthreads, 0};
        pthread_create(&th[t], NULL, verify_worker, &jobs[t]);
    }
    uint64_t bad = 0;
    for (int t = 0; t < nthreads; t++)
    {
        pthread_join(th[t], NULL);
        bad += jobs[t].bad;
    }
    return bad;
}
