/*
 * config_json.c — the reference's JSON config file (-c, default
 * /etc/pcktbatch/conf.json; src/main.c:51-94) read into pb_config_t.
 *
 * The reference reads it with PB-Common's parse_config() on json-c, both
 * un-vendored; the schema and defaults are the README's (README.md:170-578):
 * top-level "interface" and "sequences"; per sequence interface, block,
 * track, maxpckts, maxbytes, pps, bps, time, threads, delay, l4csum and the
 * eth / ip / udp / tcp / icmp objects and the payloads array.  A key that is
 * absent keeps the value clear_sequence() gave it.  This is a small
 * recursive-descent JSON reader of the build's own (RFC 8259 values; integers
 * kept exact to 64 bits); booleans and numbers are both accepted for the
 * boolean fields, as json-c's get_boolean / get_int do.
 *
 * Strings stay in the parser's memory until pb_config_free(), since
 * pb_sequence_t holds pointers (the reference's config lives to exit too).
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "config_json.h"

typedef enum
{
    J_NULL,
    J_BOOL,
    J_NUM,
    J_STR,
    J_ARR,
    J_OBJ
} jtype_t;

typedef struct jnode
{
    jtype_t t;
    int boolean;
    int negative, integral;
    uint64_t u; /* |integer| when integral */
    double d;
    char *str;
    int n;             /* children (array / object) */
    char **keys;       /* object keys */
    struct jnode *kid; /* children */
} jnode_t;

typedef struct
{
    const char *p, *end;
    int depth;
    const char *err;
} jparser_t;

/* allocations kept for the life of the strings in pb_config_t */
static void **g_keep;
static size_t g_nkeep;

static void *keep(void *ptr)
{
    if (ptr == NULL)
        return NULL;
    void **k = (void **)realloc(g_keep, (g_nkeep + 1) * sizeof *k);
    if (k == NULL)
    {
        free(ptr);
        return NULL;
    }
    g_keep = k;
    g_keep[g_nkeep++] = ptr;
    return ptr;
}

void pb_config_free(void)
{
    for (size_t i = 0; i < g_nkeep; ++i)
        free(g_keep[i]);
    free(g_keep);
    g_keep = NULL;
    g_nkeep = 0;
}

static void skip_ws(jparser_t *P)
{
    while (P->p < P->end && (*P->p == ' ' || *P->p == '\t' || *P->p == '\n' || *P->p == '\r'))
        ++P->p;
}

static int parse_value(jparser_t *P, jnode_t *out);

static int hexval(char c)
{
    if (c >= '0' && c <= '9')
        return c - '0';
    if (c >= 'a' && c <= 'f')
        return c - 'a' + 10;
    if (c >= 'A' && c <= 'F')
        return c - 'A' + 10;
    return -1;
}

static int put_utf8(char **o, uint32_t cp)
{
    char *w = *o;
    if (cp < 0x80)
        *w++ = (char)cp;
    else if (cp < 0x800)
    {
        *w++ = (char)(0xC0 | (cp >> 6));
        *w++ = (char)(0x80 | (cp & 0x3F));
    }
    else if (cp < 0x10000)
    {
        *w++ = (char)(0xE0 | (cp >> 12));
        *w++ = (char)(0x80 | ((cp >> 6) & 0x3F));
        *w++ = (char)(0x80 | (cp & 0x3F));
    }
    else
    {
        *w++ = (char)(0xF0 | (cp >> 18));
        *w++ = (char)(0x80 | ((cp >> 12) & 0x3F));
        *w++ = (char)(0x80 | ((cp >> 6) & 0x3F));
        *w++ = (char)(0x80 | (cp & 0x3F));
    }
    *o = w;
    return 0;
}

static int parse_hex4(jparser_t *P, uint32_t *v)
{
    if (P->end - P->p < 4)
        return -1;
    uint32_t x = 0;
    for (int i = 0; i < 4; ++i)
    {
        const int h = hexval(P->p[i]);
        if (h < 0)
            return -1;
        x = x << 4 | (uint32_t)h;
    }
    P->p += 4;
    *v = x;
    return 0;
}

/* string at P->p (after the opening quote) -> malloc'd UTF-8 copy */
static char *parse_string(jparser_t *P)
{
    const char *s = P->p;
    size_t cap = 1;
    while (s < P->end && *s != '"')
    {
        if (*s == '\\')
            ++s;
        ++s;
        ++cap;
    }
    if (s >= P->end)
    {
        P->err = "unterminated string";
        return NULL;
    }
    char *buf = (char *)malloc(cap * 4 + 1);
    if (buf == NULL)
    {
        P->err = "out of memory";
        return NULL;
    }
    char *w = buf;
    while (*P->p != '"')
    {
        unsigned char c = (unsigned char)*P->p++;
        if (c < 0x20)
        {
            P->err = "control character in string";
            free(buf);
            return NULL;
        }
        if (c != '\\')
        {
            *w++ = (char)c;
            continue;
        }
        c = (unsigned char)*P->p++;
        switch (c)
        {
        case '"': *w++ = '"'; break;
        case '\\': *w++ = '\\'; break;
        case '/': *w++ = '/'; break;
        case 'b': *w++ = '\b'; break;
        case 'f': *w++ = '\f'; break;
        case 'n': *w++ = '\n'; break;
        case 'r': *w++ = '\r'; break;
        case 't': *w++ = '\t'; break;
        case 'u':
        {
            uint32_t cp;
            if (parse_hex4(P, &cp))
            {
                P->err = "bad \\u escape";
                free(buf);
                return NULL;
            }
            if (cp >= 0xD800 && cp < 0xDC00 && P->end - P->p >= 6 && P->p[0] == '\\' && P->p[1] == 'u')
            {
                uint32_t lo;
                P->p += 2;
                if (parse_hex4(P, &lo) || lo < 0xDC00 || lo > 0xDFFF)
                {
                    P->err = "bad surrogate pair";
                    free(buf);
                    return NULL;
                }
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            put_utf8(&w, cp);
            break;
        }
        default:
            P->err = "bad escape";
            free(buf);
            return NULL;
        }
    }
    ++P->p; /* closing quote */
    *w = '\0';
    return buf;
}

static int parse_number(jparser_t *P, jnode_t *out)
{
    const char *s = P->p;
    out->t = J_NUM;
    out->negative = *s == '-';
    const char *q = s + out->negative;
    if (q >= P->end || *q < '0' || *q > '9')
    {
        P->err = "bad number";
        return -1;
    }
    if (*q == '0' && q + 1 < P->end && q[1] >= '0' && q[1] <= '9')
    {
        P->err = "leading zero";
        return -1;
    }
    while (q < P->end && *q >= '0' && *q <= '9')
        ++q;
    out->integral = 1;
    if (q < P->end && (*q == '.' || *q == 'e' || *q == 'E'))
        out->integral = 0;
    char tmp[64];
    const char *e = q;
    while (e < P->end && ((*e >= '0' && *e <= '9') || *e == '.' || *e == 'e' || *e == 'E' || *e == '+' || *e == '-'))
        ++e;
    if ((size_t)(e - s) >= sizeof tmp)
    {
        P->err = "number too long";
        return -1;
    }
    memcpy(tmp, s, (size_t)(e - s));
    tmp[e - s] = '\0';
    char *endp;
    out->d = strtod(tmp, &endp);
    if (*endp != '\0')
    {
        P->err = "bad number";
        return -1;
    }
    if (out->integral)
    {
        errno = 0;
        out->u = strtoull(tmp + out->negative, NULL, 10);
        if (errno == ERANGE)
            out->integral = 0;
    }
    P->p = e;
    return 0;
}

static int parse_container(jparser_t *P, jnode_t *out, int obj)
{
    out->t = obj ? J_OBJ : J_ARR;
    ++P->p;
    if (++P->depth > 64)
    {
        P->err = "nesting too deep";
        return -1;
    }
    skip_ws(P);
    int cap = 0;
    if (P->p < P->end && *P->p == (obj ? '}' : ']'))
    {
        ++P->p;
        --P->depth;
        return 0;
    }
    for (;;)
    {
        skip_ws(P);
        char *key = NULL;
        if (obj)
        {
            if (P->p >= P->end || *P->p != '"')
            {
                P->err = "expected a key";
                return -1;
            }
            ++P->p;
            key = keep(parse_string(P));
            if (key == NULL)
                return -1;
            skip_ws(P);
            if (P->p >= P->end || *P->p != ':')
            {
                P->err = "expected ':'";
                return -1;
            }
            ++P->p;
        }
        if (out->n == cap)
        {
            cap = cap ? 2 * cap : 8;
            jnode_t *k = (jnode_t *)realloc(out->kid, (size_t)cap * sizeof *k);
            char **ks = obj ? (char **)realloc(out->keys, (size_t)cap * sizeof *ks) : NULL;
            if (k == NULL || (obj && ks == NULL))
            {
                P->err = "out of memory";
                if (k)
                    out->kid = k;
                if (ks)
                    out->keys = ks;
                return -1;
            }
            out->kid = k;
            if (obj)
                out->keys = ks;
        }
        memset(&out->kid[out->n], 0, sizeof out->kid[0]);
        if (obj)
            out->keys[out->n] = key;
        ++out->n;
        if (parse_value(P, &out->kid[out->n - 1]))
            return -1;
        skip_ws(P);
        if (P->p < P->end && *P->p == ',')
        {
            ++P->p;
            continue;
        }
        if (P->p < P->end && *P->p == (obj ? '}' : ']'))
        {
            ++P->p;
            --P->depth;
            return 0;
        }
        P->err = obj ? "expected ',' or '}'" : "expected ',' or ']'";
        return -1;
    }
}

static int parse_value(jparser_t *P, jnode_t *out)
{
    skip_ws(P);
    if (P->p >= P->end)
    {
        P->err = "unexpected end";
        return -1;
    }
    const size_t left = (size_t)(P->end - P->p);
    switch (*P->p)
    {
    case '{': return parse_container(P, out, 1);
    case '[': return parse_container(P, out, 0);
    case '"':
        ++P->p;
        out->t = J_STR;
        out->str = keep(parse_string(P));
        return out->str ? 0 : -1;
    case 't':
        if (left >= 4 && !strncmp(P->p, "true", 4))
        {
            out->t = J_BOOL, out->boolean = 1, P->p += 4;
            return 0;
        }
        break;
    case 'f':
        if (left >= 5 && !strncmp(P->p, "false", 5))
        {
            out->t = J_BOOL, out->boolean = 0, P->p += 5;
            return 0;
        }
        break;
    case 'n':
        if (left >= 4 && !strncmp(P->p, "null", 4))
        {
            out->t = J_NULL, P->p += 4;
            return 0;
        }
        break;
    default:
        return parse_number(P, out);
    }
    P->err = "bad literal";
    return -1;
}

static void free_tree(jnode_t *n)
{
    for (int i = 0; i < n->n; ++i)
        free_tree(&n->kid[i]);
    free(n->kid);
    free(n->keys);
}

static const jnode_t *get(const jnode_t *o, const char *key)
{
    if (o == NULL || o->t != J_OBJ)
        return NULL;
    for (int i = o->n - 1; i >= 0; --i) /* a repeated key: the last one wins, as in json-c */
        if (strcmp(o->keys[i], key) == 0)
            return &o->kid[i];
    return NULL;
}

/* integer value of a number or boolean; 0 for anything else */
static int num(const jnode_t *v, uint64_t *out)
{
    if (v == NULL)
        return 0;
    if (v->t == J_BOOL)
    {
        *out = (uint64_t)v->boolean;
        return 1;
    }
    if (v->t != J_NUM)
        return 0;
    if (v->integral)
        *out = v->negative ? (uint64_t)(-(int64_t)v->u) : v->u;
    else
        *out = (uint64_t)(int64_t)v->d;
    return 1;
}

#define SET_NUM(obj, key, field, type)                 \
    do                                                 \
    {                                                  \
        uint64_t v_;                                   \
        if (num(get((obj), (key)), &v_))               \
            (field) = (type)v_;                        \
    } while (0)

static const char *str(const jnode_t *v)
{
    return v && v->t == J_STR ? v->str : NULL;
}

#define SET_STR(obj, key, field)                       \
    do                                                 \
    {                                                  \
        const jnode_t *n_ = get((obj), (key));          \
        if (n_ && (n_->t == J_STR || n_->t == J_NULL)) \
            (field) = str(n_);                         \
    } while (0)

static int load_sequence(const jnode_t *o, pb_sequence_t *s)
{
    SET_STR(o, "interface", s->interface);
    SET_NUM(o, "block", s->block, uint8_t);
    SET_NUM(o, "track", s->track, uint8_t);
    SET_NUM(o, "maxpckts", s->max_pckts, uint64_t);
    SET_NUM(o, "maxbytes", s->max_bytes, uint64_t);
    SET_NUM(o, "pps", s->pps, uint64_t);
    SET_NUM(o, "bps", s->bps, uint64_t);
    SET_NUM(o, "time", s->time, uint64_t);
    SET_NUM(o, "threads", s->threads, uint16_t);
    SET_NUM(o, "delay", s->delay, uint64_t);
    SET_NUM(o, "l4csum", s->l4_csum, uint8_t);

    const jnode_t *eth = get(o, "eth");
    SET_STR(eth, "smac", s->eth.src_mac);
    SET_STR(eth, "dmac", s->eth.dst_mac);

    const jnode_t *ip = get(o, "ip");
    SET_STR(ip, "sip", s->ip.src_ip);
    SET_STR(ip, "dip", s->ip.dst_ip);
    SET_STR(ip, "protocol", s->ip.protocol);
    SET_NUM(ip, "tos", s->ip.tos, uint8_t);
    SET_NUM(ip, "csum", s->ip.csum, uint8_t);
    const jnode_t *ttl = get(ip, "ttl");
    SET_NUM(ttl, "min", s->ip.min_ttl, uint8_t);
    SET_NUM(ttl, "max", s->ip.max_ttl, uint8_t);
    const jnode_t *id = get(ip, "id");
    SET_NUM(id, "min", s->ip.min_id, uint16_t);
    SET_NUM(id, "max", s->ip.max_id, uint16_t);
    const jnode_t *rg = get(ip, "ranges");
    if (rg && rg->t == J_ARR)
    {
        if (rg->n > PB_MAX_RANGES)
            return -E2BIG;
        s->ip.range_count = 0;
        for (int i = 0; i < rg->n; ++i)
            if (rg->kid[i].t == J_STR)
                s->ip.ranges[s->ip.range_count++] = rg->kid[i].str;
    }

    const jnode_t *udp = get(o, "udp");
    SET_NUM(udp, "sport", s->udp.src_port, uint16_t);
    SET_NUM(udp, "dport", s->udp.dst_port, uint16_t);
    const jnode_t *tcp = get(o, "tcp");
    SET_NUM(tcp, "sport", s->tcp.src_port, uint16_t);
    SET_NUM(tcp, "dport", s->tcp.dst_port, uint16_t);
    SET_NUM(tcp, "syn", s->tcp.syn, uint8_t);
    SET_NUM(tcp, "ack", s->tcp.ack, uint8_t);
    SET_NUM(tcp, "psh", s->tcp.psh, uint8_t);
    SET_NUM(tcp, "fin", s->tcp.fin, uint8_t);
    SET_NUM(tcp, "rst", s->tcp.rst, uint8_t);
    SET_NUM(tcp, "urg", s->tcp.urg, uint8_t);
    SET_NUM(tcp, "ece", s->tcp.ece, uint8_t);
    SET_NUM(tcp, "cwr", s->tcp.cwr, uint8_t);
    const jnode_t *icmp = get(o, "icmp");
    SET_NUM(icmp, "code", s->icmp.code, uint8_t);
    SET_NUM(icmp, "type", s->icmp.type, uint8_t);

    const jnode_t *pls = get(o, "payloads");
    if (pls && pls->t == J_ARR)
    {
        if (pls->n > PB_MAX_PAYLOADS)
            return -E2BIG;
        s->pl_cnt = 0;
        for (int i = 0; i < pls->n; ++i)
        {
            const jnode_t *p = &pls->kid[i];
            pb_payload_opt_t *po = &s->pls[s->pl_cnt++];
            memset(po, 0, sizeof *po);
            SET_STR(p, "exact", po->exact);
            SET_NUM(p, "isstatic", po->is_static, uint8_t);
            SET_NUM(p, "isfile", po->is_file, uint8_t);
            SET_NUM(p, "isstring", po->is_string, uint8_t);
            const jnode_t *ln = get(p, "length");
            SET_NUM(ln, "min", po->min_len, uint16_t);
            SET_NUM(ln, "max", po->max_len, uint16_t);
        }
    }
    return 0;
}

int pb_parse_config_text(const char *text, size_t len, pb_config_t *cfg, int *seq_cnt, const char **err)
{
    jparser_t P = {text, text + len, 0, NULL};
    jnode_t root;
    memset(&root, 0, sizeof root);
    int rc = parse_value(&P, &root);
    if (rc == 0)
    {
        skip_ws(&P);
        if (P.p != P.end)
            P.err = "trailing characters", rc = -1;
    }
    if (rc == 0 && root.t != J_OBJ)
        P.err = "the config is not a JSON object", rc = -1;
    if (rc != 0)
    {
        if (err)
            *err = P.err;
        free_tree(&root);
        return -EINVAL;
    }
    SET_STR(&root, "interface", cfg->interface);
    const jnode_t *seqs = get(&root, "sequences");
    int n = 0;
    if (seqs && seqs->t == J_ARR)
    {
        for (int i = 0; i < seqs->n && n < PB_MAX_SEQUENCES; ++i)
        {
            if (seqs->kid[i].t != J_OBJ)
                continue;
            rc = load_sequence(&seqs->kid[i], &cfg->seq[n]);
            if (rc)
            {
                if (err)
                    *err = "too many ranges or payloads in a sequence";
                free_tree(&root);
                return rc;
            }
            ++n;
        }
    }
    if (seq_cnt)
        *seq_cnt = n;
    free_tree(&root);
    return 0;
}

int pb_parse_config(const char *path, pb_config_t *cfg, int *seq_cnt, int log)
{
    FILE *f = fopen(path, "rb");
    if (f == NULL)
    {
        const int e = errno;
        if (log)
            fprintf(stderr, "Error opening config file %s (%s).\n", path, strerror(e));
        return -e;
    }
    char *buf = NULL;
    size_t len = 0, cap = 0;
    for (;;)
    {
        if (len + 4096 > cap)
        {
            cap = cap ? 2 * cap : 65536;
            char *b = (char *)realloc(buf, cap);
            if (b == NULL)
            {
                free(buf);
                fclose(f);
                return -ENOMEM;
            }
            buf = b;
        }
        const size_t r = fread(buf + len, 1, cap - len, f);
        len += r;
        if (r == 0)
            break;
    }
    fclose(f);
    const char *err = NULL;
    const int rc = pb_parse_config_text(buf, len, cfg, seq_cnt, &err);
    free(buf);
    if (rc && log)
        fprintf(stderr, "Error parsing config file %s: %s.\n", path, err ? err : "invalid");
    return rc;
}
