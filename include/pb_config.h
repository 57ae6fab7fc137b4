/*
 * pb_config.h — the sequence/config surface the packet-build hot path reads.
 *
 * Mirror of the fields of PB-Common's `struct sequence` (config.h, un-vendored
 * submodule `modules/common`) that the reference actually dereferences.  The
 * field list is taken from the reference's own uses, not from PB-Common:
 *   eth.{src_mac,dst_mac}             src/sequence.c:67-76
 *   ip.{protocol}                     src/sequence.c:79-86
 *   ip.{tos,min_ttl,max_ttl,min_id,max_id,src_ip,dst_ip}   src/sequence.c:171-198
 *   udp.{src_port,dst_port}           src/sequence.c:208-216, 503-512
 *   tcp.{src_port,dst_port,syn..cwr}  src/sequence.c:227-245, 517-526
 *   icmp.{code,type}                  src/sequence.c:254-255
 *   pls[].{exact,is_static,is_file,is_string,min_len,max_len}, pl_cnt
 *                                     src/sequence.c:264-374, 530-561
 *   ip.{ranges,range_count}           src/sequence.c:455-497
 *   l4_csum, ip.csum                  src/sequence.c:569-602
 *   host-only: block,track,max_pckts,max_bytes,pps,bps,time,threads,delay
 *                                     src/sequence.c:389-431, 633-684, 741-771
 * Types follow the README's config table (README.md:216-575): byte=u8,
 * boolean=u8, ushort=u16, ulong=u64.
 *
 * The array bounds below are this build's own: PB-Common's MAX_PAYLOADS /
 * MAX_RANGES / MAX_SEQUENCES values are not in /root/reference.
 */
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PB_MAX_SEQUENCES 256
#define PB_MAX_PAYLOADS 64
#define PB_MAX_RANGES 64
#define PB_MAX_PCKT_LEN 0xFFFF /* src/sequence.h:38 */

typedef struct pb_payload_opt
{
    const char *exact;  /* hex string, raw string (is_string) or file path (is_file) */
    uint8_t is_static;  /* payload generated once (setup) and reused */
    uint8_t is_file;
    uint8_t is_string;
    uint16_t min_len;   /* random length range; max_len == 0 -> empty payload */
    uint16_t max_len;
} pb_payload_opt_t;

typedef struct pb_sequence
{
    /* host-only fields (pacing / stop conditions / fan-out) */
    const char *interface;
    uint8_t block;
    uint8_t track;
    uint64_t max_pckts;
    uint64_t max_bytes;
    uint64_t pps;
    uint64_t bps;
    uint64_t time;
    uint16_t threads;
    uint64_t delay;

    uint8_t l4_csum;

    struct
    {
        const char *src_mac; /* "aa:bb:cc:dd:ee:ff" or NULL */
        const char *dst_mac;
    } eth;

    struct
    {
        const char *src_ip;   /* static source, or NULL -> ranges */
        const char *dst_ip;
        const char *protocol; /* "udp" (default) / "tcp" / "icmp", case-insensitive */
        uint8_t tos;
        uint8_t csum;
        uint8_t min_ttl;
        uint8_t max_ttl;
        uint16_t min_id;
        uint16_t max_id;
        const char *ranges[PB_MAX_RANGES]; /* "<ip>/<cidr>" */
        uint16_t range_count;
    } ip;

    struct
    {
        uint16_t src_port; /* 0 -> random */
        uint16_t dst_port;
    } udp;

    struct
    {
        uint16_t src_port;
        uint16_t dst_port;
        uint8_t syn, ack, psh, fin, rst, urg, ece, cwr;
    } tcp;

    struct
    {
        uint8_t code;
        uint8_t type;
    } icmp;

    pb_payload_opt_t pls[PB_MAX_PAYLOADS];
    uint16_t pl_cnt;
} pb_sequence_t;

/* PB-Common config_t (main.c:65-94 fills it): the interface and the sequences. */
typedef struct pb_config
{
    const char *interface;
    pb_sequence_t seq[PB_MAX_SEQUENCES];
} pb_config_t;

/* Declared rules for the reference quirks that are not pinned by any
 * reference fixture (DESIGN.md "Declared rules"). */
enum pb_payload_rule
{
    PB_PAYLOAD_STREAM = 0,  /* b_j = low8(rand_r(&s)) for every j < len (intended) */
    PB_PAYLOAD_LITERAL = 1, /* as compiled: shadowed loop index (sequence.c:552) */
};

enum pb_iph_fold
{
    PB_FOLD_FULL = 0,   /* RFC 1071 end-around carry until no carry */
    PB_FOLD_SINGLE = 1, /* xdp-tutorial update_iph_checksum: one fold, truncate */
};

typedef struct pb_rules
{
    uint8_t payload_rule; /* enum pb_payload_rule */
    uint8_t iph_fold;     /* enum pb_iph_fold */
} pb_rules_t;

/* Frame-index -> seed stream (DESIGN.md "Seed stream").  The reference seeds
 * each iteration from CLOCK_BOOTTIME tv_nsec (sequence.c:434-441); parity is
 * defined over this explicit per-iteration u32 stream instead:
 *   s(seq, k) = (u32) splitmix64(seed_base ^ (((u64)seq << 48) + k)),
 * k = iteration index in [0, 2^48 - 1).  k = 2^48 - 1 is reserved for the
 * setup-time seed of "static random" payloads (sequence.c:345, quirk B2). */
#define PB_STATIC_SEED_K ((uint64_t)0xFFFFFFFFFFFFull)

#ifdef __cplusplus
}
#endif
