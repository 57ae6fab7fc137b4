/*
 * main_gpu.c — pcktbatch-gpu: the reference's program entry (src/main.c)
 * with the packet build on MI355X.
 *
 * Same two-pass command line as main.c:23-94 (opterr = 0; common options,
 * then optind = 0 and the AF_XDP options of cmd_line.c plus this build's GPU
 * options), the first-sequence override (-z, README.md:101-151), sequences
 * run in order through seq_send(), shutdown_prog() on exit or SIGINT/SIGTERM.
 * The JSON config (-c, default /etc/pcktbatch/conf.json) is read first and the
 * -z overrides are applied to its first sequence afterwards, as main.c:90-103
 * does with PB-Common's parse_config() / parse_cli() (host/config_json.c).
 * Frames go through a TX ring: an AF_XDP socket per thread with --tx xsk,
 * otherwise the in-memory ring of host/xsk_ring.c, whose consumer writes a pcap
 * file with --pcap (or only counts).
 */
#include <getopt.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cmd_line.h"
#include "config_json.h"
#include "sequence_gpu.h"

typedef struct cmd_line
{
    const char *config;
    int cli, list, verbose, help;
} cmd_line_t;

static pb_config_t *cfg;

static void sign_hdl(int sig)
{
    (void)sig;
    pb_request_stop();
}

enum
{
    O_INTERFACE = 256, O_BLOCK, O_TRACK, O_MAXPCKTS, O_MAXBYTES, O_PPS, O_BPS, O_DELAY, O_THREADS, O_L4CSUM, O_SMAC,
    O_DMAC, O_MINTTL, O_MAXTTL, O_MINID, O_MAXID, O_SIP, O_DIP, O_PROTOCOL, O_TOS, O_L3CSUM, O_USPORT, O_UDPORT,
    O_TSPORT, O_TDPORT, O_SYN, O_ACK, O_PSH, O_RST, O_FIN, O_URG, O_ECE, O_CWR, O_PMIN, O_PMAX, O_PSTATIC, O_PEXACT,
    O_PFILE, O_PSTRING, O_TIME, O_SECOND_PASS,
};

static const struct option common_opts[] = {
    {"cfg", required_argument, NULL, 'c'},   {"list", no_argument, NULL, 'l'},
    {"verbose", no_argument, NULL, 'v'},     {"help", no_argument, NULL, 'h'},
    {"cli", no_argument, NULL, 'z'},         {"interface", required_argument, NULL, O_INTERFACE},
    {"block", required_argument, NULL, O_BLOCK}, {"track", required_argument, NULL, O_TRACK},
    {"maxpckts", required_argument, NULL, O_MAXPCKTS}, {"maxbytes", required_argument, NULL, O_MAXBYTES},
    {"pps", required_argument, NULL, O_PPS}, {"bps", required_argument, NULL, O_BPS},
    {"delay", required_argument, NULL, O_DELAY}, {"threads", required_argument, NULL, O_THREADS},
    {"l4csum", required_argument, NULL, O_L4CSUM}, {"smac", required_argument, NULL, O_SMAC},
    {"dmac", required_argument, NULL, O_DMAC}, {"minttl", required_argument, NULL, O_MINTTL},
    {"maxttl", required_argument, NULL, O_MAXTTL}, {"minid", required_argument, NULL, O_MINID},
    {"maxid", required_argument, NULL, O_MAXID}, {"sip", required_argument, NULL, O_SIP},
    {"dip", required_argument, NULL, O_DIP}, {"protocol", required_argument, NULL, O_PROTOCOL},
    {"tos", required_argument, NULL, O_TOS}, {"l3csum", required_argument, NULL, O_L3CSUM},
    {"usport", required_argument, NULL, O_USPORT}, {"udport", required_argument, NULL, O_UDPORT},
    {"tsport", required_argument, NULL, O_TSPORT}, {"tdport", required_argument, NULL, O_TDPORT},
    {"syn", required_argument, NULL, O_SYN}, {"ack", required_argument, NULL, O_ACK},
    {"psh", required_argument, NULL, O_PSH}, {"rst", required_argument, NULL, O_RST},
    {"fin", required_argument, NULL, O_FIN}, {"urg", required_argument, NULL, O_URG},
    {"ece", required_argument, NULL, O_ECE}, {"cwr", required_argument, NULL, O_CWR},
    {"pmin", required_argument, NULL, O_PMIN}, {"pmax", required_argument, NULL, O_PMAX},
    {"pstatic", required_argument, NULL, O_PSTATIC}, {"pexact", required_argument, NULL, O_PEXACT},
    {"pfile", required_argument, NULL, O_PFILE}, {"pstring", required_argument, NULL, O_PSTRING},
    {"time", required_argument, NULL, O_TIME},
    /* parsed in the second pass (cmd_line.c); listed here so that GNU getopt's
     * argument permutation never separates them from their values */
    {"queue", required_argument, NULL, O_SECOND_PASS}, {"batchsize", required_argument, NULL, O_SECOND_PASS},
    {"nowakeup", no_argument, NULL, O_SECOND_PASS}, {"sharedumem", no_argument, NULL, O_SECOND_PASS},
    {"skb", no_argument, NULL, O_SECOND_PASS}, {"zerocopy", no_argument, NULL, O_SECOND_PASS},
    {"copy", no_argument, NULL, O_SECOND_PASS}, {"gpus", required_argument, NULL, O_SECOND_PASS},
    {"gpu", required_argument, NULL, O_SECOND_PASS}, {"gpubatch", required_argument, NULL, O_SECOND_PASS},
    {"seed", required_argument, NULL, O_SECOND_PASS}, {"literal", no_argument, NULL, O_SECOND_PASS},
    {"singlefold", no_argument, NULL, O_SECOND_PASS}, {"pcap", required_argument, NULL, O_SECOND_PASS},
    {"tx", required_argument, NULL, O_SECOND_PASS}, {"veryrandom", no_argument, NULL, O_SECOND_PASS},
    {"umemframes", required_argument, NULL, O_SECOND_PASS}, {"umemslot", required_argument, NULL, O_SECOND_PASS},
    {NULL, 0, NULL, 0},
};

/* defaults of one sequence (README.md:216-575; PB-Common clear_sequence) */
static void clear_sequence(pb_config_t *c, int i)
{
    pb_sequence_t *s = &c->seq[i];
    memset(s, 0, sizeof *s);
    s->block = 1;
    s->delay = 1000000;
    s->l4_csum = 1;
    s->ip.csum = 1;
    s->ip.min_ttl = 64;
    s->ip.max_ttl = 64;
    s->ip.max_id = 64000;
}

/* first pass: common options and the -z overrides of sequence 0 */
static void parse_common(int argc, char **argv, cmd_line_t *cmd, pb_sequence_t *s, const char **iface)
{
    int o;
    while ((o = getopt_long(argc, argv, "c:lvhz", common_opts, NULL)) != -1)
    {
        const char *a = optarg;
        switch (o)
        {
        case 'c': cmd->config = a; break;
        case 'l': cmd->list = 1; break;
        case 'v': cmd->verbose = 1; break;
        case 'h': cmd->help = 1; break;
        case 'z': cmd->cli = 1; break;
        case O_INTERFACE: *iface = a; s->interface = a; break;
        case O_BLOCK: s->block = (uint8_t)atoi(a); break;
        case O_TRACK: s->track = (uint8_t)atoi(a); break;
        case O_MAXPCKTS: s->max_pckts = strtoull(a, NULL, 10); break;
        case O_MAXBYTES: s->max_bytes = strtoull(a, NULL, 10); break;
        case O_PPS: s->pps = strtoull(a, NULL, 10); break;
        case O_BPS: s->bps = strtoull(a, NULL, 10); break;
        case O_DELAY: s->delay = strtoull(a, NULL, 10); break;
        case O_THREADS: s->threads = (uint16_t)atoi(a); break;
        case O_L4CSUM: s->l4_csum = (uint8_t)atoi(a); break;
        case O_SMAC: s->eth.src_mac = a; break;
        case O_DMAC: s->eth.dst_mac = a; break;
        case O_MINTTL: s->ip.min_ttl = (uint8_t)atoi(a); break;
        case O_MAXTTL: s->ip.max_ttl = (uint8_t)atoi(a); break;
        case O_MINID: s->ip.min_id = (uint16_t)atoi(a); break;
        case O_MAXID: s->ip.max_id = (uint16_t)atoi(a); break;
        case O_SIP: /* "one range is supported in CIDR format" (README.md:132) */
            if (strchr(a, '/'))
            {
                s->ip.ranges[0] = a;
                s->ip.range_count = 1;
                s->ip.src_ip = NULL;
            }
            else
            {
                s->ip.src_ip = a;
            }
            break;
        case O_DIP: s->ip.dst_ip = a; break;
        case O_PROTOCOL: s->ip.protocol = a; break;
        case O_TOS: s->ip.tos = (uint8_t)atoi(a); break;
        case O_L3CSUM: s->ip.csum = (uint8_t)atoi(a); break;
        case O_USPORT: s->udp.src_port = (uint16_t)atoi(a); break;
        case O_UDPORT: s->udp.dst_port = (uint16_t)atoi(a); break;
        case O_TSPORT: s->tcp.src_port = (uint16_t)atoi(a); break;
        case O_TDPORT: s->tcp.dst_port = (uint16_t)atoi(a); break;
        case O_SYN: s->tcp.syn = (uint8_t)atoi(a); break;
        case O_ACK: s->tcp.ack = (uint8_t)atoi(a); break;
        case O_PSH: s->tcp.psh = (uint8_t)atoi(a); break;
        case O_RST: s->tcp.rst = (uint8_t)atoi(a); break;
        case O_FIN: s->tcp.fin = (uint8_t)atoi(a); break;
        case O_URG: s->tcp.urg = (uint8_t)atoi(a); break;
        case O_ECE: s->tcp.ece = (uint8_t)atoi(a); break;
        case O_CWR: s->tcp.cwr = (uint8_t)atoi(a); break;
        case O_PMIN: s->pls[0].min_len = (uint16_t)atoi(a); s->pl_cnt = 1; break;
        case O_PMAX: s->pls[0].max_len = (uint16_t)atoi(a); s->pl_cnt = 1; break;
        case O_PSTATIC: s->pls[0].is_static = (uint8_t)atoi(a); s->pl_cnt = 1; break;
        case O_PEXACT: s->pls[0].exact = a; s->pl_cnt = 1; break;
        case O_PFILE: s->pls[0].is_file = (uint8_t)atoi(a); s->pl_cnt = 1; break;
        case O_PSTRING: s->pls[0].is_string = (uint8_t)atoi(a); s->pl_cnt = 1; break;
        case O_TIME: s->time = strtoull(a, NULL, 10); break;
        default: break;
        }
    }
}

static void print_cmd_help(void)
{
    fprintf(stdout, "Usage: pcktbatch-gpu -c <configfile> | -z [overrides] [-v -l -h] [AF_XDP/GPU options]\n\n"
                    "-c --cfg => Path to the config file (default /etc/pcktbatch/conf.json).\n"
                    "-l --list => Print basic information about sequences.\n"
                    "-v --verbose => Provide verbose output.\n"
                    "-h --help => Print out help menu and exit program.\n"
                    "-z --cli => Enables the first sequence/packet override (README.md first-sequence options).\n\n"
                    "AF_XDP: --queue --nowakeup --sharedumem --batchsize --skb --zerocopy --copy\n"
                    "GPU: --gpus N --gpu I --gpubatch K --seed S --veryrandom --literal --singlefold --pcap FILE --tx xsk "
                    "--umemframes N --umemslot S\n");
}

int main(int argc, char **argv)
{
    opterr = 0; /* main.c:26 */
    cmd_line_t cmd = {0};
    cfg = (pb_config_t *)calloc(1, sizeof *cfg);
    if (cfg == NULL)
        return EXIT_FAILURE;
    for (int i = 0; i < PB_MAX_SEQUENCES; ++i)
        clear_sequence(cfg, i);
    /* getopt permutes argv (the AF_XDP pass moves the values of options it does not
     * know); the -z overrides are re-read later from this untouched copy */
    char **argv_cli = (char **)malloc(((size_t)argc + 1) * sizeof *argv_cli);
    if (argv_cli == NULL)
        return EXIT_FAILURE;
    memcpy(argv_cli, argv, ((size_t)argc + 1) * sizeof *argv_cli);
    const char *iface = NULL;
    {
        /* first pass for the common flags only (main.c:30); the -z overrides are
         * applied after the config file */
        pb_sequence_t scratch;
        memset(&scratch, 0, sizeof scratch);
        parse_common(argc, argv, &cmd, &scratch, &iface);
    }
    if (cmd.help)
    {
        print_cmd_help();
        return EXIT_SUCCESS;
    }
    struct cmd_line_af_xdp cmd_af_xdp = {0};
    cmd_line_af_xdp_defaults(&cmd_af_xdp);
    optind = 0; /* main.c:45 */
    parse_cmd_line_af_xdp(&cmd_af_xdp, argc, argv);
    pb_set_verbose(cmd.verbose);
    if (pb_af_xdp_setup(&cmd_af_xdp, cmd.verbose) != 0) /* setup_af_xdp_variables (main.c:49) */
        return EXIT_FAILURE;
    /* the seed stream's base: --seed, else drawn from CLOCK_BOOTTIME (or getrandom with
     * --veryrandom) the way the reference seeds every iteration (sequence.c:434-441) */
    pb_resolve_seed(&cmd_af_xdp);

    if (cmd.config == NULL) /* main.c:51-61 */
    {
        cmd.config = "/etc/pcktbatch/conf.json";
        if (cmd.verbose)
            fprintf(stdout, "No config specified. Using default: %s.\n", cmd.config);
    }
    int seq_cnt = 0;
    if (cmd.cli)
        fprintf(stdout, "Using command line...\n");
    const int prc = pb_parse_config(cmd.config, cfg, &seq_cnt, !cmd.cli); /* main.c:94 */
    if (prc != 0 && !cmd.cli)
        return EXIT_FAILURE;
    if (cmd.cli) /* parse_cli(): the overrides of the first sequence (main.c:96-103) */
    {
        optind = 0;
        iface = NULL;
        parse_common(argc, argv_cli, &cmd, &cfg->seq[0], &iface);
        if (iface)
            cfg->interface = iface;
        if (seq_cnt < 1)
            seq_cnt = 1;
    }
    if (cmd.list)
    {
        fprintf(stdout, "AF_XDP: queue_set=%u queue=%d nowakeup=%u sharedumem=%u batchsize=%u skb=%u zerocopy=%u copy=%u\n",
                cmd_af_xdp.queue_set, cmd_af_xdp.queue, cmd_af_xdp.no_wake_up, cmd_af_xdp.shared_umem,
                cmd_af_xdp.batch_size, cmd_af_xdp.skb_mode, cmd_af_xdp.zero_copy, cmd_af_xdp.copy);
        fprintf(stdout,
                "GPU: gpus=%d gpu=%d gpubatch=%llu seed=%llu literal=%d singlefold=%d pcap=%s tx=%s umemframes=%u "
                "umemslot=%u\n",
                cmd_af_xdp.gpus, cmd_af_xdp.gpu_first, (unsigned long long)cmd_af_xdp.gpu_batch,
                (unsigned long long)cmd_af_xdp.seed_base, cmd_af_xdp.literal_payload, cmd_af_xdp.single_fold,
                cmd_af_xdp.pcap ? cmd_af_xdp.pcap : "(none)", cmd_af_xdp.tx ? cmd_af_xdp.tx : "ring",
                cmd_af_xdp.umem_frames, cmd_af_xdp.umem_slot ? cmd_af_xdp.umem_slot : 4096u);
        for (int i = 0; i < seq_cnt; ++i)
            fprintf(stdout, "Sequence #%d: %s -> %s proto %s, %u payload(s)\n", i + 1,
                    cfg->seq[i].ip.src_ip ? cfg->seq[i].ip.src_ip
                                          : (cfg->seq[i].ip.range_count ? cfg->seq[i].ip.ranges[0] : "127.0.0.1"),
                    cfg->seq[i].ip.dst_ip ? cfg->seq[i].ip.dst_ip : "(none)",
                    cfg->seq[i].ip.protocol ? cfg->seq[i].ip.protocol : "udp", cfg->seq[i].pl_cnt);
        return EXIT_SUCCESS;
    }
    fprintf(stdout, "Seed base => 0x%016llx (%s; replay with --seed 0x%llx).\n", (unsigned long long)cmd_af_xdp.seed_base,
            cmd_af_xdp.seed_set ? "--seed" : (cmd_af_xdp.very_random ? "getrandom" : "CLOCK_BOOTTIME"),
            (unsigned long long)cmd_af_xdp.seed_base);
    for (int i = 0; i < seq_cnt && cmd_af_xdp.literal_payload; ++i)
    {
        int random = 0;
        for (int j = 0; j < cfg->seq[i].pl_cnt; ++j)
            random |= cfg->seq[i].pls[j].exact == NULL && !cfg->seq[i].pls[j].is_static && cfg->seq[i].pls[j].max_len > 0;
        if (cfg->seq[i].pl_cnt > 1 && random)
            fprintf(stderr,
                    "[%d] WARNING - --literal with several payloads follows the declared rule: the shadowed loop "
                    "(sequence.c:552) reads the other payloads' setup lengths, where the reference reads the previous "
                    "iteration's (quirk B8).\n",
                    i + 1);
    }
    pb_pcap_t *pcap = NULL;
    if (cmd_af_xdp.pcap)
    {
        pcap = pb_pcap_open(cmd_af_xdp.pcap);
        if (pcap == NULL)
        {
            fprintf(stderr, "Cannot open pcap file %s.\n", cmd_af_xdp.pcap);
            return EXIT_FAILURE;
        }
        pb_set_tx_hook(pb_pcap_tx, pcap);
    }
    signal(SIGINT, sign_hdl);
    signal(SIGTERM, sign_hdl);
    for (int i = 0; i < seq_cnt && !pb_stop_requested(); ++i)
    {
        seq_send(cfg->interface, cfg->seq[i], (uint16_t)seq_cnt, cmd_af_xdp);
        /* main.c:113 (a second between sequences; PB_SEQ_GAP_MS shortens it for tests) */
        const char *gap = getenv("PB_SEQ_GAP_MS");
        const long ms = gap ? atol(gap) : 1000;
        for (long t = 0; t < ms && !pb_stop_requested(); t += 10)
        {
            struct timespec ts = {0, (ms - t < 10 ? ms - t : 10) * 1000000L};
            nanosleep(&ts, NULL);
        }
    }
    /* shutdown_prog (sequence.c:779-824) without its exit(): the pcap file is closed
     * and the memory freed before returning */
    const int err = pb_shutdown_stats(cfg);
    pb_pcap_close(pcap);
    free(cfg);
    free(argv_cli);
    pb_config_free();
    return err ? EXIT_FAILURE : EXIT_SUCCESS;
}
