// pbgpu.cpp — C-ABI shim of libpbgpu.so (include/pbgpu.h).
//
// Host side of the drop-in seam: compiles a sequence (PB-Common sequence_t
// mirror, include/pb_config.h) into the GPU template once — the work the
// reference does in thread_hdl()'s prologue, src/sequence.c:66-374 — then
// launches the frame-build kernels per batch (the loop body,
// sequence.c:433-602) and lands frames in host memory for the AF_XDP TX path
// (af_xdp.c:200-227).  The product path has no CPU frame builder: if the HIP
// runtime or the device is missing every entry point fails with an error.
#include <arpa/inet.h>
#include <ctype.h>
#include <stddef.h>
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <new>
#include <deque>
#include <vector>

#include "../../include/pbgpu.h"
#include "pb_device.h"

extern "C" hipError_t pbk_launch_build(const pb_kargs *K, hipStream_t st);
extern "C" uint32_t pbk_build_grid(const pb_kargs *K);
extern "C" int pbk_batch_kind(const pb_kargs *K);
extern "C" hipError_t pbk_launch_batch(const pb_kargs *Ks, uint32_t wgt, hipStream_t st);
extern "C" hipError_t pbk_launch_ctr_fold(const uint32_t *slots, uint64_t n, uint32_t pairs,
                                          unsigned long long *counters, hipStream_t st);
extern "C" hipError_t pbk_launch_ctr_read(const unsigned long long *counters, uint32_t n_seq, unsigned long long *out,
                                          hipStream_t st);
extern "C" hipError_t pbk_launch_lengths(const pb_kargs *K, unsigned long long *block_sums, uint32_t nblocks,
                                         uint64_t *offsets, hipStream_t st);
extern "C" hipError_t pbk_launch_vst_lengths(const pb_kargs *K, uint32_t wgf, uint32_t *bsum, uint32_t nblk,
                                             unsigned long long *l2, uint32_t n_l2, uint64_t *offsets, hipStream_t st);
extern "C" hipError_t pbk_launch_expand_offsets(const uint32_t *off32, const unsigned long long *rstart, uint32_t wf,
                                                uint64_t n, uint64_t *offsets, hipStream_t st);
extern "C" hipError_t pbk_launch_scatter(const uint8_t *src, const uint64_t *offsets, uint64_t first, uint32_t n,
                                         uint8_t *dst, uint32_t stride, uint16_t *lens, hipStream_t st);
extern "C" hipError_t pbk_launch_fill(void *dst, uint64_t bytes, int mode, hipStream_t st);
extern "C" const char *pbk_fill_shape_name(int mode);
extern "C" hipError_t pbk_launch_scatter_fixed(const uint8_t *src, uint32_t flen, uint32_t wlen, uint32_t n,
                                               uint64_t src_lim, uint8_t *dst, uint32_t stride, hipStream_t st);

#define PB_JUMP_N (65536 + 256) // entries j = -PB_JNEG .. 65536 + 175
#define PB_SCAN_FRAMES_PER_BLOCK (256 * 8)
#define PB_VST_SCAN_MIN_WGF 32 // smallest pb_vstage_kernel workgroup the scratch is sized for
#define PB_CTR_WORDS ((size_t)PB_CTR_SHARDS * PB_CTR_STRIDE) // u64 counter words per sequence
#define PB_CTR_BYTES (sizeof(unsigned long long) * PB_CTR_WORDS * PB_MAX_SEQUENCES)

// device scratch of a frames buffer: the 3-pass length scan's block sums, or pb_vstage_kernel's
// per-workgroup length sums (u32) + their per-PB_VL_GRP group sums (u64)
static uint64_t vst_bsum_bytes(uint64_t nblk)
{
    return (nblk * 4 + 15) & ~15ull;
}
static uint64_t scan_tmp_bytes(uint64_t capacity_frames)
{
    const uint64_t a = (capacity_frames / PB_SCAN_FRAMES_PER_BLOCK + 1) * 8;
    const uint64_t nblk = capacity_frames / PB_VST_SCAN_MIN_WGF + 1;
    const uint64_t b = vst_bsum_bytes(nblk) + (nblk / PB_VL_GRP + 1) * 8;
    return a > b ? a : b;
}

namespace
{

// Shape overrides for the parity tests and A/B runs (PBGPU_* environment).  They are read in
// one place, read_opts(): at pbgpu_open into the context (landing and batch options) and at
// pbgpu_load_sequence into the slot (kernel shapes), so the build path never reads the
// environment and a loaded sequence's shape is fixed.  Every selectable shape is parity-tested
// (tests/test_gpu_kernels.py).
enum pb_kern_force
{
    PBO_K_AUTO = 0,
    PBO_K_GPF,    // PBGPU_KERNEL=gpf: the group-per-frame kernel for frames > 128 B
    PBO_K_STAGE,  // =stage: pb_stage_kernel
    PBO_K_VSTAGE, // =vstage: pb_vstage_kernel for packed variable lengths
    PBO_K_NOPAGE, // =nopage: no pb_xpage_kernel (linear small kernel)
    PBO_K_LINEAR, // =linear: neither page kernel
    PBO_K_VPAGE,  // =vpage: the page-shaped packed writer (pb_vrec_kernel + pb_vpage_kernel)
};

struct pb_opts
{
    int kernel = PBO_K_AUTO;
    uint32_t g = 0;          // PBGPU_G: lanes per frame of the staged / group kernels (8, 16, 32, 64)
    uint32_t fpw = 0;        // PBGPU_FPW: frames per workgroup of the group kernel / staged window
    uint32_t wgt = 0;        // PBGPU_WGT=64: one-wave staged workgroups
    uint32_t wgf = 0;        // PBGPU_WGF: staged frames per workgroup
    uint32_t stage_kb = 0;   // PBGPU_STAGE_KB: staged window
    uint32_t small_wgt = 0;  // PBGPU_SMALL_WGT: linear small kernel's workgroup (64 / 128 / 256)
    uint32_t fst_g = 0, fst_wgf = 0, fst_nbuf = 0; // PBGPU_FST_G / _WGF / _NBUF
    uint32_t vl_wgf = 0;     // PBGPU_VL_WGF: pb_vline_kernel's own frames per workgroup
    uint32_t vst_shape = 0;  // PBGPU_VST_SHAPE: pb_vstage_kernel shape bits (pb_kargs.vst_shape)
    bool vst_scan3 = false;  // PBGPU_VST_SCAN=3pass: pb_vstage_kernel after the 3-pass length scan
    bool xp_force = false;   // PBGPU_XP_FORCE=1: pb_xpage_kernel for every even length <= 128 B
    bool xp_static = true;   // PBGPU_XP_STATIC=0: no page kernel for static payloads
    bool xp_fa64 = false;    // PBGPU_XP_FA64=1: pb_xpage_kernel's 64-bit first-frame path at any size
    uint32_t xp_wgt = 0;     // PBGPU_XP_WGT: 256 / 512
    uint32_t xp_np = 0;      // PBGPU_XP_NP: pages per workgroup
    uint32_t xp_img = 1;     // static-payload ICMP frames: 1 pb_ximg_body in pb_batch_kernel only,
                             // 2 pb_ximg_kernel for single builds too, 0 never (PBGPU_XP_IMG)
    bool ctr_atomic = false; // PBGPU_CTR_ATOMIC=1: counts by one atomic per workgroup, no record ring
    uint32_t ctr_ring = 0;   // PBGPU_CTR_RING: record ring words (small: the fold-when-full path)
    bool batch = true;       // PBGPU_BATCH=0: pbgpu_build_batch launches every part on its own
    uint32_t batch_wgt = 512; // PBGPU_BATCH_WGT=256: pb_batch_kernel's 256-thread form
    bool seq_streams = true; // PBGPU_SEQ_STREAMS=0: span-mode builds all on the context's stream
    bool land_spin = true;   // PBGPU_LAND_SPIN=0: blocking landing waits
    bool umem_dma = false;   // PBGPU_UMEM_DMA=1: land through DMA copies, not the mapped scatter
    bool alloc_vmm = true;   // PBGPU_ALLOC=malloc: frame buffers from hipMalloc (fb_alloc)
    uint32_t alloc_chunk_mb = 64; // PBGPU_ALLOC_CHUNK_MB: fb_alloc's physical chunk
    uint32_t land_dma_min = 0xFFFFFFFFu; // PBGPU_LAND_DMA_MIN: fixed frames of at least this many bytes
                                  // land in registered UMEM by strided DMA instead of the scatter kernel
                                  // (off by default: 1500 B read 56 vs 52 GB/s landing alone on one box,
                                  // 43 vs 49 GB/s in bench.py's build + land on another)
    uint32_t vp_pages_pct = 0; // PBGPU_VP_PAGES_PCT: pb_vpage_kernel's grid as a percentage of the
                               // expected pages (tests: a short grid, so waves take several pages)
};

uint32_t opt_u32(const char *name)
{
    const char *e = getenv(name);
    return e != NULL && atoi(e) > 0 ? (uint32_t)atoi(e) : 0u;
}

bool opt_is(const char *name, const char *value)
{
    const char *e = getenv(name);
    return e != NULL && strcmp(e, value) == 0;
}

pb_opts read_opts()
{
    pb_opts o;
    const char *k = getenv("PBGPU_KERNEL");
    if (k)
        o.kernel = !strcmp(k, "gpf") ? PBO_K_GPF
                   : !strcmp(k, "stage") ? PBO_K_STAGE
                   : !strcmp(k, "vstage") ? PBO_K_VSTAGE
                   : !strcmp(k, "nopage") ? PBO_K_NOPAGE
                   : !strcmp(k, "linear") ? PBO_K_LINEAR
                   : !strcmp(k, "vpage") ? PBO_K_VPAGE
                                          : PBO_K_AUTO;
    o.g = opt_u32("PBGPU_G");
    if (o.g != 8 && o.g != 16 && o.g != 32 && o.g != 64)
        o.g = 0;
    o.fpw = opt_u32("PBGPU_FPW");
    o.wgt = opt_u32("PBGPU_WGT");
    o.wgf = opt_u32("PBGPU_WGF");
    o.stage_kb = opt_u32("PBGPU_STAGE_KB");
    o.small_wgt = opt_u32("PBGPU_SMALL_WGT");
    o.fst_g = opt_u32("PBGPU_FST_G");
    o.fst_wgf = opt_u32("PBGPU_FST_WGF");
    o.fst_nbuf = opt_u32("PBGPU_FST_NBUF");
    o.vl_wgf = opt_u32("PBGPU_VL_WGF");
    o.vst_shape = opt_u32("PBGPU_VST_SHAPE");
    o.vst_scan3 = opt_is("PBGPU_VST_SCAN", "3pass");
    o.xp_force = opt_is("PBGPU_XP_FORCE", "1");
    o.xp_static = !opt_is("PBGPU_XP_STATIC", "0");
    o.xp_fa64 = opt_is("PBGPU_XP_FA64", "1");
    o.xp_wgt = opt_u32("PBGPU_XP_WGT");
    o.xp_np = opt_u32("PBGPU_XP_NP");
    if (getenv("PBGPU_XP_IMG"))
        o.xp_img = opt_is("PBGPU_XP_IMG", "2") ? 2u : opt_is("PBGPU_XP_IMG", "0") ? 0u : 1u;
    o.ctr_atomic = opt_is("PBGPU_CTR_ATOMIC", "1");
    o.ctr_ring = opt_u32("PBGPU_CTR_RING");
    o.batch = !opt_is("PBGPU_BATCH", "0");
    o.batch_wgt = opt_u32("PBGPU_BATCH_WGT") == 256 ? 256u : 512u;
    o.seq_streams = !opt_is("PBGPU_SEQ_STREAMS", "0");
    o.land_spin = !opt_is("PBGPU_LAND_SPIN", "0");
    o.umem_dma = getenv("PBGPU_UMEM_DMA") != NULL;
    o.alloc_vmm = !opt_is("PBGPU_ALLOC", "malloc");
    o.vp_pages_pct = opt_u32("PBGPU_VP_PAGES_PCT");
    if (getenv("PBGPU_LAND_DMA_MIN"))
        o.land_dma_min = (uint32_t)atoi(getenv("PBGPU_LAND_DMA_MIN"));
    if (opt_u32("PBGPU_ALLOC_CHUNK_MB"))
        o.alloc_chunk_mb = opt_u32("PBGPU_ALLOC_CHUNK_MB");
    return o;
}

int verbose()
{
    static int v = -1;
    if (v < 0)
        v = getenv("PBGPU_VERBOSE") != NULL;
    return v;
}

#define HIPCHK(call)                                                                         \
    do                                                                                       \
    {                                                                                        \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
        {                                                                                    \
            if (verbose())                                                                   \
                fprintf(stderr, "[pbgpu] %s:%d %s -> %s\n", __FILE__, __LINE__, #call,       \
                        hipGetErrorString(e_));                                              \
            return PBGPU_EIO;                                                                \
        }                                                                                    \
    } while (0)

struct seq_slot
{
    bool loaded = false;
    pb_kargs K;              // template part; per-launch fields patched in pbgpu_build
    uint32_t fpi = 1;        // frames per iteration
    uint32_t min_flen = 0, max_flen = 0;
    uint2 *d_ranges = nullptr;
    pb_pl *d_pls = nullptr;
    uint32_t *d_lit_stop = nullptr;
    uint8_t *d_blob = nullptr;
    uint32_t *d_img = nullptr; // pb_ximg_kernel's pages (K.img)
    // per-workgroup counts of the launches not yet folded into the counters (pb_count): a
    // linear ring of u32 words, folded (pb_ctr_fold) when full, on reload and by pbgpu_counters
    uint32_t *d_ctr_slots = nullptr;
    uint64_t ctr_cap = 0, ctr_used = 0, ctr_pairs = 1; // words; words per record
    hipStream_t ctr_last = nullptr; // the stream of the last launch that wrote or folded the ring
    hipEvent_t ctr_ev = nullptr;
    pb_opts opt; // shape overrides, read when the sequence was loaded
};

struct timing_pair
{
    hipEvent_t a, b;
};

#define PB_SEQ_STREAMS 4

// What pbgpu_frames.reserved points to: the buffer's build-completion event (the landing
// stream waits on it) and the completion event of the last landing queued from it (the
// next build into the buffer waits on that, so a landing never reads frames being rebuilt)
struct frames_events
{
    hipEvent_t built = nullptr;
    hipEvent_t landed = nullptr;
    bool land_pending = false;
    hipStream_t last = nullptr; // the stream the buffer was last built on
    hipEvent_t moved = nullptr; // a build on another stream waits on this (recorded on `last`)
    // pb_vline_kernel writes 4-B offsets and region starts here; offsets[] is expanded from them
    // on first use (packed32 set until then)
    uint32_t *d_off32 = nullptr;
    unsigned long long *d_rstart = nullptr;
    // pb_vrec_kernel's records and page table (pb_vpage_kernel), allocated on first use
    uint2 *d_vrec = nullptr;
    uint2 *d_vpt = nullptr;
    bool packed32 = false;
    uint32_t wf = 0;
};

frames_events *frames_ev(pbgpu_frames *f)
{
    if (f->reserved == NULL)
        f->reserved = new (std::nothrow) frames_events();
    return (frames_events *)f->reserved;
}

} // namespace

struct pbgpu_ctx
{
    int device = 0;
    hipStream_t stream = nullptr;      // frame builds
    hipStream_t land_stream = nullptr; // UMEM landing: overlaps the next build (pbgpu_copy_to_umem)
    bool land_events = false;          // set by the first landing: builds then record a completion event
    pb_opts opt;                       // read at pbgpu_open: landing, stream and batch options
    uint2 *d_jump = nullptr;
    uint2 *d_lcg48 = nullptr;
    uint32_t *d_orbit = nullptr; // pb_vline_kernel: LCG-orbit prefix sums (built on first use, 2 MiB)
    uint32_t *d_dlog12 = nullptr; // pb_orbit_sum's discrete log mod 2^12 (16 KiB)
    uint2 *d_lcg48i = nullptr;    // pb_vpage_kernel: L^(-48 c), c < PB_VP_NCI
    uint4 *d_m16 = nullptr;       // pb_vpage_kernel: chunk byte masks by plo + phi
    uint32_t orbit_tot = 0;
    unsigned long long *d_counters = nullptr; // [PB_MAX_SEQUENCES][PB_CTR_SHARDS][PB_CTR_STRIDE]
    // the shard sums {frames, bytes} per sequence, written by pb_ctr_read into mapped pinned host
    // memory (h_ctr_sum; d_ctr_sum its device address)
    unsigned long long *h_ctr_sum = nullptr, *d_ctr_sum = nullptr;
    unsigned long long *d_img_ctr = nullptr; // counters of the load-time pb_ximg_kernel page builds (never read)
    seq_slot seqs[PB_MAX_SEQUENCES];
    std::vector<timing_pair> pending;
    std::vector<timing_pair> pool;
    int timing_mode = PBGPU_TIMING_LAUNCH;
    timing_pair span = {nullptr, nullptr}; // PBGPU_TIMING_SPAN: first-launch / call events
    uint32_t span_n = 0;                    // launches in the open span (0: none open)
    // PBGPU_TIMING_SPAN: the builds of sequence i run on seq_stream[i % PB_SEQ_STREAMS], so the
    // kernels of different sequences overlap (as the reference's non-blocking sequences run
    // their threads side by side, sequence.c:741-765); every other call first joins them
    // into `stream` (one event per stream that built since the last join)
    // counts of a slot's earlier sequences (folded in when the slot is loaded again)
    uint64_t ctr_base[PB_MAX_SEQUENCES][2] = {};
    hipStream_t seq_stream[PB_SEQ_STREAMS] = {};
    hipEvent_t seq_join[PB_SEQ_STREAMS] = {};
    bool seq_dirty[PB_SEQ_STREAMS] = {};
    bool seq_in_span[PB_SEQ_STREAMS] = {}; // has waited on span.a since it was recorded
    uint8_t *h_stage = nullptr;
    uint16_t *d_lens = nullptr; // landing: frame lengths of the mapped scatter (device), a ring
    uint16_t *h_lens = nullptr; // ... and their pinned host copy
    uint32_t lens_cap = 0;
    uint32_t lens_head = 0;     // next free entry of the ring
    size_t h_stage_bytes = 0;
    struct land_op
    {
        hipEvent_t ev;
        uint16_t *lens_out;
        uint32_t n;
        uint32_t lens_off; // variable length: entries [lens_off, lens_off + n) of the lens ring
        uint32_t fixed_len;
    };
    std::deque<land_op> landings;      // queued, not yet waited for (FIFO)
    std::vector<hipEvent_t> land_pool; // recycled landing events
    struct reg
    {
        uint8_t *host;
        size_t bytes;
        uint8_t *dev;
    };
    std::vector<reg> regs; // pbgpu_host_register'ed ranges and their device addresses
};

namespace
{

uint32_t host_rand_r(uint32_t *seed)
{
    uint32_t x = *seed, r;
    x = x * PB_LCG_A + PB_LCG_C;
    r = (x >> 16) & 0x7FFu;
    x = x * PB_LCG_A + PB_LCG_C;
    r = (r << 10) ^ ((x >> 16) & 0x3FFu);
    x = x * PB_LCG_A + PB_LCG_C;
    r = (r << 10) ^ ((x >> 16) & 0x3FFu);
    *seed = x;
    return r;
}

uint32_t host_seed(uint64_t seed_base, uint32_t seq, uint64_t k)
{
    uint64_t z = (seed_base ^ (((uint64_t)seq << 48) + k)) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)(z ^ (z >> 31));
}

pb_div make_div(uint32_t d)
{
    pb_div v;
    v.d = d;
    uint32_t l = 0;
    while ((1ull << l) < d)
        ++l;
    v.sh = 31 + l;
    v.m = (uint32_t)(((1ull << v.sh) + d - 1) / d);
    return v;
}

// jump[j + PB_JNEG] = L^(3(j+1)) as (A, C), j = -PB_JNEG ..
std::vector<uint2> make_jump_table()
{
    const uint32_t a = PB_LCG_A, c = PB_LCG_C;
    uint32_t ainv = a; // Newton: a * ainv == 1 mod 2^32
    for (int i = 0; i < 5; ++i)
        ainv *= 2u - a * ainv;
    // inverse step y -> ainv * (y - c)
    const uint32_t ia = ainv, ic = (uint32_t)(0u - ainv * c);
    // first entry: j = -PB_JNEG -> L^(3(1 - PB_JNEG))
    uint32_t A = 1, C = 0;
    for (int i = 0; i < 3 * (PB_JNEG - 1); ++i)
    {
        A = ia * A;
        C = ia * C + ic;
    }
    const uint32_t a3 = a * a * a, c3 = c * (a * a + a + 1u);
    std::vector<uint2> t(PB_JUMP_N);
    for (int j = 0; j < PB_JUMP_N; ++j)
    {
        t[j] = make_uint2(A, C);
        A = a3 * A;
        C = a3 * C + c3;
    }
    return t;
}

// pb_vline_kernel's payload sums (pbgpu_kernels.hip, pb_orbit_sum): M = L^3 mod 2^24 walks one
// orbit of all 2^24 states from 0 (full period: c odd, a = 1 mod 4); entry t holds the sums of
// the bytes (bits 16-23) at the even and the odd positions before t << PB_ORB_SH, mod 0xFFFF,
// as two u16.
std::vector<uint32_t> make_orbit_table(uint32_t *total)
{
    const uint32_t m = 0xFFFFFFu;
    const uint32_t a3 = (PB_LCG_A * PB_LCG_A * PB_LCG_A) & m, c3 = (PB_LCG_C * (PB_LCG_A * PB_LCG_A + PB_LCG_A + 1u)) & m;
    std::vector<uint32_t> t((1u << (24 - PB_ORB_SH)) + 1);
    uint32_t y = 0, pe = 0, po = 0;
    for (uint32_t k = 0; k < (1u << 24); ++k)
    {
        if ((k & ((1u << PB_ORB_SH) - 1u)) == 0)
            t[k >> PB_ORB_SH] = pe | (po << 16);
        const uint32_t b = (y >> 16) & 0xFFu;
        if (k & 1u)
            po = (po + b) % 0xFFFFu;
        else
            pe = (pe + b) % 0xFFFFu;
        y = (a3 * y + c3) & m;
    }
    t[1u << (24 - PB_ORB_SH)] = pe | (po << 16);
    *total = pe; // the even and odd totals are equal (each byte value 2^15 times per parity)
    return t;
}

int str_ieq(const char *a, const char *b)
{
    for (; *a && *b; a++, b++)
        if (tolower((unsigned char)*a) != tolower((unsigned char)*b))
            return 0;
    return *a == *b;
}

void parse_mac(const char *s, uint8_t mac[6])
{
    memset(mac, 0, 6);
    if (s)
        sscanf(s, "%hhx:%hhx:%hhx:%hhx:%hhx:%hhx", &mac[0], &mac[1], &mac[2], &mac[3], &mac[4], &mac[5]);
}

// "<ip>/<cidr>" (strtok semantics, as PB-Common rand_ip splits it); invalid
// ranges take the reference's fail path, 127.0.0.1 (sequence.c:473-482).
uint2 compile_range(const char *r)
{
    uint2 out = make_uint2(0x7F000001u, 0u);
    if (r == NULL)
        return out;
    char *cpy = strdup(r);
    if (cpy == NULL)
        return out;
    char *save = NULL;
    char *ip = strtok_r(cpy, "/", &save);
    char *cs = strtok_r(NULL, "/", &save);
    struct in_addr a;
    if (ip && cs && inet_aton(ip, &a))
    {
        int cidr = atoi(cs);
        if (cidr >= 0 && cidr <= 32)
        {
            uint32_t hm = cidr == 0 ? 0xFFFFFFFFu : (cidr == 32 ? 0u : ((1u << (32 - cidr)) - 1u));
            out = make_uint2(ntohl(a.s_addr) & ~hm, hm);
        }
    }
    free(cpy);
    return out;
}

// exact payload text -> bytes (sequence.c:269-337)
int compile_exact(const pb_payload_opt_t *po, std::vector<uint8_t> &bytes)
{
    std::vector<char> text;
    if (po->is_file)
    {
        FILE *fp = fopen(po->exact, "rb");
        if (fp)
        {
            fseek(fp, 0, SEEK_END);
            long n = ftell(fp);
            fseek(fp, 0, SEEK_SET);
            text.assign(n > 0 ? (size_t)n + 1 : 1, 0);
            if (n > 0 && fread(text.data(), 1, (size_t)n, fp) != (size_t)n)
                text.assign(1, 0);
            fclose(fp);
        }
        else
        {
            text.assign(1, 0);
        }
    }
    else
    {
        size_t n = strlen(po->exact);
        text.assign(po->exact, po->exact + n + 1);
    }
    bytes.clear();
    if (po->is_string)
    {
        size_t n = strlen(text.data());
        bytes.assign(text.data(), text.data() + n);
    }
    else
    {
        char *rest = text.data(), *tok;
        while ((tok = strtok_r(rest, " ", &rest)) != NULL)
        {
            unsigned char b = 0;
            sscanf(tok, "%2hhx", &b);
            bytes.push_back(b);
        }
    }
    return bytes.size() > PB_MAX_PCKT_LEN ? PBGPU_EINVAL : PBGPU_OK;
}

uint32_t le_word_sum(const uint8_t *p, size_t n)
{
    uint64_t s = 0;
    for (size_t j = 0; j < n; ++j)
        s += (uint64_t)p[j] << ((j & 1) * 8);
    while (s >> 16)
        s = (s & 0xFFFF) + (s >> 16);
    return (uint32_t)s;
}

template <typename T>
int upload(T **dptr, const T *src, size_t n)
{
    if (*dptr)
        (void)hipFree(*dptr);
    *dptr = nullptr;
    if (n == 0)
    {
        // an empty table is a zeroed 256-B allocation, never a null device pointer
        HIPCHK(hipMalloc((void **)dptr, 256));
        HIPCHK(hipMemset(*dptr, 0, 256));
        return PBGPU_OK;
    }
    HIPCHK(hipMalloc((void **)dptr, n * sizeof(T)));
    HIPCHK(hipMemcpy(*dptr, src, n * sizeof(T), hipMemcpyHostToDevice));
    return PBGPU_OK;
}

// Dynamic LDS that caps a launch at per_cu workgroups per CU: total LDS per workgroup just over
// 160 KiB / (per_cu + 1).  (The measured shape: 64-B pages with 41,384 B per workgroup ran 0.29-0.30
// ms per 2^25 frames, with 46,592 B 0.35 ms like 2 per CU, profiles/r05/ab/xs9.jsonl, so the
// point just past the next count's boundary is the one to take.)
#define PB_LDS_PER_CU (160u * 1024u)
#define PB_XS_WG_PER_CU 3 // pb_xsmall_kernel
uint32_t lds_cap_pad(uint32_t static_bytes, uint32_t per_cu)
{
    const uint32_t target = PB_LDS_PER_CU / (per_cu + 1u) + 512u;
    return target > static_bytes ? target - static_bytes : 0u;
}

void slot_free(seq_slot &s)
{
    if (s.d_ranges)
        (void)hipFree(s.d_ranges);
    if (s.d_pls)
        (void)hipFree(s.d_pls);
    if (s.d_lit_stop)
        (void)hipFree(s.d_lit_stop);
    if (s.d_blob)
        (void)hipFree(s.d_blob);
    if (s.d_img)
        (void)hipFree(s.d_img);
    s = seq_slot();
}

} // namespace

extern "C" {

const char *pbgpu_strerror(int err)
{
    switch (err)
    {
    case PBGPU_OK: return "ok";
    case PBGPU_ENOENT: return "sequence not loaded";
    case PBGPU_EIO: return "HIP runtime error";
    case PBGPU_ENOMEM: return "out of memory";
    case PBGPU_EINVAL: return "invalid argument or sequence";
    case PBGPU_ENOSPC: return "frames buffer too small";
    case PBGPU_ENODEV: return "no such GPU";
    case PBGPU_ENOTSUP: return "sequence not supported on the GPU path";
    default: return "unknown error";
    }
}

int pbgpu_device_count(int *n)
{
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess)
        c = 0;
    *n = c;
    return PBGPU_OK;
}

// The sequence builds issued since the last join, ordered before what follows on ctx->stream.
static int join_builds(pbgpu_ctx *ctx)
{
    for (int i = 0; i < PB_SEQ_STREAMS; ++i)
        if (ctx->seq_dirty[i])
        {
            if (ctx->seq_join[i] == nullptr)
                HIPCHK(hipEventCreateWithFlags(&ctx->seq_join[i], hipEventDisableTiming));
            HIPCHK(hipEventRecord(ctx->seq_join[i], ctx->seq_stream[i]));
            HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->seq_join[i], 0));
            ctx->seq_dirty[i] = false;
        }
    return PBGPU_OK;
}

static void slot_counts(const pbgpu_ctx *ctx, const unsigned long long *sum, int i, uint64_t *p, uint64_t *b);
static int read_counter_sums(pbgpu_ctx *ctx, int first, int n_seq);

// Launches that touch a sequence's count ring (its builds and folds) run in order, whatever
// stream each is issued on: the next one waits for the previous one's stream.
static int ctr_order(seq_slot &S, hipStream_t st)
{
    if (S.ctr_last && S.ctr_last != st)
    {
        if (S.ctr_ev == nullptr)
            HIPCHK(hipEventCreateWithFlags(&S.ctr_ev, hipEventDisableTiming));
        HIPCHK(hipEventRecord(S.ctr_ev, S.ctr_last));
        HIPCHK(hipStreamWaitEvent(st, S.ctr_ev, 0));
    }
    S.ctr_last = st;
    return PBGPU_OK;
}

// Adds the records of slot i's launches since the last fold into its counters (on st).
static int ctr_fold(pbgpu_ctx *ctx, int i, hipStream_t st)
{
    seq_slot &S = ctx->seqs[i];
    if (S.ctr_used == 0)
        return PBGPU_OK;
    const int rc = ctr_order(S, st);
    if (rc != PBGPU_OK)
        return rc;
    HIPCHK(pbk_launch_ctr_fold(S.d_ctr_slots, S.ctr_used / S.ctr_pairs, (uint32_t)S.ctr_pairs,
                               ctx->d_counters + PB_CTR_WORDS * (size_t)i, st));
    S.ctr_used = 0;
    return PBGPU_OK;
}

static void ctr_free(seq_slot &S)
{
    if (S.d_ctr_slots)
        (void)hipFree(S.d_ctr_slots);
    if (S.ctr_ev)
        (void)hipEventDestroy(S.ctr_ev);
    S.d_ctr_slots = nullptr;
    S.ctr_ev = nullptr;
    S.ctr_cap = S.ctr_used = 0;
    S.ctr_last = nullptr;
}

#define PB_CTR_RING_WORDS (8ull << 20) // count ring per sequence: 32 MiB, 64 launches of 2^25 64-B frames

#define PB_JOIN(ctx)                         \
    do                                       \
    {                                        \
        const int jrc_ = join_builds(ctx);   \
        if (jrc_ != PBGPU_OK)                \
            return jrc_;                     \
    } while (0)

int pbgpu_open(int device, pbgpu_ctx **out)
{
    if (out == NULL)
        return PBGPU_EINVAL;
    *out = NULL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return PBGPU_ENODEV;
    HIPCHK(hipSetDevice(device));
    pbgpu_ctx *ctx = new pbgpu_ctx();
    ctx->device = device;
    ctx->opt = read_opts();
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->land_stream, hipStreamNonBlocking) != hipSuccess)
    {
        if (ctx->stream)
            (void)hipStreamDestroy(ctx->stream);
        delete ctx;
        return PBGPU_EIO;
    }
    std::vector<uint2> jt = make_jump_table();
    std::vector<uint2> l48(PB_LCG48_N);
    {
        const uint32_t a3 = PB_LCG_A * PB_LCG_A * PB_LCG_A, c3 = PB_LCG_C * (PB_LCG_A * PB_LCG_A + PB_LCG_A + 1u);
        uint32_t A16 = 1, C16 = 0; // L^48 = (L^3)^16
        for (int i = 0; i < 16; ++i)
            C16 = a3 * C16 + c3, A16 = a3 * A16;
        uint32_t A = 1, C = 0;
        for (int m = 0; m < PB_LCG48_N; ++m)
        {
            l48[m] = make_uint2(A, C);
            A = A16 * A;
            C = A16 * C + C16;
        }
    }
    // L^(-48 c) (pb_vpage_kernel) and the discrete log of M = L^3 mod 2^12 (pb_orbit_sum)
    std::vector<uint2> l48i(PB_VP_NCI);
    std::vector<uint32_t> dlog12(4096);
    std::vector<uint4> m16(PB_VL_NMASK);
    for (int j = 0; j < PB_VL_NMASK; ++j) // bytes [lo, hi) of a 16-B chunk: j = lo + hi
    {
        const int lo = j > 16 ? j - 16 : 0, hi = j > 16 ? 16 : j;
        uint32_t w[4];
        for (int t = 0; t < 4; ++t)
        {
            w[t] = 0;
            for (int b = 0; b < 4; ++b)
                if (4 * t + b >= lo && 4 * t + b < hi)
                    w[t] |= 0xFFu << (8 * b);
        }
        m16[j] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    {
        uint32_t ai = PB_LCG_A; // PB_LCG_A^-1 mod 2^32 (Newton)
        for (int i = 0; i < 5; ++i)
            ai *= 2u - PB_LCG_A * ai;
        const uint32_t ci = 0u - ai * PB_LCG_C; // L^-1(x) = ai x + ci
        uint32_t A48 = 1, C48 = 0;
        for (int i = 0; i < 48; ++i)
            C48 = ai * C48 + ci, A48 = ai * A48;
        uint32_t A = 1, C = 0;
        for (uint32_t m = 0; m < PB_VP_NCI; ++m)
        {
            l48i[m] = make_uint2(A, C);
            A = A48 * A;
            C = A48 * C + C48;
        }
        const uint32_t a3 = (PB_LCG_A * PB_LCG_A * PB_LCG_A) & 0xFFFFFFu;
        const uint32_t c3 = (PB_LCG_C * (PB_LCG_A * PB_LCG_A + PB_LCG_A + 1u)) & 0xFFFFFFu;
        uint32_t x = 0;
        for (uint32_t j = 0; j < 4096; ++j)
        {
            dlog12[x & 0xFFFu] = j | (x & 0xFFF000u);
            x = (a3 * x + c3) & 0xFFFFFFu;
        }
    }
    if (upload(&ctx->d_jump, jt.data(), jt.size()) != PBGPU_OK || upload(&ctx->d_lcg48, l48.data(), l48.size()) != PBGPU_OK ||
        upload(&ctx->d_lcg48i, l48i.data(), l48i.size()) != PBGPU_OK ||
        upload(&ctx->d_dlog12, dlog12.data(), dlog12.size()) != PBGPU_OK ||
        upload(&ctx->d_m16, m16.data(), m16.size()) != PBGPU_OK ||
        hipMalloc((void **)&ctx->d_counters, PB_CTR_BYTES) != hipSuccess ||
        hipMemset(ctx->d_counters, 0, PB_CTR_BYTES) != hipSuccess ||
        hipHostMalloc((void **)&ctx->h_ctr_sum, 2 * sizeof(unsigned long long) * PB_MAX_SEQUENCES,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&ctx->d_ctr_sum, ctx->h_ctr_sum, 0) != hipSuccess)
    {
        pbgpu_close(ctx);
        return PBGPU_EIO;
    }
    *out = ctx;
    return PBGPU_OK;
}

void pbgpu_close(pbgpu_ctx *ctx)
{
    if (ctx == NULL)
        return;
    (void)hipSetDevice(ctx->device);
    for (int i = 0; i < PB_SEQ_STREAMS; ++i)
        if (ctx->seq_stream[i])
            (void)hipStreamSynchronize(ctx->seq_stream[i]);
    if (ctx->stream)
        (void)hipStreamSynchronize(ctx->stream);
    if (ctx->land_stream)
        (void)hipStreamSynchronize(ctx->land_stream);
    (void)pbgpu_land_wait(ctx, 0);
    for (hipEvent_t e : ctx->land_pool)
        (void)hipEventDestroy(e);
    for (auto &s : ctx->seqs)
    {
        ctr_free(s);
        slot_free(s);
    }
    for (auto &p : ctx->pending)
        ctx->pool.push_back(p);
    for (auto &p : ctx->pool)
    {
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    if (ctx->span.a)
    {
        (void)hipEventDestroy(ctx->span.a);
        (void)hipEventDestroy(ctx->span.b);
    }
    if (ctx->d_jump)
        (void)hipFree(ctx->d_jump);
    if (ctx->d_lcg48)
        (void)hipFree(ctx->d_lcg48);
    if (ctx->d_orbit)
        (void)hipFree(ctx->d_orbit);
    if (ctx->d_dlog12)
        (void)hipFree(ctx->d_dlog12);
    if (ctx->d_lcg48i)
        (void)hipFree(ctx->d_lcg48i);
    if (ctx->d_m16)
        (void)hipFree(ctx->d_m16);
    if (ctx->d_counters)
        (void)hipFree(ctx->d_counters);
    if (ctx->h_ctr_sum)
        (void)hipHostFree(ctx->h_ctr_sum);
    if (ctx->d_img_ctr)
        (void)hipFree(ctx->d_img_ctr);
    if (ctx->h_stage)
        (void)hipHostFree(ctx->h_stage);
    if (ctx->d_lens)
        (void)hipFree(ctx->d_lens);
    if (ctx->h_lens)
        (void)hipHostFree(ctx->h_lens);
    for (int i = 0; i < PB_SEQ_STREAMS; ++i)
    {
        if (ctx->seq_join[i])
            (void)hipEventDestroy(ctx->seq_join[i]);
        if (ctx->seq_stream[i])
            (void)hipStreamDestroy(ctx->seq_stream[i]);
    }
    if (ctx->stream)
        (void)hipStreamDestroy(ctx->stream);
    if (ctx->land_stream)
        (void)hipStreamDestroy(ctx->land_stream);
    delete ctx;
}

// sequence_t -> GPU template: thread_hdl() prologue, sequence.c:66-374.
int pbgpu_load_sequence(pbgpu_ctx *ctx, uint16_t seq_idx, const pb_sequence_t *seq, const uint8_t *src_mac,
                        const uint8_t *dst_mac, const pb_rules_t *rules, uint64_t seed_base)
{
    if (ctx == NULL || seq == NULL || seq_idx >= PB_MAX_SEQUENCES)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    {
        const int frc = ctr_fold(ctx, seq_idx, ctx->stream); // the old sequence's pending counts
        if (frc != PBGPU_OK)
            return frc;
    }
    HIPCHK(hipStreamSynchronize(ctx->stream)); // no build still reads the slot's tables
    seq_slot &S = ctx->seqs[seq_idx];
    if (S.loaded) // the slot's counts so far (their frames follow the old sequence's length)
    {
        const int rrc = read_counter_sums(ctx, seq_idx, 1);
        if (rrc != PBGPU_OK)
            return rrc;
        uint64_t p = 0, b = 0;
        slot_counts(ctx, ctx->h_ctr_sum, seq_idx, &p, &b);
        ctx->ctr_base[seq_idx][0] = p;
        ctx->ctr_base[seq_idx][1] = b;
        HIPCHK(hipMemset(ctx->d_counters + PB_CTR_WORDS * seq_idx, 0, PB_CTR_WORDS * sizeof(unsigned long long)));
    }
    {
        // the count ring (empty now) stays with the slot
        uint32_t *ring = S.d_ctr_slots;
        const uint64_t cap = S.ctr_cap;
        hipEvent_t ev = S.ctr_ev;
        slot_free(S);
        S.d_ctr_slots = ring;
        S.ctr_cap = cap;
        S.ctr_ev = ev;
        S.ctr_last = ctx->stream;
    }

    const pb_opts O = read_opts();
    pb_rules_t R = {PB_PAYLOAD_STREAM, PB_FOLD_FULL};
    if (rules)
        R = *rules;
    if (seq->ip.dst_ip == NULL) // seq_send refuses it, sequence.c:723-728
        return PBGPU_EINVAL;
    if (seq->pl_cnt > PB_MAX_PAYLOADS || seq->ip.range_count > PB_MAX_RANGES)
        return PBGPU_EINVAL;
    if (seq->ip.min_ttl > seq->ip.max_ttl || seq->ip.min_id > seq->ip.max_id)
        return PBGPU_EINVAL; // rand_num modulus <= 0: undefined in the reference

    pb_kargs K;
    memset(&K, 0, sizeof K);
    uint8_t t[64];
    memset(t, 0, sizeof t);

    uint8_t sm[6], dm[6];
    if (src_mac)
        memcpy(sm, src_mac, 6);
    else
        parse_mac(seq->eth.src_mac, sm);
    if (dst_mac)
        memcpy(dm, dst_mac, 6);
    else
        parse_mac(seq->eth.dst_mac, dm);

    uint32_t proto = 17;
    if (seq->ip.protocol && str_ieq(seq->ip.protocol, "tcp"))
        proto = 6;
    else if (seq->ip.protocol && str_ieq(seq->ip.protocol, "icmp"))
        proto = 1;
    K.proto = proto;
    K.l4len = proto == 6 ? 20 : 8;
    K.hl = 14 + 20 + K.l4len;
    if (proto == 17)
        K.csum_dw = 10, K.csum_hi = 0; // byte 40
    else if (proto == 6)
        K.csum_dw = 12, K.csum_hi = 1; // byte 50
    else
        K.csum_dw = 9, K.csum_hi = 0;  // byte 36

    // template, sequence.c:161-258
    memcpy(t + 0, dm, 6);
    memcpy(t + 6, sm, 6);
    t[12] = 0x08;
    t[13] = 0x00;
    t[14] = 0x45;
    t[15] = seq->ip.tos;
    t[23] = (uint8_t)proto;
    uint32_t flags = 0;
    if (seq->ip.min_ttl != seq->ip.max_ttl)
    {
        flags |= PBK_RND_TTL;
        K.ttl_min = seq->ip.min_ttl;
        K.ttl = make_div((uint32_t)seq->ip.max_ttl - seq->ip.min_ttl + 1);
    }
    else
    {
        t[22] = seq->ip.max_ttl;
    }
    if (seq->ip.min_id != seq->ip.max_id)
    {
        flags |= PBK_RND_ID;
        K.id_min = seq->ip.min_id;
        K.id = make_div((uint32_t)seq->ip.max_id - seq->ip.min_id + 1);
    }
    else
    {
        t[18] = (uint8_t)(seq->ip.max_id >> 8);
        t[19] = (uint8_t)seq->ip.max_id;
    }
    std::vector<uint2> ranges;
    if (seq->ip.src_ip != NULL)
    {
        struct in_addr a;
        memset(&a, 0, sizeof a);
        inet_aton(seq->ip.src_ip, &a);
        memcpy(t + 26, &a.s_addr, 4);
    }
    else if (seq->ip.range_count > 0)
    {
        flags |= PBK_RND_SADDR;
        for (int r = 0; r < seq->ip.range_count; ++r)
            ranges.push_back(compile_range(seq->ip.ranges[r]));
        K.rng = make_div(seq->ip.range_count);
    }
    else
    {
        const uint32_t lo = htonl(0x7F000001u); // sequence.c:484-490
        memcpy(t + 26, &lo, 4);
    }
    {
        struct in_addr a;
        memset(&a, 0, sizeof a);
        inet_aton(seq->ip.dst_ip, &a);
        memcpy(t + 30, &a.s_addr, 4);
    }
    if (proto == 17 || proto == 6)
    {
        const uint16_t sp = proto == 17 ? seq->udp.src_port : seq->tcp.src_port;
        const uint16_t dp = proto == 17 ? seq->udp.dst_port : seq->tcp.dst_port;
        if (sp)
            t[34] = (uint8_t)(sp >> 8), t[35] = (uint8_t)sp;
        else
            flags |= PBK_RND_SPORT;
        if (dp)
            t[36] = (uint8_t)(dp >> 8), t[37] = (uint8_t)dp;
        else
            flags |= PBK_RND_DPORT;
        K.port = make_div(65535);
        flags |= PBK_PSEUDO;
    }
    if (proto == 6)
    {
        t[46] = 5 << 4;
        t[47] = (uint8_t)((seq->tcp.fin & 1) | (seq->tcp.syn & 1) << 1 | (seq->tcp.rst & 1) << 2 |
                          (seq->tcp.psh & 1) << 3 | (seq->tcp.ack & 1) << 4 | (seq->tcp.urg & 1) << 5 |
                          (seq->tcp.ece & 1) << 6 | (seq->tcp.cwr & 1) << 7);
    }
    else if (proto == 1)
    {
        t[34] = seq->icmp.type;
        t[35] = seq->icmp.code;
    }
    if (seq->ip.csum)
        flags |= PBK_IP_CSUM;
    if (seq->l4_csum)
        flags |= PBK_L4_CSUM;
    if (R.iph_fold == PB_FOLD_SINGLE)
        flags |= PBK_IPH_SINGLE;
    if (R.payload_rule == PB_PAYLOAD_LITERAL)
        flags |= PBK_LITERAL;
    memcpy(K.tmpl, t, 64);

    // payloads, sequence.c:264-374
    std::vector<pb_pl> pls;
    std::vector<uint8_t> blob(96, 0); // >= 80 B of zeros before every static payload
    uint16_t dl_setup[PB_MAX_PAYLOADS];
    memset(dl_setup, 0, sizeof dl_setup);
    uint32_t sseed = host_seed(seed_base, seq_idx, PB_STATIC_SEED_K); // quirk B2
    int n_random = 0;
    uint32_t max_random = 0;
    for (int i = 0; i < seq->pl_cnt; ++i)
    {
        const pb_payload_opt_t *po = &seq->pls[i];
        pb_pl P;
        memset(&P, 0, sizeof P);
        std::vector<uint8_t> bytes;
        bool is_static = po->is_static;
        if (po->exact != NULL)
        {
            is_static = true;
            int rc = compile_exact(po, bytes);
            if (rc)
                return rc;
        }
        else if (po->is_static && po->max_len > 0)
        {
            if (po->min_len > po->max_len)
                return PBGPU_EINVAL;
            uint32_t s2 = sseed;
            const uint32_t len = po->min_len + host_rand_r(&s2) % ((uint32_t)po->max_len - po->min_len + 1);
            dl_setup[i] = (uint16_t)len;
            bytes.assign(len, 0);
            if (R.payload_rule == PB_PAYLOAD_LITERAL)
            {
                // the shadowed index runs while j < data_len[j], which may pass the payload's
                // own length: those draws still advance the seed, their bytes are not sent
                for (uint32_t j = 0; j < PB_MAX_PAYLOADS && j < dl_setup[j]; ++j)
                {
                    const uint8_t v = (uint8_t)host_rand_r(&sseed);
                    if (j < len)
                        bytes[j] = v;
                }
            }
            else
            {
                for (uint32_t j = 0; j < len; ++j)
                    bytes[j] = (uint8_t)host_rand_r(&sseed);
            }
        }
        if (is_static)
        {
            dl_setup[i] = (uint16_t)bytes.size();
            P.random = 0;
            P.slen = (uint32_t)bytes.size();
            P.blob_off = (uint32_t)blob.size();
            P.ssum = le_word_sum(bytes.data(), bytes.size());
            blob.insert(blob.end(), bytes.begin(), bytes.end());
            blob.insert(blob.end(), 96 + 16 - (bytes.size() & 15), 0); // >= 96 B zero pad, 16-B aligned
        }
        else if (po->max_len > 0)
        {
            if (po->min_len > po->max_len)
                return PBGPU_EINVAL;
            P.random = 1;
            P.min_len = po->min_len;
            P.len = make_div((uint32_t)po->max_len - po->min_len + 1);
            ++n_random;
            if (po->max_len > max_random)
                max_random = po->max_len;
        }
        else
        {
            P.random = 0; // non-static, max_len 0: empty payload (sequence.c:557-560)
            P.slen = 0;
            P.blob_off = 16 + 64;
        }
        if (K.hl + (P.random ? po->max_len : P.slen) > PB_MAX_PCKT_LEN)
            return PBGPU_EINVAL;
        pls.push_back(P);
    }
    if (pls.empty()) // sequence.c:364-374
    {
        pb_pl P;
        memset(&P, 0, sizeof P);
        P.blob_off = 16 + 64;
        pls.push_back(P);
    }
    // literal rule with several payloads (quirk B8, sequence.c:349 / 552): a random payload's
    // loop `for (u16 i = 0; i < data_len[i]; i++)` reads the other payloads' data_len[]
    // entries, so it draws until the first j with data_len[j] <= j.  Entries j > i hold
    // their setup values (declared rule, as the oracle); their part of the stop index is
    // fixed per payload here, the part of j <= i is found per iteration in pb_payload.
    std::vector<uint32_t> lit_stop(pls.size());
    for (size_t i = 0; i < pls.size(); ++i)
    {
        uint32_t j = (uint32_t)i + 1;
        while (j < PB_MAX_PAYLOADS && j < dl_setup[j])
            ++j;
        lit_stop[i] = j;
    }
    if ((flags & PBK_LITERAL) || max_random <= 64)
        flags |= PBK_SUM_IN_A;

    K.pl_cnt = (uint32_t)pls.size();
    K.pl0 = pls[0];
    K.flags = flags;
    K.seed_base = seed_base;
    K.seq = seq_idx;

    // frame lengths
    uint32_t minf = 0xFFFFFFFFu, maxf = 0;
    for (const pb_pl &P : pls)
    {
        const uint32_t lo = K.hl + (P.random ? P.min_len : P.slen);
        const uint32_t hi = K.hl + (P.random ? P.min_len + P.len.d - 1 : P.slen);
        minf = lo < minf ? lo : minf;
        maxf = hi > maxf ? hi : maxf;
    }
    S.min_flen = minf;
    S.max_flen = maxf;
    S.fpi = (uint32_t)pls.size();
    const bool fixed = pls.size() == 1 && (!pls[0].random || pls[0].len.d == 1);
    K.fixed_len = fixed ? minf : 0;
    if (fixed)
        K.flen = make_div(minf);
    // small fixed frames: one lane per frame (pb_small_kernel)
    if (fixed && pls.size() == 1 && minf <= 128)
    {
        K.small_ndw = minf <= 64 ? 16 : 32;
        {
            // the linear small kernel's frames per workgroup: 64 for even lengths (their 64-frame
            // regions end on 128-B lines), measured 2.5% faster than 256 on the 98-B ICMP frame
            // (0.649 vs 0.666 ms per 2^25 frames; 128: 0.666; profiles/r02/ab/small_wgt_icmp98.txt);
            // odd lengths keep 256 (line-aligned regions).  PBGPU_SMALL_WGT = 64 / 128 / 256 overrides
            const uint32_t w = O.small_wgt ? O.small_wgt : (minf % 2 == 0 ? 64u : 256u);
            K.small_wgt = (w == 64 || w == 128) ? w : 0u;
        }
        const bool xp_force = O.xp_force; // pb_xpage_kernel for any even length
        if (4096 % minf == 0 && minf == 4 * K.small_ndw && !xp_force) // pages of whole frames: pb_xsmall_kernel (64 / 128 B)
        {
            while ((minf << K.xs_fp_shift) < 4096)
                ++K.xs_fp_shift;
            K.xs_np = 256 >> K.xs_fp_shift;
            // one wave per page is fastest with few waves per CU (profiles/r05/ab/xs9.jsonl):
            // 64-B frames 0.297-0.303 ms per 2^25 at 3 workgroups per CU, 0.323-0.329 uncapped
            // (measured for 64-B frames only; 128-B pages keep the uncapped launch)
            if (K.xs_fp_shift == 6)
                K.lds_pad = lds_cap_pad(K.xs_np * PB_XPG, PB_XS_WG_PER_CU);
        }
        else if ((xp_force && minf % 2 == 0) ||
                 (O.kernel != PBO_K_NOPAGE && minf % 2 == 0 && minf >= 52 && minf <= 128 &&
                  (minf % 4 == 0 && minf <= 64 ? true : !pls[0].random && O.xp_static)))
        {
            // XCD-owned 4 KiB pages for frames cut at the page edges (pb_xpage_kernel): one slot
            // per frame touching a page, 512-thread workgroups (one pass of slots): lengths of
            // 52-64 B that are multiples of 4, and static payloads at every even length of 52-128 B
            // that does not divide 4096.  Round 4 (profiles/r04/ab/len_*.jsonl, xp_*.jsonl): static
            // payloads 5-16% faster than the linear small kernel at 54-126 B, 13% at the 98-B ICMP
            // frame (0.474-0.481 vs 0.549-0.552 ms, 4 buffers), and the rate does not depend on the
            // buffer's placement; random payloads over 64 B or of 2 mod 4 lose
            // 20-30% (each straddling frame's payload generated twice); 60-B TCP 512 vs 256
            // threads 0.296-0.298 vs 0.300-0.302 ms.  Pages per workgroup: 9 for lengths of 2 mod 4 (98 B:
            // 0.474-0.481 ms vs 0.496-0.501 at 7, 0.489-0.491 at 11, 0.574-0.577 at 5), 7 otherwise
            // (68 / 100 / 120 B: 7 faster than 9), at most the slots of one pass.
            K.xp = 1;
            K.xp_fpp = (4096 + minf - 1) / minf + 1;
            K.xp_div = make_div(K.xp_fpp);
            K.xp_inv = 1.0 / (double)minf;
            K.xp_wgt = O.xp_wgt == 256 ? 256 : 512;
            const uint32_t want = minf % 4 == 2 ? 9u : 7u;
            K.xs_np = std::max<uint32_t>(1, std::min<uint32_t>(want, 2 * PB_WG / K.xp_fpp));
            if (O.xp_np && O.xp_np * K.xp_fpp <= 2 * PB_WG) // at most two frame slots per 256 lanes
                K.xs_np = O.xp_np;
        }
        if (!pls[0].random)
        {
            const uint32_t p0 = (K.hl - 2) / 4;
            for (uint32_t j = 0; j < pls[0].slen; ++j)
            {
                const uint32_t pos = K.hl + j;
                K.stail[pos / 4 - p0] |= (uint32_t)blob[pls[0].blob_off + j] << (8 * (pos % 4));
            }
        }
    }
    {
        if (!K.small_ndw)
        {
            // lanes per frame (measured, profiles/r01/gsweep): equal-length frames take
            // the group size that wastes the fewest lanes on the frame's chunk count,
            // preferring 32 (1500-B frames: 4.2 TB/s at G=32, 3.5 at 8, 2.9 at 64);
            // packed variable-length frames take 8 (configs[2]: 3.35 TB/s at 8, 2.7
            // at 32).  PBGPU_G overrides (8, 16, 32, 64) for experiments.
            if (K.fixed_len)
            {
                const uint32_t nch = (minf + 15) / 16 + 1;
                double best = -1;
                for (uint32_t gg : {32u, 16u, 8u})
                {
                    const double util = (double)nch / (gg * ((nch + gg - 1) / gg));
                    if (util > best + 0.05)
                        best = util, K.gpf_g = gg;
                }
            }
            else
            {
                K.gpf_g = 8;
            }
            if (O.g)
                K.gpf_g = O.g;
            K.gpf_rmode = n_random == (int)pls.size() ? 1 : (n_random == 0 ? 0 : 2);
            const uint32_t ngw = PB_WG / K.gpf_g; // frames in flight per workgroup
            uint32_t fpw = O.fpw ? O.fpw : PB_WG;
            fpw = fpw < ngw ? ngw : (fpw > PB_WG ? PB_WG : fpw);
            K.gpf_fpw = fpw / ngw * ngw;

            // staged kernel (frames assembled in LDS, each window of the output written
            // as one contiguous run).  Lanes per frame G: the smallest of the group
            // sizes that waste the fewest lanes on a frame's payload chunks whose
            // 256 / G frames in flight span at most 26 KiB.  Fixed-length windows hold
            // k * 256 / G frames (~20 KiB); variable-length windows PBGPU_STAGE_KB
            // (default 24) KiB.  Measured (profiles/r01/stage): 1500-B frames 5.1 TB/s
            // at G = 16, 16 frames per window (group-per-frame: 4.1); 1024-B 5.2 at 16
            // frames; 9000-B 5.2 at G = 64.
            // variable-length frames: staged with G = 8 (configs[2], 2^23 frames: 1.81-1.86 ms
            // vs 2.01 on the group-per-frame kernel, since B writes payload chunks
            // unmasked); PBGPU_KERNEL=gpf forces the group-per-frame kernel.  A flat B
            // (one list of the window's payload chunks, checksums from LCG-cycle prefix
            // sums) measured slower: 2.1-2.5 ms
            const bool gpf_only = O.kernel == PBO_K_GPF;
            const uint32_t avg = (minf + maxf) / 2;
            const uint32_t npc = (avg - K.hl) / 16 + 2;
            double umax = 0;
            for (uint32_t gg : {8u, 16u, 32u, 64u})
                umax = std::max(umax, (double)npc / (gg * ((npc + gg - 1) / gg)));
            uint32_t sg = 64;
            for (uint32_t gg : {8u, 16u, 32u, 64u})
                if ((double)npc / (gg * ((npc + gg - 1) / gg)) >= umax - 0.02 && (PB_WG / gg) * avg <= 26 * 1024)
                {
                    sg = gg;
                    break;
                }
            if (!K.fixed_len)
                sg = 8;
            if (O.g)
                sg = O.g;
            const uint32_t wgt = O.wgt == 64 ? 64u : (uint32_t)PB_WG;
            uint32_t wgf = K.fixed_len ? 64 : 128;
            if (O.wgf && O.wgf <= PB_WG)
                wgf = O.wgf;
            wgf = std::min(wgf, wgt);
            uint32_t win, sbytes;
            if (K.fixed_len)
            {
                const uint32_t ngw2 = std::max(1u, wgt / sg);
                uint32_t fw = ngw2 * std::max(1u, (20u * 1024 * wgt / PB_WG) / (ngw2 * maxf));
                if (O.stage_kb)
                    fw = std::max(1u, O.stage_kb * 1024 / maxf);
                if (O.fpw)
                    fw = O.fpw;
                const uint32_t fit = (uint32_t)((64 * 1024 - 48 - PB_STAGE_LDS(std::max(wgf, fw))) / maxf);
                fw = std::max(1u, std::min(fw, fit)); // the stage must fit 64 KiB of LDS
                win = fw * maxf;
                sbytes = (win + 30 + 15) / 16 * 16;
            }
            else
            {
                // 24 KiB windows.  pb_vstage_kernel (configs[2], 2^25 frames, profiles/r02/ab/hv2_*):
                // 6.37 ms at 24 KiB, 6.68 at 16, 7.34 at 28 (3 workgroups per CU) since it keeps
                // only 9 header dwords per frame in LDS; with 16-dword images 16 KiB was best
                const uint32_t skb = O.stage_kb ? O.stage_kb : 24;
                sbytes = (skb * 1024 + 15) / 16 * 16;
                if (sbytes < 2 * maxf + 48)
                    sbytes = (2 * maxf + 48 + 15) / 16 * 16;
                win = sbytes - maxf - 32;
            }
            if (K.fixed_len)
            {
                const uint32_t fw = win / maxf; // whole windows per workgroup
                wgf = fw > wgt ? wgt : std::min<uint32_t>(wgt / fw * fw, fw * ((wgf + fw - 1) / fw));
            }
            else if (!O.wgf)
                wgf = std::min<uint32_t>(wgt, std::max(wgf, win / minf + 1));
            if (!gpf_only && sbytes + PB_STAGE_LDS(wgf) <= 64 * 1024)
            {
                K.gpf_g = sg;
                K.stage_win = win;
                K.stage_wgf = wgf;
                K.stage_wgt = wgt;
                K.stage_bytes = sbytes;
                // every payload random, stream rule: pb_vstage_kernel (no header pass, no
                // serial byte loops in phase A; configs[2] 1.74 vs 1.87 ms per 2^23 frames at
                // the best window of each); PBGPU_KERNEL=stage keeps pb_stage_kernel
                if (K.gpf_rmode == 1 && !(flags & PBK_LITERAL) && wgt == PB_WG && O.kernel != PBO_K_STAGE &&
                    sbytes + PB_VST_LDS(wgf) <= 64 * 1024)
                {
                    K.vst = 1;
                    K.vst_shape = O.vst_shape;
                    // phase A has one lane per slot (ghosts + own frames): as many own frames as
                    // lanes allow, which also spreads the per-workgroup work over the most windows
                    // (configs[2], 2^25 frames: 6.37 ms at 240-252 vs 6.44 at 218 and 6.50 at 200;
                    // profiles/r02/ab/wf24*)
                    // (as many as still leave 4 workgroups per CU when the window's frames fit)
                    K.stage_wgf = std::min<uint32_t>(K.stage_wgf, PB_WG - PB_VST_GHOSTS);
                    if (!O.wgf && !K.fixed_len)
                    {
                        uint32_t best = PB_WG - PB_VST_GHOSTS;
                        while (best > K.stage_wgf && K.stage_bytes + PB_VST_LDS(best) > 160 * 1024 / 4)
                            --best;
                        K.stage_wgf = best;
                    }
                }
            }
            // fixed-length staged kernel (pb_fstage_kernel): lengths > 128 B that are a
            // multiple of 4, every payload random, stream rule.  One stage buffer, then two;
            // G = the smallest of 16, 32, 64 whose stage of 256 / G frames fits 64 KiB with
            // the per-frame records; 64 frames per workgroup.  Measured on 1500-B frames
            // (profiles/r01/fstage): 1 buffer G = 16 2.12 ms per 2^23 frames, 2 buffers 2.20,
            // G = 32 2.21, G = 64 2.35, 32 / 128 frames per workgroup 2.15 / 2.20;
            // pb_stage_kernel 2.29.  PBGPU_KERNEL=stage / gpf keep the older kernels,
            // PBGPU_FST_G, PBGPU_FST_WGF, PBGPU_FST_NBUF override the shape.
            const bool fst_ok = K.fixed_len && minf > 128 && minf % 4 == 0 && K.gpf_rmode == 1 &&
                                !(flags & PBK_LITERAL) && !gpf_only && O.kernel != PBO_K_STAGE;
            // packed variable lengths, every payload random, stream rule, payloads of >= 32 B:
            // pb_vline_kernel (no LDS stage).  ICMP type 0 / code 0 is left to
            // pb_vstage_kernel: its header word sum can be 0, where the orbit sums cannot tell a
            // zero payload sum from 0xFFFF.  PBGPU_KERNEL=vstage keeps pb_vstage_kernel.
            const bool icmp00 = proto == 1 && t[34] == 0 && t[35] == 0;
            // the orbit prefix-sum table (pb_orbit_sum, pb_vline_kernel): the 2^24-step
            // walk runs once per process; each context uploads the result
            auto need_orbit = [&]() -> int {
                if (ctx->d_orbit == nullptr)
                {
                    static std::once_flag once;
                    static std::vector<uint32_t> orb;
                    static uint32_t tot = 0;
                    std::call_once(once, [] { orb = make_orbit_table(&tot); });
                    const int rc2 = upload(&ctx->d_orbit, orb.data(), orb.size());
                    if (rc2 != PBGPU_OK)
                        return rc2;
                    ctx->orbit_tot = tot;
                }
                K.orbit = ctx->d_orbit;
                K.orbit_tot = ctx->orbit_tot;
                return PBGPU_OK;
            };
            if (!K.fixed_len && K.gpf_rmode == 1 && !(flags & PBK_LITERAL) && !gpf_only && minf >= K.hl + 32 &&
                maxf <= 4096 && !icmp00 && O.kernel != PBO_K_VSTAGE && O.kernel != PBO_K_STAGE)
            {
                const uint32_t nsp = K.hl == 54 ? 5u : 4u;
                uint32_t wf = O.vl_wgf ? O.vl_wgf : PB_WG - PB_VST_GHOSTS;
                wf = std::max(32u, std::min<uint32_t>(wf, PB_WG - PB_VST_GHOSTS));
                uint32_t nl48 = 0, nlines = 0;
                for (;; wf -= 4)
                {
                    const uint64_t rmax = (uint64_t)wf * maxf + 256; // own frames + the line before the first
                    nl48 = (maxf + 31) / 16 + 1;
                    nlines = (uint32_t)(rmax / 128 + 2);
                    if (PB_VL_LDS(wf, nsp, nl48, nlines) <= 40 * 1024 || wf <= 32) // >= 4 workgroups per CU
                        break;
                }
                const int orc = need_orbit();
                if (orc != PBGPU_OK)
                    return orc;
                K.vl = 1;
                K.vl_wgf = wf;
                K.vl_nl48 = nl48;
                K.vl_nlines = nlines;
                // PBGPU_KERNEL=vpage, one payload: the page-shaped writer (pb_vrec_kernel +
                // pb_vpage_kernel).  Bit-exact and immune to the buffer placement
                // that slows pb_vline_kernel, but 7.1 vs 4.2 ms per 2^25 configs[2] frames: each
                // page's frame setup runs one lane per frame (~6 of 64 lanes), 3.4 G VALU
                // instructions per launch against 2.0 G (profiles/r06/vpage/)
                const uint32_t nfp = (4096 + minf - 1) / minf + 1;
                if (pls.size() == 1 && nfp <= 64 && O.kernel == PBO_K_VPAGE)
                {
                    K.vl = 0;
                    K.vp = 1;
                    K.vp_nfp = nfp;
                }
            }
            if (fst_ok)
            {
                const uint32_t eg = O.fst_g, ew = O.fst_wgf, en = O.fst_nbuf;
                for (uint32_t nb : {1u, 2u})
                {
                    if (en && nb != en)
                        continue;
                    for (uint32_t gg : {16u, 32u, 64u})
                    {
                        if ((eg && gg != eg) || K.hl / 4 >= gg)
                            continue;
                        const uint32_t ngw = PB_WG / gg;
                        uint32_t fw = ew ? ew : 64;
                        fw = std::max(ngw, std::min<uint32_t>(PB_WG, fw / ngw * ngw));
                        const uint32_t sb = (ngw * minf + 15) / 16 * 16;
                        if ((size_t)nb * sb + PB_FST_LDS(fw) <= 64 * 1024)
                        {
                            K.fst_g = gg;
                            K.fst_wgf = fw;
                            K.fst_sb = sb;
                            K.fst_nbuf = nb;
                            break;
                        }
                    }
                    if (K.fst_g)
                        break;
                }
            }
        }
    }
    int rc;
    if ((rc = upload(&S.d_ranges, ranges.data(), ranges.size())) != PBGPU_OK)
        return rc;
    if ((rc = upload(&S.d_pls, pls.data(), pls.size())) != PBGPU_OK)
        return rc;
    if ((rc = upload(&S.d_lit_stop, lit_stop.data(), lit_stop.size())) != PBGPU_OK)
        return rc;
    blob.insert(blob.end(), 64, 0);
    if ((rc = upload(&S.d_blob, blob.data(), blob.size())) != PBGPU_OK)
        return rc;
    K.ranges = S.d_ranges;
    K.pls = S.d_pls;
    K.lit_stop = S.d_lit_stop;
    K.blob = S.d_blob;
    K.jump = ctx->d_jump;
    K.lcg48 = ctx->d_lcg48;
    K.lcg48i = ctx->d_lcg48i;
    K.m16 = ctx->d_m16;
    K.dlog12 = ctx->d_dlog12;
    K.counters = ctx->d_counters + PB_CTR_WORDS * seq_idx;
    // pb_ximg_kernel (static-payload ICMP frames): only IPv4 ID, TTL, checksum and
    // source address vary per frame, so the stream's bytes repeat every img_np = flen / gcd(flen,
    // 4096) pages outside those fields.  Build its first img_np pages once, here, with
    // pb_xpage_kernel (counted into a scratch counter array, not the sequence's)
    if (K.xp && K.proto == 1 && !pls[0].random && K.fixed_len % 2 == 0 && O.xp_img && !O.xp_force &&
        O.kernel == PBO_K_AUTO &&
        !(K.flags & (PBK_RND_SPORT | PBK_RND_DPORT)))
    {
        uint32_t g = K.fixed_len, a = PB_XPG;
        while (a)
        {
            const uint32_t t = g % a;
            g = a;
            a = t;
        }
        const uint32_t np = K.fixed_len / g;
        const uint64_t bytes = (uint64_t)np * PB_XPG;
        HIPCHK(hipMalloc((void **)&S.d_img, bytes));
        if (ctx->d_img_ctr == nullptr)
        {
            HIPCHK(hipMalloc((void **)&ctx->d_img_ctr, PB_CTR_WORDS * sizeof(unsigned long long)));
            HIPCHK(hipMemset(ctx->d_img_ctr, 0, PB_CTR_WORDS * sizeof(unsigned long long)));
        }
        pb_kargs K2 = K;
        K2.img = nullptr;
        K2.first_iter = 0;
        K2.n_frames = (bytes + K.fixed_len - 1) / K.fixed_len + 1;
        K2.total_bytes = bytes;
        K2.out = (uint8_t *)S.d_img;
        K2.counters = ctx->d_img_ctr;
        K2.ctr_slots = nullptr;
        K2.xs_nch = np;
        K2.xs_full = np / (8 * K2.xs_np) * 8;
        K2.xs_grid = K2.xs_full + (np - K2.xs_full * K2.xs_np + K2.xs_np - 1) / K2.xs_np;
        K2.xp_fa_hi = 0;
        HIPCHK(pbk_launch_build(&K2, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        K.img = S.d_img;
        K.img_np = np;
        K.img_div = make_div(np);
        K.img_solo = O.xp_img == 2;
    }
    S.K = K;
    S.opt = O;
    S.loaded = true;
    return PBGPU_OK;
}

int pbgpu_build_size(pbgpu_ctx *ctx, uint16_t seq_idx, uint64_t n_iter, uint64_t *max_frames, uint64_t *max_bytes)
{
    if (ctx == NULL || seq_idx >= PB_MAX_SEQUENCES)
        return PBGPU_EINVAL;
    const seq_slot &S = ctx->seqs[seq_idx];
    if (!S.loaded)
        return PBGPU_ENOENT;
    const uint64_t nf = n_iter * S.fpi;
    if (max_frames)
        *max_frames = nf;
    if (max_bytes)
        *max_bytes = ((nf * S.max_flen + 15) & ~15ull) + 16;
    return PBGPU_OK;
}

// Device memory of frame buffers.  A buffer of >= PB_VMM_MIN bytes is built from physical chunks
// (hipMemCreate, alloc_chunk_mb each) mapped in creation order into one reserved VA range,
// instead of one hipMalloc: the region kernels' slow mode follows the buffer's
// physical placement; in fresh processes hipMalloc drew it 3 times in 4 (pb_fstage_kernel 8.47 ms,
// pb_vline_kernel 5.06-5.08) and chunk-mapped buffers 2 times in 40 (7.24-7.30 / 4.36-4.40 otherwise;
// profiles/r05/ab/alloc_ab2.jsonl, vmm*.jsonl, lenpass_ab.log).  Falls back to hipMalloc when the virtual-memory
// calls fail.  The blocks are kept in a process-wide table, so fb_free needs no context; callers
// free only after the work that uses a block has completed (pbgpu_frames_free synchronises first).
#define PB_VMM_MIN (64ull << 20)

namespace
{
struct vmm_block
{
    size_t bytes;
    int device; // the GPU whose memory the chunks are (fb_free synchronises it before unmapping)
    std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> chunks; // handle, size
};
std::mutex g_vmm_mu;
std::unordered_map<void *, vmm_block> g_vmm;

void vmm_release(void *va, vmm_block &B)
{
    size_t off = 0;
    for (auto &c : B.chunks)
    {
        (void)hipMemUnmap((char *)va + off, c.second);
        (void)hipMemRelease(c.first);
        off += c.second;
    }
    (void)hipMemAddressFree(va, B.bytes);
}
} // namespace

static hipError_t fb_alloc(const pbgpu_ctx *ctx, void **p, size_t bytes)
{
    *p = nullptr;
    const size_t chunk = (size_t)ctx->opt.alloc_chunk_mb << 20;
    if (!ctx->opt.alloc_vmm || bytes < PB_VMM_MIN || chunk == 0)
        return hipMalloc(p, bytes);
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = ctx->device;
    size_t gran = 0;
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) != hipSuccess || gran == 0 ||
        chunk % gran)
    {
        if (verbose())
            fprintf(stderr, "pbgpu: allocation granularity %zu B does not divide %zu-B chunks; hipMalloc\n", gran, chunk);
        (void)hipGetLastError();
        return hipMalloc(p, bytes);
    }
    vmm_block B;
    B.bytes = (bytes + gran - 1) / gran * gran;
    B.device = ctx->device;
    void *va = nullptr;
    if (hipMemAddressReserve(&va, B.bytes, chunk, nullptr, 0) != hipSuccess)
    {
        if (verbose())
            fprintf(stderr, "pbgpu: no %zu-B address reservation; hipMalloc\n", B.bytes);
        (void)hipGetLastError();
        return hipMalloc(p, bytes);
    }
    bool ok = true;
    for (size_t off = 0; off < B.bytes && ok; off += chunk)
    {
        const size_t sz = B.bytes - off < chunk ? B.bytes - off : chunk;
        hipMemGenericAllocationHandle_t h;
        if (hipMemCreate(&h, sz, &prop, 0) != hipSuccess)
        {
            ok = false;
            break;
        }
        if (hipMemMap((char *)va + off, sz, 0, h, 0) != hipSuccess)
        {
            (void)hipMemRelease(h);
            ok = false;
            break;
        }
        B.chunks.push_back({h, sz});
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if (ok && hipMemSetAccess(va, B.bytes, &acc, 1) != hipSuccess)
        ok = false;
    if (!ok)
    {
        if (verbose())
            fprintf(stderr, "pbgpu: chunk mapping failed after %zu chunks (%s); hipMalloc\n", B.chunks.size(),
                    hipGetErrorString(hipGetLastError()));
        vmm_release(va, B); // the chunks mapped so far, then the reservation
        (void)hipGetLastError();
        return hipMalloc(p, bytes);
    }
    if (verbose())
        fprintf(stderr, "pbgpu: %zu-B buffer at %p: %zu physical chunks of <= %zu B mapped in order\n", B.bytes, va,
                B.chunks.size(), chunk);
    {
        std::lock_guard<std::mutex> lk(g_vmm_mu);
        g_vmm.emplace(va, std::move(B));
    }
    *p = va;
    return hipSuccess;
}

// hipFree waits for the device; unmapping does not, so a chunk-mapped block first waits for every
// stream of its device (work queued on a caller's stream, or a free without a context, must not
// find its pages gone: a GPU page fault instead of hipFree's implicit wait)
static void fb_free(void *p)
{
    if (p == nullptr)
        return;
    {
        std::lock_guard<std::mutex> lk(g_vmm_mu);
        auto it = g_vmm.find(p);
        if (it != g_vmm.end())
        {
            int cur = -1;
            (void)hipGetDevice(&cur);
            if (hipSetDevice(it->second.device) == hipSuccess)
                (void)hipDeviceSynchronize();
            if (cur >= 0)
                (void)hipSetDevice(cur);
            vmm_release(p, it->second);
            g_vmm.erase(it);
            return;
        }
    }
    (void)hipFree(p);
}

int pbgpu_frames_alloc(pbgpu_ctx *ctx, uint64_t capacity_frames, uint64_t capacity_bytes, pbgpu_frames **out)
{
    if (ctx == NULL || out == NULL)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    pbgpu_frames *f = (pbgpu_frames *)calloc(1, sizeof *f);
    if (f == NULL)
        return PBGPU_ENOMEM;
    capacity_bytes = (capacity_bytes + 15) & ~15ull;
    // +64 B: word-granular readers (UMEM scatter) may touch a few bytes past the last frame
    if (fb_alloc(ctx, (void **)&f->data, capacity_bytes + 64) != hipSuccess ||
        fb_alloc(ctx, (void **)&f->offsets, (capacity_frames + 1) * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc((void **)&f->scan_tmp, scan_tmp_bytes(capacity_frames)) != hipSuccess)
    {
        pbgpu_frames_free(ctx, f);
        return PBGPU_ENOMEM;
    }
    f->capacity_frames = capacity_frames;
    f->capacity_bytes = capacity_bytes;
    f->total_bytes = 0;
    *out = f;
    return PBGPU_OK;
}

void pbgpu_frames_free(pbgpu_ctx *ctx, pbgpu_frames *f)
{
    if (f == NULL)
        return;
    if (ctx)
    {
        (void)hipSetDevice(ctx->device);
        (void)pbgpu_land_wait(ctx, 0);
        (void)join_builds(ctx);
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipStreamSynchronize(ctx->land_stream);
    }
    if (f->reserved)
    {
        frames_events *fe = (frames_events *)f->reserved;
        if (fe->built)
            (void)hipEventDestroy(fe->built);
        if (fe->moved)
            (void)hipEventDestroy(fe->moved);
        if (fe->d_off32)
            fb_free(fe->d_off32);
        if (fe->d_rstart)
            (void)hipFree(fe->d_rstart);
        if (fe->d_vrec)
            fb_free(fe->d_vrec);
        if (fe->d_vpt)
            (void)hipFree(fe->d_vpt);
        if (fe->landed)
            (void)hipEventDestroy(fe->landed);
        delete fe;
    }
    if (f->data)
        fb_free(f->data);
    if (f->offsets)
        fb_free(f->offsets);
    if (f->scan_tmp)
        (void)hipFree(f->scan_tmp);
    free(f);
}

static int timed_pair(pbgpu_ctx *ctx, timing_pair *p)
{
    if (!ctx->pool.empty())
    {
        *p = ctx->pool.back();
        ctx->pool.pop_back();
        return PBGPU_OK;
    }
    HIPCHK(hipEventCreate(&p->a));
    HIPCHK(hipEventCreate(&p->b));
    return PBGPU_OK;
}

// The frames' build-completion event (kept in pbgpu_frames.reserved): the
// landing stream waits on it, so landing one buffer overlaps building the next.
static int mark_built(pbgpu_ctx *ctx, pbgpu_frames *out, hipStream_t st)
{
    // only for callers that land frames: an event record per launch would cost a
    // release between back-to-back builds that are never landed (bench)
    if (!ctx->land_events)
        return PBGPU_OK;
    frames_events *fe = frames_ev(out);
    if (fe == NULL)
        return PBGPU_ENOMEM;
    if (fe->built == nullptr)
        HIPCHK(hipEventCreateWithFlags(&fe->built, hipEventDisableTiming));
    HIPCHK(hipEventRecord(fe->built, st));
    return PBGPU_OK;
}

// offsets[] of a build that wrote 4-B offsets, expanded on the context's stream (after the
// sequence streams are joined); later builds of the buffer follow it (fe->last)
static int materialize_offsets(pbgpu_ctx *ctx, const pbgpu_frames *f)
{
    frames_events *fe = (frames_events *)f->reserved;
    if (fe == NULL || !fe->packed32)
        return PBGPU_OK;
    PB_JOIN(ctx);
    HIPCHK(pbk_launch_expand_offsets(fe->d_off32, fe->d_rstart, fe->wf, f->n_frames, f->offsets, ctx->stream));
    fe->packed32 = false;
    fe->last = ctx->stream;
    if (fe->built) // a landing waits for the expansion too
        HIPCHK(hipEventRecord(fe->built, ctx->stream));
    return PBGPU_OK;
}

int pbgpu_frames_offsets(pbgpu_ctx *ctx, pbgpu_frames *f)
{
    if (ctx == NULL || f == NULL)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    return materialize_offsets(ctx, f);
}

// A part of pbgpu_build_batch's fused launch: the stream it runs on and its block size in; the
// build's kargs out (built = false: no frames, nothing to launch)
struct batch_part
{
    hipStream_t st;
    uint32_t wgt;
    pb_kargs K;
    bool built;
    uint64_t ctr_words; // count-ring words the part reserved (returned if the launch fails)
};

// Every argument check of a build, before anything is changed (pbgpu_build_batch checks all its
// parts first, so a part that cannot be built leaves the others untouched).
static int build_check(pbgpu_ctx *ctx, uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter,
                       const pbgpu_frames *out)
{
    if (ctx == NULL || out == NULL || seq_idx >= PB_MAX_SEQUENCES)
        return PBGPU_EINVAL;
    const seq_slot &S = ctx->seqs[seq_idx];
    if (!S.loaded)
        return PBGPU_ENOENT;
    const uint64_t nf = n_iter * S.fpi;
    if (nf > out->capacity_frames || nf > 0xFFFFFFFFull)
        return PBGPU_ENOSPC;
    if (first_iter + n_iter >= PB_STATIC_SEED_K)
        return PBGPU_EINVAL;
    const uint64_t max_bytes = nf * S.max_flen;
    if (((max_bytes + 15) & ~15ull) > out->capacity_bytes)
        return PBGPU_ENOSPC;
    return PBGPU_OK;
}

// pbgpu_build, or with bp: every step of it but the launch (and its timing), on bp->st
static int build_impl(pbgpu_ctx *ctx, uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter, pbgpu_frames *out,
                      batch_part *bp)
{
    {
        const int crc = build_check(ctx, seq_idx, first_iter, n_iter, out);
        if (crc != PBGPU_OK)
            return crc;
    }
    seq_slot &S = ctx->seqs[seq_idx];
    HIPCHK(hipSetDevice(ctx->device));
    const uint64_t nf = n_iter * S.fpi;

    // the stream this build runs on: the sequence's own in span mode (builds of different
    // sequences overlap), the context's otherwise (each launch timed on its own)
    hipStream_t st = ctx->stream;
    const bool span = ctx->timing_mode == PBGPU_TIMING_SPAN;
    int si = -1;
    if (bp)
        st = bp->st, bp->built = false;
    else if (span && ctx->opt.seq_streams)
    {
        si = seq_idx % PB_SEQ_STREAMS;
        if (ctx->seq_stream[si] == nullptr)
            HIPCHK(hipStreamCreateWithFlags(&ctx->seq_stream[si], hipStreamNonBlocking));
        st = ctx->seq_stream[si];
    }
    frames_events *fe = frames_ev(out);
    if (fe == NULL)
        return PBGPU_ENOMEM;
    // a buffer last built on another stream: this build follows that one
    if (fe->last && fe->last != st)
    {
        if (fe->moved == nullptr)
            HIPCHK(hipEventCreateWithFlags(&fe->moved, hipEventDisableTiming));
        HIPCHK(hipEventRecord(fe->moved, fe->last));
        HIPCHK(hipStreamWaitEvent(st, fe->moved, 0));
    }
    fe->last = st;
    fe->packed32 = false;
    // a landing queued from this buffer must have read it before the build overwrites it
    if (fe->land_pending)
    {
        HIPCHK(hipStreamWaitEvent(st, fe->landed, 0));
        fe->land_pending = false;
    }
    pb_kargs K = S.K;
    K.first_iter = first_iter;
    K.n_frames = nf;
    K.out = out->data;
    K.offsets = out->offsets;
    out->seq_idx = seq_idx;
    out->first_iter = first_iter;
    out->n_frames = nf;
    out->fixed_len = K.fixed_len;
    if (nf == 0)
    {
        out->total_bytes = 0;
        return PBGPU_OK;
    }
    if (K.fixed_len)
    {
        K.total_bytes = nf * K.fixed_len;
        out->total_bytes = K.total_bytes;
    }
    else
    {
        out->total_bytes = UINT64_MAX;
        K.vblk_sum = nullptr;
        K.vblk_l2 = nullptr;
        K.offsets_w = nullptr;
        const uint32_t wgf = K.vp ? (uint32_t)PB_WG : (K.vl ? K.vl_wgf : K.stage_wgf);
        if (K.vl || K.vp || (K.vst && K.stage_wgf >= PB_VST_SCAN_MIN_WGF && !S.opt.vst_scan3))
        {
            // pb_vline_kernel / pb_vstage_kernel: per-workgroup length sums, their scan, offsets
            // written by the build
            const uint64_t nblk = (nf + wgf - 1) / wgf;
            const uint64_t n_l2 = (nblk + PB_VL_GRP - 1) / PB_VL_GRP;
            uint32_t *bsum = reinterpret_cast<uint32_t *>(out->scan_tmp);
            unsigned long long *l2 =
                reinterpret_cast<unsigned long long *>(reinterpret_cast<uint8_t *>(out->scan_tmp) + vst_bsum_bytes(nblk));
            HIPCHK(pbk_launch_vst_lengths(&K, wgf, bsum, (uint32_t)nblk, l2, (uint32_t)n_l2, out->offsets, st));
            K.vblk_sum = bsum;
            K.vblk_l2 = l2;
            K.offsets_w = out->offsets;
            if (K.vp)
            {
                // the record pass's records (8 B per frame) and page table (8 B per page of the
                // buffer's capacity); the page grid covers the longest stream these frames can make
                if (fe->d_vrec == nullptr)
                    HIPCHK(fb_alloc(ctx, (void **)&fe->d_vrec, out->capacity_frames * sizeof(uint2)));
                if (fe->d_vpt == nullptr)
                    HIPCHK(hipMalloc((void **)&fe->d_vpt, (out->capacity_bytes / 4096 + 2) * sizeof(uint2)));
                K.vp_rec = fe->d_vrec;
                K.vp_pt = fe->d_vpt;
                // the grid covers the expected stream (one random payload of uniform length: the
                // mean frame) plus 1% and 64 pages; a longer stream is built by the same waves in
                // later rounds.  (A grid for the longest possible stream, 1.87x configs[2]'s, spent
                // ~2 ms per 2^25 frames on workgroups past the stream's end.)
                const uint64_t pages_max = (nf * S.max_flen + 4095) / 4096;
                uint64_t pages_est = (uint64_t)((double)nf * 0.5 * (S.min_flen + S.max_flen) * 1.01 / 4096.0) + 64;
                if (S.opt.vp_pages_pct)
                    pages_est = pages_est * S.opt.vp_pages_pct / 100 + 1;
                const uint64_t pages = pages_est < pages_max ? pages_est : pages_max;
                const uint64_t ppg = 32; // pages per group of 8 workgroups (4 per workgroup)
                if ((pages + ppg - 1) / ppg * 8 > 0x7FFFFFFFull)
                    return PBGPU_ENOSPC;
                K.vp_grid = (uint32_t)((pages + ppg - 1) / ppg * 8);
            }
            if (K.vl || K.vp)
            {
                // 4 B per frame and 8 B per region instead of 8 B per frame
                // (each checked on its own: a failed second allocation must not leave the pair
                // half set for the next build to launch with a null region-start array)
                if (fe->d_off32 == nullptr)
                    HIPCHK(fb_alloc(ctx, (void **)&fe->d_off32, (out->capacity_frames + 1) * sizeof(uint32_t)));
                if (fe->d_rstart == nullptr)
                    HIPCHK(hipMalloc((void **)&fe->d_rstart, (out->capacity_frames / 32 + 2) * sizeof(unsigned long long)));
                K.offsets32 = fe->d_off32;
                K.vl_rstart = fe->d_rstart;
                fe->packed32 = true;
                fe->wf = wgf;
            }
        }
        else
        {
            const uint64_t nblocks = (nf + PB_SCAN_FRAMES_PER_BLOCK - 1) / PB_SCAN_FRAMES_PER_BLOCK;
            HIPCHK(pbk_launch_lengths(&K, (unsigned long long *)out->scan_tmp, (uint32_t)nblocks, out->offsets, st));
        }
    }
    K.xs_grid = 0;
    if (bp && K.small_ndw && K.xs_np && !K.xp) // pb_batch_kernel's 64-B part at the batch's block size
        K.xs_np = bp->wgt >> K.xs_fp_shift;
    const bool img = K.img && (bp || K.img_solo); // pb_ximg_kernel / the batch's ICMP part
    if (!img)
        K.img = nullptr;
    else // one page per wave
        K.xs_np = (bp ? bp->wgt : PB_WG) / 64;
    if (K.small_ndw && K.xs_np && ((uintptr_t)K.out & 4095u) == 0 && S.opt.kernel != PBO_K_LINEAR)
    {
        // XCD-owned 4 KiB pages, xs_np per workgroup: pb_xsmall_kernel (one wave per page) takes
        // groups of 8 workgroups (pages past the stream are skipped);
        // pb_xpage_kernel and the batch's 64-B part take full groups of 8, then the tail pages in order
        const uint64_t nch = (K.total_bytes + 4095) / 4096;
        if (nch < 0x7FFFFFFFull)
        {
            K.xs_nch = (uint32_t)nch;
            const uint32_t np = K.xs_np;
            K.xs_full = (uint32_t)(nch / (8 * np) * 8);
            if ((K.xp || (bp && K.small_ndw)) && !K.img)
                K.xs_grid = K.xs_full + (uint32_t)((nch - (uint64_t)K.xs_full * np + np - 1) / np);
            else
                K.xs_grid = (uint32_t)((nch + 8ull * np - 1) / (8ull * np) * 8);
            // (PBGPU_XP_FA64=1: the 64-bit path at any size, so the tests reach it)
            K.xp_fa_hi = K.xp && ((uint64_t)nch * (4096 % K.fixed_len) >= (1ull << 31) || S.opt.xp_fa64);
        }
    }
    // the load-time occupancy cap (lds_pad) belongs to pb_xsmall_kernel's page launch alone: the
    // linear fallback (an output not 4-KiB aligned, PBGPU_KERNEL=linear) keeps its own occupancy
    if (K.xs_grid == 0)
        K.lds_pad = 0;
    timing_pair tp = {nullptr, nullptr};
    int rc = PBGPU_OK;
    // this launch's per-workgroup count records (pb_count): the next words of the sequence's
    // ring, folded into the counters first when it is full (PBGPU_CTR_ATOMIC=1: one atomic per
    // workgroup instead).  Reserved last, after everything that can fail but the launch itself;
    // a launch that fails returns them (its records would never be written)
    K.ctr_slots = nullptr;
    uint64_t words = 0;
    if (!S.opt.ctr_atomic)
    {
        const uint64_t pairs = K.fixed_len ? 1 : 2;
        words = (uint64_t)pbk_build_grid(&K) * pairs;
        if (S.ctr_pairs != pairs || S.ctr_used + words > S.ctr_cap)
        {
            if ((rc = ctr_fold(ctx, seq_idx, st)) != PBGPU_OK)
                return rc;
            S.ctr_pairs = pairs;
            if (words > S.ctr_cap)
            {
                HIPCHK(hipStreamSynchronize(st)); // the old ring's fold has read it
                if (S.d_ctr_slots)
                    (void)hipFree(S.d_ctr_slots);
                S.d_ctr_slots = nullptr;
                S.ctr_cap = 0;
                // (PBGPU_CTR_RING = words: a small ring, so the tests reach the fold-when-full path)
                const uint64_t ring = S.opt.ctr_ring ? (uint64_t)S.opt.ctr_ring : PB_CTR_RING_WORDS;
                const uint64_t cap = words > ring ? words : ring;
                HIPCHK(hipMalloc((void **)&S.d_ctr_slots, cap * sizeof(uint32_t)));
                S.ctr_cap = cap;
            }
        }
        if ((rc = ctr_order(S, st)) != PBGPU_OK)
            return rc;
        K.ctr_slots = S.d_ctr_slots + S.ctr_used;
        S.ctr_used += words;
    }
    if (bp)
    {
        bp->K = K;
        bp->built = true;
        bp->ctr_words = words;
        return PBGPU_OK;
    }
    // every error exit from here on returns the reserved count-ring words (their records would
    // never be written, and the next fold would read stale ones) and the timing pair
    auto undo = [&]() {
        S.ctr_used -= words;
        if (tp.a)
            ctx->pool.push_back(tp);
    };
#define HIPCHK_UNDO(call)                                                                    \
    do                                                                                       \
    {                                                                                        \
        const hipError_t u_ = (call);                                                        \
        if (u_ != hipSuccess)                                                                \
        {                                                                                    \
            undo();                                                                          \
            HIPCHK(u_);                                                                      \
        }                                                                                    \
    } while (0)
    if (span)
    {
        if (ctx->span_n == 0)
        {
            if (ctx->span.a == nullptr)
            {
                HIPCHK_UNDO(hipEventCreate(&ctx->span.a));
                HIPCHK_UNDO(hipEventCreate(&ctx->span.b));
            }
            HIPCHK_UNDO(hipEventRecord(ctx->span.a, ctx->stream));
            for (bool &j : ctx->seq_in_span)
                j = false;
        }
        if (si >= 0)
        {
            if (!ctx->seq_in_span[si]) // the span starts before this stream's first launch in it
            {
                HIPCHK_UNDO(hipStreamWaitEvent(st, ctx->span.a, 0));
                ctx->seq_in_span[si] = true;
            }
            ctx->seq_dirty[si] = true;
        }
        HIPCHK_UNDO(pbk_launch_build(&K, st));
        ++ctx->span_n;
        return mark_built(ctx, out, st);
    }
    if ((rc = timed_pair(ctx, &tp)) != PBGPU_OK)
    {
        undo();
        return rc;
    }
    HIPCHK_UNDO(hipEventRecord(tp.a, ctx->stream));
    HIPCHK_UNDO(pbk_launch_build(&K, ctx->stream));
#undef HIPCHK_UNDO
    // launched: its records will be written; a failing end event drops only this timing
    HIPCHK(hipEventRecord(tp.b, ctx->stream));
    if ((rc = mark_built(ctx, out, st)) != PBGPU_OK)
        return rc;
    ctx->pending.push_back(tp);
    if (ctx->pending.size() >= 4096)
    {
        double ms; // bound the pending list (this drops the older timings)
        uint32_t n;
        rc = pbgpu_kernel_time(ctx, &ms, &n);
        if (rc)
            return rc;
    }
    return PBGPU_OK;
}

int pbgpu_build(pbgpu_ctx *ctx, uint16_t seq_idx, uint64_t first_iter, uint64_t n_iter, pbgpu_frames *out)
{
    return build_impl(ctx, seq_idx, first_iter, n_iter, out, nullptr);
}


// The fused form applies: three distinct sequences of kinds 1, 2, 3 (pbk_batch_kind), into three
// distinct 4-KiB-aligned buffers, each with frames to build; order[k] = the part of kind k + 1
static bool batch_fusable(pbgpu_ctx *ctx, uint32_t n, const uint16_t *seq_idx, const uint64_t *n_iter,
                          pbgpu_frames *const *outs, uint32_t order[3])
{
    if (n != 3)
        return false;
    bool seen[3] = {false, false, false};
    for (uint32_t i = 0; i < 3; ++i)
    {
        const seq_slot &S = ctx->seqs[seq_idx[i]];
        if (!S.loaded || !S.opt.batch || S.opt.kernel == PBO_K_LINEAR)
            return false;
        const int kd = pbk_batch_kind(&S.K);
        if (kd < 1 || kd > 3 || seen[kd - 1] || n_iter[i] == 0 || ((uintptr_t)outs[i]->data & 4095u) != 0)
            return false;
        seen[kd - 1] = true;
        order[kd - 1] = i;
        for (uint32_t j = 0; j < i; ++j)
            if (seq_idx[j] == seq_idx[i] || outs[j] == outs[i])
                return false;
    }
    return true;
}

int pbgpu_build_batch(pbgpu_ctx *ctx, uint32_t n, const uint16_t *seq_idx, const uint64_t *first_iter,
                      const uint64_t *n_iter, pbgpu_frames *const *outs)
{
    if (ctx == NULL || (n && (seq_idx == NULL || first_iter == NULL || n_iter == NULL || outs == NULL)))
        return PBGPU_EINVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (outs[i] == NULL || seq_idx[i] >= PB_MAX_SEQUENCES)
            return PBGPU_EINVAL;
    // every part's arguments first: a part that cannot be built fails the call before any part
    // is launched or reserves count records
    for (uint32_t i = 0; i < n; ++i)
    {
        const int rc = build_check(ctx, seq_idx[i], first_iter[i], n_iter[i], outs[i]);
        if (rc != PBGPU_OK)
            return rc;
    }
    HIPCHK(hipSetDevice(ctx->device));
    uint32_t order[3];
    if (!batch_fusable(ctx, n, seq_idx, n_iter, outs, order))
    {
        // no fused form: one launch per part, as pbgpu_build
        for (uint32_t i = 0; i < n; ++i)
        {
            const int rc = pbgpu_build(ctx, seq_idx[i], first_iter[i], n_iter[i], outs[i]);
            if (rc != PBGPU_OK)
                return rc;
        }
        return PBGPU_OK;
    }
    // every part on the context's stream, then one launch
    hipStream_t st = ctx->stream;
    const bool span = ctx->timing_mode == PBGPU_TIMING_SPAN;
    timing_pair tp = {nullptr, nullptr};
    if (!span)
    {
        const int rc = timed_pair(ctx, &tp);
        if (rc != PBGPU_OK)
            return rc;
    }
    batch_part bp[3]; // (build_impl orders each part after its buffer's and count ring's last stream)
    pb_kargs Ks[3];
    // a failure after parts reserved count records returns them (those records are never written)
    auto unreserve = [&](uint32_t parts) {
        for (uint32_t k = 0; k < parts; ++k)
            ctx->seqs[seq_idx[order[k]]].ctr_used -= bp[k].ctr_words;
        if (tp.a)
            ctx->pool.push_back(tp);
    };
    for (uint32_t k = 0; k < 3; ++k)
    {
        const uint32_t i = order[k];
        bp[k].st = st;
        bp[k].wgt = ctx->opt.batch_wgt;
        bp[k].ctr_words = 0;
        const int rc = build_impl(ctx, seq_idx[i], first_iter[i], n_iter[i], outs[i], &bp[k]);
        if (rc != PBGPU_OK || !bp[k].built)
        {
            unreserve(k + (rc == PBGPU_OK ? 1u : 0u));
            return rc != PBGPU_OK ? rc : PBGPU_EINVAL; // (n_iter > 0 was checked: not built is unreachable)
        }
        Ks[k] = bp[k].K;
    }
    // (every error exit from here to the launch returns the three parts' reservations)
#define HIPCHK_UNRES(call)                                                                   \
    do                                                                                       \
    {                                                                                        \
        const hipError_t u_ = (call);                                                        \
        if (u_ != hipSuccess)                                                                \
        {                                                                                    \
            unreserve(3);                                                                    \
            HIPCHK(u_);                                                                      \
        }                                                                                    \
    } while (0)
    if (span && ctx->span_n == 0)
    {
        if (ctx->span.a == nullptr)
        {
            HIPCHK_UNRES(hipEventCreate(&ctx->span.a));
            HIPCHK_UNRES(hipEventCreate(&ctx->span.b));
        }
        HIPCHK_UNRES(hipEventRecord(ctx->span.a, ctx->stream));
        for (bool &j : ctx->seq_in_span)
            j = false;
    }
    if (!span)
        HIPCHK_UNRES(hipEventRecord(tp.a, st));
    HIPCHK_UNRES(pbk_launch_batch(Ks, ctx->opt.batch_wgt, st));
#undef HIPCHK_UNRES
    if (span)
        ++ctx->span_n;
    else
    {
        HIPCHK(hipEventRecord(tp.b, st));
        ctx->pending.push_back(tp);
    }
    for (uint32_t i = 0; i < 3; ++i)
    {
        const int rc = mark_built(ctx, outs[i], st);
        if (rc != PBGPU_OK)
            return rc;
    }
    return PBGPU_OK;
}

int pbgpu_sync(pbgpu_ctx *ctx)
{
    if (ctx == NULL)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PBGPU_OK;
}

int pbgpu_frames_total(pbgpu_ctx *ctx, pbgpu_frames *f, uint64_t *total)
{
    if (ctx == NULL || f == NULL)
        return PBGPU_EINVAL;
    if (f->fixed_len || f->n_frames == 0)
    {
        if (total)
            *total = f->total_bytes;
        return PBGPU_OK;
    }
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    uint64_t t = 0;
    HIPCHK(hipMemcpyAsync(&t, f->offsets + f->n_frames, sizeof t, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    f->total_bytes = t;
    if (total)
        *total = t;
    return PBGPU_OK;
}

int pbgpu_copy_packed(pbgpu_ctx *ctx, const pbgpu_frames *f, void *dst, uint64_t byte_offset, uint64_t nbytes)
{
    if (ctx == NULL || f == NULL || dst == NULL || byte_offset + nbytes > f->capacity_bytes)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    HIPCHK(hipMemcpyAsync(dst, f->data + byte_offset, nbytes, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PBGPU_OK;
}

int pbgpu_copy_offsets(pbgpu_ctx *ctx, const pbgpu_frames *f, uint64_t *dst)
{
    if (ctx == NULL || f == NULL || dst == NULL)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    if (f->fixed_len)
    {
        for (uint64_t i = 0; i <= f->n_frames; ++i)
            dst[i] = i * f->fixed_len;
        return PBGPU_OK;
    }
    PB_JOIN(ctx);
    {
        const int mrc = materialize_offsets(ctx, f);
        if (mrc != PBGPU_OK)
            return mrc;
    }
    HIPCHK(hipMemcpyAsync(dst, f->offsets, (f->n_frames + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PBGPU_OK;
}

int pbgpu_host_register(pbgpu_ctx *ctx, void *ptr, size_t bytes)
{
    if (ctx == NULL || ptr == NULL)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipHostRegister(ptr, bytes, hipHostRegisterMapped));
    void *dev = NULL;
    if (hipHostGetDevicePointer(&dev, ptr, 0) == hipSuccess && dev != NULL)
        ctx->regs.push_back({(uint8_t *)ptr, bytes, (uint8_t *)dev});
    (void)hipGetLastError();
    return PBGPU_OK;
}

int pbgpu_host_unregister(pbgpu_ctx *ctx, void *ptr)
{
    if (ctx == NULL || ptr == NULL)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    int rc = pbgpu_land_wait(ctx, 0);
    if (rc != PBGPU_OK)
        return rc;
    for (size_t i = 0; i < ctx->regs.size(); ++i)
        if (ctx->regs[i].host == (uint8_t *)ptr)
        {
            ctx->regs.erase(ctx->regs.begin() + (long)i);
            break;
        }
    HIPCHK(hipHostUnregister(ptr));
    return PBGPU_OK;
}

// device address of [p, p + n) in a registered (mapped) range, or NULL
static uint8_t *mapped(pbgpu_ctx *ctx, uint8_t *p, uint64_t n)
{
    if (ctx->opt.umem_dma)
        return NULL;
    for (const auto &r : ctx->regs)
        if (p >= r.host && p + n <= r.host + r.bytes)
            return r.dev + (p - r.host);
    void *dev = NULL; // registered outside this context
    if (hipHostGetDevicePointer(&dev, p, 0) == hipSuccess && dev != NULL)
        return (uint8_t *)dev;
    (void)hipGetLastError();
    return NULL;
}

// Wait for a landing's event without paying a blocking wait's wake-up latency on short waits,
// and without holding a core for long ones (each TX thread waits this way; the GPU box gives a
// process a 16-CPU quota): poll for up to 50 us, then poll with sched_yield() between queries
// for up to 2 ms, then block in the runtime.
static double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static hipError_t spin_wait(hipEvent_t ev)
{
    hipError_t e;
    const double t0 = now_s();
    while ((e = hipEventQuery(ev)) == hipErrorNotReady)
    {
        const double dt = now_s() - t0;
        if (dt > 2e-3)
            return hipEventSynchronize(ev);
        if (dt > 50e-6)
            sched_yield();
    }
    return e;
}

int pbgpu_land_wait(pbgpu_ctx *ctx, uint32_t keep)
{
    if (ctx == NULL)
        return PBGPU_EINVAL;
    while (ctx->landings.size() > keep)
    {
        pbgpu_ctx::land_op op = ctx->landings.front();
        // a sender waits on every landing: poll the event rather than block in the runtime
        // (a blocking wait adds its wake-up latency to each landing; PBGPU_LAND_SPIN=0 blocks)
        hipError_t e = hipSuccess;
        if (ctx->opt.land_spin)
            e = spin_wait(op.ev);
        else
            e = hipEventSynchronize(op.ev);
        ctx->landings.pop_front();
        ctx->land_pool.push_back(op.ev);
        if (e != hipSuccess)
            return PBGPU_EIO;
        if (op.lens_out)
        {
            if (op.fixed_len)
                for (uint32_t i = 0; i < op.n; ++i)
                    op.lens_out[i] = (uint16_t)op.fixed_len;
            else
                memcpy(op.lens_out, ctx->h_lens + op.lens_off, (size_t)op.n * 2);
        }
    }
    return PBGPU_OK;
}

// Landing into memory that is not registered with HIP: the queued landings
// first (in order), then a strided DMA (fixed length) or a pinned staging copy.
static int land_unmapped(pbgpu_ctx *ctx, const pbgpu_frames *f, uint8_t *dst, uint32_t slot_stride,
                         uint64_t first_frame, uint32_t n, uint16_t *lens_out)
{
    PB_JOIN(ctx);
    int rc = pbgpu_land_wait(ctx, 0);
    if (rc != PBGPU_OK)
        return rc;
    hipStream_t ls = ctx->land_stream;
    if (f->fixed_len)
    {
        // strided DMA in runs of at most 32768 rows (a 2^18-row copy failed on the runtime)
        for (uint32_t i = 0; i < n; i += 32768)
        {
            const uint32_t rows = n - i < 32768 ? n - i : 32768;
            HIPCHK(hipMemcpy2DAsync(dst + (uint64_t)i * slot_stride, slot_stride,
                                    f->data + (first_frame + i) * f->fixed_len, f->fixed_len, f->fixed_len, rows,
                                    hipMemcpyDeviceToHost, ls));
        }
        HIPCHK(hipStreamSynchronize(ls));
        if (lens_out)
            for (uint32_t i = 0; i < n; ++i)
                lens_out[i] = (uint16_t)f->fixed_len;
        return PBGPU_OK;
    }
    std::vector<uint64_t> off(n + 1);
    HIPCHK(hipMemcpyAsync(off.data(), f->offsets + first_frame, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                          ls));
    HIPCHK(hipStreamSynchronize(ls));
    const uint64_t bytes = off[n] - off[0];
    if (ctx->h_stage_bytes < bytes)
    {
        if (ctx->h_stage)
            (void)hipHostFree(ctx->h_stage);
        ctx->h_stage = NULL;
        ctx->h_stage_bytes = 0;
        HIPCHK(hipHostMalloc((void **)&ctx->h_stage, bytes, 0));
        ctx->h_stage_bytes = bytes;
    }
    HIPCHK(hipMemcpyAsync(ctx->h_stage, f->data + off[0], bytes, hipMemcpyDeviceToHost, ls));
    HIPCHK(hipStreamSynchronize(ls));
    for (uint32_t i = 0; i < n; ++i)
    {
        const uint64_t len = off[i + 1] - off[i];
        if (len > slot_stride)
            return PBGPU_EINVAL;
        memcpy(dst + (uint64_t)i * slot_stride, ctx->h_stage + (off[i] - off[0]), len);
        if (lens_out)
            lens_out[i] = (uint16_t)len;
    }
    return PBGPU_OK;
}

// send_packet()'s memcpy into UMEM slot idx * FRAME_SIZE, af_xdp.c:200-214.
// Registered (mapped) UMEM: a scatter kernel on the landing stream stores each
// frame into its slot over the host link, queued behind the build of these
// frames only; the caller waits with pbgpu_land_wait (several landings may be
// in flight: their launch and completion latencies overlap).  Unregistered
// memory: a synchronous strided DMA (fixed length) or pinned staging copy.
int pbgpu_copy_to_umem_async(pbgpu_ctx *ctx, const pbgpu_frames *f, void *umem, uint32_t slot_stride,
                             uint32_t first_slot, uint64_t first_frame, uint32_t n, uint16_t *lens_out)
{
    if (ctx == NULL || f == NULL || umem == NULL || slot_stride == 0 || first_frame + n > f->n_frames)
        return PBGPU_EINVAL;
    if (n == 0)
        return PBGPU_OK;
    // a frame longer than a slot would overrun the next slot (or, in the last slot,
    // the UMEM allocation): refused, from the fixed length or the sequence's
    // longest frame (the reference does not check, af_xdp.c:214)
    if (f->fixed_len ? f->fixed_len > slot_stride
                     : (f->seq_idx >= PB_MAX_SEQUENCES || !ctx->seqs[f->seq_idx].loaded ||
                        ctx->seqs[f->seq_idx].max_flen > slot_stride))
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    if (!f->fixed_len)
    {
        const int mrc = materialize_offsets(ctx, f);
        if (mrc != PBGPU_OK)
            return mrc;
    }
    hipStream_t ls = ctx->land_stream;
    ctx->land_events = true;
    frames_events *fe = (frames_events *)f->reserved;
    if (fe && fe->built)
        HIPCHK(hipStreamWaitEvent(ls, fe->built, 0));
    else
        HIPCHK(hipStreamSynchronize(ctx->stream));
    uint8_t *dst = (uint8_t *)umem + (uint64_t)first_slot * slot_stride;
    uint8_t *dev_dst = mapped(ctx, dst, (uint64_t)n * slot_stride);
    if (dev_dst == NULL)
        return land_unmapped(ctx, f, dst, slot_stride, first_frame, n, lens_out);
    pbgpu_ctx::land_op op = {nullptr, lens_out, n, 0, f->fixed_len};
    if (f->fixed_len && f->fixed_len >= ctx->opt.land_dma_min)
    {
        // PBGPU_LAND_DMA_MIN: the copy engine, a strided DMA on the landing stream, in runs of
        // <= 32768 rows (1500 B, 2^18 frames: 56.1 vs 52.2 GB/s for the scatter kernel landing
        // alone, 43.1 vs 49.2 in bench.py's build + land; at 64 B the engine moves 218 Mpps against
        // the kernel's 540, profiles/r06/d2h/)
        for (uint32_t i = 0; i < n; i += 32768)
        {
            const uint32_t rows = n - i < 32768 ? n - i : 32768;
            HIPCHK(hipMemcpy2DAsync(dst + (uint64_t)i * slot_stride, slot_stride,
                                    f->data + (first_frame + i) * f->fixed_len, f->fixed_len, f->fixed_len, rows,
                                    hipMemcpyDeviceToHost, ls));
        }
    }
    else if (f->fixed_len)
    {
        // a tight slot (no longer than the frame rounded up to 64 B, e.g. --umemslot 64 for 60- or
        // 64-B frames) is written whole: contiguous slots then reach the host as contiguous writes
        // (64 B: 783 Mpps into back-to-back slots against 535-541 for 64-B writes into 128-B to
        // 4-KiB slots, profiles/r06/d2h/d2h_slots.jsonl); otherwise only the frame's bytes
        const uint32_t r64 = (f->fixed_len + 63u) & ~63u;
        const uint32_t wlen = slot_stride <= r64 ? slot_stride : f->fixed_len;
        HIPCHK(pbk_launch_scatter_fixed(f->data + first_frame * f->fixed_len, f->fixed_len, wlen, n,
                                        f->capacity_bytes - first_frame * f->fixed_len, dev_dst, slot_stride, ls));
    }
    else
    {
        // lengths: a contiguous range of the context's ring (device + pinned host), FIFO
        // with the queued landings; never a stream-ordered allocation or a pageable copy
        if (ctx->lens_cap < n)
        {
            int rc = pbgpu_land_wait(ctx, 0);
            if (rc != PBGPU_OK)
                return rc;
            HIPCHK(hipStreamSynchronize(ls));
            if (ctx->d_lens)
                (void)hipFree(ctx->d_lens);
            if (ctx->h_lens)
                (void)hipHostFree(ctx->h_lens);
            ctx->d_lens = NULL;
            ctx->h_lens = NULL;
            ctx->lens_cap = 0;
            const uint32_t cap = n > (1u << 16) ? n : (1u << 16);
            HIPCHK(hipMalloc((void **)&ctx->d_lens, (size_t)cap * 2));
            HIPCHK(hipHostMalloc((void **)&ctx->h_lens, (size_t)cap * 2, 0));
            ctx->lens_cap = cap;
            ctx->lens_head = 0;
        }
        uint32_t off = ctx->lens_head + n <= ctx->lens_cap ? ctx->lens_head : 0;
        // wait for the queued landings whose ranges the new one would overwrite
        for (;;)
        {
            bool clash = false;
            for (const auto &q : ctx->landings)
                if (!q.fixed_len && q.lens_off < off + n && off < q.lens_off + q.n)
                    clash = true;
            if (!clash)
                break;
            int rc = pbgpu_land_wait(ctx, (uint32_t)ctx->landings.size() - 1);
            if (rc != PBGPU_OK)
                return rc;
        }
        HIPCHK(pbk_launch_scatter(f->data, f->offsets, first_frame, n, dev_dst, slot_stride, ctx->d_lens + off, ls));
        HIPCHK(hipMemcpyAsync(ctx->h_lens + off, ctx->d_lens + off, (size_t)n * 2, hipMemcpyDeviceToHost, ls));
        op.lens_off = off;
        ctx->lens_head = off + n;
    }
    if (!ctx->land_pool.empty())
    {
        op.ev = ctx->land_pool.back();
        ctx->land_pool.pop_back();
    }
    else
        HIPCHK(hipEventCreateWithFlags(&op.ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(op.ev, ls));
    ctx->landings.push_back(op);
    // the next pbgpu_build into this buffer waits for the landing (pbgpu.h)
    frames_events *fw = frames_ev(const_cast<pbgpu_frames *>(f));
    if (fw == NULL)
        return PBGPU_ENOMEM;
    if (fw->landed == nullptr)
        HIPCHK(hipEventCreateWithFlags(&fw->landed, hipEventDisableTiming));
    HIPCHK(hipEventRecord(fw->landed, ls));
    fw->land_pending = true;
    return PBGPU_OK;
}

int pbgpu_copy_to_umem(pbgpu_ctx *ctx, const pbgpu_frames *f, void *umem, uint32_t slot_stride, uint32_t first_slot,
                       uint64_t first_frame, uint32_t n, uint16_t *lens_out)
{
    int rc = pbgpu_copy_to_umem_async(ctx, f, umem, slot_stride, first_slot, first_frame, n, lens_out);
    if (rc == PBGPU_OK)
        rc = pbgpu_land_wait(ctx, 0);
    return rc;
}

// A slot's device counters: the shards' sums; fixed-length kernels add only the bytes they
// stored (one atomic per workgroup: each is a memory-side transaction, 0.4-1% of a small-frame
// launch's traffic as two), so their frames are bytes / length.
// sum: slot i's shard sums {frames, bytes} (read_counter_sums)
static void slot_counts(const pbgpu_ctx *ctx, const unsigned long long *sum, int i, uint64_t *p, uint64_t *b)
{
    uint64_t pp = sum[0], bb = sum[1];
    const seq_slot &S = ctx->seqs[i];
    if (S.loaded && S.K.fixed_len)
        pp = bb / S.K.fixed_len;
    *p = pp + ctx->ctr_base[i][0];
    *b = bb + ctx->ctr_base[i][1];
}

// Slots [first, first + n_seq)'s shard sums into ctx->h_ctr_sum[2 (i - first) ..], by a kernel
// writing the mapped host buffer (on ctx->stream, after everything issued there), then a stream
// synchronisation.  A pageable hipMemcpy of the shards instead (8 KiB per slot) cost 8-16 ms on
// its first use for three slots, an idle gap before bench.py's timed configs[4] steps that cost
// their first 25 launches up to 30% (profiles/r05/ab/gap.log, profiles/r05/prof/cfg/trace_c5_mix*)
static int read_counter_sums(pbgpu_ctx *ctx, int first, int n_seq)
{
    HIPCHK(pbk_launch_ctr_read(ctx->d_counters + PB_CTR_WORDS * (size_t)first, (uint32_t)n_seq,
                               ctx->d_ctr_sum, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return PBGPU_OK;
}

int pbgpu_counters(pbgpu_ctx *ctx, uint64_t *pckts, uint64_t *bytes, int n_seq)
{
    if (ctx == NULL || n_seq < 0 || n_seq > PB_MAX_SEQUENCES)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    if (n_seq == 0)
        return PBGPU_OK;
    // the launches' pending per-workgroup records first, then the shards' sums
    for (int i = 0; i < n_seq; ++i)
    {
        const int frc = ctr_fold(ctx, i, ctx->stream);
        if (frc != PBGPU_OK)
            return frc;
    }
    const int rrc = read_counter_sums(ctx, 0, n_seq);
    if (rrc != PBGPU_OK)
        return rrc;
    for (int i = 0; i < n_seq; ++i)
    {
        uint64_t p = 0, b = 0;
        slot_counts(ctx, ctx->h_ctr_sum + 2 * i, i, &p, &b);
        if (pckts)
            pckts[i] = p;
        if (bytes)
            bytes[i] = b;
    }
    return PBGPU_OK;
}

int pbgpu_set_timing(pbgpu_ctx *ctx, int mode)
{
    if (ctx == NULL || (mode != PBGPU_TIMING_LAUNCH && mode != PBGPU_TIMING_SPAN))
        return PBGPU_EINVAL;
    double ms; // close what the old mode measured
    uint32_t n;
    const int rc = pbgpu_kernel_time(ctx, &ms, &n);
    if (rc)
        return rc;
    ctx->timing_mode = mode;
    return PBGPU_OK;
}

int pbgpu_kernel_time(pbgpu_ctx *ctx, double *ms_total, uint32_t *n_launches)
{
    if (ctx == NULL)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx); // the span ends after every sequence stream's launches
    double tot = 0;
    uint32_t n = 0;
    if (ctx->span_n)
    {
        HIPCHK(hipEventRecord(ctx->span.b, ctx->stream));
        HIPCHK(hipEventSynchronize(ctx->span.b));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ctx->span.a, ctx->span.b));
        tot += ms;
        n += ctx->span_n;
        ctx->span_n = 0;
    }
    for (auto &p : ctx->pending)
    {
        HIPCHK(hipEventSynchronize(p.b));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
        tot += ms;
        ++n;
        ctx->pool.push_back(p);
    }
    ctx->pending.clear();
    if (ms_total)
        *ms_total = tot;
    if (n_launches)
        *n_launches = n;
    return PBGPU_OK;
}

int pbgpu_kernel_times(pbgpu_ctx *ctx, double *ms_each, uint32_t cap, uint32_t *n_launches)
{
    if (ctx == NULL || (cap && ms_each == NULL))
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    uint32_t n = 0;
    for (auto &p : ctx->pending)
    {
        HIPCHK(hipEventSynchronize(p.b));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
        if (n < cap)
            ms_each[n] = ms;
        ++n;
        ctx->pool.push_back(p);
    }
    ctx->pending.clear();
    if (n_launches)
        *n_launches = n;
    return PBGPU_OK;
}

static int fill_probe_buf(pbgpu_ctx *ctx, void *buf, uint64_t bytes, uint32_t reps, double *ms_per_shape,
                          int *best_shape);

int pbgpu_fill_probe_ex(pbgpu_ctx *ctx, uint64_t bytes, uint32_t reps, double *ms_per_shape, int *best_shape)
{
    if (ctx == NULL || bytes < 16 || reps == 0)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    void *buf = NULL;
    HIPCHK(hipMalloc(&buf, bytes));
    const int rc = fill_probe_buf(ctx, buf, bytes, reps, ms_per_shape, best_shape);
    (void)hipFree(buf);
    return rc;
}

int pbgpu_fill_probe_at(pbgpu_ctx *ctx, void *dst, uint64_t bytes, uint32_t reps, double *ms_per_shape)
{
    if (ctx == NULL || dst == NULL || bytes < 16 || reps == 0)
        return PBGPU_EINVAL;
    HIPCHK(hipSetDevice(ctx->device));
    PB_JOIN(ctx);
    return fill_probe_buf(ctx, dst, bytes, reps, ms_per_shape, NULL);
}

static int fill_probe_buf(pbgpu_ctx *ctx, void *buf, uint64_t bytes, uint32_t reps, double *ms_per_shape,
                          int *best_shape)
{
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    double best = 1e30;
    int bi = 0;
    for (int mode = 0; mode < PBGPU_FILL_SHAPES; ++mode) // pbk_launch_fill's shapes; the fastest is the peak
    {
        double mode_best = 1e30;
        for (int trial = 0; trial < 2; ++trial)
        {
            HIPCHK(pbk_launch_fill(buf, bytes, mode, ctx->stream)); // warm-up
            HIPCHK(hipEventRecord(a, ctx->stream));
            for (uint32_t r = 0; r < reps; ++r)
                HIPCHK(pbk_launch_fill(buf, bytes, mode, ctx->stream));
            HIPCHK(hipEventRecord(b, ctx->stream));
            HIPCHK(hipEventSynchronize(b));
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, a, b));
            mode_best = ms / reps < mode_best ? ms / reps : mode_best;
        }
        if (ms_per_shape)
            ms_per_shape[mode] = mode_best;
        if (mode_best < best)
            best = mode_best, bi = mode;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (best_shape)
        *best_shape = bi;
    return PBGPU_OK;
}

int pbgpu_fill_probe(pbgpu_ctx *ctx, uint64_t bytes, uint32_t reps, double *ms_per_launch)
{
    double ms[PBGPU_FILL_SHAPES];
    int bi = 0;
    const int rc = pbgpu_fill_probe_ex(ctx, bytes, reps, ms, &bi);
    if (rc == PBGPU_OK && ms_per_launch)
        *ms_per_launch = ms[bi];
    return rc;
}

const char *pbgpu_fill_shape_name(int shape)
{
    return pbk_fill_shape_name(shape);
}

int pbgpu_kernel_name(pbgpu_ctx *ctx, uint16_t seq_idx, char *buf, size_t n)
{
    if (ctx == NULL || seq_idx >= PB_MAX_SEQUENCES || buf == NULL || n == 0)
        return PBGPU_EINVAL;
    const seq_slot &S = ctx->seqs[seq_idx];
    if (!S.loaded)
        return PBGPU_ENOENT;
    const pb_kargs &K = S.K;
    if (K.vp)
        snprintf(buf, n, "pb_vpage_kernel<%u, %u> (after pb_vrec_kernel<%u, %u>)", K.hl,
                 (K.flags & PBK_L4_CSUM) ? 1u : 0u, K.hl, (K.flags & PBK_L4_CSUM) ? 1u : 0u);
    else if (K.vl)
        snprintf(buf, n, "pb_vline_kernel<%u, %u>", K.hl, (K.flags & PBK_L4_CSUM) ? 1u : 0u);
    else if (K.fst_g)
        snprintf(buf, n, "pb_fstage_kernel<%u, %u>", K.fst_g, (K.flags & PBK_L4_CSUM) ? 1u : 0u);
    else if (K.stage_win && K.vst)
        snprintf(buf, n, "pb_vstage_kernel<%u, %u>", K.gpf_g, (K.flags & PBK_L4_CSUM) ? 1u : 0u);
    else if (K.stage_win)
        snprintf(buf, n, "pb_stage_kernel<%u, %u>", K.gpf_g, K.gpf_rmode);
    else if (K.gpf_g)
        snprintf(buf, n, "pb_gpf_kernel<%u, %u>", K.gpf_g, K.gpf_rmode);
    else if (K.xs_np && K.img && K.img_solo && S.opt.kernel != PBO_K_LINEAR)
        snprintf(buf, n, "pb_ximg_kernel<%u>", (uint32_t)PB_WG);
    else if (K.xs_np && K.xp && S.opt.kernel != PBO_K_LINEAR)
        snprintf(buf, n, "pb_xpage_kernel<%u, %u, %s, %u, %s>%s", K.small_ndw, K.proto, K.pl0.random ? "true" : "false",
                 K.xp_wgt, K.fixed_len % 4 == 0 ? "true" : "false",
                 K.img ? " (in pbgpu_build_batch: pb_ximg_body)" : "");
    else if (K.xs_np && S.opt.kernel != PBO_K_LINEAR)
        snprintf(buf, n, "pb_xsmall_kernel<%u, %u, %s, %u>", K.small_ndw, K.proto, K.pl0.random ? "true" : "false",
                 (uint32_t)PB_WG);
    else
        snprintf(buf, n, "pb_small_kernel<%u, %u, %s, %u, %u>", K.small_ndw, K.proto, K.pl0.random ? "true" : "false",
                 K.small_wgt ? K.small_wgt : (uint32_t)PB_WG, K.fixed_len % 4 == 2 ? 2u : 0u);
    return PBGPU_OK;
}

size_t pbgpu_abi_size(int which)
{
    switch (which)
    {
    case 0: return sizeof(pb_sequence_t);
    case 1: return sizeof(pb_payload_opt_t);
    case 2: return sizeof(pbgpu_frames);
    case 3: return offsetof(pb_sequence_t, ip.ranges);
    case 4: return offsetof(pb_sequence_t, pls);
    case 5: return offsetof(pb_sequence_t, pl_cnt);
    case 6: return offsetof(pbgpu_frames, total_bytes);
    default: return 0;
    }
}

} // extern "C"
