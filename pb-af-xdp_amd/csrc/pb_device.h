// pb_device.h — device-side data layout and arithmetic shared by the frame-
// build kernels (pbgpu_kernels.hip).  CDNA4 / gfx950 only.
//
// Reference arithmetic restated:
//   rand_r        glibc, 3 LCG steps          (call sites sequence.c:345-554)
//   rand_num      min + rand_r(copy) % (max-min+1)   (PB-Common, un-vendored)
//   rand_ip       (net & ~hm) | (r0 & hm)             (PB-Common, un-vendored)
//   checksums     RFC 1071 in the little-endian word domain, as csum.h does
//                 on x86 (sequence.c:569-602)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define PB_WG 256                          // threads per workgroup (4 waves)
#define PB_IMG_DW 16                       // header image: 64 B per frame
#define PB_IMG_STRIDE 20                   // dwords per frame image row in LDS (16 used + pad: conflict-free b128 rows)
#define PB_JNEG 80                         // jump table starts at j = -80
#define PB_STAGE_L48 72                    // lcg48 entries the staged kernel keeps in LDS (> 4 + 64)
#define PB_STAGE_LDS(wgf) ((size_t)(wgf) * (16 + 8) * 4 + 4 + PB_STAGE_L48 * 8) // its LDS besides the stage
#define PB_LCG48_N 4200                    // lcg48[m] = L^(48 m), m < 4200 (> 16-B chunks of a 64 KiB frame)
#define PB_XPG 4096                        // XCD-owned page bytes (pb_xsmall_kernel, pb_xpage_kernel)
#define PB_XREG (PB_XPG + 256)             // LDS bytes per page region (128 B slack either side)
#define PBK_FILL_SHAPES 15                 // write-roofline probe shapes (pbk_launch_fill)
#define PB_XNP_MAX 8                       // pb_xsmall_kernel: pages per workgroup, 4 (64-B frames) or 8 (128-B)
#define PB_VL_GRP 32                       // length pass: build workgroups per group sum (vblk_l2 entry)
#ifndef PB_CTR_SHARDS
#define PB_CTR_SHARDS 64                   // per-sequence counter shards (workgroup b adds to shard b % 64)
#endif
#define PB_CTR_STRIDE 16                   // u64 words per shard: one 128-B line each ({frames, bytes} + pad)

// glibc LCG
#define PB_LCG_A 1103515245u
#define PB_LCG_C 12345u

enum pb_kflags : uint32_t
{
    PBK_RND_TTL = 1u << 0,
    PBK_RND_ID = 1u << 1,
    PBK_RND_SADDR = 1u << 2,
    PBK_RND_SPORT = 1u << 3,
    PBK_RND_DPORT = 1u << 4,
    PBK_IP_CSUM = 1u << 5,
    PBK_L4_CSUM = 1u << 6,
    PBK_IPH_SINGLE = 1u << 7,
    PBK_LITERAL = 1u << 8,
    PBK_SUM_IN_A = 1u << 9,   // payload sums computed per frame in phase A
    PBK_PSEUDO = 1u << 10,    // UDP/TCP pseudo header (not ICMP)
};

// n % d for n < 2^31 by multiply-shift (Granlund-Montgomery, N = 31):
// m = ceil(2^(31+l) / d), l = ceil(log2 d), sh = 31 + l.
struct pb_div
{
    uint32_t d, m, sh;
};

// one payload of the sequence (sequence_t.pls[i] after setup)
struct pb_pl
{
    uint32_t random;   // 1: length + bytes drawn per iteration
    uint32_t min_len;
    pb_div len;        // divisor max_len - min_len + 1
    uint32_t blob_off; // static bytes at blob + blob_off (16-B zero pad around)
    uint32_t slen;     // static length
    uint32_t ssum;     // static bytes' little-endian 16-bit word sum (unfolded)
};

struct pb_kargs
{
    uint32_t tmpl[16];  // header template bytes 0..63 as LE dwords, random fields 0
    uint32_t flags;
    uint32_t hl;        // 42 (UDP, ICMP) or 54 (TCP)
    uint32_t l4len;     // 8 or 20
    uint32_t proto;
    uint32_t csum_dw;   // image dword holding the L4 checksum
    uint32_t csum_hi;   // 1: checksum in the high half of that dword
    uint32_t ttl_min;
    pb_div ttl;
    uint32_t id_min;
    pb_div id;
    pb_div rng;
    pb_div port;        // 65535
    const uint2 *ranges; // {net & ~hm, hm} host order
    uint32_t pl_cnt;
    pb_pl pl0;
    const pb_pl *pls;
    const uint8_t *blob;
    const uint2 *jump;  // jump[j + PB_JNEG] = (A, C): state_j = A * st0 + C = L^(3(j+1))(st0)
    uint64_t seed_base;
    uint32_t seq;
    uint64_t first_iter;
    uint64_t n_frames;
    uint64_t total_bytes;   // fixed length only
    uint32_t fixed_len;     // 0 -> variable
    pb_div flen;            // division by fixed_len
    const uint64_t *offsets;
    uint8_t *out;
    unsigned long long *counters; // [2] pckts, bytes of this sequence
    uint32_t small_ndw;     // >0: small fixed frames, one lane per frame, NDW dwords per lane
    uint32_t gpf_g;         // >0: group-per-frame kernel with G lanes per frame
    uint32_t gpf_rmode;     // 1: all payloads random, 0: all static, 2: mixed
    uint32_t gpf_fpw;       // frames per workgroup (multiple of 256 / gpf_g, <= 256)
    uint32_t stage_win;     // >0: staged kernel, window of W workgroup bytes per stage fill (>= longest frame)
    uint32_t stage_bytes;   // its LDS stage size (multiple of 16, >= W + longest frame + 32)
    uint32_t stage_wgf;     // its frames per workgroup (<= its threads per workgroup)
    uint32_t stage_wgt;     // its threads per workgroup: 256, or 64 (one wave, barriers are wave-local)
    const uint2 *lcg48;     // lcg48[m] = L^(48 m): one 16-B chunk of payload = 48 LCG steps
    uint32_t stail[32];     // small kernel, static payload: payload bytes at frame dwords p0.. (p0 = (hl-2)/4)
    // XCD-owned small kernel (pb_xsmall_kernel), frame lengths dividing 4096: pages of 4 KiB hold
    // 1 << xs_fp_shift frames; a workgroup owns xs_np = 256 >> xs_fp_shift pages
    uint32_t xs_fp_shift;
    uint32_t xs_np;
    uint32_t xs_nch;        // pages of this launch's stream
    uint32_t xs_full;       // workgroups [0, xs_full) own XCD-strided pages; the rest take the tail pages in order
    uint32_t xs_grid;       // >0: launch pb_xsmall_kernel with this many workgroups
    // pb_xpage_kernel (the xs_* page shape for lengths % 4 == 0 that do not divide 4096)
    uint32_t xp;            // 1: use it
    uint32_t xp_fpp;        // frame slots per page: the most frames touching one page
    pb_div xp_div;          // division by xp_fpp
    double xp_inv;          // 1.0 / flen
    uint32_t xp_wgt;        // threads per workgroup: 256 (two slots per lane) or 512 (one)
    // fixed-length staged kernel (pb_fstage_kernel): frame length a multiple of 4, every
    // payload random, stream rule; one frame per G-lane group per window of 256 / G frames
    uint32_t fst_g;         // >0: launch it with G lanes per frame (16, 32, 64)
    uint32_t fst_wgf;       // frames per workgroup (a multiple of 256 / G, <= 256)
    uint32_t fst_sb;        // bytes per stage buffer (multiple of 16)
    uint32_t fst_nbuf;      // stage buffers: 2 (window w + 1 is built while w streams out) or 1
    uint32_t vst;           // 1: the stage_* shape runs pb_vstage_kernel (every payload random, stream rule)
    uint32_t vst_shape;     // pb_vstage_kernel shape options (PBGPU_VST_SHAPE; each parity-tested): bit 4 fixed
                            // 8-lane groups, bit 5 no 32-lane groups, bit 6 workgroup edges at frame starts,
                            // bit 8 no longest-first window order
    uint32_t lds_pad;       // dynamic LDS added to the build launch: caps its workgroups per CU
    // pb_vstage_kernel, variable length: per-workgroup length sums (stage_wgf frames each) and
    // their exclusive scan per PB_VL_GRP workgroups (pb_len_wgsum + pb_scan_blocks); the kernel then
    // writes offsets_w for its own frames.  Null: offsets[] was scanned beforehand (3 passes).
    const uint32_t *vblk_sum;
    const unsigned long long *vblk_l2;
    uint64_t *offsets_w;
    // (appended last: the fields above keep their kernel-argument offsets)
    // literal rule, several payloads: lit_stop[i] = min { j > i : setup data_len[j] <= j } (<= 64)
    const uint32_t *lit_stop;
    uint32_t small_wgt;     // pb_small_kernel's threads (= frames) per workgroup: 256 (0), 128 or 64
    // pb_vline_kernel (packed variable lengths, every payload random, stream rule)
    const uint32_t *orbit;  // LCG-orbit prefix sums: orbit[t] = {PE(t << PB_ORB_SH), PO(..)} mod 0xFFFF (u16 pair)
    uint32_t orbit_tot;     // PE(2^24) mod 0xFFFF (= PO(2^24)): runs that wrap the orbit
    uint32_t vl;            // 1: launch pb_vline_kernel
    uint32_t vl_wgf;        // its own frames per workgroup (<= 256 - PB_VST_GHOSTS)
    uint32_t vl_nl48;       // lcg48 entries it keeps in LDS (chunks of the longest frame + 2)
    uint32_t vl_nlines;     // its line-map entries (128-B lines of the longest workgroup region)
    // pb_vline_kernel: 4-B offsets (the low word of each frame's offset) and each workgroup
    // region's 64-bit start, instead of 8-B offsets; pbgpu.cpp expands them on first use
    uint32_t *offsets32;
    unsigned long long *vl_rstart;
    // pb_xpage_kernel: 1 when the launch's last page index times 4096 % flen reaches 2^31 (the
    // first frame of a page then takes the 64-bit path)
    uint32_t xp_fa_hi;
    // this launch's per-workgroup counts (pb_count): u32 bytes per workgroup for fixed-length
    // sequences, {frames, bytes} for variable ones, at position pb_xcd_region(blockIdx.x); the
    // host folds them into `counters` (pb_ctr_fold).  Null: one atomic per workgroup instead.
    uint32_t *ctr_slots;
    // pb_ximg_kernel (static-payload ICMP frames on XCD-owned pages, one wave per page): img holds
    // the stream's first img_np pages, built at load (the static bytes repeat with that period);
    // page c starts as a copy of page c mod img_np and each frame's IPv4 ID, TTL, checksum and
    // source address are written over it.  Null: pb_xpage_kernel.
    const uint32_t *img;
    uint32_t img_np;
    pb_div img_div;         // division by img_np
    uint32_t img_solo;      // 1: single builds too (PBGPU_XP_IMG=2); else only pb_batch_kernel's part
    // pb_orbit_sum (pb_vline_kernel, pb_vrec_kernel): the discrete log mod 2^12 by table, entry
    // y mod 2^12 = p | (M^p(0) mod 2^24 >> 12) << 12, p = the position of y on M's orbit mod 2^12
    const uint32_t *dlog12;
    // packed variable lengths as XCD-owned 4-KiB pages (pb_vrec_kernel + pb_vpage_kernel, DESIGN.md
    // 5.5): per frame {seed, L4 checksum | length << 16}; per page {the frame holding its first
    // byte, that frame's start - the page's start}
    uint32_t vp;            // 1: launch them instead of pb_vline_kernel
    uint32_t vp_nfp;        // frame slots per page (the most frames touching one page, <= 64)
    uint32_t vp_grid;       // page-kernel workgroups (4 pages each): the launch's longest possible stream
    uint2 *vp_rec;
    uint2 *vp_pt;
    const uint2 *lcg48i;    // lcg48i[c] = L^(-48 c), c < PB_VP_NCI
    const uint4 *m16;       // chunk byte masks by plo + phi (PB_VL_NMASK rows: bytes [plo, phi))
};
// pb_vpage_kernel: page-relative byte u = start - page start + PB_VP_BIAS (frames < 4 KiB start
// after the previous page's start), 16-B chunk indices u >> 4 < PB_VP_NCI
#define PB_VP_BIAS 4096u
#define PB_VP_NCI 512u
// its LDS: 33 chunk masks and a count record per wave, then per wave nfp 16-B records,
// nfp * nsp + 1 header chunks and 256 chunk marks
#define PB_VP_WAVE_LDS(nfp, nsp) ((size_t)(nfp) * 16 * (1 + (size_t)(nsp)) + 16 + 256)
#define PB_VP_LDS(nfp, nsp, nw) ((size_t)PB_VL_NMASK * 16 + 8 * (size_t)(nw) + (nw) * PB_VP_WAVE_LDS(nfp, nsp))
// pb_fstage_kernel's LDS besides the stage: header image (16 dwords) + z, checksum start per frame
#define PB_FST_LDS(wgf) ((size_t)(wgf) * (16 + 2) * 4)
// pb_vstage_kernel's LDS besides the stage: lcg48 entries, header image + start, length, z, header
// sum, build order per frame, window list
// (arrays for wgf own frames + PB_VST_GHOSTS earlier frames sharing the first 128-B line)
#define PB_VST_GHOSTS 4
#define PB_VST_PRO 576 // pb_vstage_kernel prologue records: 16 jump entries, 12 starts / S0 parts, 4 wave sums, template, 17 chunk masks (16-B multiple)
#define PB_VST_HV0 4u  // per-frame header dwords kept in LDS: [4, 13) = IPv4 from tot_len to the L4 checksum
#define PB_VST_HVN 9u  // (UDP csum dword 10, TCP 12, ICMP 9); dwords 0-3 and 13-15 are the template's
#define PB_VST_CAP(wgf) (((size_t)(wgf) + PB_VST_GHOSTS + 1) & ~(size_t)1)
// pb_vline_kernel's LDS: 256 B of prologue records, then per frame slot (own + ghosts) a 16-B
// record and nsp 16-B header chunks, a zero chunk and 17 chunk masks, the lcg48 entries, the
// line map (u16)
#define PB_VL_STEP 16384u // bytes of a workgroup's region per step (4 waves x 4 KiB)
#define PB_ORB_SH 5 // orbit prefix sums sampled every 2^PB_ORB_SH positions (2 MiB table)
#define PB_VL_NMASK 33 // pb_vline_kernel's chunk masks: one table row per (plo + phi)
#define PB_VL_LDS(wgf, nsp, nl48, nlines)                                                                       \
    ((size_t)256 + ((size_t)(wgf) + PB_VST_GHOSTS) * 16 * (1 + (size_t)(nsp)) + (1 + PB_VL_NMASK) * 16 +         \
     (size_t)(nl48) * 8 +                                                                                        \
     (((size_t)(nlines) + 7) & ~(size_t)7) * 2)
#define PB_VST_LDS(wgf) ((size_t)PB_STAGE_L48 * 8 + PB_VST_PRO + PB_VST_CAP(wgf) * (PB_VST_HVN + 5) * 4 + (PB_VST_CAP(wgf) + 2) * 4)

__device__ __forceinline__ uint32_t pb_mod(uint32_t n, const pb_div &v)
{
    uint32_t q = (uint32_t)(((uint64_t)n * v.m) >> v.sh);
    return n - q * v.d;
}

__device__ __forceinline__ uint32_t pb_divq(uint32_t n, const pb_div &v)
{
    return (uint32_t)(((uint64_t)n * v.m) >> v.sh);
}

// glibc rand_r on a copy of the seed (PB-Common rand_num takes it by value).
__device__ __forceinline__ uint32_t pb_rand_r(uint32_t s)
{
    uint32_t n1 = s * PB_LCG_A + PB_LCG_C;
    uint32_t n2 = n1 * PB_LCG_A + PB_LCG_C;
    uint32_t n3 = n2 * PB_LCG_A + PB_LCG_C;
    return (((n1 >> 16) & 0x7FFu) << 20) ^ (((n2 >> 16) & 0x3FFu) << 10) ^ ((n3 >> 16) & 0x3FFu);
}

__device__ __forceinline__ uint32_t pb_seed(uint64_t seed_base, uint32_t seq, uint64_t k)
{
    uint64_t z = (seed_base ^ (((uint64_t)seq << 48) + k)) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)(z ^ (z >> 31));
}

__device__ __forceinline__ uint32_t pb_bswap16(uint32_t v)
{
    return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu);
}

__device__ __forceinline__ uint32_t pb_fold(uint32_t s)
{
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return s;
}

__device__ __forceinline__ uint32_t pb_halves(uint32_t d)
{
    return (d & 0xFFFFu) + (d >> 16);
}

typedef unsigned short pb_u16x2 __attribute__((ext_vector_type(2)));

// acc + low16(d) + high16(d) in one v_dot2_u32_u16
__device__ __forceinline__ uint32_t pb_add_halves(uint32_t acc, uint32_t d)
{
    const pb_u16x2 one = {1, 1};
    return __builtin_amdgcn_udot2(__builtin_bit_cast(pb_u16x2, d), one, acc, false);
}
