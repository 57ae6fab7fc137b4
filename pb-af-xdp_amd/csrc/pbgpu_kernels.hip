// pbgpu_kernels.hip — MI355X (gfx950) frame-build kernels.
//
// Hot path: PB-AF-XDP thread_hdl() loop body, src/sequence.c:433-602, for a
// batch of iterations at once: per frame the seed -> r0 -> TTL / ID / source IP
// / ports / payload length (sequence.c:434-527, 548), the header image
// (sequence.c:150-258), the payload bytes (glibc rand_r low byte,
// sequence.c:552-555, in 24-bit LCG arithmetic), the L4 checksum
// (csum_tcpudp_magic / icmp_csum, sequence.c:563-594) and tot_len + the IPv4
// checksum (sequence.c:596-602), written packed into HBM.  Kernel by frame
// shape (selection in pbgpu_load_sequence):
//   pb_xsmall_kernel / pb_xpage_kernel / pb_small_kernel   frames <= 128 B, one lane per frame
//   pb_fstage_kernel                                      fixed length > 128 B, random payload
//   pb_vstage_kernel                                      packed variable length, random payload
//   pb_stage_kernel                                       static / mixed payloads, the literal rule
//   pb_gpf_kernel                                         frames too long for an LDS stage
// The template, CIDR table pointers and divisors arrive as kernel arguments
// (scalar registers); no inter-workgroup communication; no atomics to HBM
// except two counter adds per launch.
#include "pb_device.h"

#define PB_SCAN_ITEMS 8    // frames per thread in the length scan kernels

typedef uint32_t pb_u32x4 __attribute__((ext_vector_type(4)));

namespace {

struct pb_frame_pl
{
    uint32_t random;
    uint32_t plen;
    uint32_t nvalid;   // random bytes actually drawn (literal rule: <= 1)
    uint32_t st0;      // LCG state entering the payload (random)
    uint32_t blob_off; // static
    uint32_t ssum;     // static word sum (folded)
};

// L^(3 n)(s): the seed after n rand_r calls.
__device__ __forceinline__ uint32_t pb_jump(const pb_kargs &K, uint32_t s, uint32_t n)
{
    if (n == 0)
        return s;
    const uint2 t = K.jump[n - 1 + PB_JNEG];
    return t.x * s + t.y;
}

// One payload's draw from the seed state `cur` entering it (sequence.c:529-561).
__device__ __forceinline__ pb_frame_pl pb_payload_of(const pb_pl &P, uint32_t cur, uint32_t flags)
{
    pb_frame_pl r;
    if (P.random)
    {
        r.random = 1;
        r.plen = P.min_len + pb_mod(pb_rand_r(cur), P.len);
        r.nvalid = (flags & PBK_LITERAL) ? min(r.plen, 1u) : r.plen;
        r.st0 = cur;
        r.blob_off = 0;
        r.ssum = 0;
    }
    else
    {
        r.random = 0;
        r.plen = P.slen;
        r.nvalid = P.slen;
        r.st0 = 0;
        r.blob_off = P.blob_off;
        r.ssum = P.ssum;
    }
    return r;
}

// Payload i of an iteration whose seed is s (sequence.c:529-561).  The payload
// record is read in place (kernel argument or device table): a local copy chosen
// from either became a stack object, 16 B of scratch stores per lane per
// workgroup (~4% of the staged kernels' HBM writes, PMC WRITE_SIZE).
template <bool LIT = true> // false: kernels that never run the literal rule (no dead loop in them)
__device__ __forceinline__ pb_frame_pl pb_payload(const pb_kargs &K, uint32_t s, uint32_t i)
{
    if (K.pl_cnt == 1)
        return pb_payload_of(K.pl0, s, K.flags);
    if (LIT && (K.flags & PBK_LITERAL))
    {
        // literal rule, several payloads (sequence.c:545-556, quirk B8): payload p draws
        // rand_r while j < data_len[j], i.e. up to the first j with data_len[j] <= j:
        // j < p this iteration's lengths (first such j kept in `m`), j == p its own
        // draw, j > p the setup values (K.lit_stop, from pbgpu_load_sequence).  Only
        // random payloads draw; the bytes past the payload's length are not sent.
        uint32_t cur = s, m = 0xFFFFu;
        for (uint32_t p = 0; p < i; ++p)
        {
            const pb_pl &Q = K.pls[p];
            const uint32_t len = Q.random ? Q.min_len + pb_mod(pb_rand_r(cur), Q.len) : Q.slen;
            const uint32_t nv = min(min(m, K.lit_stop[p]), len <= p ? p : 0xFFFFu);
            if (Q.random)
                cur = pb_jump(K, cur, nv);
            if (m == 0xFFFFu && len <= p)
                m = p;
        }
        const pb_pl &Q = K.pls[i];
        pb_frame_pl r = pb_payload_of(Q, cur, 0u);
        if (Q.random)
            r.nvalid = min(min(min(m, K.lit_stop[i]), r.plen <= i ? i : 0xFFFFu), r.plen);
        return r;
    }
    // earlier random payloads advance the seed by one rand_r per byte
    uint32_t cur = s;
    for (uint32_t p = 0; p < i; ++p)
    {
        const pb_pl &Q = K.pls[p];
        if (Q.random)
        {
            const uint32_t len = Q.min_len + pb_mod(pb_rand_r(cur), Q.len);
            cur = pb_jump(K, cur, len);
        }
    }
    return pb_payload_of(K.pls[i], cur, K.flags);
}

__device__ __forceinline__ void pb_frame_index(const pb_kargs &K, uint64_t f, uint64_t &k, uint32_t &i)
{
    if (K.pl_cnt == 1)
    {
        k = f;
        i = 0;
    }
    else
    {
        k = f / K.pl_cnt;
        i = (uint32_t)(f - k * K.pl_cnt);
    }
}

template <bool LIT = true>
__device__ __forceinline__ uint32_t pb_frame_len(const pb_kargs &K, uint64_t f)
{
    uint64_t k;
    uint32_t i;
    pb_frame_index(K, f, k, i);
    const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + k);
    return K.hl + pb_payload<LIT>(K, s, i).plen;
}

// keep bytes [lo, hi) of dword t (byte positions 4t .. 4t+3)
__device__ __forceinline__ uint32_t pb_bytemask(int lo, int hi, int t)
{
    const int a = lo - 4 * t;
    const int b = hi - 4 * t;
    const uint32_t ge = a <= 0 ? 0xFFFFFFFFu : (a >= 4 ? 0u : (0xFFFFFFFFu << (8 * a)));
    const uint32_t lt = b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * b)));
    return ge & lt;
}

// 16-B output stores, plain and non-temporal.  Each kernel has one kind, fixed in its code (a
// run-time choice between the two gets merged into one plain store by the compiler).  Measured
// per kernel: non-temporal for the page kernels, pb_small_kernel and
// pb_vline_kernel; plain for pb_fstage_kernel and the staged kernels.
__device__ __forceinline__ void pb_st16(uint8_t *p, pb_u32x4 v)
{
    *reinterpret_cast<pb_u32x4 *>(p) = v;
}
__device__ __forceinline__ void pb_st16_nt(uint8_t *p, pb_u32x4 v)
{
    __builtin_nontemporal_store(v, reinterpret_cast<pb_u32x4 *>(p));
}

// 4 payload bytes from 4 consecutive LCG states: byte = state[23:16]
__device__ __forceinline__ uint32_t pb_pack4(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3)
{
    const uint32_t lo = __builtin_amdgcn_perm(x1, x0, 0x0C0C0602u);
    const uint32_t hi = __builtin_amdgcn_perm(x3, x2, 0x0C0C0602u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// a * x + c on the low 24 bits of x and a, one v_mad_u32_u24 (a in an SGPR, c in a
// VGPR: __umul24 with both constants uniform costs a v_and and a v_mov per use)
__device__ __forceinline__ uint32_t pb_mad24(uint32_t x, uint32_t a, uint32_t c)
{
    uint32_t r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(x), "s"(a), "v"(c));
    return r;
}

// a uniform value held in a VGPR (one v_mov outside the loops that use it)
// the same with a per-lane multiplier (lanes of one wave in groups of different sizes)
__device__ __forceinline__ uint32_t pb_mad24v(uint32_t x, uint32_t a, uint32_t c)
{
    uint32_t r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(a), "v"(c));
    return r;
}

// Opaque one-instruction forms for pb_vline_kernel's chunk addressing: the compiler schedules them
// but cannot strength-reduce them into longer loop-carried chains (it turned `ci - rc0` into three
// instructions per chunk).  a - b:
__device__ __forceinline__ uint32_t pb_subv(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_sub_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// c - 256 a, a < 2^23 (c any 32-bit value; the multiplier in an SGPR: VOP3 takes no literal here)
__device__ __forceinline__ int32_t pb_msub256(uint32_t a, uint32_t c)
{
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(-256), "v"(c));
    return r;
}
// (a << SH) + b
template <int SH>
__device__ __forceinline__ uint32_t pb_lshl_add(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(SH), "v"(b));
    return r;
}

__device__ __forceinline__ uint32_t pb_vgpr(uint32_t s)
{
    uint32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
    return v;
}

// 24-bit LCG step: three rand_r steps folded into one affine map mod 2^24.
__device__ __forceinline__ uint32_t pb_step3(uint32_t x, uint32_t a3, uint32_t c3)
{
    return __umul24(x, a3) + c3;
}

// 4 bytes of a frame-local header image starting at byte x (x may be < 0;
// bytes outside [0, 4 * PB_IMG_STRIDE) read as zero).
__device__ __forceinline__ uint32_t pb_window(const uint32_t *img, int x)
{
    const int i0 = x >> 2; // floor
    const uint32_t sh = (uint32_t)x & 3u;
    const uint32_t lo = (i0 >= 0) ? img[i0] : 0u;
    const uint32_t hi = (i0 + 1 >= 0) ? img[i0 + 1] : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Header image of one frame (sequence.c:150-258 template + sequence.c:443-527
// per-iteration fields + tot_len / udp len + IPv4 checksum, sequence.c:596-602),
// frame bytes 0..63 as little-endian dwords; the L4 checksum field stays 0.
// Returns the L4 length (header + payload).
// The source range of an iteration (sequence.c:455-497): one range is a uniform
// (scalar) load that does not wait for the seed.
// (No table unless the source is random: K.ranges may be null.)
__device__ __forceinline__ uint2 pb_range(const pb_kargs &K, uint32_t r0)
{
    if (!(K.flags & PBK_RND_SADDR))
        return make_uint2(0u, 0u);
    if (K.rng.d == 1)
        return K.ranges[0];
    return K.ranges[pb_mod(r0, K.rng)];
}

// pb_header's IPv4 part alone, for pb_ximg_body (which needs no other word of the header): dwords
// 4-7 of a frame, tot_len, ID, TTL, checksum and source address (sequence.c:443-497, 596-602);
// l4tot = the L4 length.  The checksum also covers dword 3's high half and dword 8's low half,
// which no random field touches (the same arithmetic as pb_header, tested against the oracle
// with every field random, tests/test_gpu_ximg.py).
__device__ __forceinline__ void pb_ip_words(const pb_kargs &K, uint32_t r0, uint32_t l4tot, uint2 rg, uint32_t &d4,
                                            uint32_t &d5, uint32_t &d6, uint32_t &d7)
{
    const uint32_t flags = K.flags;
    d4 = K.tmpl[4];
    d5 = K.tmpl[5];
    d6 = K.tmpl[6];
    d7 = K.tmpl[7];
    if (flags & PBK_RND_TTL) // sequence.c:443-446
        d5 |= ((K.ttl_min + pb_mod(r0, K.ttl)) & 0xFFu) << 16;
    if (flags & PBK_RND_ID) // sequence.c:449-452
        d4 |= pb_bswap16((K.id_min + pb_mod(r0, K.id)) & 0xFFFFu) << 16;
    if (flags & PBK_RND_SADDR) // sequence.c:455-497
    {
        const uint32_t sa = __builtin_bswap32(rg.x | (r0 & rg.y));
        d6 |= sa << 16;
        d7 |= sa >> 16;
    }
    d4 |= pb_bswap16(20u + l4tot); // tot_len, sequence.c:597
    if (flags & PBK_IP_CSUM) // update_iph_checksum, sequence.c:599-602
    {
        const uint32_t sum = (K.tmpl[3] >> 16) + pb_halves(d4) + pb_halves(d5) + (d6 >> 16) + pb_halves(d7) +
                             (K.tmpl[8] & 0xFFFFu);
        const uint32_t c = (flags & PBK_IPH_SINGLE) ? ~((sum & 0xFFFFu) + (sum >> 16)) : ~pb_fold(sum);
        d6 |= c & 0xFFFFu;
    }
}

__device__ __forceinline__ uint32_t pb_header(const pb_kargs &K, uint32_t r0, uint32_t plen, uint32_t (&d)[16],
                                              uint2 rg)
{
    const uint32_t flags = K.flags;
#pragma unroll
    for (int w = 0; w < 16; ++w)
        d[w] = K.tmpl[w];
    if (flags & PBK_RND_TTL) // sequence.c:443-446
        d[5] |= ((K.ttl_min + pb_mod(r0, K.ttl)) & 0xFFu) << 16;
    if (flags & PBK_RND_ID) // sequence.c:449-452
        d[4] |= pb_bswap16((K.id_min + pb_mod(r0, K.id)) & 0xFFFFu) << 16;
    if (flags & PBK_RND_SADDR) // sequence.c:455-497
    {
        const uint32_t sa = __builtin_bswap32(rg.x | (r0 & rg.y));
        d[6] |= sa << 16;
        d[7] |= sa >> 16;
    }
    if (flags & (PBK_RND_SPORT | PBK_RND_DPORT)) // sequence.c:500-527
    {
        const uint32_t port = pb_bswap16(1u + pb_mod(r0, K.port));
        if (flags & PBK_RND_SPORT)
            d[8] |= port << 16;
        if (flags & PBK_RND_DPORT)
            d[9] |= port;
    }
    const uint32_t l4tot = K.l4len + plen;
    d[4] |= pb_bswap16(20u + l4tot); // tot_len, sequence.c:597
    if (K.proto == 17u)
        d[9] |= pb_bswap16(l4tot) << 16; // udph->len, sequence.c:567
    if (flags & PBK_IP_CSUM) // update_iph_checksum, sequence.c:599-602
    {
        const uint32_t sum = (d[3] >> 16) + pb_halves(d[4]) + pb_halves(d[5]) + (d[6] >> 16) + pb_halves(d[7]) +
                             (d[8] & 0xFFFFu);
        const uint32_t c = (flags & PBK_IPH_SINGLE) ? ~((sum & 0xFFFFu) + (sum >> 16)) : ~pb_fold(sum);
        d[6] |= c & 0xFFFFu;
    }
    return l4tot;
}

} // namespace


// One payload byte = three glibc LCG steps: x -> A3 * x + C3 (mod 2^32).
constexpr uint32_t PB_A3 = PB_LCG_A * PB_LCG_A * PB_LCG_A;
constexpr uint32_t PB_C3 = PB_LCG_C * (PB_LCG_A * PB_LCG_A + PB_LCG_A + 1u);


// Workgroup b is dealt to XCD b % 8.  Region r of a launch (a workgroup's contiguous run of
// frames) taken by workgroup b: XCD x builds the x-th contiguous eighth of the regions, in
// order, instead of every eighth region (the rest, fewer than 8, keep their own index).
// Measured on the 1500-B staged kernel: 7.17 vs 8.45 ms per 2^25 frames.
__device__ __forceinline__ uint32_t pb_xcd_region(uint32_t b, uint32_t nwg)
{
    const uint32_t per = nwg >> 3;
    if (b >= 8u * per)
        return b;
    return (b & 7u) * per + (b >> 3);
}

// The reference's total_pckts / total_bytes (sequence.c:633-642), counted as work is done: each
// workgroup records the frames it built and the bytes it stored, so a skipped store or a short
// build shows in pbgpu_counters.  The record is a plain store into this launch's slot array
// (K.ctr_slots, one u32 of bytes per workgroup for fixed-length sequences, whose frames the host
// takes as bytes / length; {frames, bytes} otherwise), at the workgroup's XCD-contiguous position
// so each XCD's records fill whole lines; pb_ctr_fold adds a run of launches' records into the
// counters.  A device-scope atomic per workgroup instead executes at the memory side as its own
// 64-B request: 0.4% of a 64-B launch's HBM traffic (profiles/pmc_r03.json).  Without a slot array
// (K.ctr_slots null) the workgroup adds to shard b % PB_CTR_SHARDS (one 128-B line per shard).
// (pos: the record's index in the launch's slot array; pb_batch_kernel passes the part's own)
__device__ __forceinline__ void pb_count_at(const pb_kargs &K, uint32_t b, uint32_t pos, uint64_t frames,
                                            uint64_t bytes)
{
    if (K.ctr_slots)
    {
        if (K.fixed_len)
            K.ctr_slots[pos] = (uint32_t)bytes;
        else
            reinterpret_cast<uint2 *>(K.ctr_slots)[pos] = make_uint2((uint32_t)frames, (uint32_t)bytes);
        return;
    }
    unsigned long long *c = K.counters + (uint64_t)(b % PB_CTR_SHARDS) * PB_CTR_STRIDE;
    if (!K.fixed_len)
        atomicAdd(c, (unsigned long long)frames);
    atomicAdd(c + 1, (unsigned long long)bytes);
}
__device__ __forceinline__ void pb_count(const pb_kargs &K, uint32_t b, uint64_t frames, uint64_t bytes)
{
    pb_count_at(K, b, pb_xcd_region(blockIdx.x, gridDim.x), frames, bytes);
}

// Folds n workgroup records (pb_count's slot array; pairs = 2: {frames, bytes}, 1: bytes only)
// into a sequence's counters: a grid-stride sum, one atomic pair per workgroup.
__global__ __launch_bounds__(256) void pb_ctr_fold(const uint32_t *slots, uint64_t n, uint32_t pairs,
                                                   unsigned long long *counters)
{
    uint64_t fr = 0, by = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    {
        if (pairs == 2)
        {
            const uint2 v = reinterpret_cast<const uint2 *>(slots)[i];
            fr += v.x;
            by += v.y;
        }
        else
            by += slots[i];
    }
#pragma unroll
    for (uint32_t dd = 32; dd > 0; dd >>= 1)
    {
        fr += __shfl_xor(fr, dd, 64);
        by += __shfl_xor(by, dd, 64);
    }
    __shared__ unsigned long long s_sum[2][4];
    if ((threadIdx.x & 63u) == 0)
    {
        s_sum[0][threadIdx.x >> 6] = fr;
        s_sum[1][threadIdx.x >> 6] = by;
    }
    __syncthreads();
    if (threadIdx.x == 0)
    {
        fr = s_sum[0][0] + s_sum[0][1] + s_sum[0][2] + s_sum[0][3];
        by = s_sum[1][0] + s_sum[1][1] + s_sum[1][2] + s_sum[1][3];
        unsigned long long *c = counters + (uint64_t)(blockIdx.x % PB_CTR_SHARDS) * PB_CTR_STRIDE;
        if (fr)
            atomicAdd(c, fr);
        if (by)
            atomicAdd(c + 1, by);
    }
}

// The counters' shard sums {frames, bytes} of sequences [0, n_seq), written straight into mapped
// pinned host memory (out: its device address, 2 n_seq words): pbgpu_counters' readback without a
// DMA copy (a pageable 24-KiB hipMemcpy of three sequences' shards took 8-16 ms the first time in a
// process, an idle gap right before bench.py's timed steps; profiles/r05/ab/gap.log)
__global__ __launch_bounds__(64) void pb_ctr_read(const unsigned long long *counters, uint32_t n_seq,
                                                  unsigned long long *out)
{
    for (uint32_t w = threadIdx.x; w < 2 * n_seq; w += 64)
    {
        const unsigned long long *c = counters + (size_t)(w >> 1) * PB_CTR_SHARDS * PB_CTR_STRIDE + (w & 1u);
        unsigned long long t = 0;
        for (uint32_t k = 0; k < PB_CTR_SHARDS; ++k)
            t += c[(size_t)k * PB_CTR_STRIDE];
        out[w] = t;
    }
}

extern "C" hipError_t pbk_launch_ctr_read(const unsigned long long *counters, uint32_t n_seq, unsigned long long *out,
                                          hipStream_t st)
{
    hipLaunchKernelGGL(pb_ctr_read, dim3(1), dim3(64), 0, st, counters, n_seq, out);
    return hipGetLastError();
}

extern "C" hipError_t pbk_launch_ctr_fold(const uint32_t *slots, uint64_t n, uint32_t pairs,
                                          unsigned long long *counters, hipStream_t st)
{
    if (n == 0)
        return hipSuccess;
    const uint64_t g = (n + 4095) / 4096 < 1024 ? (n + 4095) / 4096 : 1024;
    hipLaunchKernelGGL(pb_ctr_fold, dim3((uint32_t)g), dim3(256), 0, st, slots, n, pairs, counters);
    return hipGetLastError();
}

// ---------------- small fixed-length frames: one lane per frame ----------------
//
// Frames of <= 4*NDW bytes (configs[1] 64-B UDP, configs[3] 60-B TCP SYN, the
// 98/106-B ICMP/UDP frames): each lane builds its whole frame in NDW VGPRs
// (header, payload, both checksums — sequence.c:433-602 for one iteration),
// writes it into an LDS tile at its packed byte offset, and the workgroup then
// streams the tile (256 frames, always a multiple of 16 B) to HBM with
// contiguous 16-B stores.  PROTO (17/6/1) fixes the header length and the
// checksum position at compile time; RANDOM selects the payload source.  The
// frame body is straight-line code (no data-dependent control flow on d[]).


// keep bytes [lo, hi) of a dword (byte positions 0..3), branch-free
__device__ __forceinline__ uint32_t pb_range_mask(int lo, int hi)
{
    lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
    hi = hi < 0 ? 0 : (hi > 4 ? 4 : hi);
    const uint32_t ge = (uint32_t)(0xFFFFFFFFull << (8 * lo));
    const uint32_t lt = (uint32_t)((1ull << (8 * hi)) - 1ull);
    return ge & lt;
}

// One whole frame of <= 4*NDW bytes in VGPRs (iteration k = first_iter + fidx,
// sequence.c:433-602): header fields, payload, L4 and IPv4 checksums.
template <int NDW, int PROTO, bool RANDOM>
__device__ __forceinline__ void pb_small_frame(const pb_kargs &K, uint64_t fidx, uint32_t (&d)[NDW])
{
    constexpr int HL = PROTO == 6 ? 54 : 42;
    constexpr int P0 = (HL - 2) / 4;                                 // payload byte 0 = byte 2 of dword P0
    constexpr int CDW = PROTO == 17 ? 10 : (PROTO == 6 ? 12 : 9);   // L4 checksum dword
    constexpr int CSH = PROTO == 6 ? 16 : 0;                         // ... and its half
    const uint32_t flen = K.fixed_len;
    const uint32_t flags = K.flags;
    const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + fidx);
    const uint32_t r0 = pb_rand_r(s);
    const uint32_t plen = flen - HL;
    uint32_t h[16];
    const uint32_t l4tot =
        pb_header(K, r0, plen, h,
                  pb_range(K, r0));
#pragma unroll
    for (int t = 0; t < NDW; ++t)
        d[t] = t < 16 ? h[t] : 0u;

    if (RANDOM)
    {
        // single payload: its draws start from the iteration seed (sequence.c:548-555)
        const uint32_t a3 = PB_A3, c3 = PB_C3;
        const int nv = (int)((flags & PBK_LITERAL) ? min(plen, 1u) : plen);
        uint32_t y0 = pb_step3(s, a3, c3), y1 = pb_step3(y0, a3, c3);
        uint32_t x = y1;
        d[P0] |= __builtin_amdgcn_perm(y1, y0, 0x06020C0Cu) & pb_range_mask(HL - 4 * P0, HL + nv - 4 * P0);
#pragma unroll
        for (int t = P0 + 1; t < NDW; ++t)
        {
            const uint32_t x0 = pb_step3(x, a3, c3), x1 = pb_step3(x0, a3, c3);
            const uint32_t x2 = pb_step3(x1, a3, c3), x3 = pb_step3(x2, a3, c3);
            x = x3;
            d[t] |= pb_pack4(x0, x1, x2, x3) & pb_range_mask(0, HL + nv - 4 * t);
        }
    }
    else
    {
#pragma unroll
        for (int t = P0; t < NDW; ++t)
            d[t] |= K.stail[t - P0];
    }
    // (no bytes past the frame end to clear: the template is zero past the header, the random
    // payload is masked to its length above and the static one is zero past its bytes; clearing
    // them again cost the 106-B UDP frame 8%, profiles/r03/ab/small_*)

    // L4 checksum (csum_tcpudp_magic / icmp_csum, sequence.c:569-594)
    uint32_t sum = d[8] >> 16;
    if (RANDOM)
    {
#pragma unroll
        for (int t = 9; t < NDW; ++t)
            sum = pb_add_halves(sum, d[t]);
    }
    else
    {
        // static payload: the header words, then the payload's precomputed word sum (it starts at
        // byte 2 of dword P0, an even L4 offset)
#pragma unroll
        for (int t = 9; t < P0; ++t)
            sum = pb_add_halves(sum, d[t]);
        sum += (d[P0] & 0xFFFFu) + K.pl0.ssum;
    }
    if (PROTO != 1)
        sum += (d[6] >> 16) + pb_halves(d[7]) + (d[8] & 0xFFFFu) + ((PROTO + l4tot) << 8);
    const uint32_t c = (flags & PBK_L4_CSUM) ? ((~pb_fold(sum)) & 0xFFFFu) : 0u;
    d[CDW] |= c << CSH;
}

// LDS slot swizzle of 8-B / 16-B aligned frame images: 16-B slot sl -> sl ^ ((sl >> 3) & 7),
// so lanes at a 64-B stride hit distinct banks; readers undo it with the same map.
__device__ __forceinline__ uint32_t pb_swz(uint32_t sl)
{
    return sl ^ ((sl >> 3) & 7u);
}

// Frame image d[] -> LDS tile at byte offset B (B has the frame's own alignment
// mod 16): whole 16-B / 8-B / 4-B words where the frame length allows, byte
// writes at the two ends of a frame that starts or ends inside a dword.
// two dwords at a 4-B aligned LDS address: one ds_write2_b32
typedef uint32_t pb_u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));

// SWZ = false: 16-B / 8-B frames go in unswizzled (a reader that takes the tile in order)
// AL: the frame length's alignment class when the kernel knows it (16: flen % 16 == 0, 4: % 4,
// 2: 2 mod 4; 0: any, chosen at run time) - the other paths are not compiled in
template <int NDW, bool SWZ = true, int AL = 0>
__device__ __forceinline__ void pb_small_put(uint32_t *s_tile, const uint32_t (&d)[NDW], uint32_t B, uint32_t flen)
{
    if (AL == 16)
        __builtin_assume((flen & 15u) == 0);
    else if (AL == 4)
        __builtin_assume((flen & 3u) == 0);
    else if (AL == 2)
        __builtin_assume((flen & 3u) == 2u);
    if (SWZ && (flen & 15u) == 0)
    {
        pb_u32x4 *tile16 = reinterpret_cast<pb_u32x4 *>(s_tile);
        const uint32_t slot0 = B >> 4;
#pragma unroll
        for (int t = 0; t < NDW; t += 4)
            if ((uint32_t)(4 * t) < flen)
                tile16[pb_swz(slot0 + (t >> 2))] = pb_u32x4{d[t], d[t + 1], d[t + 2], d[t + 3]};
    }
    else if (SWZ && (flen & 7u) == 0)
    {
        uint2 *tile8 = reinterpret_cast<uint2 *>(s_tile);
        const uint32_t q0 = B >> 3;
#pragma unroll
        for (int t = 0; t < NDW; t += 2)
            if ((uint32_t)(4 * t) < flen)
            {
                const uint32_t q = q0 + (t >> 1);
                tile8[(pb_swz(q >> 1) << 1) | (q & 1u)] = make_uint2(d[t], d[t + 1]);
            }
    }
    else if ((flen & 3u) == 0)
    {
        const uint32_t w0 = B >> 2;
#pragma unroll
        for (int t = 0; t < NDW; ++t)
            if ((uint32_t)(4 * t) < flen)
                s_tile[w0 + t] = d[t];
    }
    else if ((flen & 3u) == 2u)
    {
        // 2 mod 4 (98-B ICMP, 106-B UDP): frames start on even bytes, so a frame is one 16-bit
        // half dword at one end and nw = (flen - 2) / 4 whole dwords, written two per
        // ds_write2_b32 (4-B alignment is all a pair needs) instead of dword + byte writes
        const uint32_t nw = (flen - 2u) >> 2;
        const uint32_t sh = B & 2u; // 2: starts at byte 2 of a dword, the half dword comes first
        uint16_t *const half = reinterpret_cast<uint16_t *>(s_tile) + ((sh ? B : B + flen - 2u) >> 1);
        uint32_t *const row = s_tile + ((B + sh) >> 2);
        uint32_t last = 0; // d[nw], picked at the pair whose range holds nw (uniform): d[nw] with
                           // nw known only at run time compiled to a compare + select per dword
#pragma unroll
        for (int u = 0; u < NDW; u += 2)
        {
            if ((uint32_t)u == nw)
                last = d[u];
            else if ((uint32_t)u + 1u == nw && u + 1 < NDW)
                last = d[u + 1];
            if ((uint32_t)u < nw)
            {
                // v_alignbyte by sh bytes: the frame's dwords as they are (sh = 0) or moved down two
                // bytes (no select per dword)
                const uint32_t v0 = __builtin_amdgcn_alignbyte(d[u + 1], d[u], sh);
                if ((uint32_t)u + 1u < nw)
                {
                    const uint32_t v1 = __builtin_amdgcn_alignbyte(u + 2 < NDW ? d[u + 2] : 0u, d[u + 1], sh);
                    *reinterpret_cast<pb_u32x2a4 *>(row + u) = pb_u32x2a4{v0, v1};
                }
                else
                    row[u] = v0;
            }
        }
        *half = (uint16_t)(sh ? d[0] : (last & 0xFFFFu));
    }
    else
    {
        // frame starts at byte phase sh of a dword: out dword u = frame bytes [4u - sh, 4u - sh + 4)
        const uint32_t sh = B & 3u;
        uint32_t *row = s_tile + (B >> 2);
        uint8_t *rowb = reinterpret_cast<uint8_t *>(row);
        const uint32_t end = sh + flen; // row bytes this frame owns: [sh, end)
#pragma unroll
        for (int u = 0; u <= NDW; ++u)
        {
            if ((uint32_t)(4 * u) < end)
            {
                const uint32_t lo = u > 0 ? d[u - 1] : 0u;
                const uint32_t hi = u < NDW ? d[u] : 0u;
                const uint32_t v = sh ? __builtin_amdgcn_alignbyte(hi, lo, 4u - sh) : hi;
                const uint32_t b0 = u == 0 ? sh : 0u;
                const uint32_t b1 = end - 4 * u < 4 ? end - 4 * u : 4u;
                if (b0 == 0 && b1 == 4)
                    row[u] = v;
                else
                    for (uint32_t b = b0; b < b1; ++b)
                        rowb[4 * u + b] = (uint8_t)(v >> (8 * b));
            }
        }
    }
}

// Linear form: workgroup b builds frames [WGT b, WGT b + WGT) and writes their
// contiguous byte range (WGT = 256, or 128 / 64: smaller regions per workgroup).  Used when the output is not 4 KiB aligned (and under
// PBGPU_KERNEL=linear for comparison).
template <int NDW, int PROTO, bool RANDOM, int WGT, int AL = 0> // AL: pb_small_put's alignment class
__global__ __launch_bounds__(WGT) void pb_small_kernel(pb_kargs K)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t s_tile[]; // pb_small_tile_bytes(WGT, flen)
    const uint32_t tid = threadIdx.x;
    const uint64_t f0 = (uint64_t)pb_xcd_region(blockIdx.x, gridDim.x) * WGT; // XCD-contiguous regions
    const uint64_t left = K.n_frames - f0;
    const uint32_t nfr = left < WGT ? (uint32_t)left : WGT;
    const uint32_t flen = K.fixed_len;

    if (tid < nfr)
    {
        uint32_t d[NDW];
        pb_small_frame<NDW, PROTO, RANDOM>(K, f0 + tid, d);
        pb_small_put<NDW, true, AL>(s_tile, d, tid * flen, flen);
    }
    __syncthreads();

    // tile -> HBM: contiguous 16-B stores (every full tile is a multiple of 16 B)
    const uint32_t tile_bytes = nfr * flen;
    const uint32_t nchunks = (tile_bytes + 15) >> 4;
    uint8_t *const out = K.out + f0 * flen;
    const bool swz = (flen & 7u) == 0;
    for (uint32_t c = tid; c < nchunks; c += WGT)
    {
        pb_u32x4 v = reinterpret_cast<const pb_u32x4 *>(s_tile)[swz ? pb_swz(c) : c];
        if (16 * c + 16 > tile_bytes) // last chunk of the stream: zero the tail
        {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                v[t] &= pb_range_mask(0, (int)tile_bytes - (int)(16 * c + 4 * t));
        }
        pb_st16_nt(out + 16 * c, v);
    }
    if (tid == 0)
        pb_count(K, blockIdx.x, nfr, tile_bytes);
}

// XCD-owned pages, one wave per page, for frame lengths that divide 4096 (64-B configs[1]
// frames, 128-B frames).  The output stream (4 KiB aligned) is cut into 4 KiB pages of
// fp = 4096 / flen whole frames.  Workgroup b, which the dispatcher deals to XCD b % 8, owns
// NW * PPW pages, PPW = flen / 64 per wave (64 frames per wave, one per lane): wave w's page h is
// c = (((b / 8) NW + w) PPW + h) 8 + b % 8, so every XCD writes only the pages of one residue
// class mod 8, all eight inside one moving window.  A wave builds its frames into its own LDS
// page, then stores the page as four 1-KiB store instructions: no workgroup barrier, each wave
// starts storing as soon as its own frames are built.  Measured (profiles/r05/ab/xs*.jsonl,
// 2^25 64-B frames, the same buffers): 0.3177 ms at 512 threads, 0.3223 at 256, vs 0.3325 for the
// round-4 form (all four waves build, one barrier, every wave stores 1 KiB of each page); the
// stores alone in the round-4 form took 0.3359 ms and the arithmetic alone 0.190, so the store
// shape, not the arithmetic, set its time.  With the workgroups per CU capped by dynamic LDS
// (K.lds_pad, pbgpu_load_sequence) the wave-local form runs at 0.297-0.303 ms on every buffer
// (3 per CU), faster than the 4-KiB-per-workgroup plain fill beside it (0.309-0.312).

// workgroup b of nwg (b: the launch's blockIdx.x, or the part's own in pb_batch_kernel); s_tile:
// NW * PPW pages of 4 KiB
template <int NDW, int PROTO, bool RANDOM, int WGT>
__device__ __forceinline__ void pb_xsmall_body(const pb_kargs &K, uint32_t b, uint32_t nwg, uint32_t *s_tile)
{
    constexpr uint32_t NW = WGT / 64, PPW = NDW / 16; // waves; pages per wave (64 / 128-B frames)
    constexpr uint32_t FPP = 64 / PPW;                // frames per page
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t flen = K.fixed_len;
    const uint64_t T = K.total_bytes;
    const uint32_t m0 = ((b >> 3) * NW + w) * PPW; // the wave's first page's index within its XCD's class
    uint32_t *const tile = s_tile + w * PPW * (PB_XPG / 4);
    {
        const uint32_t h = lane / FPP, j = lane % FPP;
        const uint32_t c = (m0 + h) * 8 + (b & 7u);
        const uint64_t f = (uint64_t)c * FPP + j;
        if (c < K.xs_nch && f < K.n_frames)
        {
            uint32_t d[NDW];
            pb_small_frame<NDW, PROTO, RANDOM>(K, f, d);
            pb_small_put<NDW, true, 16>(tile, d, lane * flen, flen);
        }
    }
    // the wave's LDS writes before its reads (a wave's LDS operations complete in order)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (the stream's length is a multiple of 64 B: no partial chunk to mask)
#pragma unroll
    for (uint32_t u = 0; u < 4 * PPW; ++u)
    {
        const uint32_t h = u >> 2, ch = (u & 3u) * 64 + lane; // chunk ch of the wave's page h
        const uint32_t c = (m0 + h) * 8 + (b & 7u);
        const uint64_t o = (uint64_t)c * PB_XPG + 16 * ch;
        if (o < T)
            pb_st16_nt(K.out + o, reinterpret_cast<const pb_u32x4 *>(tile)[pb_swz(h * 256 + ch)]);
    }
    if (threadIdx.x == 0)
    {
        // the workgroup's stored pages: whole frames (flen divides every page)
        uint64_t by = 0;
        for (uint32_t i = 0; i < NW * PPW; ++i)
        {
            const uint32_t c = ((b >> 3) * NW * PPW + i) * 8 + (b & 7u);
            if (c < K.xs_nch)
                by += min((uint64_t)PB_XPG, T - (uint64_t)c * PB_XPG);
        }
        pb_count_at(K, b, pb_xcd_region(b, nwg), 0, by); // fixed length: frames = bytes / length on the host
    }
}

template <int NDW, int PROTO, bool RANDOM, int WGT = PB_WG>
__global__ __launch_bounds__(WGT) void pb_xsmall_kernel(pb_kargs K)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[(WGT / 64) * (NDW / 16) * (PB_XPG / 4)];
    pb_xsmall_body<NDW, PROTO, RANDOM, WGT>(K, blockIdx.x, gridDim.x, s_tile);
}

// The workgroup-wide 64-B page body, kept for pb_batch_kernel's 64-B part: all WGT lanes build,
// one barrier, then each wave stores one page (the fused launch ran the round-4 form of this body
// 1% faster than the wave-local body, 0.5335 vs 0.5386 ms per configs[4] step,
// profiles/r05/ab/mix*.jsonl: that launch runs at the xpage parts' occupancy).  Workgroup b owns pages ((b / 8) np + i) 8 + b % 8, i < np =
// WGT / 64 (the rest, fewer than 8 np, take the tail pages in order from xs_full).
template <int WGT>
__device__ __forceinline__ void pb_xsmall_wg_body(const pb_kargs &K, uint32_t b, uint32_t nwg, uint32_t *s_tile)
{
    constexpr uint32_t NPG = WGT / 64;
    const uint32_t tid = threadIdx.x;
    const uint32_t np = K.xs_np;
    const uint64_t T = K.total_bytes;
    uint32_t c0, cs;
    if (b < K.xs_full)
        c0 = (b >> 3) * (np * 8) + (b & 7u), cs = 8;
    else
        c0 = K.xs_full * np + (b - K.xs_full) * np, cs = 1;
    {
        const uint32_t i = tid >> 6, j = tid & 63u;
        const uint64_t f = ((uint64_t)(c0 + i * cs) << 6) + j;
        if (f < K.n_frames)
        {
            uint32_t d[16];
            pb_small_frame<16, 17, true>(K, f, d);
            pb_small_put<16, true, 16>(s_tile, d, i * PB_XREG + 128 + j * 64, 64);
        }
    }
    __syncthreads();
    // page i -> HBM: wave i stores page i whole, four 1-KiB store instructions (0.530 vs 0.538 ms
    // per configs[4] step for 1 KiB of every page per wave, profiles/r05/ab/mixws.jsonl)
    const uint32_t i = tid >> 6, lane = tid & 63u;
    static_assert(NPG == WGT / 64, "one page per wave");
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u)
    {
        const uint32_t ch = u * 64 + lane;
        const uint32_t c = c0 + i * cs;
        const uint64_t o = (uint64_t)c * PB_XPG + 16 * ch;
        if (i < np && c < K.xs_nch && o < T)
        {
            pb_u32x4 v = reinterpret_cast<const pb_u32x4 *>(s_tile)[pb_swz((i * PB_XREG + 128) / 16 + ch)];
            if (o + 16 > T)
            {
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    v[t] &= pb_range_mask(0, (int)(T - o) - 4 * t);
            }
            pb_st16_nt(K.out + o, v);
        }
    }
    if (tid == 0)
    {
        uint64_t by = 0;
        for (uint32_t i = 0; i < np; ++i)
        {
            const uint32_t c = c0 + i * cs;
            if (c < K.xs_nch)
                by += min((uint64_t)PB_XPG, T - (uint64_t)c * PB_XPG);
        }
        pb_count_at(K, b, pb_xcd_region(b, nwg), 0, by);
    }
}

// XCD-owned pages for frame lengths that are a multiple of 4 but do not divide
// 4096 (60-B TCP SYN, configs[3]): pb_xsmall_kernel's page ownership, with the
// frames that straddle a page edge built by both owners.  Slot j of page i is
// frame floor(4096 c_i / flen) + j (found per lane with a double reciprocal and a
// +-1 fix-up: no prologue, no barrier before the build); the frame is written
// whole into the page's LDS region, whose 128 B of slack either side take the
// bytes outside the page and are never stored.  At 60 B one frame in 69 is built
// twice.
// pb_xpage_kernel: the first frame touching page c0 = floor(4096 c0 / flen) = c0 q + floor(c0 r /
// flen) (q, r = 4096 div / mod flen), exact in 32 bits while c0 r < 2^31 (the host sets
// xp_fa_hi otherwise)
__device__ __forceinline__ uint32_t pb_xp_first_frame(const pb_kargs &K, uint32_t c0, uint32_t flen)
{
    const uint32_t q = pb_divq(PB_XPG, K.flen), r = PB_XPG - q * flen;
    return c0 * q + pb_divq(c0 * r, K.flen);
}
// ... and for any c0: a double reciprocal with a +-1 fix-up
__device__ __forceinline__ uint64_t pb_xp_first_frame64(uint32_t c0, uint32_t flen, double inv)
{
    const uint64_t p0 = (uint64_t)c0 * PB_XPG;
    uint64_t fa = (uint64_t)((double)p0 * inv);
    if (fa * flen > p0)
        --fa;
    else if ((fa + 1) * flen <= p0)
        ++fa;
    return fa;
}

// s_tile: K.xs_np page regions; workgroup b of nwg as in pb_xsmall_body
template <int NDW, int PROTO, bool RANDOM, int WGT, bool A4>
__device__ __forceinline__ void pb_xpage_body(const pb_kargs &K, uint32_t b, uint32_t nwg, uint32_t *s_tile)
{
    const uint32_t tid = threadIdx.x;
    const uint32_t flen = K.fixed_len;
    const uint32_t np = K.xs_np, fpp = K.xp_fpp;
    const uint64_t T = K.total_bytes;
    uint32_t c0, cs;
    if (b < K.xs_full)
        c0 = (b >> 3) * (np * 8) + (b & 7u), cs = 8;
    else
        c0 = K.xs_full * np + (b - K.xs_full) * np, cs = 1;

    // Page c = c0 + i cs starts at byte 4096 c = fa0 flen - rem0 + 4096 cs i: frame fa0 =
    // floor(4096 c0 / flen) and rem0 = 4096 c0 - fa0 flen are uniform (one 64-bit division
    // per workgroup), the rest is 32-bit: t = rem0 + 4096 cs i < 2^18, so page i's first frame
    // is fa0 + t / flen (exact multiply-shift) and slot j starts at byte j flen - t % flen of
    // the page.  (Per lane, a double reciprocal and 64-bit fix-ups cost ~40 VALU per slot.)
    const uint32_t fa_lo = pb_xp_first_frame(K, c0, flen);
    const uint64_t fa0 = K.xp_fa_hi ? pb_xp_first_frame64(c0, flen, K.xp_inv) : (uint64_t)fa_lo;
    const uint32_t rem0 = (uint32_t)((uint64_t)c0 * PB_XPG - fa0 * flen);
    // at most two slots per 256 lanes (np * fpp <= 512): one straight-line pass per
    // 512-thread workgroup, two unrolled passes per 256-thread one (a loop kept the
    // kernel arguments live across iterations and spilled them through v_readlane /
    // v_writelane, 41 VALU per frame)
#pragma unroll
    for (uint32_t pass = 0; pass < 512 / WGT; ++pass)
    {
        const uint32_t sl = tid + pass * WGT;
        if (sl >= np * fpp)
            break;
        const uint32_t i = pb_divq(sl, K.xp_div), j = sl - __umul24(i, fpp);
        const uint32_t c = c0 + i * cs;
        if (c >= K.xs_nch)
            continue;
        const uint32_t t = rem0 + ((i * cs) << 12);
        const uint32_t qi = pb_divq(t, K.flen);
        const int off = (int)__umul24(j, flen) - (int)(t - __umul24(qi, flen)); // (-flen, 4096 + flen)
        const uint64_t f = fa0 + qi + j;
        if (off >= (int)PB_XPG || f >= K.n_frames)
            continue;
        uint32_t d[NDW];
        pb_small_frame<NDW, PROTO, RANDOM>(K, f, d);
        if (A4)
        {
            // 4-B aligned: dword pairs (ds_write2_b32 / ds_write_b64), a last single dword
            uint32_t *row = s_tile + (i * PB_XREG + 128 + off) / 4;
#pragma unroll
            for (int t2 = 0; t2 < NDW; t2 += 2)
            {
                if ((uint32_t)(4 * t2 + 4) < flen)
                    *reinterpret_cast<pb_u32x2a4 *>(row + t2) = pb_u32x2a4{d[t2], d[t2 + 1]};
                else if ((uint32_t)(4 * t2) < flen)
                    row[t2] = d[t2];
            }
        }
        else // 2 mod 4 (98-B ICMP, 106-B UDP under PBGPU_XP_FORCE): a half dword at one end
            pb_small_put<NDW, false, 2>(s_tile, d, i * PB_XREG + 128 + off, flen);
    }
    __syncthreads();

    // page i -> HBM: wave w stores pages w, w + WGT / 64, ... whole, four 1-KiB store
    // instructions each (vs 1 KiB of every other page per wave: 60-B TCP SYN 0.280-0.282 vs
    // 0.288-0.295 ms, 98-B ICMP 0.457-0.462 vs 0.462-0.466, profiles/r05/ab/xpw3.jsonl)
    const uint32_t lane = tid & 63u;
    for (uint32_t i = tid >> 6; i < np; i += WGT / 64)
    {
        const uint32_t c = c0 + i * cs;
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
        {
            const uint32_t l = u * 64 + lane;
            const uint64_t o = (uint64_t)c * PB_XPG + 16 * l;
            if (c < K.xs_nch && o < T)
            {
                pb_u32x4 v = reinterpret_cast<const pb_u32x4 *>(s_tile)[(i * PB_XREG + 128) / 16 + l];
                if (o + 16 > T) // last chunk of the stream: zero the tail
                {
#pragma unroll
                    for (int t = 0; t < 4; ++t)
                        v[t] &= pb_range_mask(0, (int)(T - o) - 4 * t);
                }
                pb_st16_nt(K.out + o, v);
            }
        }
    }
    if (tid == 0)
    {
        // the bytes of the stored pages (fixed length: the host takes frames = bytes / length,
        // pb_count; counting each page's frame starts cost 4%, profiles/r04/ab)
        uint64_t by = 0;
        for (uint32_t i = 0; i < np; ++i)
        {
            const uint32_t c = c0 + i * cs;
            if (c < K.xs_nch)
                by += min((uint64_t)PB_XPG, T - (uint64_t)c * PB_XPG);
        }
        pb_count_at(K, b, pb_xcd_region(b, nwg), 0, by);
    }
}

// (an SGPR budget of 80, as pb_batch_kernel: 8 waves per SIMD instead of 6-7; 60-B TCP SYN
// 0.282-0.291 vs 0.302-0.308 ms, 98-B ICMP 0.457-0.471 vs 0.478-0.488 on four buffers,
// profiles/r05/ab/xp.jsonl)
template <int NDW, int PROTO, bool RANDOM, int WGT, bool A4 = true> // A4: flen % 4 == 0 (else 2 mod 4)
__global__ __launch_bounds__(WGT) __attribute__((amdgpu_num_sgpr(80))) void pb_xpage_kernel(pb_kargs K)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t s_tile[]; // K.xs_np page regions
    pb_xpage_body<NDW, PROTO, RANDOM, WGT, A4>(K, blockIdx.x, gridDim.x, s_tile);
}

// ---------------- static-payload ICMP frames: pb_ximg_kernel ----------------
//
// An ICMP echo frame with a static payload (configs[4]'s 98-B frame) varies in four header fields
// only: IPv4 ID, TTL, checksum and source address, frame bytes [18, 30) (no pseudo header: the
// ICMP checksum is a per-sequence constant).  The stream's bytes outside those windows repeat every
// img_np = flen / gcd(flen, 4096) pages (49 at 98 B), so pbgpu_load_sequence builds the first
// img_np pages once (pb_xpage_kernel into K.img).  Wave w of workgroup b owns page c =
// ((b / 8) NW + w) 8 + b % 8 (pb_xsmall_kernel's XCD ownership): it copies page c mod img_np
// (L2-resident) into its LDS page, lane j computes frame fa + j's header fields (the first frame
// touching the page, as pb_xpage_kernel) and writes its five 16-bit halves of [18, 30) that fall in
// the page, and the wave stores the page as four 1-KiB instructions after a wave barrier.  Per
// frame: the seed, rand_r and the header fields; no payload, no L4 sum, no 2-mod-4 tile write
// (pb_xpage_kernel: 282 VALU lane-ops per 98-B frame and 49% LDS bank conflicts in its tile
// writes, profiles/r05/prof/pmc_table.json).
template <int WGT>
__device__ __forceinline__ void pb_ximg_body(const pb_kargs &K, uint32_t b, uint32_t nwg, uint32_t *s_tile)
{
    constexpr uint32_t NW = WGT / 64;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const uint32_t flen = K.fixed_len;
    const uint64_t T = K.total_bytes;
    const uint32_t c = ((b >> 3) * NW + w) * 8 + (b & 7u);
    pb_u32x4 *const tile = reinterpret_cast<pb_u32x4 *>(s_tile + w * (PB_XPG / 4));
    if (c < K.xs_nch)
    {
        const uint32_t q = c - pb_divq(c, K.img_div) * K.img_np;
        const pb_u32x4 *const src = reinterpret_cast<const pb_u32x4 *>(K.img) + (size_t)q * (PB_XPG / 16);
        pb_u32x4 v[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
            v[u] = src[u * 64 + lane];
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u)
            tile[u * 64 + lane] = v[u];
        // the copy before the patches (a wave's LDS operations complete in order)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t fa = K.xp_fa_hi ? pb_xp_first_frame64(c, flen, K.xp_inv) : (uint64_t)pb_xp_first_frame(K, c, flen);
        const uint32_t rem = (uint32_t)((uint64_t)c * PB_XPG - fa * flen); // < flen
        // slots j = lane, lane + 64 (lengths under 66 B touch more than 64 frames per page)
#pragma unroll
        for (uint32_t p = 0; p < 2; ++p)
        {
            if (p && K.xp_fpp <= 64)
                break;
            const uint32_t j = lane + 64 * p;
            const int off = (int)__umul24(j, flen) - (int)rem; // frame start in the page
            const uint64_t f = fa + j;
            if (j >= K.xp_fpp || off >= (int)PB_XPG || f >= K.n_frames)
                continue;
            const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + f);
            const uint32_t r0 = pb_rand_r(s);
            uint32_t d4, d5, d6, d7;
            pb_ip_words(K, r0, K.l4len + flen - K.hl, pb_range(K, r0), d4, d5, d6, d7);
            // bytes 18-19 ID, 22-23 TTL + protocol, 24-25 checksum, 26-29 source (frames start on
            // even bytes: whole 16-bit halves)
            const uint32_t hv[5] = {d4 >> 16, d5 >> 16, d6 & 0xFFFFu, d6 >> 16, d7 & 0xFFFFu};
            constexpr int HB[5] = {18, 22, 24, 26, 28};
            uint16_t *const t16 = reinterpret_cast<uint16_t *>(tile);
#pragma unroll
            for (int i = 0; i < 5; ++i)
            {
                const int pos = off + HB[i];
                if ((uint32_t)pos < PB_XPG)
                    t16[pos >> 1] = (uint16_t)hv[i];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint8_t *const out = K.out + (uint64_t)c * PB_XPG;
        if ((uint64_t)(c + 1) * PB_XPG <= T) // (uniform) a whole page: no tail masks
        {
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u)
                pb_st16_nt(out + 16 * (u * 64 + lane), tile[u * 64 + lane]);
        }
        else
        {
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u)
            {
                const uint32_t l = u * 64 + lane;
                const uint64_t o = (uint64_t)c * PB_XPG + 16 * l;
                if (o < T)
                {
                    pb_u32x4 x = tile[l];
                    if (o + 16 > T) // last chunk of the stream: zero the tail
                    {
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            x[t] &= pb_range_mask(0, (int)(T - o) - 4 * t);
                    }
                    pb_st16_nt(out + 16 * l, x);
                }
            }
        }
    }
    if (threadIdx.x == 0)
    {
        // the workgroup's pages ascend with i: all whole unless the last one reaches the stream end
        const uint32_t cl = ((b >> 3) * NW + NW - 1) * 8 + (b & 7u);
        uint64_t by = (uint64_t)NW * PB_XPG;
        if ((uint64_t)(cl + 1) * PB_XPG > T)
        {
            by = 0;
            for (uint32_t i = 0; i < NW; ++i)
            {
                const uint32_t ci = ((b >> 3) * NW + i) * 8 + (b & 7u);
                if (ci < K.xs_nch)
                    by += min((uint64_t)PB_XPG, T - (uint64_t)ci * PB_XPG);
            }
        }
        pb_count_at(K, b, pb_xcd_region(b, nwg), 0, by);
    }
}

template <int WGT>
__global__ __launch_bounds__(WGT) __attribute__((amdgpu_num_sgpr(80))) void pb_ximg_kernel(pb_kargs K)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[(WGT / 64) * (PB_XPG / 4)];
    pb_ximg_body<WGT>(K, blockIdx.x, gridDim.x, s_tile);
}

// ---------------- several sequences in one launch: pb_batch_kernel ----------------
//
// configs[4] builds three sequences per step (64-B UDP, 60-B TCP SYN, 98-B ICMP), each a launch
// of 2^24 frames of its own page kernel.  Launched back to back or on three streams, every launch
// pays its own ramp and drain (the mix ran 0.57-0.61 ms per step against 0.55 ms for the three
// kernels' own times).  Here the three are parts of one grid: part j takes workgroups [o_j, o_j +
// g_j) (o_j a multiple of 8, so a part's workgroup b stays on XCD b % 8 and keeps its page
// ownership) and runs its kernel's body on its own kargs; the dispatcher starts part j + 1's
// workgroups while part j's last ones finish.  One block size (WGT) for all parts: the 64-B part
// runs pb_xsmall_body with WGT / 64 pages per workgroup.  Kinds (pbk_batch_kind): 1 the 64-B
// random-payload UDP page kernel, 2 the 60-B random-payload TCP one, 3 the 98-B static-payload ICMP.
struct pb_batch_args
{
    pb_kargs K[3];
    uint32_t g[3]; // the parts' workgroups
};

template <int KIND, int WGT>
__device__ __forceinline__ void pb_batch_part(const pb_kargs &K, uint32_t b, uint32_t nwg, uint32_t *s_tile)
{
    if (b >= nwg) // the padding before the next part's first workgroup
        return;
    if constexpr (KIND == 1)
        pb_xsmall_wg_body<WGT>(K, b, nwg, s_tile);
    else if constexpr (KIND == 2)
        pb_xpage_body<16, 6, true, WGT, true>(K, b, nwg, s_tile);
    else if (K.img)
        pb_ximg_body<WGT>(K, b, nwg, s_tile);
    else
        pb_xpage_body<32, 1, false, WGT, false>(K, b, nwg, s_tile);
}

// (an SGPR budget of 80: the compiler's 106 admit 6 waves per SIMD, 3 workgroups of 512 threads
// per CU, 80 admit 8: 0.5335 vs 0.5484 ms per configs[4] step, profiles/r05/ab/mix*.jsonl)
template <int WGT, int KA, int KB, int KC>
__global__ __launch_bounds__(WGT) __attribute__((amdgpu_num_sgpr(80))) void pb_batch_kernel(pb_batch_args A)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t s_tile[];
    const uint32_t b = blockIdx.x;
    const uint32_t o1 = (A.g[0] + 7u) & ~7u, o2 = o1 + ((A.g[1] + 7u) & ~7u);
    if (b < o1)
        pb_batch_part<KA, WGT>(A.K[0], b, A.g[0], s_tile);
    else if (b < o2)
        pb_batch_part<KB, WGT>(A.K[1], b - o1, A.g[1], s_tile);
    else
        pb_batch_part<KC, WGT>(A.K[2], b - o2, A.g[2], s_tile);
}

// ---------------- group per frame: any length, fixed or packed variable ----------------
//
// Workgroup = 256 frames.  Phase A: one lane per frame computes the seed,
// fields, header image + IPv4 checksum (sequence.c:433-527, 596-602) into LDS.
// Phase B: a group of G lanes streams one frame at a time: lane l of the group
// produces the frame's output-aligned 16-B chunks l, l+G, ... (payload bytes
// from the glibc LCG, sequence.c:552-555, jumped to the chunk start with
// per-lane constants L^(48 l) and advanced by L^(48 G) per step), stores every
// chunk that holds no header byte straight away, sums the payload words for
// the L4 checksum (sequence.c:569-594), reduces that sum across the group with
// lane shuffles, and finally stores the header chunks with the finished
// checksum.  Chunks shared with a neighbouring frame are written byte/dword-
// masked, so every byte of the packed stream is written exactly once.

// Sum over aligned groups of G lanes (G = 8, 16, 32, 64), result in every lane
// of the group: in-row steps by DPP (no LDS round trip), the rest by swizzle /
// shuffle.
template <int G>
__device__ __forceinline__ uint32_t pb_group_sum(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false); // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false); // quad_perm [2,3,0,1]
    if (G == 8)
        v += (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x101F); // xor 4
    if (G >= 16)
    {
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false); // row_ror:4
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false); // row_ror:8
    }
    if (G >= 32)
        v += __shfl_xor(v, 16, 64);
    if (G >= 64)
        v += __shfl_xor(v, 32, 64);
    return v;
}

// store bytes [max(0,-q0), min(16, flen-q0)) of a 16-B chunk at p (16-B aligned)
__device__ __forceinline__ void pb_store_chunk(uint8_t *p, uint32_t o0, uint32_t o1, uint32_t o2, uint32_t o3, int q0,
                                               int flen)
{
    const int a = -q0, b = flen - q0;
    if (a <= 0 && b >= 16)
    {
        pb_st16(p, pb_u32x4{o0, o1, o2, o3});
        return;
    }
    const uint32_t o[4] = {o0, o1, o2, o3};
#pragma unroll
    for (int t = 0; t < 4; ++t)
    {
        const int lo = max(a - 4 * t, 0), hi = min(b - 4 * t, 4);
        if (lo == 0 && hi == 4)
            *reinterpret_cast<uint32_t *>(p + 4 * t) = o[t];
        else
            for (int i = lo; i < hi; ++i)
                p[4 * t + i] = (uint8_t)(o[t] >> (8 * i));
    }
}

// 16 payload bytes starting at payload index j0 of a frame (random: from LCG
// state x for j0; static: blob bytes at src + j0), bytes outside [lo, hi) zeroed
__device__ __forceinline__ void pb_chunk_payload(const pb_kargs &K, bool rnd, uint32_t x, uint32_t src, int j0, int lo,
                                                 int hi, uint32_t &o0, uint32_t &o1, uint32_t &o2, uint32_t &o3)
{
    const uint32_t a3 = PB_A3, c3 = PB_C3;
    if (rnd)
    {
        uint32_t x0 = x, x1 = pb_step3(x0, a3, c3), x2 = pb_step3(x1, a3, c3), x3 = pb_step3(x2, a3, c3);
        o0 = pb_pack4(x0, x1, x2, x3);
        x0 = pb_step3(x3, a3, c3), x1 = pb_step3(x0, a3, c3), x2 = pb_step3(x1, a3, c3), x3 = pb_step3(x2, a3, c3);
        o1 = pb_pack4(x0, x1, x2, x3);
        x0 = pb_step3(x3, a3, c3), x1 = pb_step3(x0, a3, c3), x2 = pb_step3(x1, a3, c3), x3 = pb_step3(x2, a3, c3);
        o2 = pb_pack4(x0, x1, x2, x3);
        x0 = pb_step3(x3, a3, c3), x1 = pb_step3(x0, a3, c3), x2 = pb_step3(x1, a3, c3), x3 = pb_step3(x2, a3, c3);
        o3 = pb_pack4(x0, x1, x2, x3);
    }
    else
    {
        const uint8_t *bp = K.blob + src + j0;
        const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)bp & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)((uintptr_t)bp & 3);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
        o0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
        o1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
        o2 = __builtin_amdgcn_alignbyte(w3, w2, sh);
        o3 = __builtin_amdgcn_alignbyte(w4, w3, sh);
    }
    if (lo > 0 || hi < 16)
    {
        o0 &= pb_range_mask(lo, hi);
        o1 &= pb_range_mask(lo - 4, hi - 4);
        o2 &= pb_range_mask(lo - 8, hi - 8);
        o3 &= pb_range_mask(lo - 12, hi - 12);
    }
}

// RMODE: 1 every payload random, 0 every payload static, 2 mixed (multi-payload)
template <int G, int RMODE>
__global__ __launch_bounds__(PB_WG) void pb_gpf_kernel(pb_kargs K)
{
    __shared__ __attribute__((aligned(16))) uint32_t s_img[PB_WG * PB_IMG_STRIDE];
    __shared__ uint32_t s_blo[PB_WG], s_bhi[PB_WG], s_flen[PB_WG], s_z[PB_WG], s_st0[PB_WG], s_nv[PB_WG],
        s_src[PB_WG], s_hsum[PB_WG];

    const uint32_t tid = threadIdx.x;
    const uint32_t flags = K.flags;
    const uint32_t fpw = K.gpf_fpw; // frames per workgroup: a multiple of 256 / G, at most 256
    const uint64_t fwg = (uint64_t)blockIdx.x * fpw;
    const uint64_t left = K.n_frames - fwg;
    const uint32_t nfr = left < fpw ? (uint32_t)left : fpw;
    const int hl = (int)K.hl;

    // ---------------- phase A: one lane per frame ----------------
    if (tid < nfr)
    {
        const uint64_t f = fwg + tid;
        uint64_t base;
        uint32_t flen;
        if (K.fixed_len)
        {
            base = f * K.fixed_len;
            flen = K.fixed_len;
        }
        else
        {
            base = K.offsets[f];
            flen = (uint32_t)(K.offsets[f + 1] - base);
        }
        uint64_t k;
        uint32_t pi;
        pb_frame_index(K, f, k, pi);
        const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + k);
        const uint32_t r0 = pb_rand_r(s);
        const pb_frame_pl P = pb_payload(K, s, pi);
        uint32_t d[16];
        const uint32_t l4tot = pb_header(K, r0, P.plen, d, pb_range(K, r0));
        uint32_t hs = (d[8] >> 16) + pb_halves(d[9]) + pb_halves(d[10]) + pb_halves(d[11]) + pb_halves(d[12]) +
                      pb_halves(d[13]);
        if (flags & PBK_PSEUDO)
            hs += (d[6] >> 16) + pb_halves(d[7]) + (d[8] & 0xFFFFu) + ((K.proto + l4tot) << 8);
        if (!P.random)
            hs += P.ssum;
        pb_u32x4 *row = reinterpret_cast<pb_u32x4 *>(s_img + tid * PB_IMG_STRIDE);
        row[0] = pb_u32x4{d[0], d[1], d[2], d[3]};
        row[1] = pb_u32x4{d[4], d[5], d[6], d[7]};
        row[2] = pb_u32x4{d[8], d[9], d[10], d[11]};
        row[3] = pb_u32x4{d[12], d[13], d[14], d[15]};
        row[4] = pb_u32x4{0u, 0u, 0u, 0u};
        // LCG state for payload index j = -(base % 16 + hl), the first chunk's first byte
        const uint2 jt = K.jump[PB_JNEG - ((uint32_t)(base & 15u) + (uint32_t)hl)];
        s_blo[tid] = (uint32_t)base;
        s_bhi[tid] = (uint32_t)(base >> 32);
        s_flen[tid] = flen;
        s_z[tid] = P.random ? jt.x * P.st0 + jt.y : 0u;
        s_st0[tid] = P.st0;
        s_nv[tid] = P.nvalid | (P.random << 31);
        s_src[tid] = P.blob_off;
        s_hsum[tid] = hs;
    }
    __syncthreads();

    // ---------------- phase B: G lanes per frame ----------------
    // Round p gives the workgroup's 256 / G groups frames p * (256 / G) + group, so
    // the four waves write one contiguous front through the workgroup's output.
    constexpr uint32_t NGW = PB_WG / G; // frames in flight per workgroup
    const uint32_t grp = tid / G, lg = tid % G;
    const uint2 Ml = K.lcg48[lg], MG = K.lcg48[G];

    for (uint32_t p = 0; p < fpw / NGW; ++p)
    {
        const uint32_t fr = p * NGW + grp;
        if (fr >= nfr)
            break;
        const uint64_t base = ((uint64_t)s_bhi[fr] << 32) | s_blo[fr];
        const int flen = (int)s_flen[fr];
        const int s0 = (int)(base & 15u);
        const uint32_t nch = (uint32_t)(s0 + flen + 15) >> 4;
        const uint32_t nv = s_nv[fr];
        const bool rnd = RMODE == 2 ? (nv >> 31) != 0 : RMODE == 1;
        const int nvalid = (int)(nv & 0x7FFFFFFFu);
        const uint32_t src = s_src[fr];
        uint8_t *const out = K.out + (base & ~15ull);
        // Frame edges.  The 16-B chunk shared with the previous frame is stored whole
        // by this frame's chunk-0 lane, which also generates the previous frame's
        // payload tail for it (cov_in); symmetrically this frame does not store its
        // last chunk when the next frame covers it (cov_out).  Needs the neighbour in
        // this workgroup and its bytes in that chunk to be payload, not header.
        const int e = (s0 + flen) & 15;
        const bool cov_in = s0 != 0 && fr > 0 && (int)s_flen[fr - 1] - hl >= s0;
        const bool cov_out = e != 0 && fr + 1 < nfr && flen - hl >= e;
        uint32_t x = __umul24(s_z[fr], Ml.x) + Ml.y;
        uint32_t acc = 0;

        // interior chunks (all 16 bytes drawn payload): generate, sum, store.  Edge
        // chunks (header bytes, or the end of the drawn payload) are kept for later.
        int eq0 = 0, eq1 = 0;
        uint32_t ex0 = 0, ex1 = 0;
        uint32_t ne = 0;
        for (uint32_t m = lg; m < nch; m += G)
        {
            const int q0 = (int)(16 * m) - s0; // frame position of the chunk's first byte
            const int j0 = q0 - hl;            // payload index of the chunk's first byte
            if (j0 >= 0 && j0 + 16 <= nvalid)
            {
                uint32_t o0, o1, o2, o3;
                pb_chunk_payload(K, rnd, x, src, j0, 0, 16, o0, o1, o2, o3);
                if (rnd)
                    acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
                pb_st16(out + 16 * m, pb_u32x4{o0, o1, o2, o3});
            }
            else if (j0 >= nvalid && j0 >= 0)
            {
                // past the drawn bytes (literal rule): zeros up to the frame end
                if (!(m + 1 == nch && cov_out))
                    pb_store_chunk(out + 16 * m, 0u, 0u, 0u, 0u, q0, flen);
            }
            else
            {
                if (ne == 0)
                    eq0 = q0, ex0 = x;
                else
                    eq1 = q0, ex1 = x;
                ++ne;
            }
            x = __umul24(x, MG.x) + MG.y;
        }

        // edge chunks: at most two per lane (a head chunk in the first step, a tail chunk)
        uint32_t eo[2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
        {
            eo[i][0] = eo[i][1] = eo[i][2] = eo[i][3] = 0u;
            if ((uint32_t)i < ne)
            {
                const int q0 = i ? eq1 : eq0;
                bool grnd = rnd;
                uint32_t gx = i ? ex1 : ex0, gsrc = src;
                int j0 = q0 - hl, lo = -j0, hi = nvalid - j0;
                const bool special = q0 == -s0 && cov_in; // chunk 0 shared with the previous frame
                if (special)
                {
                    // the previous frame's last payload bytes fill chunk bytes [0, s0)
                    const int pf = (int)s_flen[fr - 1];
                    const uint32_t pnv = s_nv[fr - 1];
                    grnd = RMODE == 2 ? (pnv >> 31) != 0 : RMODE == 1;
                    j0 = pf - s0 - hl;
                    lo = 0;
                    hi = min((int)(pnv & 0x7FFFFFFFu) - j0, s0);
                    gsrc = s_src[fr - 1];
                    const uint2 jt = K.jump[(uint32_t)j0 + PB_JNEG];
                    gx = grnd ? jt.x * s_st0[fr - 1] + jt.y : 0u;
                }
                if (lo < 16 && hi > 0 && lo < hi)
                {
                    pb_chunk_payload(K, grnd, gx, gsrc, j0, lo, hi, eo[i][0], eo[i][1], eo[i][2], eo[i][3]);
                    if (grnd && !special)
                        acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, eo[i][0]), eo[i][1]), eo[i][2]),
                                            eo[i][3]);
                }
            }
        }

        const uint32_t sum = pb_group_sum<G>(acc);
        if ((flags & PBK_L4_CSUM) && lg == 0)
        {
            uint32_t pc = pb_fold(sum);
            if (base & 1u) // chunk sums were taken in output alignment
                pc = pb_bswap16(pc);
            const uint32_t c = (~pb_fold(pb_fold(s_hsum[fr]) + pc)) & 0xFFFFu;
            s_img[fr * PB_IMG_STRIDE + K.csum_dw] |= K.csum_hi ? (c << 16) : c;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int i = 0; i < 2; ++i)
        {
            if ((uint32_t)i < ne)
            {
                const int q0 = i ? eq1 : eq0;
                const uint32_t m = (uint32_t)(q0 + s0) >> 4;
                uint32_t o0 = eo[i][0], o1 = eo[i][1], o2 = eo[i][2], o3 = eo[i][3];
                if (q0 < hl)
                {
                    const uint32_t *img = s_img + fr * PB_IMG_STRIDE;
                    o0 |= pb_window(img, q0);
                    o1 |= pb_window(img, q0 + 4);
                    o2 |= pb_window(img, q0 + 8);
                    o3 |= pb_window(img, q0 + 12);
                }
                const bool special = q0 == -s0 && cov_in; // holds the previous frame's tail too: store whole
                if (!(m + 1 == nch && cov_out))
                    pb_store_chunk(out + 16 * m, o0, o1, o2, o3, special ? 0 : q0, special ? 16 : flen);
            }
        }
    }
    if (tid == 0 && nfr)
    {
        // every byte of the workgroup's frames is stored by exactly one of its lanes
        const uint64_t b0 = ((uint64_t)s_bhi[0] << 32) | s_blo[0];
        const uint64_t b1 = (((uint64_t)s_bhi[nfr - 1] << 32) | s_blo[nfr - 1]) + s_flen[nfr - 1];
        pb_count(K, blockIdx.x, nfr, b1 - b0);
    }
}

// ---------------- staged: frames assembled in LDS, streamed out whole ----------------
//
// Workgroup = K.stage_wgf consecutive frames (at most WGT: 256 threads, or 64,
// one wave, whose barriers cost nothing).  Phase A (one lane per
// frame) computes each frame's seed, fields, header image with the IPv4 checksum,
// payload length and LCG entry state (sequence.c:433-561, 596-602).  The frames
// then pass through an LDS stage window by window: window w holds the frames that
// start in bytes [w W, (w + 1) W) of the workgroup's output (K.stage_win = W), so
// a window's packed bytes, aligned to the absolute 16-B grid, fit the stage.
//   B  G lanes per frame: every 16-B chunk holding payload is generated whole
//      (glibc LCG, sequence.c:552-555) into the stage, its payload words summed
//      for the L4 checksum (sequence.c:569-594) and reduced over the group.  Bytes
//      a chunk covers outside the payload lie in this frame's or the next frame's
//      header, which C overwrites.
//   C  one lane per (frame, header dword): the headers with their L4 checksums,
//      byte-exact over the stage.
//   S  the window streamed to HBM as one contiguous run of 16-B stores; only the
//      two chunks shared with the neighbouring windows are byte-masked.

template <int G, int RMODE, int WGT>
__global__ __launch_bounds__(WGT) void pb_stage_kernel(pb_kargs K)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    uint8_t *const stage = reinterpret_cast<uint8_t *>(s_dyn);
    const uint32_t WF = K.stage_wgf; // frames per workgroup (<= 256)
    uint2 *const s_l48 = reinterpret_cast<uint2 *>(s_dyn + (K.stage_bytes >> 2)); // lcg48[0 .. PB_STAGE_L48)
    uint32_t *const s_img = s_dyn + (K.stage_bytes >> 2) + 2 * PB_STAGE_L48; // header image, 16 dwords per frame
    uint32_t *const s_r = s_img + WF * 16; // frame start, relative to the workgroup's 16-B chunk
    uint32_t *const s_len = s_r + WF;
    uint32_t *const s_hs = s_len + WF;     // L4 header + pseudo header (+ static payload) word sum
    uint32_t *const s_z = s_hs + WF;       // LCG state at the frame's first 16-B chunk
    uint32_t *const s_nv = s_z + WF;       // nvalid | random << 31
    uint32_t *const s_src = s_nv + WF;     // blob offset (static payload)
    uint32_t *const s_gs = s_src + WF;     // word sum of the drawn bytes B writes outside the payload
    uint32_t *const s_win = s_gs + WF;     // s_win[w]: first frame of window w, [nwin] = nfr

    const uint32_t tid = threadIdx.x;
    const uint32_t flags = K.flags;
    const int hl = (int)K.hl;
    const uint32_t W = K.stage_win;
    const uint64_t f0 = (uint64_t)blockIdx.x * WF;
    const uint64_t left = K.n_frames - f0;
    const uint32_t nfr = left < WF ? (uint32_t)left : WF;
    const uint64_t W0 = K.fixed_len ? f0 * K.fixed_len : K.offsets[f0];
    const uint64_t wbase = W0 & ~15ull;

    // ---------------- A: one lane per frame ----------------
    // the table loads are issued first; their latency hides behind the seed arithmetic
    uint2 l48v[(PB_STAGE_L48 + WGT - 1) / WGT];
#pragma unroll
    for (uint32_t i = 0; i < (PB_STAGE_L48 + WGT - 1) / WGT; ++i)
        if (tid + i * WGT < PB_STAGE_L48)
            l48v[i] = K.lcg48[tid + i * WGT];
    uint32_t my_r = 0;
    if (tid < nfr)
    {
        const uint64_t f = f0 + tid;
        uint64_t base;
        uint32_t flen;
        if (K.fixed_len)
        {
            base = f * K.fixed_len;
            flen = K.fixed_len;
        }
        else
        {
            base = K.offsets[f];
            flen = (uint32_t)(K.offsets[f + 1] - base);
        }
        my_r = (uint32_t)(base - wbase);
        // state at payload index j = -((r % 16) + hl): the first byte of the frame's first chunk
        const uint2 jt = K.jump[PB_JNEG - ((my_r & 15u) + (uint32_t)hl)];
        const uint2 rg1 = (flags & PBK_RND_SADDR) ? K.ranges[0] : make_uint2(0u, 0u);
        uint64_t k;
        uint32_t pi;
        pb_frame_index(K, f, k, pi);
        const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + k);
        const uint32_t r0 = pb_rand_r(s);
        const pb_frame_pl P = pb_payload(K, s, pi);
        uint32_t d[16];
        const uint32_t l4tot = pb_header(K, r0, P.plen, d, K.rng.d == 1 ? rg1 : pb_range(K, r0));
        uint32_t hs = (d[8] >> 16) + pb_halves(d[9]) + pb_halves(d[10]) + pb_halves(d[11]) + pb_halves(d[12]) +
                      pb_halves(d[13]);
        if (flags & PBK_PSEUDO)
            hs += (d[6] >> 16) + pb_halves(d[7]) + (d[8] & 0xFFFFu) + ((K.proto + l4tot) << 8);
        if (!P.random)
            hs += P.ssum;
        pb_u32x4 *row = reinterpret_cast<pb_u32x4 *>(s_img + tid * 16);
        row[0] = pb_u32x4{d[0], d[1], d[2], d[3]};
        row[1] = pb_u32x4{d[4], d[5], d[6], d[7]};
        row[2] = pb_u32x4{d[8], d[9], d[10], d[11]};
        row[3] = pb_u32x4{d[12], d[13], d[14], d[15]};
        s_r[tid] = my_r;
        s_len[tid] = flen;
        s_hs[tid] = hs;
        s_z[tid] = P.random ? jt.x * P.st0 + jt.y : 0u;
        s_nv[tid] = P.nvalid | (P.random << 31);
        s_src[tid] = P.blob_off;
        // B writes every payload chunk whole and unmasked: the first one also holds
        // header bytes [j0, 0) of this frame, the last one bytes [nvalid, jl + 16)
        // that belong to the next frame's header (both rewritten by C).  Their LCG
        // bytes enter B's word sum (output alignment: byte p of a chunk weighs
        // 2^(8 (p & 1))); their sum is taken here once, one lane per frame, and
        // subtracted after B's reduction.  Static payloads read zero padding there;
        // the literal rule keeps B's byte masks.
        uint32_t gs = 0;
        if (P.random && !(flags & PBK_LITERAL))
        {
            const int s0 = (int)(my_r & 15u);
            const int j0 = 16 * ((s0 + hl) >> 4) - s0 - hl; // (-16, 0]
            const int jl = 16 * ((s0 + (int)flen - 1) >> 4) - s0 - hl;
            const uint2 ja = K.jump[PB_JNEG + j0];
            uint32_t x = ja.x * P.st0 + ja.y;
            for (int p = 0; p < -j0; ++p)
            {
                gs += ((x >> 16) & 0xFFu) << (8 * (p & 1));
                x = pb_step3(x, PB_A3, PB_C3);
            }
            const int t0 = (int)P.nvalid > jl ? (int)P.nvalid : jl;
            const uint2 jb = K.jump[PB_JNEG + t0];
            x = jb.x * P.st0 + jb.y;
            for (int p = t0 - jl; p < 16; ++p)
            {
                gs += ((x >> 16) & 0xFFu) << (8 * (p & 1));
                x = pb_step3(x, PB_A3, PB_C3);
            }
        }
        s_gs[tid] = gs;
    }
#pragma unroll
    for (uint32_t i = 0; i < (PB_STAGE_L48 + WGT - 1) / WGT; ++i)
        if (tid + i * WGT < PB_STAGE_L48)
            s_l48[tid + i * WGT] = l48v[i];
    __syncthreads();
    // window starts: frame t opens windows (r_{t-1} / W, r_t / W]  (W >= the longest frame)
    if (tid < nfr)
    {
        const uint32_t w = my_r / W;
        const uint32_t wp = tid ? s_r[tid - 1] / W : 0u;
        if (tid == 0)
            s_win[0] = 0;
        for (uint32_t v = wp + 1; v <= w; ++v)
            s_win[v] = tid;
        if (tid == nfr - 1)
            s_win[w + 1] = nfr;
    }
    __syncthreads();
    const uint32_t nwin = s_r[nfr - 1] / W + 1;

    constexpr uint32_t NGW = WGT / G; // frames in flight per workgroup
    const uint32_t grp = tid / G, lg = tid % G;
    const uint2 MG = s_l48[G];
    const bool lit = (flags & PBK_LITERAL) != 0;
    for (uint32_t w = 0; w < nwin; ++w)
    {
        const uint32_t sb = s_win[w], se = s_win[w + 1];
        const uint32_t R0 = s_r[sb];                      // window bytes [R0, R1), workgroup-relative
        const uint32_t R1 = s_r[se - 1] + s_len[se - 1];
        const uint32_t sbase = R0 & ~15u;

        // ---------------- B: G lanes per frame, payload chunks -> stage ----------------
        for (uint32_t fr = sb + grp; fr < se; fr += NGW)
        {
            const uint32_t r = s_r[fr] - sbase;
            const int flen = (int)s_len[fr];
            const int s0 = (int)(r & 15u);
            const uint32_t cf = r >> 4;                   // stage chunk of the frame's first byte
            const uint32_t nch = (uint32_t)(s0 + flen + 15) >> 4;
            const uint32_t ma = (uint32_t)(s0 + hl) >> 4; // first chunk holding payload (<= 4)
            const uint32_t nv = s_nv[fr];
            const bool rnd = RMODE == 2 ? (nv >> 31) != 0 : RMODE == 1;
            const int nvalid = (int)(nv & 0x7FFFFFFFu);
            const uint32_t src = s_src[fr];
            uint32_t m = ma + lg;
            uint32_t x = 0;
            if (rnd)
            {
                const uint2 Mm = s_l48[m];
                x = __umul24(s_z[fr], Mm.x) + Mm.y;
            }
            uint32_t acc = 0;
            for (; m < nch; m += G)
            {
                const int j0 = (int)(16 * m) - s0 - hl; // payload index of the chunk's first byte
                uint32_t o0, o1, o2, o3;
                pb_chunk_payload(K, rnd, x, src, j0, 0, 16, o0, o1, o2, o3);
                if (lit && (j0 < 0 || j0 + 16 > nvalid))
                {
                    // literal rule: chunk bytes outside the drawn payload are zero (past
                    // nvalid) or header bytes of this / the next frame, rewritten by C
                    const int lo = -j0, hi = nvalid - j0;
                    o0 &= pb_range_mask(lo, hi);
                    o1 &= pb_range_mask(lo - 4, hi - 4);
                    o2 &= pb_range_mask(lo - 8, hi - 8);
                    o3 &= pb_range_mask(lo - 12, hi - 12);
                }
                if (rnd)
                    acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
                reinterpret_cast<pb_u32x4 *>(stage)[cf + m] = pb_u32x4{o0, o1, o2, o3};
                x = __umul24(x, MG.x) + MG.y;
            }
            acc = pb_group_sum<G>(acc);
            if ((flags & PBK_L4_CSUM) && lg == 0)
            {
                uint32_t pc = pb_fold(acc - s_gs[fr]);
                if (r & 1u) // chunk sums were taken in output alignment
                    pc = pb_bswap16(pc);
                const uint32_t c = (~pb_fold(pb_fold(s_hs[fr]) + pc)) & 0xFFFFu;
                s_img[fr * 16 + K.csum_dw] |= K.csum_hi ? (c << 16) : c;
            }
        }
        __syncthreads();

        // ---------------- C: headers -> stage, one lane per (frame, dword) ----------------
        for (uint32_t t = tid; t < (se - sb) * 16; t += WGT)
        {
            const uint32_t fr = sb + (t >> 4), u = t & 15u;
            const uint32_t r = s_r[fr] - sbase;
            const uint32_t sh = r & 3u;
            const uint32_t end = sh + (uint32_t)hl; // bytes of the frame's dword row the header owns: [sh, end)
            if (4 * u < end)
            {
                const uint32_t *img = s_img + fr * 16;
                const uint32_t hi = img[u];
                const uint32_t lo = u > 0 ? img[u - 1] : 0u;
                const uint32_t v = sh ? __builtin_amdgcn_alignbyte(hi, lo, 4u - sh) : hi;
                const uint32_t b0 = u == 0 ? sh : 0u;
                const uint32_t b1 = end - 4 * u < 4 ? end - 4 * u : 4u;
                const uint32_t wd = (r >> 2) + u;
                if (b0 == 0 && b1 == 4)
                    s_dyn[wd] = v;
                else
                    for (uint32_t bb = b0; bb < b1; ++bb)
                        stage[4 * wd + bb] = (uint8_t)(v >> (8 * bb));
            }
        }
        __syncthreads();

        // ---------------- S: stage -> HBM, contiguous 16-B stores ----------------
        // whole chunks [c0, c1) two per lane per step (both LDS reads in flight
        // before the stores); the chunks shared with the neighbouring windows,
        // 0 and c1, are byte-masked (a window is >= 42 B, so they differ)
        const uint32_t lo_b = R0 - sbase, hi_b = R1 - sbase;
        const uint32_t c0 = lo_b ? 1u : 0u, c1 = hi_b >> 4;
        uint8_t *const gout = K.out + wbase + sbase;
        const pb_u32x4 *const st16 = reinterpret_cast<const pb_u32x4 *>(stage);
        for (uint32_t c = c0 + tid; c < c1; c += 2 * WGT)
        {
            const bool two = c + WGT < c1;
            const pb_u32x4 v0 = st16[c];
            const pb_u32x4 v1 = two ? st16[c + WGT] : v0;
            pb_st16(gout + 16 * c, v0);
            if (two)
                pb_st16(gout + 16 * (c + WGT), v1);
        }
        if (tid == 0 && lo_b)
        {
            const pb_u32x4 v = st16[0];
            pb_store_chunk(gout, v[0], v[1], v[2], v[3], -(int)lo_b, (int)(hi_b - lo_b));
        }
        if (tid == WGT - 1 && (hi_b & 15u))
        {
            const pb_u32x4 v = st16[c1];
            pb_store_chunk(gout + 16 * c1, v[0], v[1], v[2], v[3], (int)(16 * c1) - (int)lo_b, (int)(hi_b - lo_b));
        }
        __syncthreads(); // the next window reuses the stage
    }
    if (tid == 0 && nfr) // the windows stored the workgroup's frames' bytes, each once
        pb_count(K, blockIdx.x, nfr, s_r[nfr - 1] + s_len[nfr - 1] - s_r[0]);
}

// ---------------- fixed-length staged: pb_fstage_kernel ----------------
//
// The configs[1] 1500-B shape (any fixed length > 128 B that is a multiple of 4,
// every payload random, stream rule) with the per-frame and per-window work of
// pb_stage_kernel cut down: that kernel runs VALU-bound (PMC: ~80% of the SIMD
// issue cycles) and spends ~45% of its VALU instructions outside the payload
// loop (105 per 1500-B frame, 56 in the loop).
//  * Every frame starts on a dword (flen % 4 == 0) and a window is exactly
//    NGW = 256 / G frames, so NGW * flen % 16 == 0: every window (and every
//    workgroup, WF being a multiple of NGW) starts on a 16-B boundary, and a
//    lane's frame offset, chunk range and LCG entry constant (L^(48 m)) are the
//    same in every window.
//  * Lane lg of a group takes the frame's payload chunks nch-1-lg, nch-1-lg-G, ...
//    in ascending order, so the frame's last chunk (which may also hold the next
//    frame's first dwords) is lane 0's final chunk, in the wave's final pass:
//    only it is stored dword-masked.  No two groups then write the same stage
//    bytes, and the group writes its own header right after its payload (LDS
//    operations of one wave complete in order): no header pass, one barrier per
//    window.
//  * Lane 0's checksum accumulator starts at A's per-frame constant: the header /
//    pseudo-header word sum minus the generated header bytes of the first payload
//    chunk (overwritten by the header), so the group reduction is the whole sum.
//  * One stage buffer by default (K.fst_nbuf; two, where window w + 1 is generated while window
//    w's stores drain, measured slower: 7.64-7.67 vs 7.17-7.23 ms per 2^25 1500-B frames, round 6).
template <int G, bool L4>
__global__ __launch_bounds__(PB_WG) void pb_fstage_kernel(pb_kargs K)
{
    constexpr uint32_t NGW = PB_WG / G; // frames per window
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    const uint32_t SB = K.fst_sb, NB = K.fst_nbuf, WF = K.fst_wgf;
    uint8_t *const stage = reinterpret_cast<uint8_t *>(s_dyn);
    uint32_t *const s_img = s_dyn + ((NB * SB) >> 2); // header image, 16 dwords per frame
    uint32_t *const s_z = s_img + WF * 16;             // LCG state at the frame's first 16-B chunk
    uint32_t *const s_a0 = s_z + WF;                   // lane 0's initial checksum accumulator

    const uint32_t tid = threadIdx.x;
    const uint32_t flags = K.flags;
    const uint32_t flen = K.fixed_len, hl = K.hl;
    const uint64_t f0 = (uint64_t)pb_xcd_region(blockIdx.x, gridDim.x) * WF;
    const uint64_t left = K.n_frames - f0;
    const uint32_t nfr = left < WF ? (uint32_t)left : WF;
    const uint64_t W0 = f0 * flen; // 16-B aligned

    // lane constants: group grp builds frame w * NGW + grp of every window w
    const uint32_t grp = tid / G, lg = tid % G;
    const uint32_t r = grp * flen; // frame start, relative to its window
    const uint32_t s0 = r & 15u;
    const uint32_t ma = (s0 + hl) >> 4;           // first chunk holding payload
    const uint32_t nch = (s0 + flen + 15u) >> 4;  // chunks the frame touches
    const uint32_t e4 = ((s0 + flen) & 15u) >> 2; // dwords of the frame in its last chunk (0: all 4)
    const uint32_t mlast = nch - 1u - lg;         // this lane's last chunk
    const uint32_t cnt = mlast >= ma && mlast < nch ? (mlast - ma) / G + 1u : 0u;
    const uint32_t mfirst = mlast - (cnt ? cnt - 1u : 0u) * G;
    const uint2 Mm = K.lcg48[cnt ? mfirst : 0u];
    const uint2 MG = K.lcg48[G];
    const uint32_t mgy = pb_vgpr(MG.y);
    const bool tail = lg == 0 && e4 != 0; // lane 0's final chunk is cut at dword e4

    // ---------------- A: one lane per frame ----------------
    const uint2 rg1 = (flags & PBK_RND_SADDR) ? K.ranges[0] : make_uint2(0u, 0u);
    if (tid < nfr)
    {
        const uint64_t f = f0 + tid;
        const uint32_t hs0 = (((tid % NGW) * flen) & 15u) + hl;
        const uint2 jt = K.jump[PB_JNEG - hs0];
        const int j0 = (int)(16u * (hs0 >> 4)) - (int)hs0; // (-16, 0]: header bytes in chunk ma
        const uint2 ja = K.jump[PB_JNEG + j0];
        uint64_t k;
        uint32_t pi;
        pb_frame_index(K, f, k, pi);
        const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + k);
        const uint32_t r0 = pb_rand_r(s);
        const pb_frame_pl P = pb_payload<false>(K, s, pi);
        uint32_t d[16];
        const uint32_t l4tot = pb_header(K, r0, P.plen, d, K.rng.d == 1 ? rg1 : pb_range(K, r0));
        pb_u32x4 *row = reinterpret_cast<pb_u32x4 *>(s_img + tid * 16);
        row[0] = pb_u32x4{d[0], d[1], d[2], d[3]};
        row[1] = pb_u32x4{d[4], d[5], d[6], d[7]};
        row[2] = pb_u32x4{d[8], d[9], d[10], d[11]};
        row[3] = pb_u32x4{d[12], d[13], d[14], d[15]};
        s_z[tid] = jt.x * P.st0 + jt.y;
        if (L4)
        {
            uint32_t hs = (d[8] >> 16) + pb_halves(d[9]) + pb_halves(d[10]) + pb_halves(d[11]) +
                          pb_halves(d[12]) + pb_halves(d[13]);
            if (flags & PBK_PSEUDO)
                hs += (d[6] >> 16) + pb_halves(d[7]) + (d[8] & 0xFFFFu) + ((K.proto + l4tot) << 8);
            // the generated header bytes of chunk ma, in output alignment (frames start on even bytes)
            uint32_t gs = 0;
            uint32_t x = ja.x * P.st0 + ja.y;
            for (int p = 0; p < -j0; ++p)
            {
                gs += ((x >> 16) & 0xFFu) << (8 * (p & 1));
                x = pb_step3(x, PB_A3, PB_C3);
            }
            // one's-complement arithmetic is mod 0xFFFF: add a multiple of it to stay >= 0
            s_a0[tid] = hs + 16u * 0xFFFFu - gs;
        }
    }
    __syncthreads();

    const uint32_t nwin = (nfr + NGW - 1) / NGW;
    const uint32_t hw = hl >> 2; // header dwords written whole; hl % 4 == 2: one more half dword
    uint32_t sb = 0;
    for (uint32_t w = 0; w < nwin; ++w)
    {
        uint8_t *const stg = stage + sb;
        const uint32_t nfw = min(NGW, nfr - w * NGW);
        const uint32_t fr = w * NGW + grp;
        const bool live = grp < nfw;
        // ---------------- B: payload chunks, then the group's header ----------------
        uint32_t acc = 0;
        if (live && cnt)
        {
            if (L4 && lg == 0)
                acc = s_a0[fr];
            uint32_t x = __umul24(s_z[fr], Mm.x) + Mm.y;
            pb_u32x4 *p = reinterpret_cast<pb_u32x4 *>(stg) + (r >> 4) + mfirst;
            uint32_t o0, o1, o2, o3;
            for (uint32_t i = 1; i < cnt; ++i)
            {
                pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
                if (L4)
                    acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
                *p = pb_u32x4{o0, o1, o2, o3};
                p += G;
                x = pb_mad24(x, MG.x, mgy);
            }
            // the lane's final chunk
            pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
            if (tail)
            {
                uint32_t *q = reinterpret_cast<uint32_t *>(p);
                o1 = e4 > 1u ? o1 : 0u;
                o2 = e4 > 2u ? o2 : 0u;
                o3 = 0u;
                q[0] = o0;
                if (e4 > 1u)
                    q[1] = o1;
                if (e4 > 2u)
                    q[2] = o2;
            }
            else
                *p = pb_u32x4{o0, o1, o2, o3};
            if (L4)
                acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
        }
        if (L4)
            acc = pb_group_sum<G>(acc);
        if (live && lg <= hw)
        {
            uint32_t v = s_img[fr * 16 + lg];
            if (L4)
            {
                const uint32_t c = (~pb_fold(acc)) & 0xFFFFu;
                if (lg == K.csum_dw)
                    v |= K.csum_hi ? (c << 16) : c;
            }
            uint32_t *hp = reinterpret_cast<uint32_t *>(stg + r) + lg;
            if (lg < hw)
                *hp = v;
            else if (hl & 2u)
                *reinterpret_cast<uint16_t *>(hp) = (uint16_t)v;
        }
        __syncthreads();

        // ---------------- S: the window to HBM, contiguous 16-B stores ----------------
        // window bytes [0, R1); a last chunk that is not whole (the launch's last,
        // short window) is stored dword by dword.  Lane t stores the window's chunks
        // whose absolute 16-B index is t mod 256, so each wave's store instruction
        // covers one 1 KiB-aligned block and each step of the workgroup one 4 KiB
        // page (wave stores straddling 1 KiB boundaries cost ~10% of the write
        // rate: profiles/r01/wbench, shifted pages)
        const uint32_t R1 = nfw * flen;
        const uint32_t c1 = R1 >> 4;
        const uint64_t gb = W0 + (uint64_t)w * NGW * flen;
        uint8_t *const gout = K.out + gb;
        const pb_u32x4 *const st16 = reinterpret_cast<const pb_u32x4 *>(stg);
        uint32_t c = (tid - (uint32_t)(gb >> 4)) & (PB_WG - 1u);
        for (; c + 3 * PB_WG < c1; c += 4 * PB_WG)
        {
            const pb_u32x4 v0 = st16[c], v1 = st16[c + PB_WG], v2 = st16[c + 2 * PB_WG], v3 = st16[c + 3 * PB_WG];
            pb_st16(gout + 16 * c, v0);
            pb_st16(gout + 16 * (c + PB_WG), v1);
            pb_st16(gout + 16 * (c + 2 * PB_WG), v2);
            pb_st16(gout + 16 * (c + 3 * PB_WG), v3);
        }
        for (; c < c1; c += PB_WG)
            pb_st16(gout + 16 * c, st16[c]);
        if (tid == PB_WG - 1 && (R1 & 15u))
        {
            const uint32_t *sw = reinterpret_cast<const uint32_t *>(stg) + 4 * c1;
            uint32_t *gw = reinterpret_cast<uint32_t *>(gout) + 4 * c1;
            for (uint32_t t = 0; t < ((R1 & 15u) >> 2); ++t)
                gw[t] = sw[t];
        }
        if (NB == 1)
            __syncthreads(); // the next window reuses the stage
        else
            sb = sb ? 0u : SB;
    }
    if (tid == 0)
        pb_count(K, blockIdx.x, nfr, (uint64_t)nfr * flen);
}

// ---------------- any length, every payload random: pb_vstage_kernel ----------------
//
// Packed variable-length frames (configs[2]) and fixed lengths that are not a
// multiple of 4: pb_stage_kernel's windows (frames starting in bytes
// [w W, (w + 1) W) of the workgroup's output), with the per-frame work cut
// (DESIGN.md 5.4a):
//  * phase A: one lane per slot (up to 4 earlier "ghost" frames, then the own
//    frames), lengths from the seeds, starts from a workgroup scan on top of one
//    offset; per frame only header dwords 4-12 in LDS, the rest from the template;
//  * payload pass: g lanes per frame (8/16/32 by window), every chunk holding payload
//    written once and plain (zeros outside the frame), edge chunks masked from a
//    table; the L4 sum reduced over the group and written into the frame's record;
//  * barrier, then a header pass with one lane per (frame, header chunk), ORing the
//    header into the chunks it shares with payload or with the previous frame;
//  * S: the window's chunks to HBM; the chunk shared with the next window is carried
//    into that window's stage chunk 0 instead of being stored twice, byte-masked;
//    the stage is never cleared.
// Lane lg of a group takes chunks nch-1-lg, nch-1-lg-G, ... as in pb_fstage_kernel.
template <int G, bool L4>
__global__ __launch_bounds__(PB_WG) void pb_vstage_kernel(pb_kargs K)
{
    constexpr uint32_t NGW = PB_WG / G; // frames in flight per workgroup
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    const uint32_t WF = K.stage_wgf, W = K.stage_win, SB = K.stage_bytes;
    const uint32_t CAP = (WF + PB_VST_GHOSTS + 1u) & ~1u; // frames of the workgroup's arrays: ghosts + own (rounded to even)
    pb_u32x4 *const stage = reinterpret_cast<pb_u32x4 *>(s_dyn);
    uint2 *const s_l48 = reinterpret_cast<uint2 *>(s_dyn + (SB >> 2)); // lcg48[0 .. PB_STAGE_L48)
    uint2 *const s_jt = s_l48 + PB_STAGE_L48;                          // jump[PB_JNEG - (i + hl)], i < 16
    uint64_t *const s_st0 = reinterpret_cast<uint64_t *>(s_jt + 16);   // [0, GH]: slot starts - base0; [8, 12): S0 parts
    uint32_t *const s_wsum = reinterpret_cast<uint32_t *>(s_st0 + 12); // per-wave length sums
    uint32_t *const s_tm = s_wsum + 4;                                 // the header template (16 dwords)
    pb_u32x4 *const s_m16 = reinterpret_cast<pb_u32x4 *>(s_tm + 16);   // s_m16[k]: chunk bytes >= k set, k <= 16
    // per frame only header dwords [PB_VST_HV0, PB_VST_HV0 + PB_VST_HVN) (every per-frame field and
    // the checksums); the others are the template's
    uint32_t *const s_hv = s_dyn + (SB >> 2) + 2 * PB_STAGE_L48 + PB_VST_PRO / 4;
    uint32_t *const s_r = s_hv + CAP * PB_VST_HVN;                     // frame start, workgroup-relative
    uint32_t *const s_len = s_r + CAP;
    uint32_t *const s_z = s_len + CAP;  // LCG state at the frame's first 16-B chunk
    uint32_t *const s_hs = s_z + CAP;   // header + pseudo header word sum, folded (frame alignment)
    uint32_t *const s_win = s_hs + CAP; // s_win[w]: first frame of window w, [nwin] = nfr
    uint32_t *const s_ord = s_win + CAP + 2; // frames of each window, longest first

    const uint32_t tid = threadIdx.x;
    const uint32_t bxr = pb_xcd_region(blockIdx.x, gridDim.x); // region
    const uint32_t flags = K.flags;
    const uint32_t hl = K.hl;
    // Workgroup b owns frames [f0, f0 + nown) and stores exactly the output bytes
    // [lo, hi): lo = the 128-B line holding its first frame's start (0 for b = 0), hi =
    // the next workgroup's lo.  No line is written by two workgroups (two XCDs): an
    // edge that split a line cost 5-12% of the write rate (profiles/r02/wbench,
    // shift_*.txt).  The bytes of [lo, start(f0)) belong to up to PB_VST_GHOSTS earlier
    // frames ("ghosts"), built here in full (their checksums need every byte) and
    // stored only inside [lo, hi); the bytes of the own last frames past hi are the
    // next workgroup's ghosts.
    const uint64_t f0 = (uint64_t)bxr * WF;
    const uint64_t left = K.n_frames - f0;
    const uint32_t nown = left < WF ? (uint32_t)left : WF;
    const uint64_t fe = f0 + nown;
    // (PBGPU_VST_SHAPE bit 6: the round-1 edges at the frame starts, lines split)
    const uint64_t emask = (K.vst_shape & 64u) ? ~0ull : ~127ull;

    // ---------------- A: one lane per slot; the stage starts zero ----------------
    // Slot j holds frame f0 - PB_VST_GHOSTS + j: the possible ghosts, then the own
    // frames.  The lengths come from the seeds and the starts from a workgroup scan
    // of them on top of one offset, so the global loads (that offset, the jump
    // entries, lcg48) are independent of each other and their latency overlaps the
    // seed / header arithmetic (a chain offsets -> ghosts -> offsets -> jump entry
    // was ~3 dependent load round trips per workgroup).
    constexpr uint32_t GH = PB_VST_GHOSTS;
    const int64_t fb = (int64_t)f0 - (int64_t)GH;
    // start of frame f0: fixed length, or the scanned per-workgroup length sums (l2 prefix of
    // this workgroup's group of PB_VL_GRP + the sums of the earlier workgroups of the group), or
    // offsets[] when the 3-pass scan ran
    const bool bsum = !K.fixed_len && K.vblk_sum != nullptr;
    uint64_t s0_part = 0;
    if (bsum && tid < (bxr & (PB_VL_GRP - 1u)))
        s0_part = K.vblk_sum[(bxr & ~(PB_VL_GRP - 1u)) + tid];
    const uint64_t s0_base = K.fixed_len ? f0 * K.fixed_len : (bsum ? K.vblk_l2[bxr / PB_VL_GRP] : K.offsets[f0]);
    uint2 jtv = make_uint2(0u, 0u);
    if (tid < 16u) // state at payload index -((r % 16) + hl): the first byte of the frame's first chunk
        jtv = K.jump[PB_JNEG - (tid + hl)];
    uint2 l48v[(PB_STAGE_L48 + PB_WG - 1) / PB_WG];
#pragma unroll
    for (uint32_t i = 0; i < (PB_STAGE_L48 + PB_WG - 1) / PB_WG; ++i)
        if (tid + i * PB_WG < PB_STAGE_L48)
            l48v[i] = K.lcg48[tid + i * PB_WG];
    const uint2 rg1 = (flags & PBK_RND_SADDR) ? K.ranges[0] : make_uint2(0u, 0u);
    const int64_t fj = fb + (int64_t)tid;
    const bool valid = tid < CAP && fj >= 0 && (uint64_t)fj < fe;
    uint32_t flen = 0, st0 = 0, hsf = 0;
    uint32_t d[16];
    if (valid)
    {
        uint64_t k;
        uint32_t pi;
        pb_frame_index(K, (uint64_t)fj, k, pi);
        const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + k);
        const uint32_t r0 = pb_rand_r(s);
        const pb_frame_pl P = pb_payload<false>(K, s, pi);
        const uint32_t l4tot = pb_header(K, r0, P.plen, d, K.rng.d == 1 ? rg1 : pb_range(K, r0));
        flen = K.fixed_len ? K.fixed_len : hl + P.plen;
        st0 = P.st0;
        if (L4)
        {
            uint32_t hs = (d[8] >> 16) + pb_halves(d[9]) + pb_halves(d[10]) + pb_halves(d[11]) +
                          pb_halves(d[12]) + pb_halves(d[13]);
            if (flags & PBK_PSEUDO)
                hs += (d[6] >> 16) + pb_halves(d[7]) + (d[8] & 0xFFFFu) + ((K.proto + l4tot) << 8);
            hsf = pb_fold(hs);
        }
    }
    // frame starts: exclusive scan of the slot lengths (in-wave shuffles, wave totals via LDS)
    const uint32_t lane = tid & 63u, wv = tid >> 6;
    uint32_t inc = flen;
#pragma unroll
    for (uint32_t dd = 1; dd < 64; dd <<= 1)
    {
        const uint32_t y = __shfl_up(inc, dd, 64);
        inc += lane >= dd ? y : 0u;
    }
#pragma unroll
    for (uint32_t dd = 32; dd > 0; dd >>= 1)
        s0_part += __shfl_xor(s0_part, dd, 64);
    if (lane == 63u)
        s_wsum[wv] = inc;
    if (lane == 0u)
        s_st0[8 + wv] = s0_part;
    if (tid <= GH) // slots 0 .. GH are in wave 0: no earlier waves
        s_st0[tid] = inc - flen;
    if (tid < 16u)
        s_jt[tid] = jtv;
    if (tid <= 16u)
        s_m16[tid] = pb_u32x4{pb_range_mask((int)tid, 4), pb_range_mask((int)tid - 4, 4), pb_range_mask((int)tid - 8, 4),
                              pb_range_mask((int)tid - 12, 4)};
    if (tid == 0u)
    {
        pb_u32x4 *const tm = reinterpret_cast<pb_u32x4 *>(s_tm);
        tm[0] = pb_u32x4{K.tmpl[0], K.tmpl[1], K.tmpl[2], K.tmpl[3]};
        tm[1] = pb_u32x4{K.tmpl[4], K.tmpl[5], K.tmpl[6], K.tmpl[7]};
        tm[2] = pb_u32x4{K.tmpl[8], K.tmpl[9], K.tmpl[10], K.tmpl[11]};
        tm[3] = pb_u32x4{K.tmpl[12], K.tmpl[13], K.tmpl[14], K.tmpl[15]};
    }
#pragma unroll
    for (uint32_t i = 0; i < (PB_STAGE_L48 + PB_WG - 1) / PB_WG; ++i)
        if (tid + i * PB_WG < PB_STAGE_L48)
            s_l48[tid + i * PB_WG] = l48v[i];
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < PB_WG / 64; ++w)
    {
        const uint32_t t = s_wsum[w];
        pre += w < wv ? t : 0u;
        tot += t;
    }
    uint64_t S0 = s0_base;
#pragma unroll
    for (uint32_t w = 0; w < PB_WG / 64; ++w)
        S0 += s_st0[8 + w];
    const uint64_t base0 = S0 - s_st0[GH]; // start of slot 0 (the valid ghost slots' lengths before f0)
    const uint64_t start = base0 + pre + (inc - flen);
    if (bsum && valid && tid >= GH) // own frames: the offsets the 3-pass scan would have written
        K.offsets_w[(uint64_t)fj] = start;
    // Workgroup b owns frames [f0, f0 + nown) and stores exactly the output bytes
    // [lo, hi): lo = the 128-B line holding its first frame's start (0 for b = 0), hi =
    // the next workgroup's lo.  No line is written by two workgroups (two XCDs): an
    // edge that split a line cost 5-12% of the write rate (profiles/r02/wbench,
    // shift_*.txt).  The bytes of [lo, start(f0)) belong to up to PB_VST_GHOSTS earlier
    // frames ("ghosts"), built here in full (their checksums need every byte) and
    // stored only inside [lo, hi); the bytes of the own last frames past hi are the
    // next workgroup's ghosts.
    const uint64_t lo_abs = bxr ? (S0 & emask) : 0ull;
    const uint64_t hi_abs = fe < K.n_frames ? ((base0 + tot) & emask) : base0 + tot;
    uint32_t ng = 0;
    // ghost l = frame f0 - 1 - l, present while it ends (= frame f0 - l starts) past lo;
    // the ghosts are a prefix l = 0, 1, ...
    if (bxr)
        while (ng < GH && f0 > ng && base0 + s_st0[GH - ng] > lo_abs)
            ++ng;
    const uint32_t nfr = ng + nown; // frames built: ghosts + own, array index t = slot - (GH - ng)
    const uint64_t wbase = (base0 + s_st0[GH - ng]) & ~15ull;
    const uint32_t lo_rel = (uint32_t)(lo_abs - wbase), hi_rel = (uint32_t)(hi_abs - wbase);
    const int32_t tix = (int32_t)tid - (int32_t)(GH - ng);
    if (valid && tix >= 0)
    {
        const uint32_t r = (uint32_t)(start - wbase);
        const uint2 jt = s_jt[r & 15u];
        uint32_t *const hv = s_hv + tix * PB_VST_HVN;
#pragma unroll
        for (uint32_t w = 0; w < PB_VST_HVN; ++w)
            hv[w] = d[PB_VST_HV0 + w];
        s_r[tix] = r;
        s_len[tix] = flen;
        s_z[tix] = jt.x * st0 + jt.y;
        if (L4)
            s_hs[tix] = hsf;
    }
    __syncthreads();
    const uint32_t my_r = tid < nfr ? s_r[tid] : 0u;
    // window starts: frame t opens windows (r_{t-1} / W, r_t / W]  (W >= the longest frame)
    if (tid < nfr)
    {
        const uint32_t w = my_r / W;
        const uint32_t wp = tid ? s_r[tid - 1] / W : 0u;
        if (tid == 0)
            s_win[0] = 0;
        for (uint32_t v = wp + 1; v <= w; ++v)
            s_win[v] = tid;
        if (tid == nfr - 1)
            s_win[w + 1] = nfr;
    }
    __syncthreads();
    const uint32_t nwin = s_r[nfr - 1] / W + 1;
    // the frames of a window ordered longest first, so a wave's groups build frames of
    // similar length (random lengths: the wave runs as long as its longest frame);
    // windows of more than 64 frames keep their order
    if (tid < nfr)
    {
        const uint32_t w = my_r / W;
        const uint32_t b = s_win[w], e = s_win[w + 1];
        uint32_t rank = tid - b;
        if (e - b <= 64 && !(K.vst_shape & 256u))
        {
            const uint32_t len = s_len[tid];
            rank = 0;
            for (uint32_t u = b; u < e; ++u)
            {
                const uint32_t lu = s_len[u];
                rank += (lu > len || (lu == len && u < tid)) ? 1u : 0u;
            }
        }
        s_ord[b + rank] = tid;
    }
    __syncthreads();

    for (uint32_t w = 0; w < nwin; ++w)
    {
        const uint32_t sb = s_win[w], se = s_win[w + 1];
        const uint32_t R0 = s_r[sb]; // window bytes [R0, R1), workgroup-relative
        const uint32_t R1 = s_r[se - 1] + s_len[se - 1];
        const uint32_t sbase = R0 & ~15u;

        // lanes per frame: G, or (G = 8, windows of F <= 32 frames) every lane busy — the
        // window's longest frames (s_ord is longest first) take 32 / 16 lanes: y frames of
        // 32, then x of 16, then 8 each, groups aligned to their size
        uint32_t g = G, grp0 = tid / G, lg = tid % G;
        bool any32 = false; // (workgroup-uniform) a 32-lane group exists in this window
        // the layout's counts assume 256 lanes: 32 y + 16 x == 256 for 9-16 frames, 32 F <= 256 for F <= 8
        static_assert(PB_WG == 256, "pb_vstage_kernel's 32/16/8-lane window layout is for 256-thread workgroups");
        if (G == 8 && !(K.vst_shape & 16u))
        {
            const uint32_t F = se - sb;
            uint32_t y = 0, x = 0;
            if (F <= 16u)
            {
                y = K.vst_shape & 32u ? 0u : (F <= 8u ? F : 16u - F);
                x = F - y;
            }
            else if (F <= 32u)
                x = 32u - F;
            any32 = y > 0u;
            if (tid < 32u * y)
                g = 32, grp0 = tid >> 5, lg = tid & 31u;
            else if (tid < 32u * y + 16u * x)
                g = 16, grp0 = y + ((tid - 32u * y) >> 4), lg = tid & 15u;
            else
                grp0 = y + x + ((tid - 32u * y - 16u * x) >> 3), lg = tid & 7u;
        }
        const uint2 MG = s_l48[g];

        // ---------------- B: g lanes per frame, payload chunks, then the header ----------------
        for (uint32_t k = sb + grp0; k < se; k += NGW)
        {
            const uint32_t fr = s_ord[k];
            const uint32_t r = s_r[fr] - sbase;
            const uint32_t s0 = r & 15u, cf = r >> 4;
            const uint32_t hend = s0 + hl;                   // header end, frame-chunk relative
            const uint32_t fend = s0 + s_len[fr];            // frame end
            const uint32_t ma = hend >> 4;                   // first chunk holding payload
            const uint32_t nch = (fend + 15u) >> 4;          // chunks the frame touches
            const uint32_t mlast = nch - 1u - lg;            // this lane's last chunk (wraps if none)
            const uint32_t cnt = mlast < nch && mlast >= ma ? (mlast - ma) / g + 1u : 0u;
            uint32_t acc = 0;
            if (cnt)
            {
                // edge chunks (the lane's first may be chunk ma, lane 0's last the frame's last)
                // are masked in the first and last passes only; the passes between are plain
                uint32_t m = mlast - __umul24(cnt - 1u, g);
                const uint2 Mm = s_l48[m];
                uint32_t x = __umul24(s_z[fr], Mm.x) + Mm.y;
                pb_u32x4 *p = stage + cf + m;
                auto edge = [&](uint32_t mm, pb_u32x4 *pp) {
                    uint32_t o0, o1, o2, o3;
                    pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
                    const bool last = mm + 1u == nch;
                    const int lo = mm == ma ? (int)(hend & 15u) : 0;
                    const int hi = last ? (int)(fend - 16u * mm) : 16;
                    if (lo > 0 || hi < 16)
                    {
                        // keep bytes [lo, hi): two table rows instead of four clamped 64-bit shift pairs
                        const pb_u32x4 ml = s_m16[lo], mh = s_m16[hi];
                        o0 &= ml[0] & ~mh[0];
                        o1 &= ml[1] & ~mh[1];
                        o2 &= ml[2] & ~mh[2];
                        o3 &= ml[3] & ~mh[3];
                    }
                    if (L4)
                        acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
                    // whole chunk, zeros outside [lo, hi): the header bytes (this frame's or, past
                    // the frame's end, the next frame's) are ORed in after the barrier below
                    *pp = pb_u32x4{o0, o1, o2, o3};
                };
                edge(m, p);
                for (uint32_t i = 2; i < cnt; ++i)
                {
                    x = pb_mad24v(x, MG.x, MG.y);
                    m += g;
                    p += g;
                    uint32_t o0, o1, o2, o3;
                    pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
                    if (L4)
                        acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
                    *p = pb_u32x4{o0, o1, o2, o3};
                }
                if (cnt > 1u)
                {
                    x = pb_mad24v(x, MG.x, MG.y);
                    m += g;
                    p += g;
                    edge(m, p);
                }
            }
            uint32_t *const hv = s_hv + __umul24(fr, PB_VST_HVN);
            if (L4)
            {
                if (G == 8)
                {
                    // sums over 8, 16 and 32 lanes; each lane keeps its own group's
                    const uint32_t a8 = pb_group_sum<8>(acc);
                    const uint32_t a16 = a8 + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a8, 0x128, 0xF, 0xF, false);
                    acc = g == 8 ? a8 : a16;
                    if (any32) // the cross-row step (an LDS permute) only for windows that use it
                    {
                        const uint32_t a32 = a16 + __shfl_xor(a16, 16, 64);
                        acc = g == 32 ? a32 : acc;
                    }
                }
                else
                    acc = pb_group_sum<G>(acc);
                if (lg == 0)
                {
                    // chunk sums were taken in output alignment
                    uint32_t pc = pb_fold(acc);
                    if (r & 1u)
                        pc = pb_bswap16(pc);
                    const uint32_t c = (~pb_fold(s_hs[fr] + pc)) & 0xFFFFu;
                    hv[K.csum_dw - PB_VST_HV0] |= K.csum_hi ? (c << 16) : c;
                }
            }
            // a frame without payload: its last chunk (header bytes, then the next frame's) gets
            // its plain write here, as every payload-ending chunk does in the loop above
            if (lg == 0u && fend == hend && (hend & 15u))
                stage[cf + nch - 1u] = pb_u32x4{0u, 0u, 0u, 0u};
        }
        // every chunk of the window holding payload has had its one plain write; the headers
        // are ORed into the chunks they share with payload or with the previous frame
        // One lane per (frame, header chunk), frames in window order, mh = the most header
        // chunks a frame can touch: ~F * mh lanes carry the pass (configs[2]: ~108 of 256), so
        // the other waves skip it instead of running it with one live lane in two or three
        __syncthreads();
        const uint32_t mh = (hl + 30u) >> 4;
        const uint32_t mhinv = (65536u + mh - 1u) / mh;
        const uint32_t nhl = (se - sb) * mh;
        for (uint32_t i = tid; i < nhl; i += PB_WG)
        {
            const uint32_t ti = __umul24(i, mhinv) >> 16; // i / mh (exact for i < 2^12, mh <= 8)
            const uint32_t lg = i - __umul24(ti, mh);
            const uint32_t fr = sb + ti;
            const uint32_t r = s_r[fr] - sbase;
            const uint32_t s0 = r & 15u, cf = r >> 4;
            const uint32_t hend = s0 + hl;
            const uint32_t *const hv = s_hv + __umul24(fr, PB_VST_HVN);
            // header chunks 0 .. nhc-1: the image shifted to byte s0 (the image is zero past hl);
            // the first is shared with the previous frame unless s0 == 0, the last with the
            // payload (or the next frame) unless the header ends on the chunk edge
            const uint32_t nhc = (hend + 15u) >> 4;
            if (lg < nhc)
            {
                // frame bytes [16 lg - s0, 16 lg - s0 + 16): header dwords i0 .. i0 + 4 (the frame's
                // own for [PB_VST_HV0, PB_VST_HV0 + PB_VST_HVN), else the template's); those outside
                // the 16-dword header read as zero
                const int xb = (int)(16u * lg) - (int)s0;
                const int i0 = xb >> 2;
                const uint32_t sh = (uint32_t)xb & 3u;
                uint32_t wv[5];
#pragma unroll
                for (int t = 0; t < 5; ++t)
                {
                    const int ix = i0 + t;
                    const uint32_t *src =
                        (uint32_t)(ix - (int)PB_VST_HV0) < PB_VST_HVN ? hv + (ix - (int)PB_VST_HV0) : s_tm + (ix & 15);
                    const uint32_t v = *src;
                    wv[t] = (uint32_t)ix < 16u ? v : 0u;
                }
                uint32_t h[4];
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    h[t] = __builtin_amdgcn_alignbyte(wv[t + 1], wv[t], sh);
                pb_u32x4 *p = stage + cf + lg;
                // (the workgroup's first frame has no predecessor built here: its chunk 0 is
                // written plain, zeros before the frame, bytes another workgroup stores)
                if ((lg == 0 && s0 && fr > 0u) || (lg + 1u == nhc && (hend & 15u)))
                {
                    uint32_t *q = reinterpret_cast<uint32_t *>(p);
                    atomicOr(q + 0, h[0]);
                    atomicOr(q + 1, h[1]);
                    atomicOr(q + 2, h[2]);
                    atomicOr(q + 3, h[3]);
                }
                else
                    *p = pb_u32x4{h[0], h[1], h[2], h[3]};
            }
        }
        __syncthreads();

        // ---------------- S: stage -> HBM, contiguous 16-B stores, then zero ----------------
        // the window's bytes [R0, R1) clipped to the workgroup's [lo, hi): whole chunks
        // [cf0, cf1); a chunk the window shares with a neighbouring window (same
        // workgroup) is byte-masked, stored by the lane that then zeroes it
        // A chunk shared with the next window of this workgroup is not stored here: its value
        // is carried into the next window's stage chunk 0 (the same 16 B of output) and stored
        // whole with that window (masked byte stores by one lane per window edge made S ~25%
        // of a workgroup's life).  Only workgroup edges (128-B aligned unless PBGPU_VST_SHAPE bit 6)
        // and the launch's end keep masked stores.
        const uint32_t R0c = R0 > lo_rel ? R0 : lo_rel, R1c = R1 < hi_rel ? R1 : hi_rel;
        uint32_t cf0 = 0, cf1 = 0;
        uint8_t *const gout = K.out + wbase + sbase;
        bool cout = false;
        uint32_t chc = 0;
        pb_u32x4 cv = pb_u32x4{0u, 0u, 0u, 0u};
        if (R0c < R1c)
        {
            const uint32_t lo_b = R0c - sbase, hi_b = R1c - sbase;
            const uint32_t cl = lo_b >> 4, ch = hi_b >> 4;
            const bool cin = w > 0 && R0c == R0 && (lo_b & 15u); // chunk cl holds the previous window's tail
            cout = w + 1u < nwin && R1c == R1 && (hi_b & 15u);
            chc = ch;
            cf0 = cin ? cl : (lo_b + 15u) >> 4;
            cf1 = ch;
            if (cout && tid == (ch & (PB_WG - 1u)))
                cv = stage[ch];
            if ((lo_b & 15u) && !cin && tid == (cl & (PB_WG - 1u)))
            {
                const pb_u32x4 v = stage[cl];
                pb_store_chunk(gout + 16 * cl, v[0], v[1], v[2], v[3], (int)(16 * cl) - (int)lo_b,
                               (int)(hi_b - lo_b));
            }
            if ((hi_b & 15u) && !cout && !((lo_b & 15u) && !cin && cl == ch) && tid == (ch & (PB_WG - 1u)))
            {
                const pb_u32x4 v = stage[ch];
                pb_store_chunk(gout + 16 * ch, v[0], v[1], v[2], v[3], (int)(16 * ch) - (int)lo_b,
                               (int)(hi_b - lo_b));
            }
        }
        // (one chunk per step: four LDS reads in flight, then four stores, measured 1.7%
        // slower on configs[2])
        for (uint32_t c = cf0 + ((tid - cf0) & (PB_WG - 1u)); c < cf1; c += PB_WG)
            pb_st16(gout + 16 * c, stage[c]);
        __syncthreads(); // the next window reuses the stage
        // the carried chunk is the next window's chunk 0: a header chunk there (ORed after that
        // window's payload barrier), never a payload chunk, so this plain write is its first
        if (cout && tid == (chc & (PB_WG - 1u)))
            stage[0] = cv;
    }
    if (tid == 0) // the workgroup stores exactly [lo, hi)
        pb_count(K, bxr, nown, hi_abs - lo_abs);
}

// ---------------- packed variable lengths, stores straight from registers: pb_vline_kernel ----------------
//
// configs[2].  pb_vstage_kernel assembles every window in an LDS stage between
// three barriers and spends ~200 VALU per (lane, frame) on setting up a group of lanes for each
// frame; here nothing is staged and the workgroup's waves never meet after the prologue:
//  * prologue (one lane per frame slot: up to PB_VST_GHOSTS earlier frames, then the own frames):
//    seed, fields, header image with both checksums — the L4 payload sum without the payload
//    bytes, from prefix sums over the LCG's orbit (pb_orbit_sum) — the start from a workgroup
//    scan, then per frame a 16-B record {start, end, LCG state at its first chunk} and its header
//    bytes already shifted to the frame's position in its first NSP 16-B chunks; a u16 map of the
//    region's 128-B lines to the frame holding each line's first byte;
//  * stream: the workgroup's byte region [lo, hi) (128-B aligned: no line has two writers) in
//    16-KiB steps, wave w writing bytes [4 KiB w, 4 KiB (w + 1)) of a step as four 1-KiB store
//    instructions (lane l: chunk l of each KiB).  Every chunk takes one straight-line path: the
//    line map gives the frame holding its first byte (and where the next frame starts in the
//    line), the frame's record its chunk index m and payload byte range, the L^(48 m) entry its
//    LCG state; 16 payload bytes are generated and blended under a byte mask with the frame's
//    shifted header image (header chunks) or the next frame's first header chunk (a frame edge).
// Every byte of [lo, hi) is stored exactly once, whole 16-B chunks only (the launch's last chunk
// zero-padded past the last frame).  Requires payloads of >= 32 bytes (a chunk then holds bytes
// of at most two frames, and never a payload end and the next header end).
// The L4 payload sum: payload byte j is bits 16-23 of M^(j+1)(st0), M = L^3 mod 2^24 (full
// period), so a payload is a run of consecutive orbit positions [p, p + n) of M, p = the discrete
// log of M(st0) (24 fixed steps, the PCG "distance" construction), and its word sum is a
// difference of prefix sums of the orbit's even- and odd-position bytes (K.orbit, every 32nd
// position: a 2-MiB table that stays in the XCD's L2, <= 31 LCG steps at each end; every 8th
// position, an 8-MiB table, read 7 GB per configs[2] launch through the fabric).

// discrete-log constants: M^(2^i) as (a_i, c_i) mod 2^24
constexpr uint32_t PB_M24 = 0xFFFFFFu;
constexpr uint32_t pb_orb_a(int i)
{
    uint32_t a = PB_A3 & PB_M24;
    for (int k = 0; k < i; ++k)
        a = (a * a) & PB_M24;
    return a;
}
constexpr uint32_t pb_orb_c(int i)
{
    uint32_t a = PB_A3 & PB_M24, c = PB_C3 & PB_M24;
    for (int k = 0; k < i; ++k)
    {
        c = ((a + 1u) * c) & PB_M24;
        a = (a * a) & PB_M24;
    }
    return c;
}

// M^-1 mod 2^24: y -> a^-1 (y - c)
constexpr uint32_t pb_inv24(uint32_t a)
{
    uint32_t x = a; // Newton: x = x (2 - a x), each step doubles the correct low bits (a odd)
    for (int i = 0; i < 5; ++i)
        x = x * (2u - a * x);
    return x & PB_M24;
}
constexpr uint32_t PB_A3I = pb_inv24(PB_A3 & PB_M24);
constexpr uint32_t PB_C3I = (0u - PB_A3I * (PB_C3 & PB_M24)) & PB_M24;
static_assert(((PB_A3I * (PB_A3 & PB_M24)) & PB_M24) == 1u, "M^-1");

// x * a (low 24 bits of each), one v_mul_u32_u24 with both operands in VGPRs
__device__ __forceinline__ uint32_t pb_mul24v(uint32_t x, uint32_t a)
{
    uint32_t r;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(x), "v"(a));
    return r;
}

// 0x01 in bytes [0, k) (k <= 4 taken as 4): a v_dot4_u32_u8 mask for the first k bytes
__device__ __forceinline__ uint32_t pb_ones_below(uint32_t k)
{
    return k >= 4u ? 0x01010101u : 0x01010101u & ((1u << (8u * k)) - 1u);
}

// Sums of the bytes (y_t >> 16) & 0xFF of the first dn (<= 16) states of the walk y_0 = y,
// y_(t+1) = a y_t + c (mod 2^24), split by the parity of t: returns the even-t sum, odd-t in *odd.
// Sixteen v_mad_u32_u24 (per-lane a and c: the walk runs forward or backward), the bytes packed
// four to a dword (pb_pack4) and summed under a prefix mask by v_dot4_u32_u8 (the former per-step
// compare / select / add chains compiled into v_mad_u64_u32, a quarter-rate instruction, per step)
__device__ __forceinline__ uint32_t pb_walk_sums(uint32_t y, uint32_t a, uint32_t c, uint32_t dn, uint32_t *odd)
{
    uint32_t x[16];
    x[0] = y;
#pragma unroll
    for (int t = 1; t < 16; ++t)
        x[t] = pb_mad24v(x[t - 1], a, c);
    const uint32_t e0 = pb_pack4(x[0], x[2], x[4], x[6]), e1 = pb_pack4(x[8], x[10], x[12], x[14]);
    const uint32_t o0 = pb_pack4(x[1], x[3], x[5], x[7]), o1 = pb_pack4(x[9], x[11], x[13], x[15]);
    const uint32_t ne = (dn + 1u) >> 1, no = dn >> 1; // walked even / odd positions
    const uint32_t se = __builtin_amdgcn_udot4(e1, pb_ones_below(ne > 4u ? ne - 4u : 0u),
                                               __builtin_amdgcn_udot4(e0, pb_ones_below(ne), 0u, false), false);
    *odd = __builtin_amdgcn_udot4(o1, pb_ones_below(no > 4u ? no - 4u : 0u),
                                  __builtin_amdgcn_udot4(o0, pb_ones_below(no), 0u, false), false);
    return se;
}

// Little-endian 16-bit word sum (mod 0xFFFF, in [1, 0xFFFF]) of the n >= 3 payload bytes drawn
// from the LCG state st0 entering the payload (sequence.c:552-555), payload at an even L4 offset:
// the value fold(sum of the bytes' words) takes (the orbit has no run of 3 zero bytes, so the true
// sum is never 0).  Every multiply is a full-rate 24-bit one (the states are taken mod 2^24).
__device__ __forceinline__ uint32_t pb_orbit_sum(const pb_kargs &K, uint32_t st0, uint32_t n)
{
    const uint32_t yp = pb_mad24(st0, PB_A3 & PB_M24, pb_vgpr(PB_C3)) & PB_M24; // the state of payload byte 0
    // bits 0-11 by table (K.dlog12: M mod 2^12 walks all 4096 residues from 0, so the position mod
    // 2^12 and the state there, cur = M^p(0) mod 2^24 whose low 12 bits are yp's, depend on yp mod
    // 2^12 alone; the former 12 conditional steps cost ~70 VALU per frame); bits 12-23 in closed
    // form: with N = M^4096 = (A, C), A = 1 + 2^14 u, C = 2^12 v (v odd), N^j(x) = x + j ((A - 1) x + C)
    // mod 2^24 (the dropped terms carry 2^26), so j = ((yp - cur) >> 12) / (((A - 1) >> 12) yp + v)
    // mod 2^12 (the divisor is odd)
    const uint32_t e12 = K.dlog12[yp & 0xFFFu];
    uint32_t p = e12 & 0xFFFu;
    const uint32_t cur = (e12 & 0xFFF000u) | (yp & 0xFFFu);
    {
        constexpr uint32_t A12 = pb_orb_a(12), C12 = pb_orb_c(12);
        static_assert(((A12 - 1u) & 0x3FFFu) == 0u && (C12 & 0x1FFFu) == 0x1000u, "M^4096 shape");
        const uint32_t w = pb_mad24(yp & 0xFFFu, (A12 - 1u) >> 12, pb_vgpr(C12 >> 12)) & 0xFFFu;
        uint32_t x = w; // w^-1 mod 2^12: correct to 3 bits, each Newton step doubles them
        x = pb_mul24v(x, (2u - pb_mul24v(w, x)) & 0xFFFu) & 0xFFFu;
        x = pb_mul24v(x, (2u - pb_mul24v(w, x)) & 0xFFFu) & 0xFFFu;
        const uint32_t j = pb_mul24v(((yp - cur) >> 12) & 0xFFFu, x) & 0xFFFu;
        p |= j << 12;
    }
    const uint2 jq = K.jump[n - 1 + PB_JNEG]; // L^(3n): the state one past the payload
    const uint32_t yq = pb_mad24v(yp, jq.x, jq.y) & PB_M24;
    uint32_t q = p + n, wrap = 0;
    if (q >= (1u << 24)) // the run wraps the orbit (2^24 is even: parities keep)
        q -= 1u << 24, wrap = K.orbit_tot;
    // prefix sums at p and q from the nearer sampled position (floor or ceil, <= 16 steps): walk the
    // bytes in between with M (forward, subtract) or M^-1 (backward, add); the walked bytes of
    // each parity are summed, the first walked position having parity par
    constexpr uint32_t SM = (1u << PB_ORB_SH) - 1u, HALF = (SM + 1u) >> 1;
    static_assert(HALF <= 16u, "pb_walk_sums walks at most 16 states");
    const bool fp = (p & SM) > HALF, fq = (q & SM) > HALF; // forward to the next sample
    const uint32_t ip = (p >> PB_ORB_SH) + (fp ? 1u : 0u), iq = (q >> PB_ORB_SH) + (fq ? 1u : 0u);
    const uint32_t tp = K.orbit[ip], tq = K.orbit[iq];
    const uint32_t dp = fp ? SM + 1u - (p & SM) : (p & SM), dq = fq ? SM + 1u - (q & SM) : (q & SM);
    const uint32_t ap_ = fp ? PB_A3 & PB_M24 : PB_A3I, cp_ = fp ? PB_C3 & PB_M24 : PB_C3I;
    const uint32_t aq_ = fq ? PB_A3 & PB_M24 : PB_A3I, cq_ = fq ? PB_C3 & PB_M24 : PB_C3I;
    const uint32_t y = fp ? yp : pb_mad24v(yp, pb_vgpr(PB_A3I), pb_vgpr(PB_C3I)); // backward: from position p - 1
    const uint32_t z = fq ? yq : pb_mad24v(yq, pb_vgpr(PB_A3I), pb_vgpr(PB_C3I));
    uint32_t ap1, aq1;
    const uint32_t ap0 = pb_walk_sums(y, ap_, cp_, dp, &ap1);
    const uint32_t aq0 = pb_walk_sums(z, aq_, cq_, dq, &aq1);
    // even / odd position sums of the walked bytes (the first walked position: p, or p - 1)
    const uint32_t pp = fp ? p & 1u : (p & 1u) ^ 1u, pq = fq ? q & 1u : (q & 1u) ^ 1u;
    const uint32_t sEp = pp ? ap1 : ap0, sOp = pp ? ap0 : ap1, sEq = pq ? aq1 : aq0, sOq = pq ? aq0 : aq1;
    // PE / PO at p and q, each in [0, 2 * 0xFFFF)
    const uint32_t PEp = fp ? (tp & 0xFFFFu) + 0xFFFFu - sEp : (tp & 0xFFFFu) + sEp;
    const uint32_t POp = fp ? (tp >> 16) + 0xFFFFu - sOp : (tp >> 16) + sOp;
    const uint32_t PEq = fq ? (tq & 0xFFFFu) + 0xFFFFu - sEq : (tq & 0xFFFFu) + sEq;
    const uint32_t POq = fq ? (tq >> 16) + 0xFFFFu - sOq : (tq >> 16) + sOq;
    const uint32_t de = PEq + wrap + 2u * 0xFFFFu - PEp;
    const uint32_t dO = POq + wrap + 2u * 0xFFFFu - POp;
    // payload byte j sits at orbit position p + j: even j is a word's low byte
    const uint32_t s = (p & 1u) ? dO + (de << 8) : de + (dO << 8);
    return pb_fold(s);
}

template <int HL, bool L4>
__global__ __launch_bounds__(PB_WG) void pb_vline_kernel(pb_kargs K)
{
    constexpr uint32_t GH = PB_VST_GHOSTS;
    constexpr uint32_t NSP = (15 + HL + 15) / 16; // chunks a frame's header can touch
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    const uint32_t WF = K.vl_wgf;
    const uint32_t CAP = WF + GH;
    uint2 *const s_jt = reinterpret_cast<uint2 *>(s_dyn);             // jump[PB_JNEG - (i + HL)], i < 16
    uint64_t *const s_st0 = reinterpret_cast<uint64_t *>(s_dyn + 32); // [0, GH]: slot starts - base0; [8, 12): S0 parts
    uint32_t *const s_wsum = s_dyn + 56;                              // per-wave length sums
    pb_u32x4 *const s_rec = reinterpret_cast<pb_u32x4 *>(s_dyn + 64); // {start, end, z, -} per frame slot
    pb_u32x4 *const s_img = s_rec + CAP;                              // NSP header chunks per frame slot
    pb_u32x4 *const s_m16 = s_img + CAP * NSP + 1;                    // after one zero chunk: byte masks
    uint2 *const s_l48 = reinterpret_cast<uint2 *>(s_m16 + PB_VL_NMASK);
    uint16_t *const s_map = reinterpret_cast<uint16_t *>(s_l48 + K.vl_nl48);

    const uint32_t tid = threadIdx.x;
    const uint32_t bxr = pb_xcd_region(blockIdx.x, gridDim.x); // XCD-contiguous regions
    const uint32_t flags = K.flags;
    const uint64_t f0 = (uint64_t)bxr * WF;
    const uint64_t left = K.n_frames - f0;
    const uint32_t nown = left < WF ? (uint32_t)left : WF;
    const uint64_t fe = f0 + nown;

    const uint32_t lane = tid & 63u, wv = tid >> 6;

    // ---------------- prologue: one lane per frame slot ----------------
    const int64_t fb = (int64_t)f0 - (int64_t)GH;
    uint64_t s0_part = 0;
    if (tid < (bxr & (PB_VL_GRP - 1u)))
        s0_part = K.vblk_sum[(bxr & ~(PB_VL_GRP - 1u)) + tid];
    const uint64_t s0_base = K.vblk_l2[bxr / PB_VL_GRP];
    uint2 jtv = make_uint2(0u, 0u);
    if (tid < 16u)
        jtv = K.jump[PB_JNEG - (tid + HL)];
    for (uint32_t i = tid; i < K.vl_nl48; i += PB_WG)
        s_l48[i] = K.lcg48[i];
    const uint2 rg1 = (flags & PBK_RND_SADDR) ? K.ranges[0] : make_uint2(0u, 0u);
    const int64_t fj = fb + (int64_t)tid;
    const bool valid = tid < CAP && fj >= 0 && (uint64_t)fj < fe;
    uint32_t flen = 0, st0 = 0;
    uint32_t d[16];
#pragma unroll
    for (int w = 0; w < 16; ++w)
        d[w] = 0u;
    uint32_t csum_v = 0; // the L4 checksum field, ORed into d[] after the scan
    if (valid)
    {
        uint64_t k;
        uint32_t pi;
        pb_frame_index(K, (uint64_t)fj, k, pi);
        const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + k);
        const uint32_t r0 = pb_rand_r(s);
        const pb_frame_pl P = pb_payload<false>(K, s, pi);
        const uint32_t l4tot = pb_header(K, r0, P.plen, d, K.rng.d == 1 ? rg1 : pb_range(K, r0));
        flen = HL + P.plen;
        st0 = P.st0;
        if (L4)
        {
            // csum_tcpudp_magic / icmp_csum (sequence.c:569-594): header (+ pseudo header) words
            // plus the payload's, from the orbit prefix sums
            uint32_t hs = (d[8] >> 16) + pb_halves(d[9]) + pb_halves(d[10]) + pb_halves(d[11]) + pb_halves(d[12]) +
                          pb_halves(d[13]);
            if (flags & PBK_PSEUDO)
                hs += (d[6] >> 16) + pb_halves(d[7]) + (d[8] & 0xFFFFu) + ((K.proto + l4tot) << 8);
            const uint32_t ps = pb_orbit_sum(K, P.st0, P.plen);
            const uint32_t c = (~pb_fold(pb_fold(hs) + ps)) & 0xFFFFu;
            csum_v = K.csum_hi ? (c << 16) : c;
        }
    }
    // frame starts: exclusive scan of the slot lengths (in-wave shuffles, wave totals via LDS)
    uint32_t inc = flen;
#pragma unroll
    for (uint32_t dd = 1; dd < 64; dd <<= 1)
    {
        const uint32_t y = __shfl_up(inc, dd, 64);
        inc += lane >= dd ? y : 0u;
    }
#pragma unroll
    for (uint32_t dd = 32; dd > 0; dd >>= 1)
        s0_part += __shfl_xor(s0_part, dd, 64);
    if (lane == 63u)
        s_wsum[wv] = inc;
    if (lane == 0u)
        s_st0[8 + wv] = s0_part;
    if (tid <= GH)
        s_st0[tid] = inc - flen;
    if (tid < 16u)
        s_jt[tid] = jtv;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < PB_WG / 64; ++w)
    {
        const uint32_t t = s_wsum[w];
        pre += w < wv ? t : 0u;
        tot += t;
    }
    uint64_t S0 = s0_base;
#pragma unroll
    for (uint32_t w = 0; w < PB_WG / 64; ++w)
        S0 += s_st0[8 + w];
    const uint64_t base0 = S0 - s_st0[GH]; // start of slot 0
    const uint64_t start = base0 + pre + (inc - flen);
    if (valid && tid >= GH) // own frames: the offsets' low words, the region's start
    {
        K.offsets32[(uint64_t)fj] = (uint32_t)start;
        if (tid == GH)
            K.vl_rstart[bxr] = start;
    }
    // region [lo, hi): lo = the 128-B line of the first own frame's start (0 for the first region),
    // hi = the next region's lo (the launch's end for the last)
    const bool last = fe == K.n_frames;
    const uint64_t lo_abs = bxr ? (S0 & ~127ull) : 0ull;
    const uint64_t hi_abs = last ? base0 + tot : ((base0 + tot) & ~127ull);
    // ghosts: the frames before f0 that end past lo (a prefix f0 - 1, f0 - 2, ...)
    uint32_t ng = 0;
    if (bxr)
        while (ng < GH && f0 > ng && base0 + s_st0[GH - ng] > lo_abs)
            ++ng;
    const uint32_t nfr = ng + nown; // frames with records: slot index t = tid - (GH - ng)
    const uint64_t wbase = (base0 + s_st0[GH - ng]) & ~15ull;
    const uint32_t lo_rel = (uint32_t)(lo_abs - wbase), hi_rel = (uint32_t)(hi_abs - wbase);
    const int32_t tix = (int32_t)tid - (int32_t)(GH - ng);
    if (valid && tix >= 0)
    {
        // the checksum only now: the orbit-table loads behind it (issued in the frame's field
        // computation) complete under the scan and the barrier instead of before them
#pragma unroll
        for (uint32_t w = 0; w < 16; ++w)
            d[w] |= w == K.csum_dw ? csum_v : 0u;
        const uint32_t r = (uint32_t)(start - wbase);
        const uint32_t s0 = r & 15u;
        const uint2 jt = s_jt[s0];
        // payload start and end in 1/16 B (the chunk masks are then indexed without shifts)
        s_rec[tix] = pb_u32x4{r >> 4, (r + HL) << 4, (r + flen) << 4, jt.x * st0 + jt.y};
        // the header image shifted to byte s0 of the frame's first chunk: out dword u holds image
        // bytes [4u - s0, 4u - s0 + 4)
        const uint32_t q = s0 >> 2, sh = s0 & 3u;
        uint32_t v[17];
#pragma unroll
        for (int u = 0; u < 17; ++u)
        {
            const uint32_t lo = u > 0 ? d[u - 1] : 0u, hi = u < 16 ? d[u] : 0u;
            v[u] = sh ? __builtin_amdgcn_alignbyte(hi, lo, 4u - sh) : hi;
        }
        // only the header bytes [s0, s0 + HL) of the image chunks are ever read (bytes before s0
        // belong to the previous frame's chunk and take its payload, bytes after the header this
        // frame's payload): NHW dwords from dword q, inside the frame's own NSP chunks
        constexpr uint32_t NHW = (HL + 6) / 4;
        static_assert(3 + NHW <= 4 * NSP, "image slot");
        uint32_t *const img32 = reinterpret_cast<uint32_t *>(s_img + (uint32_t)tix * NSP) + q;
#pragma unroll
        for (uint32_t u = 0; u < NHW; ++u)
            img32[u] = v[u];
    }
    __syncthreads();

    // line map
    const uint32_t R = hi_rel - lo_rel;
    const uint32_t nlines = (R + 127u) >> 7;
    if ((uint32_t)tix < nfr && tix >= 0)
    {
        const pb_u32x4 rc = s_rec[tix];
        // lines whose first byte lies in this frame: the frame holding it, and where (if at all)
        // the next frame starts in the line
        const uint32_t st = (rc[1] >> 4) - HL, end = rc[2] >> 4;
        const uint32_t a = st > lo_rel ? st - lo_rel : 0u, b = end > lo_rel ? end - lo_rel : 0u;
        const uint32_t la = (a + 127u) >> 7, lb = min((b + 127u) >> 7, nlines);
        // the next two frames' starts in the line as 16-B chunk positions c = ceil(o / 16) (1..8,
        // 8: none), kept as 8 - c in bits 0-2 and 4-6: chunk k of the line lies in frame
        // tix + (k >= c1) + (k >= c2), and k >= c <=> k + (8 - c) carries into bit 3 / 7
        const uint32_t b2 = (uint32_t)tix + 1u < nfr ? (s_rec[tix + 1][2] >> 4) - lo_rel : 0xFFFFFFFFu;
        // only the frame's last line can hold the next frame starts (o1, o2 >= 128 before it)
        for (uint32_t L = la; L + 1u < lb; ++L)
            s_map[L] = (uint16_t)((uint32_t)tix << 8);
        if (la < lb)
        {
            const uint32_t L = lb - 1u;
            const uint32_t o1 = b - (L << 7), o2 = b2 - (L << 7);
            const uint32_t c1 = o1 < 128u ? (o1 + 15u) >> 4 : 8u, c2 = o2 < 128u ? (o2 + 15u) >> 4 : 8u;
            s_map[L] = (uint16_t)(((uint32_t)tix << 8) | (8u - c1) | ((8u - c2) << 4));
        }
    }
    // chunk byte masks, indexed by plo + phi: a chunk holds a payload start (plo > 0, phi = 16) or
    // a payload end (plo = 0, phi < 16) or neither (payloads of >= 32 B), so s_m16[j] keeps bytes
    // < j for j <= 16 and bytes >= j - 16 above
    if (tid <= 32u)
    {
        const int lo = tid > 16u ? (int)tid - 16 : 0, hi = tid > 16u ? 16 : (int)tid;
        s_m16[tid] = pb_u32x4{pb_range_mask(lo, hi), pb_range_mask(lo - 4, hi - 4), pb_range_mask(lo - 8, hi - 8),
                              pb_range_mask(lo - 12, hi - 12)};
    }
    if (tid == 64u) // the header chunk after the last record's: no frame starts there
        s_img[nfr * NSP] = pb_u32x4{0u, 0u, 0u, 0u};
    __syncthreads();

    // ---------------- stream: the region in 16-KiB steps, no barriers ----------------
    // Chunk ci (16-B units from wbase) of line l: frame f holds its first byte, and its bytes are
    // f's payload bytes in [plo, phi) (one generated chunk, masked) and header bytes elsewhere:
    // f's own (chunk m < NSP of f: the shifted image, bytes < plo) or the next frame's, which
    // starts inside the chunk when phi < 16 (then m >= NSP, and image slot f * NSP + NSP is the
    // next frame's first chunk, bytes >= phi; for a chunk with neither both masks are empty).
    // One straight-line path per chunk, and every 128-B line leaves in one store instruction.
    uint8_t *const gout = K.out + wbase + lo_rel;
    const uint32_t nsteps = (R + PB_VL_STEP - 1u) / PB_VL_STEP;
    const uint32_t k = lane & 7u, kk = k | (k << 4), ck = (lo_rel >> 4) + k;
    const uint32_t lmax = nlines ? nlines - 1u : 0u;
    // chunk i of step s; clamp: lines past the region's end are computed on its last line
    auto chunk = [&](uint32_t s, uint32_t i, bool clamp) -> pb_u32x4 {
        uint32_t l = s * (PB_VL_STEP / 128u) + (wv << 5) + (i << 3) + (lane >> 3);
        if (clamp)
            l = min(l, lmax);
        const uint32_t ci = (l << 3) + ck;
        const uint32_t t = (uint32_t)s_map[l] + kk;
        const uint32_t f = (t >> 8) + __popc(t & 0x88u);
        const pb_u32x4 rc = s_rec[f];
        const uint32_t m = pb_subv(ci, rc[0]); // chunk index within frame f
        const uint2 L = s_l48[m];
        const uint32_t x = __umul24(rc[3], L.x) + L.y;
        // payload bytes [plo, phi) of the chunk, in 1/16 B: 16 plo + 16 phi is s_m16's byte offset
        const uint32_t plo16 = (uint32_t)min(max(pb_msub256(ci, rc[1]), 0), 256);
        const uint32_t phi16 = (uint32_t)min(max(pb_msub256(ci, rc[2]), 0), 256);
        const pb_u32x4 h = s_img[NSP == 4 ? pb_lshl_add<2>(f, min(m, NSP)) : f * NSP + min(m, NSP)];
        uint32_t o0, o1, o2, o3;
        pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
        const pb_u32x4 mm = *reinterpret_cast<const pb_u32x4 *>(reinterpret_cast<const uint8_t *>(s_m16) + plo16 + phi16);
        const uint32_t M0 = mm[0], M1 = mm[1], M2 = mm[2], M3 = mm[3];
        return pb_u32x4{(o0 & M0) | (h[0] & ~M0), (o1 & M1) | (h[1] & ~M1), (o2 & M2) | (h[2] & ~M2),
                        (o3 & M3) | (h[3] & ~M3)};
    };
    // steps that lie wholly inside the region: no clamp, no store guard (their four chunks' LCG
    // chains interleave instead of each running inside its own store branch)
    const uint32_t nfull = min(nsteps, R / PB_VL_STEP);
    for (uint32_t s = 0; s < nfull; ++s)
    {
        pb_u32x4 v[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
            v[i] = chunk(s, i, false);
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
            pb_st16_nt(gout + s * PB_VL_STEP + (wv << 12) + (i << 10) + (lane << 4), v[i]);
    }
    for (uint32_t s = nfull; s < nsteps; ++s)
    {
        // four independent chunks per lane, computed before any is stored
        pb_u32x4 v[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
            v[i] = chunk(s, i, true);
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
        {
            const uint32_t c0 = s * PB_VL_STEP + (wv << 12) + (i << 10) + (lane << 4);
            if (c0 < R)
                pb_st16_nt(gout + c0, v[i]);
        }
    }
    if (tid == 0) // the workgroup stores exactly [lo, hi) (the launch's last chunk zero-padded)
        pb_count(K, bxr, nown, hi_abs - lo_abs);
}

// ---------------- packed variable lengths as XCD-owned 4-KiB pages: pb_vrec_kernel + pb_vpage_kernel ----------------
//
// configs[2] in the page kernels' store shape: workgroup b's wave w owns page
// ((b / 8) 4 + w) 8 + b % 8 of the packed stream, so every XCD writes one residue class of pages
// inside one moving window and each wave retires after one page: the only store shape measured
// immune to the buffer placement that slows the region writers (pb_vline_kernel 4.9 vs 4.2 ms).
// A page finds its frames through two arrays written by the record pass, one lane per frame:
//   rec[f] = {seed, L4 checksum | length << 16}   (8 B per frame; the L4 sum by pb_orbit_sum)
//   pt[c]  = {the frame holding page c's first byte, its start - 4096 c}
// so the page kernel's per-frame work is the header image from the seed and a length scan.

// inclusive add scan over the wave's 64 lanes (DPP: row shifts, then row broadcasts)
__device__ __forceinline__ uint32_t pb_wave_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true); // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true); // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true); // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true); // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false); // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false); // row_bcast:31 -> rows 2, 3
    return v;
}

// Record pass: workgroup b takes frames [256 b, 256 b + 256) (the length pass ran at 256 frames per
// workgroup), one lane per frame: seed -> r0 -> length, header fields and the L4 checksum
// (sequence.c:434-594, as pb_vline_kernel's prologue), the start from the group sums and a
// workgroup scan; writes the frame's 4-B offset, rec[f] and, if the frame holds a page's first byte,
// pt[page].  The block sums' loads are issued first and read last.
template <int HL, bool L4>
__global__ __launch_bounds__(PB_WG) void pb_vrec_kernel(pb_kargs K)
{
    __shared__ uint32_t s_wsum[PB_WG / 64];
    __shared__ unsigned long long s_part;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint64_t f = (uint64_t)b * PB_WG + tid;
    const bool valid = f < K.n_frames;
    // the group sums before this workgroup's (PB_VL_GRP workgroups per group)
    unsigned long long part = 0;
    if (wv == 0 && lane < (b & (PB_VL_GRP - 1u)))
        part = K.vblk_sum[(b & ~(PB_VL_GRP - 1u)) + lane];
    const unsigned long long base_l2 = K.vblk_l2[b / PB_VL_GRP];
    uint32_t flen = 0, s = 0, csum = 0;
    if (valid)
    {
        s = pb_seed(K.seed_base, K.seq, K.first_iter + f);
        const uint32_t r0 = pb_rand_r(s);
        const pb_frame_pl P = pb_payload_of(K.pl0, s, K.flags);
        flen = HL + P.plen;
        if (L4)
        {
            uint32_t d[16];
            const uint2 rg1 = (K.flags & PBK_RND_SADDR) ? K.ranges[0] : make_uint2(0u, 0u);
            const uint32_t l4tot = pb_header(K, r0, P.plen, d, K.rng.d == 1 ? rg1 : pb_range(K, r0));
            uint32_t hs = (d[8] >> 16) + pb_halves(d[9]) + pb_halves(d[10]) + pb_halves(d[11]) + pb_halves(d[12]) +
                          pb_halves(d[13]);
            if (K.flags & PBK_PSEUDO)
                hs += (d[6] >> 16) + pb_halves(d[7]) + (d[8] & 0xFFFFu) + ((K.proto + l4tot) << 8);
            const uint32_t ps = pb_orbit_sum(K, P.st0, P.plen);
            csum = (~pb_fold(pb_fold(hs) + ps)) & 0xFFFFu;
        }
    }
    const uint32_t inc = pb_wave_scan(flen);
    if (wv == 0)
    {
#pragma unroll
        for (uint32_t dd = 32; dd > 0; dd >>= 1)
            part += __shfl_xor(part, dd, 64);
        if (lane == 0)
            s_part = part;
    }
    if (lane == 63u)
        s_wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (uint32_t w = 0; w < PB_WG / 64; ++w)
        pre += w < wv ? s_wsum[w] : 0u;
    const uint64_t start = base_l2 + s_part + pre + inc - flen;
    if (valid)
    {
        K.offsets32[f] = (uint32_t)start;
        if (tid == 0)
            K.vl_rstart[b] = start;
        K.vp_rec[f] = make_uint2(s, csum | (flen << 16));
        const uint64_t pg = (start + 4095u) >> 12;
        if ((pg << 12) < start + flen)
            K.vp_pt[pg] = make_uint2((uint32_t)f, (uint32_t)(start - (pg << 12)));
    }
}

// Page kernel: wave w of workgroup b builds page c (above) of the stream whose length the length
// pass's scan left in offsets_w[n_frames]:
//  * its pt entry (a scalar load) and the records of up to 64 frames from there; a length scan
//    gives each frame's page-relative start; the nf frames that start before the page's end are
//    its slots (nf <= vp_nfp);
//  * one lane per slot: r0 and the header image from the seed, the L4 checksum from the record,
//    a 16-B record {first chunk, payload start, end, LCG state at page chunk 0} and the image
//    shifted to the frame's byte offset (pb_vline_kernel's layout), and a mark at the first chunk
//    whose first byte is the frame's;
//  * lane l builds chunks l, l + 64, l + 128, l + 192 of the page: its frame is the count of marks
//    at or below the chunk (ballot + mbcnt, no map), its LCG state L^(48 ci) of the frame's state
//    at chunk 0 (per-lane constants), 16 payload bytes blended with the header image under the
//    payload's byte mask; four 1-KiB store instructions (the stream's last chunk zero-padded).
// Each workgroup's count record is {frames starting in its pages, their page bytes}; pages past the
// stream (the grid covers the longest possible one) record zeros.
// (Measured and removed, round 6: 512-thread workgroups of 8 pages, 7.24 vs 6.89 ms; the four
// pages' frame setup pooled into wave 0 before a workgroup barrier, 7.59 vs 6.93 ms, commit
// "Pooled-setup page kernel"; profiles/r06/vpage/.)
template <int HL, bool L4>
__global__ __launch_bounds__(PB_WG) void pb_vpage_kernel(pb_kargs K)
{
    constexpr uint32_t NW = PB_WG / 64; // pages (waves) per workgroup
    constexpr uint32_t NSP = (15 + HL + 15) / 16; // chunks a frame's header can touch
    constexpr uint32_t NHW = (HL + 6) / 4;       // image dwords written (pb_vline_kernel)
    static_assert(3 + NHW <= 4 * NSP, "image slot");
    extern __shared__ __attribute__((aligned(16))) uint32_t s_dyn[];
    const uint32_t NFP = K.vp_nfp;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    pb_u32x4 *const s_m16 = reinterpret_cast<pb_u32x4 *>(s_dyn);
    uint2 *const s_cnt = reinterpret_cast<uint2 *>(s_m16 + PB_VL_NMASK);
    uint8_t *const wb = reinterpret_cast<uint8_t *>(s_cnt + NW) + wv * PB_VP_WAVE_LDS(NFP, NSP);
    pb_u32x4 *const s_rec = reinterpret_cast<pb_u32x4 *>(wb);
    pb_u32x4 *const s_img = s_rec + NFP;
    uint32_t *const s_mark = reinterpret_cast<uint32_t *>(s_img + NFP * NSP + 1);

    const uint32_t b = blockIdx.x;
    const uint32_t c0 = __builtin_amdgcn_readfirstlane(((b >> 3) * NW + wv) * 8u + (b & 7u));
    // every load that does not wait for the page's records is issued here, together: the
    // stream's length and the page's pt entry (scalar; the grid's pages all have an entry, pages
    // past the stream a stale one that is not used), the lane's chunk states L^(48 ci),
    // ci = PB_VP_BIAS / 16 + 64 i + lane, and three 16 / 16 / 32-entry maps held one per lane for
    // the frames' states (read by lane shuffles): lanes 0-15 L^(3 (1 - s0 - HL)) (payload byte 0
    // at chunk byte s0 + HL), 16-31 L^(-48 j), 32-63 L^(-768 h)
    const uint64_t total = K.offsets_w[K.n_frames];
    uint2 e = K.vp_pt[c0];
    uint2 lc[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i)
        lc[i] = K.lcg48[PB_VP_BIAS / 16u + 64u * i + lane];
    const uint2 tm = lane < 16u ? K.jump[PB_JNEG - (lane + HL)] : K.lcg48i[lane < 32u ? lane - 16u : (lane - 32u) << 4];
    const uint2 rg1 = (K.flags & PBK_RND_SADDR) ? K.ranges[0] : make_uint2(0u, 0u); // one range: uniform
    // chunk byte masks by plo + phi, from the context's table (every wave writes the same rows)
    uint4 m16row = make_uint4(0u, 0u, 0u, 0u);
    if (lane < PB_VL_NMASK)
        m16row = K.m16[lane];
    uint32_t frames = 0, bytes = 0;
    // the grid is sized for the expected stream (pbgpu.cpp); a longer one is taken by later rounds
    // of the same waves (their pages keep the XCD: the stride is a multiple of 8 pages)
    for (uint64_t c = c0; (c << 12) < total; c += (uint64_t)NW * gridDim.x)
    {
        if (c != c0)
        {
            e = K.vp_pt[c];
            // the previous page's LDS reads before this page's writes
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const uint64_t f = (uint64_t)e.x + lane;
        const bool fv = f < K.n_frames;
        const uint2 r = fv ? K.vp_rec[f] : make_uint2(0u, 0u);
        const uint32_t fl = r.y >> 16;
        const int32_t st = (int32_t)e.y + (int32_t)(pb_wave_scan(fl) - fl); // page-relative start
        const bool inp = fv && st < 4096;
        const uint32_t nf = (uint32_t)__popcll(__ballot(inp)); // slots 0 .. nf - 1
        const int32_t end_last = __shfl(st + (int32_t)fl, (int)nf - 1, 64);
        const uint32_t pbytes = (uint32_t)min(end_last, 4096);
        bytes += pbytes;
        frames += nf - ((int32_t)e.y < 0 ? 1u : 0u);
        s_mark[lane] = 0u;
        if (lane < PB_VL_NMASK)
            s_m16[lane] = pb_u32x4{m16row.x, m16row.y, m16row.z, m16row.w};
        // the frame's three state maps, read from the lanes holding them (every lane takes part:
        // a shuffle reads no lane that is switched off)
        const uint32_t u = (uint32_t)(st + (int32_t)PB_VP_BIAS);
        const uint32_t s0 = u & 15u, cs = u >> 4;
        const uint32_t l1 = s0 << 2, l2 = (16u + (cs & 15u)) << 2, l3 = (32u + ((cs >> 4) & 31u)) << 2;
        const uint32_t m1a = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l1, (int)tm.x);
        const uint32_t m1c = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l1, (int)tm.y);
        const uint32_t m2a = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l2, (int)tm.x);
        const uint32_t m2c = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l2, (int)tm.y);
        const uint32_t m3a = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l3, (int)tm.x);
        const uint32_t m3c = (uint32_t)__builtin_amdgcn_ds_bpermute((int)l3, (int)tm.y);
        uint32_t k0 = 256u;
        if (inp)
        {
            const uint32_t s = r.x;
            const uint32_t r0 = pb_rand_r(s);
            uint32_t d[16];
            (void)pb_header(K, r0, fl - HL, d, K.rng.d == 1 ? rg1 : pb_range(K, r0));
            // the LCG state at the frame's first chunk (payload byte j at chunk byte s0 + HL + j),
            // taken back to page chunk 0 by L^(-48 cs) = L^(-48 (cs % 16)) L^(-768 (cs / 16))
            const uint32_t z = pb_mad24v(pb_mad24v(pb_mad24v(s, m1a, m1c), m2a, m2c), m3a, m3c);
            s_rec[lane] = pb_u32x4{cs, u + HL, u + fl, z};
            const uint32_t q = s0 >> 2, sh = s0 & 3u;
            uint32_t *const img32 = reinterpret_cast<uint32_t *>(s_img + lane * NSP) + q;
#pragma unroll
            for (uint32_t w = 0; w < NHW; ++w)
            {
                const uint32_t lo = w > 0 ? d[w - 1] : 0u, hi = d[w];
                img32[w] = sh ? __builtin_amdgcn_alignbyte(hi, lo, 4u - sh) : hi;
            }
            if (L4) // the L4 checksum's two bytes over the image's zeros (its position is the sequence's)
            {
                uint8_t *const cb = reinterpret_cast<uint8_t *>(s_img + lane * NSP) + s0 + 4u * K.csum_dw + 2u * K.csum_hi;
                cb[0] = (uint8_t)r.y;
                cb[1] = (uint8_t)(r.y >> 8);
            }
            k0 = st <= 0 ? 0u : ((uint32_t)st + 15u) >> 4;
        }
        if (lane == nf) // the chunk after the last slot's: no frame starts there
            s_img[nf * NSP] = pb_u32x4{0u, 0u, 0u, 0u};
        // the marks' zeroing before the marks (a wave's LDS operations complete in order)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (k0 < 256u) // chunk k's mark: byte k / 64 of dword k % 64
            reinterpret_cast<uint8_t *>(s_mark)[((k0 & 63u) << 2) + (k0 >> 6)] = 1u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t mk = s_mark[lane];
        const uint32_t nch = (pbytes + 15u) >> 4;
        uint8_t *const gout = K.out + ((uint64_t)c << 12) + (lane << 4);
        uint32_t pre = 0; // marks in the earlier 64-chunk quarters
        pb_u32x4 v[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
        {
            const uint64_t B = __ballot(((mk >> (8u * i)) & 0xFFu) != 0u);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(B >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)B, 0u));
            const uint32_t fi = pre + below + (uint32_t)((B >> lane) & 1u) - 1u;
            pre += (uint32_t)__popcll(B);
            const pb_u32x4 rc = s_rec[fi];
            const uint32_t ci = PB_VP_BIAS / 16u + 64u * i + lane;
            const uint32_t m = ci - rc[0]; // chunk index within frame fi
            const uint32_t x = pb_mad24v(rc[3], lc[i].x, lc[i].y);
            const int32_t pb = (int32_t)(ci << 4);
            const uint32_t plo = (uint32_t)min(max((int32_t)rc[1] - pb, 0), 16);
            const uint32_t phi = (uint32_t)min(max((int32_t)rc[2] - pb, 0), 16);
            const pb_u32x4 h = s_img[fi * NSP + min(m, NSP)];
            uint32_t o0, o1, o2, o3;
            pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
            const pb_u32x4 mm = s_m16[plo + phi];
            v[i] = pb_u32x4{(o0 & mm[0]) | (h[0] & ~mm[0]), (o1 & mm[1]) | (h[1] & ~mm[1]),
                            (o2 & mm[2]) | (h[2] & ~mm[2]), (o3 & mm[3]) | (h[3] & ~mm[3])};
        }
        if (nch == 256u)
        {
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i)
                pb_st16_nt(gout + (i << 10), v[i]);
        }
        else
        {
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i)
                if (64u * i + lane < nch)
                    pb_st16_nt(gout + (i << 10), v[i]);
        }
    }
    if (lane == 0)
        s_cnt[wv] = make_uint2(frames, bytes);
    __syncthreads();
    if (threadIdx.x == 0)
    {
        uint32_t fr = 0, by = 0;
#pragma unroll
        for (uint32_t w = 0; w < NW; ++w)
            fr += s_cnt[w].x, by += s_cnt[w].y;
        pb_count_at(K, b, pb_xcd_region(b, gridDim.x), fr, by);
    }
}

// ---------------- variable length: lengths -> offsets -> tile map ----------------

__global__ __launch_bounds__(256) void pb_len_reduce(pb_kargs K, unsigned long long *block_sums)
{
    __shared__ unsigned long long s_part[256];
    const uint64_t base = (uint64_t)blockIdx.x * 256 * PB_SCAN_ITEMS + (uint64_t)threadIdx.x * PB_SCAN_ITEMS;
    unsigned long long sum = 0;
    for (int it = 0; it < PB_SCAN_ITEMS; ++it)
    {
        const uint64_t f = base + it;
        if (f < K.n_frames)
            sum += pb_frame_len(K, f);
    }
    s_part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t w = 128; w > 0; w >>= 1)
    {
        if (threadIdx.x < w)
            s_part[threadIdx.x] += s_part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0)
        block_sums[blockIdx.x] = s_part[0];
}

// single workgroup: exclusive scan of the block sums in place, in passes of 8192 entries: coalesced
// loads into LDS (one pad word per 8 entries), 8 consecutive entries per lane, one shuffle scan per
// wave, the wave sums through LDS, coalesced stores.  A pass waits on its loads' latency (the sums
// were written by every XCD), so the passes are few: the length pass's group sums are
// 2^25 / 252 / PB_VL_GRP = 4,161 entries at configs[2]'s size, one pass.  (Strided per-lane loads or
// a chain of 64-bit row scans took 12-20 us for 8,322 entries, 4-entry passes 14 us.)
__global__ __launch_bounds__(1024) void pb_scan_blocks(unsigned long long *block_sums, uint32_t nblocks,
                                                       uint64_t *offsets, uint64_t n_frames)
{
    constexpr uint32_t IT = 8, PASS = 1024 * IT;
    __shared__ unsigned long long s_v[PASS + PASS / 8];
    __shared__ unsigned long long s_w[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    unsigned long long carry = 0;
    for (uint32_t base = 0; base < nblocks; base += PASS)
    {
        const uint32_t n = nblocks - base < PASS ? nblocks - base : PASS;
#pragma unroll
        for (uint32_t k = 0; k < IT; ++k)
        {
            const uint32_t i = k * 1024 + tid;
            s_v[i + (i >> 3)] = i < n ? block_sums[base + i] : 0ull;
        }
        __syncthreads();
        const uint32_t p0 = tid * (IT + 1); // IT consecutive entries, no pad among them
        unsigned long long v[IT], t = 0;
#pragma unroll
        for (uint32_t k = 0; k < IT; ++k)
        {
            v[k] = s_v[p0 + k];
            t += v[k];
        }
        unsigned long long x = t; // inclusive scan of the lanes' sums within the wave
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1)
        {
            const unsigned long long y = __shfl_up(x, d, 64);
            if (lane >= d)
                x += y;
        }
        if (lane == 63u)
            s_w[w] = x;
        __syncthreads();
        unsigned long long wpre = 0, tot = 0;
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j)
        {
            const unsigned long long sj = s_w[j];
            wpre += j < w ? sj : 0ull;
            tot += sj;
        }
        unsigned long long run = carry + wpre + x - t;
#pragma unroll
        for (uint32_t k = 0; k < IT; ++k)
        {
            s_v[p0 + k] = run;
            run += v[k];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < IT; ++k)
        {
            const uint32_t i = k * 1024 + tid;
            if (i < n)
                block_sums[base + i] = s_v[i + (i >> 3)];
        }
        carry += tot;
        __syncthreads(); // s_v and s_w are rewritten by the next pass
    }
    if (tid == 0)
        offsets[n_frames] = carry; // (the build kernels count frames and bytes as they store them)
}

__global__ __launch_bounds__(256) void pb_len_scan(pb_kargs K, const unsigned long long *block_sums,
                                                   uint64_t *offsets)
{
    __shared__ unsigned long long s_v[256];
    const uint64_t base = (uint64_t)blockIdx.x * 256 * PB_SCAN_ITEMS + (uint64_t)threadIdx.x * PB_SCAN_ITEMS;
    uint32_t len[PB_SCAN_ITEMS];
    unsigned long long sum = 0;
#pragma unroll
    for (int it = 0; it < PB_SCAN_ITEMS; ++it)
    {
        const uint64_t f = base + it;
        len[it] = f < K.n_frames ? pb_frame_len(K, f) : 0u;
        sum += len[it];
    }
    s_v[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1)
    {
        const unsigned long long t = threadIdx.x >= d ? s_v[threadIdx.x - d] : 0ull;
        __syncthreads();
        s_v[threadIdx.x] += t;
        __syncthreads();
    }
    unsigned long long off = block_sums[blockIdx.x] + s_v[threadIdx.x] - sum;
#pragma unroll
    for (int it = 0; it < PB_SCAN_ITEMS; ++it)
    {
        const uint64_t f = base + it;
        if (f < K.n_frames)
        {
            offsets[f] = off;
            off += len[it];
        }
    }
}

// ---------------- UMEM landing (variable length) and roofline probe ----------------

// frame first + blockIdx.x -> dst + slot * stride (mapped host memory or device)
__global__ __launch_bounds__(64) void pb_scatter_slots(const uint8_t *src, const uint64_t *offsets, uint64_t first,
                                                       uint8_t *dst, uint32_t stride, uint16_t *lens)
{
    const uint64_t f = first + blockIdx.x;
    const uint64_t o = offsets[f];
    const uint32_t len = (uint32_t)(offsets[f + 1] - o);
    if (threadIdx.x == 0)
        lens[blockIdx.x] = (uint16_t)len;
    const uint8_t *s = src + o;
    uint32_t *d = reinterpret_cast<uint32_t *>(dst + (uint64_t)blockIdx.x * stride);
    const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)s & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)((uintptr_t)s & 3);
    // whole dwords, then the frame's last 1-3 bytes one by one: nothing is
    // written past the frame's own bytes in its slot
    for (uint32_t i = threadIdx.x; i * 4 + 4 <= len; i += 64)
        d[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
    const uint32_t tail = len & 3u, i = len >> 2;
    if (threadIdx.x < tail)
        reinterpret_cast<uint8_t *>(d + i)[threadIdx.x] = s[4 * i + threadIdx.x];
}

// fixed-length frames -> slots: thread (f, i) stores dword i of slot f (f = gid / dpf) at
// dst + f * stride; straight over the host link when dst is mapped UMEM (af_xdp.c:211-214
// geometry: one frame per 4 KiB slot).  wlen bytes of each slot are written: the frame's flen,
// or the whole slot (wlen = stride, a multiple of 4) when the slot is tight, the frame's bytes
// followed by the packed stream's next ones (zeros past src_lim, the source bytes readable):
// contiguous slots then leave as contiguous host-link writes
__global__ __launch_bounds__(256) void pb_scatter_fixed(const uint8_t *src, uint32_t flen, uint32_t wlen, uint32_t dpf,
                                                        uint64_t n_dw, uint64_t src_lim, uint8_t *dst, uint32_t stride)
{
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= n_dw)
        return;
    const uint64_t f = g / dpf;
    const uint32_t i = (uint32_t)(g - f * dpf);
    const uint64_t o = f * flen + 4 * i;
    const uint8_t *s = src + o;
    const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)s & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)((uintptr_t)s & 3);
    // the frame's own dwords read at most 3 bytes past it (inside the buffer's 16-B tail pad);
    // a filler dword is read only while the stream has the bytes
    const bool rd = 4 * i < flen || o + 8 <= src_lim;
    const uint32_t v = rd ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : 0u;
    uint8_t *d = dst + f * stride + 4 * i;
    if (4 * i + 4 <= wlen)
        *reinterpret_cast<uint32_t *>(d) = v;
    else
        for (uint32_t b = 0; 4 * i + b < wlen; ++b)
            d[b] = (uint8_t)(v >> (8 * b));
}

// write-only roofline probe: each workgroup streams PER contiguous 4-KiB sweeps
// of 16-B stores (PER = 4: the linear build kernels' shape; PER = 1: 4 KiB per
// workgroup, the fastest plain fill measured, probes/wbench.hip)
template <bool NT, int PER, bool XR = false> // XR: XCD-contiguous regions (pb_xcd_region)
__global__ __launch_bounds__(256) void pb_fill_kernel(pb_u32x4 *dst, uint64_t n16, uint32_t v)
{
    const uint64_t b = (uint64_t)(XR ? pb_xcd_region(blockIdx.x, gridDim.x) : blockIdx.x) * (256 * PER);
#pragma unroll
    for (int i = 0; i < PER; ++i)
    {
        const uint64_t c = b + i * 256 + threadIdx.x;
        if (c < n16)
        {
            if (NT)
                __builtin_nontemporal_store(pb_u32x4{v, v ^ (uint32_t)c, v, (uint32_t)c}, dst + c);
            else
                dst[c] = pb_u32x4{v, v ^ (uint32_t)c, v, (uint32_t)c};
        }
    }
}

// write-only probe of pb_vline_kernel's store shape: each workgroup owns a contiguous region of
// RB KiB (XCD-contiguous regions) and writes it in 16-KiB steps, wave w the 4-KiB quarter w of a
// step as four 1-KiB store instructions
template <int RB>
__global__ __launch_bounds__(256) void pb_fillreg_kernel(pb_u32x4 *dst, uint64_t n16, uint32_t v)
{
    const uint64_t b = (uint64_t)pb_xcd_region(blockIdx.x, gridDim.x) * (RB * 64);
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    for (uint32_t s = 0; s < RB / 16; ++s)
    {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i)
        {
            const uint64_t c = b + s * 1024u + wv * 256u + i * 64u + lane;
            if (c < n16)
                dst[c] = pb_u32x4{v, v ^ (uint32_t)c, v, (uint32_t)c};
        }
    }
}

// ---------------- launch wrappers (called from pbgpu.cpp) ----------------

// pb_small_kernel's LDS tile: the workgroup's frames, not WGT slots of 4 * NDW bytes (98-B frames:
// 6.2 instead of 8.2 KiB, 26 instead of 19 workgroups per CU)
static size_t pb_small_tile_bytes(uint32_t wgt, uint32_t flen)
{
    return (((size_t)wgt * flen + 15) & ~(size_t)15) + 32;
}

// pb_small_kernel: workgroup b builds frames [wgt b, wgt b + wgt)
template <int NDW, int PROTO, bool RANDOM, int AL>
static void pbk_launch_linear(const pb_kargs *K, hipStream_t st)
{
    const uint32_t wgt = K->small_wgt ? K->small_wgt : PB_WG;
    const dim3 g((uint32_t)((K->n_frames + wgt - 1) / wgt));
    const size_t lds = pb_small_tile_bytes(wgt, K->fixed_len) + K->lds_pad;
    if (wgt == 64)
        hipLaunchKernelGGL((pb_small_kernel<NDW, PROTO, RANDOM, 64, AL>), g, dim3(64), lds, st, *K);
    else if (wgt == 128)
        hipLaunchKernelGGL((pb_small_kernel<NDW, PROTO, RANDOM, 128, AL>), g, dim3(128), lds, st, *K);
    else
        hipLaunchKernelGGL((pb_small_kernel<NDW, PROTO, RANDOM, PB_WG, AL>), g, dim3(PB_WG), lds, st, *K);
}

template <int NDW, int PROTO>
static void pbk_launch_small_p(const pb_kargs *K, uint32_t grid, hipStream_t st)
{
    if (K->xs_grid && K->img && K->img_solo)
    {
        hipLaunchKernelGGL((pb_ximg_kernel<PB_WG>), dim3(K->xs_grid), dim3(PB_WG), K->lds_pad, st, *K);
        return;
    }
    if (K->xs_grid && K->xp)
    {
        const size_t lds = (size_t)K->xs_np * PB_XREG + K->lds_pad;
        const bool w512 = K->xp_wgt == 512;
        const dim3 g(K->xs_grid);
        if (K->fixed_len % 4 == 0)
        {
            if (K->pl0.random && w512)
                hipLaunchKernelGGL((pb_xpage_kernel<NDW, PROTO, true, 512>), g, dim3(512), lds, st, *K);
            else if (K->pl0.random)
                hipLaunchKernelGGL((pb_xpage_kernel<NDW, PROTO, true, PB_WG>), g, dim3(PB_WG), lds, st, *K);
            else if (w512)
                hipLaunchKernelGGL((pb_xpage_kernel<NDW, PROTO, false, 512>), g, dim3(512), lds, st, *K);
            else
                hipLaunchKernelGGL((pb_xpage_kernel<NDW, PROTO, false, PB_WG>), g, dim3(PB_WG), lds, st, *K);
        }
        else // 2 mod 4: static-payload frames (98-B ICMP); any even length under PBGPU_XP_FORCE
        {
            if (K->pl0.random && w512)
                hipLaunchKernelGGL((pb_xpage_kernel<NDW, PROTO, true, 512, false>), g, dim3(512), lds, st, *K);
            else if (K->pl0.random)
                hipLaunchKernelGGL((pb_xpage_kernel<NDW, PROTO, true, PB_WG, false>), g, dim3(PB_WG), lds, st, *K);
            else if (w512)
                hipLaunchKernelGGL((pb_xpage_kernel<NDW, PROTO, false, 512, false>), g, dim3(512), lds, st, *K);
            else
                hipLaunchKernelGGL((pb_xpage_kernel<NDW, PROTO, false, PB_WG, false>), g, dim3(PB_WG), lds, st, *K);
        }
    }
    else if (K->xs_grid)
    {
        if (K->pl0.random)
            hipLaunchKernelGGL((pb_xsmall_kernel<NDW, PROTO, true>), dim3(K->xs_grid), dim3(PB_WG), K->lds_pad, st, *K);
        else
            hipLaunchKernelGGL((pb_xsmall_kernel<NDW, PROTO, false>), dim3(K->xs_grid), dim3(PB_WG), K->lds_pad, st, *K);
    }
    else if (K->fixed_len % 4 == 2) // 98-B ICMP, 106-B UDP: only the 2-mod-4 tile writes compiled in
    {
        if (K->pl0.random)
            pbk_launch_linear<NDW, PROTO, true, 2>(K, st);
        else
            pbk_launch_linear<NDW, PROTO, false, 2>(K, st);
    }
    else if (K->pl0.random)
        pbk_launch_linear<NDW, PROTO, true, 0>(K, st);
    else
        pbk_launch_linear<NDW, PROTO, false, 0>(K, st);
}

template <int NDW>
static void pbk_launch_small(const pb_kargs *K, uint32_t grid, hipStream_t st)
{
    if (K->proto == 17)
        pbk_launch_small_p<NDW, 17>(K, grid, st);
    else if (K->proto == 6)
        pbk_launch_small_p<NDW, 6>(K, grid, st);
    else
        pbk_launch_small_p<NDW, 1>(K, grid, st);
}

// pb_batch_kernel's part kind of a loaded sequence's kargs (0: no fused form)
extern "C" int pbk_batch_kind(const pb_kargs *K)
{
    if (!K->small_ndw || !K->xs_np || !K->fixed_len || K->pl_cnt != 1)
        return 0;
    if (K->small_ndw == 16 && !K->xp && K->proto == 17 && K->pl0.random && K->xs_fp_shift == 6)
        return 1;
    if (K->small_ndw == 16 && K->xp && K->proto == 6 && K->pl0.random && K->fixed_len % 4 == 0)
        return 2;
    if (K->small_ndw == 32 && K->xp && K->proto == 1 && !K->pl0.random && K->fixed_len % 4 == 2)
        return 3;
    return 0;
}

// One launch of the three parts Ks[0..2], of kinds 1, 2, 3 in that order, each with its page grid
// (xs_grid) set for block size wgt (256 or 512)
extern "C" hipError_t pbk_launch_batch(const pb_kargs *Ks, uint32_t wgt, hipStream_t st)
{
    pb_batch_args A;
    size_t lds = 0;
    uint32_t grid = 0;
    for (int j = 0; j < 3; ++j)
    {
        if (pbk_batch_kind(&Ks[j]) != j + 1 || Ks[j].xs_grid == 0)
            return hipErrorInvalidValue;
        A.K[j] = Ks[j];
        A.g[j] = Ks[j].xs_grid;
        grid += j < 2 ? (A.g[j] + 7u) & ~7u : A.g[j];
        const size_t l = Ks[j].img ? (size_t)(wgt / 64u) * PB_XPG // (the parts' own caps do not apply)
                                   : (size_t)(j == 0 ? wgt / 64u : Ks[j].xs_np) * PB_XREG;
        lds = l > lds ? l : lds;
    }
    if (wgt == 512)
        hipLaunchKernelGGL((pb_batch_kernel<512, 1, 2, 3>), dim3(grid), dim3(512), lds, st, A);
    else if (wgt == 256)
        hipLaunchKernelGGL((pb_batch_kernel<256, 1, 2, 3>), dim3(grid), dim3(256), lds, st, A);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// The workgroups pbk_launch_build launches for K (pb_count's records per launch)
extern "C" uint32_t pbk_build_grid(const pb_kargs *K)
{
    const uint64_t n = K->n_frames;
    uint64_t per = 0;
    if (K->vp)
        return K->vp_grid;
    if (K->vl)
        per = K->vl_wgf;
    else if (K->fst_g)
        per = K->fst_wgf;
    else if (K->gpf_g && !K->stage_win)
        per = K->gpf_fpw;
    else if (K->stage_win)
        per = K->stage_wgf;
    else if (K->small_ndw && K->xs_grid)
        return K->xs_grid;
    else if (K->small_ndw)
        per = K->small_wgt ? K->small_wgt : PB_WG;
    return per ? (uint32_t)((n + per - 1) / per) : 0u;
}

extern "C" hipError_t pbk_launch_build(const pb_kargs *K, hipStream_t st)
{
    if (K->vp)
    {
        // the record pass, then the pages (both are the build: one timed span)
        const uint32_t rgrid = (uint32_t)((K->n_frames + PB_WG - 1) / PB_WG);
        const bool l4 = (K->flags & PBK_L4_CSUM) != 0;
        const uint32_t nsp = K->hl == 54 ? 5u : 4u;
        const size_t lds = PB_VP_LDS(K->vp_nfp, nsp, 4);
#define PB_VP(HH, LL)                                                                                       \
    do                                                                                                      \
    {                                                                                                       \
        hipLaunchKernelGGL((pb_vrec_kernel<HH, LL>), dim3(rgrid), dim3(PB_WG), 0, st, *K);                  \
        hipLaunchKernelGGL((pb_vpage_kernel<HH, LL>), dim3(K->vp_grid), dim3(PB_WG), lds, st, *K);          \
    } while (0)
        if (K->hl == 54)
        {
            if (l4)
                PB_VP(54, true);
            else
                PB_VP(54, false);
        }
        else if (l4)
            PB_VP(42, true);
        else
            PB_VP(42, false);
#undef PB_VP
    }
    else if (K->vl)
    {
        const uint32_t grid = (uint32_t)((K->n_frames + K->vl_wgf - 1) / K->vl_wgf);
        const size_t lds = PB_VL_LDS(K->vl_wgf, K->hl == 54 ? 5 : 4, K->vl_nl48, K->vl_nlines) + K->lds_pad;
        const bool l4 = (K->flags & PBK_L4_CSUM) != 0;
        if (K->hl == 54)
        {
            if (l4)
                hipLaunchKernelGGL((pb_vline_kernel<54, true>), dim3(grid), dim3(PB_WG), lds, st, *K);
            else
                hipLaunchKernelGGL((pb_vline_kernel<54, false>), dim3(grid), dim3(PB_WG), lds, st, *K);
        }
        else
        {
            if (l4)
                hipLaunchKernelGGL((pb_vline_kernel<42, true>), dim3(grid), dim3(PB_WG), lds, st, *K);
            else
                hipLaunchKernelGGL((pb_vline_kernel<42, false>), dim3(grid), dim3(PB_WG), lds, st, *K);
        }
    }
    else if (K->fst_g)
    {
        const uint32_t grid = (uint32_t)((K->n_frames + K->fst_wgf - 1) / K->fst_wgf);
        const size_t lds = (size_t)K->fst_nbuf * K->fst_sb + PB_FST_LDS(K->fst_wgf) + K->lds_pad;
        const bool l4 = (K->flags & PBK_L4_CSUM) != 0;
#define PB_FST(GG)                                                                                        \
    do                                                                                                    \
    {                                                                                                     \
        if (l4)                                                                                           \
            hipLaunchKernelGGL((pb_fstage_kernel<GG, true>), dim3(grid), dim3(PB_WG), lds, st, *K);      \
        else                                                                                              \
            hipLaunchKernelGGL((pb_fstage_kernel<GG, false>), dim3(grid), dim3(PB_WG), lds, st, *K);     \
    } while (0)
        if (K->fst_g == 16)
            PB_FST(16);
        else if (K->fst_g == 32)
            PB_FST(32);
        else
            PB_FST(64);
#undef PB_FST
    }
    else if (K->gpf_g && !K->stage_win)
    {
        const uint32_t grid = (uint32_t)((K->n_frames + K->gpf_fpw - 1) / K->gpf_fpw);
        const uint32_t rm = K->gpf_rmode;
#define PB_GPF(GG, RM) hipLaunchKernelGGL((pb_gpf_kernel<GG, RM>), dim3(grid), dim3(PB_WG), 0, st, *K)
#define PB_GPF_RM(GG)      \
    if (rm == 1)           \
        PB_GPF(GG, 1);     \
    else if (rm == 0)      \
        PB_GPF(GG, 0);     \
    else                   \
        PB_GPF(GG, 2)
        if (K->gpf_g == 8)
        {
            PB_GPF_RM(8);
        }
        else if (K->gpf_g == 16)
        {
            PB_GPF_RM(16);
        }
        else if (K->gpf_g == 32)
        {
            PB_GPF_RM(32);
        }
        else
        {
            PB_GPF_RM(64);
        }
#undef PB_GPF_RM
#undef PB_GPF
    }
    else if (K->stage_win && K->vst)
    {
        const uint32_t grid = (uint32_t)((K->n_frames + K->stage_wgf - 1) / K->stage_wgf);
        const size_t lds = K->stage_bytes + PB_VST_LDS(K->stage_wgf) + K->lds_pad;
        const bool l4 = (K->flags & PBK_L4_CSUM) != 0;
#define PB_VST(GG)                                                                                    \
    do                                                                                                \
    {                                                                                                 \
        if (l4)                                                                                       \
            hipLaunchKernelGGL((pb_vstage_kernel<GG, true>), dim3(grid), dim3(PB_WG), lds, st, *K);  \
        else                                                                                          \
            hipLaunchKernelGGL((pb_vstage_kernel<GG, false>), dim3(grid), dim3(PB_WG), lds, st, *K); \
    } while (0)
        if (K->gpf_g == 8)
            PB_VST(8);
        else if (K->gpf_g == 16)
            PB_VST(16);
        else if (K->gpf_g == 32)
            PB_VST(32);
        else
            PB_VST(64);
#undef PB_VST
    }
    else if (K->stage_win)
    {
        const uint32_t grid = (uint32_t)((K->n_frames + K->stage_wgf - 1) / K->stage_wgf);
        const size_t lds = K->stage_bytes + PB_STAGE_LDS(K->stage_wgf) + K->lds_pad;
        const uint32_t rm = K->gpf_rmode;
#define PB_STG(GG, RM)                                                                                     \
    do                                                                                                     \
    {                                                                                                      \
        if (K->stage_wgt == 64)                                                                            \
            hipLaunchKernelGGL((pb_stage_kernel<GG, RM, 64>), dim3(grid), dim3(64), lds, st, *K);          \
        else                                                                                               \
            hipLaunchKernelGGL((pb_stage_kernel<GG, RM, PB_WG>), dim3(grid), dim3(PB_WG), lds, st, *K);    \
    } while (0)
#define PB_STG_RM(GG)      \
    if (rm == 1)           \
        PB_STG(GG, 1);     \
    else if (rm == 0)      \
        PB_STG(GG, 0);     \
    else                   \
        PB_STG(GG, 2)
        if (K->gpf_g == 8)
        {
            PB_STG_RM(8);
        }
        else if (K->gpf_g == 16)
        {
            PB_STG_RM(16);
        }
        else if (K->gpf_g == 32)
        {
            PB_STG_RM(32);
        }
        else
        {
            PB_STG_RM(64);
        }
#undef PB_STG_RM
#undef PB_STG
    }
    else if (K->small_ndw)
    {
        const uint32_t grid = (uint32_t)((K->n_frames + PB_WG - 1) / PB_WG);
        if (K->small_ndw == 16)
            pbk_launch_small<16>(K, grid, st);
        else
            pbk_launch_small<32>(K, grid, st);
    }
    else
        return hipErrorInvalidValue; // pbgpu_load_sequence selects one of the kernels above for every sequence
    return hipGetLastError();
}

// pb_vline_kernel's / pb_vstage_kernel's length pass: workgroup g sums the lengths of build
// workgroups [PB_VL_GRP g, PB_VL_GRP (g + 1)), 256 / PB_VL_GRP lanes per build workgroup, frames
// dealt round-robin to them (bsum[b]: build workgroup b's sum; l2[g]: the group's sum, scanned
// next by pb_scan_blocks).  One lane per build workgroup (252 frames in a row, 2 workgroups per
// CU with a third on some) took 0.090 ms per 2^25 frames (profiles/r05/prof/cfg/), 16 lanes 0.069-0.072.
__global__ __launch_bounds__(256) void pb_len_wgsum(pb_kargs K, uint32_t wgf, uint32_t nblk, uint32_t *bsum,
                                                    unsigned long long *l2)
{
    constexpr uint32_t LPB = PB_WG / PB_VL_GRP; // lanes per build workgroup
    static_assert(LPB >= 1 && LPB <= 64 && (LPB & (LPB - 1)) == 0, "PB_VL_GRP: a power of 2 in [4, 256]");
    __shared__ unsigned long long s_w[PB_WG / 64];
    const uint32_t b = blockIdx.x * PB_VL_GRP + threadIdx.x / LPB;
    const uint32_t sub = threadIdx.x & (LPB - 1u);
    uint32_t sum = 0;
    if (b < nblk)
    {
        const uint64_t fa = (uint64_t)b * wgf;
        const uint64_t fz = fa + wgf < K.n_frames ? fa + wgf : K.n_frames;
#pragma unroll 4
        for (uint64_t f = fa + sub; f < fz; f += LPB)
            sum += pb_frame_len<false>(K, f);
    }
#pragma unroll
    for (uint32_t dd = LPB / 2; dd > 0; dd >>= 1)
        sum += __shfl_xor(sum, dd, 64);
    if (b < nblk && sub == 0)
        bsum[b] = sum;
    // group sum: every lane group's sum once (its first lane)
    unsigned long long v = sub == 0 ? sum : 0u;
#pragma unroll
    for (uint32_t dd = 32; dd > 0; dd >>= 1)
        v += __shfl_xor(v, dd, 64);
    if ((threadIdx.x & 63u) == 0)
        s_w[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0)
    {
        unsigned long long t = 0;
#pragma unroll
        for (uint32_t i = 0; i < PB_WG / 64; ++i)
            t += s_w[i];
        l2[blockIdx.x] = t;
    }
}

extern "C" hipError_t pbk_launch_vst_lengths(const pb_kargs *K, uint32_t wgf, uint32_t *bsum, uint32_t nblk,
                                             unsigned long long *l2, uint32_t n_l2, uint64_t *offsets, hipStream_t st)
{
    hipLaunchKernelGGL(pb_len_wgsum, dim3(n_l2), dim3(PB_WG), 0, st, *K, wgf, nblk, bsum, l2);
    hipLaunchKernelGGL(pb_scan_blocks, dim3(1), dim3(1024), 0, st, l2, n_l2, offsets, K->n_frames);
    return hipGetLastError();
}

extern "C" hipError_t pbk_launch_lengths(const pb_kargs *K, unsigned long long *block_sums, uint32_t nblocks,
                                         uint64_t *offsets, hipStream_t st)
{
    hipLaunchKernelGGL(pb_len_reduce, dim3(nblocks), dim3(256), 0, st, *K, block_sums);
    hipLaunchKernelGGL(pb_scan_blocks, dim3(1), dim3(1024), 0, st, block_sums, nblocks, offsets, K->n_frames);
    hipLaunchKernelGGL(pb_len_scan, dim3(nblocks), dim3(256), 0, st, *K, (const unsigned long long *)block_sums,
                       offsets);
    return hipGetLastError();
}

extern "C" hipError_t pbk_launch_scatter_fixed(const uint8_t *src, uint32_t flen, uint32_t wlen, uint32_t n,
                                               uint64_t src_lim, uint8_t *dst, uint32_t stride, hipStream_t st)
{
    const uint32_t dpf = (wlen + 3) / 4;
    const uint64_t n_dw = (uint64_t)n * dpf;
    hipLaunchKernelGGL(pb_scatter_fixed, dim3((uint32_t)((n_dw + 255) / 256)), dim3(256), 0, st, src, flen, wlen, dpf,
                       n_dw, src_lim, dst, stride);
    return hipGetLastError();
}

// offsets[f] from pb_vline_kernel's 32-bit low words: region r = f / wf starts at rstart[r] and
// spans < 2^32 bytes, so the frame's offset is rstart[r] plus the 32-bit difference of low words.
__global__ __launch_bounds__(256) void pb_expand_offsets(const uint32_t *off32, const unsigned long long *rstart,
                                                         uint32_t wf, uint64_t n, uint64_t *offsets)
{
    const uint64_t f = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (f >= n)
        return;
    const unsigned long long r0 = rstart[(uint32_t)f / wf];
    offsets[f] = r0 + (uint32_t)(off32[f] - (uint32_t)r0);
}

extern "C" hipError_t pbk_launch_expand_offsets(const uint32_t *off32, const unsigned long long *rstart, uint32_t wf,
                                                uint64_t n, uint64_t *offsets, hipStream_t st)
{
    hipLaunchKernelGGL(pb_expand_offsets, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, off32, rstart, wf, n,
                       offsets);
    return hipGetLastError();
}

extern "C" hipError_t pbk_launch_scatter(const uint8_t *src, const uint64_t *offsets, uint64_t first, uint32_t n,
                                         uint8_t *dst, uint32_t stride, uint16_t *lens, hipStream_t st)
{
    hipLaunchKernelGGL(pb_scatter_slots, dim3(n), dim3(64), 0, st, src, offsets, first, dst, stride, lens);
    return hipGetLastError();
}

// 8 KiB per 512-thread workgroup, one plain 16-B store per lane
__global__ __launch_bounds__(512) void pb_fill512_kernel(pb_u32x4 *dst, uint64_t n16, uint32_t v)
{
    const uint64_t c = (uint64_t)blockIdx.x * 512 + threadIdx.x;
    if (c < n16)
        dst[c] = pb_u32x4{v, v ^ (uint32_t)c, v, (uint32_t)c};
}

// Write-roofline probe shapes (probes/wbench.hip, profiles/r02/wbench: the fastest plain
// fills found; dynamic LDS caps the workgroups per CU, and fewer concurrent writers
// write faster down to 4 per CU):
//  0  16 KiB per workgroup, 4 plain 16-B stores per lane     4  4 KiB, LDS-capped at 5 workgroups / CU
//  1  the same, non-temporal                                 5  4 KiB, 4 workgroups / CU
//  2  4 KiB per workgroup, one plain store per lane (8 / CU)  6  4 KiB, 3 workgroups / CU
//  3  4 KiB, LDS-capped at 6 workgroups / CU                 7  8 KiB per 512-thread workgroup, 1 store / lane
//  8  hipMemsetD32Async (the runtime's fill)
//  9-11  shapes 0, 2 and 5 with XCD-contiguous regions (each XCD fills its own eighth, as the
//        staged build kernels write since pb_xcd_region)
//  12-14 pb_vline_kernel's shape: a 208 / 64 / 16-KiB region per workgroup in 16-KiB steps,
//        5 workgroups / CU, XCD-contiguous
extern "C" const char *pbk_fill_shape_name(int mode)
{
    static const char *names[PBK_FILL_SHAPES] = {
        "16KiB/wg 4 st/lane", "16KiB/wg 4 st/lane nt", "4KiB/wg 1 st/lane (8 wg/CU)", "4KiB/wg 1 st/lane, 6 wg/CU",
        "4KiB/wg 1 st/lane, 5 wg/CU", "4KiB/wg 1 st/lane, 4 wg/CU", "4KiB/wg 1 st/lane, 3 wg/CU",
        "8KiB/512-thread wg 1 st/lane", "hipMemsetD32Async", "16KiB/wg 4 st/lane, XCD-contiguous",
        "4KiB/wg 1 st/lane (8 wg/CU), XCD-contiguous", "4KiB/wg 1 st/lane, 4 wg/CU, XCD-contiguous",
        "208KiB region/wg 16KiB steps, 5 wg/CU", "64KiB region/wg 16KiB steps, 5 wg/CU",
        "16KiB region/wg, 5 wg/CU"};
    return mode >= 0 && mode < PBK_FILL_SHAPES ? names[mode] : "?";
}

extern "C" hipError_t pbk_launch_fill(void *dst, uint64_t bytes, int mode, hipStream_t st)
{
    const uint64_t n16 = bytes / 16;
    const uint32_t g4 = (uint32_t)((n16 + 1023) / 1024), g1 = (uint32_t)((n16 + 255) / 256);
    static const uint32_t cap_lds[4] = {27136u, 32768u, 40960u, 54272u}; // 6, 5, 4, 3 workgroups per CU
    switch (mode)
    {
    case 0:
        hipLaunchKernelGGL((pb_fill_kernel<false, 4>), dim3(g4), dim3(256), 0, st, (pb_u32x4 *)dst, n16, 0x5A5A5A5Au);
        break;
    case 1:
        hipLaunchKernelGGL((pb_fill_kernel<true, 4>), dim3(g4), dim3(256), 0, st, (pb_u32x4 *)dst, n16, 0x5A5A5A5Au);
        break;
    case 2:
    case 3:
    case 4:
    case 5:
    case 6:
        hipLaunchKernelGGL((pb_fill_kernel<false, 1>), dim3(g1), dim3(256), mode == 2 ? 0u : cap_lds[mode - 3], st,
                           (pb_u32x4 *)dst, n16, 0x5A5A5A5Au);
        break;
    case 7:
        hipLaunchKernelGGL(pb_fill512_kernel, dim3((uint32_t)((n16 + 511) / 512)), dim3(512), 0, st, (pb_u32x4 *)dst,
                           n16, 0x5A5A5A5Au);
        break;
    case 9:
        hipLaunchKernelGGL((pb_fill_kernel<false, 4, true>), dim3(g4), dim3(256), 0, st, (pb_u32x4 *)dst, n16,
                           0x5A5A5A5Au);
        break;
    case 10:
    case 11:
        hipLaunchKernelGGL((pb_fill_kernel<false, 1, true>), dim3(g1), dim3(256), mode == 10 ? 0u : cap_lds[2], st,
                           (pb_u32x4 *)dst, n16, 0x5A5A5A5Au);
        break;
    case 12:
        hipLaunchKernelGGL((pb_fillreg_kernel<208>), dim3((uint32_t)((n16 + 208 * 64 - 1) / (208 * 64))), dim3(256),
                           cap_lds[1], st, (pb_u32x4 *)dst, n16, 0x5A5A5A5Au);
        break;
    case 13:
        hipLaunchKernelGGL((pb_fillreg_kernel<64>), dim3((uint32_t)((n16 + 64 * 64 - 1) / (64 * 64))), dim3(256),
                           cap_lds[1], st, (pb_u32x4 *)dst, n16, 0x5A5A5A5Au);
        break;
    case 14:
        hipLaunchKernelGGL((pb_fillreg_kernel<16>), dim3((uint32_t)((n16 + 16 * 64 - 1) / (16 * 64))), dim3(256),
                           cap_lds[1], st, (pb_u32x4 *)dst, n16, 0x5A5A5A5Au);
        break;
    default:
        return hipMemsetD32Async((hipDeviceptr_t)dst, 0x5A5A5A5Au, bytes / 4, st);
    }
    return hipGetLastError();
}
