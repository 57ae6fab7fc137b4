// r06_vdiag.hip — where pb_vline_kernel's and pb_fstage_kernel's time goes (tool only, never
// linked into libpbgpu.so): copies of the kernels with compile-time cuts, timed beside the product
// build and the write-roofline fills on the same buffers.  The pb_vline_kernel copy is the
// mid-round-6 kernel (57.5 VALU per 16-B chunk); its DIAG 16 / 48 forms prototyped the addressing
// trim the product now carries (48.5), and its timings are in profiles/r06/vdiag/.
//   DIAG 0: the copied kernel uncut
//   DIAG 1: chunks without payload bytes (a state word in every dword; lookups, masks, blend kept)
//   DIAG 2: no chunk work: constant stores in the kernel's stream geometry (prologue kept)
//   DIAG 4: no orbit sums in the prologue (the L4 checksum wrong; everything else kept)
//   DIAG 16: opaque chunk index / bounds; DIAG 32 (with 16: 48): bounds in 1/16 B, image slot by one
//            v_lshl_add (bit-exact, checked by scripts/r06/vdiag.py)
// pb_fstage_kernel copy (pr6v_fst): DIAG 1 no payload bytes, 2 no payload pass, 8 no checksum
// accumulation, 16 L4 sums from the orbit prefix sums in a second wave (needs the orbit table:
// a packed-frame sequence loaded first; refused otherwise).
// Built by scripts/r06/build_vdiag.sh into pb-af-xdp_amd/lib/libpbprobe6v.so, driven by
// scripts/r06/vdiag.py.
#include "r06_probe.hip"

namespace
{

// opaque VALU forms (the compiler may schedule them but not rewrite them into longer chains)
__device__ __forceinline__ uint32_t pr6v_sub(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_sub_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// c - 16 a (a < 2^23, c < 2^23 signed)
__device__ __forceinline__ int32_t pr6v_msub16(uint32_t a, uint32_t c)
{
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, -16, %2" : "=v"(r) : "v"(a), "v"(c));
    return r;
}

// c - 256 a with the multiplier in an SGPR (VOP3 takes no literal on gfx950)
__device__ __forceinline__ int32_t pr6v_msub256(uint32_t a, uint32_t c)
{
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(-256), "v"(c));
    return r;
}
// (a << sh) + b, kept as one v_lshl_add_u32
template <int SH>
__device__ __forceinline__ uint32_t pr6v_lshl_add(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(SH), "v"(b));
    return r;
}

template <int HL, bool L4, int DIAG>
__global__ __launch_bounds__(PB_WG) void pr6v_vline(pb_kargs K)
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
            const uint32_t ps = (DIAG & 4) ? P.st0 : pb_orbit_sum(K, P.st0, P.plen);
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
        if (DIAG & 32) // payload bounds in 1/16 B: the chunk masks index without shifts
            s_rec[tix] = pb_u32x4{r >> 4, (r + HL) << 4, (r + flen) << 4, jt.x * st0 + jt.y};
        else
            s_rec[tix] = pb_u32x4{r >> 4, r + HL, r + flen, jt.x * st0 + jt.y};
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
        pb_u32x4 rc = s_rec[tix];
        if (DIAG & 32)
            rc[1] >>= 4, rc[2] >>= 4;
        // lines whose first byte lies in this frame: the frame holding it, and where (if at all)
        // the next frame starts in the line
        const uint32_t st = rc[1] - HL;
        const uint32_t a = st > lo_rel ? st - lo_rel : 0u, b = rc[2] > lo_rel ? rc[2] - lo_rel : 0u;
        const uint32_t la = (a + 127u) >> 7, lb = min((b + 127u) >> 7, nlines);
        // the next two frames' starts in the line as 16-B chunk positions c = ceil(o / 16) (1..8,
        // 8: none), kept as 8 - c in bits 0-2 and 4-6: chunk k of the line lies in frame
        // tix + (k >= c1) + (k >= c2), and k >= c <=> k + (8 - c) carries into bit 3 / 7
        const uint32_t b2 = (uint32_t)tix + 1u < nfr ? (s_rec[tix + 1][2] >> ((DIAG & 32) ? 4 : 0)) - lo_rel : 0xFFFFFFFFu;
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
        if (DIAG & 2) // no chunk work: the stream's stores alone
            return pb_u32x4{s, i, lane, 0x5EEDu};
        uint32_t l = s * (PB_VL_STEP / 128u) + (wv << 5) + (i << 3) + (lane >> 3);
        if (clamp)
            l = min(l, lmax);
        const uint32_t ci = (l << 3) + ck;
        const uint32_t t = (uint32_t)s_map[l] + kk;
        const uint32_t f = (t >> 8) + __popc(t & 0x88u);
        const pb_u32x4 rc = s_rec[f];
        const uint32_t m = (DIAG & 16) ? pr6v_sub(ci, rc[0]) : ci - rc[0]; // chunk index within frame f
        const uint2 L = s_l48[m];
        const uint32_t x = __umul24(rc[3], L.x) + L.y;
        const int32_t pb = (int32_t)(ci << 4);
        pb_u32x4 h, mm;
        if (DIAG & 32)
        {
            // plo, phi in 1/16 B: s_m16 is indexed by (plo + phi) 16-B rows, i.e. bytes
            const uint32_t plo16 = (uint32_t)min(max(pr6v_msub256(ci, rc[1]), 0), 256);
            const uint32_t phi16 = (uint32_t)min(max(pr6v_msub256(ci, rc[2]), 0), 256);
            mm = *reinterpret_cast<const pb_u32x4 *>(reinterpret_cast<const uint8_t *>(s_m16) + plo16 + phi16);
            h = s_img[pr6v_lshl_add<2>(f, min(m, NSP))];
        }
        else
        {
            const int32_t p1 = (DIAG & 16) ? pr6v_msub16(ci, rc[1]) : (int32_t)rc[1] - pb;
            const int32_t p2 = (DIAG & 16) ? pr6v_msub16(ci, rc[2]) : (int32_t)rc[2] - pb;
            const uint32_t plo = (uint32_t)min(max(p1, 0), 16);
            const uint32_t phi = (uint32_t)min(max(p2, 0), 16);
            h = s_img[f * NSP + min(m, NSP)];
            mm = s_m16[plo + phi]; // payload bytes [plo, phi)
        }
        uint32_t o0, o1, o2, o3;
        if (DIAG & 1) // no payload bytes: one state word in every dword
            o0 = o1 = o2 = o3 = x;
        else
            pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
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


template <int G, bool L4, int DIAG>
__global__ __launch_bounds__(PB_WG) void pr6v_fstage(pb_kargs K)
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
            s_a0[tid] = (DIAG & 16) ? hs : hs + 16u * 0xFFFFu - gs;
        }
    }
    else if ((DIAG & 16) && L4 && tid >= 64u && tid - 64u < nfr)
    {
        // wave 1: the payload's word sum of frame tid - 64 from the orbit prefix sums (pb_orbit_sum),
        // beside wave 0's headers: the payload pass then sums nothing
        uint64_t k;
        uint32_t pi;
        pb_frame_index(K, f0 + (tid - 64u), k, pi);
        const uint32_t s = pb_seed(K.seed_base, K.seq, K.first_iter + k);
        const pb_frame_pl P = pb_payload<false>(K, s, pi);
        s_a0[WF + tid - 64u] = pb_orbit_sum(K, P.st0, P.plen);
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
        if (live && cnt && !(DIAG & 2))
        {
            if (L4 && lg == 0 && !(DIAG & 16))
                acc = s_a0[fr];
            uint32_t x = __umul24(s_z[fr], Mm.x) + Mm.y;
            pb_u32x4 *p = reinterpret_cast<pb_u32x4 *>(stg) + (r >> 4) + mfirst;
            uint32_t o0, o1, o2, o3;
            // DIAG 32: the chunk loop unrolled by two (one counter / compare / address step per pair)
            uint32_t i0 = 1;
            if (DIAG & 32)
                for (; i0 + 1u < cnt; i0 += 2u)
                {
                    pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
                    acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
                    p[0] = pb_u32x4{o0, o1, o2, o3};
                    x = pb_mad24(x, MG.x, mgy);
                    pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
                    acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
                    p[G] = pb_u32x4{o0, o1, o2, o3};
                    p += 2 * G;
                    x = pb_mad24(x, MG.x, mgy);
                }
            for (uint32_t i = i0; i < cnt; ++i)
            {
                if (DIAG & 1)
                    o0 = o1 = o2 = o3 = x;
                else
                    pb_chunk_payload(K, true, x, 0, 0, 0, 16, o0, o1, o2, o3);
                if (L4 && !(DIAG & 24))
                    acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
                *p = pb_u32x4{o0, o1, o2, o3};
                p += G;
                x = pb_mad24(x, MG.x, mgy);
            }
            // the lane's final chunk
            if (DIAG & 1)
                o0 = o1 = o2 = o3 = x;
            else
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
            if (L4 && !(DIAG & 16))
                acc = pb_add_halves(pb_add_halves(pb_add_halves(pb_add_halves(acc, o0), o1), o2), o3);
        }
        if (L4 && !(DIAG & 16))
            acc = pb_group_sum<G>(acc);
        if (live && lg <= hw)
        {
            uint32_t v = s_img[fr * 16 + lg];
            if (L4)
            {
                const uint32_t c = (DIAG & 16) ? (~pb_fold(pb_fold(s_a0[fr]) + s_a0[WF + fr])) & 0xFFFFu
                                               : (~pb_fold(acc)) & 0xFFFFu;
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


} // namespace

extern "C" {

// the product build's kargs for `seq` into `out`, then the DIAG copy timed (reps launches)
int pr6v_run(pbgpu_ctx *ctx, uint16_t seq, uint64_t first, uint64_t n, pbgpu_frames *out, int diag, int reps,
             double *ms)
{
    HIPCHK(hipSetDevice(ctx->device));
    pb_kargs K;
    int rc = pr6_kargs(ctx, seq, first, n, out, &K);
    if (rc != PBGPU_OK)
        return rc;
    if (!K.vl || K.hl != 42 || !(K.flags & PBK_L4_CSUM))
        return PBGPU_EINVAL;
    const uint32_t grid = (uint32_t)((K.n_frames + K.vl_wgf - 1) / K.vl_wgf);
    const size_t lds = PB_VL_LDS(K.vl_wgf, 4, K.vl_nl48, K.vl_nlines) + K.lds_pad;
    hipStream_t st = ctx->stream;
    auto launch = [&]() -> hipError_t {
        switch (diag)
        {
        case 0: hipLaunchKernelGGL((pr6v_vline<42, true, 0>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 1: hipLaunchKernelGGL((pr6v_vline<42, true, 1>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 2: hipLaunchKernelGGL((pr6v_vline<42, true, 2>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 4: hipLaunchKernelGGL((pr6v_vline<42, true, 4>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 5: hipLaunchKernelGGL((pr6v_vline<42, true, 5>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 6: hipLaunchKernelGGL((pr6v_vline<42, true, 6>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 16: hipLaunchKernelGGL((pr6v_vline<42, true, 16>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 17: hipLaunchKernelGGL((pr6v_vline<42, true, 17>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 48: hipLaunchKernelGGL((pr6v_vline<42, true, 48>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 49: hipLaunchKernelGGL((pr6v_vline<42, true, 49>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    };
    return pr6_time(ctx, reps, ms, launch);
}

// the product build (pbk_launch_build) of a packed-frame sequence with its workgroups capped at
// per_cu per CU by dynamic LDS (0: as the library launches it)
int pr6v_build_cap(pbgpu_ctx *ctx, uint16_t seq, uint64_t first, uint64_t n, pbgpu_frames *out, uint32_t per_cu,
                   int reps, double *ms)
{
    HIPCHK(hipSetDevice(ctx->device));
    pb_kargs K;
    int rc = pr6_kargs(ctx, seq, first, n, out, &K);
    if (rc != PBGPU_OK)
        return rc;
    if (!K.vl)
        return PBGPU_EINVAL;
    const uint32_t base = (uint32_t)PB_VL_LDS(K.vl_wgf, K.hl == 54 ? 5 : 4, K.vl_nl48, K.vl_nlines);
    K.lds_pad = per_cu ? lds_cap_pad(base, per_cu) : 0u;
    return pr6_time(ctx, reps, ms, [&] { return pbk_launch_build(&K, ctx->stream); });
}

// the same for pb_fstage_kernel (fixed frames > 128 B): DIAG 0 uncut, 1 no payload bytes, 2 no
// payload pass (the stage stored as it is), 8 no checksum accumulation
int pr6v_fst(pbgpu_ctx *ctx, uint16_t seq, uint64_t first, uint64_t n, pbgpu_frames *out, int diag, int reps,
             double *ms)
{
    HIPCHK(hipSetDevice(ctx->device));
    pb_kargs K;
    int rc = pr6_kargs(ctx, seq, first, n, out, &K);
    if (rc != PBGPU_OK)
        return rc;
    if (!K.fst_g || K.fst_g != 16 || !(K.flags & PBK_L4_CSUM))
        return PBGPU_EINVAL;
    if (diag & 16)
    {
        // pb_orbit_sum reads the orbit table, which the library builds only for packed-frame
        // sequences: a configs[2]-shaped sequence must have been loaded first
        if (ctx->d_orbit == nullptr || ctx->d_dlog12 == nullptr)
            return PBGPU_EINVAL;
        K.orbit = ctx->d_orbit;
        K.orbit_tot = ctx->orbit_tot;
    }
    const uint32_t grid = (uint32_t)((K.n_frames + K.fst_wgf - 1) / K.fst_wgf);
    const size_t lds = (size_t)K.fst_nbuf * K.fst_sb + PB_FST_LDS(K.fst_wgf) + 4 * K.fst_wgf + K.lds_pad;
    hipStream_t st = ctx->stream;
    auto launch = [&]() -> hipError_t {
        switch (diag)
        {
        case 0: hipLaunchKernelGGL((pr6v_fstage<16, true, 0>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 1: hipLaunchKernelGGL((pr6v_fstage<16, true, 1>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 2: hipLaunchKernelGGL((pr6v_fstage<16, true, 2>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 8: hipLaunchKernelGGL((pr6v_fstage<16, true, 8>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 9: hipLaunchKernelGGL((pr6v_fstage<16, true, 9>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 16: hipLaunchKernelGGL((pr6v_fstage<16, true, 16>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        case 32: hipLaunchKernelGGL((pr6v_fstage<16, true, 32>), dim3(grid), dim3(PB_WG), lds, st, K); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    };
    return pr6_time(ctx, reps, ms, launch);
}

} // extern "C"
