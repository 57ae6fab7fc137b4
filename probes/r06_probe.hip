// r06_probe.hip — round-6 gate probe for a page-shaped packed writer (tool only, never linked
// into libpbgpu.so).
//
// Question: can a packed variable-length writer in the page kernels' store
// shape (one 4-KiB page per wave, short-lived workgroups: the only shape measured immune to the
// slow placement) keep the page fill's rate once each page has to find its frames
// through records written by a pre-pass?
//  * pr6_rec_kernel: the record pre-pass, one lane per frame (frames [256 b, 256 b + 256) per
//    workgroup, started from a length pass at 256 frames per workgroup): seed, fields, L4 checksum
//    (orbit sums), start; writes rec[f] = {seed, csum | flen << 16}, the 4-B offset and, for the
//    frame holding a page's first byte, pt[page] = {f, start - 4096 page}.
//  * pr6_gate<XMAP, LOADS>: the page kernel's skeleton: wave w of workgroup b owns one page, loads
//    its pt entry and the 64 records from there, scans the lengths, and stores 4 KiB of bytes that
//    depend on the loaded records (no frame bytes: the verdict's "template store" gate).
//    XMAP 0: pb_xsmall_kernel's XCD-strided pages; 1: XCD-contiguous eighths.  LOADS 0: the same
//    stores without the loads (the bare store shape).
//  * pr6_check: the records against a finished product build of the same frames.
// Built by scripts/r06/build_probe.sh into pb-af-xdp_amd/lib/libpbprobe6.so; driven by
// scripts/r06/probe.py.
#include "../pb-af-xdp_amd/csrc/pbgpu_kernels.hip"
#include "../pb-af-xdp_amd/csrc/pbgpu.cpp"

namespace
{

template <int HL, bool L4>
__global__ __launch_bounds__(256) void pr6_rec_kernel(pb_kargs K, uint2 *rec, uint2 *pt, uint32_t *off32,
                                                      unsigned long long *rstart)
{
    __shared__ uint32_t s_wsum[4];
    __shared__ unsigned long long s_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint64_t f = (uint64_t)b * 256u + tid;
    const bool valid = f < K.n_frames;
    if (wv == 0)
    {
        unsigned long long part = lane < (b & (PB_VL_GRP - 1u)) ? K.vblk_sum[(b & ~(PB_VL_GRP - 1u)) + lane] : 0ull;
#pragma unroll
        for (uint32_t dd = 32; dd > 0; dd >>= 1)
            part += __shfl_xor(part, dd, 64);
        if (lane == 0)
            s_base = K.vblk_l2[b / PB_VL_GRP] + part;
    }
    uint32_t flen = 0, s = 0, csum = 0;
    if (valid)
    {
        s = pb_seed(K.seed_base, K.seq, K.first_iter + f);
        const uint32_t r0 = pb_rand_r(s);
        const pb_frame_pl P = pb_payload<false>(K, s, 0);
        uint32_t d[16];
        const uint2 rg1 = (K.flags & PBK_RND_SADDR) ? K.ranges[0] : make_uint2(0u, 0u);
        const uint32_t l4tot = pb_header(K, r0, P.plen, d, K.rng.d == 1 ? rg1 : pb_range(K, r0));
        flen = HL + P.plen;
        if (L4)
        {
            uint32_t hs = (d[8] >> 16) + pb_halves(d[9]) + pb_halves(d[10]) + pb_halves(d[11]) + pb_halves(d[12]) +
                          pb_halves(d[13]);
            if (K.flags & PBK_PSEUDO)
                hs += (d[6] >> 16) + pb_halves(d[7]) + (d[8] & 0xFFFFu) + ((K.proto + l4tot) << 8);
            const uint32_t ps = pb_orbit_sum(K, P.st0, P.plen);
            csum = (~pb_fold(pb_fold(hs) + ps)) & 0xFFFFu;
        }
    }
    uint32_t inc = flen;
#pragma unroll
    for (uint32_t dd = 1; dd < 64; dd <<= 1)
    {
        const uint32_t y = __shfl_up(inc, dd, 64);
        inc += lane >= dd ? y : 0u;
    }
    if (lane == 63u)
        s_wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w)
        pre += w < wv ? s_wsum[w] : 0u;
    const uint64_t start = s_base + pre + inc - flen;
    if (valid)
    {
        off32[f] = (uint32_t)start;
        if (tid == 0)
            rstart[b] = start;
        rec[f] = make_uint2(s, csum | (flen << 16));
        const uint64_t pg = (start + 4095u) >> 12;
        if ((pg << 12) < start + flen)
            pt[pg] = make_uint2((uint32_t)f, (uint32_t)(start - (pg << 12)));
    }
}

template <int XMAP, int LOADS, int WGT = 256>
__global__ __launch_bounds__(WGT) void pr6_gate(uint8_t *out, const uint2 *pt, const uint2 *rec, uint64_t n,
                                                uint32_t npages)
{
    constexpr uint32_t NW = WGT / 64;
    const uint32_t b = blockIdx.x, lane = threadIdx.x & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t c;
    if (XMAP == 0)
        c = ((b >> 3) * NW + wv) * 8u + (b & 7u);
    else
        c = pb_xcd_region(b, gridDim.x) * NW + wv;
    if (c >= npages)
        return;
    pb_u32x4 v;
    if (LOADS)
    {
        const uint2 e = pt[c];
        const uint64_t f = (uint64_t)e.x + lane;
        const uint2 r = f < n ? rec[f] : make_uint2(0u, 0u);
        const uint32_t fl = r.y >> 16;
        uint32_t inc = fl;
#pragma unroll
        for (uint32_t dd = 1; dd < 64; dd <<= 1)
        {
            const uint32_t y = __shfl_up(inc, dd, 64);
            inc += lane >= dd ? y : 0u;
        }
        const int32_t st = (int32_t)e.y + (int32_t)(inc - fl);
        v = pb_u32x4{r.x, r.y, (uint32_t)st, c};
    }
    else
        v = pb_u32x4{lane, b, 0x5EEDu, c};
    uint8_t *const p = out + ((uint64_t)c << 12) + (lane << 4);
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i)
        pb_st16_nt(p + (i << 10), v ^ i);
}

// records vs a finished product build (offs: its expanded offsets): counts of mismatching
// offsets, lengths, checksums and page entries
__global__ __launch_bounds__(256) void pr6_check(const uint8_t *out, const uint64_t *offs, const uint2 *rec,
                                                 const uint2 *pt, const uint32_t *off32, uint64_t n, uint32_t npages,
                                                 uint32_t cpos, uint32_t l4, unsigned long long *bad)
{
    unsigned long long e0 = 0, e1 = 0, e2 = 0, e3 = 0;
    const uint64_t g0 = (uint64_t)blockIdx.x * 256 + threadIdx.x, gs = (uint64_t)gridDim.x * 256;
    for (uint64_t f = g0; f < n; f += gs)
    {
        const uint64_t o = offs[f], fl = offs[f + 1] - o;
        e0 += off32[f] != (uint32_t)o;
        e1 += (rec[f].y >> 16) != fl;
        if (l4)
            e2 += ((uint32_t)out[o + cpos] | ((uint32_t)out[o + cpos + 1] << 8)) != (rec[f].y & 0xFFFFu);
    }
    for (uint64_t c = g0; c < npages; c += gs)
    {
        const uint2 e = pt[c];
        const uint64_t a = c << 12;
        const bool okp = e.x < n && offs[e.x] <= a && a < offs[e.x + 1] && (uint32_t)(offs[e.x] - a) == e.y;
        e3 += !okp;
    }
    if (e0)
        atomicAdd(bad + 0, e0);
    if (e1)
        atomicAdd(bad + 1, e1);
    if (e2)
        atomicAdd(bad + 2, e2);
    if (e3)
        atomicAdd(bad + 3, e3);
}

template <typename F>
int pr6_time(pbgpu_ctx *ctx, int reps, double *ms, F launch)
{
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    HIPCHK(launch());
    HIPCHK(hipEventRecord(a, ctx->stream));
    for (int r = 0; r < reps; ++r)
        HIPCHK(launch());
    HIPCHK(hipEventRecord(b, ctx->stream));
    HIPCHK(hipEventSynchronize(b));
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *ms = t / reps;
    return PBGPU_OK;
}

// the product kargs of a build of `seq` into `out` (its length pass queued on the context's stream)
int pr6_kargs(pbgpu_ctx *ctx, uint16_t seq, uint64_t first, uint64_t n, pbgpu_frames *out, pb_kargs *K)
{
    seq_slot &S = ctx->seqs[seq];
    const uint64_t used = S.ctr_used;
    batch_part bp;
    bp.st = ctx->stream;
    bp.wgt = 256;
    const int rc = build_impl(ctx, seq, first, n, out, &bp);
    S.ctr_used = used;
    if (rc != PBGPU_OK)
        return rc;
    *K = bp.K;
    K->ctr_slots = nullptr;
    K->counters = ctx->d_counters + PB_CTR_WORDS * (size_t)(PB_MAX_SEQUENCES - 1);
    return PBGPU_OK;
}

struct pr6_bufs
{
    uint2 *rec = nullptr, *pt = nullptr;
    uint32_t *off32 = nullptr, *bsum = nullptr;
    unsigned long long *rstart = nullptr, *l2 = nullptr, *bad = nullptr;
    uint64_t cap = 0;
};
pr6_bufs B6;

} // namespace

extern "C" {

// scratch for n frames: records, page table, offsets, length-pass sums
int pr6_alloc(pbgpu_ctx *ctx, uint64_t n, uint64_t max_bytes)
{
    HIPCHK(hipSetDevice(ctx->device));
    const uint64_t np = max_bytes / 4096 + 2, nb = n / 256 + 2;
    HIPCHK(hipMalloc((void **)&B6.rec, n * sizeof(uint2)));
    HIPCHK(hipMalloc((void **)&B6.pt, np * sizeof(uint2)));
    HIPCHK(hipMalloc((void **)&B6.off32, (n + 1) * sizeof(uint32_t)));
    HIPCHK(hipMalloc((void **)&B6.rstart, nb * sizeof(unsigned long long)));
    HIPCHK(hipMalloc((void **)&B6.bsum, nb * sizeof(uint32_t)));
    HIPCHK(hipMalloc((void **)&B6.l2, (nb / PB_VL_GRP + 2) * sizeof(unsigned long long)));
    HIPCHK(hipMalloc((void **)&B6.bad, 4 * sizeof(unsigned long long)));
    B6.cap = n;
    return PBGPU_OK;
}

// the pre-pass over configs[2]-shaped sequence `seq`, iterations [first, first + n), into `out`'s
// offsets (total) and the scratch; ms[0] the length pass + scan, ms[1] the record pass
int pr6_prep(pbgpu_ctx *ctx, uint16_t seq, uint64_t first, uint64_t n, pbgpu_frames *out, int reps, double *ms)
{
    HIPCHK(hipSetDevice(ctx->device));
    pb_kargs K;
    int rc = pr6_kargs(ctx, seq, first, n, out, &K);
    if (rc != PBGPU_OK)
        return rc;
    if (!K.vl || n > B6.cap || K.pl_cnt != 1)
        return PBGPU_EINVAL;
    const uint32_t nblk = (uint32_t)((n + 255) / 256), nl2 = (nblk + PB_VL_GRP - 1) / PB_VL_GRP;
    K.vblk_sum = B6.bsum;
    K.vblk_l2 = B6.l2;
    hipStream_t st = ctx->stream;
    auto lens = [&]() { return pbk_launch_vst_lengths(&K, 256, B6.bsum, nblk, B6.l2, nl2, out->offsets, st); };
    auto recs = [&]() -> hipError_t {
        const bool l4 = (K.flags & PBK_L4_CSUM) != 0;
        if (K.hl == 54)
        {
            if (l4)
                hipLaunchKernelGGL((pr6_rec_kernel<54, true>), dim3(nblk), dim3(256), 0, st, K, B6.rec, B6.pt,
                                   B6.off32, B6.rstart);
            else
                hipLaunchKernelGGL((pr6_rec_kernel<54, false>), dim3(nblk), dim3(256), 0, st, K, B6.rec, B6.pt,
                                   B6.off32, B6.rstart);
        }
        else if (l4)
            hipLaunchKernelGGL((pr6_rec_kernel<42, true>), dim3(nblk), dim3(256), 0, st, K, B6.rec, B6.pt, B6.off32,
                               B6.rstart);
        else
            hipLaunchKernelGGL((pr6_rec_kernel<42, false>), dim3(nblk), dim3(256), 0, st, K, B6.rec, B6.pt, B6.off32,
                               B6.rstart);
        return hipGetLastError();
    };
    if ((rc = pr6_time(ctx, reps, &ms[0], lens)) != PBGPU_OK)
        return rc;
    return pr6_time(ctx, reps, &ms[1], recs);
}

// the scratch's records against `out` as the product built it (offsets expanded first);
// bad[4]: offsets, lengths, checksums, page entries
int pr6_check_out(pbgpu_ctx *ctx, uint16_t seq, pbgpu_frames *out, uint64_t total, unsigned long long *bad)
{
    HIPCHK(hipSetDevice(ctx->device));
    int rc = pbgpu_frames_offsets(ctx, out);
    if (rc != PBGPU_OK)
        return rc;
    const pb_kargs &K = ctx->seqs[seq].K;
    HIPCHK(hipMemsetAsync(B6.bad, 0, 4 * sizeof(unsigned long long), ctx->stream));
    const uint32_t np = (uint32_t)((total + 4095) / 4096);
    hipLaunchKernelGGL(pr6_check, dim3(2048), dim3(256), 0, ctx->stream, out->data, out->offsets, B6.rec, B6.pt,
                       B6.off32, out->n_frames, np, 4 * K.csum_dw + 2 * K.csum_hi,
                       (K.flags & PBK_L4_CSUM) ? 1u : 0u, B6.bad);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(ctx->stream));
    HIPCHK(hipMemcpy(bad, B6.bad, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return PBGPU_OK;
}

// the gate kernel over `total` bytes at dst: variant 0 XCD-strided pages, 1 XCD-contiguous,
// 2 / 3 the same without loads; lds_pad caps workgroups per CU
int pr6_gate_run(pbgpu_ctx *ctx, void *dst, uint64_t total, uint64_t n, int variant, uint32_t lds_pad, int reps,
                 double *ms)
{
    HIPCHK(hipSetDevice(ctx->device));
    const uint32_t np = (uint32_t)((total + 4095) / 4096);
    hipStream_t st = ctx->stream;
    uint8_t *o = (uint8_t *)dst;
    const dim3 g0((np + 31) / 32 * 8), g1((np + 3) / 4);
    auto launch = [&]() -> hipError_t {
        switch (variant)
        {
        case 0: hipLaunchKernelGGL((pr6_gate<0, 1>), g0, dim3(256), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 1: hipLaunchKernelGGL((pr6_gate<1, 1>), g1, dim3(256), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 2: hipLaunchKernelGGL((pr6_gate<0, 0>), g0, dim3(256), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 3: hipLaunchKernelGGL((pr6_gate<1, 0>), g1, dim3(256), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        // store shapes without loads: pages per workgroup 1, 2, 8 (64-, 128-, 512-thread workgroups)
        case 4: hipLaunchKernelGGL((pr6_gate<0, 0, 64>), dim3((np + 7) / 8 * 8), dim3(64), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 5: hipLaunchKernelGGL((pr6_gate<1, 0, 64>), dim3(np), dim3(64), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 6: hipLaunchKernelGGL((pr6_gate<0, 0, 128>), dim3((np + 15) / 16 * 8), dim3(128), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 7: hipLaunchKernelGGL((pr6_gate<1, 0, 128>), dim3((np + 1) / 2), dim3(128), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 8: hipLaunchKernelGGL((pr6_gate<0, 0, 512>), dim3((np + 63) / 64 * 8), dim3(512), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 9: hipLaunchKernelGGL((pr6_gate<1, 0, 512>), dim3((np + 7) / 8), dim3(512), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        // the same shapes with the loads
        case 10: hipLaunchKernelGGL((pr6_gate<0, 1, 64>), dim3((np + 7) / 8 * 8), dim3(64), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 11: hipLaunchKernelGGL((pr6_gate<0, 1, 128>), dim3((np + 15) / 16 * 8), dim3(128), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        case 12: hipLaunchKernelGGL((pr6_gate<0, 1, 512>), dim3((np + 63) / 64 * 8), dim3(512), lds_pad, st, o, B6.pt, B6.rec, n, np); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    };
    return pr6_time(ctx, reps, ms, launch);
}

// the product build of `seq` into `out`, reps launches (the length pass included, as pbgpu_build)
int pr6_build(pbgpu_ctx *ctx, uint16_t seq, uint64_t first, uint64_t n, pbgpu_frames *out, int reps, double *ms)
{
    HIPCHK(hipSetDevice(ctx->device));
    pb_kargs K;
    int rc = pr6_kargs(ctx, seq, first, n, out, &K);
    if (rc != PBGPU_OK)
        return rc;
    return pr6_time(ctx, reps, ms, [&] { return pbk_launch_build(&K, ctx->stream); });
}

// a write-roofline fill shape (pbk_launch_fill) over dst
int pr6_fill(pbgpu_ctx *ctx, void *dst, uint64_t bytes, int mode, int reps, double *ms)
{
    HIPCHK(hipSetDevice(ctx->device));
    return pr6_time(ctx, reps, ms, [&] { return pbk_launch_fill(dst, bytes, mode, ctx->stream); });
}

} // extern "C"
