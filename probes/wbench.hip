// wbench.hip — HBM write-pattern microbenchmark (gfx950).  Two jobs:
//  1. the write-roofline denominator: search store shapes (workgroup size,
//     stores per lane, page ownership, non-temporal, the runtime's memset and
//     copy paths) for the fastest plain fill of the same bytes;
//  2. the address-map probe behind the frame kernels' store layout: blocks of G
//     bytes written at a stride of M blocks (one residue class only) show the
//     interleave granularity and how many independent units it spreads over, and
//     a window model (contiguous per-workgroup windows, optional LDS source,
//     compute delay and occupancy limit) reproduces the staged kernels' store
//     pattern without their arithmetic.
// Usage: wbench <bytes> [section ...]   sections: shapes sparse win memset (default: all)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
    do                                                                               \
    {                                                                                \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess)                                                         \
        {                                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

template <bool NT>
__device__ __forceinline__ void st16(uint8_t *p, u32x4 v)
{
    if (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4 *>(p));
    else
        *reinterpret_cast<u32x4 *>(p) = v;
}

// Page-list fill.  Workgroup b writes `ppw` pages of 2^pgs bytes; its chunk list
// (ppw * 2^pgs / 16 chunks of 16 B) is dealt to the lanes round robin, so every
// wave store instruction writes WG*16 contiguous bytes of one page.
//   mode 0  linear:      page = b * ppw + i
//   mode 1  XCD-owned:   page = ((b / 8) * ppw + i) * 8 + b % 8   (blocks are dealt to XCDs round robin)
//   mode 2  XCD pairs:   mode 1 with two adjacent pages per slot (residue classes mod 16 in pairs)
template <int WG, bool NT>
__global__ __launch_bounds__(WG) void fill_pages(uint8_t *dst, uint32_t pgs, uint32_t ppw, uint32_t mode)
{
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t cpp = (1u << pgs) >> 4; // chunks per page
    const uint32_t nq = ppw * cpp;
    for (uint32_t q = t; q < nq; q += WG)
    {
        const uint32_t i = q / cpp, o = (q % cpp) * 16;
        uint64_t pg;
        if (mode == 0)
            pg = (uint64_t)b * ppw + i;
        else if (mode == 1)
            pg = ((uint64_t)(b >> 3) * ppw + i) * 8 + (b & 7u);
        else
            pg = (((uint64_t)(b >> 3) * (ppw >> 1) + (i >> 1)) * 8 + (b & 7u)) * 2 + (i & 1u);
        st16<NT>(dst + (pg << pgs) + o, u32x4{b, q, 2u, 3u});
    }
}

// Sparse probe: 4 KiB (or one block, if larger) per workgroup, written as blocks
// of 2^gs bytes at a stride of M blocks, residue `res` only.
__global__ __launch_bounds__(256) void fill_sparse(uint8_t *dst, uint32_t gs, uint32_t M, uint32_t res)
{
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t per = gs > 12 ? (1u << (gs - 12)) : 1u; // stores per lane
    const uint64_t wgb = (uint64_t)256 * 16 * per;          // data bytes per workgroup
    for (uint32_t i = 0; i < per; ++i)
    {
        const uint64_t o = (uint64_t)b * wgb + ((uint64_t)i * 256 + t) * 16; // data offset
        const uint64_t bi = o >> gs, within = o & ((1ull << gs) - 1);
        st16<false>(dst + ((bi * M + res) << gs) + within, u32x4{b, i, 2u, 3u});
    }
}

// Window model of the staged kernels' stores: workgroup b writes `nwin` windows
// of `wb` bytes (a multiple of 16), one after another.  Between windows a
// dependent VALU chain of `delay` steps stands in for the frame build; with
// from_lds the chunks are read from LDS (ds_read_b128) and a barrier closes each
// window, as the kernels do.  Dynamic LDS (launch argument) limits occupancy.
//   mode 0: the workgroup's region is contiguous (b * nwin * wb)
//   mode 1: windows are whole 4 KiB pages, XCD-owned as fill_pages mode 1
__global__ __launch_bounds__(256) void fill_win(uint8_t *dst, uint32_t wb, uint32_t nwin, uint32_t delay,
                                                uint32_t from_lds, uint32_t mode)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t nc = wb >> 4;
    uint32_t x = t * 2654435761u + b;
    for (uint32_t w = 0; w < nwin; ++w)
    {
        for (uint32_t d = 0; d < delay; ++d)
            x = __umul24(x, 1103515245u) + 12345u;
        if (from_lds)
        {
            for (uint32_t q = t; q < nc; q += 256)
                reinterpret_cast<u32x4 *>(lds)[q] = u32x4{x, q, w, b};
            __syncthreads();
        }
        for (uint32_t q = t; q < nc; q += 256)
        {
            uint64_t a;
            if (mode == 0)
                a = ((uint64_t)b * nwin + w) * wb + 16ull * q;
            else
            {
                const uint32_t ppw = wb >> 12;
                const uint64_t pg = ((uint64_t)(b >> 3) * nwin * ppw + (uint64_t)w * ppw + (q >> 8)) * 8 + (b & 7u);
                a = (pg << 12) + 16ull * (q & 255u);
            }
            const u32x4 v = from_lds ? reinterpret_cast<const u32x4 *>(lds)[q] : u32x4{x, q, w, b};
            st16<false>(dst + a, v);
        }
        if (from_lds)
            __syncthreads();
    }
}

// Window model by workgroup size (from LDS, a barrier per window, linear or
// XCD-owned pages as fill_win).
template <int WG>
__global__ __launch_bounds__(WG) void fill_win2(uint8_t *dst, uint32_t wb, uint32_t nwin, uint32_t mode, uint32_t delay)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t nc = wb >> 4;
    uint32_t x = t * 2654435761u + b;
    for (uint32_t w = 0; w < nwin; ++w)
    {
        for (uint32_t d = 0; d < delay; ++d)
            x = __umul24(x, 1103515245u) + 12345u;
        for (uint32_t q = t; q < nc; q += WG)
            reinterpret_cast<u32x4 *>(lds)[q] = u32x4{x, q, w, b};
        __syncthreads();
        for (uint32_t q = t; q < nc; q += WG)
        {
            uint64_t a;
            if (mode == 0)
                a = ((uint64_t)b * nwin + w) * wb + 16ull * q;
            else
            {
                const uint32_t ppw = wb >> 12;
                const uint64_t pg = ((uint64_t)(b >> 3) * nwin * ppw + (uint64_t)w * ppw + (q >> 8)) * 8 + (b & 7u);
                a = (pg << 12) + 16ull * (q & 255u);
            }
            st16<false>(dst + a, reinterpret_cast<const u32x4 *>(lds)[q]);
        }
        __syncthreads();
    }
}

// Frame-owned pages (the store side of a frame kernel for frames > 128 B):
// frames of L bytes are packed; a frame owns the 128-B lines from the one holding
// its first byte up to (not including) the one holding its end, so every line
// has one writer.  Workgroup b owns `ppw` XCD-strided 4 KiB pages (mode 1) or
// consecutive pages (mode 0) and writes the lines of every frame whose first line
// lies in one of its pages: a contiguous range [R(p), R(p + 1)) per page that
// starts inside page p and may end inside page p + 1.  Lane t stores byte 16 t of
// each 4 KiB grid page the range touches (1 KiB-aligned wave stores, masked at
// the range ends).
__device__ __forceinline__ uint64_t fown_start(uint64_t p, uint32_t L)
{
    const uint64_t a = p << 12;
    uint64_t f = a / L;
    while (((f * L) & ~127ull) < a)
        ++f;
    return (f * L) & ~127ull;
}

__global__ __launch_bounds__(256) void fill_fown(uint8_t *dst, uint32_t L, uint32_t ppw, uint32_t mode)
{
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    for (uint32_t i = 0; i < ppw; ++i)
    {
        const uint64_t p = mode ? ((uint64_t)(b >> 3) * ppw + i) * 8 + (b & 7u) : (uint64_t)b * ppw + i;
        const uint64_t r0 = fown_start(p, L), r1 = fown_start(p + 1, L);
#pragma unroll
        for (uint32_t g = 0; g < 2; ++g)
        {
            const uint64_t a = ((p + g) << 12) + 16ull * t;
            if (a >= r0 && a < r1)
                st16<false>(dst + a, u32x4{b, i, g, 3u});
        }
    }
}

// Paced page fill: a dependent chain of d0 24-bit multiply-adds before the first
// page and d1 before each further one (standing in for frame arithmetic), with
// dynamic LDS limiting the workgroups per CU.  fill_pages' page maps (mode 0/1).
__global__ __launch_bounds__(256) void fill_paced(uint8_t *dst, uint32_t ppw, uint32_t mode, uint32_t d0, uint32_t d1)
{
    extern __shared__ uint32_t lds_dummy[];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    uint32_t x = t * 2654435761u + b;
    for (uint32_t d = 0; d < d0; ++d)
        x = __umul24(x, 1103515245u) + 12345u;
    for (uint32_t i = 0; i < ppw; ++i)
    {
        if (i)
            for (uint32_t d = 0; d < d1; ++d)
                x = __umul24(x, 1103515245u) + 12345u;
        const uint64_t pg = mode ? ((uint64_t)(b >> 3) * ppw + i) * 8 + (b & 7u) : (uint64_t)b * ppw + i;
        st16<false>(dst + (pg << 12) + 16 * t, u32x4{x, i, 2u, 3u});
    }
    if (x == 0x12345678u && t == 999) // keep the chain
        lds_dummy[0] = x;
}

// Frame-owned blocks with precomputed bounds (no division in the kernel): block b
// of 2^bs bytes writes the lines [R[b], R[b + 1]) of the frames whose first line
// starts in it (R from the host, as fill_fown defines them), WG threads with one
// 16-B store per lane per grid chunk of the region; mode 1 maps blocks to
// workgroups XCD-strided.
template <int WG>
__global__ __launch_bounds__(WG) void fill_fown2(uint8_t *dst, const uint64_t *R, uint32_t bs, uint32_t mode, uint32_t nblk)
{
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t blk = mode ? ((b >> 3) + (b & 7u) * (nblk >> 3)) : b; // mode 1: XCD x owns a contiguous run of blocks
    const uint64_t r0 = R[blk], r1 = R[blk + 1];
    const uint64_t g0 = r0 & ~(uint64_t)(WG * 16 - 1);
    for (uint64_t a = g0 + 16ull * t; a < r1; a += WG * 16)
        if (a >= r0)
            st16<false>(dst + a, u32x4{b, t, 2u, 3u});
}

// Shared boundary lines: workgroup b writes [b S + d(b), (b + 1) S + d(b + 1)) in
// windows of wb bytes from LDS (a barrier per window), d(b) = 16 * ((b * 37) % 8) * on:
// with on = 1 every workgroup edge splits a 128-B line between two workgroups
// (usually on two XCDs), as packed variable-length frames do.
__global__ __launch_bounds__(256) void fill_shift(uint8_t *dst, uint32_t S, uint32_t wb, uint32_t on)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint64_t r0 = (uint64_t)b * S + 16u * (((b * 37u) % 8u) * on);
    const uint64_t r1 = (uint64_t)(b + 1) * S + 16u * ((((b + 1) * 37u) % 8u) * on);
    for (uint64_t w0 = r0; w0 < r1; w0 += wb)
    {
        const uint32_t nc = (uint32_t)((r1 - w0 < wb ? r1 - w0 : wb) >> 4);
        for (uint32_t q = t; q < nc; q += 256)
            reinterpret_cast<u32x4 *>(lds)[q] = u32x4{b, q, 2u, 3u};
        __syncthreads();
        for (uint32_t q = t; q < nc; q += 256)
            st16<false>(dst + w0 + 16ull * q, reinterpret_cast<const u32x4 *>(lds)[q]);
        __syncthreads();
    }
}

// Strided page ownership: workgroup b writes `ppw` 4 KiB pages at a stride of S
// pages, page = ((b / S) * ppw + i) * S + b % S (S = 1: linear 4*ppw KiB; S = 8:
// the XCD-owned layout).  Separates "8 XCDs own 8 residues" from "concurrent
// pages of one workgroup far apart".
__global__ __launch_bounds__(256) void fill_stride(uint8_t *dst, uint32_t ppw, uint32_t S)
{
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    for (uint32_t i = 0; i < ppw; ++i)
    {
        const uint64_t pg = ((uint64_t)(b / S) * ppw + i) * S + (b % S);
        st16<false>(dst + (pg << 12) + 16 * t, u32x4{b, i, 2u, 3u});
    }
}

// Half-chip ownership probe: does the 4 KiB XCD-residue effect come from one
// memory unit per XCD, or from the half of the chip (IOD) an XCD sits on?
// Workgroup b (XCD x = b % 8, the k = b / 8-th of that XCD) writes one block of
// `bpp` consecutive 4 KiB pages; the blocks alternate between two page-residue
// halves ({0..3}, {4..7} for bpp = 4), and XCD x writes only half grp(x):
//   group 0: grp = x / 4   group 1: grp = x % 2   group 2: grp = (x / 2) % 2
// the XCD's rank j in its half picks the block: block = (k * 4 + j) * 2 + grp.
template <int WG>
__global__ __launch_bounds__(WG) void fill_half(uint8_t *dst, uint32_t bpp, uint32_t group)
{
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint32_t x = b & 7u, k = b >> 3;
    uint32_t grp, j;
    if (group == 0)
        grp = x >> 2, j = x & 3u;
    else if (group == 1)
        grp = x & 1u, j = x >> 1;
    else
        grp = (x >> 1) & 1u, j = (x & 1u) | ((x >> 2) << 1);
    const uint64_t blk = ((uint64_t)k * 4 + j) * 2 + grp;
    const uint64_t base = blk * bpp * 4096ull;
    for (uint32_t q = t; q < bpp * 256u; q += WG)
        st16<false>(dst + base + 16ull * q, u32x4{b, q, 2u, 3u});
}

// Persistent grid-stride windows: `grid` workgroups (about one resident set)
// loop over windows g = b, b + grid, ... of wb bytes each (the byte offset of
// window g is g * wb, so wb need not be a multiple of 128: windows then split
// lines between workgroups), staged in LDS with a barrier per window as the
// staged kernels do.  At any moment the resident workgroups write neighbouring
// windows: the concurrent write footprint is ~grid * wb, against grid * (a
// workgroup's whole region) for contiguous per-workgroup regions.
__global__ __launch_bounds__(256) void fill_gwin(uint8_t *dst, uint32_t wb, uint64_t nwin)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    for (uint64_t g = b; g < nwin; g += gridDim.x)
    {
        const uint64_t w0 = g * wb;
        const uint32_t c0 = (uint32_t)(w0 & 15u);          // window start inside its first chunk
        const uint32_t nc = (c0 + wb + 15u) >> 4;
        for (uint32_t q = t; q < nc; q += 256)
            reinterpret_cast<u32x4 *>(lds)[q] = u32x4{(uint32_t)g, q, 2u, 3u};
        __syncthreads();
        uint8_t *const base = dst + (w0 & ~15ull);
        for (uint32_t q = t; q < nc; q += 256)
        {
            const u32x4 v = reinterpret_cast<const u32x4 *>(lds)[q];
            if ((q == 0 && c0) || (q == nc - 1 && ((c0 + wb) & 15u)))
            {
                // edge chunk shared with the neighbouring window: its own dwords only
                const int lo = q == 0 ? (int)c0 : 0, hi = q == nc - 1 && ((c0 + wb) & 15u) ? (int)((c0 + wb) & 15u) : 16;
                uint32_t *w = reinterpret_cast<uint32_t *>(base + 16ull * q);
                for (int i = lo / 4; i < hi / 4; ++i)
                    w[i] = v[i];
            }
            else
                st16<false>(base + 16ull * q, v);
        }
        __syncthreads();
    }
}

// Kernel timing: best of 3 trials, each the mean of `reps` back-to-back launches
// after one untimed launch.
template <typename F>
double timeit(F launch, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    double best = 1e30;
    for (int trial = 0; trial < 3; ++trial)
    {
        launch();
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r)
            launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms / reps < best)
            best = ms / reps;
    }
    CK(hipGetLastError());
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return best;
}

static uint64_t g_bytes;
static void rep(const char *name, uint64_t bytes, double ms)
{
    printf("%-56s %9.4f ms %9.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

template <int WG, bool NT>
static void pages_case(uint8_t *buf, uint32_t pgs, uint32_t ppw, uint32_t mode)
{
    const uint64_t pgb = 1ull << pgs;
    const uint64_t wgbytes = pgb * ppw;
    const uint32_t grid = (uint32_t)(g_bytes / wgbytes / 8 * 8); // whole XCD rounds
    const uint64_t bytes = (uint64_t)grid * wgbytes;
    char nm[96];
    static const char *mn[] = {"linear", "xcd", "xcd-pair"};
    snprintf(nm, sizeof nm, "pages %s wg=%d page=%llu ppw=%u st/lane=%llu%s", mn[mode], WG,
             (unsigned long long)pgb, ppw, (unsigned long long)(wgbytes / 16 / WG), NT ? " nt" : "");
    rep(nm, bytes, timeit([&] { hipLaunchKernelGGL((fill_pages<WG, NT>), dim3(grid), dim3(WG), 0, 0, buf, pgs, ppw, mode); }, 20));
}

static bool want(int argc, char **argv, const char *s)
{
    if (argc <= 2)
        return true;
    for (int i = 2; i < argc; ++i)
        if (!strcmp(argv[i], s))
            return true;
    return false;
}

int main(int argc, char **argv)
{
    g_bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : (2ull << 30));
    const uint64_t sparse_data = g_bytes / 2 < (1ull << 30) ? g_bytes / 2 : (1ull << 30);
    const uint64_t alloc = 2 * g_bytes + 8192 > 32 * sparse_data + (1 << 20) ? 2 * g_bytes + 8192 : 32 * sparse_data + (1 << 20); // sparse strides up to 32 blocks
    uint8_t *buf;
    CK(hipMalloc(&buf, alloc));
    CK(hipMemset(buf, 0, alloc));
    CK(hipDeviceSynchronize());
    printf("# wbench: %llu bytes per fill\n", (unsigned long long)g_bytes);

    if (want(argc, argv, "shapes"))
    {
        // one store per lane per 4 KiB page, every workgroup size; 2 / 4 stores per lane
        pages_case<64, false>(buf, 10, 1, 0);   // 1 KiB per 64-thread workgroup
        pages_case<64, false>(buf, 12, 1, 0);   // 4 KiB per 64-thread workgroup (4 stores / lane)
        pages_case<128, false>(buf, 11, 1, 0);  // 2 KiB per 128-thread workgroup
        pages_case<128, false>(buf, 12, 1, 0);  // 4 KiB per 128-thread workgroup (2 / lane)
        pages_case<256, false>(buf, 12, 1, 0);  // the round-1 best shape
        pages_case<256, false>(buf, 13, 1, 0);  // 8 KiB per workgroup (2 / lane)
        pages_case<256, false>(buf, 12, 2, 0);
        pages_case<256, false>(buf, 12, 4, 0);
        pages_case<512, false>(buf, 13, 1, 0);  // 8 KiB per 512-thread workgroup (1 / lane)
        pages_case<512, false>(buf, 12, 2, 0);
        pages_case<1024, false>(buf, 14, 1, 0); // 16 KiB per 1024-thread workgroup (1 / lane)
        pages_case<1024, false>(buf, 12, 4, 0);
        // XCD-owned 4 KiB pages
        pages_case<64, false>(buf, 12, 1, 1);
        pages_case<64, false>(buf, 12, 4, 1);
        pages_case<128, false>(buf, 12, 2, 1);
        pages_case<256, false>(buf, 12, 1, 1);
        pages_case<256, false>(buf, 12, 2, 1);
        pages_case<256, false>(buf, 12, 4, 1);
        pages_case<256, false>(buf, 12, 8, 1);
        pages_case<256, false>(buf, 12, 16, 1);
        pages_case<512, false>(buf, 12, 2, 1);
        pages_case<512, false>(buf, 12, 8, 1);
        pages_case<1024, false>(buf, 12, 4, 1);
        pages_case<1024, false>(buf, 12, 16, 1);
        pages_case<256, false>(buf, 12, 4, 2);
        pages_case<256, false>(buf, 11, 4, 1); // 2 KiB pages, XCD-owned
        pages_case<256, false>(buf, 13, 2, 1); // 8 KiB pages, XCD-owned
        // non-temporal
        pages_case<256, true>(buf, 12, 1, 0);
        pages_case<256, true>(buf, 12, 4, 1);
        pages_case<1024, true>(buf, 14, 1, 0);
    }
    if (want(argc, argv, "win2"))
    {
        struct W
        {
            int wg;
            uint32_t wb, nwin, lds, mode, delay;
        } cases[] = {
            {1024, 16384, 1, 16384, 0, 0},   {1024, 24576, 1, 24576, 0, 0},  {1024, 32768, 1, 32768, 0, 0},
            {1024, 49152, 1, 49152, 0, 0},   {1024, 65536, 1, 65536, 0, 0},  {1024, 98304, 1, 98304, 0, 0},
            {512, 8192, 1, 8192, 0, 0},      {512, 16384, 1, 16384, 0, 0},   {512, 24576, 1, 24576, 0, 0},
            {512, 49152, 1, 49152, 0, 0},    {256, 8192, 1, 8192, 0, 0},     {256, 16384, 1, 16384, 0, 0},
            {1024, 49152, 1, 49152, 0, 300}, {1024, 49152, 1, 49152, 0, 1500}, {1024, 16384, 1, 16384, 0, 1500},
            {512, 24576, 1, 24576, 0, 1500}, {1024, 49152, 1, 49152, 1, 0},  {1024, 49152, 1, 49152, 1, 1500},
            {1024, 98304, 1, 98304, 1, 0},   {1024, 49152, 2, 49152, 0, 0},
        };
        for (const W &c : cases)
        {
            const uint64_t wgbytes = (uint64_t)c.wb * c.nwin;
            const uint32_t grid = (uint32_t)(g_bytes / wgbytes / 8 * 8);
            char nm[128];
            snprintf(nm, sizeof nm, "win2 %s wg=%d wb=%u nwin=%u lds=%u delay=%u st/lane/win=%.1f", c.mode ? "xcd" : "linear",
                     c.wg, c.wb, c.nwin, c.lds, c.delay, c.wb / 16.0 / c.wg);
            auto L = [&] {
                if (c.wg == 256)
                    hipLaunchKernelGGL(fill_win2<256>, dim3(grid), dim3(256), c.lds, 0, buf, c.wb, c.nwin, c.mode, c.delay);
                else if (c.wg == 512)
                    hipLaunchKernelGGL(fill_win2<512>, dim3(grid), dim3(512), c.lds, 0, buf, c.wb, c.nwin, c.mode, c.delay);
                else
                    hipLaunchKernelGGL(fill_win2<1024>, dim3(grid), dim3(1024), c.lds, 0, buf, c.wb, c.nwin, c.mode, c.delay);
            };
            rep(nm, (uint64_t)grid * wgbytes, timeit(L, 10));
        }
    }
    if (want(argc, argv, "fown"))
    {
        for (uint32_t L : {1500u, 1024u, 824u, 4096u})
            for (uint32_t mode : {0u, 1u})
                for (uint32_t ppw : {1u, 4u, 8u})
                {
                    const uint32_t grid = (uint32_t)((g_bytes - 65536) / (4096ull * ppw) / 8 * 8);
                    char nm[96];
                    snprintf(nm, sizeof nm, "fown %s L=%u pages/wg=%u", mode ? "xcd" : "linear", L, ppw);
                    rep(nm, (uint64_t)grid * 4096 * ppw,
                        timeit([&] { hipLaunchKernelGGL(fill_fown, dim3(grid), dim3(256), 0, 0, buf, L, ppw, mode); }, 20));
                }
    }
    if (want(argc, argv, "paced"))
    {
        struct P
        {
            uint32_t ppw, mode, d0, d1, lds;
        } cases[] = {
            {1, 0, 0, 0, 0},    {1, 0, 8, 0, 0},    {1, 0, 16, 0, 0},   {1, 0, 32, 0, 0},   {1, 0, 64, 0, 0},
            {1, 0, 128, 0, 0},  {1, 0, 256, 0, 0},  {1, 1, 0, 0, 0},    {1, 1, 32, 0, 0},   {1, 1, 128, 0, 0},
            {4, 1, 0, 0, 0},    {4, 1, 32, 0, 0},   {4, 1, 32, 32, 0},  {4, 1, 128, 128, 0}, {4, 0, 32, 32, 0},
            {4, 0, 128, 128, 0}, {8, 1, 64, 64, 0}, {16, 1, 64, 64, 0}, {1, 0, 0, 0, 40960}, {1, 0, 0, 0, 81920},
            {1, 0, 32, 0, 40960}, {4, 1, 32, 32, 40960}, {4, 1, 32, 32, 81920},
        };
        for (const P &c : cases)
        {
            const uint32_t grid = (uint32_t)(g_bytes / (4096ull * c.ppw) / 8 * 8);
            char nm[96];
            snprintf(nm, sizeof nm, "paced %s pages/wg=%u d0=%u d1=%u lds=%u", c.mode ? "xcd" : "linear", c.ppw, c.d0, c.d1,
                     c.lds);
            rep(nm, (uint64_t)grid * 4096 * c.ppw,
                timeit([&] { hipLaunchKernelGGL(fill_paced, dim3(grid), dim3(256), c.lds, 0, buf, c.ppw, c.mode, c.d0, c.d1); }, 20));
        }
    }
    if (want(argc, argv, "occ"))
    {
        // workgroups per CU limited by dynamic LDS: 8 (none), 6, 5, 4, 3, 2 of 256 threads
        const uint32_t ldsv[] = {0u, 24576u, 30720u, 40960u, 53248u, 81920u};
        for (uint32_t mode : {0u, 1u})
            for (uint32_t ppw : {1u, 4u})
                for (uint32_t lds : ldsv)
                {
                    const uint32_t grid = (uint32_t)(g_bytes / (4096ull * ppw) / 8 * 8);
                    char nm[96];
                    snprintf(nm, sizeof nm, "occ %s pages/wg=%u lds=%u (wg/cu=%u)", mode ? "xcd" : "linear", ppw, lds,
                             lds ? (163840u / lds < 8 ? 163840u / lds : 8u) : 8u);
                    rep(nm, (uint64_t)grid * 4096 * ppw,
                        timeit([&] { hipLaunchKernelGGL(fill_paced, dim3(grid), dim3(256), lds, 0, buf, ppw, mode, 0u, 0u); }, 20));
                }
        for (uint32_t mode : {0u, 1u})
            for (uint32_t lds : ldsv)
            {
                if (lds && lds < 24576)
                    continue;
                const uint32_t wb = 24576, nwin = 4;
                const uint32_t l = lds ? lds : 24576;
                const uint32_t grid = (uint32_t)(g_bytes / ((uint64_t)wb * nwin) / 8 * 8);
                char nm[96];
                snprintf(nm, sizeof nm, "occ win %s wb=24576 nwin=4 from-lds lds=%u", mode ? "xcd" : "linear", l);
                rep(nm, (uint64_t)grid * wb * nwin,
                    timeit([&] { hipLaunchKernelGGL(fill_win, dim3(grid), dim3(256), l, 0, buf, wb, nwin, 0u, 1u, mode); }, 10));
            }
    }
    if (want(argc, argv, "fown2"))
    {
        for (uint32_t L : {1500u, 824u})
            for (uint32_t bs : {12u, 13u, 14u})
            {
                const uint32_t nblk = (uint32_t)(((g_bytes - 65536) >> bs) / 8 * 8);
                std::vector<uint64_t> R(nblk + 1);
                for (uint32_t i = 0; i <= nblk; ++i)
                {
                    const uint64_t a = (uint64_t)i << bs;
                    uint64_t f = a / L;
                    while (((f * L) & ~127ull) < a)
                        ++f;
                    R[i] = (f * L) & ~127ull;
                }
                uint64_t *dR;
                CK(hipMalloc(&dR, R.size() * 8));
                CK(hipMemcpy(dR, R.data(), R.size() * 8, hipMemcpyHostToDevice));
                const uint64_t bytes = R[nblk] - R[0];
                for (uint32_t mode : {0u})
                {
                    char nm[96];
                    snprintf(nm, sizeof nm, "fown2 L=%u block=%u wg=256", L, 1u << bs);
                    rep(nm, bytes, timeit([&] { hipLaunchKernelGGL(fill_fown2<256>, dim3(nblk), dim3(256), 0, 0, buf, dR, bs, mode, nblk); }, 20));
                    snprintf(nm, sizeof nm, "fown2 L=%u block=%u wg=512", L, 1u << bs);
                    rep(nm, bytes, timeit([&] { hipLaunchKernelGGL(fill_fown2<512>, dim3(nblk), dim3(512), 0, 0, buf, dR, bs, mode, nblk); }, 20));
                    snprintf(nm, sizeof nm, "fown2 L=%u block=%u wg=1024", L, 1u << bs);
                    rep(nm, bytes, timeit([&] { hipLaunchKernelGGL(fill_fown2<1024>, dim3(nblk), dim3(1024), 0, 0, buf, dR, bs, mode, nblk); }, 20));
                }
                CK(hipFree(dR));
            }
    }
    if (want(argc, argv, "shift"))
    {
        for (uint32_t S : {114688u, 24576u})
            for (uint32_t on : {0u, 1u, 0u, 1u})
            {
                const uint32_t grid = (uint32_t)((g_bytes - 4096) / S / 8 * 8);
                char nm[96];
                snprintf(nm, sizeof nm, "shift region=%u window=16384 split-lines=%u", S, on);
                rep(nm, (uint64_t)grid * S,
                    timeit([&] { hipLaunchKernelGGL(fill_shift, dim3(grid), dim3(256), 29288, 0, buf, S, 16384u, on); }, 20));
            }
    }
    if (want(argc, argv, "stride"))
    {
        for (uint32_t ppw : {2u, 4u, 8u})
            for (uint32_t S : {1u, 2u, 4u, 8u, 16u, 32u, 64u, 128u, 7u, 9u})
            {
                const uint32_t grid = (uint32_t)(g_bytes / (4096ull * ppw) / (8 * S) * (8 * S));
                char nm[96];
                snprintf(nm, sizeof nm, "stride pages=%u stride=%u", ppw, S);
                rep(nm, (uint64_t)grid * 4096 * ppw,
                    timeit([&] { hipLaunchKernelGGL(fill_stride, dim3(grid), dim3(256), 0, 0, buf, ppw, S); }, 20));
            }
    }
    if (want(argc, argv, "half"))
    {
        // one XCD-owned page per workgroup (the reference shape), then 8 / 16 KiB blocks by half
        {
            const uint32_t grid = (uint32_t)(g_bytes / 4096 / 8 * 8);
            rep("half baseline xcd page wg=256", (uint64_t)grid * 4096,
                timeit([&] { hipLaunchKernelGGL(fill_stride, dim3(grid), dim3(256), 0, 0, buf, 1u, 8u); }, 20));
        }
        for (uint32_t bpp : {2u, 4u})
            for (uint32_t group : {0u, 1u, 2u})
            {
                const uint32_t grid = (uint32_t)(g_bytes / (4096ull * bpp) / 8 * 8);
                char nm[96];
                snprintf(nm, sizeof nm, "half bpp=%u group=%u wg=256", bpp, group);
                rep(nm, (uint64_t)grid * 4096 * bpp,
                    timeit([&] { hipLaunchKernelGGL(fill_half<256>, dim3(grid), dim3(256), 0, 0, buf, bpp, group); }, 20));
                snprintf(nm, sizeof nm, "half bpp=%u group=%u wg=%u", bpp, group, 256 * bpp);
                if (bpp == 2)
                    rep(nm, (uint64_t)grid * 4096 * bpp,
                        timeit([&] { hipLaunchKernelGGL(fill_half<512>, dim3(grid), dim3(512), 0, 0, buf, bpp, group); }, 20));
                else
                    rep(nm, (uint64_t)grid * 4096 * bpp,
                        timeit([&] { hipLaunchKernelGGL(fill_half<1024>, dim3(grid), dim3(1024), 0, 0, buf, bpp, group); }, 20));
            }
    }
    if (want(argc, argv, "gwin"))
    {
        // staged windows, persistent grid-stride vs contiguous per-workgroup regions
        // (fill_win mode 0 at 4 windows per workgroup); 1500-B-frame windows: 16 frames
        // (24,000 B, edges split lines) and 32 frames (48,000 B, line-aligned)
        for (uint32_t wb : {24576u, 24000u, 48000u, 16384u, 8192u})
            for (uint32_t wpc : {5u, 4u, 3u})
            {
                const uint32_t lds = 163840u / wpc - 512u < 65536u ? 163840u / wpc - 512u : 65536u;
                if (lds < wb + 16)
                    continue;
                const uint64_t nwin = (g_bytes - 65536) / wb;
                const uint32_t grid = 256u * wpc;
                char nm[96];
                snprintf(nm, sizeof nm, "gwin wb=%u grid=%u (%u per CU)", wb, grid, wpc);
                rep(nm, nwin * wb, timeit([&] { hipLaunchKernelGGL(fill_gwin, dim3(grid), dim3(256), lds, 0, buf, wb, nwin); }, 20));
            }
    }
    if (want(argc, argv, "memset"))
    {
        rep("hipMemsetD32Async", g_bytes,
            timeit([&] { CK(hipMemsetD32Async((hipDeviceptr_t)buf, 0x5EEDBA5Eu, g_bytes / 4, 0)); }, 20));
        rep("hipMemsetAsync (bytes)", g_bytes, timeit([&] { CK(hipMemsetAsync(buf, 0x5E, g_bytes, 0)); }, 20));
        // a device-to-device copy writes g_bytes (and reads as many)
        rep("hipMemcpyAsync D2D (bytes written)", g_bytes,
            timeit([&] { CK(hipMemcpyAsync(buf, buf + g_bytes + 4096, g_bytes, hipMemcpyDeviceToDevice, 0)); }, 20));
    }
    if (want(argc, argv, "sparse"))
    {
        // G bytes at a stride of M blocks: the interleave granularity and its width
        const uint64_t data = sparse_data;
        for (uint32_t gs : {8u, 10u, 12u, 13u, 14u})
            for (uint32_t M : {1u, 2u, 4u, 8u, 16u, 32u})
            {
                const uint32_t per = gs > 12 ? (1u << (gs - 12)) : 1u;
                const uint32_t grid = (uint32_t)(data / (4096ull * per));
                char nm[96];
                snprintf(nm, sizeof nm, "sparse block=%u stride=%u blocks (residue 0)", 1u << gs, M);
                rep(nm, (uint64_t)grid * 4096 * per,
                    timeit([&] { hipLaunchKernelGGL(fill_sparse, dim3(grid), dim3(256), 0, 0, buf, gs, M, 0u); }, 10));
            }
    }
    if (want(argc, argv, "win"))
    {
        // the staged kernels' store pattern without their arithmetic
        struct W
        {
            uint32_t wb, nwin, delay, from_lds, lds, mode;
        } cases[] = {
            {24576, 4, 0, 0, 0, 0},     {24576, 4, 0, 1, 24576, 0}, {24576, 4, 0, 1, 30720, 0},
            {24576, 4, 200, 1, 30720, 0}, {24576, 1, 0, 1, 30720, 0}, {24576, 16, 0, 1, 30720, 0},
            {24576, 4, 0, 1, 30720, 1}, {24576, 4, 200, 1, 30720, 1}, {24576, 1, 0, 1, 30720, 1},
            {4096, 24, 0, 1, 30720, 1}, {4096, 24, 0, 1, 30720, 0},  {16384, 6, 0, 1, 30720, 1},
            {16384, 6, 0, 1, 20480, 1}, {16384, 6, 0, 1, 16384, 0},
        };
        for (const W &c : cases)
        {
            const uint64_t wgbytes = (uint64_t)c.wb * c.nwin;
            const uint32_t grid = (uint32_t)(g_bytes / wgbytes / 8 * 8);
            char nm[128];
            snprintf(nm, sizeof nm, "win %s wb=%u nwin=%u delay=%u lds=%u%s", c.mode ? "xcd" : "linear", c.wb, c.nwin,
                     c.delay, c.lds, c.from_lds ? " from-lds" : "");
            rep(nm, (uint64_t)grid * wgbytes,
                timeit([&] {
                    hipLaunchKernelGGL(fill_win, dim3(grid), dim3(256), c.lds, 0, buf, c.wb, c.nwin, c.delay, c.from_lds,
                                       c.mode);
                },
                       10));
        }
    }
    CK(hipFree(buf));
    return 0;
}
