// wbench.hip — HBM write-pattern microbenchmark (gfx950): which store shapes
// reach the write roofline.  Decides the frame-build kernel's store layout.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

// grid-stride fill, 16 B per lane per iteration
template <bool NT>
__global__ __launch_bounds__(256) void fill_gs(u32x4 *dst, uint64_t n16)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    {
        u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
        if (NT)
            __builtin_nontemporal_store(v, dst + i);
        else
            dst[i] = v;
    }
}

// one-shot: each thread writes PER 16-B chunks, block covers contiguous 256*PER*16 B
template <bool NT, int PER>
__global__ __launch_bounds__(256) void fill_block(uint8_t *dst, uint32_t misalign)
{
    uint8_t *base = dst + (uint64_t)blockIdx.x * 256 * PER * 16 + misalign;
#pragma unroll
    for (int i = 0; i < PER; ++i)
    {
        u32x4 v = {(uint32_t)blockIdx.x, (uint32_t)i, 2u, 3u};
        u32x4 *p = (u32x4 *)(base + ((uint64_t)i * 256 + threadIdx.x) * 16);
        if (NT)
            __builtin_nontemporal_store(v, p);
        else
            *p = v;
    }
}

// frame-per-lane: lane writes 64 contiguous bytes as 4 x 16 B (stride 64 B across lanes)
template <bool NT>
__global__ __launch_bounds__(256) void fill_lane64(uint8_t *dst)
{
    uint8_t *base = dst + ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i)
    {
        u32x4 v = {(uint32_t)blockIdx.x, (uint32_t)i, 2u, 3u};
        if (NT)
            __builtin_nontemporal_store(v, (u32x4 *)(base + 16 * i));
        else
            *(u32x4 *)(base + 16 * i) = v;
    }
}

// frame-per-lane through an LDS transpose: lanes write 64 B rows to LDS, then
// the workgroup streams the 16 KiB tile out with contiguous dwordx4 stores
template <bool NT>
__global__ __launch_bounds__(256) void fill_lane64_lds(uint8_t *dst)
{
    __shared__ __attribute__((aligned(16))) uint32_t tile[256 * 20]; // 80-B padded rows
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        *(u32x4 *)(tile + t * 20 + 4 * i) = u32x4{(uint32_t)blockIdx.x, (uint32_t)i, t, 3u};
    __syncthreads();
    uint8_t *base = dst + (uint64_t)blockIdx.x * 256 * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i)
    {
        const uint32_t c = i * 256 + t; // chunk: frame c / 4, part c % 4
        u32x4 v = *(const u32x4 *)(tile + (c >> 2) * 20 + 4 * (c & 3));
        if (NT)
            __builtin_nontemporal_store(v, (u32x4 *)(base + 16 * c));
        else
            *(u32x4 *)(base + 16 * c) = v;
    }
}

// dword stores, contiguous per wave (4 B/lane)
__global__ __launch_bounds__(256) void fill_dword(uint32_t *dst)
{
    uint32_t *base = dst + (uint64_t)blockIdx.x * 256 * 16;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        __builtin_nontemporal_store((uint32_t)i, base + i * 256 + threadIdx.x);
}


// persistent: grid of G blocks; block b writes chunks b, b+G, ... of CH bytes (16 B per lane per store)
template <int WG, int PER>
__global__ __launch_bounds__(WG) void fill_chunk(uint8_t *dst, uint64_t nchunks)
{
    for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x)
    {
        uint8_t *base = dst + c * (uint64_t)WG * PER * 16;
#pragma unroll
        for (int i = 0; i < PER; ++i)
        {
            u32x4 v = {(uint32_t)c, (uint32_t)i, 2u, 3u};
            *(u32x4 *)(base + ((uint64_t)i * WG + threadIdx.x) * 16) = v;
        }
    }
}

// one-shot blocks of WG threads, PER 16-B stores each
template <int WG, int PER>
__global__ __launch_bounds__(WG) void fill_wg(uint8_t *dst)
{
    uint8_t *base = dst + (uint64_t)blockIdx.x * WG * PER * 16;
#pragma unroll
    for (int i = 0; i < PER; ++i)
    {
        u32x4 v = {(uint32_t)blockIdx.x, (uint32_t)i, 2u, 3u};
        *(u32x4 *)(base + ((uint64_t)i * WG + threadIdx.x) * 16) = v;
    }
}

// one-shot blocks, wave-major order: wave w writes its own contiguous PER KiB
template <int WG, int PER>
__global__ __launch_bounds__(WG) void fill_wave(uint8_t *dst)
{
    const uint32_t w = threadIdx.x / 64, l = threadIdx.x % 64;
    uint8_t *base = dst + (uint64_t)blockIdx.x * WG * PER * 16 + (uint64_t)w * PER * 1024;
#pragma unroll
    for (int i = 0; i < PER; ++i)
    {
        u32x4 v = {(uint32_t)blockIdx.x, (uint32_t)i, 2u, 3u};
        *(u32x4 *)(base + ((uint64_t)i * 64 + l) * 16) = v;
    }
}

// XCD-aware: block b (dealt to XCD b % 8) writes PER chunks of CH bytes, chunk index ((b/8)*PER + i)*8 + (b+ROT)%8
template <int WG, int PER, int CH, int ROT>
__global__ __launch_bounds__(WG) void fill_xcd(uint8_t *dst)
{
    const uint32_t b = blockIdx.x;
    constexpr int SPC = CH / (WG * 16); // stores per chunk per lane
#pragma unroll
    for (int i = 0; i < PER; ++i)
    {
        const uint64_t c = ((uint64_t)(b >> 3) * PER + i) * 8 + ((b + ROT) & 7);
#pragma unroll
        for (int s = 0; s < SPC; ++s)
        {
            u32x4 v = {b, (uint32_t)i, 2u, 3u};
            *(u32x4 *)(dst + c * CH + ((uint64_t)s * WG + threadIdx.x) * 16) = v;
        }
    }
}

// XCD-aware with arbitrary chunk bytes CB (multiple of 16, <= WG*16*SPC): chunk c at c*CB + off
template <int WG, int PER, int SPC>
__global__ __launch_bounds__(WG) void fill_xcdb(uint8_t *dst, uint32_t CB, uint32_t off)
{
    const uint32_t b = blockIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i)
    {
        const uint64_t c = ((uint64_t)(b >> 3) * PER + i) * 8 + (b & 7);
#pragma unroll
        for (int s = 0; s < SPC; ++s)
        {
            const uint32_t o = (s * WG + threadIdx.x) * 16;
            u32x4 v = {b, (uint32_t)i, 2u, 3u};
            if (o < CB)
                *(u32x4 *)(dst + off + c * CB + o) = v;
        }
    }
}

template <typename F>
double timeit(F launch, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv)
{
    const uint64_t bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : (4ull << 30));
    uint8_t *buf;
    CK(hipMalloc(&buf, bytes + 4096));
    const int reps = 20;
    auto rep = [&](const char *name, double ms) {
        printf("%-40s %8.3f ms  %8.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    if (argc > 2)
    {
        // size / shape sweep of plain 16-B stores (argv[2] = any): which shape and buffer size reach the write ceiling
#define WG_CASE(WG, PER)                                                                                           \
    {                                                                                                              \
        char nm[64];                                                                                               \
        snprintf(nm, 64, "wg=%d per=%d", WG, PER);                                                                 \
        rep(nm, timeit([&] { hipLaunchKernelGGL((fill_wg<WG, PER>), dim3(bytes / (WG * PER * 16)), dim3(WG), 0, 0, buf); }, reps)); \
    }
        WG_CASE(256, 1) WG_CASE(256, 4)
#define XC_CASE(WG, PER, CH, ROT)                                                                                  \
    {                                                                                                              \
        char nm[64];                                                                                               \
        snprintf(nm, 64, "xcd wg=%d per=%d ch=%d rot=%d", WG, PER, CH, ROT);                                        \
        rep(nm, timeit([&] { hipLaunchKernelGGL((fill_xcd<WG, PER, CH, ROT>), dim3(bytes / ((uint64_t)PER * CH)), dim3(WG), 0, 0, buf); }, reps)); \
    }
        XC_CASE(256, 4, 4096, 0)
#define XB_CASE(WG, PER, SPC, CB, OFF)                                                                             \
    {                                                                                                              \
        char nm[64];                                                                                               \
        snprintf(nm, 64, "xcdb wg=%d per=%d cb=%d off=%d", WG, PER, CB, OFF);                                      \
        rep(nm, timeit([&] { hipLaunchKernelGGL((fill_xcdb<WG, PER, SPC>), dim3((bytes - 65536) / ((uint64_t)PER * CB)), dim3(WG), 0, 0, buf, (uint32_t)CB, (uint32_t)OFF); }, reps)); \
    }
        XB_CASE(256, 4, 1, 4096, 0) XB_CASE(256, 4, 1, 4096, 256) XB_CASE(256, 4, 1, 4096, 1024) XB_CASE(256, 4, 1, 4096, 2048)
        XB_CASE(256, 4, 1, 3840, 0) XB_CASE(256, 4, 1, 3584, 0) XB_CASE(256, 4, 2, 6144, 0) XB_CASE(256, 4, 2, 5120, 0)
        XB_CASE(256, 1, 1, 3840, 0) XB_CASE(256, 1, 1, 4096, 2048) XB_CASE(256, 1, 2, 6000, 0) XB_CASE(256, 2, 2, 6000, 0)
        XB_CASE(256, 1, 4, 12288, 0) XB_CASE(256, 2, 4, 12288, 0) XB_CASE(256, 1, 4, 16384, 0)
#define CH_CASE(WG, PER, G)                                                                                        \
    {                                                                                                              \
        char nm[64];                                                                                               \
        snprintf(nm, 64, "persistent wg=%d per=%d grid=%d", WG, PER, G);                                           \
        rep(nm, timeit([&] { hipLaunchKernelGGL((fill_chunk<WG, PER>), dim3(G), dim3(WG), 0, 0, buf, bytes / (WG * PER * 16)); }, reps)); \
    }
        CH_CASE(1024, 8, 256)
        CK(hipFree(buf));
        return 0;
    }
    const uint64_t n16 = bytes / 16;
    for (int g : {1024, 2048, 4096, 8192, 16384, 65536})
    {
        char nm[64];
        snprintf(nm, 64, "grid-stride nt grid=%d", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL(fill_gs<true>, dim3(g), dim3(256), 0, 0, (u32x4 *)buf, n16); },
                       reps));
        snprintf(nm, 64, "grid-stride plain grid=%d", g);
        rep(nm, timeit([&] { hipLaunchKernelGGL(fill_gs<false>, dim3(g), dim3(256), 0, 0, (u32x4 *)buf, n16); },
                       reps));
    }
    const uint32_t nb4 = (uint32_t)(bytes / (256 * 4 * 16));
    const uint32_t nb16 = (uint32_t)(bytes / (256 * 16 * 16));
    rep("block PER=4 nt aligned", timeit([&] { hipLaunchKernelGGL((fill_block<true, 4>), dim3(nb4), dim3(256), 0, 0, buf, 0u); }, reps));
    rep("block PER=4 plain aligned", timeit([&] { hipLaunchKernelGGL((fill_block<false, 4>), dim3(nb4), dim3(256), 0, 0, buf, 0u); }, reps));
    rep("block PER=16 nt aligned", timeit([&] { hipLaunchKernelGGL((fill_block<true, 16>), dim3(nb16), dim3(256), 0, 0, buf, 0u); }, reps));
    rep("block PER=16 plain aligned", timeit([&] { hipLaunchKernelGGL((fill_block<false, 16>), dim3(nb16), dim3(256), 0, 0, buf, 0u); }, reps));
    rep("block PER=4 nt misalign 4", timeit([&] { hipLaunchKernelGGL((fill_block<true, 4>), dim3(nb4), dim3(256), 0, 0, buf, 4u); }, reps));
    rep("block PER=4 nt misalign 2", timeit([&] { hipLaunchKernelGGL((fill_block<true, 4>), dim3(nb4), dim3(256), 0, 0, buf, 2u); }, reps));
    rep("block PER=4 nt misalign 1", timeit([&] { hipLaunchKernelGGL((fill_block<true, 4>), dim3(nb4), dim3(256), 0, 0, buf, 1u); }, reps));
    rep("block PER=4 plain misalign 4", timeit([&] { hipLaunchKernelGGL((fill_block<false, 4>), dim3(nb4), dim3(256), 0, 0, buf, 4u); }, reps));
    rep("lane64 nt (4x16B, 64B lane stride)", timeit([&] { hipLaunchKernelGGL(fill_lane64<true>, dim3(nb4), dim3(256), 0, 0, buf); }, reps));
    rep("lane64 plain", timeit([&] { hipLaunchKernelGGL(fill_lane64<false>, dim3(nb4), dim3(256), 0, 0, buf); }, reps));
    rep("lane64 via LDS nt", timeit([&] { hipLaunchKernelGGL(fill_lane64_lds<true>, dim3(nb4), dim3(256), 0, 0, buf); }, reps));
    rep("lane64 via LDS plain", timeit([&] { hipLaunchKernelGGL(fill_lane64_lds<false>, dim3(nb4), dim3(256), 0, 0, buf); }, reps));
    rep("dword nt contiguous", timeit([&] { hipLaunchKernelGGL(fill_dword, dim3(nb16), dim3(256), 0, 0, (uint32_t *)buf); }, reps));
    CK(hipFree(buf));
    return 0;
}
