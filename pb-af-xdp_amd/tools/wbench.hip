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
