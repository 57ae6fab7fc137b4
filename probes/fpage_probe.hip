// fpage_probe.hip — can a page-owned writer build 1500-B frames at the 4 KiB
// page fill rate?  (the fast store shape is one 4 KiB page per
// short-lived workgroup; pb_fstage_kernel's frame windows top out near 6 TB/s.)
//
// Probe only, wrong bytes on purpose: workgroup b writes page b of a packed
// stream of 1500-B frames, one 16-B chunk per lane.  Each lane finds its frame
// and position, gets the frame's seed (from a per-frame record written by a
// pre-pass, or by splitmix64 in the lane), enters the payload LCG through a
// jump table at its position and generates its 16 bytes (16 v_mad_u32_u24 +
// 12 v_perm_b32, as the frame kernels do); header dwords are a template ORed
// with seed bits.  No L4 checksums: a real writer would take them (and the
// header fields) from the per-frame record, so the "rec" variant's load is the
// one it would pay.  Compared with a plain fill of the same bytes.
// Usage: fpage_probe [frames]   (default 2^23)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

constexpr uint32_t FLEN = 1500, HL = 42;
constexpr uint32_t LA = 1103515245u, LC = 12345u;
constexpr uint32_t A3 = LA * LA * LA, C3 = LC * (LA * LA + LA + 1u);

__device__ __forceinline__ uint32_t splitmix(uint64_t k)
{
    uint64_t z = (0x5EEDBA5Eull ^ k) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)(z ^ (z >> 31));
}

__device__ __forceinline__ uint32_t pack4(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3)
{
    const uint32_t lo = __builtin_amdgcn_perm(x1, x0, 0x0C0C0602u);
    const uint32_t hi = __builtin_amdgcn_perm(x3, x2, 0x0C0C0602u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

__global__ __launch_bounds__(256) void seeds_kernel(uint32_t *rec, uint64_t n)
{
    const uint64_t f = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (f < n)
        rec[f] = splitmix(f);
}

// MODE 0: seeds from rec[]; MODE 1: splitmix in the lane
template <int MODE>
__global__ __launch_bounds__(256) void fpage_kernel(uint8_t *out, const uint32_t *rec, const uint2 *jump, uint64_t total)
{
    extern __shared__ uint32_t lds_pad[];
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    const uint64_t o = (uint64_t)b * 4096 + 16 * t;
    if (o >= total)
        return;
    const uint64_t pf = ((uint64_t)b * 4096) / FLEN; // frame holding the page's first byte (uniform)
    const uint32_t r = (uint32_t)((uint64_t)b * 4096 - pf * FLEN);
    const uint32_t rel = r + 16 * t;                    // < 1500 + 4096
    const uint32_t df = rel / FLEN;
    const uint32_t p = rel - df * FLEN;                  // chunk start in its frame
    const uint64_t f = pf + df;
    uint32_t s, s2;
    if (MODE == 0)
    {
        s = rec[f];
        s2 = p + 16 > FLEN ? rec[f + 1] : 0u;
    }
    else
    {
        s = splitmix(f);
        s2 = p + 16 > FLEN ? splitmix(f + 1) : 0u;
    }
    const int j0 = (int)p - (int)HL;
    const uint2 e = jump[j0 < 0 ? 0 : j0];
    uint32_t x = e.x * s + e.y;
    uint32_t o4[4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
    {
        const uint32_t x0 = x, x1 = __umul24(x0, A3) + C3, x2 = __umul24(x1, A3) + C3, x3 = __umul24(x2, A3) + C3;
        o4[d] = pack4(x0, x1, x2, x3);
        x = __umul24(x3, A3) + C3;
    }
#pragma unroll
    for (int d = 0; d < 4; ++d)
    {
        const uint32_t pos = p + 4 * d;
        if (pos < 44) // header dword of this frame
            o4[d] = (0x45000000u + pos) | (s & 0xFFu);
        else if (pos >= FLEN) // header dword of the next frame
            o4[d] = (0x45000000u + pos - FLEN) | (s2 & 0xFFu);
    }
    *reinterpret_cast<u32x4 *>(out + o) = u32x4{o4[0], o4[1], o4[2], o4[3]};
}

__global__ __launch_bounds__(256) void fill_page(uint8_t *out, uint64_t total)
{
    const uint64_t o = (uint64_t)blockIdx.x * 4096 + 16 * threadIdx.x;
    if (o < total)
        *reinterpret_cast<u32x4 *>(out + o) = u32x4{(uint32_t)o, 1u, 2u, 3u};
}

template <typename F>
static double timeit(F launch, int reps)
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
        best = ms / reps < best ? ms / reps : best;
    }
    CK(hipGetLastError());
    return best;
}

int main(int argc, char **argv)
{
    const uint64_t nf = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 23);
    const uint64_t total = nf * FLEN;
    const uint32_t pages = (uint32_t)((total + 4095) / 4096);
    // jump[j] = L^(3 (j + 1)) as (A, C) mod 2^32
    std::vector<uint2> jt(FLEN);
    uint32_t A = A3, C = C3;
    for (uint32_t j = 0; j < FLEN; ++j)
    {
        jt[j] = make_uint2(A, C);
        C = A3 * C + C3;
        A = A3 * A;
    }
    uint8_t *out;
    uint32_t *rec;
    uint2 *jump;
    CK(hipMalloc(&out, total + 8192));
    CK(hipMalloc(&rec, (nf + 2) * 4));
    CK(hipMalloc(&jump, FLEN * sizeof(uint2)));
    CK(hipMemcpy(jump, jt.data(), FLEN * sizeof(uint2), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(seeds_kernel, dim3((uint32_t)((nf + 2 + 255) / 256)), dim3(256), 0, 0, rec, nf + 2);
    CK(hipDeviceSynchronize());
    printf("# fpage_probe: %llu frames of %u B = %.2f GB, %u pages\n", (unsigned long long)nf, FLEN, total / 1e9, pages);
    auto rep = [&](const char *nm, double ms) {
        printf("%-44s %8.4f ms %8.1f GB/s\n", nm, ms, total / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    rep("fill, 4 KiB page per workgroup", timeit([&] { hipLaunchKernelGGL(fill_page, dim3(pages), dim3(256), 0, 0, out, total); }, 10));
    for (uint32_t pad : {0u, 20480u, 32768u})
    {
        char nm[96];
        snprintf(nm, sizeof nm, "page writer, seed record  lds_pad=%u", pad);
        rep(nm, timeit([&] { hipLaunchKernelGGL(fpage_kernel<0>, dim3(pages), dim3(256), pad, 0, out, rec, jump, total); }, 10));
        snprintf(nm, sizeof nm, "page writer, splitmix     lds_pad=%u", pad);
        rep(nm, timeit([&] { hipLaunchKernelGGL(fpage_kernel<1>, dim3(pages), dim3(256), pad, 0, out, rec, jump, total); }, 10));
    }
    rep("seed pre-pass (4 B per frame)", timeit([&] {
            hipLaunchKernelGGL(seeds_kernel, dim3((uint32_t)((nf + 2 + 255) / 256)), dim3(256), 0, 0, rec, nf + 2);
        }, 10));
    CK(hipFree(out));
    CK(hipFree(rec));
    CK(hipFree(jump));
    return 0;
}
