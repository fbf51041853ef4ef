// Bandwidth experiments on the x3 image passes (csrc/kernels_gemm_x3.hip to_x3_kernel: f32 ->
// BN affine -> exact three-way bf16 split, 4 B read + 6 B written per element), on the config-2
// activation shapes.  Variants are compared bit for bit with the library kernel.
//   V1: R rows in flight per thread (all loads first), R = 4
//   V2: V1 with non-temporal loads of the f32 source (read once)
//   V3: V1 with a grid of 4 blocks per CU walking row blocks (grid-stride)
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3_pass_exp.hip -o /tmp/x3_pass_exp
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../thyroid-nodule-image-segmentation-unet-ddti_amd/csrc/kernels_gemm_x3.hip"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

namespace {

template <int R, bool NT, bool GS>
__global__ __launch_bounds__(256) void to_x3_v(const float* __restrict__ src, int C,
                                               const float* __restrict__ scale,
                                               const float* __restrict__ shift, int64_t P,
                                               uint16_t* __restrict__ dst, int rpb) {
    const int g8 = C / 8, G = min(g8, 256);
    const int r0 = threadIdx.x / G, rstep = 256 / G;
    if (r0 >= rstep) return;
    const int nblk = (int)((P + rpb - 1) / rpb);
    for (int blk = blockIdx.x; blk < nblk; blk += GS ? gridDim.x : nblk) {
        const int64_t mb = (int64_t)blk * rpb;
        const int64_t me = min(mb + rpb, P);
        for (int oct = threadIdx.x % G; oct < g8; oct += G) {
            const int c = oct * 8;
            float sc[8], sh[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f32x4 a = *(const f32x4*)(scale + c + 4 * h), b = *(const f32x4*)(shift + c + 4 * h);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    sc[4 * h + j] = a[j];
                    sh[4 * h + j] = b[j];
                }
            }
            uint16_t* dcol = dst + (c >> 5) * 96 + (c & 31);
            for (int64_t m = mb + r0; m < me; m += R * rstep) {
                f32x4 v[R][2];
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const int64_t mi = m + i * rstep;
                    if (mi < me) {
                        const f32x4* sp = (const f32x4*)(src + mi * C + c);
                        if constexpr (NT) {
                            v[i][0] = __builtin_nontemporal_load(sp);
                            v[i][1] = __builtin_nontemporal_load(sp + 1);
                        } else {
                            v[i][0] = sp[0];
                            v[i][1] = sp[1];
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const int64_t mi = m + i * rstep;
                    if (mi >= me) break;
                    float w[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) w[j] = __builtin_fmaf(sc[j], v[i][j >> 2][j & 3], sh[j]);
                    x3_store8(w, dcol + mi * 3 * (int64_t)C);
                }
            }
        }
    }
}

__global__ void fill_rand(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        p[i] = ((x & 0xFFFFFF) / 16777216.0f - 0.5f);
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 20;
    struct Shape {
        const char* name;
        int64_t P;
        int C;
    } shapes[] = {{"L0 2.1M x 64", 32LL * 256 * 256, 64},
                  {"L1 524K x 128", 32LL * 128 * 128, 128},
                  {"L2 131K x 256", 32LL * 64 * 64, 256},
                  {"L3 32K x 512", 32LL * 32 * 32, 512},
                  {"L4 8K x 1024", 32LL * 16 * 16, 1024}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int ncu = 256;
    for (const Shape& sh : shapes) {
        const int64_t n = sh.P * sh.C;
        float *x, *sc, *sf;
        uint16_t *ref, *out;
        CK(hipMalloc(&x, n * 4));
        CK(hipMalloc(&sc, sh.C * 4));
        CK(hipMalloc(&sf, sh.C * 4));
        CK(hipMalloc(&ref, n * 6));
        CK(hipMalloc(&out, n * 6));
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, x, (size_t)n, 7u);
        hipLaunchKernelGGL(fill_rand, dim3(1), dim3(256), 0, 0, sc, (size_t)sh.C, 9u);
        hipLaunchKernelGGL(fill_rand, dim3(1), dim3(256), 0, 0, sf, (size_t)sh.C, 11u);
        auto timeit = [&](auto fn) {
            CK((hipError_t)fn());
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < iters; ++i) fn();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            return ms / iters;
        };
        const double bytes = 10.0 * n;
        const float tl = timeit([&] { return k_to_x3(x, sh.C, 0, sh.C, sc, sf, 0, sh.P, ref, sh.C, 0, 0); });
        printf("%-16s library: %.3f ms %.2f TB/s\n", sh.name, tl, bytes / tl / 1e9);
        std::vector<uint16_t> r(n * 3), q(n * 3);
        CK(hipMemcpy(r.data(), ref, n * 6, hipMemcpyDeviceToHost));
        auto variant = [&](const char* name, auto fn) {
            CK(hipMemset(out, 0, n * 6));
            const float t = timeit(fn);
            CK(hipMemcpy(q.data(), out, n * 6, hipMemcpyDeviceToHost));
            printf("    %-28s %.3f ms %.2f TB/s  %s\n", name, t, bytes / t / 1e9,
                   memcmp(q.data(), r.data(), n * 6) == 0 ? "bit-identical" : "DIFFERS");
            fflush(stdout);
        };
        for (int rpb : {256, 512, 1024}) {
            const int nb = (int)((sh.P + rpb - 1) / rpb);
            char nm[64];
            snprintf(nm, sizeof nm, "R2 rpb %d", rpb);
            variant(nm, [&] {
                hipLaunchKernelGGL((to_x3_v<2, false, false>), dim3(nb), dim3(256), 0, 0, x, sh.C, sc, sf, sh.P, out, rpb);
                return (int)hipGetLastError();
            });
            snprintf(nm, sizeof nm, "R4 rpb %d", rpb);
            variant(nm, [&] {
                hipLaunchKernelGGL((to_x3_v<4, false, false>), dim3(nb), dim3(256), 0, 0, x, sh.C, sc, sf, sh.P, out, rpb);
                return (int)hipGetLastError();
            });
            snprintf(nm, sizeof nm, "R4 nt rpb %d", rpb);
            variant(nm, [&] {
                hipLaunchKernelGGL((to_x3_v<4, true, false>), dim3(nb), dim3(256), 0, 0, x, sh.C, sc, sf, sh.P, out, rpb);
                return (int)hipGetLastError();
            });
            snprintf(nm, sizeof nm, "R4 grid-stride 8/CU rpb %d", rpb);
            variant(nm, [&] {
                hipLaunchKernelGGL((to_x3_v<4, false, true>), dim3(std::min(nb, 8 * ncu)), dim3(256), 0, 0, x, sh.C,
                                   sc, sf, sh.P, out, rpb);
                return (int)hipGetLastError();
            });
        }
        CK(hipFree(x)); CK(hipFree(sc)); CK(hipFree(sf)); CK(hipFree(ref)); CK(hipFree(out));
    }
    return 0;
}
