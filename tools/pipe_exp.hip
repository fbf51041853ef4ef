// Speed-of-light ablations of the software-pipelined f32 row GEMM (kernels_gemm_pipe.hip,
// template argument XP): times the kernel with parts of its chunk loop removed on one
// layer shape, interleaved over rounds in one process.  Results are garbage for XP != 0;
// only the times matter.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pipe_exp.hip -o pipe_exp
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "../thyroid-nodule-image-segmentation-unet-ddti_amd/csrc/kernels_gemm_pipe.hip"

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

__global__ void fill_rand(float* p, size_t n, unsigned seed, float scale) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = scale * ((x & 0xFFFFFF) / 16777216.0f - 0.5f);
    }
}

static float* dalloc(size_t n, unsigned seed, float scale) {
    float* p;
    CK(hipMalloc(&p, n * sizeof(float)));
    hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, p, n, seed, scale);
    return p;
}

// variant v: XP = v % 100, prefetch depth 1 + v / 100
template <int V>
static void go_fwd(const RowGemmArgs& g) {
    using T = std::conditional_t<(V >= 100), PipeTile2, PipeTile0>;
    const dim3 grid(((g.M + 127) / 128) * (g.N / 128));
    hipLaunchKernelGGL((rowgemm_pipe_kernel<G_CONV3, OP_AFFINE, E_BIAS_RELU_STATS, T, V % 100>), grid,
                       dim3(256), 0, 0, g);
}
template <int V>
static void go_dgrad(const RowGemmArgs& g) {
    using T = std::conditional_t<(V >= 100), PipeTile2, PipeTile0>;
    const dim3 grid(((g.M + 127) / 128) * (g.N / 128));
    hipLaunchKernelGGL((rowgemm_pipe_kernel<G_CONV3, OP_PLAIN, E_STORE, T, V % 100>), grid, dim3(256), 0, 0, g);
}


// N = 64 tiles (experiment): 128x64 / 4 waves of 64x32 (library tile 1 / 3), 256x64 / 4 waves
// of 64x64 (one block per CU), 128x64 / 2 waves of 64x64
using N64a = PipeTile1;
using N64b = PipeTile<256, 64, 64, 64, 1, 1>;
using N64c = PipeTile<256, 64, 64, 64, 1, 2>;
using N64d = PipeTile<128, 64, 64, 64, 2, 1>;
using N64e = PipeTile3;
template <class T, bool FWD, int XP = 0>
static void go64(const RowGemmArgs& g) {
    const dim3 grid(((g.M + T::BM - 1) / T::BM) * (g.N / T::BN));
    if (FWD)
        hipLaunchKernelGGL((rowgemm_pipe_kernel<G_CONV3, OP_AFFINE, E_BIAS_RELU_STATS, T, XP>), grid,
                           dim3(T::THREADS), 0, 0, g);
    else
        hipLaunchKernelGGL((rowgemm_pipe_kernel<G_CONV3, OP_PLAIN, E_STORE, T, XP>), grid, dim3(T::THREADS), 0, 0, g);
}

struct Shape { const char* name; int N, H, W, Cin, Cout; };

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    const int iters = 5;
    Shape shapes[] = {
        {"L1 128->128 @128", 32, 128, 128, 128, 128},
        {"L2 256->256 @64", 32, 64, 64, 256, 256},
    };
    // vx[v]: XCD-contiguous tile order (RowGemmArgs::xcd)
    constexpr int NV = 8;
    const int xps[NV] = {0, 0, 100, 100, 2, 16, 116, 31};
    const int vx[NV] = {0, 1, 0, 1, 0, 0, 1, 0};
    typedef void (*Fn)(const RowGemmArgs&);
    const Fn fwd[NV] = {go_fwd<0>, go_fwd<0>, go_fwd<100>, go_fwd<100>, go_fwd<2>, go_fwd<16>, go_fwd<116>, go_fwd<31>};
    const Fn dgr[NV] = {go_dgrad<0>, go_dgrad<0>, go_dgrad<100>, go_dgrad<100>, go_dgrad<2>, go_dgrad<16>, go_dgrad<116>, go_dgrad<31>};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Shape& sh : shapes) {
        const int M = sh.N * sh.H * sh.W;
        float* x = dalloc((size_t)M * sh.Cin, 1, 2.f);
        float* w = dalloc((size_t)sh.Cout * 9 * sh.Cin, 2, 0.1f);
        float* sc = dalloc(sh.Cin, 3, 1.f);
        float* shf = dalloc(sh.Cin, 4, 1.f);
        float* bias = dalloc(sh.Cout, 5, 1.f);
        float* y = dalloc((size_t)M * sh.Cout, 6, 0.f);
        float* st = dalloc((size_t)(M / 64 + 1) * 2 * sh.Cout, 7, 0.f);
        float* dz = dalloc((size_t)M * sh.Cout, 8, 1.f);
        float* xo = dalloc((size_t)M * sh.Cin, 9, 0.f);
        const double flop = 2.0 * M * sh.Cout * 9.0 * sh.Cin;
        double best[2][NV] = {};
        for (int r = 0; r < rounds; ++r)
            for (int v = 0; v < NV; ++v)
                for (int op = 0; op < 2; ++op) {
                    RowGemmArgs g{};
                    g.H = sh.H; g.W = sh.W; g.M = M; g.amode = G_CONV3; g.bt = w; g.xcd = vx[v];
                    if (op == 0) {
                        g.N = sh.Cout; g.K = 9 * sh.Cin; g.a = x; g.lda = sh.Cin; g.C = sh.Cin;
                        g.ascale = sc; g.ashift = shf; g.emode = E_BIAS_RELU_STATS; g.bias = bias;
                        g.stats = st; g.out = y; g.ldo = sh.Cout;
                    } else {
                        g.N = sh.Cin; g.K = 9 * sh.Cout; g.a = dz; g.lda = sh.Cout; g.C = sh.Cout;
                        g.emode = E_STORE; g.out = xo; g.ldo = sh.Cin;
                    }
                    const Fn f = op ? dgr[v] : fwd[v];
                    f(g);
                    CK(hipGetLastError());
                    CK(hipEventRecord(e0, 0));
                    for (int it = 0; it < iters; ++it) f(g);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    const double tf = flop * iters / (ms * 1e-3) / 1e12;
                    if (tf > best[op][v]) best[op][v] = tf;
                }
        for (int op = 0; op < 2; ++op) {
            printf("%-18s %-5s", sh.name, op ? "dgrad" : "fwd");
            for (int v = 0; v < NV; ++v) printf("  xp%d%s %6.1f", xps[v], vx[v] ? "x" : "", best[op][v]);
            printf("\n");
        }
        fflush(stdout);
        CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(sc)); CK(hipFree(shf)); CK(hipFree(bias));
        CK(hipFree(y)); CK(hipFree(st)); CK(hipFree(dz)); CK(hipFree(xo));
    }
    {  // N = 64 outputs: forward 64->64 and 128->64 at 256^2 (N = Cout = 64), dgrad of 64->64
        // r04: ablations of the library's N = 64 tiles (19 = PipeTile3 forward, 25 = PipeTile6
        // dgrad): xp16 no epilogue, xp2 no loop global loads, xp31 MFMAs only
        constexpr int NV64 = 8;
        typedef void (*Fn)(const RowGemmArgs&);
        const Fn f64[NV64] = {go64<PipeTile3, true>, go64<PipeTile3, true, 16>, go64<PipeTile3, true, 2>,
                              go64<PipeTile3, true, 31>, go64<PipeTile6, true>, go64<PipeTile6, true, 16>,
                              go64<PipeTile6, true, 2>, go64<PipeTile6, true, 31>};
        const Fn d64[NV64] = {go64<PipeTile3, false>, go64<PipeTile3, false, 16>, go64<PipeTile3, false, 2>,
                              go64<PipeTile3, false, 31>, go64<PipeTile6, false>, go64<PipeTile6, false, 16>,
                              go64<PipeTile6, false, 2>, go64<PipeTile6, false, 31>};
        const char* nm[NV64] = {"t19", "t19/xp16", "t19/xp2", "t19/xp31", "t25", "t25/xp16", "t25/xp2", "t25/xp31"};
        Shape s64[] = {{"L0 64->64 @256", 32, 256, 256, 64, 64}, {"L0 128->64 @256", 32, 256, 256, 128, 64}};
        for (const Shape& sh : s64) {
            const int M = sh.N * sh.H * sh.W;
            float* x = dalloc((size_t)M * sh.Cin, 1, 2.f);
            float* w = dalloc((size_t)sh.Cout * 9 * sh.Cin, 2, 0.1f);
            float* sc = dalloc(sh.Cin, 3, 1.f);
            float* shf = dalloc(sh.Cin, 4, 1.f);
            float* bias = dalloc(sh.Cout, 5, 1.f);
            float* y = dalloc((size_t)M * sh.Cout, 6, 0.f);
            float* st = dalloc((size_t)(M / 64 + 1) * 2 * sh.Cout, 7, 0.f);
            float* dz = dalloc((size_t)M * sh.Cin, 8, 1.f);
            float* xo = dalloc((size_t)M * sh.Cin, 9, 0.f);
            const double flop = 2.0 * M * sh.Cout * 9.0 * sh.Cin;
            double best[2][NV64] = {};
            for (int r = 0; r < rounds; ++r)
                for (int v = 0; v < NV64; ++v)
                    for (int op = 0; op < 2; ++op) {
                        if (op == 1 && sh.Cin != 64) continue;
                        RowGemmArgs g{};
                        g.H = sh.H; g.W = sh.W; g.M = M; g.amode = G_CONV3; g.bt = w;
                        if (op == 0) {
                            g.N = sh.Cout; g.K = 9 * sh.Cin; g.a = x; g.lda = sh.Cin; g.C = sh.Cin;
                            g.ascale = sc; g.ashift = shf; g.emode = E_BIAS_RELU_STATS; g.bias = bias;
                            g.stats = st; g.out = y; g.ldo = sh.Cout;
                        } else {  // dgrad of a Cin -> 64 conv: N = Cin = 64, K = 9 * 64
                            g.N = sh.Cin; g.K = 9 * sh.Cout; g.a = dz; g.lda = sh.Cout; g.C = sh.Cout;
                            g.emode = E_STORE; g.out = xo; g.ldo = sh.Cin;
                        }
                        const Fn f = op ? d64[v] : f64[v];
                        f(g);
                        CK(hipGetLastError());
                        CK(hipEventRecord(e0, 0));
                        for (int it = 0; it < iters; ++it) f(g);
                        CK(hipEventRecord(e1, 0));
                        CK(hipEventSynchronize(e1));
                        float ms;
                        CK(hipEventElapsedTime(&ms, e0, e1));
                        const double tf = flop * iters / (ms * 1e-3) / 1e12;
                        if (tf > best[op][v]) best[op][v] = tf;
                    }
            for (int op = 0; op < 2; ++op) {
                printf("%-18s %-5s", sh.name, op ? "dgrad" : "fwd");
                for (int v = 0; v < NV64; ++v) printf("  %s %6.1f", nm[v], best[op][v]);
                printf("\n");
            }
            fflush(stdout);
            CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(sc)); CK(hipFree(shf)); CK(hipFree(bias));
            CK(hipFree(y)); CK(hipFree(st)); CK(hipFree(dz)); CK(hipFree(xo));
        }
    }
    return 0;
}
