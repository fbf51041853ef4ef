// Probe for the split-bf16 fp32 row GEMM (csrc/kernels_gemm_x3.hip) against the f32-MFMA
// pipelined kernel (csrc/kernels_gemm_pipe.hip) on the 3x3 conv GEMMs of BASELINE config 2
// (bs 32, 256^2, models/model.py UNet): time per launch of each, max |difference| between
// them, and both kernels' errors against an fp64 dot product on sampled outputs.
// Second part: the x3 weight gradient against the f32 library kernels (launch_wgrad, linked
// from lib/libunet_hip.so), slabs summed on the host.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3_probe.hip -o /tmp/x3_probe \
//          -L thyroid-nodule-image-segmentation-unet-ddti_amd/lib -lunet_hip
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <cmath>
#include <vector>

#include "../thyroid-nodule-image-segmentation-unet-ddti_amd/csrc/kernels_gemm_pipe.hip"
#include "../thyroid-nodule-image-segmentation-unet-ddti_amd/csrc/kernels_gemm_x3.hip"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void fill_rand(float* p, size_t n, unsigned seed, float scale, int relu) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        float v = scale * ((x & 0xFFFFFF) / 16777216.0f - 0.5f);
        p[i] = relu ? fmaxf(v, 0.f) : v;
    }
}

struct Shape {
    const char* name;
    int N, H, W, Cin, Cout;
};

static void probe_wgrad(int iters, void* zero);

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 5;
    const int what = argc > 2 ? atoi(argv[2]) : 3;  // bit 0 row GEMMs, bit 1 weight gradients,
                                                     // bit 2 speed-of-light ablations of tile 0
    Shape shapes[] = {
        {"L0 64->64 @256", 32, 256, 256, 64, 64},     {"L0 128->64 @256", 32, 256, 256, 128, 64},
        {"L0 64->128 @256 (dgrad)", 32, 256, 256, 64, 128},
        {"L1 64->128 @128", 32, 128, 128, 64, 128},   {"L1 128->128 @128", 32, 128, 128, 128, 128},
        {"L1 256->128 @128", 32, 128, 128, 256, 128}, {"L2 256->256 @64", 32, 64, 64, 256, 256},
        {"L3 512->512 @32", 32, 32, 32, 512, 512},    {"L4 1024->1024 @16", 32, 16, 16, 1024, 1024},
    };
    void* zero;
    CK(hipMalloc(&zero, 256));
    CK(hipMemset(zero, 0, 256));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (what & 2) probe_wgrad(iters, zero);
    for (const Shape& sh : shapes) {
        if (!(what & 5)) break;
        const int M = sh.N * sh.H * sh.W, N = sh.Cout, C = sh.Cin, K = 9 * C;
        float *x, *w, *y32, *yx3;
        uint16_t *x3, *w3;
        CK(hipMalloc(&x, (size_t)M * C * 4));
        CK(hipMalloc(&w, (size_t)N * K * 4));
        CK(hipMalloc(&y32, (size_t)M * N * 4));
        CK(hipMalloc(&yx3, (size_t)M * N * 4));
        CK(hipMalloc(&x3, (size_t)M * C * 6));
        CK(hipMalloc(&w3, (size_t)N * K * 6));
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, x, (size_t)M * C, 17u, 4.f, 1);
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, w, (size_t)N * K, 91u,
                           2.f / sqrtf((float)K), 0);
        CK((hipError_t)k_to_x3(x, C, 0, C, nullptr, nullptr, 0, M, x3, C, 0, 0));
        CK((hipError_t)k_to_x3(w, K, 0, K, nullptr, nullptr, 0, N, w3, K, 0, 0));
        RowGemmArgs g{};
        g.H = sh.H;
        g.W = sh.W;
        g.M = M;
        g.N = N;
        g.K = K;
        g.a = x;
        g.lda = C;
        g.C = C;
        g.amode = G_CONV3;
        g.bt = w;
        g.out = y32;
        g.ldo = N;
        g.emode = E_STORE;
        g.xcd = 1;
        RowGemmArgs h = g;
        h.a = nullptr;
        h.bt = nullptr;
        h.a16 = x3;
        h.bt16 = w3;
        h.zero16 = zero;
        h.out = yx3;
        const double fl = 2.0 * M * N * K;
        const int ptile = N % 128 == 0 ? 2 : 5;
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
        if (what & 4) {  // ablations: 1 no A DMA, 2 no B DMA, 4 no LDS reads, 8 no waits / barriers
            if (N % 128) continue;
            const float t0 = timeit([&] { return launch_rowgemm_x3(h, 0, 0); });
            printf("%-26s M=%d N=%d K=%d  x3 tile 0: %.3f ms %.1f TF/s\n", sh.name, M, N, K, t0, fl / t0 / 1e9);
            for (int xp : {1, 2, 3, 4, 8, 12, 7, 15}) {
                const float tx = timeit([&] { return launch_rowgemm_x3_xp(h, xp, 0); });
                printf("    xp %2d: %.3f ms %.1f TF/s\n", xp, tx, fl / tx / 1e9);
            }
            fflush(stdout);
            CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(y32)); CK(hipFree(yx3)); CK(hipFree(x3)); CK(hipFree(w3));
            continue;
        }
        const float t32 = timeit([&] { return launch_rowgemm_pipe(g, ptile, 0); });
        // the split pass of the activation (per layer in a real step; weights are per step)
        const float tsp = timeit([&] { return k_to_x3(x, C, 0, C, nullptr, nullptr, 0, M, x3, C, 0, 0); });
        printf("%-26s M=%d N=%d K=%d  f32 pipe tile %d: %.3f ms %.1f TF/s | split pass %.3f ms\n", sh.name,
               M, N, K, ptile, t32, fl / t32 / 1e9, tsp);
        std::vector<float> r32((size_t)M * N);
        CK(hipMemcpy(r32.data(), y32, r32.size() * 4, hipMemcpyDeviceToHost));
        std::vector<float> hx, hw;
        bool host_loaded = false;
        for (int tile = 0; tile <= 7; ++tile) {
            int bm = 0, bn = 0;
            if (rowgemm_x3_tile_dims(tile, &bm, &bn) != 0 || N % bn) continue;
            CK(hipMemset(yx3, 0, (size_t)M * N * 4));
            const float tx = timeit([&] { return launch_rowgemm_x3(h, tile, 0); });
            std::vector<float> rx((size_t)M * N);
            CK(hipMemcpy(rx.data(), yx3, rx.size() * 4, hipMemcpyDeviceToHost));
            double md = 0, mref = 0;
            for (size_t i = 0; i < rx.size(); ++i) {
                md = std::max(md, (double)fabsf(rx[i] - r32[i]));
                mref = std::max(mref, (double)fabsf(r32[i]));
            }
            // fp64 errors on sampled outputs
            if (!host_loaded) {
                hx.resize((size_t)M * C);
                hw.resize((size_t)N * K);
                CK(hipMemcpy(hx.data(), x, hx.size() * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hw.data(), w, hw.size() * 4, hipMemcpyDeviceToHost));
                host_loaded = true;
            }
            double e32 = 0, ex3 = 0, s2 = 0, mx32 = 0, mxx3 = 0;
            unsigned st = 12345;
            for (int smp = 0; smp < 2000; ++smp) {
                st = st * 1664525u + 1013904223u;
                const int m = (int)(st % (unsigned)M);
                st = st * 1664525u + 1013904223u;
                const int n = (int)(st % (unsigned)N);
                const int img = m / (sh.H * sh.W), yy = (m / sh.W) % sh.H, xx = m % sh.W;
                double acc = 0;
                for (int t = 0; t < 9; ++t) {
                    const int sy = yy + t / 3 - 1, sx = xx + t % 3 - 1;
                    if (sy < 0 || sy >= sh.H || sx < 0 || sx >= sh.W) continue;
                    const float* xr = &hx[((size_t)(img * sh.H + sy) * sh.W + sx) * C];
                    const float* wr = &hw[(size_t)n * K + t * C];
                    for (int c = 0; c < C; ++c) acc += (double)xr[c] * wr[c];
                }
                const double d32 = r32[(size_t)m * N + n] - acc, dx3 = rx[(size_t)m * N + n] - acc;
                e32 += d32 * d32;
                ex3 += dx3 * dx3;
                s2 += acc * acc;
                mx32 = std::max(mx32, fabs(d32));
                mxx3 = std::max(mxx3, fabs(dx3));
            }
            printf("    x3 tile %d (%dx%d): %.3f ms %.1f TF/s (x%.2f)  max|x3-f32|/max|f32| %.2e  "
                   "rms err vs fp64: f32 %.2e x3 %.2e  max: f32 %.2e x3 %.2e\n",
                   tile, bm, bn, tx, fl / tx / 1e9, t32 / tx, md / mref, sqrt(e32 / s2), sqrt(ex3 / s2),
                   mx32, mxx3);
            fflush(stdout);
        }
        CK(hipFree(x));
        CK(hipFree(w));
        CK(hipFree(y32));
        CK(hipFree(yx3));
        CK(hipFree(x3));
        CK(hipFree(w3));
    }
    return 0;
}

static void probe_wgrad(int iters, void* zero) {
    Shape shapes[] = {
        {"L0 64x64 @256", 32, 256, 256, 64, 64},      {"L0 128x64 @256", 32, 256, 256, 128, 64},
        {"L1 128x128 @128", 32, 128, 128, 128, 128},  {"L1 256x128 @128", 32, 128, 128, 256, 128},
        {"L2 256x256 @64", 32, 64, 64, 256, 256},     {"L3 512x512 @32", 32, 32, 32, 512, 512},
        {"L4 1024x1024 @16", 32, 16, 16, 1024, 1024},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Shape& sh : shapes) {
        const int P = sh.N * sh.H * sh.W, CA = sh.Cin, CB = sh.Cout, Mw = 9 * CA, Nw = CB;
        // split-K over pixels: >= 1536 blocks of 128x128
        int splits = std::max(1, 1536 / std::max(1, (Mw / 128) * std::max(1, Nw / 128)));
        int pps = (P + splits - 1) / splits;
        pps = (pps + 255) / 256 * 256;
        splits = (P + pps - 1) / pps;
        float *x, *dz, *slab;
        uint16_t *x3, *dz3;
        CK(hipMalloc(&x, (size_t)P * CA * 4));
        CK(hipMalloc(&dz, (size_t)P * CB * 4));
        CK(hipMalloc(&x3, (size_t)P * CA * 6));
        CK(hipMalloc(&dz3, (size_t)P * CB * 6));
        CK(hipMalloc(&slab, (size_t)splits * Mw * Nw * 4));
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, x, (size_t)P * CA, 23u, 4.f, 1);
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, dz, (size_t)P * CB, 29u, 1e-3f, 0);
        CK((hipError_t)k_to_x3(x, CA, 0, CA, nullptr, nullptr, 0, P, x3, CA, 0, 0));
        CK((hipError_t)k_to_x3(dz, CB, 0, CB, nullptr, nullptr, 0, P, dz3, CB, 0, 0));
        WgradArgs w{};
        w.H = sh.H;
        w.W = sh.W;
        w.P = P;
        w.a = x;
        w.lda = CA;
        w.CA = CA;
        w.amode = G_CONV3;
        w.b = dz;
        w.ldb = CB;
        w.CB = CB;
        w.bmode = G_IDENT;
        w.Mw = Mw;
        w.Nw = Nw;
        w.pps = pps;
        w.splits = splits;
        w.slab = slab;
        w.xcd = 1;
        WgradArgs v = w;
        v.a = (const float*)x3;
        v.b = (const float*)dz3;
        v.zero16 = zero;
        const double fl = 2.0 * P * Mw * Nw;
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
        auto reduce = [&]() {
            std::vector<float> hs((size_t)splits * Mw * Nw);
            CK(hipMemcpy(hs.data(), slab, hs.size() * 4, hipMemcpyDeviceToHost));
            std::vector<double> r((size_t)Mw * Nw, 0.0);
            for (int sp = 0; sp < splits; ++sp)
                for (size_t i = 0; i < r.size(); ++i) r[i] += hs[(size_t)sp * Mw * Nw + i];
            return r;
        };
        // f32 library tiles: row3 128x128 (23) / 64x64 (20) where they fit, one-tap 128x128 (0)
        const int f32tiles[] = {23, 21, 22, 20, 0, 7};
        float tbest = 1e30f;
        int fbest = -1;
        std::vector<double> r32;
        for (int t : f32tiles) {
            int bm, bn, bkp;
            if (wgrad_tile_dims(t, &bm, &bn, &bkp)) continue;
            if (CA % bm || Nw % bn || pps % bkp) continue;
            CK(hipMemset(slab, 0, (size_t)splits * Mw * Nw * 4));
            if (launch_wgrad(w, t, 0) != 0) continue;
            const float tt = timeit([&] { return launch_wgrad(w, t, 0); });
            if (tt < tbest) {
                tbest = tt;
                fbest = t;
                r32 = reduce();
            }
        }
        printf("%-20s P=%d Mw=%d Nw=%d splits=%d  f32 wgrad tile %d: %.3f ms %.1f TF/s\n", sh.name, P, Mw,
               Nw, splits, fbest, tbest, fl / tbest / 1e9);
        std::vector<float> hx((size_t)P * CA), hd((size_t)P * CB);
        CK(hipMemcpy(hx.data(), x, hx.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hd.data(), dz, hd.size() * 4, hipMemcpyDeviceToHost));
        for (int tile = 0; tile <= 6; ++tile) {
            int bm = 0, bn = 0;
            if (wgrad_x3_tile_dims(tile, &bm, &bn) != 0 || CA % bm || Nw % bn) continue;
            CK(hipMemset(slab, 0, (size_t)splits * Mw * Nw * 4));
            const float tx = timeit([&] { return launch_wgrad_x3(v, tile, 0); });
            std::vector<double> rx = reduce();
            double md = 0, mref = 0;
            for (size_t i = 0; i < rx.size(); ++i) {
                md = std::max(md, fabs(rx[i] - r32[i]));
                mref = std::max(mref, fabs(r32[i]));
            }
            // fp64 reference on sampled weights: dW[(t, ci)][co] = sum_p x[p + tap][ci] dz[p][co]
            double e32 = 0, ex3 = 0, s2 = 0;
            unsigned st = 777;
            for (int smp = 0; smp < 64; ++smp) {
                st = st * 1664525u + 1013904223u;
                const int m = (int)(st % (unsigned)Mw);
                st = st * 1664525u + 1013904223u;
                const int n = (int)(st % (unsigned)Nw);
                const int t = m / CA, ci = m % CA;
                double acc = 0;
                for (int pix = 0; pix < P; ++pix) {
                    const int img = pix / (sh.H * sh.W), yy = (pix / sh.W) % sh.H, xx = pix % sh.W;
                    const int sy = yy + t / 3 - 1, sx = xx + t % 3 - 1;
                    if (sy < 0 || sy >= sh.H || sx < 0 || sx >= sh.W) continue;
                    acc += (double)hx[((size_t)(img * sh.H + sy) * sh.W + sx) * CA + ci] * hd[(size_t)pix * CB + n];
                }
                const double d32 = r32[(size_t)m * Nw + n] - acc, dx3 = rx[(size_t)m * Nw + n] - acc;
                e32 += d32 * d32;
                ex3 += dx3 * dx3;
                s2 += acc * acc;
            }
            printf("    x3 wgrad tile %d (%dx%d): %.3f ms %.1f TF/s (x%.2f)  max|x3-f32|/max|f32| %.2e  "
                   "rms err vs fp64: f32 %.2e x3 %.2e\n",
                   tile, bm, bn, tx, fl / tx / 1e9, tbest / tx, md / mref, sqrt(e32 / s2), sqrt(ex3 / s2));
            fflush(stdout);
        }
        CK(hipFree(x));
        CK(hipFree(dz));
        CK(hipFree(x3));
        CK(hipFree(dz3));
        CK(hipFree(slab));
    }
}
