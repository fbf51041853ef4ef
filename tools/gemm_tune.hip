// Tile tuning harness for the implicit-GEMM conv kernels (run on the GPU box).
// Includes kernels_gemm.hip directly, allocates one layer's operands with random data and
// times every instantiated tile on it, interleaved over rounds in ONE process
// (cdna_hip_programming.md §5.4 rule 24).  Prints TF/s per (shape, variant).
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_tune.hip -o gemm_tune
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <cmath>
#include <vector>

#include "../thyroid-nodule-image-segmentation-unet-ddti_amd/csrc/kernels_gemm.hip"

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

struct Shape { const char* name; int N, H, W, Cin, Cout; };

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    const int iters = 5;
    Shape shapes[] = {
        {"L0 64->64 @256", 32, 256, 256, 64, 64},
        {"L0 128->64 @256", 32, 256, 256, 128, 64},
        {"L1 128->128 @128", 32, 128, 128, 128, 128},
        {"L2 256->256 @64", 32, 64, 64, 256, 256},
        {"L3 512->512 @32", 32, 32, 32, 512, 512},
        {"L4 1024->1024 @16", 32, 16, 16, 1024, 1024},
    };
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
        const double flop = 2.0 * M * sh.Cout * 9.0 * sh.Cin;
        // forward (CONV3 + affine + stats) per tile, dgrad (CONV3 store) per tile
        const int NT = 13, NW = 17;
        std::vector<std::vector<double>> best(2, std::vector<double>(NT, 0));
        std::vector<std::vector<double>> rerr(2, std::vector<double>(NT, 0));
        std::vector<float> rref[2];
        float* xo = dalloc((size_t)M * sh.Cin, 9, 0.f);
        for (int r = 0; r < rounds; ++r) {
            for (int tile = 0; tile < NT; ++tile) {
                if (tile == 6) continue;  // bf16-oriented BK64 tile
                for (int op = 0; op < 2; ++op) {
                    RowGemmArgs g{};
                    g.H = sh.H; g.W = sh.W; g.M = M;
                    if (op == 0) {
                        g.N = sh.Cout; g.K = 9 * sh.Cin; g.a = x; g.lda = sh.Cin; g.C = sh.Cin;
                        g.ascale = sc; g.ashift = shf; g.emode = E_BIAS_RELU_STATS; g.bias = bias;
                        g.stats = st; g.out = y; g.ldo = sh.Cout;
                    } else {
                        g.N = sh.Cin; g.K = 9 * sh.Cout; g.a = dz; g.lda = sh.Cout; g.C = sh.Cout;
                        g.emode = E_STORE; g.out = xo; g.ldo = sh.Cin;
                    }
                    g.amode = G_CONV3; g.bt = w;
                    if (launch_rowgemm(g, tile, 0) != 0) continue;
                    if (r == 0) {  // output vs the first tile that ran
                        CK(hipDeviceSynchronize());
                        const size_t no = (size_t)M * (op ? sh.Cin : sh.Cout);
                        std::vector<float> h(no);
                        CK(hipMemcpy(h.data(), op ? xo : y, no * 4, hipMemcpyDeviceToHost));
                        if (rref[op].empty()) {
                            rref[op] = h;
                        } else {
                            double md = 0, mx = 0;
                            for (size_t i = 0; i < no; ++i) {
                                md = std::max(md, (double)std::abs(h[i] - rref[op][i]));
                                mx = std::max(mx, (double)std::abs(rref[op][i]));
                            }
                            rerr[op][tile] = md / (mx > 0 ? mx : 1);
                        }
                    }
                    CK(hipEventRecord(e0, 0));
                    for (int it = 0; it < iters; ++it) launch_rowgemm(g, tile, 0);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    const double tf = flop * iters / (ms * 1e-3) / 1e12;
                    if (tf > best[op][tile]) best[op][tile] = tf;
                }
            }
            // wgrad tiles
        }
        for (int op = 0; op < 2; ++op) {
            printf("%-20s %-5s", sh.name, op ? "dgrad" : "fwd");
            for (int tile = 0; tile < NT; ++tile) printf("  t%d %6.1f", tile, best[op][tile]);
            printf("\n%-20s %-5s rel.err:", sh.name, op ? "dgrad" : "fwd");
            for (int tile = 0; tile < NT; ++tile) printf("  t%d %.1e", tile, rerr[op][tile]);
            printf("\n");
        }
        // wgrad over the tile table
        // ids 0..7: pixel-major LDS (wgrad_kernel); 10, 15: channel-major (wgradT_kernel);
        // 20..24: one row of taps per block (wgrad_row3_kernel); wx: XCD-contiguous order
        const int wids[NW] = {0, 1, 2, 3, 4, 5, 6, 7, 10, 15, 20, 21, 22, 23, 24, 7, 0};
        const int wx[NW] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1};
        double wb[NW] = {};
        double werr[NW] = {};
        int wsplit[NW] = {};
        std::vector<double> wref;
        float* slab = nullptr;
        size_t slab_n = 0;
        for (int r = 0; r < rounds; ++r)
            for (int v = 0; v < NW; ++v) {
                int bm, bn, bkp;
                if (wgrad_tile_dims(wids[v], &bm, &bn, &bkp) != 0) continue;
                if (sh.Cin % bm || sh.Cout % bn) continue;
                const long tiles = (long)(9 * sh.Cin / (bm * wgrad_tile_taps(wids[v]))) * (sh.Cout / bn);
                long sp = (2048 + tiles - 1) / tiles;
                if (sp > M / (8 * bkp)) sp = M / (8 * bkp);
                if (sp < 1) sp = 1;
                long pps = ((M + sp - 1) / sp + 127) / 128 * 128;
                const int splits = (int)((M + pps - 1) / pps);
                const size_t need = (size_t)splits * 9 * sh.Cin * sh.Cout;
                if (need > slab_n) {
                    if (slab) CK(hipFree(slab));
                    CK(hipMalloc(&slab, need * 4));
                    slab_n = need;
                }
                WgradArgs a{};
                a.H = sh.H; a.W = sh.W; a.P = M; a.a = x; a.lda = sh.Cin; a.CA = sh.Cin;
                a.amode = G_CONV3; a.ascale = sc; a.ashift = shf; a.b = dz; a.ldb = sh.Cout;
                a.CB = sh.Cout; a.bmode = G_IDENT; a.Mw = 9 * sh.Cin; a.Nw = sh.Cout;
                a.pps = (int)pps; a.splits = splits; a.slab = slab; a.xcd = wx[v];
                if (launch_wgrad(a, wids[v], 0) != 0) continue;
                if (r == 0) {  // split-reduced result vs the first tile that ran
                    CK(hipDeviceSynchronize());
                    const size_t nw = (size_t)9 * sh.Cin * sh.Cout;
                    std::vector<float> h((size_t)splits * nw);
                    CK(hipMemcpy(h.data(), slab, h.size() * 4, hipMemcpyDeviceToHost));
                    std::vector<double> red(nw, 0.0);
                    for (int sp2 = 0; sp2 < splits; ++sp2)
                        for (size_t i = 0; i < nw; ++i) red[i] += h[(size_t)sp2 * nw + i];
                    if (wref.empty()) {
                        wref = red;
                    } else {
                        double md = 0, mx = 0;
                        for (size_t i = 0; i < nw; ++i) {
                            md = std::max(md, std::abs(red[i] - wref[i]));
                            mx = std::max(mx, std::abs(wref[i]));
                        }
                        werr[v] = md / (mx > 0 ? mx : 1);
                    }
                }
                CK(hipEventRecord(e0, 0));
                for (int it = 0; it < iters; ++it) launch_wgrad(a, wids[v], 0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double tf = flop * iters / (ms * 1e-3) / 1e12;
                if (tf > wb[v]) wb[v] = tf;
                wsplit[v] = splits;
            }
        printf("%-20s wgrad", sh.name);
        for (int v = 0; v < NW; ++v)
            printf("  w%d%s/s%d %6.1f", wids[v], wx[v] ? "x" : "", wsplit[v], wb[v]);
        printf("\n%-20s wgrad rel.err vs first tile:", sh.name);
        for (int v = 0; v < NW; ++v) printf("  w%d %.1e", wids[v], werr[v]);
        printf("\n");
        fflush(stdout);
        CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(sc)); CK(hipFree(shf)); CK(hipFree(bias));
        CK(hipFree(y)); CK(hipFree(st)); CK(hipFree(dz)); CK(hipFree(xo));
        if (slab) CK(hipFree(slab));
    }
    return 0;
}
