// Bandwidth-bound kernels around the MFMA convolutions: weight repacking, the Cin=1 first
// conv, BatchNorm statistics / finalisation / backward, 2x2 max-pool, the 1x1 head, the
// BCE + Dice + FocalTversky loss, AdamW and the eval mask readout.
//
// All reductions are deterministic: fixed per-block partial sums followed by fixed-order
// reductions (no float atomics), so two runs of the same inputs are bit-identical.
// Layout everywhere: NHWC, channel stride `ld`, channel offset `off` (concat slices).
#include "kernels_misc.h"
#include "gemm_common.h"  // Pix, decode, pix_advance (and x3_split.h)

namespace {

// one AdamW element (torch optim/adam.py _single_tensor_adam, documented at adamw_kernel below)
__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v,
                                           const AdamwScalars& a) {
#pragma clang fp contract(off)
    if (a.gscale != 1.f) g = g * a.gscale;
    p = p * a.decay;
    const float d = g - m;
    m = a.lerp_small ? __builtin_fmaf(a.w1, d, m) : __builtin_fmaf(a.w1 - 1.f, d, g);
    v = v * a.b2;
    v = __builtin_fmaf(a.w2 * g, g, v);
    const float den = __builtin_sqrtf(v) / a.bc2_sqrt + a.eps;
    p = p + (a.neg_step * m) / den;
}

// (r06) the fused AdamW of the packed weights (unet_adamw_repack): the pack kernel updates
// each weight tile from the arena-shaped p / g / m / v before it packs it, so the forward reads
// no f32 weight again.  Pointers point at the tensor's first element.
struct AdamTile {
    float* p;
    const float* g;
    float* m;
    float* v;
    AdamwScalars a;
};
// N elements of one thread at once: every load of the batch issues before the first store
// (element by element, each element's p / m / v stores held the next element's loads back:
// the fused kernel then ran slower than unet_adamw + the repack)
template <int N>
__device__ __forceinline__ void adam_batch(const AdamTile& t, const int64_t (&ix)[N], const bool (&ok)[N],
                                           float (&out)[N]) {
    float p[N], g[N], m[N], v[N];
#pragma unroll
    for (int k = 0; k < N; ++k)
        if (ok[k]) {
            p[k] = t.p[ix[k]];
            g[k] = t.g[ix[k]];
            m[k] = t.m[ix[k]];
            v[k] = t.v[ix[k]];
        }
#pragma unroll
    for (int k = 0; k < N; ++k)
        if (ok[k]) {
            adamw_elem(p[k], g[k], m[k], v[k], t.a);
            t.p[ix[k]] = p[k];
            t.m[ix[k]] = m[k];
            t.v[ix[k]] = v[k];
            out[k] = p[k];
        }
}
template <bool ADAM>
__device__ __forceinline__ float pack_load(const float* __restrict__ w, const AdamTile& t, int64_t i) {
    if constexpr (ADAM) {
        float p = t.p[i], m = t.m[i], v = t.v[i];
        adamw_elem(p, t.g[i], m, v, t.a);
        t.p[i] = p;
        t.m[i] = m;
        t.v[i] = v;
        return p;
    } else {
        return w[i];
    }
}

// -------------------------------------------------------------------------------------
// Weight packing.  torch Conv2d weight W[co][ci][ky][kx] (models/model.py:36,39):
//   fwd  : Wf[co][tap][ci]                    (Bt of the forward row-GEMM, k = tap*Cin+ci)
//   dgrad: Wd[ci][tap'][co] = W[co][ci][8-tap'] (flipped taps, k = tap'*Cout+co)
// torch ConvTranspose2d weight W[ci][co][a][b] (models/model.py:19,49):
//   fwd  : Tf[(ab*Cout+co)][ci]
//   dgrad: Td[ci][ab*Cout+co]
// -------------------------------------------------------------------------------------
// OUT = float (f32 MFMA images) or __bf16 (bf16 MFMA images, round to nearest even).
// 3x3: one block per LDS tile of 32 co x 32 ci x 9 taps: the torch rows (ci, tap
// contiguous) are read with unit stride, and both images are written as 32-element runs
// (ci runs of Wf, co runs of Wd) rather than an element-wise stride-9 / stride-9*Cout
// scatter.  Row stride 289 floats: both LDS read patterns are conflict-free.
template <class OUT, bool ADAM = false>
__device__ void pack_conv3_tile(const float* __restrict__ w, OUT* __restrict__ wf,
                                OUT* __restrict__ wd, int cin, int cout, int ci0, int co0,
                                float* tile, const AdamTile& at = AdamTile{}) {
    constexpr int T = 32, RS = T * 9 + 1;
    const int nci = min(T, cin - ci0), nco = min(T, cout - co0);
    const int tid = threadIdx.x;
    if (nci == T && nco == T) {
        // full tile: 36 independent loads per thread in flight before the LDS stores
        constexpr int NK = T * T * 9 / 256;
        float v[NK];
        if constexpr (ADAM) {
            constexpr int CH = 12;  // 48 loads in flight per thread
#pragma unroll
            for (int k0 = 0; k0 < NK; k0 += CH) {
                int64_t ix[CH];
                bool ok[CH];
                float o[CH];
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    const int e = tid + 256 * (k0 + k);
                    const int co_l = e / (T * 9), r = e - co_l * (T * 9);
                    ix[k] = ((int64_t)(co0 + co_l) * cin + ci0) * 9 + r;
                    ok[k] = true;
                }
                adam_batch<CH>(at, ix, ok, o);
#pragma unroll
                for (int k = 0; k < CH; ++k) v[k0 + k] = o[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int e = tid + 256 * k;  // e = co_l * 288 + (ci_l * 9 + tap)
                const int co_l = e / (T * 9), r = e - co_l * (T * 9);
                v[k] = w[((int64_t)(co0 + co_l) * cin + ci0) * 9 + r];
            }
        }
#pragma unroll
        for (int k = 0; k < T * T * 9 / 256; ++k) {
            const int e = tid + 256 * k;
            const int co_l = e / (T * 9), r = e - co_l * (T * 9);
            tile[co_l * RS + r] = v[k];
        }
    } else {
        for (int e = tid; e < T * T * 9; e += 256) {  // e = co_l * 288 + (ci_l * 9 + tap)
            const int co_l = e / (T * 9), r = e - co_l * (T * 9);
            if (co_l < nco && r < nci * 9)
                tile[co_l * RS + r] = pack_load<ADAM>(w, at, ((int64_t)(co0 + co_l) * cin + ci0) * 9 + r);
        }
    }
    __syncthreads();
    const int l = tid & 31, g = tid >> 5;  // 8 groups of 32 lanes
    // Wf[co][tap][ci]: rows (co_l, tap), lanes over ci
    for (int row = g; row < T * 9; row += 8) {
        const int co_l = row / 9, tap = row - co_l * 9;
        if (co_l < nco && l < nci)
            wf[((int64_t)(co0 + co_l) * 9 + tap) * cin + ci0 + l] = (OUT)tile[co_l * RS + l * 9 + tap];
    }
    if (!wd) return;
    // Wd[ci][8-tap][co]: rows (ci_l, tap), lanes over co
    for (int row = g; row < T * 9; row += 8) {
        const int ci_l = row / 9, tap = row - ci_l * 9;
        if (ci_l < nci && l < nco)
            wd[((int64_t)(ci0 + ci_l) * 9 + (8 - tap)) * cout + co0 + l] =
                (OUT)tile[l * RS + ci_l * 9 + tap];
    }
}

// ConvT: one block per LDS tile of 32 ci x 32 co x 4 taps (ab).  The torch rows (co, ab
// contiguous per ci) are read with unit stride; Tf rows (ab, co) are written as 32-element ci
// runs and Td rows (ci) as 32-element co runs per ab (the element-wise form scattered every
// Tf element cin apart).  LDS tile [ci_l][ab][co_l], ab stride 40, row stride 161 floats:
// the fill (lanes over (co_l, ab)), the Tf read (lanes over ci) and the Td read (lanes over
// co) are all conflict-free (the r02 [ci_l][co_l * 4 + ab] image read Td at a 4-float lane
// stride: 4-way conflicts, 4.19 M extra LDS cycles per config-4 repack).
template <class OUT, bool ADAM = false>
__device__ void pack_convT_tile(const float* __restrict__ w, OUT* __restrict__ tf,
                                OUT* __restrict__ td, int cin, int cout, int co0, int ci0,
                                float* tile, const AdamTile& at = AdamTile{}) {
    constexpr int T = 32, AS = 40, RS = 4 * AS + 1;  // tile: [ci_l][ab][co_l]
    const int nci = min(T, cin - ci0), nco = min(T, cout - co0);
    const int tid = threadIdx.x;
    if constexpr (ADAM) {  // 16 elements per thread, loads batched (adam_batch)
        constexpr int NK = T * T * 4 / 256;
        int64_t ix[NK];
        bool ok[NK];
        float o[NK];
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int e = tid + 256 * k;
            const int ci_l = e / (T * 4), r = e - ci_l * (T * 4);
            ok[k] = ci_l < nci && r < nco * 4;
            ix[k] = ((int64_t)(ci0 + ci_l) * cout + co0) * 4 + r;
        }
        adam_batch<NK>(at, ix, ok, o);
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int e = tid + 256 * k;
            const int ci_l = e / (T * 4), r = e - ci_l * (T * 4);
            if (ok[k]) tile[ci_l * RS + (r & 3) * AS + (r >> 2)] = o[k];
        }
    } else {
        for (int e = tid; e < T * T * 4; e += 256) {  // e = ci_l * 128 + (co_l * 4 + ab)
            const int ci_l = e / (T * 4), r = e - ci_l * (T * 4);
            if (ci_l < nci && r < nco * 4)
                tile[ci_l * RS + (r & 3) * AS + (r >> 2)] = w[((int64_t)(ci0 + ci_l) * cout + co0) * 4 + r];
        }
    }
    __syncthreads();
    const int l = tid & 31, g = tid >> 5;  // 8 groups of 32 lanes
    // Tf[(ab * cout + co)][ci]: rows (ab, co_l), lanes over ci
    for (int row = g; row < 4 * T; row += 8) {
        const int ab = row / T, co_l = row - ab * T;
        if (co_l < nco && l < nci)
            tf[((int64_t)ab * cout + co0 + co_l) * cin + ci0 + l] = (OUT)tile[l * RS + ab * AS + co_l];
    }
    if (!td) return;
    // Td[ci][ab * cout + co]: rows (ci_l, ab), lanes over co
    for (int row = g; row < 4 * T; row += 8) {
        const int ci_l = row >> 2, ab = row & 3;
        if (ci_l < nci && l < nco)
            td[(int64_t)(ci0 + ci_l) * 4 * cout + ab * cout + co0 + l] = (OUT)tile[ci_l * RS + ab * AS + l];
    }
}

// Every 3x3 / ConvT weight image of the network in ONE launch (the per-layer launches were
// 21 small grids per step, most of them too small to fill the chip): block b runs tile
// b - block0 of the last job with block0 <= b; the job table travels as a kernel argument.
// ADAM (r06, unet_adamw_repack): each tile is first AdamW-updated in place (p, m, v of the
// arena-shaped pointers in `ad`, the same adamw_elem as adamw_kernel: bit-identical), and the
// updated values are what it packs.
struct AdamArena {
    float* p;
    const float* g;
    float* m;
    float* v;
};
template <class OUT, bool ADAM = false>
__global__ __launch_bounds__(256) void pack_all_kernel(PackJobs jobs, const float* __restrict__ prm,
                                                       float* __restrict__ pack, AdamArena ad,
                                                       AdamwScalars a) {
    __shared__ float tile[32 * (32 * 9 + 1)];
    const int b = blockIdx.x;
    int j = 0;
    for (int k = 1; k < jobs.n; ++k)
        if (jobs.j[k].block0 <= b) j = k;
    const PackJob& J = jobs.j[j];
    const int local = b - J.block0, ix = local % J.tx, iy = local / J.tx;
    OUT* f = (OUT*)(pack + J.f);
    OUT* d = J.d >= 0 ? (OUT*)(pack + J.d) : nullptr;
    AdamTile at{};
    if constexpr (ADAM) at = AdamTile{ad.p + J.w, ad.g + J.w, ad.m + J.w, ad.v + J.w, a};
    const float* w = ADAM ? nullptr : prm + J.w;
    if (J.kind == 0)
        pack_conv3_tile<OUT, ADAM>(w, f, d, J.cin, J.cout, ix * 32, iy * 32, tile, at);
    else
        pack_convT_tile<OUT, ADAM>(w, f, d, J.cin, J.cout, ix * 32, iy * 32, tile, at);
}

// (r06) AdamW of the arena elements the fused pack does not cover (biases, BN affine, the
// first conv and the head): a grid-stride walk over the concatenation of the ranges, each
// index mapped to its range by binary search in the table (the kernel argument)
__global__ __launch_bounds__(256) void adamw_ranges_kernel(AdamRanges t, AdamArena ad, AdamwScalars a) {
    const int64_t total = t.cum[t.n];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = t.n - 1;
        while (lo < hi) {  // the last range with cum <= i
            const int mid = (lo + hi + 1) >> 1;
            if (t.cum[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        const int64_t e = t.off[lo] + (i - t.cum[lo]);
        float p = ad.p[e], m = ad.m[e], v = ad.v[e];
        adamw_elem(p, ad.g[e], m, v, a);
        ad.p[e] = p;
        ad.m[e] = m;
        ad.v[e] = v;
    }
}

// 1x1 conv weight W[co][ci] -> its dgrad image Wt[ci][co] (models/mod.py:83 skip)
__global__ void pack_1x1_t_kernel(const float* __restrict__ w, float* __restrict__ wt, int cin,
                                  int cout) {
    const int64_t n = (int64_t)cin * cout;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int ci = (int)(i % cin), co = (int)(i / cin);
        wt[(int64_t)ci * cout + co] = w[i];
    }
}

// Block-level combine of per-thread channel partials.  Threads are laid out as
// (row group g = tid / tpr, channel quad q = tid % tpr); acc[NV] holds NV quantities per
// channel-quad.  Writes out[v*C + 4q + j] for row group 0.  smem: 256*NV*4 floats.
template <int NV>
__device__ void block_combine(const f32x4 (&acc)[NV], int tpr, int C, float* out, float* smem) {
    const int tid = threadIdx.x;
    const int g = tid / tpr, q = tid % tpr;
    const int groups = blockDim.x / tpr;
    f32x4* s = (f32x4*)smem;
#pragma unroll
    for (int v = 0; v < NV; ++v) s[v * blockDim.x + tid] = acc[v];
    __syncthreads();
    if (g == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            f32x4 a = s[v * blockDim.x + q];
            for (int k = 1; k < groups; ++k) a += s[v * blockDim.x + k * tpr + q];
            *(f32x4*)(out + v * C + 4 * q) = a;
        }
    }
}

// f64 variant (BN-backward partials, where downstream differences of the sums cancel).
// smem holds component (v, j) of every thread contiguously ([v][j][thread]): consecutive
// lanes touch consecutive doubles, conflict-free (the [thread][v][j] order put lanes 32 B
// apart, an 8-way bank conflict on every store and load: 499,712 extra LDS cycles per
// max-pool backward launch in r02).  Same summation order as before: bit-identical.
// Row groups: the nt / tpr complete ones (threads past them hold zeros and are not read);
// only the first nq channel quads are written (a last pass over C / 4 > 256 quads).
template <int NV>
__device__ void block_combine_d(const double (&acc)[NV][4], int tpr, int C, float* out,
                                double* smem, int nq = 1 << 30) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const int g = tid / tpr, q = tid % tpr;
    const int groups = nt / tpr;
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int j = 0; j < 4; ++j) smem[(v * 4 + j) * nt + tid] = acc[v][j];
    __syncthreads();
    if (g == 0 && q < nq) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double a = 0.0;
                for (int k = 0; k < groups; ++k) a += smem[(v * 4 + j) * nt + k * tpr + q];
                out[v * C + 4 * q + j] = (float)a;
            }
    }
}

// -------------------------------------------------------------------------------------
// Conv2d(1 -> C, 3x3, pad 1) + bias + ReLU + BN partials (encoder1.0, model.py:10,36-37),
// or bias-free without ReLU (encoders.0.0 of mod.py:45).  K = 9 is too small for MFMA;
// one thread computes 4 channels of one pixel.
// -------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void conv_first_fwd_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias,
                                                            float* __restrict__ y, int P, int H,
                                                            int W, int C, int relu,
                                                            float* partial) {
    __shared__ __attribute__((aligned(16))) float smem[256 * 2 * 4];
    extern __shared__ float xs[];  // x[r0 - W - 1, r1 + W + 1): every tap of the block's pixels
    const int tpr = C / 4, rpp = 256 / tpr;
    const int q = threadIdx.x % tpr, g = threadIdx.x / tpr;
    float wr[4][9];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 9; ++t) wr[j][t] = w[(4 * q + j) * 9 + t];
    const f32x4 b = bias ? *(const f32x4*)(bias + 4 * q) : f32x4{0, 0, 0, 0};
    f32x4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const int per = (P + gridDim.x - 1) / gridDim.x;
    const int r0 = blockIdx.x * per;
    const int r1 = min(P, r0 + per);
    // in_channels = 1: the image is one float per pixel, so the taps of the block's pixel range
    // are one contiguous slice of x (the 16 lanes of a pixel then read it from LDS instead of
    // issuing 9 global loads each)
    const int xb = r0 - W - 1, xn = per + 2 * W + 2;
    for (int i = threadIdx.x; i < xn; i += blockDim.x) {
        const int gi = xb + i;
        xs[i] = (gi >= 0 && gi < P) ? x[gi] : 0.f;
    }
    __syncthreads();
    // U pixels per trip (m, m + rpp, ..., their 9 U image loads issued together), pixel
    // coordinates walked incrementally: no integer division per pixel.  Each thread still sums
    // its pixels in increasing m, so the partials are those of one pixel per trip.
    constexpr int U = 4;
    Pix at[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        at[u] = decode(min(r0 + g, P - 1), H, W);
        pix_advance(at[u], u * rpp, H, W);
    }
    for (int m0 = r0 + g; m0 < r1; m0 += U * rpp) {
        float xv[U][9];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int sy = at[u].y + tap / 3 - 1, sx = at[u].x + tap % 3 - 1;
                const bool ok = sy >= 0 && sy < H && sx >= 0 && sx < W && m0 + u * rpp < r1;
                xv[u][tap] = ok ? xs[m0 + u * rpp + (tap / 3 - 1) * W + tap % 3 - 1 - xb] : 0.f;
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int m = m0 + u * rpp;
            pix_advance(at[u], U * rpp, H, W);
            if (m >= r1) continue;
            f32x4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float s = 0.f;
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) s = fmaf(xv[u][tap], wr[j][tap], s);
                o[j] = relu ? fmaxf(s + b[j], 0.f) : s + b[j];
            }
            __builtin_nontemporal_store(o, (f32x4*)(y + (int64_t)m * C + 4 * q));
            acc[0] += o;
            acc[1] += o * o;
        }
    }
    block_combine<2>(acc, tpr, C, partial + (int64_t)blockIdx.x * 2 * C, smem);
}

// dW[co][tap] = sum_p x_tap(p) dz[p][co], db[co] = sum_p dz[p][co]; partial [G][10*C]
// laid out as [tap][C] for tap 0..8 then bias.
__global__ __launch_bounds__(256) void conv_first_wgrad_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ dout,
                                                              const float* __restrict__ y,
                                                              const float* __restrict__ coef,
                                                              int P, int H, int W, int C,
                                                              int mask, float* partial) {
    __shared__ __attribute__((aligned(16))) float smem[256 * 10 * 4];
    extern __shared__ float xs[];  // x[r0 - W - 1, r1 + W + 1), as conv_first_fwd_kernel
    const int tpr = C / 4, rpp = 256 / tpr;
    const int q = threadIdx.x % tpr, g = threadIdx.x / tpr;
    f32x4 acc[10];
#pragma unroll
    for (int v = 0; v < 10; ++v) acc[v] = f32x4{0, 0, 0, 0};
    const int per = (P + gridDim.x - 1) / gridDim.x;
    const int r0 = blockIdx.x * per;
    const int r1 = min(P, r0 + per);
    const int xb = r0 - W - 1, xn = per + 2 * W + 2;
    for (int i = threadIdx.x; i < xn; i += blockDim.x) {
        const int gi = xb + i;
        xs[i] = (gi >= 0 && gi < P) ? x[gi] : 0.f;
    }
    __syncthreads();
    const f32x4 ka = *(const f32x4*)(coef + 4 * q), kb = *(const f32x4*)(coef + C + 4 * q);
    const f32x4 kc = *(const f32x4*)(coef + 2 * C + 4 * q), km = *(const f32x4*)(coef + 3 * C + 4 * q);
    Pix at = decode(min(r0 + g, P - 1), H, W);
    // two pixels per trip (both pixels' loads issued first); each thread still adds its pixels
    // in increasing m, so the partials are bit-identical to one pixel per trip
    auto accum = [&](int m, const Pix& pq, const f32x4& dv, const f32x4& yv) {
        const f32x4 dd = bn_dz4(ka, dv, kb, yv, km, kc);
        f32x4 d;
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = (!mask || yv[j] > 0.f) ? dd[j] : 0.f;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int sy = pq.y + tap / 3 - 1, sx = pq.x + tap % 3 - 1;
            const bool ok = sy >= 0 && sy < H && sx >= 0 && sx < W;
            const float xv = ok ? xs[m + (tap / 3 - 1) * W + tap % 3 - 1 - xb] : 0.f;
            acc[tap] += xv * d;
        }
        acc[9] += d;
    };
    for (int m = r0 + g; m < r1; m += 2 * rpp) {
        const int m2 = m + rpp;
        const Pix p1 = at;
        pix_advance(at, rpp, H, W);
        const Pix p2 = at;
        pix_advance(at, rpp, H, W);
        const f32x4 dv = *(const f32x4*)(dout + (int64_t)m * C + 4 * q);
        const f32x4 yv = *(const f32x4*)(y + (int64_t)m * C + 4 * q);
        f32x4 dw{0, 0, 0, 0}, yw{0, 0, 0, 0};
        if (m2 < r1) {
            dw = *(const f32x4*)(dout + (int64_t)m2 * C + 4 * q);
            yw = *(const f32x4*)(y + (int64_t)m2 * C + 4 * q);
        }
        accum(m, p1, dv, yv);
        if (m2 < r1) accum(m2, p2, dw, yw);
    }
    block_combine<10>(acc, tpr, C, partial + (int64_t)blockIdx.x * 10 * C, smem);
}

// -------------------------------------------------------------------------------------
// Deterministic reductions of partial rows.
// -------------------------------------------------------------------------------------
// out[g][c] = sum_{r in slice g} in[r][c], c < ncols.  grid (ceil(ncols/256), G).
__global__ void reduce_rows_kernel(const float* __restrict__ in, int R, int ncols,
                                   float* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncols) return;
    const int G = gridDim.y, g = blockIdx.y;
    const int per = (R + G - 1) / G;
    const int r0 = g * per, r1 = min(R, r0 + per);
    float s = 0.f;
    for (int r = r0; r < r1; ++r) s += in[(int64_t)r * ncols + c];
    out[(int64_t)g * ncols + c] = s;
}

// Column sums of G partial rows for the 64 columns of this block: thread (cx, ry) sums rows
// ry, ry+16, ... (8 loads in flight), then the 16 row groups are added in fixed order.
// Returns the column total in threads ry == 0 (others return 0).  blockDim = (64, 16).
template <int NQ>
__device__ void colsum16(const float* __restrict__ part, int G, int stride, int qstride, int col,
                         bool ok, double (&out)[NQ]) {
    __shared__ double red[NQ][16][64];
    const int cx = threadIdx.x, ry = threadIdx.y;
    double acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
    if (ok) {
        int g = ry;
        for (; g + 16 * 7 < G; g += 16 * 8) {
            float v[NQ][8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int q = 0; q < NQ; ++q)
                    v[q][u] = part[(int64_t)(g + 16 * u) * stride + q * qstride + col];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int q = 0; q < NQ; ++q) acc[q] += v[q][u];
        }
        for (; g < G; g += 16)
#pragma unroll
            for (int q = 0; q < NQ; ++q) acc[q] += part[(int64_t)g * stride + q * qstride + col];
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) red[q][ry][cx] = acc[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        double t = 0.0;
        if (ry == 0)
            for (int k = 0; k < 16; ++k) t += red[q][k][cx];
        out[q] = t;
    }
}

// BatchNorm2d train finalisation (torch/nn/modules/batchnorm.py semantics): batch mean,
// biased var for normalisation, running stats r = (1-m) r + m * stat with unbiased var.
// Emits the fused affine (scale, shift) consumers apply in their load path, and keeps
// mean / invstd for the backward.
__device__ void bn_train_final(int c, int C, const double (&sq)[2], double count,
                               const float* __restrict__ gamma, const float* __restrict__ beta,
                               float* rmean, float* rvar, int64_t* nbt, float momentum, float eps,
                               float* __restrict__ scale, float* __restrict__ shift,
                               float* __restrict__ mean_out, float* __restrict__ invstd_out) {
    if (c == 0 && nbt) *nbt += 1;
    if (c >= C) return;
    const double s = sq[0], q = sq[1];
    const double mean = s / count;
    double var = q / count - mean * mean;
    if (var < 0) var = 0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = gamma[c] * invstd;
    scale[c] = sc;
    shift[c] = beta[c] - (float)mean * sc;
    mean_out[c] = (float)mean;
    invstd_out[c] = invstd;
    if (rmean) {
        const double unb = count > 1 ? var * count / (count - 1) : var;
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mean;
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
}

__global__ void bn_finalize_train_kernel(const float* __restrict__ part, int G, int C,
                                         double count, const float* __restrict__ gamma,
                                         const float* __restrict__ beta, float* rmean,
                                         float* rvar, int64_t* nbt, float momentum, float eps,
                                         float* __restrict__ scale, float* __restrict__ shift,
                                         float* __restrict__ mean_out,
                                         float* __restrict__ invstd_out) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    double sq[2];
    colsum16<2>(part, G, 2 * C, C, c, c < C, sq);
    if (threadIdx.y != 0) return;
    bn_train_final(c, C, sq, count, gamma, beta, rmean, rvar, nbt, momentum, eps, scale, shift,
                   mean_out, invstd_out);
}

__global__ void bn_finalize_eval_kernel(int C, const float* __restrict__ gamma,
                                        const float* __restrict__ beta,
                                        const float* __restrict__ rmean,
                                        const float* __restrict__ rvar, float eps,
                                        float* __restrict__ scale, float* __restrict__ shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float invstd = 1.f / sqrtf(rvar[c] + eps);
    const float sc = gamma[c] * invstd;
    scale[c] = sc;
    shift[c] = beta[c] - rmean[c] * sc;
}

// -------------------------------------------------------------------------------------
// MaxPool2d(2) of BN(y) (model.py:17,56-58).  BN is applied before the max (the two do not
// commute when gamma < 0).  idx keeps the winning window position with torch's tie rule:
// scan order (0,0),(0,1),(1,0),(1,1), first strict maximum wins.
// -------------------------------------------------------------------------------------
// relu: BN -> ReLU order (mod.py:46-47); the max of ReLU(v) is ReLU(max v) and the winner
// only differs where every candidate is <= 0, where the ReLU blocks its gradient anyway.
// One pooled pixel: BN affine of the four window values, torch's tie rule, optional ReLU.
// (r06) PoolImg: operand images the pass also writes from the values it forms anyway -- the
// bf16 pooled image of the next encoder conv (pool16, [pooled pixels][C]) and, at full
// resolution, the skip half of the decoder conv's kept image of this level (skip16: bf16
// [pixels][ldk] at channel offset so; skip3: its x3 split, [pixels][ldk / 32][3][32]) with the
// affine and ReLU k_to_bf16 / k_to_x3 would apply (same fma, same RNE): their prep passes then
// have nothing left to convert.
struct PoolImg {
    uint16_t* pool16;
    uint16_t* skip16;
    uint16_t* skip3;
    int ldk, so;
};
__device__ __forceinline__ void maxpool_px(const float* __restrict__ y, int ld, int off, f32x4 sc,
                                           f32x4 sh, int relu, int H, int W, int img, int yo,
                                           int xo, int c, float* __restrict__ out,
                                           uint8_t* __restrict__ idx, int64_t o,
                                           uint16_t* __restrict__ out3 = nullptr, int C = 0,
                                           PoolImg pi = PoolImg{}) {
    typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
    f32x4 best;
    uint32_t bi = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t pin = ((int64_t)img * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1);
        const f32x4 yv = *(const f32x4*)(y + pin * ld + off + c);
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = __builtin_fmaf(yv[j], sc[j], sh[j]);
        if (pi.skip16 || pi.skip3) {  // the skip half's operand image: op(BN(y)) at this pixel
            f32x4 t = v;
            if (relu)
#pragma unroll
                for (int j = 0; j < 4; ++j) t[j] = fmaxf(t[j], 0.f);
            const int cc = pi.so + c;
            if (pi.skip16) {
                u16x4 b;
#pragma unroll
                for (int j = 0; j < 4; ++j) b[j] = __builtin_bit_cast(uint16_t, (__bf16)t[j]);
                *(u16x4*)(pi.skip16 + pin * pi.ldk + cc) = b;
            }
            if (pi.skip3) {
                u16x4 h, m, l;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    uint16_t hj, mj, lj;
                    x3_split(t[j], X3CvtDev{}, hj, mj, lj);
                    h[j] = hj;
                    m[j] = mj;
                    l[j] = lj;
                }
                uint16_t* d = pi.skip3 + pin * 3 * pi.ldk + (cc >> 5) * 96 + (cc & 31);
                *(u16x4*)d = h;
                *(u16x4*)(d + 32) = m;
                *(u16x4*)(d + 64) = l;
            }
        }
        if (k == 0) {
            best = v;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (v[j] > best[j] || v[j] != v[j]) {
                    best[j] = v[j];
                    bi = (bi & ~(0xFFu << (8 * j))) | ((uint32_t)k << (8 * j));
                }
        }
    }
    if (relu)
#pragma unroll
        for (int j = 0; j < 4; ++j) best[j] = fmaxf(best[j], 0.f);
    if (out) *(f32x4*)(out + o) = best;
    if (pi.pool16) {  // bf16 (RNE) straight into the next conv's operand image [pixels][C]
        u16x4 b;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = __builtin_bit_cast(uint16_t, (__bf16)best[j]);
        *(u16x4*)(pi.pool16 + o) = b;
    }
    if (out3) {  // the x3 split straight into the next conv's operand image [pixels][C / 32][3][32]
        u16x4 h, m, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint16_t hj, mj, lj;
            x3_split(best[j], X3CvtDev{}, hj, mj, lj);
            h[j] = hj;
            m[j] = mj;
            l[j] = lj;
        }
        uint16_t* d = out3 + (o / C) * 3 * C + (c >> 5) * 96 + (c & 31);
        *(u16x4*)d = h;
        *(u16x4*)(d + 32) = m;
        *(u16x4*)(d + 64) = l;
    }
    *(uint32_t*)(idx + o) = bi;
}

// Row form (N*H*W < 2^31): a thread keeps one channel quad and its affine in registers and
// walks pooled pixels with 32-bit index math (threads past the last complete row group of
// tpr = min(C / 4, 256) idle, and so do the quads past C / 4 in a last pass).
__global__ __launch_bounds__(256) void maxpool_bn_kernel(const float* __restrict__ y, int ld,
                                                         int off, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, int relu,
                                                         int N, int H, int W, int C,
                                                         float* __restrict__ out,
                                                         uint8_t* __restrict__ idx,
                                                         uint16_t* __restrict__ out3, PoolImg pi) {
    const int Ho = H / 2, Wo = W / 2, c4n = C / 4;
    const int tpr = c4n < 256 ? c4n : 256, rpp = 256 / tpr;
    const int PO = N * Ho * Wo;
    for (int cb = 0; cb < c4n; cb += tpr) {
        const int c = 4 * (cb + (int)threadIdx.x % tpr);
        const bool cin = c < C;
        const f32x4 sc = scale && cin ? *(const f32x4*)(scale + c) : f32x4{1.f, 1.f, 1.f, 1.f};
        const f32x4 sh = shift && cin ? *(const f32x4*)(shift + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        // each block walks one contiguous range of pooled pixels, the coordinates advanced
        // incrementally (no integer division per pixel)
        const int per = (PO + gridDim.x - 1) / gridDim.x;
        const int r0 = blockIdx.x * per, r1 = min(PO, r0 + per);
        const int g = (int)threadIdx.x / tpr;
        if (g >= rpp || c >= C) continue;  // partial row group (tpr does not divide 256) / pass
        Pix at = decode(min(r0 + g, PO - 1), Ho, Wo);
        for (int po = r0 + g; po < r1; po += rpp) {
            maxpool_px(y, ld, off, sc, sh, relu, H, W, at.img, at.y, at.x, c, out, idx,
                       (int64_t)po * C + c, out3, C, pi);
            pix_advance(at, rpp, Ho, Wo);
        }
    }
}

// Any C % 4 == 0: one thread per (pooled pixel, channel quad).
__global__ void maxpool_bn_any_kernel(const float* __restrict__ y, int ld, int off,
                                      const float* __restrict__ scale,
                                      const float* __restrict__ shift, int relu, int N, int H,
                                      int W, int C, float* __restrict__ out,
                                      uint8_t* __restrict__ idx, uint16_t* __restrict__ out3, PoolImg pi) {
    const int Ho = H / 2, Wo = W / 2, c4n = C / 4;
    const int64_t total = (int64_t)N * Ho * Wo * c4n;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c4 = (int)(i % c4n);
        const int64_t po = i / c4n;
        const int xo = (int)(po % Wo);
        const int64_t t = po / Wo;
        const int yo = (int)(t % Ho), img = (int)(t / Ho);
        const f32x4 sc = scale ? *(const f32x4*)(scale + 4 * c4) : f32x4{1.f, 1.f, 1.f, 1.f};
        const f32x4 sh = shift ? *(const f32x4*)(shift + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
        maxpool_px(y, ld, off, sc, sh, relu, H, W, img, yo, xo, 4 * c4, out, idx, po * C + 4 * c4, out3, C, pi);
    }
}

// do[p][c] = (idx routes dpool to p) + dskip[p][c]  (skip grad comes from the decoder's
// concat slice, model.py:64-70 / mod.py:64, so the encoder output's two consumers are
// summed here), plus the BN-backward column partials of do against the BN input y (same
// NHWC slice as the skip): partial[G][2][C] = {sum do, sum do*y}.  With mscale/mshift
// (BN -> ReLU order) do is first masked by the ReLU, [mscale*y + mshift > 0].
// One thread per channel quad, pooled pixels strided over the block's row groups.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const float* __restrict__ dp,
                                                         const uint8_t* __restrict__ idx,
                                                         const float* __restrict__ dskip, int ldskip,
                                                         int offskip, const float* __restrict__ y,
                                                         int ldy, int offy,
                                                         const float* __restrict__ mscale,
                                                         const float* __restrict__ mshift, int N,
                                                         int H, int W, int C,
                                                         float* __restrict__ dout, float* partial) {
    __shared__ double smem[256 * 2 * 4];
    const int Ho = H / 2, Wo = W / 2;
    // tpr need not divide 256 (C = 96, 192, ...: the threads past the last complete row
    // group idle) nor C / 4 (the last pass over C / 4 > 256 quads idles its upper quads)
    const int tpr = C / 4 < 256 ? C / 4 : 256, rpp = 256 / tpr;
    const int64_t PO = (int64_t)N * Ho * Wo;
    double acc[2][4];
    for (int c0 = 0; c0 < C; c0 += 4 * tpr) {
        const int q = threadIdx.x % tpr, g = threadIdx.x / tpr;
        const int c = c0 + 4 * q;
        const bool live = g < rpp && c < C;
        f32x4 ms = {0, 0, 0, 0}, mb = ms;
        if (mscale && live) {
            ms = *(const f32x4*)(mscale + c);
            mb = *(const f32x4*)(mshift + c);
        }
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[v][j] = 0.0;
        const int64_t per = (PO + gridDim.x - 1) / gridDim.x;
        const int64_t r0 = blockIdx.x * per, r1 = r0 + per < PO ? r0 + per : PO;
        Pix at = decode((int)min(r0 + g, PO - 1), Ho, Wo);  // N*H*W < 2^31 (launcher)
        for (int64_t po = r0 + g; live && po < r1; po += rpp) {
            const int xo = at.x, yo = at.y, img = at.img;
            pix_advance(at, rpp, Ho, Wo);
            const f32x4 gp = *(const f32x4*)(dp + po * C + c);
            const uint32_t bi = *(const uint32_t*)(idx + po * C + c);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int64_t pin = ((int64_t)img * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1);
                f32x4 v = *(const f32x4*)(dskip + pin * ldskip + offskip + c);
                const f32x4 yv = y ? *(const f32x4*)(y + pin * ldy + offy + c) : f32x4{0, 0, 0, 0};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (((bi >> (8 * j)) & 0xFF) == (uint32_t)k) v[j] += gp[j];
                    // (explicit fma: bn_dz_x3's fused pool source recomputes this mask, r05)
                    if (mscale && !(__builtin_fmaf(ms[j], yv[j], mb[j]) > 0.f)) v[j] = 0.f;
                }
                if (dout) *(f32x4*)(dout + pin * C + c) = v;  // (null: the dz pass recomputes it)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][j] += v[j];
                    acc[1][j] += (double)v[j] * yv[j];
                }
            }
        }
        if (partial)
            block_combine_d<2>(acc, tpr, C, partial + (int64_t)blockIdx.x * 2 * C + c0, smem,
                               (C - c0) / 4);
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------
// BatchNorm backward (train mode).  The producer of the BN-output gradient leaves column
// partials [G][2][C] = {S1 = sum do, S2 = sum do*y} (y = BN input; with BN -> ReLU order
// do is already masked by the ReLU).  From them: dgamma = invstd (S2 - mean S1),
// dbeta = S1 and the coefficients of dz = A do + B (y - mean) + Cc, coef[4][C] (model.py order additionally
// masks dz by [y > 0], the ReLU in front of the BN: model.py:37-38,40-41).
// -------------------------------------------------------------------------------------
__device__ void bn_bwd_final(int c, int C, const double (&ss)[2], double count,
                             const float* __restrict__ gamma, const float* __restrict__ mean,
                             const float* __restrict__ invstd, float* __restrict__ coef,
                             float* __restrict__ dgamma, float* __restrict__ dbeta) {
    if (c >= C) return;
    const double s1 = ss[0], s2 = ss[1];
    const double is = invstd[c], mu = mean[c];
    const double sdxh = is * (s2 - mu * s1);
    const double k = (double)gamma[c] * is;
    // centred form dz = A do + B (y - mean) + Cc: B (y - mean) is formed from the small
    // centred value, not as B y + (large constant), which cancelled to a few ulp of B * mean
    coef[c] = (float)k;
    coef[C + c] = (float)(-k * is * sdxh / count);
    coef[2 * C + c] = (float)(-k * s1 / count);
    coef[3 * C + c] = (float)mu;
    dgamma[c] = (float)sdxh;
    dbeta[c] = (float)s1;
}

__global__ void bn_bwd_finalize2_kernel(const float* __restrict__ part, int G, int C, double count,
                                        const float* __restrict__ gamma,
                                        const float* __restrict__ mean,
                                        const float* __restrict__ invstd, float* __restrict__ coef,
                                        float* __restrict__ dgamma, float* __restrict__ dbeta) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    double ss[2];
    colsum16<2>(part, G, 2 * C, C, c, c < C, ss);
    if (threadIdx.y != 0) return;
    bn_bwd_final(c, C, ss, count, gamma, mean, invstd, coef, dgamma, dbeta);
}


// dz = A do + B (y - mean) + C in place, masked by [y > 0] when `mask` (ReLU before the BN).
// Row form (C / 4 <= 256): each thread keeps one channel quad and its coefficients in
// registers and walks pixel rows, so there is no per-element index division.
__global__ __launch_bounds__(256) void bn_dz_rows_kernel(float* __restrict__ d,
                                                         const float* __restrict__ y, int ld,
                                                         int off, int64_t P, int C,
                                                         const float* __restrict__ coef, int mask) {
    const int tpr = C / 4, rpp = 256 / tpr;
    if ((int)threadIdx.x >= rpp * tpr) return;  // partial row group (tpr does not divide 256)
    const int c = (threadIdx.x % tpr) * 4;
    const f32x4 ka = *(const f32x4*)(coef + c), kb = *(const f32x4*)(coef + C + c),
                kc = *(const f32x4*)(coef + 2 * C + c), km = *(const f32x4*)(coef + 3 * C + c);
    for (int64_t m = (int64_t)blockIdx.x * rpp + threadIdx.x / tpr; m < P;
         m += (int64_t)gridDim.x * rpp) {
        f32x4* pd = (f32x4*)(d + m * C + c);
        const f32x4 v = *(const f32x4*)(y + m * ld + off + c);
        const f32x4 r = bn_dz4(ka, *pd, kb, v, km, kc);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (!mask || v[j] > 0.f) ? r[j] : 0.f;
        *pd = o;
    }
}

// bn_dz for the bf16 GEMMs: dz as the dense bf16 image the LDS-DMA dgrad / wgrad read
// (round to nearest even, as k_to_bf16), and the f32 dz in place only when another consumer
// still reads it (f32 != 0).  8 channels per thread.
// POOL (r06, option pool_fuse on the bf16 path): `d` is not read; do = [fma(msc, y, msh) > 0]
// (dskip + [winner == window position] dpool), the max-pool backward's sum recomputed from its
// inputs (as kernels_gemm_x3.hip bn_dz_x3_kernel<2>), so maxpool_bwd stores no full-resolution do
struct Dz16Pool {
    const float* dp;       // d pooled [N][H/2][W/2][C]
    const uint8_t* idx;    // winner index per pooled element
    const float* dskip;    // the concat gradient's skip half (offset applied), row stride ldskip
    int ldskip;
    const float *msc, *msh;  // BN -> ReLU mask affine, or null
    int H, W;              // full-resolution grid
    float rH, rW;
};
// HEAD (r06, option head_fuse on the bf16 path): the last conv's do = [BN -> ReLU: fma(y, sc, sh)
// > 0] dl[m] w[c], head_bwd's expression bit for bit (one output channel), as
// kernels_gemm_x3.hip bn_dz_x3_kernel<1>: head_bwd stores no full-resolution f32 do
struct Dz16Head {
    const float* dl;       // d logits [P]
    const float* w;        // head weights [C]
    const float *sc, *sh;  // the last BN's forward affine
    int relu;
};
template <int SRC>  // 0: do from memory, 1: Dz16Head, 2: Dz16Pool
__global__ __launch_bounds__(256) void bn_dz16_kernel(float* __restrict__ d, const float* __restrict__ y,
                                                      int ld, int off, int64_t P, int C,
                                                      const float* __restrict__ coef, int mask,
                                                      int tpr, __bf16* __restrict__ dz16, int f32, Dz16Pool pl,
                                                      Dz16Head hd) {
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    constexpr bool POOL = SRC == 2, HEAD = SRC == 1;
    constexpr int U = 4;  // rows per thread per trip: 16 independent 16-B loads in flight
    const int rpp = 256 / tpr;
    const int c_first = (threadIdx.x % tpr) * 8;
    for (int64_t m0 = (int64_t)blockIdx.x * rpp * U + threadIdx.x / tpr; m0 < P;
         m0 += (int64_t)gridDim.x * rpp * U) {
        for (int c = c_first; c < C; c += tpr * 8) {
            // the BN -> ReLU mask affine of this thread's 8 channels, in registers (loaded per
            // element inside the row loop, the fused pass ran 1.5x slower than the unfused pair)
            f32x4 msc[2], msh[2], hw[2], hs[2], hh[2];
            if (POOL && pl.msc) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    msc[h] = *(const f32x4*)(pl.msc + c + 4 * h);
                    msh[h] = *(const f32x4*)(pl.msh + c + 4 * h);
                }
            }
            if constexpr (HEAD) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    hw[h] = *(const f32x4*)(hd.w + c + 4 * h);
                    hs[h] = *(const f32x4*)(hd.sc + c + 4 * h);
                    hh[h] = *(const f32x4*)(hd.sh + c + 4 * h);
                }
            }
            f32x4 dv[U][2], yv[U][2];
            f32x4 gp[U][2];
            float dl[U];
            uint32_t wi[U][2];
            int kk[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t m = m0 + u * rpp;
                if (m < P) {
                    int64_t po = 0;
                    if constexpr (HEAD) dl[u] = hd.dl[m];
                    if constexpr (POOL) {
                        const Pix q = decode_fast((int)m, pl.H, pl.W, pl.rH, pl.rW);
                        po = ((int64_t)q.img * (pl.H >> 1) + (q.y >> 1)) * (pl.W >> 1) + (q.x >> 1);
                        kk[u] = (q.y & 1) * 2 + (q.x & 1);
                        const uint2 w2 = *(const uint2*)(pl.idx + po * C + c);
                        wi[u][0] = w2.x;
                        wi[u][1] = w2.y;
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if constexpr (POOL) {
                            dv[u][h] = *(const f32x4*)(pl.dskip + m * pl.ldskip + c + 4 * h);
                            gp[u][h] = *(const f32x4*)(pl.dp + po * C + c + 4 * h);
                        } else if constexpr (!HEAD) {
                            dv[u][h] = *(const f32x4*)(d + m * C + c + 4 * h);
                        }
                        yv[u][h] = *(const f32x4*)(y + m * ld + off + c + 4 * h);
                    }
                }
            }
            if constexpr (POOL) {
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (((wi[u][h] >> (8 * j)) & 0xFF) == (uint32_t)kk[u]) dv[u][h][j] += gp[u][h][j];
                            if (pl.msc && !(__builtin_fmaf(msc[h][j], yv[u][h][j], msh[h][j]) > 0.f))
                                dv[u][h][j] = 0.f;
                        }
            }
            if constexpr (HEAD) {
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const bool on = !hd.relu || __builtin_fmaf(yv[u][h][j], hs[h][j], hh[h][j]) > 0.f;
                            dv[u][h][j] = on ? dl[u] * hw[h][j] : 0.f;
                        }
            }
            f32x4 ka[2], kb[2], kc[2], km[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                ka[h] = *(const f32x4*)(coef + c + 4 * h);
                kb[h] = *(const f32x4*)(coef + C + c + 4 * h);
                kc[h] = *(const f32x4*)(coef + 2 * C + c + 4 * h);
                km[h] = *(const f32x4*)(coef + 3 * C + c + 4 * h);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t m = m0 + u * rpp;
                if (m >= P) break;
                bf16x8 o16;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const f32x4 v = yv[u][h];
                    const f32x4 r = bn_dz4(ka[h], dv[u][h], kb[h], v, km[h], kc[h]);
                    f32x4 o;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        o[j] = (!mask || v[j] > 0.f) ? r[j] : 0.f;
                        o16[4 * h + j] = (__bf16)o[j];
                    }
                    if (SRC == 0 && f32) *(f32x4*)(d + m * C + c + 4 * h) = o;
                }
                *(bf16x8*)(dz16 + m * C + c) = o16;
            }
        }
    }
}

__global__ void bn_dz_kernel(float* __restrict__ d, const float* __restrict__ y, int ld, int off,
                             int64_t P, int C, const float* __restrict__ coef, int mask) {
    const int c4n = C / 4;
    const int64_t total = P * c4n;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % c4n) * 4;
        const int64_t m = i / c4n;
        f32x4* pd = (f32x4*)(d + m * C + c);
        const f32x4 v = *(const f32x4*)(y + m * ld + off + c);
        const f32x4 r = *(const f32x4*)(coef + c) * (*pd) +
                        *(const f32x4*)(coef + C + c) * (v - *(const f32x4*)(coef + 3 * C + c)) +
                        *(const f32x4*)(coef + 2 * C + c);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (!mask || v[j] > 0.f) ? r[j] : 0.f;
        *pd = o;
    }
}

// bf16 operand image for the LDS-DMA GEMMs (kernels_gemm16.hip): dst[m][c] (dense, ld C) =
// bf16(op(src[m * ld + off + c])), op = scale * x + shift when scale is set, then ReLU on
// channels c < relu (BN -> ReLU order, models/mod.py:46-47; a [skip, up] concat has it on
// the skip half only).  Round to nearest even -- the rounding the register-staged bf16 GEMMs
// apply when they stage the same values.  tpr threads per row, 8 channels each.
__global__ __launch_bounds__(256) void to_bf16_kernel(const float* __restrict__ src, int ld, int off,
                                                      int C, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, int relu,
                                                      int64_t P, int tpr, __bf16* __restrict__ dst,
                                                      int dld) {
    typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
    constexpr int U = 4;  // rows per thread per trip: 8 independent 16-B loads in flight
    const int rpp = 256 / tpr;
    const int c_first = (threadIdx.x % tpr) * 8;
    for (int64_t m0 = (int64_t)blockIdx.x * rpp * U + threadIdx.x / tpr; m0 < P;
         m0 += (int64_t)gridDim.x * rpp * U) {
        for (int c = c_first; c < C; c += tpr * 8) {
            f32x4 v[U][2];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t m = m0 + u * rpp;
                if (m < P) {
                    const float* row = src + m * ld + off + c;
                    v[u][0] = *(const f32x4*)row;
                    v[u][1] = *(const f32x4*)(row + 4);
                }
            }
            f32x4 sc0 = {1.f, 1.f, 1.f, 1.f}, sc1 = sc0, sh0 = {0.f, 0.f, 0.f, 0.f}, sh1 = sh0;
            if (scale) {
                sc0 = *(const f32x4*)(scale + c);
                sc1 = *(const f32x4*)(scale + c + 4);
                sh0 = *(const f32x4*)(shift + c);
                sh1 = *(const f32x4*)(shift + c + 4);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t m = m0 + u * rpp;
                if (m >= P) break;
                f32x4 v0 = v[u][0], v1 = v[u][1];
                if (scale) {
                    v0 = v0 * sc0 + sh0;
                    v1 = v1 * sc1 + sh1;
                }
                if (c < relu) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        v0[j] = fmaxf(v0[j], 0.f);
                        v1[j] = fmaxf(v1[j], 0.f);
                    }
                }
                bf16x8 o;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    o[j] = (__bf16)v0[j];
                    o[4 + j] = (__bf16)v1[j];
                }
                *(bf16x8*)(dst + m * dld + c) = o;
            }
        }
    }
}

// bias gradient from the wgrad kernels' column sums: out[co] = sum_s sum_tap slab[s][tap*C+co]
__global__ void bias_reduce_kernel(const float* __restrict__ slab, int S, int taps, int C,
                                   float* __restrict__ out) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    double t = 0.0;
    for (int tap = 0; tap < taps; ++tap) {
        double v[1];
        colsum16<1>(slab + tap * C, S, taps * C, 0, c, c < C, v);
        t += v[0];
        __syncthreads();
    }
    if (threadIdx.y == 0 && c < C) out[c] = (float)t;
}

// ConvT bias gradient partials for the LDS-DMA weight gradient (which has no B' column
// sums): bslab[s][ab*C + c] = sum over the coarse pixels m of split s (pps per split) of
// d[fine(m, ab)][off + c], i.e. the column sums of the G_UP2-gathered B' operand the
// register-staged kernel forms, accumulated in f64 and rounded once, as it does.
// Block = (split, ab, 64 channels); thread (quad q = tid % 16, row group g = tid / 16).
__global__ __launch_bounds__(256) void up2_bias_partials_kernel(const float* __restrict__ d, int ld,
                                                                int off, int H, int W, int64_t P,
                                                                int C, int pps,
                                                                float* __restrict__ bslab) {
    __shared__ double red[16][64];
    const int split = blockIdx.x, ab = blockIdx.y, c0 = blockIdx.z * 64;
    const int tid = threadIdx.x, q = tid & 15, g = tid >> 4;
    const int a = ab >> 1, b = ab & 1;
    const int64_t pbeg = (int64_t)split * pps, pend = min(pbeg + pps, P);
    const int c = c0 + 4 * q;
    const bool ok = c < C;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    const int HW = H * W;
    constexpr int U = 8;  // 8 independent row loads in flight per thread
    for (int64_t m0 = pbeg + g; m0 < pend && ok; m0 += 16 * U) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t m = m0 + 16 * u;
            if (m < pend) {
                // 32-bit index math (the launcher guarantees 4 P < 2^31)
                const int mm = (int)m;
                const int n = mm / HW;
                const int r = mm - n * HW;
                const int i = r / W, j = r - i * W;
                const int64_t f = (int64_t)n * 4 * HW + (2 * i + a) * (2 * W) + (2 * j + b);
                v[u] = *(const f32x4*)(d + f * ld + off + c);
            } else {
                v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            s0 += v[u][0];
            s1 += v[u][1];
            s2 += v[u][2];
            s3 += v[u][3];
        }
    }
    red[g][4 * q] = s0;
    red[g][4 * q + 1] = s1;
    red[g][4 * q + 2] = s2;
    red[g][4 * q + 3] = s3;
    __syncthreads();
    if (tid < 64 && c0 + tid < C) {
        double t = 0.0;
        for (int k = 0; k < 16; ++k) t += red[k][tid];
        bslab[(int64_t)split * 4 * C + ab * C + c0 + tid] = (float)t;
    }
}

// out[c] = sum over G partial rows (fixed order), optional scatter stride
__global__ void sum_partials_kernel(const float* __restrict__ part, int G, int ncols,
                                    float* __restrict__ out) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    double s[1];
    colsum16<1>(part, G, ncols, 0, c, c < ncols, s);
    if (threadIdx.y == 0 && c < ncols) out[c] = (float)s[0];
}

// Sum the split-K slabs of a wgrad and scatter into the torch weight layout.
//   conv3 : slab [S][tap*Cin+ci][co] -> grad[co][ci][tap]
//   conv1 : slab [S][ci][co]         -> grad[co][ci]         (kind 2)
//   convT : slab [S][ci][ab*Cout+co] -> grad[ci][co][ab]
__global__ void slab_reduce_kernel(const float* __restrict__ slab, int S, int Mw, int Nw,
                                   int kind, int cin, int cout, float* __restrict__ grad) {
    // 4 consecutive n per thread (float4 loads); the S slabs are summed in a fixed
    // association (four interleaved partial sums, then combined) with 8 loads in flight.
    const int64_t total = (int64_t)Mw * Nw;
    const int64_t nq = total / 4;
    for (int64_t iq = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; iq < nq;
         iq += (int64_t)gridDim.x * blockDim.x) {
        const f32x4* sp = (const f32x4*)slab + iq;
        const int64_t stride = total / 4;
        f32x4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
        int k = 0;
        for (; k + 8 <= S; k += 8) {
            f32x4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = sp[(int64_t)(k + u) * stride];
            a0 += v[0] + v[4];
            a1 += v[1] + v[5];
            a2 += v[2] + v[6];
            a3 += v[3] + v[7];
        }
        for (; k < S; ++k) a0 += sp[(int64_t)k * stride];
        const f32x4 s4 = (a0 + a1) + (a2 + a3);
        const int64_t i0 = iq * 4;
        const int m = (int)(i0 / Nw), n0 = (int)(i0 % Nw);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + j;
            int64_t o;
            if (kind == 0) {
                const int tap = m / cin, ci = m - tap * cin;
                o = ((int64_t)n * cin + ci) * 9 + tap;
            } else if (kind == 2) {  // 1x1 conv: slab [ci][co] -> grad[co][ci]
                o = (int64_t)n * cin + m;
            } else {
                const int ab = n / cout, co = n - ab * cout;
                o = ((int64_t)m * cout + co) * 4 + ab;
            }
            grad[o] = s4[j];
        }
    }
}

// Many-slab reduce (S >= 32: the narrow layers, whose split-K runs hundreds of slices):
// 16 lanes per 4-column quad walk the slabs k = lane, lane + 16, ... (8 loads in flight),
// and the 16 partial sums are combined in lane order through LDS -- a fixed association, so
// deterministic, with 16x more threads and 16x shorter chains than one thread per quad.
__global__ __launch_bounds__(256) void slab_reduce_wide_kernel(const float* __restrict__ slab, int S,
                                                               int Mw, int Nw, int kind, int cin,
                                                               int cout, float* __restrict__ grad) {
    __shared__ f32x4 red[16][17];
    const int64_t total = (int64_t)Mw * Nw;
    const int64_t nq = total / 4;
    const int ql = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const int64_t iq = (int64_t)blockIdx.x * 16 + ql;
    f32x4 a0 = {0, 0, 0, 0}, a1 = a0;
    if (iq < nq) {
        const f32x4* sp = (const f32x4*)slab + iq;
        const int64_t stride = total / 4;
        int k = sl;
        for (; k + 16 * 7 < S; k += 16 * 8) {
            f32x4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = sp[(int64_t)(k + 16 * u) * stride];
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                a0 += v[u];
                a1 += v[u + 1];
            }
        }
        for (; k < S; k += 16) a0 += sp[(int64_t)k * stride];
    }
    red[sl][ql] = a0 + a1;
    __syncthreads();
    if (sl != 0 || iq >= nq) return;
    f32x4 s4 = red[0][ql];
#pragma unroll
    for (int j = 1; j < 16; ++j) s4 += red[j][ql];
    const int64_t i0 = iq * 4;
    const int m = (int)(i0 / Nw), n0 = (int)(i0 % Nw);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = n0 + j;
        int64_t o;
        if (kind == 0) {
            const int tap = m / cin, ci = m - tap * cin;
            o = ((int64_t)n * cin + ci) * 9 + tap;
        } else if (kind == 2) {
            o = (int64_t)n * cin + m;
        } else {
            const int ab = n / cout, co = n - ab * cout;
            o = ((int64_t)m * cout + co) * 4 + ab;
        }
        grad[o] = s4[j];
    }
}

// (r06) 2x2 ConvT weight gradient, slab rows m = ci, columns n = ab * cout + co ->
// grad[ci][co][ab]: one thread per (ci, co) reads its four ab columns (coalesced along co) and
// stores one float4 (slab_reduce_kernel wrote each float 16 B from the next, which on the
// 4096 -> 2048 ConvT of config 4 ran its 268 MB at 1.3 TB/s).  Per element the S slabs are
// summed in exactly slab_reduce_kernel's association: identical bits.
__global__ __launch_bounds__(256) void slab_reduce_convT_kernel(const float* __restrict__ slab, int S,
                                                                int cin, int cout,
                                                                float* __restrict__ grad) {
    const int64_t total = (int64_t)cin * 4 * cout;
    const int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (q >= (int64_t)cin * cout) return;
    const int ci = (int)(q / cout), co = (int)(q - (int64_t)ci * cout);
    f32x4 r;
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) {
        const float* sp = slab + (int64_t)ci * 4 * cout + ab * cout + co;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int k = 0;
        for (; k + 8 <= S; k += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = sp[(int64_t)(k + u) * total];
            a0 += v[0] + v[4];
            a1 += v[1] + v[5];
            a2 += v[2] + v[6];
            a3 += v[3] + v[7];
        }
        for (; k < S; ++k) a0 += sp[(int64_t)k * total];
        r[ab] = (a0 + a1) + (a2 + a3);
    }
    *(f32x4*)(grad + q * 4) = r;
}

// 3x3 weight gradient, slab rows m = tap * cin + ci, columns n = co -> grad[co][ci][tap]
// through an LDS tile of 32 co x 32 ci x 9 taps: reads stay coalesced along n, and each co
// writes one contiguous run of 32 * 9 floats (the row-per-thread kernel above scatters every
// float 9 * cin apart, which on the 4096-channel layers made this pass HBM-write-bound at a
// small fraction of the bandwidth).  Per element the S slabs are summed in exactly the
// association of slab_reduce_kernel, so both kernels give identical bits.
// CI = input channels per tile: 32 for the transposing copy (S == 1: 36 loads per thread in
// flight), 8 when slabs are summed (each thread walks S slabs per element with 8 loads in
// flight; the 4x smaller tile gives 4x the blocks, which is what keeps enough loads in flight
// on layers with only 256 32x32 tiles).
template <int CI>
__global__ __launch_bounds__(256) void slab_reduce_conv3_kernel(const float* __restrict__ slab, int S,
                                                                int cin, int cout,
                                                                float* __restrict__ grad) {
    constexpr int ROWS = 9 * CI;  // (tap, ci) rows of the tile
    __shared__ float tile[32][ROWS + 1];
    const int n0 = blockIdx.x * 32, c0 = blockIdx.y * CI;
    const int Nw = cout;
    const int64_t total = (int64_t)9 * cin * cout;
    const int nl = threadIdx.x & 31, rr = threadIdx.x >> 5;
    if (S == 1) {  // a transposing copy: all loads of the thread in flight at once
        constexpr int NV = ROWS / 8;
        float v[NV];
#pragma unroll
        for (int it = 0; it < NV; ++it) {
            const int row = rr + 8 * it, tap = row / CI, cl = row - tap * CI;
            v[it] = slab[(int64_t)(tap * cin + c0 + cl) * Nw + n0 + nl];
        }
#pragma unroll
        for (int it = 0; it < NV; ++it) {
            const int row = rr + 8 * it, tap = row / CI, cl = row - tap * CI;
            tile[nl][cl * 9 + tap] = v[it];
        }
    }
    for (int row = S == 1 ? ROWS : rr; row < ROWS; row += 8) {
        const int tap = row / CI, cl = row - tap * CI;
        const int64_t e = (int64_t)(tap * cin + c0 + cl) * Nw + n0 + nl;
        const float* sp = slab + e;
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int k = 0;
        for (; k + 8 <= S; k += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = sp[(int64_t)(k + u) * total];
            a0 += v[0] + v[4];
            a1 += v[1] + v[5];
            a2 += v[2] + v[6];
            a3 += v[3] + v[7];
        }
        for (; k < S; ++k) a0 += sp[(int64_t)k * total];
        tile[nl][cl * 9 + tap] = (a0 + a1) + (a2 + a3);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 32 * ROWS; i += 256) {
        const int n = i / ROWS, off = i - n * ROWS;
        grad[((int64_t)(n0 + n) * cin + c0) * 9 + off] = tile[n][off];
    }
}

// conv-first wgrad partials [G][10][C] -> grad w[co][0][tap], b[co]
__global__ void conv_first_wgrad_finalize_kernel(const float* __restrict__ part, int G, int C,
                                                 float* __restrict__ gw, float* __restrict__ gb) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    double sv[1];
    colsum16<1>(part, G, 10 * C, 0, i, i < 10 * C, sv);
    if (threadIdx.y != 0 || i >= 10 * C) return;
    const float s = (float)sv[0];
    const int tap = i / C, c = i - tap * C;
    if (tap < 9)
        gw[c * 9 + tap] = s;
    else if (gb)
        gb[c] = s;
}

// -------------------------------------------------------------------------------------
// 1x1 head Conv2d(C -> O) (model.py:30) on BN(y), fused BN affine.  16 lanes per pixel.
// logits are NCHW (N, O, H, W).
// -------------------------------------------------------------------------------------
__global__ void head_fwd_kernel(const float* __restrict__ y, int C, const float* __restrict__ scale,
                                const float* __restrict__ shift, int relu,
                                const float* __restrict__ w,
                                const float* __restrict__ b, int O, int P, int HW,
                                float* __restrict__ logits) {
    const int lpp = C / 4;  // lanes per pixel (C == 64 -> 16)
    // U pixels per thread, strided by the grid's pixel count (their loads issued together:
    // a one-pixel thread left too few bytes in flight, 3.8 TB/s); 32-bit index math
    // (P * lpp < 2^31: the launcher's thread count)
    constexpr int U = 4;
    const int gt = blockIdx.x * blockDim.x + threadIdx.x;
    const int pix0 = gt / lpp;
    const int q = gt - pix0 * lpp;
    const int stride = gridDim.x * (blockDim.x / lpp);  // pixels per grid sweep
    const f32x4 sc = scale ? *(const f32x4*)(scale + 4 * q) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 sh = scale ? *(const f32x4*)(shift + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int pb = pix0; pb < P; pb += U * stride) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int pix = pb + u * stride;
            v[u] = pix < P ? __builtin_nontemporal_load((const f32x4*)(y + (int64_t)pix * C + 4 * q))
                           : f32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int pix = pb + u * stride;
            f32x4 a = v[u];
            if (scale)  // explicit fma: the same activation as the backward's ReLU mask
#pragma unroll
                for (int j = 0; j < 4; ++j) a[j] = __builtin_fmaf(a[j], sc[j], sh[j]);
            if (relu)
#pragma unroll
                for (int j = 0; j < 4; ++j) a[j] = fmaxf(a[j], 0.f);
            for (int o = 0; o < O; ++o) {
                const f32x4 wv = *(const f32x4*)(w + o * C + 4 * q);
                float s = a[0] * wv[0] + a[1] * wv[1] + a[2] * wv[2] + a[3] * wv[3];
                for (int d = lpp / 2; d >= 1; d >>= 1) s += __shfl_xor(s, d);
                if (pix < P && q == 0) {
                    const int img = pix / HW, hw = pix - img * HW;
                    logits[((int64_t)img * O + o) * HW + hw] = s + b[o];
                }
            }
        }
    }
}

// do[p][c] = sum_o dl[p][o] w[o][c];  partial dW[o][c] = sum dl * act(y)_c, db[o] = sum dl.
// partial layout [G][O*C + O]; bnpart [G][2][C] = {sum do, sum do*y} for the BN backward.
// relu (BN -> ReLU order): act = ReLU(BN(y)) and do is masked by that ReLU.
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ y, int C,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift, int relu,
                                                      const float* __restrict__ w, int O, int P,
                                                      int HW, const float* __restrict__ dlog,
                                                      float* __restrict__ dout, float* partial,
                                                      float* bnpart) {
    __shared__ float red[256 * 5];
    __shared__ double smem4[256 * 2 * 4];
    double bq[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    const int lpp = C / 4, rpp = 256 / lpp;
    const int q = threadIdx.x % lpp, g = threadIdx.x / lpp;
    const f32x4 sc = scale ? *(const f32x4*)(scale + 4 * q) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 sh = shift ? *(const f32x4*)(shift + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    // O <= 4 supported for the fused partials
    f32x4 aw[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    float ab[4] = {0, 0, 0, 0};
    const int per = (P + gridDim.x - 1) / gridDim.x;
    const int r0 = blockIdx.x * per, r1 = min(P, r0 + per);
    // two pixels per trip, both pixels' loads issued first (P < 2^31: 32-bit pixel math);
    // each thread still accumulates its pixels in increasing m (same partials)
    auto one = [&](int m, const f32x4& yr, const float (&dl)[4]) {
        f32x4 v;  // explicit fma: bn_dz_x3's fused head source recomputes this mask (r05)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = __builtin_fmaf(yr[j], sc[j], sh[j]);
        if (relu)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
        f32x4 d = {0, 0, 0, 0};
        for (int o = 0; o < O; ++o) {
            d += dl[o] * *(const f32x4*)(w + o * C + 4 * q);
            aw[o] += dl[o] * v;
            ab[o] += dl[o];
        }
        if (relu)
#pragma unroll
            for (int j = 0; j < 4; ++j) d[j] = v[j] > 0.f ? d[j] : 0.f;
        if (dout) *(f32x4*)(dout + (int64_t)m * C + 4 * q) = d;  // (null: the dz pass recomputes it)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bq[0][j] += d[j];
            bq[1][j] += (double)d[j] * yr[j];
        }
    };
    for (int m = r0 + g; m < r1; m += 2 * rpp) {
        const int m2 = m + rpp;
        const bool two = m2 < r1;
        const f32x4 y1 = *(const f32x4*)(y + (int64_t)m * C + 4 * q);
        const f32x4 y2 = two ? *(const f32x4*)(y + (int64_t)m2 * C + 4 * q) : f32x4{0, 0, 0, 0};
        float d1[4] = {0, 0, 0, 0}, d2[4] = {0, 0, 0, 0};
        {
            const int img = m / HW, hw = m - img * HW;
            for (int o = 0; o < O; ++o) d1[o] = dlog[((int64_t)img * O + o) * HW + hw];
        }
        if (two) {
            const int img = m2 / HW, hw = m2 - img * HW;
            for (int o = 0; o < O; ++o) d2[o] = dlog[((int64_t)img * O + o) * HW + hw];
        }
        one(m, y1, d1);
        if (two) one(m2, y2, d2);
    }
    if (bnpart) block_combine_d<2>(bq, lpp, C, bnpart + (int64_t)blockIdx.x * 2 * C, smem4);
    __syncthreads();
    // combine over row groups through LDS, one quantity at a time
    float* out = partial + (int64_t)blockIdx.x * (O * C + O);
    for (int o = 0; o < O; ++o) {
        for (int j = 0; j < 4; ++j) {
            red[threadIdx.x] = aw[o][j];
            __syncthreads();
            if (g == 0) {
                float s = 0.f;
                for (int k = 0; k < rpp; ++k) s += red[k * lpp + q];
                out[o * C + 4 * q + j] = s;
            }
            __syncthreads();
        }
        red[threadIdx.x] = ab[o];
        __syncthreads();
        if (threadIdx.x == 0) {
            float s = 0.f;
            for (int k = 0; k < rpp; ++k) s += red[k * lpp];  // q == 0 lanes carry the sum
            out[O * C + o] = s;
        }
        __syncthreads();
    }
}

// -------------------------------------------------------------------------------------
// Residual block of models/mod.py:ResUNet (:73-86): out = ReLU(BN2(z2) + skip(x)).
// -------------------------------------------------------------------------------------
// First block (Cin = 1): skip is a per-channel scale of the image, out[p][c] =
// ReLU(s[c] z[p][c] + t[c] + ws[c] x[p]).  One thread per (pixel, channel quad).
__global__ void res_first_fwd_kernel(const float* __restrict__ x, const float* __restrict__ ws,
                                     const float* __restrict__ z, const float* __restrict__ sc,
                                     const float* __restrict__ sh, int64_t P, int C,
                                     float* __restrict__ out, int ldo, int offo) {
    const int c4n = C / 4;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < P * c4n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % c4n) * 4;
        const int64_t m = i / c4n;
        const float xv = x[m];
        const f32x4 zv = *(const f32x4*)(z + m * C + c);
        f32x4 o = zv * *(const f32x4*)(sc + c) + *(const f32x4*)(sh + c) + xv * *(const f32x4*)(ws + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = fmaxf(o[j], 0.f);
        *(f32x4*)(out + m * ldo + offo + c) = o;
    }
}

// Backward entry of a residual block: du = dout [out > 0] (in place) and the BN2 partials
// partial[G][2][C] = {sum du, sum du z2} (z2 = conv output before BN2, dense [P][C]).
__global__ __launch_bounds__(256) void res_bwd_prep_kernel(float* __restrict__ d,
                                                          const float* __restrict__ out, int ldo,
                                                          int offo, const float* __restrict__ z,
                                                          int64_t P, int C, float* partial) {
    __shared__ double smem[256 * 2 * 4];
    const int tpr = C / 4 < 256 ? C / 4 : 256, rpp = 256 / tpr;
    double acc[2][4];
    for (int c0 = 0; c0 < C; c0 += 4 * tpr) {
        const int q = threadIdx.x % tpr, g = threadIdx.x / tpr;
        const int c = c0 + 4 * q;
        const bool live = g < rpp && c < C;  // (maxpool_bwd_kernel: partial groups / passes)
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[v][j] = 0.0;
        const int64_t per = (P + gridDim.x - 1) / gridDim.x;
        const int64_t r0 = blockIdx.x * per, r1 = r0 + per < P ? r0 + per : P;
        for (int64_t m = r0 + g; live && m < r1; m += rpp) {
            f32x4* pd = (f32x4*)(d + m * C + c);
            f32x4 v = *pd;
            const f32x4 ov = *(const f32x4*)(out + m * ldo + offo + c);
            const f32x4 zv = *(const f32x4*)(z + m * C + c);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = ov[j] > 0.f ? v[j] : 0.f;
                acc[0][j] += v[j];
                acc[1][j] += (double)v[j] * zv[j];
            }
            *pd = v;
        }
        block_combine_d<2>(acc, tpr, C, partial + (int64_t)blockIdx.x * 2 * C + c0, smem,
                           (C - c0) / 4);
        __syncthreads();
    }
}

// First block's skip weight gradient: partial[G][C] = sum_p x[p] du[p][c].
__global__ __launch_bounds__(256) void res_first_wgrad_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ du, int P,
                                                             int C, float* partial) {
    __shared__ __attribute__((aligned(16))) float smem[256 * 1 * 4];
    const int tpr = C / 4, rpp = 256 / tpr;
    const int q = threadIdx.x % tpr, g = threadIdx.x / tpr;
    f32x4 acc[1] = {{0, 0, 0, 0}};
    const int per = (P + gridDim.x - 1) / gridDim.x;
    const int r0 = blockIdx.x * per, r1 = min(P, r0 + per);
    for (int m = r0 + g; m < r1; m += rpp)
        acc[0] += x[m] * *(const f32x4*)(du + (int64_t)m * C + 4 * q);
    block_combine<1>(acc, tpr, C, partial + (int64_t)blockIdx.x * C, smem);
}

// -------------------------------------------------------------------------------------
// Losses (utils/trainer.py:85-88; models/loss.py:13-46).  Per sample:
//   stats[n] = {I = sum p t, Sp = sum p, St = sum t, Sbce = sum bce_elem}
// bce_elem = (1 - t) x - log_sigmoid(x), log_sigmoid(x) = min(x,0) - log1p(exp(-|x|))
// (ATen binary_cross_entropy_with_logits), p = 1 / (1 + exp(-x)).
// (r06) G = loss_groups(per) blocks per sample (a function of the sample size only, so a
// sample's statistics carry the same bits whatever the batch or its split over ranks) each
// write the four sums of one contiguous chunk to part[n][g]; loss_sums_kernel adds the G
// chunks of a sample in order.  One block per sample left 8 CUs streaming config 4's logits
// (0.31 ms for 17 MB).
// -------------------------------------------------------------------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ void loss_elem(float xv, float tv, float (&a)[4]) {
    const float pv = sigmoidf_(xv);
    a[0] += pv * tv;
    a[1] += pv;
    a[2] += tv;
    a[3] += (1.f - tv) * xv - (fminf(xv, 0.f) - log1pf(expf(-fabsf(xv))));
}

__global__ __launch_bounds__(256) void loss_stats_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ t, int64_t per,
                                                        int G, float* __restrict__ part) {
    __shared__ float red[4][4];
    const int n = blockIdx.x / G, g = blockIdx.x - n * G;
    const int64_t chunk = (per + G - 1) / G;
    const int64_t i0 = g * chunk, i1 = min(per, i0 + chunk);
    const float* xs = x + n * per;
    const float* ts = t + n * per;
    float a[4] = {0, 0, 0, 0};
    if ((per & 3) == 0 && (chunk & 3) == 0 && ((((uintptr_t)x) | ((uintptr_t)t)) & 15) == 0) {
        for (int64_t i = i0 + 4 * threadIdx.x; i < i1; i += 4 * blockDim.x) {
            const f32x4 xv = *(const f32x4*)(xs + i), tv = *(const f32x4*)(ts + i);
#pragma unroll
            for (int j = 0; j < 4; ++j) loss_elem(xv[j], tv[j], a);
        }
    } else {
        for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) loss_elem(xs[i], ts[i], a);
    }
    for (int k = 0; k < 4; ++k)
        for (int d = 32; d >= 1; d >>= 1) a[k] += __shfl_xor(a[k], d);
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    if (ln == 0)
        for (int k = 0; k < 4; ++k) red[k][wv] = a[k];
    __syncthreads();
    if (threadIdx.x < 4)
        part[4 * (int64_t)blockIdx.x + threadIdx.x] =
            (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

// Batch sums of the per-sample statistics (double, fixed sample order):
//   sums = {Σ bce_elem, Σ_n dice_n, TP = Σ I, Σ p, Σ t, samples, elements, 0}
// These are the only cross-sample quantities of the three losses, so under data
// parallelism an all-reduce (SUM) of `sums` turns every rank's local batch into the
// reference's gathered batch (nn.DataParallel computes the loss on the gathered logits,
// utils/trainer.py:28-30,85-90; FocalTversky's TP/FP/FN are global, models/loss.py:41-45).
__global__ __launch_bounds__(256) void loss_sums_kernel(const float* __restrict__ part, int G,
                                                       float* __restrict__ stats, int N,
                                                       int64_t per, double* __restrict__ sums) {
    for (int j = threadIdx.x; j < 4 * N; j += blockDim.x) {  // a sample's chunks, in order
        const int n = j >> 2, k = j & 3;
        float v = 0.f;
        for (int g = 0; g < G; ++g) v += part[4 * ((int64_t)n * G + g) + k];
        stats[j] = v;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double bce = 0, dice = 0, tp = 0, sp = 0, st = 0;
    for (int n = 0; n < N; ++n) {
        const double I = stats[4 * n], P = stats[4 * n + 1], T = stats[4 * n + 2];
        bce += stats[4 * n + 3];
        dice += (2.0 * I + 1.0) / (P + T + 1.0);  // models/loss.py:23, smooth = 1
        tp += I;
        sp += P;
        st += T;
    }
    sums[0] = bce;
    sums[1] = dice;
    sums[2] = tp;
    sums[3] = sp;
    sums[4] = st;
    sums[5] = (double)N;
    sums[6] = (double)per * N;
    sums[7] = 0.0;
}

// losses = {bce_mean, dice_loss, focal} of the (possibly all-reduced) batch sums
__global__ void loss_finalize_kernel(const double* __restrict__ sums, float alpha, float beta,
                                     float gamma, float* __restrict__ losses) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const double tp = sums[2], fp = sums[3] - tp, fn = sums[4] - tp, sm = 1e-6;  // loss.py:41-43
    const double ti = (tp + sm) / (tp + alpha * fp + beta * fn + sm);              // loss.py:44
    losses[0] = (float)(sums[0] / sums[6]);
    losses[1] = (float)(1.0 - sums[1] / sums[5]);
    losses[2] = (float)pow(1.0 - ti, (double)gamma);                               // loss.py:45
}

// dlogits of w[0]*bce + w[1]*dice + w[2]*focal for this rank's samples; the batch
// normalisers (elements, samples) and the focal TP/FP/FN come from `sums`, so with
// all-reduced sums every rank writes its slice of the gathered batch's gradient and the
// ranks' weight gradients SUM to the reference's (DataParallel's reduce-add).
__global__ void loss_bwd_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                int64_t per, int N, const float* __restrict__ stats,
                                const double* __restrict__ sums, const float* __restrict__ w,
                                float alpha, float beta, float gamma, float* __restrict__ dx) {
    const int64_t total = per * N;
    const float wb = w[0], wd = w[1], wf = w[2];
    const float inv_total = (float)(1.0 / sums[6]);
    const float inv_n = (float)(1.0 / sums[5]);
    // focal-tversky scalars (models/loss.py:41-45), formed once in double
    const double tpd = sums[2], smd = 1e-6;
    const double Ad = tpd + smd;
    const double Bdd = tpd + alpha * (sums[3] - tpd) + beta * (sums[4] - tpd) + smd;
    const double tid = Ad / Bdd;
    const float A = (float)Ad, Bd = (float)Bdd;
    const float dLdti = (wf != 0.f) ? (float)(-gamma * pow(fmax(1.0 - tid, 0.0), gamma - 1.0)) : 0.f;
    const float inv_B2 = (float)(1.0 / (Bdd * Bdd));
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int n = (int)(i / per);
        const float xv = x[i], tv = t[i];
        const float pv = sigmoidf_(xv);
        float g = wb * (pv - tv) * inv_total;  // d bce_mean / dx
        const float I = stats[4 * n], U = stats[4 * n + 1] + stats[4 * n + 2];
        const float dd = (2.f * tv * (U + 1.f) - (2.f * I + 1.f)) / ((U + 1.f) * (U + 1.f));
        float gp = -wd * dd * inv_n;  // d dice_loss / dp
        if (wf != 0.f) {
            const float dti = (tv * Bd - A * (tv + alpha * (1.f - tv) - beta * tv)) * inv_B2;
            gp += wf * dLdti * dti;
        }
        g += gp * pv * (1.f - pv);
        dx[i] = g;
    }
}

// -------------------------------------------------------------------------------------
// AdamW (utils/trainer.py:41,92; torch optim/adam.py _single_tensor_adam with decoupled
// weight decay).  The element update is torch's CPU op sequence with each op rounded
// where ATen rounds it; the scalars were formed in double on the host and rounded to
// float once, as ATen casts a Python-float Scalar (runtime.hip: unet_adamw):
//   param.mul_(1 - lr*wd)                      p * decay
//   exp_avg.lerp_(grad, 1 - beta1)             ATen lerp_vec: fma(w, g - m, m) for |w| < 0.5,
//                                              else fma(w - 1, g - m, g)
//   exp_avg_sq.mul_(beta2)                     v * b2
//     .addcmul_(grad, grad, value=1 - beta2)   fma(w2 * g, g, v)  (ATen's vectorised
//                                              self + s*t1*t2, contracted by the compiler)
//   denom = (exp_avg_sq.sqrt() / bc2_sqrt).add_(eps)
//   param.addcdiv_(exp_avg, denom, value=-step_size)   p + (-step * m) / denom
// Contraction is switched off so the compiler cannot fuse any other pair; sqrt and the
// divisions are IEEE correctly rounded (HIP's default).  This matches the oracle's AdamW
// bit for bit except where the host's vectorised sqrtf is not correctly rounded
// (tests/test_gpu_parity.py::test_adamw_bitwise_vs_oracle).
// -------------------------------------------------------------------------------------
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, int64_t n,
                             AdamwScalars a) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        float pi = p[i], mi = m[i], vi = v[i];
        adamw_elem(pi, g[i], mi, vi, a);
        p[i] = pi;
        m[i] = mi;
        v[i] = vi;
    }
}

// 16-B vectorised form (same per-element code): 28 B/parameter in 7 dwordx4 accesses
__global__ void adamw4_kernel(float4* __restrict__ p, const float4* __restrict__ g,
                              float4* __restrict__ m, float4* __restrict__ v, int64_t n4,
                              AdamwScalars a) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        float4 pi = p[i], mi = m[i], vi = v[i];
        const float4 gi = g[i];
        adamw_elem(pi.x, gi.x, mi.x, vi.x, a);
        adamw_elem(pi.y, gi.y, mi.y, vi.y, a);
        adamw_elem(pi.z, gi.z, mi.z, vi.z, a);
        adamw_elem(pi.w, gi.w, mi.w, vi.w, a);
        p[i] = pi;
        m[i] = mi;
        v[i] = vi;
    }
}

// sigmoid(x) > 0.5 masks + confusion counts (utils/trainer.py:101-107,217-242):
//   counts[0..3] = TP, FP, FN, TN with targets cast to an integer (astype(int)/astype(uint8):
//                  only t == 1 is positive, utils/utils.py:233-251, trainer.py:220)
//   counts[4..5] = |pred & t!=0|, |pred | t!=0| (astype(bool), calculate_iou utils.py:225-231)
// Integer counts: atomics are exact, the result is deterministic.
__global__ void mask_counts_kernel(const float* __restrict__ x, const float* __restrict__ t,
                                   int64_t n, uint8_t* __restrict__ mask,
                                   unsigned long long* __restrict__ counts) {
    unsigned long long c[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const bool pr = sigmoidf_(x[i]) > 0.5f;
        const float tv = t[i];
        const uint8_t tu = (uint8_t)(int)tv;  // numpy astype(uint8) truncation of {0,1} floats
        const bool pos = tu == 1, neg = tu == 0;
        if (mask) mask[i] = pr ? 1 : 0;
        c[0] += pr && pos;
        c[1] += pr && neg;
        c[2] += !pr && pos;
        c[3] += !pr && neg;
        c[4] += pr && (tv != 0.f);
        c[5] += pr || (tv != 0.f);
    }
    for (int k = 0; k < 6; ++k) {
        unsigned long long s = c[k];
        for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(counts + k, s);
    }
}

// NCHW (N,C,H,W) -> NHWC for in_channels > 1
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int HW,
                                    float* __restrict__ y) {
    const int64_t total = (int64_t)N * C * HW;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        const int64_t p = i / C;
        const int64_t img = p / HW, hw = p % HW;
        y[i] = x[(img * C + c) * HW + hw];
    }
}

inline int grid_for(int64_t n, int block = 256, int cap = 8192) {
    int64_t g = (n + block - 1) / block;
    if (g > cap) g = cap;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

// ============================ host launchers ============================
#define LAUNCH_CHECK() return (int)hipGetLastError()

int k_pack_all(const PackJobs& jobs, const float* prm, float* pack, int bf16, hipStream_t s) {
    if (jobs.n < 1 || jobs.n > MAX_PACK_JOBS) return -1;
    const PackJob& last = jobs.j[jobs.n - 1];
    const int blocks = last.block0 + last.tx * last.ty;
    if (bf16)
        hipLaunchKernelGGL(pack_all_kernel<__bf16>, dim3(blocks), dim3(256), 0, s, jobs, prm, pack, AdamArena{},
                           AdamwScalars{});
    else
        hipLaunchKernelGGL(pack_all_kernel<float>, dim3(blocks), dim3(256), 0, s, jobs, prm, pack, AdamArena{},
                           AdamwScalars{});
    LAUNCH_CHECK();
}
int k_pack_adamw(const PackJobs& jobs, const AdamRanges& rest, float* p, const float* g, float* m, float* v,
                 const AdamwScalars& a, float* pack, int bf16, hipStream_t s) {
    if (jobs.n < 1 || jobs.n > MAX_PACK_JOBS || rest.n < 0 || rest.n > MAX_ADAM_RANGES) return -1;
    const PackJob& last = jobs.j[jobs.n - 1];
    const int blocks = last.block0 + last.tx * last.ty;
    const AdamArena ad{p, g, m, v};
    if (bf16)
        hipLaunchKernelGGL((pack_all_kernel<__bf16, true>), dim3(blocks), dim3(256), 0, s, jobs, nullptr, pack, ad, a);
    else
        hipLaunchKernelGGL((pack_all_kernel<float, true>), dim3(blocks), dim3(256), 0, s, jobs, nullptr, pack, ad, a);
    HIP_OK(hipGetLastError());
    if (rest.n > 0 && rest.cum[rest.n] > 0)
        hipLaunchKernelGGL(adamw_ranges_kernel, dim3(grid_for(rest.cum[rest.n], 256, 1024)), dim3(256), 0, s, rest,
                           ad, a);
    LAUNCH_CHECK();
}
int k_conv_first_fwd(const float* x, const float* w, const float* b, float* y, int P, int H, int W,
                     int C, int relu, float* partial, int G, hipStream_t s) {
    if (C % 4 || C > 1024) return -1;
    const size_t xs = sizeof(float) * ((P + G - 1) / G + 2 * (size_t)W + 2);  // staged x slice
    if (xs > 56 * 1024) return -1;
    hipLaunchKernelGGL(conv_first_fwd_kernel, dim3(G), dim3(256), xs, s, x, w, b, y, P, H, W, C,
                       relu, partial);
    LAUNCH_CHECK();
}
int k_conv_first_wgrad(const float* x, const float* dout, const float* y, const float* coef, int P,
                       int H, int W, int C, int mask, float* partial, int G, float* gw, float* gb,
                       hipStream_t s) {
    if (C % 4 || C > 1024) return -1;
    const size_t xs = sizeof(float) * ((P + G - 1) / G + 2 * (size_t)W + 2);  // staged x slice
    if (xs > 56 * 1024) return -1;
    hipLaunchKernelGGL(conv_first_wgrad_kernel, dim3(G), dim3(256), xs, s, x, dout, y, coef, P, H, W,
                       C, mask, partial);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(conv_first_wgrad_finalize_kernel, dim3((10 * C + 63) / 64), dim3(64, 16), 0,
                       s, partial, G, C, gw, gb);
    LAUNCH_CHECK();
}
int k_reduce_rows(const float* in, int R, int ncols, float* out, int G, hipStream_t s) {
    hipLaunchKernelGGL(reduce_rows_kernel, dim3((ncols + 255) / 256, G), dim3(256), 0, s, in, R,
                       ncols, out);
    LAUNCH_CHECK();
}
int k_bn_finalize_train(const float* part, int G, int C, double count, const float* gamma,
                        const float* beta, float* rmean, float* rvar, int64_t* nbt, float momentum,
                        float eps, float* scale, float* shift, float* mean, float* invstd,
                        hipStream_t s) {
    hipLaunchKernelGGL(bn_finalize_train_kernel, dim3((C + 63) / 64), dim3(64, 16), 0, s, part, G,
                       C, count, gamma, beta, rmean, rvar, nbt, momentum, eps, scale, shift, mean,
                       invstd);
    LAUNCH_CHECK();
}
int k_bn_finalize_eval(int C, const float* gamma, const float* beta, const float* rmean,
                       const float* rvar, float eps, float* scale, float* shift, hipStream_t s) {
    hipLaunchKernelGGL(bn_finalize_eval_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma,
                       beta, rmean, rvar, eps, scale, shift);
    LAUNCH_CHECK();
}
int k_maxpool_bn(const float* y, int ld, int off, const float* scale, const float* shift, int relu,
                 int N, int H, int W, int C, float* out, uint8_t* idx, hipStream_t s, uint16_t* out3,
                 uint16_t* pool16, uint16_t* skip16, uint16_t* skip3, int ldk, int so) {
    const int64_t n = (int64_t)N * (H / 2) * (W / 2) * (C / 4);
    const int c4n = C / 4;
    if ((!out && !out3 && !pool16) || (out3 && C % 32)) return -1;
    if ((skip16 || skip3) && (so % 4 || ldk % 4 || so + C > ldk || (skip3 && (so % 32 || ldk % 32))))
        return -1;
    const PoolImg pi{pool16, skip16, skip3, ldk, so};
    if (C % 4 == 0 && c4n >= 1 && (int64_t)N * H * W < (1ll << 31))
        hipLaunchKernelGGL(maxpool_bn_kernel, dim3(grid_for(n)), dim3(256), 0, s, y, ld, off, scale,
                           shift, relu, N, H, W, C, out, idx, out3, pi);
    else
        hipLaunchKernelGGL(maxpool_bn_any_kernel, dim3(grid_for(n)), dim3(256), 0, s, y, ld, off,
                           scale, shift, relu, N, H, W, C, out, idx, out3, pi);
    LAUNCH_CHECK();
}
int k_maxpool_bwd(const float* dp, const uint8_t* idx, const float* dskip, int ldskip, int offskip,
                  const float* y, int ldy, int offy, const float* mscale, const float* mshift,
                  int N, int H, int W, int C, float* dout, float* partial, int G, hipStream_t s) {
    if ((int64_t)N * H * W >= (1ll << 31)) return -1;  // 32-bit pixel index math
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(G), dim3(256), 0, s, dp, idx, dskip, ldskip,
                       offskip, y, ldy, offy, mscale, mshift, N, H, W, C, dout, partial);
    LAUNCH_CHECK();
}
int k_bn_bwd_finalize2(const float* part, int G, int C, double count, const float* gamma,
                       const float* mean, const float* invstd, float* coef, float* dgamma,
                       float* dbeta, hipStream_t s) {
    hipLaunchKernelGGL(bn_bwd_finalize2_kernel, dim3((C + 63) / 64), dim3(64, 16), 0, s, part, G, C,
                       count, gamma, mean, invstd, coef, dgamma, dbeta);
    LAUNCH_CHECK();
}
int k_bn_dz(float* d, const float* y, int ld, int off, int64_t P, int C, const float* coef, int mask,
            hipStream_t s) {
    if (C % 4 == 0 && C >= 4 && C <= 1024)
        hipLaunchKernelGGL(bn_dz_rows_kernel, dim3(grid_for(P * (C / 4))), dim3(256), 0, s, d, y, ld,
                           off, P, C, coef, mask);
    else
        hipLaunchKernelGGL(bn_dz_kernel, dim3(grid_for(P * (C / 4))), dim3(256), 0, s, d, y, ld, off,
                           P, C, coef, mask);
    LAUNCH_CHECK();
}
int k_to_bf16(const float* src, int ld, int off, int C, const float* scale, const float* shift,
              int relu, int64_t P, uint16_t* dst, hipStream_t s, int dld) {
    if (dld == 0) dld = C;
    if (C % 8 || ld % 4 || off % 4 || dld % 8 || dld < C || (scale == nullptr) != (shift == nullptr))
        return -1;
    const int c8 = C / 8;
    const int tpr = c8 >= 256 ? 256 : c8;
    if (256 % tpr || (c8 > 256 && c8 % 256)) return -1;
    hipLaunchKernelGGL(to_bf16_kernel, dim3(grid_for((P + 3) / 4 * tpr)), dim3(256), 0, s, src, ld, off, C,
                       scale, shift, relu, P, tpr, (__bf16*)dst, dld);
    LAUNCH_CHECK();
}
int k_bn_dz16(float* d, const float* y, int ld, int off, int64_t P, int C, const float* coef,
              int mask, uint16_t* dz16, int f32, hipStream_t s, const float* hdl, const float* hw,
              const float* hsc, const float* hsh, int hrelu) {
    if (C % 8 || ld % 4 || off % 4) return -1;
    const int c8 = C / 8;
    const int tpr = c8 >= 256 ? 256 : c8;
    if (256 % tpr || (c8 > 256 && c8 % 256)) return -1;
    if (hdl) {  // do recomputed from the head: no do to read, none to write back
        if (!hw || !hsc || !hsh || f32) return -1;
        hipLaunchKernelGGL(bn_dz16_kernel<1>, dim3(grid_for((P + 3) / 4 * tpr)), dim3(256), 0, s, nullptr, y, ld,
                           off, P, C, coef, mask, tpr, (__bf16*)dz16, 0, Dz16Pool{},
                           Dz16Head{hdl, hw, hsc, hsh, hrelu});
        LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(bn_dz16_kernel<0>, dim3(grid_for((P + 3) / 4 * tpr)), dim3(256), 0, s, d, y, ld, off,
                       P, C, coef, mask, tpr, (__bf16*)dz16, f32, Dz16Pool{}, Dz16Head{});
    LAUNCH_CHECK();
}
int k_bn_dz16_pool(const float* y, int ld, int off, int64_t P, int C, const float* coef, int mask,
                   uint16_t* dz16, const float* dp, const uint8_t* idx, const float* dskip, int ldskip,
                   const float* msc, const float* msh, int N, int H, int W, hipStream_t s) {
    if (C % 8 || ld % 4 || off % 4 || ldskip % 4) return -1;
    if (!dp || !idx || !dskip || H % 2 || W % 2 || (int64_t)N * H * W != P || P >= (1LL << 24)) return -1;
    const int c8 = C / 8;
    const int tpr = c8 >= 256 ? 256 : c8;
    if (256 % tpr || (c8 > 256 && c8 % 256)) return -1;
    const Dz16Pool pl{dp, idx, dskip, ldskip, msc, msh, H, W, 1.f / (float)H, 1.f / (float)W};
    hipLaunchKernelGGL(bn_dz16_kernel<2>, dim3(grid_for((P + 3) / 4 * tpr)), dim3(256), 0, s, nullptr, y, ld,
                       off, P, C, coef, mask, tpr, (__bf16*)dz16, 0, pl, Dz16Head{});
    LAUNCH_CHECK();
}
int k_bias_reduce(const float* slab, int S, int taps, int C, float* out, hipStream_t s) {
    hipLaunchKernelGGL(bias_reduce_kernel, dim3((C + 63) / 64), dim3(64, 16), 0, s, slab, S, taps, C,
                       out);
    LAUNCH_CHECK();
}
int k_up2_bias_partials(const float* d, int ld, int off, int H, int W, int64_t P, int C, int pps,
                        int splits, float* bslab, hipStream_t s) {
    if (C % 4 || ld % 4 || off % 4 || pps < 1 || splits < 1 || 4 * P >= (1ll << 31)) return -1;
    hipLaunchKernelGGL(up2_bias_partials_kernel, dim3(splits, 4, (C + 63) / 64), dim3(256), 0, s, d,
                       ld, off, H, W, P, C, pps, bslab);
    LAUNCH_CHECK();
}
int k_sum_partials(const float* part, int G, int ncols, float* out, hipStream_t s) {
    hipLaunchKernelGGL(sum_partials_kernel, dim3((ncols + 63) / 64), dim3(64, 16), 0, s, part, G,
                       ncols, out);
    LAUNCH_CHECK();
}
int k_slab_reduce(const float* slab, int S, int Mw, int Nw, int kind, int cin, int cout,
                  float* grad, hipStream_t s) {
    if (kind == 0 && S == 1 && cin % 32 == 0 && cout % 32 == 0 && (cin / 32) * (cout / 32) >= 128) {
        hipLaunchKernelGGL(slab_reduce_conv3_kernel<32>, dim3(cout / 32, cin / 32), dim3(256), 0, s, slab,
                           S, cin, cout, grad);
        LAUNCH_CHECK();
    }
    if (kind == 0 && S > 1 && S < 32 && cin % 8 == 0 && cout % 32 == 0 && (cin / 8) * (cout / 32) >= 256) {
        hipLaunchKernelGGL(slab_reduce_conv3_kernel<8>, dim3(cout / 32, cin / 8), dim3(256), 0, s, slab,
                           S, cin, cout, grad);
        LAUNCH_CHECK();
    }
    if (kind == 1 && S < 32 && Mw == cin && Nw == 4 * cout && ((uintptr_t)grad & 15) == 0) {
        hipLaunchKernelGGL(slab_reduce_convT_kernel, dim3((int)(((int64_t)cin * cout + 255) / 256)), dim3(256),
                           0, s, slab, S, cin, cout, grad);
        LAUNCH_CHECK();
    }
    if (Nw % 4) return -1;
    if (S >= 32) {
        hipLaunchKernelGGL(slab_reduce_wide_kernel, dim3((int)(((int64_t)Mw * Nw / 4 + 15) / 16)),
                           dim3(256), 0, s, slab, S, Mw, Nw, kind, cin, cout, grad);
        LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(slab_reduce_kernel, dim3(grid_for((int64_t)Mw * Nw / 4)), dim3(256), 0, s,
                       slab, S, Mw, Nw, kind, cin, cout, grad);
    LAUNCH_CHECK();
}
int k_pack_1x1_t(const float* w, float* wt, int cin, int cout, hipStream_t s) {
    hipLaunchKernelGGL(pack_1x1_t_kernel, dim3(grid_for((int64_t)cin * cout)), dim3(256), 0, s, w, wt,
                       cin, cout);
    LAUNCH_CHECK();
}
int k_res_first_fwd(const float* x, const float* ws, const float* z, const float* sc,
                    const float* sh, int64_t P, int C, float* out, int ldo, int offo, hipStream_t s) {
    if (C % 4) return -1;
    hipLaunchKernelGGL(res_first_fwd_kernel, dim3(grid_for(P * (C / 4))), dim3(256), 0, s, x, ws, z,
                       sc, sh, P, C, out, ldo, offo);
    LAUNCH_CHECK();
}
int k_res_bwd_prep(float* d, const float* out, int ldo, int offo, const float* z, int64_t P, int C,
                   float* partial, int G, hipStream_t s) {
    if (C % 4) return -1;
    hipLaunchKernelGGL(res_bwd_prep_kernel, dim3(G), dim3(256), 0, s, d, out, ldo, offo, z, P, C,
                       partial);
    LAUNCH_CHECK();
}
int k_res_first_wgrad(const float* x, const float* du, int P, int C, float* partial, int G,
                      float* gw, hipStream_t s) {
    if (C % 4 || C > 1024) return -1;
    hipLaunchKernelGGL(res_first_wgrad_kernel, dim3(G), dim3(256), 0, s, x, du, P, C, partial);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(sum_partials_kernel, dim3((C + 63) / 64), dim3(64, 16), 0, s, partial, G, C,
                       gw);
    LAUNCH_CHECK();
}
int k_head_fwd(const float* y, int C, const float* scale, const float* shift, int relu,
               const float* w, const float* b, int O, int P, int HW, float* logits, hipStream_t s) {
    if (C % 4 || C / 4 > 64 || (C / 4 & (C / 4 - 1))) return -1;  // lanes per pixel: pow2 <= 64
    const int64_t threads = (int64_t)P * (C / 4);
    if (threads + 255 >= (1ll << 31)) return -1;  // the kernel's 32-bit thread index
    // 4 pixels per thread (head_fwd_kernel U), at most 8192 blocks (a grid-stride remainder)
    hipLaunchKernelGGL(head_fwd_kernel, dim3(grid_for((threads + 3) / 4)), dim3(256), 0, s, y,
                       C, scale, shift, relu, w, b, O, P, HW, logits);
    LAUNCH_CHECK();
}
int k_head_bwd(const float* y, int C, const float* scale, const float* shift, int relu,
               const float* w, int O, int P, int HW, const float* dlog, float* dout, float* partial,
               float* bnpart, int G, hipStream_t s) {
    if (C % 4 || C / 4 > 256 || O > 4) return -1;
    hipLaunchKernelGGL(head_bwd_kernel, dim3(G), dim3(256), 0, s, y, C, scale, shift, relu, w, O, P,
                       HW, dlog, dout, partial, bnpart);
    LAUNCH_CHECK();
}
int loss_groups(int64_t per) { return (int)std::min<int64_t>(256, std::max<int64_t>(1, per / 4096)); }
int k_loss_stats(const float* x, const float* t, int N, int64_t per, float* stats, double* sums,
                 float* part, hipStream_t s) {
    const int G = loss_groups(per);
    hipLaunchKernelGGL(loss_stats_kernel, dim3(N * G), dim3(256), 0, s, x, t, per, G, part);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(loss_sums_kernel, dim3(1), dim3(256), 0, s, part, G, stats, N, per, sums);
    LAUNCH_CHECK();
}
int k_loss_finalize(const double* sums, float alpha, float beta, float gamma, float* losses,
                    hipStream_t s) {
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(64), 0, s, sums, alpha, beta, gamma,
                       losses);
    LAUNCH_CHECK();
}
int k_loss_bwd(const float* x, const float* t, int N, int64_t per, const float* stats,
               const double* sums, const float* w, float alpha, float beta, float gamma, float* dx,
               hipStream_t s) {
    hipLaunchKernelGGL(loss_bwd_kernel, dim3(grid_for(per * N)), dim3(256), 0, s, x, t, per, N,
                       stats, sums, w, alpha, beta, gamma, dx);
    LAUNCH_CHECK();
}
int k_adamw(float* p, const float* g, float* m, float* v, int64_t n, const AdamwScalars& a,
            hipStream_t s) {
    if ((n & 3) == 0 && ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0)
        hipLaunchKernelGGL(adamw4_kernel, dim3(grid_for(n / 4, 256, 16384)), dim3(256), 0, s,
                           (float4*)p, (const float4*)g, (float4*)m, (float4*)v, n / 4, a);
    else
        hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n, 256, 16384)), dim3(256), 0, s, p, g, m, v,
                           n, a);
    LAUNCH_CHECK();
}
int k_mask_counts(const float* x, const float* t, int64_t n, uint8_t* mask, int64_t* counts,
                  hipStream_t s) {
    hipLaunchKernelGGL(mask_counts_kernel, dim3(grid_for(n, 256, 2048)), dim3(256), 0, s, x, t, n,
                       mask, (unsigned long long*)counts);
    LAUNCH_CHECK();
}
int k_nchw_to_nhwc(const float* x, int N, int C, int HW, float* y, hipStream_t s) {
    hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for((int64_t)N * C * HW)), dim3(256), 0, s, x,
                       N, C, HW, y);
    LAUNCH_CHECK();
}

namespace {
// one tensor per blockIdx.y; grid-stride over its padded (expand) or real (compact) elements
__global__ __launch_bounds__(256) void pad_copy_kernel(const PadDesc* __restrict__ table,
                                                       const float* __restrict__ src,
                                                       float* __restrict__ dst, int expand) {
    const PadDesc d = table[blockIdx.y];
    int64_t rd[4], pd[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rd[k] = (int64_t)d.seg[k] * d.nseg[k];
        pd[k] = (int64_t)d.pseg[k] * d.nseg[k];
    }
    const int64_t n = expand ? d.pnumel : d.rnumel;
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * blockDim.x) {
        // decode j over the (padded or real) dims, innermost last
        int64_t rem = j, ridx = 0, pidx = 0, rstride = 1, pstride = 1;
        bool valid = true;
#pragma unroll
        for (int k = 3; k >= 0; --k) {
            const int64_t ext = expand ? pd[k] : rd[k];
            const int64_t i = rem % ext;
            rem /= ext;
            int64_t sg, w;
            if (expand) {
                sg = i / d.pseg[k];
                w = i - sg * d.pseg[k];
                valid = valid && w < d.seg[k];
            } else {
                sg = i / d.seg[k];
                w = i - sg * d.seg[k];
            }
            ridx += (sg * d.seg[k] + w) * rstride;
            pidx += (sg * d.pseg[k] + w) * pstride;
            rstride *= rd[k];
            pstride *= pd[k];
        }
        if (expand)
            dst[d.poff + j] = valid ? src[d.roff + ridx] : 0.f;
        else
            dst[d.roff + j] = src[d.poff + pidx];
    }
}

__global__ void fill_kernel(float* __restrict__ p, int64_t n, float v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}
}  // namespace
int k_pad_copy(const PadDesc* table, int n, int64_t max_numel, const float* src, float* dst,
               int expand, hipStream_t s) {
    if (n <= 0) return 0;
    const int64_t nb = (max_numel + 255) / 256;
    const unsigned bx = (unsigned)(nb < 1024 ? nb : 1024);
    hipLaunchKernelGGL(pad_copy_kernel, dim3(bx > 0 ? bx : 1, n), dim3(256), 0, s, table, src, dst,
                       expand);
    LAUNCH_CHECK();
}
int k_fill(float* p, int64_t n, float v, hipStream_t s) {
    hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, s, p, n, v);
    LAUNCH_CHECK();
}

// -------------------------------------------------------------------------------------
// Input pipeline: PIL-exact bilinear resize of a uint8 image + ToTensor scaling
// (utils/transforms.py:143-156: TF.resize on a PIL image = Image.resize(size, BILINEAR),
// then TF.to_tensor = float(u8) / 255).  Pillow's 8-bit resampler (libImaging/Resample.c)
// is two separable passes with fixed-point coefficients (22 fraction bits) and a clip to
// uint8 after EACH pass, horizontal first.  One thread per output pixel recomputes the
// horizontal-pass values of the rows it needs (identical integers to Pillow's temporary
// image), so the result is bit-exact.  Coefficients / bounds come from the host
// (runtime.hip: pil_resample_plan), in Pillow's layout: k[out][ksize], b[out] = {min, n}.
// -------------------------------------------------------------------------------------
namespace {
constexpr int PIL_PRECISION_BITS = 32 - 8 - 2;

__device__ __forceinline__ int pil_clip8(int v) {
    if (v >= (1 << PIL_PRECISION_BITS << 8)) return 255;
    if (v <= 0) return 0;
    return v >> PIL_PRECISION_BITS;
}

__global__ void resize_u8_pil_kernel(const uint8_t* __restrict__ src, int H, int W,
                                     float* __restrict__ dst, int OH, int OW,
                                     const int* __restrict__ kh, const int* __restrict__ bh, int ksh,
                                     const int* __restrict__ kv, const int* __restrict__ bv, int ksv,
                                     int need_h, int need_v, float divisor) {
    const int64_t n = (int64_t)OH * OW;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int yy = (int)(i / OW), xx = (int)(i % OW);
        // horizontal pass value of source row y at output column xx
        auto hval = [&](int y) -> int {
            if (!need_h) return src[(int64_t)y * W + xx];
            const int xmin = bh[2 * xx], xn = bh[2 * xx + 1];
            int ss = 1 << (PIL_PRECISION_BITS - 1);
            for (int x = 0; x < xn; ++x) ss += (int)src[(int64_t)y * W + xmin + x] * kh[xx * ksh + x];
            return pil_clip8(ss);
        };
        int v;
        if (need_v) {
            const int ymin = bv[2 * yy], yn = bv[2 * yy + 1];
            int ss = 1 << (PIL_PRECISION_BITS - 1);
            for (int y = 0; y < yn; ++y) ss += hval(ymin + y) * kv[yy * ksv + y];
            v = pil_clip8(ss);
        } else {
            v = hval(yy);
        }
        dst[i] = (float)v / divisor;  // TF.to_tensor divides (torch div), not x * (1/255)
    }
}
}  // namespace

int k_resize_u8(const uint8_t* src, int H, int W, float* dst, int OH, int OW, const int* kh,
                const int* bh, int ksh, const int* kv, const int* bv, int ksv, int need_h,
                int need_v, float divisor, hipStream_t s) {
    hipLaunchKernelGGL(resize_u8_pil_kernel, dim3(grid_for((int64_t)OH * OW)), dim3(256), 0, s, src,
                       H, W, dst, OH, OW, kh, bh, ksh, kv, bv, ksv, need_h, need_v, divisor);
    LAUNCH_CHECK();
}
