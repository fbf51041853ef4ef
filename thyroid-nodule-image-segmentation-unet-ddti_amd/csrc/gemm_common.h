// Shared device helpers of the row-GEMM kernels (kernels_gemm.hip: f32 and register-staged
// bf16; kernels_gemm16.hip: LDS-DMA bf16): MFMA wrappers, pixel decode, the implicit-conv
// row gather and the epilogues (bias / ReLU / BN statistics, ConvTranspose scatter, BN-backward
// partials, residual close), so every kernel family stores identical results.
#pragma once
#include "common.h"
#include "x3_split.h"

namespace {

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// bf16 operands (BF kernels): 8 bf16 per lane, k = 8 * (lane >> 5) + j
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma32_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// 16x16x32 (r05): lane l feeds A row slot l & 15 / B column slot l & 15 with k = 8 (l >> 4) + j
// and holds D rows 4 (l >> 4) + i, column l & 15.  Under load the chip holds a higher clock on
// this shape than on 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH.md, DVFS item 7).
__device__ __forceinline__ f32x4 mfma16_bf16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// A row slot rs of a 16-row block -> row within the block, chosen so that 2 x 2 blocks of
// 16 x 16 hold, after one exchange between lanes l and l ^ 16 per register pair, exactly the
// 32x32x16 accumulator layout of their 32 x 32 block (acc16_to32)
__device__ __forceinline__ int m16_row(int rs) { return ((rs >> 2) & 1) * 8 + (rs >> 3) * 4 + (rs & 3); }

// [bm][bn] 16x16 blocks (rows via m16_row) -> one 32x32x16-layout f32x16
__device__ __forceinline__ void acc16_to32(const f32x4 (&a)[2][2], f32x16& acc, int lane) {
    const bool odd = (lane >> 4) & 1;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float v0 = a[bm][0][i], v1 = a[bm][1][i];
            const float p0 = __shfl_xor(v0, 16), p1 = __shfl_xor(v1, 16);
            acc[8 * bm + i] = odd ? p1 : v0;
            acc[8 * bm + 4 + i] = odd ? v1 : p0;
        }
}

// f32x4 -> 4 bf16 (round to nearest even; v_cvt_pk_bf16_f32)
__device__ __forceinline__ bf16x4 to_bf16x4(f32x4 v) {
    return bf16x4{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
}

struct Pix {
    int img, y, x;
};

// Blocks are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), each with its
// own L2.  Give XCD x the contiguous logical tiles [x*n/8, (x+1)*n/8) instead, so tiles
// that share input rows (3x3 halos, the taps and channel slices of one pixel range) hit
// the same L2.
__device__ __forceinline__ int xcd_remap(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7, i = b >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// (r06) remapped block -> (tile_m, tile_n).  gm <= 1: M-major (consecutive blocks walk the N
// tiles of one M tile).  gm > 1: groups of gm M tiles, each group walking its N tiles with the
// group's M tiles fastest, so a run of consecutive blocks -- the blocks one XCD holds at once,
// after xcd_remap -- covers a gm x (run / gm) rectangle of tiles instead of one or two M tiles
// x every N tile.  Where the weight matrix is large (config 4's 16² / 32² levels: 75-151 MB of
// bf16 weights, every XCD re-reading all of it under M-major order) that cuts the distinct A and
// B rows per XCD L2.  The order never changes what a tile computes: bit-identical.
__device__ __forceinline__ void tile_mn(int bid, int ntm, int ntn, int gm, int& tm, int& tn) {
    if (gm <= 1) {
        tm = bid / ntn;
        tn = bid - tm * ntn;
        return;
    }
    const int per = gm * ntn, grp = bid / per, first = grp * gm;
    const int gs = min(ntm - first, gm);
    const int r = bid - grp * per;
    tn = r / gs;
    tm = first + (r - tn * gs);
}

__device__ __forceinline__ Pix decode(int m, int H, int W) {
    Pix r;
    int t = m / W;
    r.x = m - t * W;
    r.img = t / H;
    r.y = t - r.img * H;
    return r;
}

// q += d pixels (row-major over H x W images), without dividing
__device__ __forceinline__ void pix_advance(Pix& q, int d, int H, int W) {
    q.x += d;
    while (q.x >= W) {
        q.x -= W;
        if (++q.y == H) {
            q.y = 0;
            ++q.img;
        }
    }
}

// Division by a per-launch constant through an f32 reciprocal plus one correction step:
// exact while the quotient stays below 2^22 (P / W < 4M pixel rows here).
__device__ __forceinline__ int fdiv(int n, int d, float rd) {
    int q = (int)((float)n * rd);
    const int r = n - q * d;
    q += (r >= d) ? 1 : 0;
    q -= (r < 0) ? 1 : 0;
    return q;
}

__device__ __forceinline__ Pix decode_fast(int m, int H, int W, float rH, float rW) {
    Pix r;
    const int t = fdiv(m, W, rW);
    r.x = m - t * W;
    r.img = fdiv(t, H, rH);
    r.y = t - r.img * H;
    return r;
}

// Source pixel of row pixel `q` (on grid HxW) for `tap` in MODE; `valid` false for
// zero-padding taps (the returned index is then the row pixel itself, always in range).
template <int MODE>
__device__ __forceinline__ int gather_src(int tap, int m, Pix q, int H, int W, bool& valid) {
    if constexpr (MODE == G_CONV3) {
        const int yy = q.y + tap / 3 - 1, xx = q.x + tap % 3 - 1;
        valid = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W);
        return valid ? (q.img * H + yy) * W + xx : m;
    } else if constexpr (MODE == G_UP2) {
        valid = true;
        const int a = tap >> 1, b = tap & 1;
        return (q.img * 2 * H + 2 * q.y + a) * (2 * W) + 2 * q.x + b;
    } else {
        valid = true;
        return m;
    }
}

// ------------------------------------------------------------------------------------
// Row-GEMM epilogue: accumulators acc[MT][NT] of wave (wm, wn) of the BM x BN block tile at
// (m0, n0); tile_m indexes the block row; smem (>= (BM / 64) * 2 * BN doubles) is free
// scratch (the caller has finished with its LDS images).
//
// BN partials (E_BIAS_RELU_STATS / E_STATS / E_STORE_BN) are emitted per 128-ROW GROUP
// whatever the tile: partial row tile_m * (BM / 128) + g.  Inside a group the sum runs in a
// fixed order -- per lane over each 64-row unit's 32 rows in (mt, r) order, the two lane
// halves combined, then unit 0 + unit 1 -- so a 128x128 tile (two 64-row waves), a 256x128
// tile (four) and a 256x256 tile (two 128-row waves, two units each) produce bit-identical
// partial rows, and the tile choice changes speed only (tests/test_gpu_mod.py).  The
// squared terms are explicit fmas: left to -ffp-contract, hipcc fused them in some tile
// instantiations and not in others (a 1-ulp invstd difference between 128- and 256-row
// tiles, tools/diag_tile.py).
// ------------------------------------------------------------------------------------
// PRELOAD: the epilogues that read memory (E_STORE_BN, E_RESID, E_ADD) issue all 16 loads
// of an accumulator first -- a load under `if (m < M)` makes hipcc wait for each one before
// the next, which dominated the short-K bf16 GEMMs; the long-K f32 kernels keep the
// per-element form (fewer live registers, measured 4 % faster on their dgrads).
template <int EMODE, int BM, int BN, int WM, int WN, bool PRELOAD = false>
__device__ __forceinline__ void row_epilogue(const RowGemmArgs& p, f32x16 (&acc)[WM / 32][WN / 32],
                                             int m0, int n0, int tile_m, int wm, int wn,
                                             int lane, int tid, float* smem) {
    constexpr int MT = WM / 32, NT = WN / 32, WAVES_M = BM / WM;
    constexpr int U = WM / 64;           // 64-row units per wave
    constexpr int GB = BM / 128;         // 128-row BN groups per block
    constexpr int THREADS = 64 * WAVES_M * (BN / WN);
    static_assert(WM % 64 == 0 && BM % 128 == 0, "BN partial groups need 64-row units");
    const int li = lane & 31, lh = lane >> 5;
    const int H = p.H, W = p.W;
    // FULL: the block tile lies inside M, so no row needs a guard.  Row (mt, r) of the wave
    // then has a wave-uniform base address (SGPRs) and each lane a fixed 32-bit byte offset
    // (4 lh rows + its column): one store per element, no per-element branch or 64-bit
    // address arithmetic.  Same values, same order as the guarded path.
    const bool full = m0 + BM <= p.M;
    const int wrow = __builtin_amdgcn_readfirstlane(m0 + wm * WM);
    auto urow = [&](const float* base, int ld, int off, int mt, int r) {
        return (const char*)(base + (size_t)(wrow + mt * 32 + (r & 3) + 8 * (r >> 2)) * ld + off);
    };
    if constexpr (EMODE == E_BIAS_RELU_STATS || EMODE == E_STATS) {
        constexpr bool BR = EMODE == E_BIAS_RELU_STATS;
        float s1[U][NT], s2[U][NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int n = n0 + wn * WN + nt * 32 + li;
            const float b = BR ? p.bias[n] : 0.f;
#pragma unroll
            for (int u = 0; u < U; ++u) s1[u][nt] = s2[u][nt] = 0.f;
            if (full) {
                const unsigned lo = (unsigned)(4 * lh * p.ldo + n) * 4u;
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float v = BR ? fmaxf(acc[mt][nt][r] + b, 0.f) : acc[mt][nt][r];
                        *(float*)(urow(p.out, p.ldo, p.ooff, mt, r) + lo) = v;
                        s1[mt / 2][nt] += v;
                        s2[mt / 2][nt] = __builtin_fmaf(v, v, s2[mt / 2][nt]);
                    }
            } else {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                        if (m < p.M) {
                            const float v = BR ? fmaxf(acc[mt][nt][r] + b, 0.f) : acc[mt][nt][r];
                            p.out[(size_t)m * p.ldo + p.ooff + n] = v;
                            s1[mt / 2][nt] += v;
                            s2[mt / 2][nt] = __builtin_fmaf(v, v, s2[mt / 2][nt]);
                        }
                    }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                s1[u][nt] += __shfl_xor(s1[u][nt], 32);
                s2[u][nt] += __shfl_xor(s2[u][nt], 32);
            }
        }
        // combine the 64-row units of each 128-row group (LDS is free after the loop)
        __syncthreads();
        float* red = smem;  // [BM / 64][2][BN]
        if (lh == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int ub = wm * U + u;
                    red[(ub * 2 + 0) * BN + wn * WN + nt * 32 + li] = s1[u][nt];
                    red[(ub * 2 + 1) * BN + wn * WN + nt * 32 + li] = s2[u][nt];
                }
        }
        __syncthreads();
        for (int i = tid; i < GB * BN; i += THREADS) {
            const int g = i / BN, col = i - g * BN;
            float a = 0.f, q = 0.f;
#pragma unroll
            for (int w = 2 * g; w < 2 * g + 2; ++w) {
                a += red[(w * 2 + 0) * BN + col];
                q += red[(w * 2 + 1) * BN + col];
            }
            if (m0 + g * 128 < p.M) {
                const size_t row = (size_t)tile_m * GB + g;
                p.stats[row * 2 * p.N + n0 + col] = a;
                p.stats[row * 2 * p.N + p.N + n0 + col] = q;
            }
        }
    } else if constexpr (EMODE == E_STORE_BN) {
        // BN-backward partials are differences of nearly equal sums downstream (sum do can be
        // 1e-3 of sum |do|): accumulate in f64, round once per 128-row group.
        const bool emask = p.escale != nullptr;
        double q[U][NT][2];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int n = n0 + wn * WN + nt * 32 + li;
            const float es = emask ? p.escale[n] : 0.f, eb = emask ? p.eshift[n] : 0.f;
#pragma unroll
            for (int u = 0; u < U; ++u) q[u][nt][0] = q[u][nt][1] = 0.0;
            const unsigned lo = (unsigned)(4 * lh * p.ldo + n) * 4u;
            const unsigned ly = (unsigned)(4 * lh * p.ldey + n) * 4u;
#pragma unroll
            for (int mt = 0; mt < MT && !PRELOAD && full; ++mt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float v = acc[mt][nt][r];
                    const float y = *(const float*)(urow(p.ey, p.ldey, p.offey, mt, r) + ly);
                    if (emask && !(es * y + eb > 0.f)) v = 0.f;
                    *(float*)(urow(p.out, p.ldo, p.ooff, mt, r) + lo) = v;
                    q[mt / 2][nt][0] += v;
                    q[mt / 2][nt][1] = __builtin_fma((double)v, (double)y, q[mt / 2][nt][1]);
                }
#pragma unroll
            for (int mt = 0; mt < MT && !PRELOAD && !full; ++mt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (m < p.M) {
                        float v = acc[mt][nt][r];
                        const float y = p.ey[(size_t)m * p.ldey + p.offey + n];
                        if (emask && !(es * y + eb > 0.f)) v = 0.f;
                        p.out[(size_t)m * p.ldo + p.ooff + n] = v;
                        q[mt / 2][nt][0] += v;
                        q[mt / 2][nt][1] = __builtin_fma((double)v, (double)y, q[mt / 2][nt][1]);
                    }
                }
#pragma unroll
            for (int mt = 0; mt < MT && PRELOAD && full; ++mt) {
                float yv[16];  // all 16 loads first, then the stores (no guards: full tile)
#pragma unroll
                for (int r = 0; r < 16; ++r) yv[r] = *(const float*)(urow(p.ey, p.ldey, p.offey, mt, r) + ly);
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float y = yv[r];
                    float v = acc[mt][nt][r];
                    if (emask && !(es * y + eb > 0.f)) v = 0.f;
                    *(float*)(urow(p.out, p.ldo, p.ooff, mt, r) + lo) = v;
                    q[mt / 2][nt][0] += v;
                    q[mt / 2][nt][1] = __builtin_fma((double)v, (double)y, q[mt / 2][nt][1]);
                }
            }
#pragma unroll
            for (int mt = 0; mt < MT && PRELOAD && !full; ++mt) {
                // all 16 loads first (rows past M clamped, their products zeroed below)
                float yv[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    yv[r] = p.ey[(size_t)(m < p.M ? m : p.M - 1) * p.ldey + p.offey + n];
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    const float y = yv[r];
                    float v = acc[mt][nt][r];
                    if (emask && !(es * y + eb > 0.f)) v = 0.f;
                    if (m < p.M) p.out[(size_t)m * p.ldo + p.ooff + n] = v;
                    v = m < p.M ? v : 0.f;
                    q[mt / 2][nt][0] += v;
                    q[mt / 2][nt][1] = __builtin_fma((double)v, (double)y, q[mt / 2][nt][1]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < 2; ++j) q[u][nt][j] += __shfl_xor(q[u][nt][j], 32);
        }
        __syncthreads();
        double* red = (double*)smem;  // [BM / 64][2][BN]
        if (lh == 0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        red[((wm * U + u) * 2 + j) * BN + wn * WN + nt * 32 + li] = q[u][nt][j];
        }
        __syncthreads();
        for (int i = tid; i < GB * BN; i += THREADS) {
            const int g = i / BN, col = i - g * BN;
            if (m0 + g * 128 >= p.M) continue;
            const size_t row = (size_t)tile_m * GB + g;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                double a = 0.0;
#pragma unroll
                for (int w = 2 * g; w < 2 * g + 2; ++w) a += red[(w * 2 + j) * BN + col];
                p.stats[(row * 2 + j) * p.N + n0 + col] = (float)a;
            }
        }
    } else if constexpr (EMODE == E_CONVT) {
        // one pixel decode per accumulator row (f32-reciprocal division), shared by the NT
        // column groups: with K = Cin as short as 128 the epilogue is a large part of the
        // block, and an integer-division decode per element cost more than its MFMAs
        const float rH = 1.f / (float)H, rW = 1.f / (float)W;
        int coff[NT], co_[NT];
        float bb[NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int n = n0 + wn * WN + nt * 32 + li;
            const int ab = n / p.cout, co = n - ab * p.cout;
            coff[nt] = (ab >> 1) * (2 * W) + (ab & 1);  // (a, b) offset in the output grid
            co_[nt] = co;
            bb[nt] = p.bias[co];
        }
        if (p.out3) {
            // x3 split straight into the consumer's operand image (as k_to_x3), two channels per
            // store: lanes li, li ^ 1 hold neighbouring columns of the same rows, so for each
            // pair of accumulator rows (r, r + 1) the even lane stores row r and the odd lane row
            // r + 1, each for both columns (4-B stores, half the 2-B store instructions)
            const int odd = li & 1;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int r2 = 0; r2 < 8; ++r2) {
                    const int row = 2 * r2 + odd;
                    const int m = m0 + wm * WM + mt * 32 + (row & 3) + 8 * (row >> 2) + 4 * lh;
                    const Pix q = decode_fast(m < p.M ? m : 0, H, W, rH, rW);
                    const size_t ob = (size_t)(q.img * 2 * H + 2 * q.y) * (2 * W) + 2 * q.x;
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) {
                        const float v0 = acc[mt][nt][2 * r2] + bb[nt], v1 = acc[mt][nt][2 * r2 + 1] + bb[nt];
                        const float recv = __shfl_xor(odd ? v0 : v1, 1);
                        const float ve = odd ? recv : v0, vo = odd ? v1 : recv;  // columns li & ~1, li | 1
                        if (m >= p.M) continue;
                        uint16_t he, me, le, ho, mo, lo;
                        x3_split(ve, X3CvtDev{}, he, me, le);
                        x3_split(vo, X3CvtDev{}, ho, mo, lo);
                        const int ch = p.ooff + co_[nt] - odd;
                        uint16_t* d = p.out3 + (ob + coff[nt]) * 3 * (size_t)p.ldo + (ch >> 5) * 96 + (ch & 31);
                        *(uint32_t*)d = (uint32_t)he | ((uint32_t)ho << 16);
                        *(uint32_t*)(d + 32) = (uint32_t)me | ((uint32_t)mo << 16);
                        *(uint32_t*)(d + 64) = (uint32_t)le | ((uint32_t)lo << 16);
                    }
                }
            return;
        }
        if (p.out16 && ((p.ldo | p.ooff | p.cout) & 1) == 0) {
            // bf16 straight into the consumer's operand image (RNE, as k_to_bf16), two channels
            // per 4-B store with the out3 pairing above (r06: half the store instructions)
            const int odd = li & 1;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int r2 = 0; r2 < 8; ++r2) {
                    const int row = 2 * r2 + odd;
                    const int m = m0 + wm * WM + mt * 32 + (row & 3) + 8 * (row >> 2) + 4 * lh;
                    const Pix q = decode_fast(m < p.M ? m : 0, H, W, rH, rW);
                    const size_t ob = (size_t)(q.img * 2 * H + 2 * q.y) * (2 * W) + 2 * q.x;
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) {
                        const float v0 = acc[mt][nt][2 * r2] + bb[nt], v1 = acc[mt][nt][2 * r2 + 1] + bb[nt];
                        const float recv = __shfl_xor(odd ? v0 : v1, 1);
                        const float ve = odd ? recv : v0, vo = odd ? v1 : recv;  // columns li & ~1, li | 1
                        if (m >= p.M) continue;
                        const uint32_t be = __builtin_bit_cast(uint16_t, (__bf16)ve);
                        const uint32_t bo = __builtin_bit_cast(uint16_t, (__bf16)vo);
                        *(uint32_t*)(p.out16 + (ob + coff[nt]) * p.ldo + p.ooff + co_[nt] - odd) = be | (bo << 16);
                    }
                }
            return;
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (m >= p.M) continue;
                const Pix q = decode_fast(m, H, W, rH, rW);
                const size_t ob = (size_t)(q.img * 2 * H + 2 * q.y) * (2 * W) + 2 * q.x;
                if (p.out16) {  // (odd ld / offset / cout: one 2-B store per element)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        ((__bf16*)p.out16)[(ob + coff[nt]) * p.ldo + p.ooff + co_[nt]] =
                            (__bf16)(acc[mt][nt][r] + bb[nt]);
                } else {
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        p.out[(ob + coff[nt]) * p.ldo + p.ooff + co_[nt]] = acc[mt][nt][r] + bb[nt];
                }
            }
    } else if constexpr (EMODE == E_RESID || EMODE == E_ADD) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int n = n0 + wn * WN + nt * 32 + li;
            const float es = EMODE == E_RESID ? p.escale[n] : 0.f;
            const float eb = EMODE == E_RESID ? p.eshift[n] : 0.f;
#pragma unroll
            for (int mt = 0; mt < MT && !PRELOAD; ++mt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (m >= p.M) continue;
                    float* o = p.out + (size_t)m * p.ldo + p.ooff + n;
                    if constexpr (EMODE == E_RESID)
                        *o = fmaxf(acc[mt][nt][r] + (es * p.ey[(size_t)m * p.ldey + p.offey + n] + eb),
                                   0.f);
                    else
                        *o += acc[mt][nt][r];
                }
#pragma unroll
            for (int mt = 0; mt < MT && PRELOAD; ++mt) {
                float xv[16];  // ey (E_RESID) or the current out (E_ADD), loaded up front
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    m = m < p.M ? m : p.M - 1;
                    xv[r] = EMODE == E_RESID ? p.ey[(size_t)m * p.ldey + p.offey + n]
                                             : p.out[(size_t)m * p.ldo + p.ooff + n];
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (m >= p.M) continue;
                    float* o = p.out + (size_t)m * p.ldo + p.ooff + n;
                    if constexpr (EMODE == E_RESID)
                        *o = fmaxf(acc[mt][nt][r] + (es * xv[r] + eb), 0.f);
                    else
                        *o = xv[r] + acc[mt][nt][r];
                }
            }
        }
    } else {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int n = n0 + wn * WN + nt * 32 + li;
            const unsigned lo = (unsigned)(4 * lh * p.ldo + n) * 4u;
            if (full) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        *(float*)(urow(p.out, p.ldo, p.ooff, mt, r) + lo) = acc[mt][nt][r];
            } else {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = m0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                        if (m < p.M) p.out[(size_t)m * p.ldo + p.ooff + n] = acc[mt][nt][r];
                    }
            }
        }
    }
}

}  // namespace
