// Shared definitions for the gfx950 UNet kernels (internal; the public ABI is
// include/unet_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// BN(+ReLU) backward value dz = A do + B (y - mean) + C in one explicit rounding order,
// shared by every kernel that forms it (the bn_dz passes, the OP_DZ GEMM loaders,
// conv_first_wgrad): left to -ffp-contract, hipcc contracted the same source expression
// differently per kernel, and the fused-loader and materialised paths disagreed in the last
// bit.
__device__ __forceinline__ f32x4 bn_dz4(f32x4 a, f32x4 d, f32x4 b, f32x4 y, f32x4 mu, f32x4 c) {
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = __builtin_fmaf(a[j], d[j], __builtin_fmaf(b[j], y[j] - mu[j], c[j]));
    return r;
}

// How the rows of a GEMM operand are gathered from an NHWC activation.
//   G_CONV3: 3x3 / pad 1 taps on the row grid (tap t -> dy = t/3-1, dx = t%3-1),
//            out-of-image taps read as zero (post-BN zero padding, models/model.py:36).
//   G_IDENT: one tap, row = pixel.
//   G_UP2  : four taps (a,b) = (t>>1, t&1) reading pixel (2y+a, 2x+b) of a grid twice
//            the row grid (ConvTranspose2d k2 s2, models/model.py:19,49).
enum GatherMode { G_CONV3 = 0, G_IDENT = 1, G_UP2 = 2 };

static inline int gather_taps(int mode) { return mode == G_CONV3 ? 9 : (mode == G_UP2 ? 4 : 1); }

// Epilogues of the pixel-row GEMM.
//   E_STORE          : out[m][n] = acc            (dgrad)
//   E_BIAS_RELU_STATS: out[m][n] = relu(acc+b[n]) + per-block column sum / sum of squares
//                      for the following BatchNorm (models/model.py:36-38)
//   E_CONVT          : ConvTranspose2d scatter, n = (a*2+b)*cout + co ->
//                      out[(2y+a, 2x+b)][co] = acc + b[co]  (models/model.py:19)
//   E_STORE_BN       : out[m][n] = acc, and the result is the gradient `do` of a BatchNorm
//                      output: per-block column partials {sum do, sum do*y} for the BN
//                      backward (y = ey, the BN input).  With escale/eshift set (BN -> ReLU
//                      order, models/mod.py:46-47) do is first masked by the ReLU that
//                      follows the BN: do *= [escale*y + eshift > 0], stored masked.
//   E_STATS          : out[m][n] = acc + per-block column sum / sum of squares (a bias-free
//                      conv feeding BN directly, models/mod.py:45-46)
//   E_RESID          : out[m][n] = ReLU(acc + escale[n] * ey[m][n] + eshift[n]): the 1x1 skip
//                      conv of a residual block closing the block, ReLU(BN2(z2) + skip(x))
//                      (models/mod.py:86)
//   E_ADD            : out[m][n] += acc (the skip conv's input gradient already there)
enum EpiMode {
    E_STORE = 0, E_BIAS_RELU_STATS = 1, E_CONVT = 2, E_STORE_BN = 3, E_STATS = 4, E_RESID = 5,
    E_ADD = 6
};

// What the A (row GEMM) / B' (wgrad) loader applies to the gathered values:
//   OP_PLAIN : raw values
//   OP_AFFINE: per-channel BN affine scale*x + shift (forward consumers of a BN output)
//   OP_AFFINE_RELU: the same followed by ReLU on channels [0, arelu) (BN -> ReLU order,
//              models/mod.py:46-47; a concat [skip, up] has ReLU on the skip half only)
//   OP_DZ    : BN+ReLU backward on the fly, dz = [y > 0] (A*do + B*(y - mean) + C) per
//              channel, from do (the operand pointer), y (its BN input) and
//              coef = [A | B | C | mean]
enum LoadOp { OP_PLAIN = 0, OP_AFFINE = 1, OP_DZ = 2, OP_AFFINE_RELU = 3 };

struct RowGemmArgs {
    int H, W;        // row grid (rows = Nimg*H*W pixels)
    int M, N, K;     // GEMM sizes; K = taps * C
    const float* a;  // NHWC source of A rows
    int lda, aoff, C, amode;
    const float* ascale;  // per-channel affine applied to valid A values (BN fused in the
    const float* ashift;  // consumer's prologue); null = identity
    int arelu;            // OP_AFFINE_RELU: ReLU after the affine on channels [0, arelu)
    const float* bt;      // B^T, row-major [N][K] (f32 MFMA)
    const uint16_t* bt16; // or: B^T as bf16 (bf16 MFMA, f32 accumulate); exactly one is set
    float* out;
    int ldo, ooff;
    const float* bias;
    float* stats;  // [M/BM][2][N] partial (sum, sumsq) or, E_STORE_BN, (sum do, sum do*y)
    int cout;      // E_CONVT
    int emode;
    const float* ay;     // OP_DZ: BN input y of the A operand (ld, off)
    int lday, offay;
    const float* acoef;  // OP_DZ: [4][C] coefficients (A, B, Cc, mean: A do + B (y - mean) + Cc)
    const float* ey;     // E_STORE_BN: BN input y at the output position (ld, off)
    int ldey, offey;
    const float* escale;  // E_STORE_BN, BN -> ReLU order: affine of that BN (ReLU mask)
    const float* eshift;
    int xcd;              // remap blocks so each XCD gets a contiguous range of tiles
    const uint16_t* a16;  // rowgemm16: A as a dense bf16 image [pixels][lda] (prepared operand)
    const void* zero16;   // rowgemm16: >= 16 zero bytes (padding taps / rows past M)
    uint16_t* out16;      // E_CONVT: store bf16(result) into this image (ld ldo, offset ooff)
                          // instead of f32 into out (the bf16 consumer's operand image)
    uint16_t* out3;       // E_CONVT: store the x3 split of the result into this x3 image (ldo
                          // channels per row, channel offset ooff) instead of f32 into out
    int tgm;              // (r06) tile order: 0 / 1 M-major, > 1 groups of tgm M tiles
                          // (gemm_common.h tile_mn), -1 = the launcher's choice (tile_group_auto)
};

// (r06) group size of tile_mn for a grid of ntm x ntn tiles whose blocks hold `slots` block
// slots per XCD: the power of two that minimises the A + B rows one XCD's concurrently resident
// blocks touch (both operands stream K elements per row, so rows are the cost).  M-major when
// there are fewer than four N tiles (the weights fit the L2 anyway).
inline int tile_group_auto(int64_t M, int N, int BM, int BN, int slots) {
    const int64_t ntm = (M + BM - 1) / BM, ntn = N / BN;
    if (ntn < 4 || ntm < 2) return 1;
    const int64_t run = std::min<int64_t>(slots, (ntm * ntn + 7) / 8);
    int best = 1;
    int64_t bc = -1;
    for (int64_t gm = 1; gm <= ntm && gm <= run; gm *= 2) {
        const int64_t mspan = std::min<int64_t>(ntm, gm * ((run + gm * ntn - 1) / (gm * ntn)));
        const int64_t nspan = std::min<int64_t>(ntn, (run + gm - 1) / gm);
        const int64_t cost = mspan * BM + nspan * BN;
        if (bc < 0 || cost < bc) bc = cost, best = (int)gm;
    }
    return best;
}

struct WgradArgs {
    int H, W;   // pixel grid of the reduction rows (P = Nimg*H*W)
    int P;
    const float* a;  // A' rows: gather(a, amode, tapA) channels [ca0, ca0+BM)
    int lda, aoff, CA, amode;
    const float* ascale;
    const float* ashift;
    int arelu;       // ReLU after the affine on A' channels [0, arelu)
    const float* b;  // B' rows: gather(b, bmode, tapB) channels [cb0, cb0+BN)
    int ldb, boff, CB, bmode;
    int Mw, Nw;      // tapsA*CA, tapsB*CB
    int pps;         // pixels per split (multiple of the pixel chunk)
    int splits;
    float* slab;     // [splits][Mw][Nw]
    const float* by;     // OP_DZ on B': BN input y (ld, off) and coef [4][CB]
    int ldby, offby;
    const float* bcoef;
    float* bias_slab;    // optional [splits][Nw]: column sums of B' (the bias gradient)
    int bf16;            // bf16 MFMA (operands rounded to bf16 in LDS, f32 accumulate)
    const void* zero16;  // wgrad16: >= 16 zero bytes (padding taps / pixels past the split)
    int xcd;             // remap blocks so each XCD gets a contiguous range of tiles
    float* dzout;        // OP_DZ on B': the blocks of the first A' tile also store the dz
    int lddz;            // they formed ([P][lddz], channels cb0..), for the dgrad to read
    int bdznomask;       // OP_DZ on B', BN -> ReLU order (models/mod.py): dz is not masked by
                         // [y > 0] (the producer of do already applied the ReLU mask)
};

#define HIP_OK(x)                                   \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) return (int)e_;       \
    } while (0)

// host launchers (kernels_gemm.hip)
// row-GEMM tile ids: register-staged 0 = 128x128 (two LDS images), 1 = 128x64, 4 = 128x128,
// 6 = 128x128 64-K chunks (bf16), 13 = 128x32, 14 = 256x32; software-pipelined (kernels_gemm_pipe.hip)
// 18 = 128x128, 19 = 128x64 (loading two chunks ahead), 25 / 26 = 128x64 at three blocks per CU
// (one / two chunks ahead)
int launch_rowgemm(const RowGemmArgs& a, int tile, hipStream_t s);
int rowgemm_tile_dims(int tile, int* bm, int* bn, int* bk);
int rowgemm_tile_dbuf(int tile);
// software-pipelined f32 row GEMM (kernels_gemm_pipe.hip); tile 2 = 128x128, 3 = 128x64 (two
// chunks ahead), 4 / 5 = 128x64 at three blocks per CU
int rowgemm_pipe_ok(const RowGemmArgs& a);
int launch_rowgemm_pipe(const RowGemmArgs& a, int tile, hipStream_t s);
// wgrad tile ids (kernels_gemm.hip WGRAD_TILES): 0 = 128x128, 3 = 64x128 two waves,
// 5 = 128x64 four waves, 7 = 64x64 three waves / SIMD, 8 = 64x32, 9 = 32x32;
// 20.. = one row of 3x3 taps per block (3 accumulator sets; BM = channels of ONE tap):
// 20 = 64x64, 21 = 128x64, 22 = 64x128, 23 = 128x128
int launch_rowgemm16(const RowGemmArgs& a, int tile, hipStream_t s);
int rowgemm16_tile_dims(int tile, int* bm, int* bn, int* stages = nullptr);
int wgrad16g_tile_dims(int tile, int* bm, int* bn, int* stages = nullptr);
int launch_wgrad(const WgradArgs& a, int tile, hipStream_t s);
int launch_wgrad16(const WgradArgs& a, int tile, hipStream_t s);
int wgrad_tile_dims(int tile, int* bm, int* bn, int* bkp);
int wgrad_tile_taps(int tile);  // taps of the M dimension one block covers (3 for 20..)
// f32 GEMMs on bf16 MFMAs through exact three-way operand splits (kernels_gemm_x3.hip):
// x3 images bf16 [rows][C / 32][3][32] (hi, mid, lo planes per 32-channel group).  Row GEMM:
// a16 / bt16 are x3 images (lda channels per A row, aoff a channel offset); tiles 0 =
// 256x128, 1 = 128x128, 2 = 128x64, 3 = 256x64; tap-row halo tiles 4 = 256x128, 6 = 128x64.
// Weight gradient: a / b are x3 images; tiles 0 = 128x128, 1 = 64x64; tap-row tiles 2 = 64x128,
// 4 = 64x64.
int launch_rowgemm_x3(const RowGemmArgs& a, int tile, hipStream_t s);
int rowgemm_x3_tile_dims(int tile, int* bm, int* bn);
int launch_wgrad_x3(const WgradArgs& a, int tile, hipStream_t s);
int wgrad_x3_tile_dims(int tile, int* bm, int* bn);
// x3 image of op(src) (BN affine if scale, ReLU on channels < relu) into dst [P][dld] at
// channel offset doff
int k_to_x3(const float* src, int ld, int off, int C, const float* scale, const float* shift,
            int relu, int64_t P, uint16_t* dst, int dld, int doff, hipStream_t s);
// BN-backward dz (bn_dz4) as an x3 image; bpart (optional): [x3_dz_blocks(P)][C] column sums
// hdl != null (r05): `d` is not read; do = [hrelu: fma(y, hsc, hsh) > 0] hdl[m] hw[c] (the 1x1
// head's backward with one output channel, head_bwd's expression)
int k_bn_dz_x3(const float* d, const float* y, int ld, int off, int64_t P, int C, const float* coef,
               int mask, uint16_t* dz3, float* bpart, hipStream_t s, const float* hdl = nullptr,
               const float* hw = nullptr, const float* hsc = nullptr, const float* hsh = nullptr,
               int hrelu = 0);
// the same with do = [msc: fma(msc, y, msh) > 0] (dskip + [idx == window position] dp): the
// encoder block's second conv, maxpool_bwd's expression (r05; dskip offset applied, N H W the
// full-resolution grid, P = N H W < 2^24 for the f32-reciprocal pixel decode)
int k_bn_dz_x3_pool(const float* y, int ld, int off, int64_t P, int C, const float* coef, int mask,
                    uint16_t* dz3, float* bpart, const float* dp, const uint8_t* idx, const float* dskip,
                    int ldskip, const float* msc, const float* msh, int N, int H, int W, hipStream_t s);
int x3_dz_blocks(int64_t P);
// register-staged bf16 wgrad tile ids (a.bf16): 0 = 128x128/32 px, 2 = 64x64/64,
// 3 = 128x64/64, 4 = 64x128/64
int wgrad16_tile_dims(int tile, int* bm, int* bn, int* bkp);
