// Implicit-GEMM kernels for the UNet convolutions on gfx950, fp32 in / fp32 accumulate on
// the matrix cores (v_mfma_f32_32x32x2_f32: exact f32 fmaf chains at 64 FLOP/clk/SIMD).
//
// Two families cover every conv-shaped op of models/model.py:UNet:
//
//  rowgemm  C[m][n] = sum_k A[m][k] * Bt[n][k], rows m = output pixels (NHWC), k = (tap, c)
//           * Conv2d 3x3 pad 1 forward        (model.py:36,39)  A = gather G_CONV3 of the
//             BN-normalised input (affine applied in the load, zero padding kept zero),
//             Bt = weights packed [Cout][tap][Cin]; epilogue bias + ReLU (model.py:37,40)
//             + BatchNorm batch-stat partials.
//           * Conv2d 3x3 dgrad                 A = gather G_CONV3 of dZ, Bt = flipped weights
//             packed [Cin][tap'][Cout].
//           * ConvTranspose2d k2 s2 forward    (model.py:19,49) A = G_IDENT, Bt = [(a,b,co)][ci],
//             epilogue scatters the 2x2 output pixels into the concat buffer's channel slice
//             (torch.cat([up, skip]) of model.py:64-70 costs no copy).
//           * ConvTranspose2d dgrad            A = gather G_UP2 of dOut, Bt = [ci][(a,b,co)].
//  wgrad    C[m][n] = sum_p A'[p][m] * B'[p][n], reduction over pixels p, split over `splits`
//           slices into fp32 slabs (deterministic: the slab reducer adds them in order).
//
// Tiling: 256 threads = 4 waves (2x2), block tile BM x BN, wave tile (BM/2) x (BN/2) made of
// 32x32 MFMA accumulators.  Operands go HBM/L2 -> registers (issued one K-chunk ahead) ->
// LDS -> registers.  K-order inside an 8-wide chunk is permuted so each lane fetches its
// four k values with one ds_read_b128: lane half h owns k = 4h..4h+3 and MFMA step s sums
// k = s (h=0) and k = 4+s (h=1) -- A and B use the same permutation, so the product is the
// same sum in a different order.
#include <type_traits>

#include "gemm_common.h"

namespace {

// ------------------------------------------------------------------------------------
// Row GEMM.  Pipeline per K-chunk: issue the NEXT chunk's global loads into registers
// (raw: no arithmetic depends on them, so nothing waits for them here), run the MFMAs of
// the current chunk from LDS, then apply the BN affine / zero padding to the landed
// registers and write them to the other LDS image, one barrier.
// ------------------------------------------------------------------------------------
// Tile configuration of the row GEMM: block tile BM x BN, wave tile WM x WN (32x32 MFMA
// accumulators), K-chunk BK, DBUF = two LDS images (one barrier per chunk).
// OCC = waves per SIMD the register allocation must allow (launch_bounds' second argument).
// PRIO: raise the wave's issue priority (s_setprio 1) for its MFMA phase of each K-chunk
// and drop it for the commit phase, so a SIMD's matrix pipe is fed first when its co-
// resident waves (other blocks) are staging.
template <int BM_, int BN_, int WM_, int WN_, int BK_, bool DBUF_, int OCC_ = 1, bool PRIO_ = false>
struct RowTile {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = BK_;
    static constexpr bool DBUF = DBUF_;
    static constexpr int OCC = OCC_;
    static constexpr bool PRIO = PRIO_;
    static constexpr int WAVES = (BM / WM) * (BN / WN);
    static constexpr int THREADS = 64 * WAVES;
};

// BF: bf16 MFMA (v_mfma_f32_32x32x16_bf16, f32 accumulate).  A is still gathered as f32
// (activations stay f32 in HBM) and rounded to bf16 when it is written to LDS; Bt is a bf16
// weight image (p.bt16).  LDS rows are K-contiguous bf16 with an 8-element pad (80 B /
// 144 B row stride: the 16 lanes of a ds_read_b128 phase hit disjoint banks).
template <int AMODE, int AOP, int EMODE, class T, bool BF>
__global__ __launch_bounds__(T::THREADS, T::OCC) void rowgemm_kernel(RowGemmArgs p) {
    constexpr bool AFFINE = AOP == OP_AFFINE || AOP == OP_AFFINE_RELU, ADZ = AOP == OP_DZ;
    constexpr bool ARELU = AOP == OP_AFFINE_RELU;
    constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, BK = T::BK;
    constexpr bool DBUF = T::DBUF;
    constexpr int NTH = T::THREADS;
    constexpr int WAVES_N = BN / WN;
    constexpr int NBUF = DBUF ? 2 : 1;
    constexpr int LDK = BF ? BK + 8 : BK + 4;  // row stride in elements (bf16 or f32)
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int F4R = BK / 4;
    constexpr int RPP = NTH / F4R;
    constexpr int AP = BM / RPP, BP = BF ? 1 : BN / RPP;
    static_assert(AP * RPP == BM && (BF || BP * RPP == BN), "loader shape");
    constexpr int F8R = BK / 8, RPP8 = NTH / F8R;  // bf16 B image: 8 elements per lane
    constexpr int BP8 = BF ? BN / RPP8 : 1;
    static_assert(!BF || BP8 * RPP8 == BN, "bf16 B loader shape");
    constexpr int IMG = (BM + BN) * LDK;  // elements per LDS image
    constexpr int SMEM_F = BF ? (NBUF * IMG + 1) / 2 : NBUF * IMG;
    __shared__ __attribute__((aligned(16))) float smem[SMEM_F];
    static_assert(SMEM_F * 4 >= (BM / 64) * 2 * BN * 8, "epilogue scratch (row_epilogue)");

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tile_m = bid / ntn, tile_n = bid - tile_m * ntn;
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    const int H = p.H, W = p.W;

    const int lrow = tid / F4R, lc4 = tid % F4R;
    Pix rq[AP];
    int rm[AP];
    bool rok[AP];  // row inside M (the last M tile may be partial)
#pragma unroll
    for (int i = 0; i < AP; ++i) {
        const int m = m0 + lrow + i * RPP;
        rok[i] = m < p.M;
        rm[i] = rok[i] ? m : p.M - 1;
        rq[i] = decode(rm[i], H, W);
    }

    f32x4 ra[AP], rb[BP], rsc, rsh, rcc, rmu;
    uint4 rb8[BP8];
    f32x4 ry[ADZ ? AP : 1];
    unsigned vmask = 0;
    bool rrelu = false;
    const int brow8 = tid / F8R, bc8 = tid % F8R;

    auto issue = [&](int kc) {
        const int k0 = kc * BK;
        const int tap = k0 / p.C;
        const int c = k0 - tap * p.C + lc4 * 4;
        if constexpr (AFFINE) {
            rsc = *(const f32x4*)(p.ascale + c);
            rsh = *(const f32x4*)(p.ashift + c);
            if constexpr (ARELU) rrelu = c < p.arelu;
        }
        if constexpr (ADZ) {
            rsc = *(const f32x4*)(p.acoef + c);
            rsh = *(const f32x4*)(p.acoef + p.C + c);
            rcc = *(const f32x4*)(p.acoef + 2 * p.C + c);
            rmu = *(const f32x4*)(p.acoef + 3 * p.C + c);
        }
        vmask = 0;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            bool valid;
            const int src = gather_src<AMODE>(tap, rm[i], rq[i], H, W, valid);
            vmask |= (valid && rok[i]) ? (1u << i) : 0u;
            ra[i] = *(const f32x4*)(p.a + (size_t)src * p.lda + p.aoff + c);
            if constexpr (ADZ) ry[i] = *(const f32x4*)(p.ay + (size_t)src * p.lday + p.offay + c);
        }
        if constexpr (BF) {
#pragma unroll
            for (int i = 0; i < BP8; ++i)
                rb8[i] = *(const uint4*)(p.bt16 + (size_t)(n0 + brow8 + i * RPP8) * p.K + k0 + bc8 * 8);
        } else {
#pragma unroll
            for (int i = 0; i < BP; ++i)
                rb[i] = *(const f32x4*)(p.bt + (size_t)(n0 + lrow + i * RPP) * p.K + k0 + lc4 * 4);
        }
    };
    auto commit = [&](int buf) {
        float* as = smem + buf * IMG;
        float* bs = as + BM * LDK;
        __bf16* as16 = (__bf16*)smem + buf * IMG;
        __bf16* bs16 = as16 + BM * LDK;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            f32x4 v = ra[i];
            if constexpr (AFFINE) {
                v = v * rsc + rsh;
                if (ARELU && rrelu)
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
            }
            if constexpr (ADZ) {
                const f32x4 d = bn_dz4(rsc, v, rsh, ry[i], rmu, rcc);
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = ry[i][j] > 0.f ? d[j] : 0.f;
            }
            if (!((vmask >> i) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (BF)
                *(bf16x4*)&as16[(lrow + i * RPP) * LDK + lc4 * 4] = to_bf16x4(v);
            else
                *(f32x4*)&as[(lrow + i * RPP) * LDK + lc4 * 4] = v;
        }
        if constexpr (BF) {
#pragma unroll
            for (int i = 0; i < BP8; ++i) *(uint4*)&bs16[(brow8 + i * RPP8) * LDK + bc8 * 8] = rb8[i];
        } else {
#pragma unroll
            for (int i = 0; i < BP; ++i) *(f32x4*)&bs[(lrow + i * RPP) * LDK + lc4 * 4] = rb[i];
        }
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int li = lane & 31, lh = lane >> 5;
    const int nk = p.K / BK;
    issue(0);
    commit(0);
    __syncthreads();
    for (int kc = 0; kc < nk; ++kc) {
        const int cur = DBUF ? (kc & 1) : 0;
        if (kc + 1 < nk) issue(kc + 1);
        if constexpr (T::PRIO) __builtin_amdgcn_s_setprio(1);
        if constexpr (BF) {
            const __bf16* as16 = (const __bf16*)smem + cur * IMG;
            const __bf16* bs16 = as16 + BM * LDK;
#pragma unroll
            for (int kk = 0; kk < BK / 16; ++kk) {
                bf16x8 af[MT], bf[NT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    af[mt] = *(const bf16x8*)&as16[(wm * WM + mt * 32 + li) * LDK + kk * 16 + lh * 8];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    bf[nt] = *(const bf16x8*)&bs16[(wn * WN + nt * 32 + li) * LDK + kk * 16 + lh * 8];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[mt][nt] = mfma32_bf16(af[mt], bf[nt], acc[mt][nt]);
            }
        } else {
            const float* as = smem + cur * IMG;
            const float* bs = as + BM * LDK;
#pragma unroll
            for (int kk = 0; kk < BK / 8; ++kk) {
                f32x4 af[MT], bf[NT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    af[mt] = *(const f32x4*)&as[(wm * WM + mt * 32 + li) * LDK + kk * 8 + lh * 4];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    bf[nt] = *(const f32x4*)&bs[(wn * WN + nt * 32 + li) * LDK + kk * 8 + lh * 4];
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
                            acc[mt][nt] = mfma32(af[mt][s], bf[nt][s], acc[mt][nt]);
            }
        }
        if constexpr (T::PRIO) __builtin_amdgcn_s_setprio(0);
        if constexpr (DBUF) {
            // the other image was last read in iteration kc-1, which every wave finished
            // before the barrier that ended it
            if (kc + 1 < nk) commit(cur ^ 1);
            __syncthreads();
        } else {
            __syncthreads();
            if (kc + 1 < nk) {
                commit(0);
                __syncthreads();
            }
        }
    }

    row_epilogue<EMODE, BM, BN, WM, WN>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, smem);
}

// ------------------------------------------------------------------------------------
// Skinny row GEMM (N = 32 outputs: the narrow networks' level 0; tile 15).  With one wave per 64-row band holding the whole
// N, every A row feeds exactly one wave, so staging A through LDS (tile 14) bought no reuse
// and held the CU to one 83-KB block of four waves.  Here every MFMA operand comes from
// global memory straight into registers, in the layout the LDS-staged tiles read (lane half h
// owns k = 4h..4h+3 of each 8-k group: one dwordx4 of A per accumulator row band and one of
// Bt per 32 columns, which every wave of the CU shares through L1), one chunk of GK 8-k
// groups loaded ahead of the MFMAs.  No LDS in the main loop and no barriers: the four waves
// of a block run independently, several blocks per CU.  Same K order, same MFMA sequence per
// element and the same epilogue as the LDS-staged tiles: bit-identical results.
// ------------------------------------------------------------------------------------
template <int AMODE, int AOP, int EMODE, int NT, int GK, int OCC>
__global__ __launch_bounds__(256, OCC) void rowgemm_direct_kernel(RowGemmArgs p) {
    constexpr bool AFFINE = AOP == OP_AFFINE || AOP == OP_AFFINE_RELU;
    constexpr bool ARELU = AOP == OP_AFFINE_RELU;
    static_assert(AOP != OP_DZ, "plain / affine A operands only");
    static_assert(GK == 1 || GK == 2 || GK == 4, "a chunk is 8, 16 or 32 k of one tap");
    constexpr int BM = 256, BN = 32 * NT, WM = 64, WN = BN, MT = 2, KC = 8 * GK;
    constexpr int CMAX = 256;  // affine operands: per-channel scale / shift staged in LDS
    __shared__ __attribute__((aligned(16))) float smem[(BM / 64) * 2 * BN * 2];  // epilogue
    __shared__ __attribute__((aligned(16))) float aff[AFFINE ? 2 * CMAX : 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if constexpr (AFFINE) {
        for (int i = tid; i < p.C; i += 256) {
            aff[i] = p.ascale[i];
            aff[CMAX + i] = p.ashift[i];
        }
        __syncthreads();
    }
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tile_m = bid / ntn, tile_n = bid - tile_m * ntn;
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    const int H = p.H, W = p.W, C = p.C;
    const int li = lane & 31, lh = lane >> 5;

    Pix rq[MT];
    int rm[MT];
    bool rok[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = m0 + wave * WM + mt * 32 + li;
        rok[mt] = m < p.M;
        rm[mt] = rok[mt] ? m : p.M - 1;
        rq[mt] = decode(rm[mt], H, W);
    }
    const float* brow = p.bt + (size_t)(n0 + li) * p.K + 4 * lh;

    // chunk kc = KC k of one tap: A[mt][g], Bt[nt][g] for its GK 8-k groups
    struct Chunk {
        f32x4 a[MT][GK], b[NT][GK];
        int c0;  // the lane's first channel (affine lookup)
        unsigned vmask;
        bool relu;
    };
    auto load = [&](int kc, Chunk& ch) {
        const int k0 = kc * KC;
        const int tap = k0 / C;
        const int c0 = k0 - tap * C + 4 * lh;
        ch.vmask = 0;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            bool valid;
            const int src = gather_src<AMODE>(tap, rm[mt], rq[mt], H, W, valid);
            ch.vmask |= (valid && rok[mt]) ? (1u << mt) : 0u;
            const float* ar = p.a + (size_t)src * p.lda + p.aoff + c0;
#pragma unroll
            for (int g = 0; g < GK; ++g) ch.a[mt][g] = *(const f32x4*)(ar + 8 * g);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int g = 0; g < GK; ++g)
                ch.b[nt][g] = *(const f32x4*)(brow + (size_t)nt * 32 * p.K + k0 + 8 * g);
        ch.c0 = c0;
        // (the ReLU span is a multiple of 32 channels: a chunk lies in one half of a concat)
        if constexpr (ARELU) ch.relu = c0 - 4 * lh < p.arelu;
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

    auto compute = [&](const Chunk& ch) {
#pragma unroll
        for (int g = 0; g < GK; ++g) {
            f32x4 av[MT], sc = {}, sh = {};
            if constexpr (AFFINE) {
                sc = *(const f32x4*)&aff[ch.c0 + 8 * g];
                sh = *(const f32x4*)&aff[CMAX + ch.c0 + 8 * g];
            }
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                f32x4 v = ch.a[mt][g];
                if constexpr (AFFINE) {
                    v = v * sc + sh;
                    if (ARELU && ch.relu)
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
                }
                if (!((ch.vmask >> mt) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
                av[mt] = v;
            }
            // the LDS-staged tiles' order per accumulator: k-steps st = 0..3 of each group
#pragma unroll
            for (int st = 0; st < 4; ++st)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[mt][nt] = mfma32(av[mt][st], ch.b[nt][g][st], acc[mt][nt]);
        }
    };
    // two register sets, one chunk ahead (unrolled by two: no set copies)
    const int nk = p.K / KC;
    Chunk c0, c1;
    load(0, c0);
    for (int kc = 0; kc < nk; kc += 2) {
        if (kc + 1 < nk) load(kc + 1, c1);
        compute(c0);
        if (kc + 1 >= nk) break;
        if (kc + 2 < nk) load(kc + 2, c0);
        compute(c1);
    }
    // PRELOAD: the short-K (64 .. 576) GEMMs of this tile are epilogue-heavy; the reading
    // epilogues (BN partials, residual close / add) issue each accumulator's 16 loads first
    row_epilogue<EMODE, BM, BN, WM, WN, true>(p, acc, m0, n0, tile_m, wave, 0, lane, tid, smem);
}


// ------------------------------------------------------------------------------------
// Weight-gradient GEMM (reduction over pixels), same issue / compute / commit pipeline.
// ------------------------------------------------------------------------------------
// wgrad tile: block BM x BN, wave tile WM x WN, pixels per chunk BKP.
template <int BM_, int BN_, int WM_, int WN_, int BKP_, int OCC_ = 1>
struct WgTile {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BKP = BKP_;
    static constexpr int THREADS = 64 * (BM / WM) * (BN / WN);
    static constexpr int OCC = OCC_;
};

template <int AMODE, int AOP, int BMODE, bool BDZ, class T>
__global__ __launch_bounds__(T::THREADS, T::OCC) void wgrad_kernel(WgradArgs p) {
    constexpr bool AFFINE = AOP == OP_AFFINE || AOP == OP_AFFINE_RELU;
    constexpr bool ARELU = AOP == OP_AFFINE_RELU;
    constexpr int BM = T::BM, BN = T::BN, BKP = T::BKP, WM = T::WM, WN = T::WN;
    constexpr int NTH = T::THREADS;
    constexpr int WAVES_N = BN / WN;
    constexpr int LDA = BM + 4, LDB = BN + 4;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int AF = BM / 4, BF = BN / 4;          // float4 per pixel row
    constexpr int ARPP = NTH / AF, BRPP = NTH / BF;  // rows per pass
    constexpr int AP = BKP / ARPP, BP = BKP / BRPP;
    static_assert(AP * ARPP == BKP && BP * BRPP == BKP, "loader shape");
    __shared__ __attribute__((aligned(16))) float As[BKP * LDA];
    __shared__ __attribute__((aligned(16))) float Bs[BKP * LDB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int tiles_n = p.Nw / BN, tiles_m = p.Mw / BM;
    int idx = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tn = idx % tiles_n;
    idx /= tiles_n;
    const int tm = idx % tiles_m;
    const int split = idx / tiles_m;
    const int tapA = (tm * BM) / p.CA, ca0 = tm * BM - tapA * p.CA;
    const int tapB = (tn * BN) / p.CB, cb0 = tn * BN - tapB * p.CB;
    const int H = p.H, W = p.W;
    const float rH = 1.f / (float)H, rW = 1.f / (float)W;

    const int ac4 = tid % AF, arow = tid / AF;
    const int bc4 = tid % BF, brow = tid / BF;
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
    bool arl = false;
    if constexpr (AFFINE) {
        sc = *(const f32x4*)(p.ascale + ca0 + ac4 * 4);
        sh = *(const f32x4*)(p.ashift + ca0 + ac4 * 4);
        if constexpr (ARELU) arl = ca0 + ac4 * 4 < p.arelu;
    }

    f32x4 ca = {0, 0, 0, 0}, cb = ca, cc = ca, cm = ca;  // OP_DZ coefficients of this thread's columns
    if constexpr (BDZ) {
        ca = *(const f32x4*)(p.bcoef + cb0 + bc4 * 4);
        cb = *(const f32x4*)(p.bcoef + p.CB + cb0 + bc4 * 4);
        cc = *(const f32x4*)(p.bcoef + 2 * p.CB + cb0 + bc4 * 4);
        cm = *(const f32x4*)(p.bcoef + 3 * p.CB + cb0 + bc4 * 4);
    }
    const bool bsum = p.bias_slab != nullptr && tm == 0;
    double bacc[4] = {0.0, 0.0, 0.0, 0.0};  // f64: the bias gradient is a small sum of +/- terms

    const int pbeg = split * p.pps;
    int pend = pbeg + p.pps;
    if (pend > p.P) pend = p.P;
    const int nchunks = (pend - pbeg + BKP - 1) / BKP;

    f32x4 ryb[BDZ ? BP : 1];
    int bm_row[BDZ ? BP : 1];
    const bool dzw = BDZ && p.dzout != nullptr && tm == 0 && BMODE == G_IDENT;
    f32x4 ra[AP], rb[BP];
    unsigned amask = 0, bmask = 0;
    auto issue = [&](int pc) {
        amask = bmask = 0;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            int m = pc + arow + i * ARPP;
            const bool in = m < pend;
            m = in ? m : pend - 1;
            bool valid;
            const Pix q = AMODE == G_IDENT ? Pix{0, 0, 0} : decode_fast(m, H, W, rH, rW);
            const int src = gather_src<AMODE>(tapA, m, q, H, W, valid);
            amask |= (valid && in) ? (1u << i) : 0u;
            ra[i] = *(const f32x4*)(p.a + (size_t)src * p.lda + p.aoff + ca0 + ac4 * 4);
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            int m = pc + brow + i * BRPP;
            const bool in = m < pend;
            m = in ? m : pend - 1;
            bool valid;
            const Pix q = BMODE == G_IDENT ? Pix{0, 0, 0} : decode_fast(m, H, W, rH, rW);
            const int src = gather_src<BMODE>(tapB, m, q, H, W, valid);
            bmask |= (valid && in) ? (1u << i) : 0u;
            rb[i] = *(const f32x4*)(p.b + (size_t)src * p.ldb + p.boff + cb0 + bc4 * 4);
            if constexpr (BDZ) {
                ryb[i] = *(const f32x4*)(p.by + (size_t)src * p.ldby + p.offby + cb0 + bc4 * 4);
                bm_row[i] = src;
            }
        }
    };
    auto commit = [&]() {
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            f32x4 v = ra[i];
            if constexpr (AFFINE) {
                v = v * sc + sh;
                if (ARELU && arl)
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
            }
            if (!((amask >> i) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
            *(f32x4*)&As[(arow + i * ARPP) * LDA + ac4 * 4] = v;
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            f32x4 v = rb[i];
            if constexpr (BDZ) {
                const f32x4 d = bn_dz4(ca, v, cb, ryb[i], cm, cc);
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (p.bdznomask || ryb[i][j] > 0.f) ? d[j] : 0.f;
                // the first A' tile's blocks (tap 0, channels 0..BM) hand dz to the dgrad
                if (dzw && ((bmask >> i) & 1u))
                    *(f32x4*)(p.dzout + (size_t)bm_row[i] * p.lddz + cb0 + bc4 * 4) = v;
            }
            if (!((bmask >> i) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (bsum)
#pragma unroll
                for (int j = 0; j < 4; ++j) bacc[j] += v[j];
            *(f32x4*)&Bs[(brow + i * BRPP) * LDB + bc4 * 4] = v;
        }
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int li = lane & 31, lh = lane >> 5;
    if (nchunks > 0) {
        issue(pbeg);
        commit();
        __syncthreads();
    }
    for (int c = 0; c < nchunks; ++c) {
        if (c + 1 < nchunks) issue(pbeg + (c + 1) * BKP);
#pragma unroll
        for (int kk = 0; kk < BKP / 8; ++kk)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int pr = kk * 8 + lh * 4 + s;
                float af[MT], bf[NT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) af[mt] = As[pr * LDA + wm * WM + mt * 32 + li];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) bf[nt] = Bs[pr * LDB + wn * WN + nt * 32 + li];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32(af[mt], bf[nt], acc[mt][nt]);
            }
        __syncthreads();
        if (c + 1 < nchunks) {
            commit();
            __syncthreads();
        }
    }

    if (bsum) {  // column sums of B' for the bias gradient: combine the row groups in order
        __syncthreads();
        double* red = (double*)As;  // [NTH][4]; As holds >= BKP*LDA floats >= 8*NTH
#pragma unroll
        for (int j = 0; j < 4; ++j) red[tid * 4 + j] = bacc[j];
        __syncthreads();
        if (tid < BF) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double t = 0.0;
                for (int g = 0; g < BRPP; ++g) t += red[(g * BF + tid) * 4 + j];
                p.bias_slab[(size_t)split * p.Nw + tn * BN + tid * 4 + j] = (float)t;
            }
        }
    }

    float* slab = p.slab + (size_t)split * p.Mw * p.Nw;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = tm * BM + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int n = tn * BN + wn * WN + nt * 32 + li;
                slab[(size_t)m * p.Nw + n] = acc[mt][nt][r];
            }
}

// ------------------------------------------------------------------------------------
// Weight gradient of a 3x3 conv, one ROW of taps per block (dy fixed, dx = 0..2).
// dW[(dy,dx)][ci][co] = sum_p x[p + (dy-1, dx-1)][ci] * dz[p][co]: for a chunk of BKP
// pixels of one image row (W % BKP == 0, so a chunk never crosses a row) the three dx
// taps read the same input row shifted by one pixel.  The block stages that row ONCE
// with a one-pixel halo on each side (BKP + 2 LDS rows, zero outside the image), stages
// the dz chunk once, and feeds three accumulator sets from it: A' of tap dx at chunk
// pixel k is LDS row k + dx.  Against the one-tap tiles this reads each dz chunk 3x
// instead of 9x per layer and does a third of the staging per MFMA.  Same K order,
// split-K slabs, bias column sums and loaders (OP_AFFINE / OP_AFFINE_RELU on x, OP_DZ on
// dz) as wgrad_kernel; slab rows m = (3*dy + dx)*CA + ci, the one-tap layout.
// ------------------------------------------------------------------------------------
template <int AOP, bool BDZ, class T>
__global__ __launch_bounds__(T::THREADS, T::OCC) void wgrad_row3_kernel(WgradArgs p) {
    constexpr bool AFFINE = AOP == OP_AFFINE || AOP == OP_AFFINE_RELU;
    constexpr bool ARELU = AOP == OP_AFFINE_RELU;
    constexpr int BM = T::BM, BN = T::BN, BKP = T::BKP, WM = T::WM, WN = T::WN;
    constexpr int NTH = T::THREADS;
    constexpr int WAVES_N = BN / WN;
    constexpr int LDA = BM + 4, LDB = BN + 4;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int AF = BM / 4, BF = BN / 4;          // float4 per pixel row
    constexpr int ARPP = NTH / AF, BRPP = NTH / BF;  // rows per pass
    constexpr int HROWS = BKP + 2;                   // chunk + halo
    constexpr int AROWS = HROWS;
    constexpr int AP = (AROWS + ARPP - 1) / ARPP, BP = BKP / BRPP;
    static_assert(ARPP * AF == NTH && BP * BRPP == BKP, "loader shape");
    __shared__ __attribute__((aligned(16))) float As[AROWS * LDA];
    __shared__ __attribute__((aligned(16))) float Bs[BKP * LDB];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ctm = p.CA / BM;                       // channel tiles per tap row
    const int tiles_n = p.Nw / BN, tiles_m = 3 * ctm;
    int idx = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tn = idx % tiles_n;
    idx /= tiles_n;
    const int tm = idx % tiles_m;
    const int split = idx / tiles_m;
    const int dy = tm / ctm, ca0 = (tm - dy * ctm) * BM;  // tap row
    const int tapB = (tn * BN) / p.CB, cb0 = tn * BN - tapB * p.CB;
    const int H = p.H, W = p.W;

    const int ac4 = tid % AF, arow = tid / AF;
    const int bc4 = tid % BF, brow = tid / BF;
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
    bool arl = false;
    if constexpr (AFFINE) {
        sc = *(const f32x4*)(p.ascale + ca0 + ac4 * 4);
        sh = *(const f32x4*)(p.ashift + ca0 + ac4 * 4);
        if constexpr (ARELU) arl = ca0 + ac4 * 4 < p.arelu;
    }
    f32x4 ca = {0, 0, 0, 0}, cb = ca, cc = ca, cm = ca;
    if constexpr (BDZ) {
        ca = *(const f32x4*)(p.bcoef + cb0 + bc4 * 4);
        cb = *(const f32x4*)(p.bcoef + p.CB + cb0 + bc4 * 4);
        cc = *(const f32x4*)(p.bcoef + 2 * p.CB + cb0 + bc4 * 4);
        cm = *(const f32x4*)(p.bcoef + 3 * p.CB + cb0 + bc4 * 4);
    }
    const bool bsum = p.bias_slab != nullptr && tm == 0;
    double bacc[4] = {0.0, 0.0, 0.0, 0.0};

    const int pbeg = split * p.pps;
    int pend = pbeg + p.pps;
    if (pend > p.P) pend = p.P;
    const int nchunks = (pend - pbeg + BKP - 1) / BKP;

    f32x4 ryb[BDZ ? BP : 1];
    int bm_row[BDZ ? BP : 1];
    const bool dzw = BDZ && p.dzout != nullptr && tm == 0;
    f32x4 ra[AP], rb[BP];
    unsigned amask = 0, bmask = 0;
    auto issue = [&](int pc) {
        amask = bmask = 0;
        const Pix q = decode(pc, H, W);  // chunk start; the chunk stays on this row
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const int r0 = arow + i * ARPP, r = r0;
            const int yy = q.y + dy - 1;
            const bool rowok = (yy >= 0) & (yy < H);
            const int rbase = (q.img * H + (rowok ? yy : q.y)) * W;
            const int xx = q.x + r - 1;
            const bool valid = rowok & (r0 < AROWS) & (xx >= 0) & (xx < W);
            amask |= valid ? (1u << i) : 0u;
            const int src = valid ? rbase + xx : pc;
            ra[i] = *(const f32x4*)(p.a + (size_t)src * p.lda + p.aoff + ca0 + ac4 * 4);
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            int m = pc + brow + i * BRPP;
            const bool in = m < pend;
            m = in ? m : pend - 1;
            bmask |= in ? (1u << i) : 0u;
            rb[i] = *(const f32x4*)(p.b + (size_t)m * p.ldb + p.boff + cb0 + bc4 * 4);
            if constexpr (BDZ) {
                ryb[i] = *(const f32x4*)(p.by + (size_t)m * p.ldby + p.offby + cb0 + bc4 * 4);
                bm_row[i] = m;
            }
        }
    };
    auto commit = [&]() {
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const int r = arow + i * ARPP;
            if (AP * ARPP > AROWS && r >= AROWS) break;
            f32x4 v = ra[i];
            if constexpr (AFFINE) {
                v = v * sc + sh;
                if (ARELU && arl)
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
            }
            if (!((amask >> i) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
            *(f32x4*)&As[r * LDA + ac4 * 4] = v;
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            f32x4 v = rb[i];
            if constexpr (BDZ) {
                const f32x4 d = bn_dz4(ca, v, cb, ryb[i], cm, cc);
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = (p.bdznomask || ryb[i][j] > 0.f) ? d[j] : 0.f;
                // the first A' tile's blocks (tap row 0, channels 0..BM) hand dz to the dgrad
                if (dzw && ((bmask >> i) & 1u))
                    *(f32x4*)(p.dzout + (size_t)bm_row[i] * p.lddz + cb0 + bc4 * 4) = v;
            }
            if (!((bmask >> i) & 1u)) v = f32x4{0.f, 0.f, 0.f, 0.f};
            if (bsum)
#pragma unroll
                for (int j = 0; j < 4; ++j) bacc[j] += v[j];
            *(f32x4*)&Bs[(brow + i * BRPP) * LDB + bc4 * 4] = v;
        }
    };

    constexpr int NTAP = 3;
    f32x16 acc[NTAP][MT][NT];
#pragma unroll
    for (int d = 0; d < NTAP; ++d)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[d][i][j][r] = 0.f;

    const int li = lane & 31, lh = lane >> 5;
    if (nchunks > 0) {
        issue(pbeg);
        commit();
        __syncthreads();
    }
    for (int c = 0; c < nchunks; ++c) {
        if (c + 1 < nchunks) issue(pbeg + (c + 1) * BKP);
#pragma unroll
        for (int kk = 0; kk < BKP / 8; ++kk)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int pr = kk * 8 + lh * 4 + s;
                float bf[NT];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) bf[nt] = Bs[pr * LDB + wn * WN + nt * 32 + li];
#pragma unroll
                for (int d = 0; d < NTAP; ++d) {
                    // tap dx = d reads halo row pr + dx
                    const int ar = pr + d;
                    float af[MT];
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) af[mt] = As[ar * LDA + wm * WM + mt * 32 + li];
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
                            acc[d][mt][nt] = mfma32(af[mt], bf[nt], acc[d][mt][nt]);
                }
            }
        __syncthreads();
        if (c + 1 < nchunks) {
            commit();
            __syncthreads();
        }
    }

    if (bsum) {  // column sums of B' for the bias gradient: combine the row groups in order
        __syncthreads();
        double* red = (double*)As;  // [NTH][4]
        static_assert(AROWS * LDA >= 8 * NTH, "bias reduction scratch");
#pragma unroll
        for (int j = 0; j < 4; ++j) red[tid * 4 + j] = bacc[j];
        __syncthreads();
        if (tid < BF) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double t = 0.0;
                for (int g = 0; g < BRPP; ++g) t += red[(g * BF + tid) * 4 + j];
                p.bias_slab[(size_t)split * p.Nw + tn * BN + tid * 4 + j] = (float)t;
            }
        }
    }

    float* slab = p.slab + (size_t)split * p.Mw * p.Nw;
#pragma unroll
    for (int d = 0; d < NTAP; ++d)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = (3 * dy + d) * p.CA + ca0 + wm * WM + mt * 32 + (r & 3) +
                                  8 * (r >> 2) + 4 * lh;
                    const int n = tn * BN + wn * WN + nt * 32 + li;
                    slab[(size_t)m * p.Nw + n] = acc[d][mt][nt][r];
                }
}

// ------------------------------------------------------------------------------------
// Weight-gradient GEMM with a channel-major LDS image ("transposed" loader).  The MFMA
// operands of the pixel reduction are consecutive PIXELS of one channel per lane, so the
// loader works on 4-pixel x 4-channel units: four f32x4 loads (one per pixel), the BN
// affine / ReLU / padding applied in f32, then a register transpose into four 16-B
// (f32) or 8-B (bf16) rows of channel-major, pixel-contiguous LDS images ([BM][BKP+pad]
// and [BN][BKP+pad]).  f32 (BF = false): each lane then reads its 4 pixels of a k-group
// with one ds_read_b128 and feeds 4 v_mfma_f32_32x32x2_f32 (the row GEMM's K permutation,
// applied to both operands); bf16 (BF = true): 8 pixels, one v_mfma_f32_32x32x16_bf16.
// Bias column sums of B' are taken from the f32 values.
// ------------------------------------------------------------------------------------
template <int AMODE, int AOP, int BMODE, class T, bool BF>
__global__ __launch_bounds__(T::THREADS, T::OCC) void wgradT_kernel(WgradArgs p) {
    constexpr bool AFFINE = AOP == OP_AFFINE || AOP == OP_AFFINE_RELU;
    constexpr bool ARELU = AOP == OP_AFFINE_RELU;
    constexpr int BM = T::BM, BN = T::BN, BKP = T::BKP, WM = T::WM, WN = T::WN;
    constexpr int NTH = T::THREADS;
    constexpr int WAVES_N = BN / WN;
    constexpr int LDP = BF ? BKP + 8 : BKP + 4;       // LDS row (pixels) in elements
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int AQ = BM / 4, BQ = BN / 4;           // channel quads
    constexpr int APQ = NTH / AQ, BPQ = NTH / BQ;     // pixel quads per pass
    constexpr int AP = (BKP / 4) / APQ, BP = (BKP / 4) / BPQ;
    static_assert(AP * APQ == BKP / 4 && BP * BPQ == BKP / 4 && AP >= 1 && BP >= 1, "loader");
    using E = typename std::conditional<BF, __bf16, float>::type;
    constexpr int IMG_F = BF ? ((BM + BN) * LDP + 1) / 2 : (BM + BN) * LDP;
    constexpr int SMEM_F = IMG_F > 8 * NTH ? IMG_F : 8 * NTH;
    __shared__ __attribute__((aligned(16))) float smem[SMEM_F];
    E* As = (E*)smem;
    E* Bs = As + BM * LDP;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int tiles_n = p.Nw / BN, tiles_m = p.Mw / BM;
    int idx = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tn = idx % tiles_n;
    idx /= tiles_n;
    const int tm = idx % tiles_m;
    const int split = idx / tiles_m;
    const int tapA = (tm * BM) / p.CA, ca0 = tm * BM - tapA * p.CA;
    const int tapB = (tn * BN) / p.CB, cb0 = tn * BN - tapB * p.CB;
    const int H = p.H, W = p.W;
    const float rH = 1.f / (float)H, rW = 1.f / (float)W;

    const int aq = tid % AQ, apq = tid / AQ;
    const int bq = tid % BQ, bpq = tid / BQ;
    f32x4 sc = {1.f, 1.f, 1.f, 1.f}, sh = {0.f, 0.f, 0.f, 0.f};
    bool arl = false;
    if constexpr (AFFINE) {
        sc = *(const f32x4*)(p.ascale + ca0 + aq * 4);
        sh = *(const f32x4*)(p.ashift + ca0 + aq * 4);
        if constexpr (ARELU) arl = ca0 + aq * 4 < p.arelu;
    }
    const bool bsum = p.bias_slab != nullptr && tm == 0;
    double bacc[4] = {0.0, 0.0, 0.0, 0.0};

    const int pbeg = split * p.pps;
    int pend = pbeg + p.pps;
    if (pend > p.P) pend = p.P;
    const int nchunks = (pend - pbeg + BKP - 1) / BKP;

    f32x4 ra[AP][4], rb[BP][4];
    unsigned amask = 0, bmask = 0;
    auto issue = [&](int pc) {
        amask = bmask = 0;
#pragma unroll
        for (int i = 0; i < AP; ++i)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int m = pc + 4 * (apq + i * APQ) + u;
                const bool in = m < pend;
                m = in ? m : pend - 1;
                bool valid;
                const Pix q = AMODE == G_IDENT ? Pix{0, 0, 0} : decode_fast(m, H, W, rH, rW);
                const int src = gather_src<AMODE>(tapA, m, q, H, W, valid);
                amask |= (valid && in) ? (1u << (4 * i + u)) : 0u;
                ra[i][u] = *(const f32x4*)(p.a + (size_t)src * p.lda + p.aoff + ca0 + aq * 4);
            }
#pragma unroll
        for (int i = 0; i < BP; ++i)
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                int m = pc + 4 * (bpq + i * BPQ) + u;
                const bool in = m < pend;
                m = in ? m : pend - 1;
                bool valid;
                const Pix q = BMODE == G_IDENT ? Pix{0, 0, 0} : decode_fast(m, H, W, rH, rW);
                const int src = gather_src<BMODE>(tapB, m, q, H, W, valid);
                bmask |= (valid && in) ? (1u << (4 * i + u)) : 0u;
                rb[i][u] = *(const f32x4*)(p.b + (size_t)src * p.ldb + p.boff + cb0 + bq * 4);
            }
    };
    auto commit = [&]() {
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            f32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                v[u] = ra[i][u];
                if constexpr (AFFINE) {
                    v[u] = v[u] * sc + sh;
                    if (ARELU && arl)
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[u][j] = fmaxf(v[u][j], 0.f);
                }
                if (!((amask >> (4 * i + u)) & 1u)) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            const int pp = 4 * (apq + i * APQ);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if constexpr (BF)
                    *(bf16x4*)&As[(aq * 4 + j) * LDP + pp] =
                        bf16x4{(__bf16)v[0][j], (__bf16)v[1][j], (__bf16)v[2][j], (__bf16)v[3][j]};
                else
                    *(f32x4*)&As[(aq * 4 + j) * LDP + pp] = f32x4{v[0][j], v[1][j], v[2][j], v[3][j]};
            }
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            f32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                v[u] = rb[i][u];
                if (!((bmask >> (4 * i + u)) & 1u)) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (bsum)
#pragma unroll
                    for (int j = 0; j < 4; ++j) bacc[j] += v[u][j];
            }
            const int pp = 4 * (bpq + i * BPQ);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if constexpr (BF)
                    *(bf16x4*)&Bs[(bq * 4 + j) * LDP + pp] =
                        bf16x4{(__bf16)v[0][j], (__bf16)v[1][j], (__bf16)v[2][j], (__bf16)v[3][j]};
                else
                    *(f32x4*)&Bs[(bq * 4 + j) * LDP + pp] = f32x4{v[0][j], v[1][j], v[2][j], v[3][j]};
            }
        }
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int li = lane & 31, lh = lane >> 5;
    if (nchunks > 0) {
        issue(pbeg);
        commit();
        __syncthreads();
    }
    for (int c = 0; c < nchunks; ++c) {
        if (c + 1 < nchunks) issue(pbeg + (c + 1) * BKP);
        if constexpr (BF) {
#pragma unroll
            for (int kk = 0; kk < BKP / 16; ++kk) {
                bf16x8 af[MT], bf[NT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    af[mt] = *(const bf16x8*)&As[(wm * WM + mt * 32 + li) * LDP + kk * 16 + lh * 8];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    bf[nt] = *(const bf16x8*)&Bs[(wn * WN + nt * 32 + li) * LDP + kk * 16 + lh * 8];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[mt][nt] = mfma32_bf16(af[mt], bf[nt], acc[mt][nt]);
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < BKP / 8; ++kk) {
                f32x4 af[MT], bf[NT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
                    af[mt] = *(const f32x4*)&As[(wm * WM + mt * 32 + li) * LDP + kk * 8 + lh * 4];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    bf[nt] = *(const f32x4*)&Bs[(wn * WN + nt * 32 + li) * LDP + kk * 8 + lh * 4];
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
                            acc[mt][nt] = mfma32(af[mt][s4], bf[nt][s4], acc[mt][nt]);
            }
        }
        __syncthreads();
        if (c + 1 < nchunks) {
            commit();
            __syncthreads();
        }
    }

    if (bsum) {  // column sums of B' for the bias gradient: combine the pixel groups in order
        __syncthreads();
        double* red = (double*)smem;  // [NTH][4]
#pragma unroll
        for (int j = 0; j < 4; ++j) red[tid * 4 + j] = bacc[j];
        __syncthreads();
        if (tid < BQ) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                double t = 0.0;
                for (int g = 0; g < BPQ; ++g) t += red[(g * BQ + tid) * 4 + j];
                p.bias_slab[(size_t)split * p.Nw + tn * BN + tid * 4 + j] = (float)t;
            }
        }
    }

    float* slab = p.slab + (size_t)split * p.Mw * p.Nw;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = tm * BM + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int n = tn * BN + wn * WN + nt * 32 + li;
                slab[(size_t)m * p.Nw + n] = acc[mt][nt][r];
            }
}

}  // namespace

// ------------------------------------------------------------------------------------
// host dispatch
// ------------------------------------------------------------------------------------
// Tile table (tuned on MI355X with tools/gemm_tune.hip).  The runtime picks a tile id per
// layer; ROWGEMM_TILES lists what is instantiated.
using RowTile0 = RowTile<128, 128, 64, 64, 32, true>;
using RowTile1 = RowTile<128, 64, 64, 32, 32, false>;
using RowTile4 = RowTile<128, 128, 64, 64, 32, false>;
using RowTile6 = RowTile<128, 128, 64, 64, 64, true>;  // bf16: 4 MFMA k-steps per barrier
// (r02: 256x128 with 4 waves of 128x64, 128x128 with 2 waves of 128x64 and 128x64 with 2
// waves of 64x64 measured 3-17 % slower than these defaults; not kept)
// 32-output tiles (the 32-channel level 0 of the reference grid's narrow networks,
// config/config.yaml base_filters 16 / 24 / 32, padded to 32): 128 x 32 (2 waves) and
// 256 x 32 (4 waves), two LDS images
using RowTile13 = RowTile<128, 32, 64, 32, 32, true, 2>;
using RowTile14 = RowTile<256, 32, 64, 32, 32, true>;
// (r01-r03: 256x64, 128x128 with 64-K chunks, 256x128, three waves per SIMD and
// MFMA-phase s_setprio variants measured at or below these; not kept)
#define ROWGEMM_TILES(X) \
    X(0, RowTile0) X(1, RowTile1) X(4, RowTile4) X(6, RowTile6) X(13, RowTile13) X(14, RowTile14)

template <int AMODE, int AOP, int EMODE, class T, bool BF>
static int rowgemm_go(const RowGemmArgs& a, hipStream_t s) {
    if constexpr (BF && T::BN < 64) {  // the bf16 B loader needs 64-column tiles
        return -1;
    } else {
        if (a.N % T::BN || a.K % T::BK || a.C % T::BK) return -1;
        if (EMODE == E_CONVT && (a.cout % T::BN) && (T::BN % a.cout)) return -1;  // per-column map
        const dim3 grid(((a.M + T::BM - 1) / T::BM) * (a.N / T::BN));
        hipLaunchKernelGGL((rowgemm_kernel<AMODE, AOP, EMODE, T, BF>), grid, dim3(T::THREADS), 0, s, a);
        return (int)hipGetLastError();
    }
}

// tile 15 = 256x32 (32-k chunks, two waves per SIMD)
template <int AMODE, int AOP, int EMODE, int NT, int GK, int OCC>
static int rowgemm_direct_go(const RowGemmArgs& a, hipStream_t s) {
    if constexpr (AOP == OP_DZ) {
        return -1;
    } else {
        constexpr int BN = 32 * NT;
        if (a.N % BN || a.K % 32 || a.C % 32 || !a.bt || a.bt16) return -1;
        if (EMODE == E_CONVT && (a.cout % BN) && (BN % a.cout)) return -1;
        // affine operands stage at most 256 channels of scale / shift: the LDS-staged tile
        if (AOP != OP_PLAIN && a.C > 256) {
            if constexpr (NT == 1) return rowgemm_go<AMODE, AOP, EMODE, RowTile14, false>(a, s);
            return -1;
        }
        const dim3 grid(((a.M + 255) / 256) * (a.N / BN));
        hipLaunchKernelGGL((rowgemm_direct_kernel<AMODE, AOP, EMODE, NT, GK, OCC>), grid, dim3(256), 0, s, a);
        return (int)hipGetLastError();
    }
}

template <int AMODE, int AOP, int EMODE, bool BF>
static int rowgemm_tile(const RowGemmArgs& a, int tile, hipStream_t s) {
    if constexpr (!BF) {
        // (r04 A/B, not kept: 16-k chunks at four waves per SIMD for 32 outputs, and the
        // same kernel for 64 / 96 outputs -- slower / neutral against tiles 19/25 and 15)
        if (tile == 15) return rowgemm_direct_go<AMODE, AOP, EMODE, 1, 4, 2>(a, s);
    }
#define RG_CASE(id, T) \
    if (tile == id) return rowgemm_go<AMODE, AOP, EMODE, T, BF>(a, s);
    ROWGEMM_TILES(RG_CASE)
#undef RG_CASE
    return -1;
}

int rowgemm_tile_dims(int tile, int* bm, int* bn, int* bk) {
    if (tile == 15) {  // rowgemm_direct_kernel (operands straight from global memory)
        *bm = 256;
        *bn = 32;
        *bk = 32;
        return 0;
    }
    if (tile == 18 || tile == 19) {  // rowgemm_pipe_kernel (loads two chunks ahead)
        *bm = 128;
        *bn = tile % 2 == 0 ? 128 : 64;
        *bk = 32;
        return 0;
    }
    if (tile == 25 || tile == 26) {  // rowgemm_pipe_kernel 128x64, three blocks per CU
        *bm = 128;
        *bn = 64;
        *bk = 32;
        return 0;
    }
#define RG_DIMS(id, T)   \
    if (tile == id) {    \
        *bm = T::BM;     \
        *bn = T::BN;     \
        *bk = T::BK;     \
        return 0;        \
    }
    ROWGEMM_TILES(RG_DIMS)
#undef RG_DIMS
    return -1;
}

int rowgemm_tile_dbuf(int tile) {
    if (tile == 15) return 3;  // operands straight from global memory
    if (tile == 18 || tile == 19 || tile == 25 || tile == 26) return 2;  // pipelined
#define RG_DB(id, T) \
    if (tile == id) return T::DBUF ? 1 : 0;
    ROWGEMM_TILES(RG_DB)
#undef RG_DB
    return 0;
}

// BF (bf16 MFMA) is instantiated for the combinations of the BN -> ReLU network
// (models/mod.py) only; the ReLU -> BN network runs f32.
template <bool BF>
static int rowgemm_dispatch(const RowGemmArgs& a, int tile, hipStream_t s) {
    const bool aff = a.ascale != nullptr, dz = a.acoef != nullptr;
    if (a.amode == G_CONV3 && a.emode == E_STATS) {  // BN -> ReLU order (models/mod.py)
        if (a.arelu) return rowgemm_tile<G_CONV3, OP_AFFINE_RELU, E_STATS, BF>(a, tile, s);
        if (!aff) return rowgemm_tile<G_CONV3, OP_PLAIN, E_STATS, BF>(a, tile, s);
        return -1;
    }
    if (a.amode == G_CONV3 && (a.emode == E_STORE || a.emode == E_STORE_BN) && !dz)
        return a.emode == E_STORE ? rowgemm_tile<G_CONV3, OP_PLAIN, E_STORE, BF>(a, tile, s)
                                  : rowgemm_tile<G_CONV3, OP_PLAIN, E_STORE_BN, BF>(a, tile, s);
    if (a.amode == G_IDENT && a.emode == E_CONVT && aff && a.arelu)
        return rowgemm_tile<G_IDENT, OP_AFFINE_RELU, E_CONVT, BF>(a, tile, s);
    if (a.amode == G_UP2 && !aff && !dz && a.emode == E_STORE_BN)
        return rowgemm_tile<G_UP2, OP_PLAIN, E_STORE_BN, BF>(a, tile, s);
    if constexpr (!BF) {
        // residual network (models/mod.py:ResUNet): plain operands everywhere
        if (!aff && !dz) {
            if (a.amode == G_IDENT && a.emode == E_RESID)
                return rowgemm_tile<G_IDENT, OP_PLAIN, E_RESID, false>(a, tile, s);
            if (a.amode == G_IDENT && a.emode == E_STORE)
                return rowgemm_tile<G_IDENT, OP_PLAIN, E_STORE, false>(a, tile, s);
            if (a.amode == G_CONV3 && a.emode == E_ADD)
                return rowgemm_tile<G_CONV3, OP_PLAIN, E_ADD, false>(a, tile, s);
            if (a.amode == G_IDENT && a.emode == E_CONVT)
                return rowgemm_tile<G_IDENT, OP_PLAIN, E_CONVT, false>(a, tile, s);
            if (a.amode == G_UP2 && a.emode == E_STORE)
                return rowgemm_tile<G_UP2, OP_PLAIN, E_STORE, false>(a, tile, s);
        }
        if (a.amode == G_CONV3 && a.emode == E_BIAS_RELU_STATS)
            return aff ? rowgemm_tile<G_CONV3, OP_AFFINE, E_BIAS_RELU_STATS, false>(a, tile, s)
                       : rowgemm_tile<G_CONV3, OP_PLAIN, E_BIAS_RELU_STATS, false>(a, tile, s);
        if (a.amode == G_IDENT && a.emode == E_CONVT && aff && !a.arelu)
            return rowgemm_tile<G_IDENT, OP_AFFINE, E_CONVT, false>(a, tile, s);
    }
    return -1;  // combination not instantiated
}

int launch_rowgemm(const RowGemmArgs& a, int tile, hipStream_t s) {
    if (a.M < 1 || a.K != gather_taps(a.amode) * a.C) return -1;
    const bool aff = a.ascale != nullptr, dz = a.acoef != nullptr;
    if (aff && dz) return -1;
    if ((a.emode == E_STORE_BN || a.emode == E_RESID) != (a.ey != nullptr)) return -1;
    if ((a.escale != nullptr) != (a.eshift != nullptr) || (a.arelu && !aff)) return -1;
    if (a.emode == E_RESID && !a.escale) return -1;
    if ((a.bt != nullptr) == (a.bt16 != nullptr)) return -1;  // exactly one weight image
    // ids 18, 19, 25, 26: the software-pipelined f32 kernel (128x128 / 128x64 loading two chunks
    // ahead; 25 / 26: 128x64 at three blocks per CU); operands it does not take (bf16 weights,
    // > 2 GB offsets) run the same tile shape on the register-staged kernel
    if (tile == 18 || tile == 19 || tile == 25 || tile == 26) {
        if (rowgemm_pipe_ok(a)) return launch_rowgemm_pipe(a, tile <= 19 ? tile - 16 : tile - 21, s);
        tile = tile == 18 ? 4 : 1;
    }
    return a.bt16 ? rowgemm_dispatch<true>(a, tile, s) : rowgemm_dispatch<false>(a, tile, s);
}

// wgrad tiles: (BM, BN, pixels per chunk).  Narrow tiles take deeper pixel chunks so the
// per-chunk staging cost is spread over as many MFMAs as the 128x128 tile's.
using WgTile0 = WgTile<128, 128, 64, 64, 32>;  // 4 waves
using WgTile3 = WgTile<64, 128, 64, 64, 32>;   // 2 waves
using WgTile5 = WgTile<128, 64, 64, 32, 32>;   // 4 waves
using WgTile7 = WgTile<64, 64, 32, 32, 32, 3>;
// 32-channel operands (narrow level 0): 64 x 32 (2 waves), 32 x 32 (1 wave)
using WgTile8 = WgTile<64, 32, 32, 32, 32>;
using WgTile9 = WgTile<32, 32, 32, 32, 32>;
#define WGRAD_TILES(X) \
    X(0, WgTile0) X(3, WgTile3) X(5, WgTile5) X(7, WgTile7) X(8, WgTile8) X(9, WgTile9)

#define WG_DIMS_R3(id, T) \
    if (tile == id) {     \
        *bm = T::BM;      \
        *bn = T::BN;      \
        *bkp = T::BKP;    \
        return 0;         \
    }
// one-row-of-taps tiles (wgrad_row3_kernel, ids 20..): BM x BN per tap, 3 taps per block
using Wr3Tile0 = WgTile<64, 64, 32, 32, 32>;    // 4 waves, 3 x 32x32 per wave
using Wr3Tile1 = WgTile<128, 64, 64, 32, 32>;   // 4 waves, 3 x 64x32
using Wr3Tile2 = WgTile<64, 128, 32, 64, 32>;   // 4 waves, 3 x 32x64
using Wr3Tile3 = WgTile<128, 128, 64, 64, 32>;  // 4 waves, 3 x 64x64 (192 accumulators)
// 32-channel operands (the narrow networks' level 0, r04): one / two waves of 3 x 32x32
using Wr3Tile4 = WgTile<32, 32, 32, 32, 32>;    // Cin = Cout = 32
using Wr3Tile5 = WgTile<64, 32, 32, 32, 32>;    // Cin 64 (a [skip | up] concat), Cout 32
using Wr3Tile6 = WgTile<32, 64, 32, 32, 32>;    // Cin 32, Cout 64
// (r03: 64-pixel chunks, 16-pixel rows, all three tap rows per block and a software-
// pipelined schedule of these tiles measured at or below them; not kept)
#define WGRAD_ROW3_TILES(X) \
    X(20, Wr3Tile0) X(21, Wr3Tile1) X(22, Wr3Tile2) X(23, Wr3Tile3) X(24, Wr3Tile4) X(25, Wr3Tile5) \
    X(26, Wr3Tile6)

// a row3 block covers three taps (its split-K partition counts them)
int wgrad_tile_taps(int tile) { return tile >= 20 ? 3 : 1; }

int wgrad_tile_dims(int tile, int* bm, int* bn, int* bkp) {
    WGRAD_ROW3_TILES(WG_DIMS_R3)
#define WG_DIMS(id, T) \
    if (tile == id) {  \
        *bm = T::BM;   \
        *bn = T::BN;   \
        *bkp = T::BKP; \
        return 0;      \
    }
    WGRAD_TILES(WG_DIMS)
#undef WG_DIMS
    return -1;
}

template <int AOP, bool BDZ>
static int wgrad_row3_tile(const WgradArgs& a, int tile, hipStream_t s) {
#define WR3_CASE(id, T)                                                                       \
    if (tile == id) {                                                                         \
        if (a.Mw != 9 * a.CA || a.CA % T::BM || a.Nw % T::BN || a.CB % T::BN ||               \
            a.pps % T::BKP || a.W % T::BKP)                                                   \
            return -1;                                                                        \
        const dim3 grid(3 * (a.CA / T::BM) * (a.Nw / T::BN) * a.splits);                      \
        hipLaunchKernelGGL((wgrad_row3_kernel<AOP, BDZ, T>), grid, dim3(T::THREADS), 0, s, a); \
        return (int)hipGetLastError();                                                        \
    }
    WGRAD_ROW3_TILES(WR3_CASE)
#undef WR3_CASE
    return -1;
}

template <int AMODE, int AOP, int BMODE, bool BDZ>
static int wgrad_tile(const WgradArgs& a, int tile, hipStream_t s) {
#define WG_CASE(id, T)                                                                        \
    if (tile == id) {                                                                         \
        if (a.Mw % T::BM || a.Nw % T::BN || a.CA % T::BM || a.CB % T::BN || a.pps % T::BKP) \
            return -1;                                                                        \
        const dim3 grid((a.Mw / T::BM) * (a.Nw / T::BN) * a.splits);                          \
        hipLaunchKernelGGL((wgrad_kernel<AMODE, AOP, BMODE, BDZ, T>), grid, dim3(T::THREADS), 0, s, a); \
        return (int)hipGetLastError();                                                        \
    }
    WGRAD_TILES(WG_CASE)
#undef WG_CASE
    return -1;
}

// channel-major wgrad tiles of the register-staged bf16 path (wgradT_kernel): 4-pixel x
// 4-channel loader units
using Wg16Tile0 = WgTile<128, 128, 64, 64, 32>;
using Wg16Tile2 = WgTile<64, 64, 32, 32, 64>;
using Wg16Tile3 = WgTile<128, 64, 64, 32, 64>;
using Wg16Tile4 = WgTile<64, 128, 32, 64, 64>;
#define WGRAD16_TILES(X) X(0, Wg16Tile0) X(2, Wg16Tile2) X(3, Wg16Tile3) X(4, Wg16Tile4)

int wgrad16_tile_dims(int tile, int* bm, int* bn, int* bkp) {
#define WG16_DIMS(id, T) \
    if (tile == id) {    \
        *bm = T::BM;     \
        *bn = T::BN;     \
        *bkp = T::BKP;   \
        return 0;        \
    }
    WGRAD16_TILES(WG16_DIMS)
#undef WG16_DIMS
    return -1;
}

#define WG16_CASE(id, T)                                                                      \
    if (tile == id) {                                                                         \
        if (a.Mw % T::BM || a.Nw % T::BN || a.CA % T::BM || a.CB % T::BN || a.pps % T::BKP) \
            return -1;                                                                        \
        const dim3 grid((a.Mw / T::BM) * (a.Nw / T::BN) * a.splits);                          \
        hipLaunchKernelGGL((wgradT_kernel<AMODE, AOP, BMODE, T, true>), grid, dim3(T::THREADS), 0, s, a); \
        return (int)hipGetLastError();                                                        \
    }

template <int AMODE, int AOP, int BMODE>
static int wgradT_tile(const WgradArgs& a, int tile, hipStream_t s) {
    WGRAD16_TILES(WG16_CASE)
    return -1;
}
#undef WG16_CASE

int launch_wgrad(const WgradArgs& a, int tile, hipStream_t s) {
    if (a.P < 1) return -1;
    if (a.bf16) {  // BN -> ReLU network only (no OP_DZ loaders)
        const bool aff = a.ascale != nullptr;
        if (a.bcoef || (a.arelu && !aff) || (aff && !a.arelu)) return -1;
        if (a.amode == G_CONV3 && a.bmode == G_IDENT)
            return aff ? wgradT_tile<G_CONV3, OP_AFFINE_RELU, G_IDENT>(a, tile, s)
                       : wgradT_tile<G_CONV3, OP_PLAIN, G_IDENT>(a, tile, s);
        if (a.amode == G_IDENT && a.bmode == G_UP2 && aff)
            return wgradT_tile<G_IDENT, OP_AFFINE_RELU, G_UP2>(a, tile, s);
        return -1;
    }
    const bool aff = a.ascale != nullptr, dz = a.bcoef != nullptr;
    if (a.arelu && !aff) return -1;
    if (a.arelu && dz && !a.bdznomask) return -1;  // BN -> ReLU A' operands come with an unmasked dz
    if (tile >= 20) {  // one row of 3x3 taps per block (wgrad_row3_kernel)
        if (a.amode != G_CONV3 || a.bmode != G_IDENT) return -1;
        if (dz && a.arelu) return wgrad_row3_tile<OP_AFFINE_RELU, true>(a, tile, s);
        if (dz) return aff ? wgrad_row3_tile<OP_AFFINE, true>(a, tile, s)
                           : wgrad_row3_tile<OP_PLAIN, true>(a, tile, s);
        if (a.arelu) return wgrad_row3_tile<OP_AFFINE_RELU, false>(a, tile, s);
        return aff ? wgrad_row3_tile<OP_AFFINE, false>(a, tile, s)
                   : wgrad_row3_tile<OP_PLAIN, false>(a, tile, s);
    }
    if (a.amode == G_CONV3 && a.bmode == G_IDENT && dz) {
        if (a.arelu) return wgrad_tile<G_CONV3, OP_AFFINE_RELU, G_IDENT, true>(a, tile, s);
        return aff ? wgrad_tile<G_CONV3, OP_AFFINE, G_IDENT, true>(a, tile, s)
                   : wgrad_tile<G_CONV3, OP_PLAIN, G_IDENT, true>(a, tile, s);
    }
    if (a.amode == G_CONV3 && a.bmode == G_IDENT && !dz) {
        if (a.arelu) return wgrad_tile<G_CONV3, OP_AFFINE_RELU, G_IDENT, false>(a, tile, s);
        return aff ? wgrad_tile<G_CONV3, OP_AFFINE, G_IDENT, false>(a, tile, s)
                   : wgrad_tile<G_CONV3, OP_PLAIN, G_IDENT, false>(a, tile, s);
    }
    if (a.amode == G_IDENT && a.bmode == G_UP2 && aff && !dz)
        return a.arelu ? wgrad_tile<G_IDENT, OP_AFFINE_RELU, G_UP2, false>(a, tile, s)
                       : wgrad_tile<G_IDENT, OP_AFFINE, G_UP2, false>(a, tile, s);
    // residual network: plain operands (skip 1x1 conv; ConvT of a materialised block output)
    if (a.amode == G_IDENT && a.bmode == G_IDENT && !aff && !dz)
        return wgrad_tile<G_IDENT, OP_PLAIN, G_IDENT, false>(a, tile, s);
    if (a.amode == G_IDENT && a.bmode == G_UP2 && !aff && !dz)
        return wgrad_tile<G_IDENT, OP_PLAIN, G_UP2, false>(a, tile, s);
    return -1;
}
