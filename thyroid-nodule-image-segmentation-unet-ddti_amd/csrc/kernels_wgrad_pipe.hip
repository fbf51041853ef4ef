// Software-pipelined weight gradient of a 3x3 conv, one ROW of taps per block (gfx950, f32
// in / f32 accumulate on v_mfma_f32_32x32x2_f32).
//
// Same contract, K order and numerics as wgrad_row3_kernel (kernels_gemm.hip): dW[(dy,dx)]
// [ci][co] = sum_p x[p + (dy-1, dx-1)][ci] * dz[p][co] over pixel chunks of BKP pixels of
// one image row; the block stages the chunk's input row once with a one-pixel halo and
// feeds the three dx taps from it; split-K slabs, bias column sums (f64 per lane, combined
// in order) and the BN affine / ReLU / OP_DZ loaders are those of the one-tap kernels, so
// the two kernels write identical bits.
//
// What differs is the schedule (the reasoning of kernels_gemm_pipe.hip): two LDS images;
// during chunk c's MFMAs the wave commits chunk c+1 (loaded into registers one chunk
// earlier) into the other image and issues chunk c+2's global loads; one barrier per chunk;
// the loop body is branch-free (tail chunks re-load the last chunk into the image nobody
// reads; the bias sums add zero outside the tm == 0 blocks) so sched_group_barrier can
// spread the commit's ds_writes and the loads between the 3 x MT x NT x BKP / 2 MFMAs.
#include "gemm_common.h"

namespace {

template <int BM_, int BN_, int WM_, int WN_, int BKP_, int OCC_ = 1>
struct Wr3PipeTile {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BKP = BKP_, OCC = OCC_;
    static constexpr int THREADS = 64 * (BM / WM) * (BN / WN);
};

template <int AOP, bool BDZ, class T>
__global__ __launch_bounds__(T::THREADS, T::OCC) void wgrad_row3_pipe_kernel(WgradArgs p) {
    constexpr bool AFFINE = AOP == OP_AFFINE || AOP == OP_AFFINE_RELU;
    constexpr bool ARELU = AOP == OP_AFFINE_RELU;
    constexpr int BM = T::BM, BN = T::BN, BKP = T::BKP, WM = T::WM, WN = T::WN;
    constexpr int NTH = T::THREADS;
    constexpr int WAVES_N = BN / WN;
    constexpr int LDA = BM + 4, LDB = BN + 4;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int AF = BM / 4, BF = BN / 4;          // float4 per pixel row
    constexpr int ARPP = NTH / AF, BRPP = NTH / BF;  // rows per pass
    constexpr int AROWS = BKP + 2;                   // chunk + halo
    constexpr int AP = (AROWS + ARPP - 1) / ARPP, BP = BKP / BRPP;
    constexpr int AIMG = AP * ARPP * LDA;            // rows past AROWS: written, never read
    constexpr int BIMG = BKP * LDB;
    static_assert(ARPP * AF == NTH && BP * BRPP == BKP, "loader shape");
    __shared__ __attribute__((aligned(16))) float As[2 * AIMG];
    __shared__ __attribute__((aligned(16))) float Bs[2 * BIMG];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ctm = p.CA / BM;  // channel tiles per tap row
    const int tiles_n = p.Nw / BN, tiles_m = 3 * ctm;
    int idx = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tn = idx % tiles_n;
    idx /= tiles_n;
    const int tm = idx % tiles_m;
    const int split = idx / tiles_m;
    const int dy = tm / ctm, ca0 = (tm - dy * ctm) * BM;
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
    f32x4 ra[AP], rb[BP];
    unsigned amask = 0, bmask = 0;
    const float* abase = p.a + p.aoff + ca0 + ac4 * 4;
    const float* bbase = p.b + p.boff + cb0 + bc4 * 4;
    auto issue = [&](int c) {
        const int pc = pbeg + c * BKP;
        amask = bmask = 0;
        const Pix q = decode(pc, H, W);  // chunk start; the chunk stays on this row
        const int yy = q.y + dy - 1;
        const bool rowok = (yy >= 0) & (yy < H);
        const int rbase = (q.img * H + (rowok ? yy : q.y)) * W;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const int r = arow + i * ARPP;
            const int xx = q.x + r - 1;
            const bool valid = rowok & (r < AROWS) & (xx >= 0) & (xx < W);
            amask |= valid ? (1u << i) : 0u;
            const int src = valid ? rbase + xx : pc;
            ra[i] = *(const f32x4*)(abase + (size_t)src * p.lda);
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            int m = pc + brow + i * BRPP;
            const bool in = m < pend;
            m = in ? m : pend - 1;
            bmask |= in ? (1u << i) : 0u;
            rb[i] = *(const f32x4*)(bbase + (size_t)m * p.ldb);
            if constexpr (BDZ)
                ryb[i] = *(const f32x4*)(p.by + (size_t)m * p.ldby + p.offby + cb0 + bc4 * 4);
        }
    };
    // live: a real chunk (false for the tail repeat, which must not enter the bias sums)
    auto commit = [&](int buf, bool live) {
        const bool bs_on = bsum && live;
        float* as = As + buf * AIMG;
        float* bs = Bs + buf * BIMG;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            f32x4 v = ra[i];
            if constexpr (AFFINE) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float t = __builtin_fmaf(v[j], sc[j], sh[j]);
                    v[j] = (ARELU && arl) ? fmaxf(t, 0.f) : t;
                }
            }
            const bool keep = (amask >> i) & 1u;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = keep ? v[j] : 0.f;
            *(f32x4*)&as[(arow + i * ARPP) * LDA + ac4 * 4] = v;
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            f32x4 v = rb[i];
            if constexpr (BDZ) {
                const f32x4 d = bn_dz4(ca, v, cb, ryb[i], cm, cc);
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = ryb[i][j] > 0.f ? d[j] : 0.f;
            }
            const bool keep = (bmask >> i) & 1u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = keep ? v[j] : 0.f;
                bacc[j] += bs_on ? (double)v[j] : 0.0;
            }
            *(f32x4*)&bs[(brow + i * BRPP) * LDB + bc4 * 4] = v;
        }
    };

    f32x16 acc[3][MT][NT];
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[d][i][j][r] = 0.f;

    const int li = lane & 31, lh = lane >> 5;
    constexpr int NMF = 3 * MT * NT * BKP / 2;  // MFMAs per chunk
    constexpr int NDSW = AP + BP;
    constexpr int NVM = AP + BP * (BDZ ? 2 : 1);
    static_assert(NDSW + NVM <= NMF, "schedule shape");
    if (nchunks > 0) {
        issue(0);
        commit(0, true);
        issue(nchunks > 1 ? 1 : 0);
        __syncthreads();
    }
    for (int c = 0; c < nchunks; ++c) {
        const float* as = As + (c & 1) * AIMG;
        const float* bs = Bs + (c & 1) * BIMG;
        commit((c + 1) & 1, c + 1 < nchunks);  // chunk c+1 (tail: a repeat, unread)
        issue(c + 2 < nchunks ? c + 2 : nchunks - 1);
#pragma unroll
        for (int kk = 0; kk < BKP / 8; ++kk)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int pr = kk * 8 + lh * 4 + s;
                float bf[NT];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) bf[nt] = bs[pr * LDB + wn * WN + nt * 32 + li];
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    float af[MT];
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) af[mt] = as[(pr + d) * LDA + wm * WM + mt * 32 + li];
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
                            acc[d][mt][nt] = mfma32(af[mt], bf[nt], acc[d][mt][nt]);
                }
            }
        // spread the commit (ds_write + its VALU) and the next loads over the first MFMAs
#pragma unroll
        for (int i = 0; i < NDSW; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);  // VALU
            __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
        }
#pragma unroll
        for (int i = 0; i < NVM; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU
            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
        }
        __syncthreads();
    }

    if (bsum) {  // column sums of B' for the bias gradient: combine the row groups in order
        double* red = (double*)As;  // [NTH][4]
        static_assert(2 * AIMG >= 8 * NTH, "bias reduction scratch");
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

    // slab rows m = (3*dy + d)*CA + ca0 + ...: wave-uniform row bases, per-lane offsets
    float* slab = p.slab + (size_t)split * p.Mw * p.Nw;
    const unsigned lo = (unsigned)(4 * lh * p.Nw + tn * BN + wn * WN + li) * 4u;
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = (3 * dy + d) * p.CA + ca0 + wm * WM + mt * 32 + (r & 3) + 8 * (r >> 2);
                    *(float*)((char*)(slab + (size_t)m * p.Nw + nt * 32) + lo) = acc[d][mt][nt][r];
                }
}

// pipelined counterparts of kernels_gemm.hip's Wr3Tile0..3
using Wr3P0 = Wr3PipeTile<64, 64, 32, 32, 32>;
using Wr3P1 = Wr3PipeTile<128, 64, 64, 32, 32>;
using Wr3P2 = Wr3PipeTile<64, 128, 32, 64, 32>;
using Wr3P3 = Wr3PipeTile<128, 128, 64, 64, 32>;
using Wr3P4 = Wr3PipeTile<128, 64, 64, 32, 32, 2>;  // Wr3P1 at two waves per SIMD

template <int AOP, bool BDZ, class T>
static int wr3p_go(const WgradArgs& a, hipStream_t s) {
    if (a.Mw != 9 * a.CA || a.CA % T::BM || a.Nw % T::BN || a.CB % T::BN || a.pps % T::BKP ||
        a.W % T::BKP)
        return -1;
    const dim3 grid(3 * (a.CA / T::BM) * (a.Nw / T::BN) * a.splits);
    hipLaunchKernelGGL((wgrad_row3_pipe_kernel<AOP, BDZ, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

template <int AOP, bool BDZ>
static int wr3p_tile(const WgradArgs& a, int tile, hipStream_t s) {
    switch (tile) {
        case 0: return wr3p_go<AOP, BDZ, Wr3P0>(a, s);
        case 1: return wr3p_go<AOP, BDZ, Wr3P1>(a, s);
        case 2: return wr3p_go<AOP, BDZ, Wr3P2>(a, s);
        case 3: return wr3p_go<AOP, BDZ, Wr3P3>(a, s);
        case 4: return wr3p_go<AOP, BDZ, Wr3P4>(a, s);
    }
    return -1;
}

}  // namespace

// tile 0..3: the shapes of kernels_gemm.hip's row3 tiles 20..23; 4 = tile 1 at two waves per SIMD
int launch_wgrad_row3_pipe(const WgradArgs& a, int tile, hipStream_t s) {
    if (a.P < 1 || a.bf16 || a.amode != G_CONV3 || a.bmode != G_IDENT) return -1;
    const bool aff = a.ascale != nullptr, dz = a.bcoef != nullptr;
    if (a.arelu && (!aff || dz)) return -1;
    if (dz) return aff ? wr3p_tile<OP_AFFINE, true>(a, tile, s) : wr3p_tile<OP_PLAIN, true>(a, tile, s);
    if (a.arelu) return wr3p_tile<OP_AFFINE_RELU, false>(a, tile, s);
    return aff ? wr3p_tile<OP_AFFINE, false>(a, tile, s) : wr3p_tile<OP_PLAIN, false>(a, tile, s);
}
