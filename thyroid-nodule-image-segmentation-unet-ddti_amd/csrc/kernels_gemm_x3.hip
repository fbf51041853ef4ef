// fp32 row GEMM on the bf16 matrix cores through an exact three-way operand split.
//
// gfx950 runs f32-input MFMAs (v_mfma_f32_32x32x2_f32) at 1/16 of the bf16 rate.  Every f32
// value v splits EXACTLY into three bf16 pieces, v = h + m + l:
//   h = bf16_rne(v), m = bf16_rne(v - h), l = bf16_rne(v - h - m)
// (each difference is exact in f32; h holds the top 8 significand bits, m the next 8, l the
// last 8, so nothing is left over for normal v).  A product then is the sum of the nine
// piece products; the six kept here,
//   Ah*Bh + Ah*Bm + Am*Bh + Ah*Bl + Am*Bm + Al*Bh,
// drop Am*Bl, Al*Bm, Al*Bl, at most ~2^-25 |a b| together -- below the 2^-24 unit roundoff
// of one f32 operation.  Each piece product is exact in the MFMA (8 x 8 significand bits)
// and accumulates in f32, so a K-long dot product carries the rounding of an f32
// accumulation chain, like the f32 MFMA path: this is f32 arithmetic, not a bf16
// approximation (tests/test_gpu_x3.py holds it to the f32 kernels' own error vs fp64).
// Six bf16 MFMAs cost 6 x 32 = 192 cycles per 32x32x16 block against 8 x 64 = 512 for the
// f32 MFMA: a 2.67x higher peak (≈419 vs 157.3 TFLOP/s).
//
// "x3 image": the split operand in HBM, bf16 [rows][C / 32][3][32] -- per 32-channel group
// the h, m and l planes side by side, 192 contiguous bytes.  One K-chunk (one tap, 32
// channels) of one row is then one 192-B LDS row, and an LDS-DMA wave-instruction (1 KB)
// covers 5 1/3 such rows: the gathered activation rows cost 2 cache lines per chunk instead
// of 3 for separate planes.
//
// LDS image per stage: [BM + BN rows][192 B]; 16-B slot s of plane q of row r holds global
// chunk s ^ ((r >> 2) & 3) (the XOR on the DMA source address, the destination stays
// lane-linear).  The 16 lanes of a ds_read_b128 phase read one (plane, chunk) of 16
// consecutive rows: 16-B units r * 12 + 4 q + (c ^ ((r >> 2) & 3)) mod 16 are all distinct,
// conflict-free.  Pipeline per chunk as kernels_gemm16.hip: issue chunk k + S - 1, wait for
// chunk k's DMA, barrier, 2 k-steps x MT x NT x 6 MFMAs, barrier.
#include <algorithm>
#include <type_traits>

#include "gemm_common.h"

namespace {

typedef __attribute__((address_space(3))) void x3_lds_void;
typedef __attribute__((address_space(1))) void x3_gbl_void;

__device__ __forceinline__ void x3_dma16(const void* src, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((x3_gbl_void*)src, (x3_lds_void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void x3_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void x3_wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// the six kept piece products of one 32x32x16 block, smallest first
__device__ __forceinline__ f32x16 mfma_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
    c = mfma32_bf16(a[2], b[0], c);
    c = mfma32_bf16(a[1], b[1], c);
    c = mfma32_bf16(a[0], b[2], c);
    c = mfma32_bf16(a[1], b[0], c);
    c = mfma32_bf16(a[0], b[1], c);
    return mfma32_bf16(a[0], b[0], c);
}

template <int BM_, int BN_, int WM_, int WN_, int S_, int OCC_>
struct TileX3 {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, S = S_, OCC = OCC_;
    static constexpr int BK = 32;  // K per chunk (one tap, 32 channels), per plane
    static constexpr int WAVES = (BM / WM) * (BN / WN);
    static constexpr int THREADS = 64 * WAVES;
};

template <int AMODE, int EMODE, class T>
__global__ __launch_bounds__(T::THREADS, T::OCC) void rowgemm_x3_kernel(RowGemmArgs p) {
    constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, S = T::S, BK = T::BK;
    constexpr int WAVES = T::WAVES, WAVES_N = BN / WN;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int RB = 192;  // bytes per LDS row: 3 planes x 32 bf16
    static_assert((BM * RB) % (1024 * WAVES) == 0 && (BN * RB) % (1024 * WAVES) == 0, "loader");
    constexpr int AI = BM * RB / (1024 * WAVES), BI = BN * RB / (1024 * WAVES);
    constexpr int GPC = AI + BI;
    constexpr int DIST = S - 1;
    static_assert(DIST >= 1 && DIST <= 3, "stages");
    constexpr int STAGE = (BM + BN) * RB;
    constexpr int RED = 2 * (BM / 64) * BN * 8;
    constexpr int SMEM = STAGE * S > RED ? STAGE * S : RED;
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    auto swz = [](int r) { return (r >> 2) & 3; };

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tile_m = bid / ntn, tile_n = bid - tile_m * ntn;
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    const int H = p.H, W = p.W, C = p.C, K = p.K;
    const size_t rowa = 3 * (size_t)p.lda, rowb = 3 * (size_t)K;  // x3 row strides (bf16)

    // loader: lane `lane` of instruction j fills stage bytes (j WAVES + wave) KB + 16 lane,
    // i.e. row r = that / 192, plane q, slot s; it sources element q 32 + 8 (s ^ swz(r)) of
    // the row's 96-element group
    Pix aq[AI];
    int am[AI], ace[AI];
    bool aok[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int r = o / RB, w = o - r * RB;
        const int m = m0 + r;
        aok[j] = m < p.M;
        am[j] = aok[j] ? m : p.M - 1;
        aq[j] = decode(am[j], H, W);
        ace[j] = (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(r)) << 3);
    }
    const uint16_t* bsrc[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int r = o / RB, w = o - r * RB;
        bsrc[j] = p.bt16 + (size_t)(n0 + r) * rowb + (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(BM + r)) << 3);
    }
    const uint16_t* zero = (const uint16_t*)p.zero16;
    const uint16_t* a16 = p.a16 + (size_t)p.aoff * 3;

    auto issue = [&](int kc, int st) {
        const int k0 = kc * BK;
        const int tap = k0 / C;
        const int c0 = k0 - tap * C;
        char* base = smem + st * STAGE;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            bool valid;
            const int src = gather_src<AMODE>(tap, am[j], aq[j], H, W, valid);
            const uint16_t* g = (valid && aok[j]) ? a16 + (size_t)src * rowa + c0 * 3 + ace[j] : zero;
            x3_dma16(g, base + (j * WAVES + wave) * 1024);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j)
            x3_dma16(bsrc[j] + k0 * 3, base + BM * RB + (j * WAVES + wave) * 1024);
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int li = lane & 31, lh = lane >> 5;
    int aro[MT], afx[MT], bro[NT], bfx[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int r = wm * WM + mt * 32 + li;
        aro[mt] = r * RB;
        afx[mt] = swz(r);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int r = BM + wn * WN + nt * 32 + li;
        bro[nt] = r * RB;
        bfx[nt] = swz(r);
    }

    const int nk = K / BK;
#pragma unroll
    for (int s = 0; s < DIST; ++s)
        if (s < nk) issue(s, s);
    for (int kc = 0; kc < nk; ++kc) {
        if (kc + DIST < nk) issue(kc + DIST, (kc + DIST) % S);
        const int ahead = min(DIST, nk - 1 - kc);
        if constexpr (DIST >= 3) {
            if (ahead >= 3) x3_wait_vm<3 * GPC>();
            else if (ahead == 2) x3_wait_vm<2 * GPC>();
            else if (ahead == 1) x3_wait_vm<GPC>();
            else x3_wait_vm<0>();
        } else if constexpr (DIST == 2) {
            if (ahead >= 2) x3_wait_vm<2 * GPC>();
            else if (ahead == 1) x3_wait_vm<GPC>();
            else x3_wait_vm<0>();
        } else {
            if (ahead >= 1) x3_wait_vm<GPC>();
            else x3_wait_vm<0>();
        }
        x3_barrier();
        const char* base = smem + (kc % S) * STAGE;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            const int c = kk * 2 + lh;
            bf16x8 af[MT][3], bfr[NT][3];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    af[mt][q] = *(const bf16x8*)(base + aro[mt] + q * 64 + ((c ^ afx[mt]) << 4));
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    bfr[nt][q] = *(const bf16x8*)(base + bro[nt] + q * 64 + ((c ^ bfx[nt]) << 4));
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma_x3(af[mt], bfr[nt], acc[mt][nt]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        x3_barrier();
    }
    row_epilogue<EMODE, BM, BN, WM, WN, true>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)smem);
}

// tiles: 0 = 256x128 (8 waves of 64x64, 2 stages, 144 KB), 1 = 128x128 (4 waves of 64x64,
// 3 stages), 2 = 256x64 (4 waves of 64x64, 2 stages), 3 = 256x128 (4 waves of 128x64),
// 4 = 128x128 (4 waves, 2 stages: 96 KB)
using TX0 = TileX3<256, 128, 64, 64, 2, 1>;
using TX1 = TileX3<128, 128, 64, 64, 3, 1>;
using TX2 = TileX3<256, 64, 64, 64, 2, 1>;
using TX3 = TileX3<256, 128, 128, 64, 2, 1>;
using TX4 = TileX3<128, 128, 64, 64, 2, 1>;
#define ROWGEMM_X3_TILES(X) X(0, TX0) X(1, TX1) X(2, TX2) X(3, TX3) X(4, TX4)

template <int AMODE, int EMODE, class T>
static int x3_go(const RowGemmArgs& a, hipStream_t s) {
    if (a.N % T::BN || a.C % 32 || a.K % 32) return -1;
    if (EMODE == E_CONVT && (a.cout % T::BN) && (T::BN % a.cout)) return -1;
    const dim3 grid(((a.M + T::BM - 1) / T::BM) * (a.N / T::BN));
    hipLaunchKernelGGL((rowgemm_x3_kernel<AMODE, EMODE, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

template <int AMODE, int EMODE>
static int x3_tile(const RowGemmArgs& a, int tile, hipStream_t s) {
#define X3_CASE(id, T) \
    if (tile == id) return x3_go<AMODE, EMODE, T>(a, s);
    ROWGEMM_X3_TILES(X3_CASE)
#undef X3_CASE
    return -1;
}

// x3 image of op(src) (f32 [P][ld] at channel offset off, C channels; scale / shift: the
// BN affine, ReLU on channels < relu) into dst [P][dld / 32][3][32] at channel offset doff.
// One thread per 8 channels of a row.
__global__ void to_x3_kernel(const float* __restrict__ src, int ld, int off, int C,
                             const float* __restrict__ scale, const float* __restrict__ shift,
                             int relu, int64_t P, uint16_t* __restrict__ dst, int dld, int doff) {
    const int g8 = C / 8;
    const int64_t n = P * g8;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / g8;
        const int c = (int)(i - r * g8) * 8;
        const float* s = src + r * ld + off + c;
        const f32x4 v0 = *(const f32x4*)s, v1 = *(const f32x4*)(s + 4);
        float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        if (scale) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float t = __builtin_fmaf(scale[c + j], v[j], shift[c + j]);
                if (c + j < relu) t = fmaxf(t, 0.f);
                v[j] = t;
            }
        }
        bf16x8 h, m, l;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const __bf16 hj = (__bf16)v[j];
            const float r1 = v[j] - (float)hj;
            const __bf16 mj = (__bf16)r1;
            const float r2 = r1 - (float)mj;
            h[j] = hj;
            m[j] = mj;
            l[j] = (__bf16)r2;
        }
        const int cc = doff + c;
        uint16_t* d = dst + r * 3 * (int64_t)dld + (cc >> 5) * 96 + (cc & 31);
        *(bf16x8*)d = h;
        *(bf16x8*)(d + 32) = m;
        *(bf16x8*)(d + 64) = l;
    }
}

}  // namespace

int rowgemm_x3_tile_dims(int tile, int* bm, int* bn) {
#define X3_DIMS(id, T)  \
    if (tile == id) {   \
        *bm = T::BM;    \
        *bn = T::BN;    \
        return 0;       \
    }
    ROWGEMM_X3_TILES(X3_DIMS)
#undef X3_DIMS
    return -1;
}

// A: x3 image (a16, lda channels per row, channel offset aoff), Bt: x3 weights [N][K]
int launch_rowgemm_x3(const RowGemmArgs& a, int tile, hipStream_t s) {
    if (!a.a16 || !a.bt16 || !a.zero16 || a.M < 1 || a.K != gather_taps(a.amode) * a.C) return -1;
    if (a.aoff % 32 || a.lda % 32) return -1;
    if ((a.emode == E_STORE_BN || a.emode == E_RESID) != (a.ey != nullptr)) return -1;
    if (a.ascale || a.acoef) return -1;  // the x3 image already holds op(A)
    if (a.amode == G_CONV3) {
        if (a.emode == E_BIAS_RELU_STATS) return x3_tile<G_CONV3, E_BIAS_RELU_STATS>(a, tile, s);
        if (a.emode == E_STATS) return x3_tile<G_CONV3, E_STATS>(a, tile, s);
        if (a.emode == E_STORE) return x3_tile<G_CONV3, E_STORE>(a, tile, s);
        if (a.emode == E_STORE_BN) return x3_tile<G_CONV3, E_STORE_BN>(a, tile, s);
        if (a.emode == E_ADD) return x3_tile<G_CONV3, E_ADD>(a, tile, s);
    }
    if (a.amode == G_UP2) {
        if (a.emode == E_STORE_BN) return x3_tile<G_UP2, E_STORE_BN>(a, tile, s);
        if (a.emode == E_STORE) return x3_tile<G_UP2, E_STORE>(a, tile, s);
    }
    if (a.amode == G_IDENT && a.emode == E_CONVT) return x3_tile<G_IDENT, E_CONVT>(a, tile, s);
    return -1;
}

int k_to_x3(const float* src, int ld, int off, int C, const float* scale, const float* shift,
            int relu, int64_t P, uint16_t* dst, int dld, int doff, hipStream_t s) {
    if (C % 32 || dld % 32 || doff % 32 || ld % 4 || off % 4) return -1;
    const int64_t n = P * (C / 8);
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(to_x3_kernel, dim3(blocks), dim3(256), 0, s, src, ld, off, C, scale, shift,
                       relu, P, dst, dld, doff);
    return (int)hipGetLastError();
}
