// bf16 row GEMM staged by LDS-DMA (global_load_lds_dwordx4) for the bf16-MFMA path
// (BASELINE config 4: models/mod.py UNet(base 128, depth 5) at 512x512).
//
// Same GEMM as kernels_gemm.hip's rowgemm (C[m][n] = sum_k A[m][k] * Bt[n][k], rows m =
// output pixels, k = (tap, channel)), but both operands are bf16 in HBM: A is a dense
// [pixels][C] bf16 image of the conv input with its BatchNorm affine and ReLU already
// applied (k_to_bf16, one pass per layer), Bt the packed bf16 weights.  With no arithmetic
// left between HBM and the matrix cores, each lane's 16 bytes go straight into LDS
// (global_load_lds_dwordx4: per-lane source address, lane-linear LDS destination), several
// K-chunks ahead, so the loads of chunks k+1..k+S-1 stream while chunk k feeds the MFMAs --
// the register-staged kernel could keep only one chunk in flight and was latency-bound at
// ~12 % of the bf16 peak.
//
// LDS image per stage: [BM + BN rows][64 bf16] = 128-B rows.  One wave-instruction fills 8
// rows (lane l -> row l/8, 16-B slot l%8).  Slot s of row r holds global chunk s ^ f(r),
// f(r) = (r >> 1) & 7 (the XOR is applied to the SOURCE address, the destination stays
// lane-linear); an MFMA lane reading chunk c of row r addresses slot c ^ f(r).  Each 16-lane
// phase of ds_read_b128 (rows r .. in one 256-B bank row pair) then hits 16 distinct slots.
// Padding taps and rows past M read a zeroed 16-B page instead of the activation.
//
// Pipeline per K-chunk (S stages): issue chunk k+S-1, s_waitcnt vmcnt(#chunks still allowed
// in flight x loads per chunk), s_barrier (every wave's DMA for chunk k has landed), MFMAs
// from stage k % S, s_barrier (stage free for reuse).  Raw s_barrier, not __syncthreads():
// the latter's fence would drain the DMAs still in flight.
#include <type_traits>

#include "gemm_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_wave_base, 16, 0, 0);
}

// s_barrier with compiler fences: the builtin itself does not order memory operations, so
// without them ds_reads could be hoisted above it (or sunk below it)
__device__ __forceinline__ void block_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// block tile BM x BN, wave tile WM x WN, S LDS stages of BK = 64 K each; prefetch distance
// S-1 chunks, a second barrier after each chunk's MFMAs frees its stage.
// (r01-r03 variants measured at or below this schedule and not kept: 32-K chunks with 4-5
// stages and one barrier per chunk, DMA issue interleaved between the MFMAs, LDS fragments
// read one k-step ahead, 16x16x32 MFMAs with / without s_setprio, a ping-pong schedule of two
// wave groups one barrier apart)
template <int BM_, int BN_, int WM_, int WN_, int S_, int OCC_>
struct Tile16 {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, S = S_, OCC = OCC_;
    static constexpr int BK = 64;
    static constexpr int WAVES = (BM / WM) * (BN / WN);
    static constexpr int THREADS = 64 * WAVES;
};

template <int AMODE, int EMODE, class T>
__global__ __launch_bounds__(T::THREADS, T::OCC) void rowgemm16_kernel(RowGemmArgs p) {
    constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, S = T::S, BK = T::BK;
    constexpr int WAVES = T::WAVES, WAVES_N = BN / WN;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int RB = 2 * BK;             // bytes per LDS row
    constexpr int LPR = RB / 16;           // 16-B chunks (DMA lanes) per row
    constexpr int RPI = 64 / LPR;          // rows per DMA wave-instruction (1 KB)
    constexpr int RPB = 256 / RB;          // rows per 256-B bank row
    // slot of chunk c in row r: c ^ swz(r).  A 16-lane ds_read_b128 phase reads one chunk of
    // 16 rows; with RPB rows per bank row and LPR slots per row, XORing by (r / RPB) mod LPR
    // spreads them over all 16 slots of the 256-B bank row.
    auto swz = [](int r) { return (r / RPB) & (LPR - 1); };
    constexpr int AI = BM / (RPI * WAVES), BI = BN / (RPI * WAVES);  // DMA instructions per chunk
    static_assert(AI * RPI * WAVES == BM && BI * RPI * WAVES == BN, "loader shape");
    constexpr int GPC = AI + BI;
    constexpr int DIST = S - 1;  // chunks in flight beyond the current one
    static_assert(DIST >= 1, "stages");
    constexpr int STAGE = (BM + BN) * RB;  // bytes
    constexpr int RED = 2 * (BM / 64) * BN * 8;  // epilogue scratch (f64 partials per 64-row unit)
    constexpr int SMEM = STAGE * S > RED ? STAGE * S : RED;
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    int tile_m, tile_n;
    tile_mn(bid, (p.M + BM - 1) / BM, ntn, p.tgm, tile_m, tile_n);
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    const int H = p.H, W = p.W, C = p.C, K = p.K;

    // loader rows: instruction j of this wave fills rows (j * WAVES + wave) * RPI .. + RPI-1
    const int lr = lane / LPR, slot = lane % LPR;
    Pix aq[AI];
    int am[AI], ach[AI];
    bool aok[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int r = (j * WAVES + wave) * RPI + lr;
        const int m = m0 + r;
        aok[j] = m < p.M;
        am[j] = aok[j] ? m : p.M - 1;
        aq[j] = decode(am[j], H, W);
        ach[j] = (slot ^ swz(r)) * 8;
    }
    const uint16_t* bsrc[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int r = (j * WAVES + wave) * RPI + lr;
        bsrc[j] = p.bt16 + (size_t)(n0 + r) * K + (slot ^ swz(r)) * 8;
    }
    const uint16_t* zero = (const uint16_t*)p.zero16;

    // DMA pieces [j0, j1) of chunk kc into stage st (pieces 0..AI-1 = A rows, then B rows)
    auto issue = [&](int kc, int st) {
        const int k0 = kc * BK;
        const int tap = k0 / C;
        const int c0 = k0 - tap * C;
        char* base = smem + st * STAGE;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            bool valid;
            const int src = gather_src<AMODE>(tap, am[j], aq[j], H, W, valid);
            const uint16_t* g = (valid && aok[j]) ? p.a16 + (size_t)src * p.lda + c0 + ach[j] : zero;
            glds16(g, base + (j * WAVES + wave) * 1024);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) glds16(bsrc[j] + k0, base + BM * RB + (j * WAVES + wave) * 1024);
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int li = lane & 31, lh = lane >> 5;
    // LDS read offsets (bytes) of this lane's rows; the chunk XOR depends on the row only
    int aro[MT], afx[MT], bro[NT], bfx[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int r = wm * WM + mt * 32 + li;
        aro[mt] = r * RB;
        afx[mt] = swz(r);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int r = wn * WN + nt * 32 + li;
        bro[nt] = (BM + r) * RB;
        bfx[nt] = swz(r);
    }

    const int nk = K / BK;
#pragma unroll
    for (int s = 0; s < DIST; ++s)
        if (s < nk) issue(s, s);
    constexpr int INFL = DIST;  // chunks issued after kc before its wait
    for (int kc = 0; kc < nk; ++kc) {
        if (kc + DIST < nk) issue(kc + DIST, (kc + DIST) % S);
        // chunks issued after kc that may stay in flight
        const int ahead = min(INFL, nk - 1 - kc);
        if constexpr (INFL >= 3) {
            if (ahead >= 3) wait_vm<3 * GPC>();
            else if (ahead == 2) wait_vm<2 * GPC>();
            else if (ahead == 1) wait_vm<GPC>();
            else wait_vm<0>();
        } else if constexpr (INFL == 2) {
            if (ahead >= 2) wait_vm<2 * GPC>();
            else if (ahead == 1) wait_vm<GPC>();
            else wait_vm<0>();
        } else if constexpr (INFL == 1) {
            if (ahead >= 1) wait_vm<GPC>();
            else wait_vm<0>();
        } else {
            wait_vm<0>();
        }
        block_barrier();
        const char* base = smem + (kc % S) * STAGE;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            const int c = kk * 2 + lh;
            bf16x8 af[MT], bfr[NT];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
                af[mt] = *(const bf16x8*)(base + aro[mt] + ((c ^ afx[mt]) << 4));
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                bfr[nt] = *(const bf16x8*)(base + bro[nt] + ((c ^ bfx[nt]) << 4));
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32_bf16(af[mt], bfr[nt], acc[mt][nt]);
        }
        // this stage's ds_reads must have returned before any wave restages it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        block_barrier();
    }
    row_epilogue<EMODE, BM, BN, WM, WN, true>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)smem);
}

// ------------------------------------------------------------------------------------
// Tap-row halo variant of the 3x3 conv GEMM (tile 19, G_CONV3 only, W >= 16).  The
// one-tap kernel restages the block's 256 A rows for each of the 9 taps; here a stage holds
// the HALO of one tap row dy -- the block's image rows shifted by dy - 1, one extra pixel
// either side (ROWS x (SEG + 2) rows, <= 288) -- with the B rows of the three taps (dy, 0..2),
// and the three dx taps read A rows h + dx from the same halo.  Per 32-channel stage: 17-18
// A + 48 B DMA pieces of 1 KB feed 48 MFMAs per wave (one-tap kernel: 32 + 32 pieces per 32
// MFMAs), i.e. 25 % fewer LDS-DMA bytes per MFMA and 1.5x the MFMAs between barriers.
//   geometry: SEG = min(W, 256) output pixels per image row of the tile, ROWS = 256 / SEG
//   (W a power of two: a tile is ROWS whole rows, or half a 512-pixel row); halo row
//   h = r (SEG + 2) + xl + 1 holds pixel (row r shifted by dy - 1, column x0 + xl),
//   xl = -1 .. SEG; output pixel (r, xo) reads halo row r (SEG + 2) + xo + dx for tap dx.
//   LDS rows are 64 B (32 bf16); chunk c of row r sits in slot c ^ ((r >> 2) & 3), which
//   keeps the shifted, row-jumping A reads at most 2-way conflicted (W = 16; none otherwise).
//   K order: dy, 32-channel slice, dx, k -- a reordering of the one-tap kernel's sum, so
//   results agree with the other tiles to fp32 rounding, not bitwise.
// ------------------------------------------------------------------------------------
// BM x BN block tiles: 256 x 256 (tile 19) and 512 x 128 (tile 20, the 128-output layers of
// config 4's level 0: 8 waves of 128 x 64 either way).
// (r05, removed in r06: waves 4..7 running each stage's last tap after the next barrier, with
// and without the next DMA behind the first tap's reads; the same kernel on 16x16x32 MFMAs:
// +1 % kernel, -0.4 % step, profiles/r05_1tap16_ab.txt)
template <int EMODE, int BM, int BN>
__global__ __launch_bounds__(512, 1) void rowgemm16_row3_kernel(RowGemmArgs p) {
    constexpr int WM = 128, WN = 64, BK = 32, WAVES_N = BN / WN;
    constexpr int WAVES = (BM / WM) * WAVES_N;
    static_assert(WAVES == 8, "512 threads");
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int RB = 2 * BK, LPR = RB / 16, RPI = 64 / LPR;  // 64-B rows, 16 rows / piece
    auto swz = [](int r) { return (r >> 2) & 3; };
    constexpr int AR = (BM / 16) * 18;        // halo rows held (W = 16: BM / 16 rows x 18)
    constexpr int AI = (AR / RPI + WAVES - 1) / WAVES;  // A pieces per wave (w, w + 8, ...)
    constexpr int BR = 3 * BN;                // B rows: taps dx = 0..2 x BN outputs
    constexpr int BI = BR / (RPI * WAVES);    // 6 / 3
    static_assert(BI * RPI * WAVES == BR && (AR / RPI) <= AI * WAVES, "loader shape");
    constexpr int STAGE = (AR + BR) * RB;     // 66 KB / 60 KB
    constexpr int SMEM = 2 * STAGE;
    static_assert(SMEM >= 2 * (BM / 64) * BN * 8, "epilogue scratch");
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    int tile_m, tile_n;
    tile_mn(bid, (p.M + BM - 1) / BM, ntn, p.tgm, tile_m, tile_n);
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    const int H = p.H, W = p.W, C = p.C, K = p.K;
    const int SEG = W < BM ? W : BM, HW = SEG + 2;
    const int AROWS = (BM / SEG) * HW;
    const int NA = (AROWS + RPI - 1) / RPI;           // A pieces per stage (17 or 18)
    const bool a3 = (AI - 1) * WAVES + wave < NA;     // this wave issues its last A piece

    const int lr = lane / LPR, slot = lane % LPR;
    int acen[AI], ayr[AI], ach[AI];  // pixel at dy = 1 (-1: padding), its image row, chunk
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int h = (j * WAVES + wave) * RPI + lr;
        const int r = h / HW, xl = h - r * HW - 1;
        const int mrow = m0 + r * SEG;  // first output pixel of the tile's image row r
        bool ok = h < AROWS && mrow < p.M;
        const Pix q = decode(ok ? mrow : 0, H, W);
        ok = ok && q.x + xl >= 0 && q.x + xl < W;
        acen[j] = ok ? mrow + xl : -1;
        ayr[j] = q.y;
        ach[j] = (slot ^ swz(h)) * 8;
    }
    const uint16_t* bsrc[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int rb = (j * WAVES + wave) * RPI + lr;
        const int dx = rb / BN, nl = rb - dx * BN;
        bsrc[j] = p.bt16 + (size_t)(n0 + nl) * K + dx * C + (slot ^ swz(rb)) * 8;
    }
    const uint16_t* zero = (const uint16_t*)p.zero16;
    const int CC = C / BK;  // channel slices per tap row
    auto issue = [&](int s) {
        const int dy = s / CC, c0 = (s - dy * CC) * BK;
        char* base = smem + (s & 1) * STAGE;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            if (j == AI - 1 && !a3) continue;
            const int yy = ayr[j] + dy - 1;
            const bool valid = acen[j] >= 0 && yy >= 0 && yy < H;
            const uint16_t* g =
                valid ? p.a16 + (size_t)(acen[j] + (dy - 1) * W) * p.lda + c0 + ach[j] : zero;
            glds16(g, base + (j * WAVES + wave) * 1024);
        }
        const int kb = dy * 3 * C + c0;
#pragma unroll
        for (int j = 0; j < BI; ++j) glds16(bsrc[j] + kb, base + AR * RB + (j * WAVES + wave) * 1024);
    };

    f32x16 acc[MT][NT];
    const int ns = 3 * CC;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int lh = lane >> 5, li = lane & 31;
    int ahb[MT], bro[NT], bfx[NT];  // halo row of output pixel at dx = 0; B row offsets
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int mo = wm * WM + mt * 32 + li;
        const int r = mo / SEG;
        ahb[mt] = r * HW + (mo - r * SEG);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int r = wn * WN + nt * 32 + li;
        bro[nt] = (AR + r) * RB;
        bfx[nt] = swz(r);  // rows dx * 256 + r share it
    }

    issue(0);
    for (int s = 0; s < ns; ++s) {
        // one barrier per stage: wait for stage s, barrier (every wave's DMA landed, every wave
        // done reading stage s - 1), then restage s - 1's buffer with s + 1.  (r04: issuing
        // before the wait and a second barrier after the MFMAs gave the same bits, 3 % slower.)
        wait_vm<0>();
        block_barrier();
        if (s + 1 < ns) issue(s + 1);
        const char* base = smem + (s & 1) * STAGE;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int kk = 0; kk < BK / 16; ++kk) {
                const int c = kk * 2 + lh;
                bf16x8 af[MT], bfr[NT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const int h = ahb[mt] + dx;
                    af[mt] = *(const bf16x8*)(base + h * RB + ((c ^ swz(h)) << 4));
                }
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    bfr[nt] = *(const bf16x8*)(base + bro[nt] + dx * BN * RB + ((c ^ bfx[nt]) << 4));
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma32_bf16(af[mt], bfr[nt], acc[mt][nt]);
            }
        // this stage's ds_reads must have returned before any wave restages it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    block_barrier();  // the epilogue reuses the stage memory
    row_epilogue<EMODE, BM, BN, WM, WN, true>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)smem);
}

template <int EMODE, int BM, int BN>
static int rg16r3_go(const RowGemmArgs& a, hipStream_t s) {
    // BM % W == 0 or W % BM == 0 keeps a tile on whole rows / row segments; W >= 16 bounds the halo
    if (a.amode != G_CONV3 || a.N % BN || a.C % 32 || a.K != 9 * a.C) return -1;
    if (a.W < 16 || (BM % a.W && a.W % BM)) return -1;
    const dim3 grid(((a.M + BM - 1) / BM) * (a.N / BN));
    hipLaunchKernelGGL((rowgemm16_row3_kernel<EMODE, BM, BN>), grid, dim3(512), 0, s, a);
    return (int)hipGetLastError();
}

// tiles: 0 = 128x128, 2 stages (64 KB LDS, 2 blocks/CU); 2 = 256x128, 8 waves, 2 stages
// (96 KB); 4 = 256x256, 8 waves of 128x64, 2 stages (128 KB); 6 = 512x128, 8 waves of 128x64,
// 2 stages (160 KB); 19 / 20 = the tap-row halo kernel at 256x256 / 512x128
using T16_0 = Tile16<128, 128, 64, 64, 2, 2>;
using T16_2 = Tile16<256, 128, 64, 64, 2, 1>;
using T16_4 = Tile16<256, 256, 128, 64, 2, 1>;
using T16_6 = Tile16<512, 128, 128, 64, 2, 1>;
// (r06, not kept: 128x128 with three / four stages at one block per CU for the deep levels' small
// grids, config 4 -1.2 %, profiles/r06_c4_ab.txt)
#define ROWGEMM16_TILES(X) X(0, T16_0) X(2, T16_2) X(4, T16_4) X(6, T16_6)

template <int AMODE, int EMODE, class T>
static int rg16_go(const RowGemmArgs& a, hipStream_t s) {
    if (a.N % T::BN || a.C % T::BK || a.K % T::BK) return -1;
    if (EMODE == E_CONVT && (a.cout % T::BN)) return -1;
    const dim3 grid(((a.M + T::BM - 1) / T::BM) * (a.N / T::BN));
    hipLaunchKernelGGL((rowgemm16_kernel<AMODE, EMODE, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

template <int AMODE, int EMODE>
static int rg16_tile(const RowGemmArgs& a0, int tile, hipStream_t s) {
    RowGemmArgs a = a0;
    if (a.tgm < 0) {  // tile order: the group size for this tile's grid (two blocks per CU on tile 0)
        int bm = 0, bn = 0;
        if (rowgemm16_tile_dims(tile, &bm, &bn, nullptr) != 0) return -1;
        a.tgm = tile_group_auto(a.M, a.N, bm, bn, tile == 0 ? 64 : 32);
    }
    if (tile == 19 || tile == 20) {
        if constexpr (AMODE == G_CONV3)
            return tile == 19 ? rg16r3_go<EMODE, 256, 256>(a, s) : rg16r3_go<EMODE, 512, 128>(a, s);
        return -1;
    }
#define RG16_CASE(id, T) \
    if (tile == id) return rg16_go<AMODE, EMODE, T>(a, s);
    ROWGEMM16_TILES(RG16_CASE)
#undef RG16_CASE
    return -1;
}

// ------------------------------------------------------------------------------------
// Weight gradient on LDS-DMA bf16 operands: dW[m][n] = sum_p A'[p][m] * B'[p][n], the
// reduction over pixels p split into `splits` slices of pps pixels, each block writing its
// fp32 tile of slab[split] (k_slab_reduce sums the slices in fixed order).  A' = gather of
// the conv input's bf16 image (tap = m / CA), B' = the bf16 image of dz (G_IDENT) or of the
// ConvT output gradient (G_UP2, tap = n / CB).
//
// The MFMA wants 8 consecutive PIXELS of one channel per lane, while the images are
// pixel-major (NHWC).  LDS holds [BKP pixels][128 channels] (256-B rows, filled by
// global_load_lds: one wave-instruction = 4 pixel rows) and the operands are read with
// ds_read_b64_tr_b16, which hands lane i of each 16-lane group column i of a 4-row x
// 16-column block: two such reads give a lane channel c's pixels 8h .. 8h+7.  The 16-B
// chunk ch of pixel row r sits in slot ch ^ ((r & 3) << 2), so the four rows a group reads
// land in four different bank quarters (conflict-free per 32-lane half).
// ------------------------------------------------------------------------------------
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4;

// ds_read_b64_tr_b16 as inline asm: through the builtin, hipcc cannot tell the read from
// the LDS-DMA writes still in flight and drains them (s_waitcnt vmcnt(0)) before every
// k-step.  An asm read is outside hipcc's wait bookkeeping, so the caller waits lgkmcnt
// itself and fences the MFMAs behind it with sched_barrier (cdna_hip_programming.md rule 18).
template <int OFF>
__device__ __forceinline__ short4v ds_tr16(unsigned addr) {
    short4v r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
    return r;
}

__device__ __forceinline__ unsigned lds_u32(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int BM_, int BN_, int WM_, int WN_, int BKP_, int S_, int OCC_>
struct WTile16 {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BKP = BKP_, S = S_, OCC = OCC_;
    static constexpr int WAVES = (BM / WM) * (BN / WN);
    static constexpr int THREADS = 64 * WAVES;
};

template <int AMODE, int BMODE, class T>
__global__ __launch_bounds__(T::THREADS, T::OCC) void wgrad16_kernel(WgradArgs p) {
    constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, BKP = T::BKP, S = T::S;
    constexpr int WAVES = T::WAVES, WAVES_N = BN / WN;
    constexpr int MT = WM / 32, NT = WN / 32;
    static_assert(BM % 128 == 0 && BN % 128 == 0 && BM <= 512 && BN <= 512, "pixel rows");
    constexpr int RA = 2 * BM, RBB = 2 * BN;   // bytes per pixel row of the A' / B' images
    constexpr int LA = RA / 16, LB = RBB / 16;  // lanes per pixel row in a DMA instruction
    constexpr int PA = 64 / LA, PB = 64 / LB;   // pixel rows per DMA instruction
    constexpr int AI = BKP / (PA * WAVES), BI = BKP / (PB * WAVES);  // DMA instructions per chunk
    static_assert(AI * PA * WAVES == BKP && BI * PB * WAVES == BKP, "loader shape");
    constexpr int GPC = AI + BI;
    constexpr int STAGE = BKP * (RA + RBB);
    __shared__ __attribute__((aligned(1024))) char smem[STAGE * S];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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
    const int pbeg = split * p.pps;
    const int pend = min(pbeg + p.pps, p.P);
    const int nk = (pend - pbeg + BKP - 1) / BKP;

    // loader: instruction j of this wave fills pixel rows (j * WAVES + wave) * PA .. (A');
    // lane l -> row l / LA, slot l % LA holding global chunk slot ^ ((row & 3) << 2)
    const int lra = lane / LA, lrb = lane / LB;
    const uint16_t* a16 = (const uint16_t*)p.a;
    const uint16_t* b16 = (const uint16_t*)p.b;
    const uint16_t* zero = (const uint16_t*)p.zero16;

    auto issue = [&](int kc, int st) {
        const int pc = pbeg + kc * BKP;
        char* base = smem + st * STAGE;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            const int row = (j * WAVES + wave) * PA + lra;
            const int gcha = ((lane % LA) ^ ((row & 3) << 2)) * 8;
            const int pix = pc + row;
            const bool in = pix < pend;
            const int m = in ? pix : pend - 1;
            bool valid;
            const Pix q = AMODE == G_IDENT ? Pix{0, 0, 0} : decode_fast(m, H, W, rH, rW);
            const int src = gather_src<AMODE>(tapA, m, q, H, W, valid);
            const uint16_t* g = (valid && in) ? a16 + (size_t)src * p.lda + ca0 + gcha : zero;
            glds16(g, base + (j * WAVES + wave) * 1024);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int row = (j * WAVES + wave) * PB + lrb;
            const int gchb = ((lane % LB) ^ ((row & 3) << 2)) * 8;
            const int pix = pc + row;
            const bool in = pix < pend;
            const int m = in ? pix : pend - 1;
            bool valid;
            const Pix q = BMODE == G_IDENT ? Pix{0, 0, 0} : decode_fast(m, H, W, rH, rW);
            const int src = gather_src<BMODE>(tapB, m, q, H, W, valid);
            const uint16_t* g = (valid && in) ? b16 + (size_t)src * p.ldb + cb0 + gchb : zero;
            glds16(g, base + BKP * RA + (j * WAVES + wave) * 1024);
        }
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // transposed-read addresses (bytes within a stage, k-step 0, read t = 0): lane l of
    // group g = l / 16 supplies row 8 (g >> 1) + q, columns 16 (g & 1) + 4 p (l % 16 = 4q + p)
    const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const int trow = 8 * (g >> 1) + qq;  // + 4 t + 16 kk: (row & 3) stays qq
    int aoff[MT], boff[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int col = wm * WM + mt * 32 + 16 * (g & 1) + 4 * pp;
        aoff[mt] = trow * RA + (((col >> 3) ^ (qq << 2)) << 4) + ((col >> 2) & 1) * 8;
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = wn * WN + nt * 32 + 16 * (g & 1) + 4 * pp;
        boff[nt] = BKP * RA + trow * RBB + (((col >> 3) ^ (qq << 2)) << 4) + ((col >> 2) & 1) * 8;
    }

#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nk) issue(s, s);
    for (int kc = 0; kc < nk; ++kc) {
        if (kc + S - 1 < nk) issue(kc + S - 1, (kc + S - 1) % S);
        const int ahead = min(S - 1, nk - 1 - kc);
        if constexpr (S >= 3) {
            if (ahead >= 2) wait_vm<2 * GPC>();
            else if (ahead == 1) wait_vm<GPC>();
            else wait_vm<0>();
        } else {
            if (ahead >= 1) wait_vm<GPC>();
            else wait_vm<0>();
        }
        block_barrier();
        const unsigned sb = lds_u32(smem) + (kc % S) * STAGE;
        // fragments of k-step kk (A then B; two transposed reads each), software-pipelined:
        // the reads of kk + 1 are in flight while the MFMAs of kk run
        short4v fa[2][MT][2], fb[2][NT][2];
        auto load = [&](auto KK) {
            constexpr int kk = decltype(KK)::value, set = kk & 1;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                fa[set][mt][0] = ds_tr16<kk * 16 * RA>(sb + aoff[mt]);
                fa[set][mt][1] = ds_tr16<kk * 16 * RA + 4 * RA>(sb + aoff[mt]);
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                fb[set][nt][0] = ds_tr16<kk * 16 * RBB>(sb + boff[nt]);
                fb[set][nt][1] = ds_tr16<kk * 16 * RBB + 4 * RBB>(sb + boff[nt]);
            }
        };
        auto mma = [&](auto KK) {
            constexpr int set = decltype(KK)::value & 1;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[mt][nt] = mfma32_bf16(*(const bf16x8*)fa[set][mt], *(const bf16x8*)fb[set][nt],
                                              acc[mt][nt]);
        };
        static_assert(BKP == 64, "four k-steps per chunk");
        constexpr int RD = 2 * (MT + NT);  // reads per k-step
        load(std::integral_constant<int, 0>{});
        load(std::integral_constant<int, 1>{});
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 0>{});
        __builtin_amdgcn_sched_barrier(0);
        load(std::integral_constant<int, 2>{});
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 1>{});
        __builtin_amdgcn_sched_barrier(0);
        load(std::integral_constant<int, 3>{});
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 2>{});
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 3>{});
        block_barrier();
    }

    const int li = lane & 31, lh = lane >> 5;
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
// Tap-row weight gradient (3x3 convs, W % 64 == 0): one block computes the three dx taps of
// one tap row dy for a 128-channel (ci) x 128-channel (co) tile over its split's pixels.  A
// 64-pixel chunk never crosses an image row (pps and W are multiples of 64), so the A'
// operands of the three taps are the SAME 66 halo pixel rows of source row y + dy - 1
// (columns x0 - 1 .. x0 + 64, zero outside the image), read at row offsets dx = 0, 1, 2;
// the one-tap kernel streams a shifted copy of them per tap.  LDS stage: [68 halo rows][128
// ci] + [64 pixel rows][128 co] bf16 (33 KB; 3 stages, one block of 8 waves per CU).  Wave
// tile 32 (ci) x 64 (co) per tap: 6 accumulators, 10 transposed reads per 6 MFMAs.
// Same operands, pixel chunks, k-steps and split partition as wgrad16_kernel, so every
// element's sum is the same sequence of MFMAs: bit-identical to the one-tap tiles.
// ------------------------------------------------------------------------------------
// (r05-r06, removed: four waves of 32 x 128 per tap at 3 stages, and 3 stages of this tile --
// bit-identical, slower)
template <int S>
__global__ __launch_bounds__(512, 1) void wgrad16_row3_kernel(WgradArgs p) {
    constexpr int BM = 128, BN = 128, WM = 32, WN = 64, BKP = 64;
    constexpr int WAVES_N = BN / WN, WAVES = (BM / WM) * WAVES_N;  // 4 x 2 / 4 x 1 waves
    constexpr int NT = WN / 32;
    constexpr int RA = 2 * BM, RBB = 2 * BN;    // 256-B pixel rows
    constexpr int LA = RA / 16, LB = RBB / 16;  // 16 lanes per row in a DMA instruction
    constexpr int PA = 64 / LA, PB = 64 / LB;   // 4 rows per DMA instruction
    constexpr int AROWS = BKP + 2;              // halo rows
    constexpr int NA = (AROWS + PA - 1) / PA;   // 17 A' pieces
    constexpr int AI = (NA + WAVES - 1) / WAVES;  // 3 (the third: wave 0 only)
    constexpr int BI = BKP / (PB * WAVES);      // 2
    static_assert(BI * PB * WAVES == BKP && (AI - 1) * WAVES < NA, "loader shape");
    constexpr int AST = NA * PA * RA;           // A' bytes per stage (68 rows)
    constexpr int STAGE = AST + BKP * RBB;
    __shared__ __attribute__((aligned(1024))) char smem[STAGE * S];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int tiles_n = p.Nw / BN, tiles_m = p.CA / BM;
    int idx = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tn = idx % tiles_n;
    idx /= tiles_n;
    const int tm = idx % tiles_m;
    idx /= tiles_m;
    const int dy = idx % 3;
    const int split = idx / 3;
    const int ca0 = tm * BM, cb0 = tn * BN;
    const int H = p.H, W = p.W;
    const float rH = 1.f / (float)H, rW = 1.f / (float)W;
    const int pbeg = split * p.pps;
    const int pend = min(pbeg + p.pps, p.P);
    const int nk = (pend - pbeg + BKP - 1) / BKP;
    const bool a3 = (AI - 1) * WAVES + wave < NA;  // this wave issues a third A' piece

    const int lra = lane / LA, lrb = lane / LB;
    const uint16_t* a16 = (const uint16_t*)p.a;
    const uint16_t* b16 = (const uint16_t*)p.b;
    const uint16_t* zero = (const uint16_t*)p.zero16;

    auto issue = [&](int kc, int st) {
        const int pc = pbeg + kc * BKP;  // first output pixel of the chunk (one image row)
        const Pix q = decode_fast(pc, H, W, rH, rW);
        const int yy = q.y + dy - 1;
        const bool rowok = yy >= 0 && yy < H;
        const int srow = (q.img * H + yy) * W;  // source row's first pixel (when rowok)
        char* base = smem + st * STAGE;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            if (j == AI - 1 && !a3) continue;
            const int row = (j * WAVES + wave) * PA + lra;  // halo row: column x0 - 1 + row
            const int gcha = ((lane % LA) ^ ((row & 3) << 2)) * 8;
            const int xx = q.x - 1 + row;
            const bool ok = rowok && row < AROWS && xx >= 0 && xx < W;
            const uint16_t* g = ok ? a16 + (size_t)(srow + xx) * p.lda + ca0 + gcha : zero;
            glds16(g, base + (j * WAVES + wave) * 1024);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int row = (j * WAVES + wave) * PB + lrb;
            const int gchb = ((lane % LB) ^ ((row & 3) << 2)) * 8;
            const int pix = pc + row;
            const uint16_t* g = pix < pend ? b16 + (size_t)pix * p.ldb + cb0 + gchb : zero;
            glds16(g, base + AST + (j * WAVES + wave) * 1024);
        }
    };

    f32x16 acc[3][NT];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // transposed reads (wgrad16_kernel's addressing): lane l of group g = l / 16 supplies row
    // 8 (g >> 1) + qq (+ 4 t + 16 kk, + dx for tap dx), columns 16 (g & 1) + 4 pp
    const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    int aoff[3], boff[NT];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
        const int row = 8 * (g >> 1) + qq + dx;  // (row & 3) == ((qq + dx) & 3) for every kk, t
        const int col = wm * WM + 16 * (g & 1) + 4 * pp;
        aoff[dx] = row * RA + (((col >> 3) ^ ((row & 3) << 2)) << 4) + ((col >> 2) & 1) * 8;
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int row = 8 * (g >> 1) + qq;
        const int col = wn * WN + nt * 32 + 16 * (g & 1) + 4 * pp;
        boff[nt] = AST + row * RBB + (((col >> 3) ^ (qq << 2)) << 4) + ((col >> 2) & 1) * 8;
    }

#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nk) issue(s, s);
    for (int kc = 0; kc < nk; ++kc) {
        // one barrier per chunk: chunks kc + 1 .. kc + S - 2 may stay in flight; then
        // restage the buffer every wave finished reading in chunk kc - 1.  (r04: issuing
        // before the wait and a second barrier after the MFMAs, the same bits, 2 % slower.)
        const int ahead = min(S - 2, nk - 1 - kc);
        if (a3) {
            constexpr int G = AI + BI;
            if (ahead >= 2) wait_vm<2 * G>();
            else if (ahead == 1) wait_vm<G>();
            else wait_vm<0>();
        } else {
            constexpr int G = AI - 1 + BI;
            if (ahead >= 2) wait_vm<2 * G>();
            else if (ahead == 1) wait_vm<G>();
            else wait_vm<0>();
        }
        block_barrier();
        if (kc + S - 1 < nk) issue(kc + S - 1, (kc + S - 1) % S);
        const unsigned sb = lds_u32(smem) + (kc % S) * STAGE;
        short4v fa[2][3][2], fb[2][NT][2];
        auto load = [&](auto KK) {
            constexpr int kk = decltype(KK)::value, set = kk & 1;
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                fa[set][dx][0] = ds_tr16<kk * 16 * RA>(sb + aoff[dx]);
                fa[set][dx][1] = ds_tr16<kk * 16 * RA + 4 * RA>(sb + aoff[dx]);
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                fb[set][nt][0] = ds_tr16<kk * 16 * RBB>(sb + boff[nt]);
                fb[set][nt][1] = ds_tr16<kk * 16 * RBB + 4 * RBB>(sb + boff[nt]);
            }
        };
        auto mma = [&](auto KK) {
            constexpr int set = decltype(KK)::value & 1;
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[dx][nt] = mfma32_bf16(*(const bf16x8*)fa[set][dx], *(const bf16x8*)fb[set][nt],
                                              acc[dx][nt]);
        };
        static_assert(BKP == 64, "four k-steps per chunk");
        constexpr int RD = 2 * (3 + NT);  // reads per k-step
        load(std::integral_constant<int, 0>{});
        load(std::integral_constant<int, 1>{});
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 0>{});
        __builtin_amdgcn_sched_barrier(0);
        load(std::integral_constant<int, 2>{});
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 1>{});
        __builtin_amdgcn_sched_barrier(0);
        load(std::integral_constant<int, 3>{});
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 2>{});
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 3>{});
    }

    const int li = lane & 31, lh = lane >> 5;
    float* slab = p.slab + (size_t)split * p.Mw * p.Nw;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = (3 * dy + dx) * p.CA + ca0 + wm * WM + (r & 3) + 8 * (r >> 2) + 4 * lh;
                const int n = cb0 + wn * WN + nt * 32 + li;
                slab[(size_t)m * p.Nw + n] = acc[dx][nt][r];
            }
}

// ------------------------------------------------------------------------------------
// (r06) The tap-row bf16 weight gradient on v_mfma_f32_16x16x32_bf16 (tiles 6 / 7).  The x3
// weight gradient's r05 lessons carried over: the 16x16x32 shape (the chip holds a higher clock
// on it at equal cycles per FLOP, MI355X_MICROARCH.md DVFS item 7) and, tile 7, the re-read
// stagger of x3_wsched = 10.
//   Same block (128 ci x 128 co x the three dx taps of one dy, 8 waves of 32 ci x 64 co per tap),
//   same halo staging (68 + 64 rows of 256 B per 64-pixel chunk) and split partition as
//   wgrad16_row3_kernel; per chunk two k-steps of 32 pixels, a wave's 32 x 64 tap tile as 2 x 4
//   blocks of 16 x 16 (24 MFMAs per k-step, 20 transposed reads).  Lane l of group g = l / 16
//   supplies the k values 8 g .. 8 g + 7 = pixel rows 4 g + qq (first transposed read) and
//   16 + 4 g + qq (second), the same rows for A' and B', column l & 15 of its block.
//   LDS swizzle: 16-B slot s of pixel row r holds global chunk s ^ ((r & 7) << 1): a 32-lane half
//   reads 32 B of eight consecutive rows (A': rows shifted by dx), which then fall on eight
//   different 32-B bank sections.
//   LAG (tile 7): four stages with the DMA two chunks ahead, so a chunk's stage stays intact one
//   chunk longer; waves 4..7 (each sharing a SIMD with wave w - 4) run each chunk's second k-step
//   at the start of the next chunk, re-reading its fragments from that stage, so their matrix
//   work opens the segment while their partner waits for its first fragments.
//   The sums run 32 products per MFMA step (16 on the 32x32x16 kernel): f32 rounding apart from
//   tiles 3..5, bit-identical between 6 and 7 (same MFMAs in the same order per accumulator).
//   SEGW (r06): W % 64 == 0 (64), or the deep levels' W = 32 / 16 (config 4's 32^2 level and
//   16^2 bottleneck, which ran the one-tap kernel): a 64-pixel chunk is then 64 / W whole image
//   rows (H W % 64 == 0, so it never leaves its image), staged as 64 / W halo segments of W + 2
//   pixels at a segment stride of 40 / 24 rows -- multiples of 8, so the row & 7 swizzle of a
//   fragment read is the same in every segment -- and a k-step's 32 pixels read segment rows
//   (one segment of 32, or two of 16).
template <int S, bool LAG, int SEGW = 64>
__global__ __launch_bounds__(512, 1) void wgrad16_row3_m16_kernel(WgradArgs p) {
    constexpr int BM = 128, BN = 128, WM = 32, WN = 64, BKP = 64;
    constexpr int WAVES_N = BN / WN, WAVES = (BM / WM) * WAVES_N;  // 4 x 2
    constexpr int RA = 2 * BM, RBB = 2 * BN;     // 256-B pixel rows
    constexpr int LA = RA / 16, LB = RBB / 16;   // 16 lanes per row in a DMA instruction
    constexpr int PA = 64 / LA, PB = 64 / LB;    // 4 rows per DMA instruction
    static_assert(SEGW == 64 || SEGW == 32 || SEGW == 16, "segment width");
    constexpr int NSEG = BKP / SEGW;             // image rows per chunk (W < 64)
    constexpr int SS = SEGW == 64 ? BKP : SEGW == 32 ? 40 : 24;  // halo segment stride (rows)
    constexpr int AROWS = (NSEG - 1) * SS + SEGW + 2;            // halo rows: 66 / 74 / 90
    constexpr int NA = (AROWS + PA - 1) / PA;    // 17 / 19 / 23 A' pieces
    constexpr int AI = (NA + WAVES - 1) / WAVES;  // 3 (the third: wave 0 only)
    constexpr int BI = BKP / (PB * WAVES);       // 2
    static_assert(BI * PB * WAVES == BKP && (AI - 1) * WAVES < NA, "loader shape");
    constexpr int AST = NA * PA * RA;            // A' bytes per stage (68 rows)
    constexpr int STAGE = AST + BKP * RBB;
    constexpr int DIST = LAG ? 2 : S - 1;        // chunks the DMA runs ahead
    static_assert(!LAG || S == 4, "the stagger reads a stage one chunk after its own");
    static_assert(DIST <= S - 1 && DIST >= 1, "stages");
    __shared__ __attribute__((aligned(1024))) char smem[STAGE * S];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int tiles_n = p.Nw / BN, tiles_m = p.CA / BM;
    int idx = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tn = idx % tiles_n;
    idx /= tiles_n;
    const int tm = idx % tiles_m;
    idx /= tiles_m;
    const int dy = idx % 3;
    const int split = idx / 3;
    const int ca0 = tm * BM, cb0 = tn * BN;
    const int H = p.H, W = p.W;
    const float rH = 1.f / (float)H, rW = 1.f / (float)W;
    const int pbeg = split * p.pps;
    const int pend = min(pbeg + p.pps, p.P);
    const int nk = (pend - pbeg + BKP - 1) / BKP;
    const bool a3 = (AI - 1) * WAVES + wave < NA;  // this wave issues a third A' piece
    const bool lag = LAG && wave >= 4;

    const int lra = lane / LA, lrb = lane / LB;
    const uint16_t* a16 = (const uint16_t*)p.a;
    const uint16_t* b16 = (const uint16_t*)p.b;
    const uint16_t* zero = (const uint16_t*)p.zero16;
    auto swz = [](int sl, int row) { return sl ^ ((row & 7) << 1); };

    auto issue = [&](int kc, int st) {
        const int pc = pbeg + kc * BKP;  // first output pixel of the chunk (one image row / NSEG rows)
        const Pix q = decode_fast(pc, H, W, rH, rW);
        char* base = smem + st * STAGE;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            if (j == AI - 1 && !a3) continue;
            const int row = (j * WAVES + wave) * PA + lra;  // halo row
            const int gcha = swz(lane % LA, row) * 8;
            // segment sg (image row q.y + sg), column xx of halo row `row` (segment offset - 1)
            const int sg = SEGW == 64 ? 0 : row / SS;
            const int xx = (SEGW == 64 ? q.x : 0) - 1 + row - sg * SS;
            const int yy = q.y + sg + dy - 1;
            const bool ok = row < AROWS && sg < NSEG && xx >= 0 && xx < W && yy >= 0 && yy < H;
            const uint16_t* g = ok ? a16 + (size_t)((q.img * H + yy) * W + xx) * p.lda + ca0 + gcha : zero;
            glds16(g, base + (j * WAVES + wave) * 1024);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int row = (j * WAVES + wave) * PB + lrb;
            const int gchb = swz(lane % LB, row) * 8;
            const int pix = pc + row;
            const uint16_t* g = pix < pend ? b16 + (size_t)pix * p.ldb + cb0 + gchb : zero;
            glds16(g, base + AST + (j * WAVES + wave) * 1024);
        }
    };

    f32x4 acc[3][2][4];
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int b = 0; b < 8; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[d][b >> 2][b & 3][r] = 0.f;

    const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const int trow = 4 * g + qq;
    int aoff[3][2], boff[4];
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
        const int col = wm * WM + 16 * bm + 4 * pp;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const int row = trow + dx;  // (+ 16, + 32 kk: the same row & 7)
            aoff[dx][bm] = row * RA + (swz(col >> 3, row) << 4) + ((col >> 2) & 1) * 8;
        }
    }
#pragma unroll
    for (int bn = 0; bn < 4; ++bn) {
        const int col = wn * WN + 16 * bn + 4 * pp;
        boff[bn] = AST + trow * RBB + (swz(col >> 3, trow) << 4) + ((col >> 2) & 1) * 8;
    }
    struct Frag {
        short4v a[3][2][2], b[4][2];
    };
    // the fragments of k-step KK (pixels 32 KK ..) of the stage at byte sb
    auto load = [&](Frag& f, unsigned sb, auto KK) {
        constexpr int kk = decltype(KK)::value;
#pragma unroll
        for (int bn = 0; bn < 4; ++bn) {
            f.b[bn][0] = ds_tr16<kk * 32 * RBB>(sb + boff[bn]);
            f.b[bn][1] = ds_tr16<kk * 32 * RBB + 16 * RBB>(sb + boff[bn]);
        }
        // halo rows of the k-step's two 16-pixel halves (the same row & 7 as kk = 0's)
        constexpr int R0 = SEGW == 64 ? kk * 32 : SEGW == 32 ? kk * SS : 2 * kk * SS;
        constexpr int R1 = SEGW == 16 ? R0 + SS : R0 + 16;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int bm = 0; bm < 2; ++bm) {
                f.a[dx][bm][0] = ds_tr16<R0 * RA>(sb + aoff[dx][bm]);
                f.a[dx][bm][1] = ds_tr16<R1 * RA>(sb + aoff[dx][bm]);
            }
    };
    auto mma = [&](const Frag& f) {
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int bm = 0; bm < 2; ++bm)
#pragma unroll
                for (int bn = 0; bn < 4; ++bn)
                    acc[dx][bm][bn] = mfma16_bf16(*(const bf16x8*)f.a[dx][bm], *(const bf16x8*)f.b[bn],
                                                  acc[dx][bm][bn]);
    };
    // a k-step takes 20 transposed reads; lgkmcnt counts at most 15, so the first k-step's wait
    // leaves 15 of the second's 20 in flight
    constexpr int RD = 15;
    using K0 = std::integral_constant<int, 0>;
    using K1 = std::integral_constant<int, 1>;
    const unsigned sbase = lds_u32(smem);

#pragma unroll
    for (int s = 0; s < DIST; ++s)
        if (s < nk) issue(s, s);
    // one chunk loop per role (separately register-allocated paths)
    auto run = [&](auto LAGC) {
        constexpr bool LG = decltype(LAGC)::value;
        for (int kc = 0; kc < nk; ++kc) {
            // one barrier per chunk: chunks kc + 1 .. kc + DIST - 1 may stay in flight; then
            // restage the slot every wave finished reading (chunk kc - 1 without the stagger,
            // kc - 2 with it)
            const int ahead = min(DIST - 1, nk - 1 - kc);
            if (a3) {
                constexpr int G = AI + BI;
                if (ahead >= 2) wait_vm<2 * G>();
                else if (ahead == 1) wait_vm<G>();
                else wait_vm<0>();
            } else {
                constexpr int G = AI - 1 + BI;
                if (ahead >= 2) wait_vm<2 * G>();
                else if (ahead == 1) wait_vm<G>();
                else wait_vm<0>();
            }
            block_barrier();
            if (kc + DIST < nk) issue(kc + DIST, (kc + DIST) % S);
            const unsigned sb = sbase + (kc % S) * STAGE;
            Frag f0, f1;
            if constexpr (LG) {  // chunk kc - 1's second k-step, then this chunk's first
                if (kc > 0) {
                    load(f1, sbase + ((kc + S - 1) % S) * STAGE, K1{});
                    load(f0, sb, K0{});
                    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
                    __builtin_amdgcn_sched_barrier(0);
                    mma(f1);
                    __builtin_amdgcn_sched_barrier(0);
                } else {
                    load(f0, sb, K0{});
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                mma(f0);
            } else {
                load(f0, sb, K0{});
                load(f1, sb, K1{});
                asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
                __builtin_amdgcn_sched_barrier(0);
                mma(f0);
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                mma(f1);
            }
        }
        if (LG && nk > 0) {  // the last chunk's second k-step (its stage is not restaged any more)
            Frag f1;
            load(f1, sbase + ((nk - 1) % S) * STAGE, K1{});
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            mma(f1);
        }
    };
    if (lag) run(std::true_type{});
    else run(std::false_type{});

    float* slab = p.slab + (size_t)split * p.Mw * p.Nw;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
            for (int bn = 0; bn < 4; ++bn)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m = (3 * dy + dx) * p.CA + ca0 + wm * WM + 16 * bm + 4 * g + i;
                    const int n = cb0 + wn * WN + 16 * bn + (lane & 15);
                    slab[(size_t)m * p.Nw + n] = acc[dx][bm][bn][i];
                }
}

// wgrad16 tiles: 0 = 128x128, 64 pixels per stage, 2 stages (64 KB, 2 blocks/CU);
// 2 = 256x256, 8 waves of 128x64, 2 stages (128 KB, 1 block/CU)
// (r01-r02, not kept: 3-stage 128x128, 256x128 / 128x256 at 3 stages)
using W16_0 = WTile16<128, 128, 64, 64, 64, 2, 2>;
using W16_2 = WTile16<256, 256, 128, 64, 64, 2, 1>;
#define WGRAD16G_TILES(X) X(0, W16_0) X(2, W16_2)

template <int AMODE, int BMODE, class T>
static int wg16_go(const WgradArgs& a, hipStream_t s) {
    if (a.Mw % T::BM || a.Nw % T::BN || a.CA % T::BM || a.CB % T::BN || a.pps % T::BKP) return -1;
    const dim3 grid((a.Mw / T::BM) * (a.Nw / T::BN) * a.splits);
    hipLaunchKernelGGL((wgrad16_kernel<AMODE, BMODE, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

}  // namespace

int wgrad16g_tile_dims(int tile, int* bm, int* bn, int* stages) {
    if (tile == 4 || tile == 7) {  // tap-row: 128 x 128 per tap, three taps per block, 4 stages
        *bm = *bn = 128;
        if (stages) *stages = 4;
        return 0;
    }
#define WG16_DIMS(id, T)          \
    if (tile == id) {             \
        *bm = T::BM;              \
        *bn = T::BN;              \
        if (stages) *stages = T::S; \
        return 0;                 \
    }
    WGRAD16G_TILES(WG16_DIMS)
#undef WG16_DIMS
    return -1;
}

int rowgemm16_tile_dims(int tile, int* bm, int* bn, int* stages) {
    if (tile == 19 || tile == 20) {  // tap-row halo 256x256 / 512x128
        *bm = tile == 19 ? 256 : 512;
        *bn = tile == 19 ? 256 : 128;
        if (stages) *stages = 2;
        return 0;
    }
#define RG16_DIMS(id, T)          \
    if (tile == id) {             \
        *bm = T::BM;              \
        *bn = T::BN;              \
        if (stages) *stages = T::S; \
        return 0;                 \
    }
    ROWGEMM16_TILES(RG16_DIMS)
#undef RG16_DIMS
    return -1;
}

// The combinations of the BN -> ReLU network (models/mod.py): conv forward (E_STATS),
// conv dgrad (E_STORE / E_STORE_BN), ConvT forward (E_CONVT), ConvT dgrad (G_UP2, E_STORE_BN).
int launch_rowgemm16(const RowGemmArgs& a, int tile, hipStream_t s) {
    if (a.M < 1 || a.K != gather_taps(a.amode) * a.C || !a.a16 || !a.bt16 || !a.zero16) return -1;
    if (a.ascale || a.acoef || a.arelu) return -1;  // operands arrive prepared (k_to_bf16)
    if ((a.emode == E_STORE_BN) != (a.ey != nullptr)) return -1;
    if ((a.escale != nullptr) != (a.eshift != nullptr)) return -1;
    if (a.amode == G_CONV3 && a.emode == E_STATS) return rg16_tile<G_CONV3, E_STATS>(a, tile, s);
    if (a.amode == G_CONV3 && a.emode == E_STORE) return rg16_tile<G_CONV3, E_STORE>(a, tile, s);
    if (a.amode == G_CONV3 && a.emode == E_STORE_BN) return rg16_tile<G_CONV3, E_STORE_BN>(a, tile, s);
    if (a.amode == G_IDENT && a.emode == E_CONVT) return rg16_tile<G_IDENT, E_CONVT>(a, tile, s);
    if (a.amode == G_UP2 && a.emode == E_STORE_BN) return rg16_tile<G_UP2, E_STORE_BN>(a, tile, s);
    return -1;
}

// Weight gradient from bf16 images: a / b point at uint16 images [pixels][lda] /
// [pixels][ldb] (aoff / boff must be 0: the images are dense), zero16 at a zeroed page.
// 3x3 conv (A' G_CONV3, B' G_IDENT) and ConvT (A' G_IDENT, B' G_UP2); no bias column sums.
int launch_wgrad16(const WgradArgs& a, int tile, hipStream_t s) {
    if (a.aoff || a.boff || a.ascale || a.bcoef || a.bias_slab || !a.zero16 || a.P < 1) return -1;
    if (tile == 4 || tile == 7) {  // tap-row kernel: 3x3 conv layers, W % 64 == 0 (4: 32x32x16, 4 LDS
                                   // stages; 7: 16x16x32 with the re-read stagger, r06, and also
                                   // W = 32 / 16 with H W % 64 == 0)
        const bool deep = tile == 7 && (a.W == 32 || a.W == 16) && (a.H * a.W) % 64 == 0;
        if (a.amode != G_CONV3 || a.bmode != G_IDENT || a.Mw != 9 * a.CA || a.Nw != a.CB ||
            a.CA % 128 || a.CB % 128 || (a.W % 64 && !deep) || a.pps % 64 || a.P % 64)
            return -1;
        const dim3 grid((a.CA / 128) * 3 * (a.Nw / 128) * a.splits);
        if (tile == 7 && a.W == 32)
            hipLaunchKernelGGL((wgrad16_row3_m16_kernel<4, true, 32>), grid, dim3(512), 0, s, a);
        else if (tile == 7 && a.W == 16)
            hipLaunchKernelGGL((wgrad16_row3_m16_kernel<4, true, 16>), grid, dim3(512), 0, s, a);
        else if (tile == 7)
            hipLaunchKernelGGL((wgrad16_row3_m16_kernel<4, true>), grid, dim3(512), 0, s, a);
        else
            hipLaunchKernelGGL((wgrad16_row3_kernel<4>), grid, dim3(512), 0, s, a);
        return (int)hipGetLastError();
    }
#define WG16G(AM, BMD)                                   \
    do {                                                 \
        if (tile == 0) return wg16_go<AM, BMD, W16_0>(a, s); \
        if (tile == 2) return wg16_go<AM, BMD, W16_2>(a, s); \
        return -1;                                       \
    } while (0)
    if (a.amode == G_CONV3 && a.bmode == G_IDENT) WG16G(G_CONV3, G_IDENT);
    if (a.amode == G_IDENT && a.bmode == G_UP2) WG16G(G_IDENT, G_UP2);
#undef WG16G
    return -1;
}
