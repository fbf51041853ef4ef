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

// block tile BM x BN, wave tile WM x WN, S LDS stages of 64 K each
template <int BM_, int BN_, int WM_, int WN_, int S_, int OCC_>
struct Tile16 {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, S = S_, OCC = OCC_;
    static constexpr int BK = 64;
    static constexpr int WAVES = (BM / WM) * (BN / WN);
    static constexpr int THREADS = 64 * WAVES;
};

template <int AMODE, int EMODE, class T>
__global__ __launch_bounds__(T::THREADS, T::OCC) void rowgemm16_kernel(RowGemmArgs p) {
    constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, S = T::S;
    constexpr int WAVES = T::WAVES, WAVES_N = BN / WN;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int AI = BM / (8 * WAVES), BI = BN / (8 * WAVES);  // DMA instructions per chunk
    static_assert(AI * 8 * WAVES == BM && BI * 8 * WAVES == BN, "loader shape");
    constexpr int GPC = AI + BI;
    constexpr int STAGE = (BM + BN) * 128;  // bytes
    constexpr int RED = 2 * (BM / WM) * BN * 8;  // epilogue scratch (f64 partials)
    constexpr int SMEM = STAGE * S > RED ? STAGE * S : RED;
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tile_m = bid / ntn, tile_n = bid - tile_m * ntn;
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    const int H = p.H, W = p.W, C = p.C, K = p.K;

    // loader rows: instruction j of this wave fills rows (j * WAVES + wave) * 8 .. + 7
    const int lr = lane >> 3, slot = lane & 7;
    Pix aq[AI];
    int am[AI], ach[AI];
    bool aok[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int r = (j * WAVES + wave) * 8 + lr;
        const int m = m0 + r;
        aok[j] = m < p.M;
        am[j] = aok[j] ? m : p.M - 1;
        aq[j] = decode(am[j], H, W);
        ach[j] = (slot ^ ((r >> 1) & 7)) * 8;
    }
    const uint16_t* bsrc[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int r = (j * WAVES + wave) * 8 + lr;
        bsrc[j] = p.bt16 + (size_t)(n0 + r) * K + (slot ^ ((r >> 1) & 7)) * 8;
    }
    const uint16_t* zero = (const uint16_t*)p.zero16;

    auto issue = [&](int kc, int st) {
        const int k0 = kc * 64;
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
        for (int j = 0; j < BI; ++j) glds16(bsrc[j] + k0, base + BM * 128 + (j * WAVES + wave) * 1024);
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
        aro[mt] = r * 128;
        afx[mt] = (r >> 1) & 7;
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int r = BM + wn * WN + nt * 32 + li;
        bro[nt] = r * 128;
        bfx[nt] = ((r - BM) >> 1) & 7;
    }

    const int nk = K / 64;
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nk) issue(s, s);
    for (int kc = 0; kc < nk; ++kc) {
        if (kc + S - 1 < nk) issue(kc + S - 1, (kc + S - 1) % S);
        // chunks issued after kc that may stay in flight
        const int ahead = min(S - 1, nk - 1 - kc);
        if constexpr (S >= 4) {
            if (ahead >= 3) wait_vm<3 * GPC>();
            else if (ahead == 2) wait_vm<2 * GPC>();
            else if (ahead == 1) wait_vm<GPC>();
            else wait_vm<0>();
        } else if constexpr (S == 3) {
            if (ahead >= 2) wait_vm<2 * GPC>();
            else if (ahead == 1) wait_vm<GPC>();
            else wait_vm<0>();
        } else {
            if (ahead >= 1) wait_vm<GPC>();
            else wait_vm<0>();
        }
        block_barrier();
        const char* base = smem + (kc % S) * STAGE;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
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
    row_epilogue<EMODE, BM, BN, WM, WN>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)smem);
}

// tiles: 0 = 128x128, 2 stages (64 KB LDS, 2 blocks/CU); 1 = 128x128, 3 stages (96 KB);
// 2 = 256x128, 8 waves, 2 stages (96 KB); 3 = 128x128, 4 stages (128 KB)
using T16_0 = Tile16<128, 128, 64, 64, 2, 2>;
using T16_1 = Tile16<128, 128, 64, 64, 3, 1>;
using T16_2 = Tile16<256, 128, 64, 64, 2, 1>;
using T16_3 = Tile16<128, 128, 64, 64, 4, 1>;
#define ROWGEMM16_TILES(X) X(0, T16_0) X(1, T16_1) X(2, T16_2) X(3, T16_3)

template <int AMODE, int EMODE, class T>
static int rg16_go(const RowGemmArgs& a, hipStream_t s) {
    if (a.N % T::BN || a.C % 64 || a.K % 64) return -1;
    if (EMODE == E_CONVT && (a.cout % T::BN)) return -1;
    const dim3 grid(((a.M + T::BM - 1) / T::BM) * (a.N / T::BN));
    hipLaunchKernelGGL((rowgemm16_kernel<AMODE, EMODE, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

template <int AMODE, int EMODE>
static int rg16_tile(const RowGemmArgs& a, int tile, hipStream_t s) {
#define RG16_CASE(id, T) \
    if (tile == id) return rg16_go<AMODE, EMODE, T>(a, s);
    ROWGEMM16_TILES(RG16_CASE)
#undef RG16_CASE
    return -1;
}

}  // namespace

int rowgemm16_tile_dims(int tile, int* bm, int* bn) {
#define RG16_DIMS(id, T) \
    if (tile == id) {    \
        *bm = T::BM;     \
        *bn = T::BN;     \
        return 0;        \
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
