// f32 row GEMM with both operands staged by LDS-DMA (global_load_lds_dwordx4) on gfx950.
//
// Same contract, K order and numerics as rowgemm_kernel / rowgemm_pipe_kernel (f32 operands,
// v_mfma_f32_32x32x2_f32, K in 32-wide (tap, channel) chunks, the same in-chunk lane
// permutation, the same epilogues): the three kernels store identical bits.
//
// The register-staged kernels spend the wave's issue slots on the loads' address
// arithmetic, the BN-affine / padding commit and its ds_writes, and wait for each chunk's
// loads before committing it (tools/pipe_exp.hip: +10 % with the loop's global loads
// removed).  Here no instruction sits between HBM and LDS: each lane's 16 B go straight
// into the LDS image (per-lane source address, lane-linear destination, the layout and
// XOR swizzle of kernels_gemm16.hip: an f32 chunk row is 32 x 4 B = 128 B, the byte
// geometry of a 64-deep bf16 row), S - 1 chunks ahead.  Padding taps and rows past M read
// a zeroed 16-B page.  The BN prologue of the forward A operand moves to the MFMA side:
// after its ds_read, each A fragment (4 channels of one row) gets fma(x, scale, shift),
// the ReLU on the channels below arelu and the padding select, from a per-block LDS copy
// of scale / shift and a per-row 9-bit tap mask -- the values rowgemm_kernel's commit
// writes, so the products are the same.
#include <type_traits>

#include "gemm_common.h"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)lds_wave_base, 16, 0, 0);
}

// s_barrier with compiler fences (the builtin alone does not order memory operations)
__device__ __forceinline__ void block_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ds_read_b128 as inline asm: a compiler-visible LDS read makes hipcc drain every LDS-DMA in
// flight first (s_waitcnt vmcnt(0): it cannot tell which stage a DMA writes), which
// serialised the prefetch.  An asm read is outside hipcc's wait bookkeeping, so the caller
// counts lgkmcnt itself and fences the consumers with sched_barrier.
template <int OFF>
__device__ __forceinline__ f32x4 ds_read16(unsigned addr) {
    f32x4 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
    return r;
}

template <int N>
__device__ __forceinline__ void wait_lgkm() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int BM_, int BN_, int WM_, int WN_, int S_, int OCC_>
struct DmaTile {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, S = S_, OCC = OCC_, BK = 32;
    static constexpr int WAVES = (BM / WM) * (BN / WN);
    static constexpr int THREADS = 64 * WAVES;
};

constexpr int DMA_MAXC = 1024;  // channels of the per-block scale / shift copy

template <int AMODE, int AOP, int EMODE, class T>
__global__ __launch_bounds__(T::THREADS, T::OCC) void rowgemm_dma_kernel(RowGemmArgs p) {
    static_assert(AOP != OP_DZ, "OP_DZ operands run on rowgemm_kernel");
    constexpr bool AFFINE = AOP == OP_AFFINE || AOP == OP_AFFINE_RELU;
    constexpr bool ARELU = AOP == OP_AFFINE_RELU;
    constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, S = T::S, BK = T::BK;
    constexpr int WAVES = T::WAVES, WAVES_N = BN / WN;
    constexpr int MT = WM / 32, NT = WN / 32, KG = BK / 8;
    constexpr int RB = 4 * BK;    // bytes per LDS row (128)
    constexpr int LPR = RB / 16;  // 16-B slots per row (8)
    constexpr int RPI = 64 / LPR; // rows per DMA wave-instruction (8)
    constexpr int RPB = 256 / RB; // rows per 256-B bank row (2)
    auto swz = [](int r) { return (r / RPB) & (LPR - 1); };
    constexpr int AI = BM / (RPI * WAVES), BI = BN / (RPI * WAVES);
    static_assert(AI * RPI * WAVES == BM && BI * RPI * WAVES == BN, "loader shape");
    constexpr int GPC = AI + BI;  // DMA instructions per chunk per wave
    static_assert(S == 2 || S == 3, "two or three LDS stages");
    constexpr int STAGE = (BM + BN) * RB;
    static_assert(STAGE >= 2 * (BM / 64) * BN * 8, "epilogue scratch");
    // The two stages are separate LDS objects and the chunk loop is unrolled by two, so
    // every ds_read and every DMA names its stage statically: hipcc's wait insertion can then
    // tell a read of one stage from the DMA still in flight into the other and waits only
    // for the former (with one array it drained every DMA before each read, the prefetch
    // included).
    __shared__ __attribute__((aligned(1024))) char st0[STAGE];
    __shared__ __attribute__((aligned(1024))) char st1[STAGE];
    __shared__ __attribute__((aligned(1024))) char st2[S == 3 ? STAGE : 16];
    __shared__ __attribute__((aligned(16))) float sct[AFFINE ? 2 * DMA_MAXC : 4];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tile_m = bid / ntn, tile_n = bid - tile_m * ntn;
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    const int H = p.H, W = p.W, C = p.C, K = p.K;

    if constexpr (AFFINE) {  // per-block copy of the BN affine of the A channels
        for (int i = tid; i < C; i += T::THREADS) {
            sct[i] = p.ascale[i];
            sct[DMA_MAXC + i] = p.ashift[i];
        }
        __syncthreads();  // before any DMA is in flight (its fence would drain them)
    }

    // DMA rows: instruction j of this wave fills rows (j * WAVES + wave) * RPI + lane / LPR
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
        ach[j] = (slot ^ swz(r)) * 4;
    }
    const float* bsrc[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int r = (j * WAVES + wave) * RPI + lr;
        bsrc[j] = p.bt + (size_t)(n0 + r) * K + (slot ^ swz(r)) * 4;
    }
    const float* zero = (const float*)p.zero16;
    const float* abase = p.a + p.aoff;

    auto issue = [&](int kc, char* base) {
        const int k0 = kc * BK;
        const int tap = k0 / C;
        const int c0 = k0 - tap * C;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            bool valid;
            const int src = gather_src<AMODE>(tap, am[j], aq[j], H, W, valid);
            const float* g = (valid && aok[j]) ? abase + (size_t)src * p.lda + c0 + ach[j] : zero;
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
    int aro[MT], afx[MT], bro[NT], bfx[NT];
    unsigned tmask[MT];  // AFFINE: bit t = tap t of this lane's MFMA row reads inside the image
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int r = wm * WM + mt * 32 + li;
        aro[mt] = r * RB;
        afx[mt] = swz(r);
        unsigned bits = 0;
        const int m = m0 + r;
        if (m < p.M) {
            const Pix q = decode(m, H, W);
            if constexpr (AMODE == G_CONV3) {
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int yy = q.y + t / 3 - 1, xx = q.x + t % 3 - 1;
                    bits |= ((yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)) ? (1u << t) : 0u;
                }
            } else {
                bits = 0x1ffu;
            }
        }
        tmask[mt] = bits;
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int r = wn * WN + nt * 32 + li;
        bro[nt] = (BM + r) * RB;
        bfx[nt] = swz(r);
    }

    const int nk = K / BK;
    // per-lane LDS byte offsets of the MFMA fragments of k-group kg (slot (2 kg + lh) ^ swizzle)
    unsigned aofs[KG][MT], bofs[KG][NT];
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) aofs[kg][mt] = aro[mt] + (((kg * 2 + lh) ^ afx[mt]) << 4);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) bofs[kg][nt] = bro[nt] + (((kg * 2 + lh) ^ bfx[nt]) << 4);
    }
    const unsigned sct_lane = lds_addr(sct) + lh * 16;
    constexpr int RD = MT + NT + (AFFINE ? 2 : 0);  // asm reads per k-group
    auto compute = [&](int kc, const char* base) {
        const int k0 = kc * BK;
        const int tap = k0 / C, c0 = k0 - tap * C;
        const unsigned sb = lds_addr(base);
        const unsigned sa = sct_lane + c0 * 4;
        f32x4 af[2][MT], bf[2][NT], sc[2], sh[2];
        // fragments of k-group kg into register set kg & 1 (in flight until the counted wait)
        auto load = [&](auto KG_) {
            constexpr int kg = decltype(KG_)::value, set = kg & 1;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) af[set][mt] = ds_read16<0>(sb + aofs[kg][mt]);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) bf[set][nt] = ds_read16<0>(sb + bofs[kg][nt]);
            if constexpr (AFFINE) {
                sc[set] = ds_read16<kg * 32>(sa);
                sh[set] = ds_read16<DMA_MAXC * 4 + kg * 32>(sa);
            }
        };
        auto mma = [&](auto KG_) {
            constexpr int kg = decltype(KG_)::value, set = kg & 1;
            if constexpr (AFFINE) {  // rowgemm_kernel's commit arithmetic, on the fragment
                const int ch = c0 + kg * 8 + lh * 4;  // the fragment's 4 channels
                const bool rl = ARELU && ch < p.arelu;
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const bool keep = (tmask[mt] >> tap) & 1u;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float t = __builtin_fmaf(af[set][mt][j], sc[set][j], sh[set][j]);
                        const float u = rl ? fmaxf(t, 0.f) : t;
                        af[set][mt][j] = keep ? u : 0.f;
                    }
                }
            }
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[mt][nt] = mfma32(af[set][mt][s], bf[set][nt][s], acc[mt][nt]);
        };
        static_assert(KG == 4, "four k-groups per chunk");
        load(std::integral_constant<int, 0>{});
        load(std::integral_constant<int, 1>{});
        wait_lgkm<RD>();
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 0>{});
        __builtin_amdgcn_sched_barrier(0);
        load(std::integral_constant<int, 2>{});
        wait_lgkm<RD>();
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 1>{});
        __builtin_amdgcn_sched_barrier(0);
        load(std::integral_constant<int, 3>{});
        wait_lgkm<RD>();
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 2>{});
        __builtin_amdgcn_sched_barrier(0);
        wait_lgkm<0>();
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 3>{});
        // every wave's reads of this stage have returned (waited above) before any restages it
        block_barrier();
    };
    if constexpr (S == 3) {
        // chunk c in stage c % 3; chunks kc + 1 and kc + 2 fly during chunk kc's MFMAs (kc + 2
        // restages the image chunk kc - 1 left, free since compute's closing barrier)
        issue(0, st0);
        if (nk > 1) issue(1, st1);
        auto stage = [&](int kc, const char* cur, char* nxt2) {
            if (kc + 2 < nk) {
                issue(kc + 2, nxt2);
                wait_vm<2 * GPC>();
            } else if (kc + 1 < nk) {
                wait_vm<GPC>();
            } else {
                wait_vm<0>();
            }
            block_barrier();
            compute(kc, cur);
        };
        for (int kc = 0; kc < nk; kc += 3) {
            stage(kc, st0, st2);
            if (kc + 1 >= nk) break;
            stage(kc + 1, st1, st0);
            if (kc + 2 >= nk) break;
            stage(kc + 2, st2, st1);
        }
        row_epilogue<EMODE, BM, BN, WM, WN>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)st0);
        return;
    }
    // even chunks in st0, odd chunks in st1; chunk kc+1's DMA flies during chunk kc's MFMAs
    issue(0, st0);
    for (int kc = 0; kc < nk; kc += 2) {
        if (kc + 1 < nk) {
            issue(kc + 1, st1);
            wait_vm<GPC>();
        } else {
            wait_vm<0>();
        }
        block_barrier();
        compute(kc, st0);
        if (kc + 1 >= nk) break;
        if (kc + 2 < nk) {
            issue(kc + 2, st0);
            wait_vm<GPC>();
        } else {
            wait_vm<0>();
        }
        block_barrier();
        compute(kc + 1, st1);
    }
    row_epilogue<EMODE, BM, BN, WM, WN>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)st0);
}

using DmaTile0 = DmaTile<128, 128, 64, 64, 2, 2>;  // 2 stages, 64 KB (+8 KB affine table)
using DmaTile1 = DmaTile<128, 64, 64, 32, 2, 2>;
// N = 64 with two chunks in flight: 3 stages of 24 KB, two blocks per CU
using DmaTile2 = DmaTile<128, 64, 64, 32, 3, 2>;

template <int AMODE, int AOP, int EMODE, class T>
static int dma_go(const RowGemmArgs& a, hipStream_t s) {
    if (a.N % T::BN || a.K % T::BK || a.C % T::BK) return -1;
    if (EMODE == E_CONVT && (a.cout % T::BN)) return -1;
    const dim3 grid(((a.M + T::BM - 1) / T::BM) * (a.N / T::BN));
    hipLaunchKernelGGL((rowgemm_dma_kernel<AMODE, AOP, EMODE, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

template <int AMODE, int AOP, int EMODE>
static int dma_tile(const RowGemmArgs& a, int tile, hipStream_t s) {
    if (tile == 0) return dma_go<AMODE, AOP, EMODE, DmaTile0>(a, s);
    if (tile == 1) return dma_go<AMODE, AOP, EMODE, DmaTile1>(a, s);
    if (tile == 2) return dma_go<AMODE, AOP, EMODE, DmaTile2>(a, s);
    return -1;
}

}  // namespace

int rowgemm_dma_ok(const RowGemmArgs& a) {
    if (a.bt == nullptr || a.bt16 != nullptr || a.acoef != nullptr || a.zero16 == nullptr) return 0;
    if (a.K % 32 || a.C % 32 || a.N % 64) return 0;
    if (a.ascale != nullptr && a.C > DMA_MAXC) return 0;
    return 1;
}

// tile: 0 = 128x128, 1 = 128x64 (two LDS stages each)
int launch_rowgemm_dma(const RowGemmArgs& a, int tile, hipStream_t s) {
    if (!rowgemm_dma_ok(a) || a.M < 1 || a.K != gather_taps(a.amode) * a.C) return -1;
    const bool aff = a.ascale != nullptr;
    if ((a.emode == E_STORE_BN || a.emode == E_RESID) != (a.ey != nullptr)) return -1;
    if ((a.escale != nullptr) != (a.eshift != nullptr) || (a.arelu && !aff)) return -1;
    if (a.emode == E_RESID && !a.escale) return -1;
    if (a.amode == G_CONV3 && a.emode == E_BIAS_RELU_STATS)
        return aff ? dma_tile<G_CONV3, OP_AFFINE, E_BIAS_RELU_STATS>(a, tile, s)
                   : dma_tile<G_CONV3, OP_PLAIN, E_BIAS_RELU_STATS>(a, tile, s);
    if (a.amode == G_CONV3 && a.emode == E_STATS) {
        if (a.arelu) return dma_tile<G_CONV3, OP_AFFINE_RELU, E_STATS>(a, tile, s);
        if (!aff) return dma_tile<G_CONV3, OP_PLAIN, E_STATS>(a, tile, s);
        return -1;
    }
    if (aff) {
        if (a.amode == G_IDENT && a.emode == E_CONVT)
            return a.arelu ? dma_tile<G_IDENT, OP_AFFINE_RELU, E_CONVT>(a, tile, s)
                           : dma_tile<G_IDENT, OP_AFFINE, E_CONVT>(a, tile, s);
        return -1;
    }
    if (a.amode == G_CONV3) {
        if (a.emode == E_STORE) return dma_tile<G_CONV3, OP_PLAIN, E_STORE>(a, tile, s);
        if (a.emode == E_STORE_BN) return dma_tile<G_CONV3, OP_PLAIN, E_STORE_BN>(a, tile, s);
        if (a.emode == E_ADD) return dma_tile<G_CONV3, OP_PLAIN, E_ADD>(a, tile, s);
    }
    if (a.amode == G_UP2) {
        if (a.emode == E_STORE_BN) return dma_tile<G_UP2, OP_PLAIN, E_STORE_BN>(a, tile, s);
        if (a.emode == E_STORE) return dma_tile<G_UP2, OP_PLAIN, E_STORE>(a, tile, s);
    }
    if (a.amode == G_IDENT) {
        if (a.emode == E_CONVT) return dma_tile<G_IDENT, OP_PLAIN, E_CONVT>(a, tile, s);
        if (a.emode == E_RESID) return dma_tile<G_IDENT, OP_PLAIN, E_RESID>(a, tile, s);
        if (a.emode == E_STORE) return dma_tile<G_IDENT, OP_PLAIN, E_STORE>(a, tile, s);
    }
    return -1;
}
