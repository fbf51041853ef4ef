// Software-pipelined f32 row GEMM (implicit 3x3 / ConvT / 1x1 conv) for gfx950.
//
// Same contract and numerics as rowgemm_kernel (kernels_gemm.hip, f32 path): C[m][n] =
// sum_k A[m][k] * Bt[n][k] on v_mfma_f32_32x32x2_f32, K walked in 32-wide chunks in the same
// order with the same in-chunk lane permutation, the same prologue (BN affine, ReLU, zero
// padding) and the same epilogues (row_epilogue), so the two kernels store identical bits.
//
// What differs is the schedule.  rowgemm_kernel runs each chunk as [global loads] [MFMAs]
// [commit VALU + ds_write] [barrier]: the address arithmetic and the commit execute while the
// wave's matrix pipe is idle, which measured as 78 % MFMA-busy however many waves share a SIMD
// (co-resident waves fall into the same phase).  Here one wave keeps its pipe fed:
//   * the whole chunk's MFMA operands (KG x (MT + NT) f32x4) are pulled from LDS into
//     registers right after the chunk's barrier, so the LDS image is free while the MFMAs run;
//   * two LDS images: during chunk kc's MFMAs the wave commits chunk kc+1 (loaded into
//     registers one chunk earlier) into the other image and issues chunk kc+2's global loads;
//     one barrier per chunk;
//   * __builtin_amdgcn_sched_group_barrier interleaves that work between the MFMAs, and the
//     next chunk's ds_reads with the last MFMAs of this one (the loop body is branch-free:
//     the tail chunks re-load / re-commit the last chunk into the image nobody reads);
//   * the gather keeps per-row 9-bit tap masks and 32-bit byte offsets, so a chunk costs a
//     handful of VALU per loaded row (uniform chunk bases live in SGPRs).
// Host contract (launch_rowgemm_pipe): f32 operands, K % 32 == C % 32 == 0, N % BN == 0, and
// every A / Bt byte offset below 2^31.
#include "gemm_common.h"

namespace {

// DEPTH: chunks whose global loads are in flight in registers (2 = issued two chunks before
// their commit; costs one more stage of registers).  SWZ: unpadded, XOR-swizzled LDS rows
// (see the kernel), 8/9 of the padded images' space.
template <int BM_, int BN_, int WM_, int WN_, int OCC_, int DEPTH_ = 1, bool SWZ_ = false>
struct PipeTile {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = 32, OCC = OCC_;
    static constexpr int DEPTH = DEPTH_;
    static constexpr bool SWZ = SWZ_;
    static constexpr int WAVES = (BM / WM) * (BN / WN);
    static constexpr int THREADS = 64 * WAVES;
};

// XP: speed-of-light ablations for tools/pipe_exp.hip only (bit 0 drops the loop barrier,
// 1 the loop's global loads, 2 its ds_writes, 3 its ds_reads, 4 the epilogue); the library
// instantiates XP = 0.
template <int AMODE, int AOP, int EMODE, class T, int XP = 0>
__global__ __launch_bounds__(T::THREADS, T::OCC) void rowgemm_pipe_kernel(RowGemmArgs p) {
    static_assert(AOP != OP_DZ, "OP_DZ operands run on rowgemm_kernel");
    constexpr bool AFFINE = AOP == OP_AFFINE || AOP == OP_AFFINE_RELU;
    constexpr bool ARELU = AOP == OP_AFFINE_RELU;
    constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, BK = T::BK;
    constexpr int NTH = T::THREADS, WAVES_N = BN / WN;
    // LDS images: rows of BK + 4 f32 (the padding makes the 16-lane groups of ds_read_b128
    // conflict-free), or, SWZ, unpadded 128-B rows with 16-B chunk c of row r in slot
    // c ^ ((r >> 1) & 7): the groups (rows r0 + {0-3, 12-15, 20-27} or {4-11, 16-19, 28-31},
    // one chunk) again hit 16 distinct slots, in 8/9 of the space (the 128x64 tile then fits
    // three blocks per CU).  The XOR costs the 128x128 tile ~0.8 % (A/B on one box), so only
    // the three-block tiles use it.
    constexpr bool SWZ = T::SWZ;
    constexpr int LDK = SWZ ? BK : BK + 4;
    auto swz = [](int r) { return SWZ ? (r >> 1) & 7 : 0; };
    constexpr int MT = WM / 32, NT = WN / 32, KG = BK / 8;
    constexpr int F4R = BK / 4, RPP = NTH / F4R;
    constexpr int AP = BM / RPP, BP = BN / RPP;
    static_assert(AP * RPP == BM && BP * RPP == BN, "loader shape");
    constexpr int IMG = (BM + BN) * LDK;
    __shared__ __attribute__((aligned(16))) float smem[2 * IMG];
    static_assert(2 * IMG * 4 >= (BM / 64) * 2 * BN * 8, "epilogue scratch (row_epilogue)");

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ntn = p.N / BN;
    const int ntiles = ((p.M + BM - 1) / BM) * ntn;  // = gridDim.x
    const int H = p.H, W = p.W, C = p.C;

    // loader rows: lrow + i * RPP, 16 B (4 channels) per lane, F4R lanes per 128-B row
    const int lrow = tid / F4R, lc4 = tid % F4R;
    int tile_m, m0, n0;
    unsigned aoff[AP];  // byte offset of the row's tap-0 source (+ the lane's 4 channels)
    unsigned tmask[AP]; // bit t: tap t reads inside the image (and the row is inside M)
    unsigned boff[BP];
    // tile of block v and its gather offsets / tap masks
    auto setup = [&](int v) {
        const int bid = p.xcd ? xcd_remap(v, ntiles) : v;
        tile_m = bid / ntn;
        const int tile_n = bid - tile_m * ntn;
        m0 = tile_m * BM;
        n0 = tile_n * BN;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const int m = m0 + lrow + i * RPP;
            const bool ok = m < p.M;
            const int mm = ok ? m : p.M - 1;
            const Pix q = decode(mm, H, W);
            int base = mm;
            unsigned bits = 0;
            if constexpr (AMODE == G_CONV3) {
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const int yy = q.y + t / 3 - 1, xx = q.x + t % 3 - 1;
                    bits |= ((yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)) ? (1u << t) : 0u;
                }
            } else if constexpr (AMODE == G_UP2) {
                base = (q.img * 2 * H + 2 * q.y) * (2 * W) + 2 * q.x;
                bits = 0xfu;
            } else {
                bits = 1u;
            }
            tmask[i] = ok ? bits : 0u;
            aoff[i] = (unsigned)(base * p.lda + lc4 * 4) * 4u;
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) boff[i] = (unsigned)((n0 + lrow + i * RPP) * p.K + lc4 * 4) * 4u;
    };
    setup(blockIdx.x);
    const char* abytes = (const char*)(p.a + p.aoff);

    // one chunk's global loads, held in registers until its commit
    struct Stage {
        f32x4 ra[AP], rb[BP], rsc, rsh;
        unsigned vbits;
        bool rrelu;
    };

    // global loads of chunk kc into registers (raw; the commit applies the prologue)
    auto issue = [&](Stage& st, int kc) {
        const int k0 = kc * BK;
        const int tap = k0 / C;
        const int c0 = k0 - tap * C;
        int doff;  // row offset of this tap relative to tap 0 (uniform)
        if constexpr (AMODE == G_CONV3)
            doff = (tap / 3 - 1) * W + (tap % 3 - 1);
        else if constexpr (AMODE == G_UP2)
            doff = (tap >> 1) * (2 * W) + (tap & 1);
        else
            doff = 0;
        const unsigned dbytes = (unsigned)(doff * p.lda) * 4u;
        const char* ab = abytes + (size_t)c0 * 4;
        if constexpr (AFFINE) {
            st.rsc = *(const f32x4*)(p.ascale + c0 + lc4 * 4);
            st.rsh = *(const f32x4*)(p.ashift + c0 + lc4 * 4);
            if constexpr (ARELU) st.rrelu = c0 + lc4 * 4 < p.arelu;
        }
        st.vbits = 0;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            const unsigned v = (tmask[i] >> tap) & 1u;
            st.vbits |= v << i;
            // invalid taps read the row's own pixel (always in range) and are zeroed at commit
            const unsigned off = aoff[i] + (v ? dbytes : 0u);
            st.ra[i] = *(const f32x4*)(ab + off);
        }
        const char* bb = (const char*)(p.bt + k0);
#pragma unroll
        for (int i = 0; i < BP; ++i) st.rb[i] = *(const f32x4*)(bb + boff[i]);
    };
    auto commit = [&](const Stage& st, int buf) {
        float* as = smem + buf * IMG;
        float* bs = as + BM * LDK;
#pragma unroll
        for (int i = 0; i < AP; ++i) {
            f32x4 v = st.ra[i];
            if constexpr (AFFINE) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float t = __builtin_fmaf(v[j], st.rsc[j], st.rsh[j]);
                    v[j] = (ARELU && st.rrelu) ? fmaxf(t, 0.f) : t;
                }
            }
            const bool keep = (st.vbits >> i) & 1u;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = keep ? v[j] : 0.f;
            const int r = lrow + i * RPP;
            *(f32x4*)&as[r * LDK + ((lc4 ^ swz(r)) << 2)] = v;
        }
#pragma unroll
        for (int i = 0; i < BP; ++i) {
            const int r = lrow + i * RPP;
            *(f32x4*)&bs[r * LDK + ((lc4 ^ swz(r)) << 2)] = st.rb[i];
        }
    };

    const int li = lane & 31, lh = lane >> 5;
    const int sl = swz(li);  // = swz(row) of every operand row (row bases are multiples of 32)
    static_assert(WM % 32 == 0 && WN % 32 == 0, "operand row bases");
    f32x4 af[KG][MT], bf[KG][NT];
    // MFMA operands of k-group kg (8 k) of the chunk in image buf
    auto read_kg = [&](int buf, int kg) {
        const float* as = smem + buf * IMG;
        const float* bs = as + BM * LDK;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
            af[kg][mt] = *(const f32x4*)&as[(wm * WM + mt * 32 + li) * LDK + (((2 * kg + lh) ^ sl) << 2)];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
            bf[kg][nt] = *(const f32x4*)&bs[(wn * WN + nt * 32 + li) * LDK + (((2 * kg + lh) ^ sl) << 2)];
    };

    f32x16 acc[MT][NT];
    auto mfma_kg = [&](int kg) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[mt][nt] = mfma32(af[kg][mt][s], bf[kg][nt][s], acc[mt][nt]);
    };

    constexpr int NMF = 4 * MT * NT;              // MFMAs per k-group
    constexpr int NDSW = AP + BP;                 // commit ds_writes
    constexpr int NVM = AP + BP + (AFFINE ? 2 : 0);  // global loads per chunk
    constexpr int NDSR = MT + NT;                 // ds_reads per k-group
    static_assert(NDSW <= NMF && NVM <= NMF, "schedule shape");

    const int nk = p.K / BK;
    auto clampk = [&](int j) { return j < nk ? j : nk - 1; };
    constexpr int D = T::DEPTH;  // chunks in flight in registers (1 or 2)
    Stage S[D];
    issue(S[0], 0);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    commit(S[0], 0);
    // the prologue's chunks are issued in order, each behind a scheduling fence: loads of
    // chunk 2 hoisted between chunk 1's would make the loop's first commit wait for (almost)
    // every load in flight -- the wait counts are merged over the loop entry and back edge
#pragma unroll
    for (int d = 0; d < D; ++d) {
        __builtin_amdgcn_sched_barrier(0);
        issue(S[(1 + d) % D], clampk(1 + d));
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
#pragma unroll
    for (int kg = 0; kg < KG; ++kg) read_kg(0, kg);
    // Per chunk kc (registers hold its operands; the stages hold chunks kc+1 .. kc+D):
    //   A: k-group 0 MFMAs | commit chunk kc+1 into image nb          -> barrier
    //   B: k-group 1 MFMAs | ds_read next k-group 0, issue chunk kc+1+D into the freed stage
    //   C, D: k-groups 2, 3 | ds_read next k-groups 1, 2
    //   E: ds_read next k-group 3 (lands under the next chunk's phase A)
    // sched_barrier(0) fences keep each phase's reads behind the MFMAs that free their
    // registers.  Tail chunks re-load / re-commit the last chunk into the image nobody reads.
    auto body = [&](int kc, Stage& st) {
        const int nb = (kc + 1) & 1;
        if constexpr (!(XP & 4)) commit(st, nb);
        mfma_kg(0);
#pragma unroll
        for (int i = 0; i < NMF; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU
            if (i < NDSW) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // DS write
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(XP & 1)) __syncthreads();
        if constexpr (!(XP & 8)) read_kg(nb, 0);
        if constexpr (!(XP & 2)) issue(st, clampk(kc + 1 + D));
        mfma_kg(1);
        __builtin_amdgcn_sched_group_barrier(0x100, NDSR, 0);  // DS read
#pragma unroll
        for (int i = 0; i < NMF; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // VALU
            if (i < NVM) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kg = 2; kg < KG; ++kg) {
            if constexpr (!(XP & 8)) read_kg(nb, kg - 1);
            mfma_kg(kg);
#pragma unroll
            for (int i = 0; i < NMF; ++i) {
                if (i < NDSR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (!(XP & 8)) read_kg(nb, KG - 1);
    };
    // chunk kc commits stage (kc + 1) % D: unrolled by D so the stage is static
    int kc = 0;
    for (; kc + D <= nk; kc += D) {
#pragma unroll
        for (int d = 0; d < D; ++d) body(kc + d, S[(1 + d) % D]);
    }
    if constexpr (D == 2) {
        if (kc < nk) body(kc, S[1]);
    }

    if constexpr (XP & 16) {  // keep the accumulators live: one store per lane
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) v += acc[i][j][r];
        p.out[(size_t)blockIdx.x * NTH + tid] = v;
    } else {
        row_epilogue<EMODE, BM, BN, WM, WN>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, smem);
    }
}

// 4 waves of 64x64 (74 KB LDS) / 4 waves of 64x32 (N = 64 outputs), loading two chunks ahead
// (r02-r03 tiles 0 / 1 loaded one chunk ahead: 1-2 % slower, removed in r06)
using PipeTile2 = PipeTile<128, 128, 64, 64, 2, 2>;
using PipeTile3 = PipeTile<128, 64, 64, 32, 2, 2>;
// N = 64 at three blocks per CU (48 KB of LDS each): a third resident block to overlap the
// epilogues of the short-K (576) level-0 GEMMs; 5 loads two chunks ahead
using PipeTile4 = PipeTile<128, 64, 64, 32, 3, 1, true>;
using PipeTile5 = PipeTile<128, 64, 64, 32, 3, 2, true>;
// (r02-r03, not kept: 128x256 / 256x128 eight-wave tiles for the short-K ConvT GEMMs, 256x64
// on 64x64 wave tiles, persistent blocks walking several tiles -- 0-12 % slower or neutral,
// DESIGN.md §3)

template <int AMODE, int AOP, int EMODE, class T>
static int pipe_go(const RowGemmArgs& a, hipStream_t s) {
    // (E_CONVT: the epilogue maps every column to its (a, b, co) on its own, so a tile may
    // span several taps -- the 128x256 tile covers all four of a 64-channel ConvT)
    if (a.N % T::BN || a.K % T::BK || a.C % T::BK) return -1;
    if (EMODE == E_CONVT && (a.cout % T::BN) && (T::BN % a.cout)) return -1;
    const dim3 grid(((a.M + T::BM - 1) / T::BM) * (a.N / T::BN));
    hipLaunchKernelGGL((rowgemm_pipe_kernel<AMODE, AOP, EMODE, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

template <int AMODE, int AOP, int EMODE>
static int pipe_tile(const RowGemmArgs& a, int tile, hipStream_t s) {
    if (tile == 2) return pipe_go<AMODE, AOP, EMODE, PipeTile2>(a, s);
    if (tile == 3) return pipe_go<AMODE, AOP, EMODE, PipeTile3>(a, s);
    if (tile == 4) return pipe_go<AMODE, AOP, EMODE, PipeTile4>(a, s);
    if (tile == 5) return pipe_go<AMODE, AOP, EMODE, PipeTile5>(a, s);
    return -1;
}

}  // namespace

int rowgemm_pipe_ok(const RowGemmArgs& a) {
    if (a.bt == nullptr || a.bt16 != nullptr || a.acoef != nullptr) return 0;
    if (a.K % 32 || a.C % 32 || a.N % 64) return 0;
    // 32-bit byte offsets: every A source row (G_UP2 reads a grid 4x the rows) and Bt
    const long long arows = a.amode == G_UP2 ? 4LL * a.M : (long long)a.M;
    if ((arows * a.lda + a.C) * 4 >= (1LL << 31)) return 0;
    if ((long long)a.N * a.K * 4 >= (1LL << 31)) return 0;
    return 1;
}

// tile: 2 = 128x128, 3 = 128x64 (loading two chunks ahead), 4 / 5 = 128x64 at three blocks per
// CU (one / two chunks ahead)
int launch_rowgemm_pipe(const RowGemmArgs& a, int tile, hipStream_t s) {
    if (!rowgemm_pipe_ok(a) || a.M < 1 || a.K != gather_taps(a.amode) * a.C) return -1;
    const bool aff = a.ascale != nullptr;
    if ((a.emode == E_STORE_BN || a.emode == E_RESID) != (a.ey != nullptr)) return -1;
    if ((a.escale != nullptr) != (a.eshift != nullptr) || (a.arelu && !aff)) return -1;
    if (a.emode == E_RESID && !a.escale) return -1;
    if (a.amode == G_CONV3 && a.emode == E_BIAS_RELU_STATS)
        return aff ? pipe_tile<G_CONV3, OP_AFFINE, E_BIAS_RELU_STATS>(a, tile, s)
                   : pipe_tile<G_CONV3, OP_PLAIN, E_BIAS_RELU_STATS>(a, tile, s);
    if (a.amode == G_CONV3 && a.emode == E_STATS) {
        if (a.arelu) return pipe_tile<G_CONV3, OP_AFFINE_RELU, E_STATS>(a, tile, s);
        if (!aff) return pipe_tile<G_CONV3, OP_PLAIN, E_STATS>(a, tile, s);
        return -1;
    }
    if (aff) {
        if (a.amode == G_IDENT && a.emode == E_CONVT)
            return a.arelu ? pipe_tile<G_IDENT, OP_AFFINE_RELU, E_CONVT>(a, tile, s)
                           : pipe_tile<G_IDENT, OP_AFFINE, E_CONVT>(a, tile, s);
        return -1;
    }
    if (a.amode == G_CONV3) {
        if (a.emode == E_STORE) return pipe_tile<G_CONV3, OP_PLAIN, E_STORE>(a, tile, s);
        if (a.emode == E_STORE_BN) return pipe_tile<G_CONV3, OP_PLAIN, E_STORE_BN>(a, tile, s);
        if (a.emode == E_ADD) return pipe_tile<G_CONV3, OP_PLAIN, E_ADD>(a, tile, s);
    }
    if (a.amode == G_UP2) {
        if (a.emode == E_STORE_BN) return pipe_tile<G_UP2, OP_PLAIN, E_STORE_BN>(a, tile, s);
        if (a.emode == E_STORE) return pipe_tile<G_UP2, OP_PLAIN, E_STORE>(a, tile, s);
    }
    if (a.amode == G_IDENT) {
        if (a.emode == E_CONVT) return pipe_tile<G_IDENT, OP_PLAIN, E_CONVT>(a, tile, s);
        if (a.emode == E_RESID) return pipe_tile<G_IDENT, OP_PLAIN, E_RESID>(a, tile, s);
        if (a.emode == E_STORE) return pipe_tile<G_IDENT, OP_PLAIN, E_STORE>(a, tile, s);
    }
    return -1;
}
