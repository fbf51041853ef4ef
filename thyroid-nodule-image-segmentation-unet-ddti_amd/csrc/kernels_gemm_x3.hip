// fp32 row GEMM on the bf16 matrix cores through an exact three-way operand split.
//
// gfx950 runs f32-input MFMAs (v_mfma_f32_32x32x2_f32) at 1/16 of the bf16 rate.  Every f32
// value v splits EXACTLY into three bf16 pieces, v = h + m + l:
//   h = bf16_rne(v), m = bf16_rne(v - h), l = bf16_rne(v - h - m)
// (each difference is exact in f32; h holds the top 8 significand bits, m the next 8, l the
// last 8, so nothing is left over for normal v).  A product then is the sum of the nine
// piece products; the six kept here,
//   Ah*Bh + Ah*Bm + Am*Bh + Ah*Bl + Am*Bm + Al*Bh,
// drop Am*Bl, Al*Bm, Al*Bl: with |m| <= 2^-8 |a|, |l| <= 2^-16 |a| they total at most
// 2^-24 + 2^-24 + 2^-32 ~ 2^-23 |a b| (worst case; the unit roundoff of one f32 operation is
// 2^-24, and the split accumulators below make the K-long sum ~3x MORE accurate than the f32
// MFMA kernels' in practice, profiles/r04_x3_probe_splitacc.txt).  Range edges (huge, inf,
// NaN, subnormal pieces): x3_split.h.  Each piece product is exact in the MFMA (8 x 8 significand bits)
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
// LDS image per stage: [BM rows][192 B] (A) then [BN rows][192 B] (B, at the A region's
// whole-KB end); 16-B slot s of plane q of row r (counted within its region) holds global
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

// the same with the five small products in their own accumulator (split accumulation: the
// large one then takes one rounding per 16 products)
__device__ __forceinline__ void mfma_x3s(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16& hi,
                                         f32x16& lo) {
    lo = mfma32_bf16(a[2], b[0], lo);
    lo = mfma32_bf16(a[1], b[1], lo);
    lo = mfma32_bf16(a[0], b[2], lo);
    lo = mfma32_bf16(a[1], b[0], lo);
    lo = mfma32_bf16(a[0], b[1], lo);
    hi = mfma32_bf16(a[0], b[0], hi);
}

// the six products of one 16x16x32 block (the same pieces and order; 32 k per instruction)

__device__ __forceinline__ void mfma_x3s16(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4& hi, f32x4& lo) {
    lo = mfma16_bf16(a[2], b[0], lo);
    lo = mfma16_bf16(a[1], b[1], lo);
    lo = mfma16_bf16(a[0], b[2], lo);
    lo = mfma16_bf16(a[1], b[0], lo);
    lo = mfma16_bf16(a[0], b[1], lo);
    hi = mfma16_bf16(a[0], b[0], hi);
}

template <int BM_, int BN_, int WM_, int WN_, int S_, int OCC_, int SA_ = 0>
struct TileX3 {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, S = S_, OCC = OCC_, SA = SA_;
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
    // DMA instructions per wave and chunk: every wave issues the same count; rows past BM /
    // BN (when a region is not a whole number of instructions per wave) read the zero page
    constexpr int AI = (BM * RB + 1024 * WAVES - 1) / (1024 * WAVES);
    constexpr int BI = (BN * RB + 1024 * WAVES - 1) / (1024 * WAVES);
    constexpr int AREG = AI * WAVES * 1024;  // bytes of the A region of a stage
    constexpr int DIST = S - 1;
    static_assert(DIST >= 1 && DIST <= 3, "stages");
    constexpr int STAGE = AREG + BI * WAVES * 1024;
    constexpr int RED = 2 * (BM / 64) * BN * 8;
    constexpr int SMEM = STAGE * S > RED ? STAGE * S : RED;
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    auto swz = [](int r) { return (r >> 2) & 3; };

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    int tile_m, tile_n;
    tile_mn(bid, (p.M + BM - 1) / BM, ntn, p.tgm, tile_m, tile_n);
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
        aok[j] = m < p.M && r < BM;
        am[j] = m < p.M ? m : p.M - 1;
        aq[j] = decode(am[j], H, W);
        ace[j] = (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(r)) << 3);
    }
    const uint16_t* bsrc[BI];
    bool bok[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int r = o / RB, w = o - r * RB;
        bok[j] = r < BN;
        bsrc[j] = p.bt16 + (size_t)(n0 + (bok[j] ? r : 0)) * rowb + (w >> 6) * 32 +
                  ((((w >> 4) & 3) ^ swz(r)) << 3);
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
            x3_dma16(bok[j] ? bsrc[j] + k0 * 3 : zero, base + AREG + (j * WAVES + wave) * 1024);
    };
    constexpr int GPC = AI + BI;  // DMA pieces per chunk

    constexpr int SA = T::SA;
    f32x16 acc[MT][NT], acl[SA ? MT : 1][SA ? NT : 1];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[i][j][r] = 0.f;
                if constexpr (SA) acl[i][j][r] = 0.f;
            }

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
        const int r = wn * WN + nt * 32 + li;
        bro[nt] = AREG + r * RB;
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
                for (int nt = 0; nt < NT; ++nt) {
                    if constexpr (SA) mfma_x3s(af[mt], bfr[nt], acc[mt][nt], acl[mt][nt]);
                    else acc[mt][nt] = mfma_x3(af[mt], bfr[nt], acc[mt][nt]);
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        x3_barrier();
    }
    if constexpr (SA) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[mt][nt] += acl[mt][nt];
    }
    row_epilogue<EMODE, BM, BN, WM, WN, true>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)smem);
}

// ------------------------------------------------------------------------------------
// Tap-row halo variant of the x3 3x3-conv GEMM (tile 4: 256 x 128, 8 waves of 64 x 64,
// W >= 16 a power of two).  The one-tap kernel restages the block's 256 A rows for each of the
// 9 taps, and its A gather is what holds it at ~0.55 of its MFMA-only speed (profiles/
// r04_x3_ablation.txt).  Here one stage holds the HALO of one tap row dy for one 32-channel
// group -- the block's image rows shifted by dy - 1, one extra pixel either side (ROWS x
// (SEG + 2) <= 288 x3 rows) -- and the three dx taps read A rows h + dx from it: a third of
// the A staging.  The x3 rows are 192 B, so the halo and the B rows of three taps (3 x 24 KB)
// cannot be double-buffered together; B streams per sub-step (dy, group, dx) through its own
// two-slot ring instead (2 x 56 KB halo + 2 x 24 KB B = 160 KB).  Per sub-step: wait for its
// B, barrier, issue B of the next sub-step (and, on dx = 0, the next group's halo) into the
// slot the previous sub-step read, 2 k-steps x 4 x 6 MFMAs per wave.
//   geometry (as rowgemm16_row3_kernel): SEG = min(W, 256) output pixels per image row of the
//   tile, ROWS = 256 / SEG; halo row h = r (SEG + 2) + xl + 1 holds pixel (row r shifted by
//   dy - 1, column x0 + xl), xl = -1 .. SEG; output pixel (r, xo) reads halo row
//   r (SEG + 2) + xo + dx for tap dx.  16 consecutive output pixels stay in one image row
//   (SEG >= 16), so a ds_read_b128 phase reads 16 consecutive halo rows: conflict-free.
//   K order: dy, channel group, dx, k -- a reordering of the one-tap kernel's sum, so results
//   agree with the other tiles to f32 rounding, not bitwise.
// ------------------------------------------------------------------------------------
// BN = 128 (8 waves of 64 x 64) or 64 (8 waves of 64 x 32, B pieces padded to 2 per wave).
//
// Schedule (r05, profiles/r05_halo_sched.txt, r05_halo_m16.txt).  The eight waves pair up on the
// four SIMDs (wave w and w + 4), and when both run the same program they reach the barrier, the
// DMA issue (100-185 cycles per LDS-DMA piece inside a busy phase, MI355X_MICROARCH.md) and the
// post-barrier fragment reads together, leaving the matrix pipe idle.  So:
//   LAG  waves 4..7 run each sub-step's second 32-row half after the next barrier, from
//        fragments they read before it (held in registers): their pipe work starts while their
//        partner waits for its first fragments
//   LATE the DMA of the next sub-step is issued after the first fragment reads
// The next group's halo is spread over the current group's three sub-steps (AC pieces each).
// Same MFMAs in the same order per accumulator with or without them: bit-identical.
// (r04-r05, measured and removed in r06: the 32x32x16 body of the same kernel, 5-18 % slower per
// launch; waves 0..3 issuing every DMA; a quarter stagger; re-reading the deferred A half; the
// loader state recomputed per piece; a 512 x 64 tile over 16-channel groups, 1.103 vs 1.032 ms.)
// The same halo GEMM on v_mfma_f32_16x16x32_bf16 (r05).  Under load the chip holds a higher clock
// on the 16x16x32 shape than on 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH.md, DVFS
// item 7); with this kernel's LDS traffic and DMA unchanged, swapping the shape alone measured
// -9..-18 % time per launch (tools/x3_halo_exp.hip flag 8192, profiles/r05_halo_m16.txt).
//   A wave's 64 x 64 tile is 2 x 2 blocks of 32 x 32, each computed as 2 x 2 MFMA blocks of
//   16 x 16 with K = 32 = one channel group per instruction (one k-step per sub-step).  Lane l
//   feeds A row slot l & 15 and B column slot l & 15 with channels 8 (l >> 4) .. + 8; the A row
//   slot rs of 16-row block bm is image row bm 16 + 8 ((rs >> 2) & 1) + 4 (rs >> 3) + (rs & 3),
//   so that lanes l and l ^ 16 together hold what the 32x32x16 layout gives lanes l and l ^ 16
//   (x3_acc16_to32: one exchange per register pair, then the same epilogue).
//   LDS swizzle: 16-B slot c of row r at c ^ ((r >> 1) & 2) -- the 16 lanes of a ds_read_b128
//   phase read rows r0 .. r0 + 15 at two channel slots (lane groups {0-3,12-15,20-27} etc.),
//   and this XOR puts them on 16 distinct bank quads for any r0.
//   Stagger (LAG): waves 4..7 run the second 32-row half's MFMAs after the next barrier.
// ------------------------------------------------------------------------------------
template <int BM, int BN, bool LAG>
__device__ __forceinline__ void x3r3_body16(const RowGemmArgs& p, char* smem, int wave, int lane,
                                            f32x4 (&hi)[2][BN / 64][2][2], f32x4 (&lo)[2][BN / 64][2][2],
                                            int m0, int n0) {
    constexpr int BK = 32, WM = 64, WN = BN / 2, WAVES_N = 2, WAVES = (BM / WM) * WAVES_N;
    constexpr int NT = WN / 32;
    constexpr int RB = 192, AR = BM / 16 * 18;
    constexpr int AREG = ((AR * RB + 1024 * WAVES - 1) / (1024 * WAVES)) * WAVES * 1024;
    constexpr int BREG = ((BN * RB + 1024 * WAVES - 1) / (1024 * WAVES)) * WAVES * 1024;
    constexpr int AI = AREG / (1024 * WAVES), BI = BREG / (1024 * WAVES);  // pieces per wave
    constexpr int AC = (AI + 2) / 3;
    auto swz = [](int r) { return (r >> 1) & 2; };
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int H = p.H, W = p.W, C = p.C, K = p.K;
    const int SEG = W < BM ? W : BM, HW = SEG + 2;
    const int AROWS = (BM / SEG) * HW;
    const size_t rowa = 3 * (size_t)p.lda, rowb = 3 * (size_t)K;
    // loader state packed to 3 registers per piece pair (the staggered waves hold a second
    // fragment set): pixel index, y * 128 + element offset in the 192-B row, B element offset
    int acen[AI], apk[AI], boff[BI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {  // piece j's A state: pixel at dy = 1 (-1: padding / past the halo)
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int h = o / RB, w = o - h * RB;
        const int r = h / HW, xl = h - r * HW - 1;
        const int mrow = m0 + r * SEG;
        bool ok = h < AROWS && mrow < p.M;
        const Pix q = decode(ok ? mrow : 0, H, W);
        ok = ok && q.x + xl >= 0 && q.x + xl < W;
        acen[j] = ok ? mrow + xl : -1;
        apk[j] = q.y * 128 + (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(h)) << 3);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int r = o / RB, w = o - r * RB;
        boff[j] = r < BN ? (int)((n0 + r) * rowb) + (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(r)) << 3) : -1;
    }
    const uint16_t* zero = (const uint16_t*)p.zero16;
    const uint16_t* a16 = p.a16 + (size_t)p.aoff * 3;
    const int CC = C / BK;
    const int NG = 3 * CC;
    const int ns = 9 * CC;
    auto issue_a = [&](int g, int j0, int j1) {
        const int dy = g / CC, c0 = (g - dy * CC) * BK;
        char* base = smem + (g & 1) * AREG;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            if (j < j0 || j >= j1) continue;
            const int yy = (apk[j] >> 7) + dy - 1;
            const bool valid = acen[j] >= 0 && yy >= 0 && yy < H;
            // 32 x 32 -> 64-bit row offset plus a 32-bit in-row offset (no 64-bit loop invariants)
            const uint64_t off = (uint64_t)(uint32_t)(acen[j] + (dy - 1) * W) * (uint32_t)rowa +
                                 (uint32_t)(c0 * 3 + (apk[j] & 127));
            const uint16_t* src = valid ? a16 + off : zero;
            x3_dma16(src, base + (j * WAVES + wave) * 1024);
        }
    };
    auto issue_b = [&](int s) {
        const int g = s / 3, dx = s - g * 3;
        const int dy = g / CC, c0 = (g - dy * CC) * BK;
        const int k0 = (dy * 3 + dx) * C + c0;
        char* base = smem + 2 * AREG + (s & 1) * BREG;
#pragma unroll
        for (int j = 0; j < BI; ++j)
            x3_dma16(boff[j] >= 0 ? p.bt16 + boff[j] + k0 * 3 : zero, base + (j * WAVES + wave) * 1024);
    };
    // during sub-step s: B(s + 1), then the halo pieces [dx AC, (dx + 1) AC) of group g + 1 into
    // the buffer group g - 1 read (free since the barrier that opened group g)
    auto issue = [&](int s) {
        const int g = s / 3, dx = s - g * 3;
        if (s + 1 < ns) issue_b(s + 1);
        if (g + 1 < NG) issue_a(g + 1, dx * AC, dx * AC + AC);
    };
    const int ks = lane >> 4, rs = lane & 15;
    const int rperm = m16_row(rs);
    // B rows wn WN + nt 32 + bn 16 + rs: one swizzle for all of them, bit 2 of rs
    const int bfx = (rs >> 1) & 2;
    int ahb[2][2], bro[NT][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int bm = 0; bm < 2; ++bm) {
            const int mo = wm * WM + mt * 32 + bm * 16 + rperm;
            const int r = mo / SEG;
            ahb[mt][bm] = r * HW + (mo - r * SEG);
        }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) {
            const int r = wn * WN + nt * 32 + bn * 16 + rs;
            bro[nt][bn] = r * RB;
        }
    // LAG: the previous sub-step's deferred fragments (the second 32-row half)
    bf16x8 ha[2][3], hb[NT][2][3];
    auto mma = [&](const bf16x8 (&af)[2][3], const bf16x8* bf, int mt) {
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int bn = 0; bn < 2; ++bn)
                    mfma_x3s16(af[bm], *(const bf16x8(*)[3])(bf + (nt * 2 + bn) * 3), hi[mt][nt][bm][bn],
                               lo[mt][nt][bm][bn]);
    };
    issue_a(0, 0, AI);
    issue_b(0);
    for (int s = 0; s < ns; ++s) {
        const int g = s / 3, dx = s - g * 3;
        // one barrier per sub-step: wait for B(s) and, entering a group, the last halo pieces of
        // g (the pieces of g + 1 issued during s - 1, younger than B(s), may stay in flight); the
        // barrier then also means every wave finished reading s - 1, so slot (s + 1) & 1 and
        // halo buffer (g + 1) & 1 are free
        if (dx >= 1 && g + 1 < NG) x3_wait_vm<AC>();
        else x3_wait_vm<0>();
        x3_barrier();
        const char* abase = smem + (g & 1) * AREG;
        if constexpr (LAG) {
            if (s > 0) mma(ha, &hb[0][0][0], 1);
            // the held registers free before this sub-step's reads (256 VGPRs at two waves / SIMD)
            __builtin_amdgcn_sched_barrier(0);
        }
        const char* bbase = smem + 2 * AREG + (s & 1) * BREG;
        bf16x8 af[2][3], bfr[NT][2][3];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    bfr[nt][bn][q] = *(const bf16x8*)(bbase + bro[nt][bn] + q * 64 + ((ks ^ bfx) << 4));
#pragma unroll
        for (int bm = 0; bm < 2; ++bm) {
            const int h = ahb[0][bm] + dx;
#pragma unroll
            for (int q = 0; q < 3; ++q) af[bm][q] = *(const bf16x8*)(abase + h * RB + q * 64 + ((ks ^ swz(h)) << 4));
        }
        issue(s);  // LATE: the next sub-step's DMA behind the first fragment reads
        mma(af, &bfr[0][0][0], 0);
        if constexpr (LAG) __builtin_amdgcn_sched_barrier(0);  // A of the held half after A0 died
        bf16x8 af1[2][3];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm) {
            const int h = ahb[1][bm] + dx;
#pragma unroll
            for (int q = 0; q < 3; ++q) af1[bm][q] = *(const bf16x8*)(abase + h * RB + q * 64 + ((ks ^ swz(h)) << 4));
        }
        if constexpr (LAG) {
#pragma unroll
            for (int bm = 0; bm < 2; ++bm)
#pragma unroll
                for (int q = 0; q < 3; ++q) ha[bm][q] = af1[bm][q];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int bn = 0; bn < 2; ++bn)
#pragma unroll
                    for (int q = 0; q < 3; ++q) hb[nt][bn][q] = bfr[nt][bn][q];
        } else {
            mma(af1, &bfr[0][0][0], 1);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if constexpr (LAG) mma(ha, &hb[0][0][0], 1);
}

// the 16x16x32 accumulators (hi + lo) in the 32x32x16 register layout: lanes l and l ^ 16 swap
// one register of each pair (x3r3_body16's row order makes that the whole difference)
template <int NT>
__device__ __forceinline__ void x3_acc16_to32(const f32x4 (&hi)[2][NT][2][2], const f32x4 (&lo)[2][NT][2][2],
                                              f32x16 (&acc)[2][NT], int lane) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            f32x4 a[2][2];
#pragma unroll
            for (int b = 0; b < 4; ++b) a[b >> 1][b & 1] = hi[mt][nt][b >> 1][b & 1] + lo[mt][nt][b >> 1][b & 1];
            acc16_to32(a, acc[mt][nt], lane);
        }
}

// BM = 256 (tile 4 / 256 x 128): 8 waves, one block per CU (160 KB), staggered; BM = 128 (tile 6,
// 128 x 64): 4 waves of 64 x 32, 80 KB, two blocks per CU -- independent blocks run out of phase,
// so one block's prologue, epilogue and barrier stalls overlap the other's MFMAs (the short-K
// level-0 GEMMs), and no wave holds deferred fragments
template <int EMODE, int BN = 128, int BM = 256>
__global__ __launch_bounds__(BM / 64 * 2 * 64, BM == 256 ? 1 : 2) void rowgemm_x3_row3_kernel(RowGemmArgs p) {
    constexpr int WM = 64, WN = BN / 2, NT = WN / 32, WAVES = BM / 64 * 2;
    constexpr int RB = 192, AR = BM / 16 * 18, WB = 1024 * WAVES;
    constexpr int SMEM = 2 * ((AR * RB + WB - 1) / WB) * WB + 2 * ((BN * RB + WB - 1) / WB) * WB;  // 160 / 80 KB
    static_assert(SMEM >= 2 * (BM / 64) * BN * 8, "epilogue scratch");
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / 2, wn = wave % 2;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    int tile_m, tile_n;
    tile_mn(bid, (p.M + BM - 1) / BM, ntn, p.tgm, tile_m, tile_n);
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    f32x16 acc[2][NT];
    f32x4 h16[2][NT][2][2], l16[2][NT][2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) h16[i][j][b >> 1][b & 1][r] = l16[i][j][b >> 1][b & 1][r] = 0.f;
    if (BM == 256 && wave >= 4)
        x3r3_body16<BM, BN, BM == 256>(p, smem, wave, lane, h16, l16, m0, n0);
    else
        x3r3_body16<BM, BN, false>(p, smem, wave, lane, h16, l16, m0, n0);
    x3_acc16_to32(h16, l16, acc, lane);
    x3_barrier();  // the epilogue reuses the stage memory
    row_epilogue<EMODE, BM, BN, WM, WN, true>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)smem);
}

template <int EMODE, int BN, int BM = 256>
static int x3r3_go(const RowGemmArgs& a, hipStream_t s) {
    // BM % W == 0 or W % BM == 0 keeps a tile on whole rows / row segments; W >= 16 bounds the halo
    if (a.amode != G_CONV3 || a.N % BN || a.C % 32 || a.K != 9 * a.C) return -1;
    if (a.W < 16 || (BM % a.W && a.W % BM)) return -1;
    const dim3 grid(((a.M + BM - 1) / BM) * (a.N / BN));
    hipLaunchKernelGGL((rowgemm_x3_row3_kernel<EMODE, BN, BM>), grid, dim3(BM / 64 * 2 * 64), 0, s, a);
    return (int)hipGetLastError();
}
// tiles (split accumulators; probe: profiles/r04_x3_probe_*.txt): 0 = 256x128 (8 waves of
// 64x64, 2 stages, 144 KB, one block per CU), 1 = 128x128 (4 waves, 2 stages: grids below 256
// blocks of tile 0), 2 = 128x64 (4 waves of 64x32, two blocks per CU: the 64-output layers),
// 3 = 256x64 (8 waves of 64x32, B region padded to 16 KB)
using TX0 = TileX3<256, 128, 64, 64, 2, 1, 1>;
using TX1 = TileX3<128, 128, 64, 64, 2, 1, 1>;
using TX2 = TileX3<128, 64, 64, 32, 2, 2, 1>;
using TX3 = TileX3<256, 64, 64, 32, 2, 1, 1>;
#define ROWGEMM_X3_TILES(X) X(0, TX0) X(1, TX1) X(2, TX2) X(3, TX3)

template <int AMODE, int EMODE, class T>
static int x3_go(const RowGemmArgs& a, hipStream_t s) {
    if (a.N % T::BN || a.C % 32 || a.K % 32) return -1;
    if (EMODE == E_CONVT && (a.cout % T::BN) && (T::BN % a.cout)) return -1;
    const dim3 grid(((a.M + T::BM - 1) / T::BM) * (a.N / T::BN));
    hipLaunchKernelGGL((rowgemm_x3_kernel<AMODE, EMODE, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

template <int AMODE, int EMODE>
static int x3_tile(const RowGemmArgs& a0, int tile, hipStream_t s) {
    RowGemmArgs a = a0;
    if (a.tgm < 0) {  // tile order: the group size for this tile's grid (two blocks per CU on 128 x 64)
        int bm = 0, bn = 0;
        if (rowgemm_x3_tile_dims(tile, &bm, &bn) != 0) return -1;
        a.tgm = tile_group_auto(a.M, a.N, bm, bn, (tile == 2 || tile == 6) ? 64 : 32);
    }
    if (tile == 4 || tile == 6) {  // tap-row halo kernel (3x3 convs): 256 x 128 / 128 x 64
        // (r04, not kept: 4-wave 128x64 / 64x128 wave tiles, within noise of 8 waves; B
        // straight from global memory into registers instead of the LDS ring, one barrier per
        // halo group, bit-identical but 222 -> 161 TF/s: the per-wave B loads cost more than
        // the ring's barriers; 256 x 64 as 4 waves of 64 x 64, bit-identical, 589 -> 584 img/s;
        // 256 x 64 with a three-slot B ring, B two sub-steps ahead: bit-identical, no gain;
        // r05: 256 x 64 on 8 waves, 0.2 % slower than 128 x 64, removed in r06)
        if constexpr (AMODE == G_CONV3)
            return tile == 4 ? x3r3_go<EMODE, 128>(a, s) : x3r3_go<EMODE, 64, 128>(a, s);
        return -1;
    }
    // (r05, removed in r06: the one-tap tiles on 16x16x32, config 2 within noise,
    // profiles/r05_1tap16_ab.txt; a 128 x 32 tile for the narrow widths' 32-channel layers, slower
    // than the f32 MFMA kernels there, profiles/r05_x3_n32_ab.txt)
#define X3_CASE(id, T) \
    if (tile == id) return x3_go<AMODE, EMODE, T>(a, s);
    ROWGEMM_X3_TILES(X3_CASE)
#undef X3_CASE
    return -1;
}

// ------------------------------------------------------------------------------------
// Weight gradient on x3 images: dW[m][n] = sum_p A'[p][m] * B'[p][n] over the pixels p of
// one split (slab[split], reduced in fixed order by k_slab_reduce).  A' = gather of the
// conv input's x3 image (tap = m / CA), B' = the x3 image of dz (G_IDENT) or of the ConvT
// output gradient (G_UP2, tap = n / CB).  The MFMA wants 8 consecutive PIXELS of one channel
// per lane: LDS holds [BKP pixel rows][BM / 32 groups][3 planes][32] (the x3 row as it lies in
// HBM, RA = 6 BM bytes) and the fragments come from ds_read_b64_tr_b16 (lane i of a 16-lane
// group receives column i of a 4-row x 16-column block), as wgrad16_kernel, the 16-B slots
// of each pixel row permuted by x3_tswz.
// ------------------------------------------------------------------------------------
typedef short x3_short4 __attribute__((ext_vector_type(4)));

// LDS slot of global 16-B slot sl in pixel row `row` of an RB-byte stage row (an involution,
// used by the loader and the reader alike): the four rows a 32-lane half reads (rows r0..r0+3,
// 64 B of one plane each) must fall into four different 64-B bank quarters.  RB % 256 == 0:
// XOR the quarter by row & 3; RB % 256 == 128 (BM = 64): rows r, r + 1 already differ by half
// a bank row, XOR by bit 1 of the row; RB = 192 (BM = 32): the rows are spread already.
template <int RB>
__device__ __forceinline__ int x3_tswz(int sl, int row) {
    if constexpr (RB % 256 == 0) return sl ^ ((row & 3) << 2);
    else if constexpr (RB % 256 == 128) return sl ^ (((row >> 1) & 1) << 2);
    else return sl;
}

// the same for the 16x16x32 weight gradient (r05): a 32-lane half reads 32 B (16 columns) of
// eight consecutive pixel rows r0 .. r0 + 7 (and, in its second read, of rows r0 + 16 ..), so
// the 32-B slot pairs of those rows must fall on eight different 32-B bank sections: RB % 256
// == 0: XOR the pair by row & 7; == 128: rows of one parity share a 128-B half, XOR the pair by
// (row >> 1) & 3; 192: rows r, r + 4 share a 64-B quarter, XOR the pair by (row >> 2) & 1.
// Invariant under row + 16; pairs (and 16-B halves of a plane) stay whole.
template <int RB>
__device__ __forceinline__ int x3_tswz16(int sl, int row) {
    if constexpr (RB % 256 == 0) return sl ^ ((row & 7) << 1);
    else if constexpr (RB % 256 == 128) return sl ^ (((row >> 1) & 3) << 1);
    else return sl ^ (((row >> 2) & 1) << 1);
}

template <int OFF>
__device__ __forceinline__ x3_short4 x3_tr16(unsigned addr) {
    x3_short4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
    return r;
}

__device__ __forceinline__ unsigned x3_lds_u32(const void* p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int BM_, int BN_, int WM_, int WN_, int S_, int SA_ = 0>
struct WTileX3 {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, S = S_, SA = SA_;
    static constexpr int BKP = 32;  // pixels per chunk (two 16-pixel k-steps)
    static constexpr int WAVES = (BM / WM) * (BN / WN);
    static constexpr int THREADS = 64 * WAVES;
};

template <int AMODE, int BMODE, class T>
__global__ __launch_bounds__(T::THREADS, 1) void wgrad_x3_kernel(WgradArgs p) {
    constexpr int BM = T::BM, BN = T::BN, WM = T::WM, WN = T::WN, BKP = T::BKP, S = T::S;
    constexpr int WAVES = T::WAVES, WAVES_N = BN / WN;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int RA = 6 * BM, RBB = 6 * BN;  // bytes per pixel row of the A' / B' stage images
    static_assert((BKP * RA) % (1024 * WAVES) == 0 && (BKP * RBB) % (1024 * WAVES) == 0, "loader");
    constexpr int AI = BKP * RA / (1024 * WAVES), BI = BKP * RBB / (1024 * WAVES);
    constexpr int GPC = AI + BI;
    static_assert(S >= 2 && S <= 3, "stages");
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

    // loader: lane of instruction j fills stage byte o = (j WAVES + wave) KB + 16 lane: pixel
    // row o / RA, 16-B slot s = (o % RA) / 16, sourcing global slot x3_tswz(s, row) of the
    // row's x3 segment
    int arow[AI], aele[AI], brow[BI], bele[BI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int r = o / RA, sl = (o - r * RA) >> 4;
        arow[j] = r;
        aele[j] = x3_tswz<RA>(sl, r) * 8;
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int r = o / RBB, sl = (o - r * RBB) >> 4;
        brow[j] = r;
        bele[j] = x3_tswz<RBB>(sl, r) * 8;
    }
    const uint16_t* a16 = (const uint16_t*)p.a + (size_t)(p.aoff + ca0) * 3;
    const uint16_t* b16 = (const uint16_t*)p.b + (size_t)(p.boff + cb0) * 3;
    const size_t rowa = 3 * (size_t)p.lda, rowb = 3 * (size_t)p.ldb;
    const uint16_t* zero = (const uint16_t*)p.zero16;

    auto issue = [&](int kc, int st) {
        const int pc = pbeg + kc * BKP;
        char* base = smem + st * STAGE;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            const int pix = pc + arow[j];
            const bool in = pix < pend;
            const int m = in ? pix : pend - 1;
            bool valid;
            const Pix q = AMODE == G_IDENT ? Pix{0, 0, 0} : decode_fast(m, H, W, rH, rW);
            const int src = gather_src<AMODE>(tapA, m, q, H, W, valid);
            const uint16_t* g = (valid && in) ? a16 + (size_t)src * rowa + aele[j] : zero;
            x3_dma16(g, base + (j * WAVES + wave) * 1024);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int pix = pc + brow[j];
            const bool in = pix < pend;
            const int m = in ? pix : pend - 1;
            bool valid;
            const Pix q = BMODE == G_IDENT ? Pix{0, 0, 0} : decode_fast(m, H, W, rH, rW);
            const int src = gather_src<BMODE>(tapB, m, q, H, W, valid);
            const uint16_t* g = (valid && in) ? b16 + (size_t)src * rowb + bele[j] : zero;
            x3_dma16(g, base + BKP * RA + (j * WAVES + wave) * 1024);
        }
    };

    constexpr int SA = T::SA;
    f32x16 acc[MT][NT], acl[SA ? MT : 1][SA ? NT : 1];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[i][j][r] = 0.f;
                if constexpr (SA) acl[i][j][r] = 0.f;
            }

    // transposed-read addresses (bytes within a stage, k-step 0): lane l of group g = l / 16
    // supplies row 8 (g >> 1) + qq, columns 16 (g & 1) + 4 pp (l % 16 = 4 qq + pp) of plane q
    const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const int trow = 8 * (g >> 1) + qq;  // + 4 t + 16 kk: (row & 3) stays qq
    auto slot = [](int col, int q) { return (col >> 5) * 12 + q * 4 + ((col & 31) >> 3); };
    int aoff[MT][3], boff[NT][3];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int col = wm * WM + mt * 32 + 16 * (g & 1) + 4 * pp;
            aoff[mt][q] = trow * RA + (x3_tswz<RA>(slot(col, q), trow) << 4) + ((col >> 2) & 1) * 8;
        }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int col = wn * WN + nt * 32 + 16 * (g & 1) + 4 * pp;
            boff[nt][q] = BKP * RA + trow * RBB + (x3_tswz<RBB>(slot(col, q), trow) << 4) + ((col >> 2) & 1) * 8;
        }

#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (s < nk) issue(s, s);
    for (int kc = 0; kc < nk; ++kc) {
        if (kc + S - 1 < nk) issue(kc + S - 1, (kc + S - 1) % S);
        const int ahead = min(S - 1, nk - 1 - kc);
        if constexpr (S >= 3) {
            if (ahead >= 2) x3_wait_vm<2 * GPC>();
            else if (ahead == 1) x3_wait_vm<GPC>();
            else x3_wait_vm<0>();
        } else {
            if (ahead >= 1) x3_wait_vm<GPC>();
            else x3_wait_vm<0>();
        }
        x3_barrier();
        const unsigned sb = x3_lds_u32(smem) + (kc % S) * STAGE;
        x3_short4 fa[2][MT][3][2], fb[2][NT][3][2];
        auto load = [&](auto KK) {
            constexpr int kk = decltype(KK)::value;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    fa[kk][mt][q][0] = x3_tr16<kk * 16 * RA>(sb + aoff[mt][q]);
                    fa[kk][mt][q][1] = x3_tr16<kk * 16 * RA + 4 * RA>(sb + aoff[mt][q]);
                }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    fb[kk][nt][q][0] = x3_tr16<kk * 16 * RBB>(sb + boff[nt][q]);
                    fb[kk][nt][q][1] = x3_tr16<kk * 16 * RBB + 4 * RBB>(sb + boff[nt][q]);
                }
        };
        auto mma = [&](auto KK) {
            constexpr int kk = decltype(KK)::value;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    bf16x8 a3[3], b3[3];
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
                        a3[q] = *(const bf16x8*)fa[kk][mt][q];
                        b3[q] = *(const bf16x8*)fb[kk][nt][q];
                    }
                    if constexpr (SA) mfma_x3s(a3, b3, acc[mt][nt], acl[mt][nt]);
                    else acc[mt][nt] = mfma_x3(a3, b3, acc[mt][nt]);
                }
        };
        static_assert(BKP == 32, "two k-steps per chunk");
        load(std::integral_constant<int, 0>{});
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        load(std::integral_constant<int, 1>{});
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 0>{});
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(std::integral_constant<int, 1>{});
        x3_barrier();
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
                slab[(size_t)m * p.Nw + n] = SA ? acc[mt][nt][r] + acl[SA ? mt : 0][SA ? nt : 0][r]
                                                : acc[mt][nt][r];
            }
}

// ------------------------------------------------------------------------------------
// Tap-row weight gradient on x3 images (3x3 convs, W % 32 == 0): one block computes the three
// dx taps of one tap row dy for a BM (ci) x BN (co) tile over its split's pixels.  A 32-pixel
// chunk never crosses an image row, so the A' operands of the three taps are the same 34
// halo pixels of source row y + dy - 1 (columns x0 - 1 .. x0 + 32, zero outside the image),
// read at row offsets dx = 0, 1, 2: a third of the one-tap kernel's A' staging per MFMA.
// 16x16x32 MFMAs (r05): the chip holds a higher clock on that shape at equal cycles per FLOP.
// Stage: [AR halo rows][6 BM B] + [32 pixel rows][6 BN B]; the loader gives every wave the same
// instruction count (rows past the halo / chunk read zeros).
// ------------------------------------------------------------------------------------
//
// LAG (r05 schedule 10, the 64 x 128 tile): four LDS stages with the DMA two chunks ahead, so a
// stage stays intact one chunk longer; waves 4..7 (each sharing a SIMD with wave w - 4) run each
// chunk's second 16-column half at the start of the next chunk, re-reading its fragments from
// that stage, while their partner waits for its first fragments (MI355X_MICROARCH.md "two waves
// per SIMD" item 9); the next DMA goes behind the first fragment reads.  Without LAG (the 128 x
// 64 and 64 x 64 tiles) the DMA runs S - 1 chunks ahead.  Same MFMAs in the same order per
// accumulator, same split partition: bit-identical.  (r04-r05, removed in r06: the 32x32x16
// body, 1.6-1.9 % slower over the step, and its staggered / late-DMA variants.)
template <int BM, int BN, int S = 3, int OCC = 1, bool LAG = false, bool W16 = false>
__global__ __launch_bounds__((BM / 32) * (BN / 32) * 64, OCC) void wgrad_x3_row3_kernel(WgradArgs p) {
    constexpr int WAVES = (BM / 32) * (BN / 32), BKP = 32;
    constexpr int WAVES_N = BN / 32;
    static_assert(S >= 2 && S <= 4, "stages");
    static_assert(!LAG || (S == 4 && WAVES == 8), "the stagger: four stages, waves w / w + 4");
    constexpr int LW = WAVES;                   // waves issuing the DMA
    constexpr int DIST = LAG ? 2 : S - 1;       // chunks the DMA runs ahead
    constexpr bool LATE = LAG;                  // the DMA issued after the first fragment reads
    constexpr int RA = 6 * BM, RBB = 6 * BN;
    // halo pixel rows per stage: 34 (one 32-pixel row segment) plus room for W = 16's two image
    // rows of 16 + 2 (r05: the 16x16 level's 3x3 weight gradients on this kernel too)
    constexpr int HALO = BKP + 4;
    constexpr int AREG = (HALO * RA + 1024 * WAVES - 1) / (1024 * WAVES) * WAVES * 1024;  // per stage
    constexpr int BREG = (BKP * RBB + 1024 * WAVES - 1) / (1024 * WAVES) * WAVES * 1024;
    constexpr int AI = AREG / (1024 * LW), BI = BREG / (1024 * LW);  // pieces per issuing wave
    constexpr int GPC = AI + BI;
    constexpr int STAGE = AREG + BREG;
    __shared__ __attribute__((aligned(1024))) char smem[STAGE * S];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const bool issuer = wave < LW;
    const bool lag = LAG && wave >= 4;
    const int tiles_n = p.CB / BN, tiles_m = p.CA / BM;
    int idx = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tn = idx % tiles_n;
    idx /= tiles_n;
    const int dy = idx % 3;
    idx /= 3;
    const int tm = idx % tiles_m;
    const int split = idx / tiles_m;
    const int ca0 = tm * BM, cb0 = tn * BN;
    const int H = p.H, W = p.W;
    const int pbeg = split * p.pps;
    const int pend = min(pbeg + p.pps, p.P);
    const int nk = (pend - pbeg) / BKP;  // pps, P multiples of 32

    // loader: lane of piece j fills stage byte o = (j LW + wave) KB + 16 lane: pixel row o / RA,
    // 16-B slot (o % RA) / 16, sourcing slot x3_tswz16 of it (recomputed per piece to stay
    // within 256 VGPRs)
    // W16 (launched for W = 16 only): two 18-row halo segments, swizzle by row mod 18 (its own
    // instance: one kernel holding both loops costs 1-6 spilled VGPRs)
    using W16T = std::integral_constant<bool, W16>;
    auto apiece = [&](int j, int& r, int& e, auto W16C) {
        constexpr bool TW = decltype(W16C)::value;
        const int o = ((j * LW + wave) * 64 + lane) * 16;
        r = o / RA;
        e = x3_tswz16<RA>((o - r * RA) >> 4, TW ? r % 18 : r) * 8;
    };
    auto bpiece = [&](int j, int& r, int& e) {
        const int o = ((j * LW + wave) * 64 + lane) * 16;
        r = o / RBB;
        e = x3_tswz16<RBB>((o - r * RBB) >> 4, r) * 8;
    };
    const uint16_t* a16 = (const uint16_t*)p.a + (size_t)(p.aoff + ca0) * 3;
    const uint16_t* b16 = (const uint16_t*)p.b + (size_t)(p.boff + cb0) * 3;
    const size_t rowa = 3 * (size_t)p.lda, rowb = 3 * (size_t)p.ldb;
    const uint16_t* zero = (const uint16_t*)p.zero16;

    auto issue = [&](int kc, int st, auto W16C) {
        constexpr bool TW = decltype(W16C)::value;
        const int pc = pbeg + kc * BKP;  // wave-uniform: the chunk's image row and first column
        const int t = pc / W, x0 = pc - t * W;
        const int img = t / H, y = t - img * H;
        const int yy = y + dy - 1;
        const bool rowok = yy >= 0 && yy < H;
        const int rowbase = (img * H + yy) * W;
        char* base = smem + st * STAGE;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            int ar, ae;
            apiece(j, ar, ae, W16C);
            // W = 16 (w16): halo row ar = 18 seg + xl + 1 holds image row y + seg + dy - 1,
            // column xl (the chunk is image rows y, y + 1; y even, H even)
            const int seg = TW ? ar / 18 : 0;
            const int xx = TW ? ar - seg * 18 - 1 : x0 - 1 + ar;
            const bool segok = TW ? (seg < 2 && yy + seg >= 0 && yy + seg < H) : (rowok && ar < BKP + 2);
            const bool ok = segok && xx >= 0 && xx < W;
            const uint16_t* g = ok ? a16 + (size_t)(rowbase + seg * W + xx) * rowa + ae : zero;
            x3_dma16(g, base + (j * LW + wave) * 1024);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            int br, be;
            bpiece(j, br, be);
            const bool ok = br < BKP;
            const uint16_t* g = ok ? b16 + (size_t)(pc + br) * rowb + be : zero;
            x3_dma16(g, base + AREG + (j * LW + wave) * 1024);
        }
    };

    // 16x16x32: per chunk ONE k-step of 32 pixels; a wave's 32 x 32 x 3-tap tile is 2 x 2
    // blocks of 16 x 16 per tap.  Lane l of group g = l / 16 supplies the k values 8 g .. 8 g
    // + 7 = pixel rows 4 g + qq (first transposed read) and 16 + 4 g + qq (second), the same
    // rows for A' and B' (any k order sums the same products), column l & 15 of its block.
    f32x4 hi[3][2][2], lo[3][2][2];
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) hi[d][b >> 1][b & 1][r] = lo[d][b >> 1][b & 1][r] = 0.f;
    const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const int trow = 4 * g + qq;
    auto slot = [](int col, int q) { return (col >> 5) * 12 + q * 4 + ((col & 31) >> 3); };
    int aoff[3][2][3], boff[2][3];
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
        const int col = wm * 32 + 16 * bm + 4 * pp;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int q = 0; q < 3; ++q)
                aoff[dx][bm][q] = (trow + dx) * RA + (x3_tswz16<RA>(slot(col, q), trow + dx) << 4) + ((col >> 2) & 1) * 8;
        // (trow + dx <= 17: the same swizzle row for W = 16's row-mod-18 rule)
        const int colb = wn * 32 + 16 * bm + 4 * pp;
#pragma unroll
        for (int q = 0; q < 3; ++q)
            boff[bm][q] = AREG + trow * RBB + (x3_tswz16<RBB>(slot(colb, q), trow) << 4) + ((colb >> 2) & 1) * 8;
    }
    const unsigned sbase = x3_lds_u32(smem);
    auto rd = [](x3_short4 (&f)[2], unsigned addr, auto ROWB) {
        constexpr int rb = decltype(ROWB)::value;
        f[0] = x3_tr16<0>(addr);
        f[1] = x3_tr16<16 * rb>(addr);
    };
    // A' second read: pixel rows 16 + 4 g + qq sit 16 halo rows on, or 18 at W = 16 (a
    // compile-time offset per loop instance: an added address per read costs 18 VGPRs)
    auto rda = [](x3_short4 (&f)[2], unsigned addr, auto W16C) {
        constexpr int off = decltype(W16C)::value ? 18 * RA : 16 * RA;
        f[0] = x3_tr16<0>(addr);
        f[1] = x3_tr16<off>(addr);
    };
    using IRB = std::integral_constant<int, RBB>;
    auto mma = [&](const x3_short4 (&fa)[3][3][2], const x3_short4 (&fb)[2][3][2], int bm) {
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) {
            bf16x8 b3[3];
#pragma unroll
            for (int q = 0; q < 3; ++q) b3[q] = *(const bf16x8*)fb[bn][q];
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                bf16x8 a3[3];
#pragma unroll
                for (int q = 0; q < 3; ++q) a3[q] = *(const bf16x8*)fa[dx][q];
                mfma_x3s16(a3, b3, hi[dx][bm][bn], lo[dx][bm][bn]);
            }
        }
    };
    // schedule 10 (LG): waves 4..7 run each chunk's second 16-column half (bm = 1) at the
    // start of the next chunk, re-reading its fragments from the chunk's stage (four
    // stages, DMA two chunks ahead: a stage stays intact one chunk longer) -- the stagger
    // of the halo GEMM's schedule 9 without held registers
    auto loop = [&](auto W16C, auto LGC) {
    constexpr bool LG = decltype(LGC)::value;
    if (issuer) {
#pragma unroll
        for (int s = 0; s < DIST; ++s)
            if (s < nk) issue(s, s, W16C);
    }
    for (int kc = 0; kc < nk; ++kc) {
        if (issuer) {
            if (DIST >= 2 && kc + 1 < nk) x3_wait_vm<GPC>();
            else x3_wait_vm<0>();
        }
        x3_barrier();
        if (!LATE && issuer && kc + DIST < nk) issue(kc + DIST, (kc + DIST) % S, W16C);
        if constexpr (LG) {
            if (kc > 0) {
                const unsigned sp = sbase + ((kc + S - 1) % S) * STAGE;
                x3_short4 pb[2][3][2], pa[3][3][2];
#pragma unroll
                for (int bn = 0; bn < 2; ++bn)
#pragma unroll
                    for (int q = 0; q < 3; ++q) rd(pb[bn][q], sp + boff[bn][q], IRB{});
#pragma unroll
                for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                    for (int q = 0; q < 3; ++q) rda(pa[dx][q], sp + aoff[dx][1][q], W16C);
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                mma(pa, pb, 1);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        const unsigned sb = sbase + (kc % S) * STAGE;
        x3_short4 fb[2][3][2], fa[3][3][2], fa1[3][3][2];
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
#pragma unroll
            for (int q = 0; q < 3; ++q) rd(fb[bn][q], sb + boff[bn][q], IRB{});
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int q = 0; q < 3; ++q) rda(fa[dx][q], sb + aoff[dx][0][q], W16C);
        if (LATE && issuer && kc + DIST < nk) {
            __builtin_amdgcn_sched_barrier(0);
            issue(kc + DIST, (kc + DIST) % S, W16C);
            __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (LG) {
            mma(fa, fb, 0);
            continue;
        }
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
            for (int q = 0; q < 3; ++q) rda(fa1[dx][q], sb + aoff[dx][1][q], W16C);
        __builtin_amdgcn_sched_barrier(0);
        mma(fa, fb, 0);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        mma(fa1, fb, 1);
    }
    if constexpr (LG) {
        if (nk > 0) {  // the last chunk's second half (its stage is not restaged any more)
            const unsigned sp = sbase + ((nk - 1) % S) * STAGE;
            x3_short4 pb[2][3][2], pa[3][3][2];
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
#pragma unroll
                for (int q = 0; q < 3; ++q) rd(pb[bn][q], sp + boff[bn][q], IRB{});
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                for (int q = 0; q < 3; ++q) rda(pa[dx][q], sp + aoff[dx][1][q], W16C);
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            mma(pa, pb, 1);
        }
    }
    };
    if (lag) loop(W16T{}, std::true_type{});
    else loop(W16T{}, std::false_type{});
    float* slab = p.slab + (size_t)split * p.Mw * p.Nw;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m = (dy * 3 + dx) * p.CA + ca0 + wm * 32 + 16 * bm + 4 * g + i;
                    const int n = cb0 + wn * 32 + 16 * bn + (lane & 15);
                    slab[(size_t)m * p.Nw + n] = hi[dx][bm][bn][i] + lo[dx][bm][bn][i];
                }
}

// tiles (split accumulators): 0 = 128x128 (8 waves of 64x32), 1 = 64x64 (4 waves of 32x32);
// three LDS stages of 32 pixels
using WX0 = WTileX3<128, 128, 64, 32, 3, 1>;
using WX1 = WTileX3<64, 64, 32, 32, 3, 1>;
#define WGRAD_X3_TILES(X) X(0, WX0) X(1, WX1)

template <int AMODE, int BMODE, class T>
static int wx3_go(const WgradArgs& a, hipStream_t s) {
    if (a.Mw % T::BM || a.Nw % T::BN || a.CA % T::BM || a.CB % T::BN || a.pps % T::BKP) return -1;
    const dim3 grid((a.Mw / T::BM) * (a.Nw / T::BN) * a.splits);
    hipLaunchKernelGGL((wgrad_x3_kernel<AMODE, BMODE, T>), grid, dim3(T::THREADS), 0, s, a);
    return (int)hipGetLastError();
}

// exact three-way split of 8 f32 values into their hi / mid / lo bf16 pieces, stored at d,
// d + 32, d + 64 (one 32-channel group of an x3 row)
// (x3_split.h: the range edges -- huge, +-inf, NaN -- keep their values)
typedef uint16_t x3_u16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ void x3_store8(const float (&v)[8], uint16_t* d) {
    x3_u16x8 h, m, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        uint16_t hj, mj, lj;
        x3_split(v[j], X3CvtDev{}, hj, mj, lj);
        h[j] = hj;
        m[j] = mj;
        l[j] = lj;
    }
    *(x3_u16x8*)d = h;
    *(x3_u16x8*)(d + 32) = m;
    *(x3_u16x8*)(d + 64) = l;
}

// Rows per block of the two image passes: 256, or fewer where that leaves the grid short of
// ~1024 blocks (the deep levels: 8k rows x 1024 channels made 32 blocks, 1.2 TB/s;
// profiles/r05_x3_pass_exp.txt).  bn_dz_x3's bias partials come one row per block, so the
// caller sizes its reduction with x3_dz_blocks (the same rule).
__host__ __device__ inline int x3_rows_per_block(int64_t P) {
    return P >= 256 * 1024 ? 256 : P >= 128 * 1024 ? 128 : 64;
}
constexpr int X3_RIF = 4;  // rows in flight per thread (all loads before any arithmetic)

// x3 image of op(src) (f32 [P][ld] at channel offset off, C channels; scale / shift: the
// BN affine, ReLU on channels < relu) into dst [P][dld / 32][3][32] at channel offset doff.
// A block covers rpb rows; thread t handles channel octet t % (C / 8) of rows t / (C / 8) +
// k 256 / (C / 8), X3_RIF rows in flight; the affine is loaded once per thread.
__global__ __launch_bounds__(256) void to_x3_kernel(const float* __restrict__ src, int ld, int off, int C,
                                                    const float* __restrict__ scale,
                                                    const float* __restrict__ shift, int relu, int64_t P,
                                                    uint16_t* __restrict__ dst, int dld, int doff, int rpb) {
    const int g8 = C / 8, G = min(g8, 256);  // octets per pass (C > 2048: several passes)
    const int r0 = threadIdx.x / G, rstep = 256 / G;
    if (r0 >= rstep) return;
    const int64_t mb = (int64_t)blockIdx.x * rpb;
    const int64_t me = min(mb + rpb, P);
    for (int oct = threadIdx.x % G; oct < g8; oct += G) {
        const int c = oct * 8;
        float sc[8], sh[8];
        if (scale) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f32x4 a = *(const f32x4*)(scale + c + 4 * h), b = *(const f32x4*)(shift + c + 4 * h);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    sc[4 * h + j] = a[j];
                    sh[4 * h + j] = b[j];
                }
            }
        }
        const int cc = doff + c;
        uint16_t* dcol = dst + (cc >> 5) * 96 + (cc & 31);
        for (int64_t m = mb + r0; m < me; m += X3_RIF * rstep) {
            f32x4 v[X3_RIF][2];
#pragma unroll
            for (int i = 0; i < X3_RIF; ++i) {
                const int64_t mi = m + i * rstep;
                if (mi < me) {
                    const float* sp = src + mi * ld + off + c;
                    v[i][0] = *(const f32x4*)sp;
                    v[i][1] = *(const f32x4*)(sp + 4);
                }
            }
#pragma unroll
            for (int i = 0; i < X3_RIF; ++i) {
                const int64_t mi = m + i * rstep;
                if (mi >= me) break;
                float w[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float t = v[i][j >> 2][j & 3];
                    if (scale) {
                        t = __builtin_fmaf(sc[j], t, sh[j]);
                        if (c + j < relu) t = fmaxf(t, 0.f);
                    }
                    w[j] = t;
                }
                x3_store8(w, dcol + mi * 3 * (int64_t)dld);
            }
        }
    }
}

// dz = [!mask || y > 0] (A do + B (y - mean) + C) per channel (bn_dz4, the f32 path's
// rounding order) as the x3 image dz3 [P][C / 32][3][32]; with bpart, also the per-block
// column sums of dz (the conv bias gradient; k_sum_partials adds the G rows in f64).  A
// block covers rpb rows (x3_rows_per_block); thread t handles channel octet t % (C / 8) of
// rows t / (C / 8) + k 256 / (C / 8), X3_RIF rows in flight (the column sums add each thread's
// rows in ascending order).
// HEAD (r05): the last conv's `do` is not read from memory but recomputed from the 1x1 head:
// do[m][c] = [BN->ReLU: fma(y, sc, sh) > 0] dl[m] w[c] (head_bwd's expression, bit for bit;
// out_channels = 1), so head_bwd need not store the 64-channel f32 do at full resolution.
struct DzHead {
    const float* dl;     // d logits [P] (NCHW with one channel = pixel order)
    const float* w;      // head weights [C]
    const float *sc, *sh;  // the last BN's forward affine
    int relu;            // BN -> ReLU: mask by the activation
};
// POOL (r05): the encoder block's second conv: do = [BN->ReLU: fma(msc, y, msh) > 0] (dskip +
// [winner == window position] dp) -- maxpool_bwd's expression, so it need not store do
struct DzPool {
    const float* dp;       // d pooled [N][H/2][W/2][C]
    const uint8_t* idx;    // winner index per pooled element
    const float* dskip;    // the concat gradient's skip half (offset applied), row stride ldskip
    int ldskip;
    const float *msc, *msh;  // BN -> ReLU mask affine, or null
    int H, W;              // full-resolution grid
    float rH, rW;
};

template <int SRC>  // 0: do from memory, 1: DzHead, 2: DzPool
__global__ __launch_bounds__(256) void bn_dz_x3_kernel(const float* __restrict__ d, const float* __restrict__ y,
                                                       int ld, int off, int64_t P, int C,
                                                       const float* __restrict__ coef, int mask,
                                                       uint16_t* __restrict__ dz3, float* __restrict__ bpart,
                                                       int rpb, DzHead hd, DzPool pl) {
    constexpr bool HEAD = SRC == 1, POOL = SRC == 2;
    __shared__ float red[256 * 8];
    const int g8 = C / 8, G = min(g8, 256);  // octets per pass (bias sums: C <= 2048, one pass)
    const int r0 = threadIdx.x / G, rstep = 256 / G;
    const bool active = r0 < rstep;  // threads past the last complete row group idle
    const int64_t mb = (int64_t)blockIdx.x * rpb;
    const int64_t me = min(mb + rpb, P);
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int oct = threadIdx.x % G; active && oct < g8; oct += G) {
        const int c = oct * 8;
        f32x4 ka[2], kb[2], kc[2], km[2], hw[2], hs[2], hh[2], msc[2], msh[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (POOL && pl.msc) {  // the BN -> ReLU mask affine, in registers (r06)
                msc[h] = *(const f32x4*)(pl.msc + c + 4 * h);
                msh[h] = *(const f32x4*)(pl.msh + c + 4 * h);
            }
            ka[h] = *(const f32x4*)(coef + c + 4 * h);
            kb[h] = *(const f32x4*)(coef + C + c + 4 * h);
            kc[h] = *(const f32x4*)(coef + 2 * C + c + 4 * h);
            km[h] = *(const f32x4*)(coef + 3 * C + c + 4 * h);
            if constexpr (HEAD) {
                hw[h] = *(const f32x4*)(hd.w + c + 4 * h);
                hs[h] = *(const f32x4*)(hd.sc + c + 4 * h);
                hh[h] = *(const f32x4*)(hd.sh + c + 4 * h);
            }
        }
        for (int64_t m = mb + r0; m < me; m += X3_RIF * rstep) {
            f32x4 dv[X3_RIF][2], yv[X3_RIF][2];
            float dl[X3_RIF];
            f32x4 gp[X3_RIF][2];
            uint32_t wi[X3_RIF][2];
            int kk[X3_RIF];
#pragma unroll
            for (int i = 0; i < X3_RIF; ++i) {
                const int64_t mi = m + i * rstep;
                if (mi < me) {
                    if constexpr (HEAD) dl[i] = hd.dl[mi];
                    int64_t po = 0;
                    if constexpr (POOL) {
                        const Pix q = decode_fast((int)mi, pl.H, pl.W, pl.rH, pl.rW);
                        po = ((int64_t)q.img * (pl.H >> 1) + (q.y >> 1)) * (pl.W >> 1) + (q.x >> 1);
                        kk[i] = (q.y & 1) * 2 + (q.x & 1);
                        const uint2 w2 = *(const uint2*)(pl.idx + po * C + c);
                        wi[i][0] = w2.x;
                        wi[i][1] = w2.y;
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if constexpr (POOL) {
                            dv[i][h] = *(const f32x4*)(pl.dskip + mi * pl.ldskip + c + 4 * h);
                            gp[i][h] = *(const f32x4*)(pl.dp + po * C + c + 4 * h);
                        } else if constexpr (!HEAD) {
                            dv[i][h] = *(const f32x4*)(d + mi * C + c + 4 * h);
                        }
                        yv[i][h] = *(const f32x4*)(y + mi * ld + off + c + 4 * h);
                    }
                }
            }
            if constexpr (POOL) {
#pragma unroll
                for (int i = 0; i < X3_RIF; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (((wi[i][h] >> (8 * j)) & 0xFF) == (uint32_t)kk[i]) dv[i][h][j] += gp[i][h][j];
                            if (pl.msc && !(__builtin_fmaf(msc[h][j], yv[i][h][j], msh[h][j]) > 0.f))
                                dv[i][h][j] = 0.f;
                        }
            }
            if constexpr (HEAD) {
#pragma unroll
                for (int i = 0; i < X3_RIF; ++i)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const bool on = !hd.relu || __builtin_fmaf(yv[i][h][j], hs[h][j], hh[h][j]) > 0.f;
                            dv[i][h][j] = on ? dl[i] * hw[h][j] : 0.f;
                        }
            }
#pragma unroll
            for (int i = 0; i < X3_RIF; ++i) {
                const int64_t mi = m + i * rstep;
                if (mi >= me) break;
                float v[8];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const f32x4 r = bn_dz4(ka[h], dv[i][h], kb[h], yv[i][h], km[h], kc[h]);
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[4 * h + j] = (!mask || yv[i][h][j] > 0.f) ? r[j] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) cs[j] += v[j];
                x3_store8(v, dz3 + mi * 3 * (int64_t)C + (c >> 5) * 96 + (c & 31));
            }
        }
    }
    if (!bpart) return;  // (the launcher allows bias sums for C <= 2048 only)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = active ? cs[j] : 0.f;
    __syncthreads();
    // column c + j: the rstep row groups' sums in fixed order
    for (int i = threadIdx.x; i < C; i += 256) {
        const int o8 = i >> 3, j = i & 7;
        float a = 0.f;
        for (int r = 0; r < rstep; ++r) a += red[(r * g8 + o8) * 8 + j];
        bpart[(size_t)blockIdx.x * C + i] = a;
    }
}

}  // namespace

int rowgemm_x3_tile_dims(int tile, int* bm, int* bn) {
    if (tile == 4 || tile == 6) {  // tap-row halo 256 x 128 / 128 x 64
        *bm = tile == 6 ? 128 : 256;
        *bn = tile == 4 ? 128 : 64;
        return 0;
    }
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
    if (P < 1) return -1;
    const int rpb = x3_rows_per_block(P);
    const int blocks = (int)((P + rpb - 1) / rpb);
    hipLaunchKernelGGL(to_x3_kernel, dim3(blocks), dim3(256), 0, s, src, ld, off, C, scale, shift,
                       relu, P, dst, dld, doff, rpb);
    return (int)hipGetLastError();
}

// tap-row tiles (BM ci x BN co per tap, three taps per block): 2 = 64x128, 4 = 64x64 (r05-r06
// tile 3, 128x64, measured 20 % slower than 4 on config 2's 128 -> 64 conv and was removed)
static const int WX3R3_DIMS[5][2] = {{0, 0}, {0, 0}, {64, 128}, {0, 0}, {64, 64}};

int wgrad_x3_tile_dims(int tile, int* bm, int* bn) {
    if (tile == 2 || tile == 4) {
        *bm = WX3R3_DIMS[tile][0];
        *bn = WX3R3_DIMS[tile][1];
        return 0;
    }
#define WX3_DIMS(id, T) \
    if (tile == id) {   \
        *bm = T::BM;    \
        *bn = T::BN;    \
        return 0;       \
    }
    WGRAD_X3_TILES(WX3_DIMS)
#undef WX3_DIMS
    return -1;
}

// Weight gradient from x3 images: a / b point at uint16 x3 images (lda / ldb channels per
// row, channel offsets aoff / boff multiples of 32), zero16 at a zeroed page.  3x3 conv (A'
// G_CONV3, B' G_IDENT) and ConvT (A' G_IDENT, B' G_UP2); no bias column sums.
// (r04, not kept: the tap-row tiles on 64-pixel chunks, four k-steps per barrier pair:
// bit-identical, config 2 within noise, profiles/r04_x3_halo_ab.txt)
int launch_wgrad_x3(const WgradArgs& a, int tile, hipStream_t s) {
    if (a.ascale || a.bcoef || a.bias_slab || !a.zero16 || a.P < 1) return -1;
    if (a.aoff % 32 || a.boff % 32 || a.lda % 32 || a.ldb % 32) return -1;
    if (tile == 2 || tile == 4) {  // tap-row kernel: 3x3 convs, W % 32 == 0 or W = 16 with an even H
        int bm = 0, bn = 0;
        wgrad_x3_tile_dims(tile, &bm, &bn);
        const bool w16 = a.W == 16 && a.H % 2 == 0;
        if (a.amode != G_CONV3 || a.bmode != G_IDENT || a.Mw != 9 * a.CA || a.Nw != a.CB ||
            a.CA % bm || a.CB % bn || (a.W % 32 && !w16) || a.pps % 32 || a.P % 32)
            return -1;
        const dim3 grid((a.CA / bm) * 3 * (a.CB / bn) * a.splits);
        // 64 x 128: four stages with the stagger (r05 schedule 10); 64 x 64 without it
        if (tile == 2 && w16)
            hipLaunchKernelGGL((wgrad_x3_row3_kernel<64, 128, 4, 1, true, true>), grid, dim3(512), 0, s, a);
        else if (tile == 2)
            hipLaunchKernelGGL((wgrad_x3_row3_kernel<64, 128, 4, 1, true>), grid, dim3(512), 0, s, a);
        else if (w16)  // 64 x 64: four waves, two LDS stages, two blocks per CU
            hipLaunchKernelGGL((wgrad_x3_row3_kernel<64, 64, 2, 2, false, true>), grid, dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((wgrad_x3_row3_kernel<64, 64, 2, 2>), grid, dim3(256), 0, s, a);
        return (int)hipGetLastError();
    }
#define WX3G(AM, BMD)                                        \
    do {                                                     \
        if (tile == 0) return wx3_go<AM, BMD, WX0>(a, s);    \
        if (tile == 1) return wx3_go<AM, BMD, WX1>(a, s);    \
        return -1;                                           \
    } while (0)
    if (a.amode == G_CONV3 && a.bmode == G_IDENT) WX3G(G_CONV3, G_IDENT);
    if (a.amode == G_IDENT && a.bmode == G_UP2) WX3G(G_IDENT, G_UP2);
#undef WX3G
    return -1;
}

int x3_dz_blocks(int64_t P) {
    const int rpb = x3_rows_per_block(P);
    return (int)((P + rpb - 1) / rpb);
}

int k_bn_dz_x3(const float* d, const float* y, int ld, int off, int64_t P, int C, const float* coef,
               int mask, uint16_t* dz3, float* bpart, hipStream_t s, const float* hdl, const float* hw,
               const float* hsc, const float* hsh, int hrelu) {
    if (C % 32 || (bpart && C > 2048) || ld % 4 || off % 4 || P < 1) return -1;
    if (hdl) {
        if (!hw || !hsc || !hsh) return -1;
        const DzHead hd{hdl, hw, hsc, hsh, hrelu};
        hipLaunchKernelGGL(bn_dz_x3_kernel<1>, dim3(x3_dz_blocks(P)), dim3(256), 0, s, d, y, ld, off, P, C,
                           coef, mask, dz3, bpart, x3_rows_per_block(P), hd, DzPool{});
    } else {
        hipLaunchKernelGGL(bn_dz_x3_kernel<0>, dim3(x3_dz_blocks(P)), dim3(256), 0, s, d, y, ld, off, P, C,
                           coef, mask, dz3, bpart, x3_rows_per_block(P), DzHead{}, DzPool{});
    }
    return (int)hipGetLastError();
}

int k_bn_dz_x3_pool(const float* y, int ld, int off, int64_t P, int C, const float* coef, int mask,
                    uint16_t* dz3, float* bpart, const float* dp, const uint8_t* idx, const float* dskip,
                    int ldskip, const float* msc, const float* msh, int N, int H, int W, hipStream_t s) {
    if (C % 32 || (bpart && C > 2048) || ld % 4 || off % 4 || ldskip % 4 || P < 1) return -1;
    if (!dp || !idx || !dskip || H % 2 || W % 2 || (int64_t)N * H * W != P || P >= (1LL << 24)) return -1;
    const DzPool pl{dp, idx, dskip, ldskip, msc, msh, H, W, 1.f / (float)H, 1.f / (float)W};
    hipLaunchKernelGGL(bn_dz_x3_kernel<2>, dim3(x3_dz_blocks(P)), dim3(256), 0, s, nullptr, y, ld, off, P, C,
                       coef, mask, dz3, bpart, x3_rows_per_block(P), DzHead{}, pl);
    return (int)hipGetLastError();
}
