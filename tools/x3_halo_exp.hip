// Experiments on the tap-row halo x3 GEMM (csrc/kernels_gemm_x3.hip rowgemm_x3_row3_kernel):
// a copy of the kernel with schedule flags, timed on the config-2 3x3 GEMM shapes and compared
// bit for bit with the library kernel.  Timing-only flags (XP) compute garbage on purpose.
//   FLAGS: 1 no A DMA, 2 no B DMA, 4 no LDS fragment reads, 8 no waits / barriers (XP);
//          16 s_setprio 1 for waves 4..7; 32 DMA issue after the first k-step's reads;
//          64 stagger: waves 4..7 run each sub-step's second k-step MFMAs after the next
//             barrier from fragments held in registers (MicroArch "two waves per SIMD" item 9)
//          128 the next sub-step's first k-step A fragments read before its barrier when it
//             stays in the same halo group (only B needs the barrier)
//          1024 / 2048 (timing only): B / A DMA from the same rows every sub-step (always L2 hits)
//          256 explicit fragment pipeline (k-step 0 reads, then k-step 1 reads one per k-step-0
//             MFMA, then the k-step-1 MFMAs)
//          8192 (timing only): each 32x32x16 MFMA replaced by two 16x16x32 MFMAs on slices of
//             the same accumulators (the same FLOPs in the other shape; MI355X_MICROARCH.md DVFS
//             item 7: the 16x16x32 loop holds a higher clock)
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/x3_halo_exp.hip -o /tmp/x3_halo_exp
//   run:   /tmp/x3_halo_exp [iters] [flag list, e.g. 0,16,64,80]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <algorithm>
#include <vector>

#include "../thyroid-nodule-image-segmentation-unet-ddti_amd/csrc/kernels_gemm_x3.hip"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

namespace {

__device__ __forceinline__ f32x4 m16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int F>
__device__ __forceinline__ void mx3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16& hi, f32x16& lo) {
    if constexpr (F & 8192) {
        f32x4 l0 = {lo[0], lo[1], lo[2], lo[3]}, l1 = {lo[4], lo[5], lo[6], lo[7]};
        f32x4 h0 = {hi[0], hi[1], hi[2], hi[3]}, h1 = {hi[4], hi[5], hi[6], hi[7]};
        l0 = m16(a[2], b[0], l0); l1 = m16(a[2], b[1], l1);
        l0 = m16(a[1], b[1], l0); l1 = m16(a[1], b[2], l1);
        l0 = m16(a[0], b[2], l0); l1 = m16(a[0], b[0], l1);
        l0 = m16(a[1], b[0], l0); l1 = m16(a[1], b[2], l1);
        l0 = m16(a[0], b[1], l0); l1 = m16(a[0], b[2], l1);
        h0 = m16(a[0], b[0], h0); h1 = m16(a[0], b[1], h1);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            lo[i] = l0[i]; lo[4 + i] = l1[i]; hi[i] = h0[i]; hi[4 + i] = h1[i];
        }
    } else {
        mfma_x3s(a, b, hi, lo);
    }
}

template <int BN, int F, bool LAG>
__device__ __forceinline__ void halo_body(const RowGemmArgs& p, char* smem, int wave, int lane,
                                          f32x16 (&acc)[2][BN / 64], f32x16 (&acl)[2][BN / 64], int m0,
                                          int n0) {
    constexpr int BM = 256, BK = 32, WM = 64, WN = BN / 2, WAVES_N = 2, WAVES = 8;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int RB = 192, AR = 288;
    constexpr int AI = (AR * RB + 1024 * WAVES - 1) / (1024 * WAVES);
    constexpr int BI = (BN * RB + 1024 * WAVES - 1) / (1024 * WAVES);
    constexpr int AREG = AI * WAVES * 1024, BREG = BI * WAVES * 1024;
    auto swz = [](int r) { return (r >> 2) & 3; };
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int H = p.H, W = p.W, C = p.C, K = p.K;
    const int SEG = W < BM ? W : BM, HW = SEG + 2;
    const int AROWS = (BM / SEG) * HW;
    const size_t rowa = 3 * (size_t)p.lda, rowb = 3 * (size_t)K;
    int acen[AI], ayr[AI], ace[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int h = o / RB, w = o - h * RB;
        const int r = h / HW, xl = h - r * HW - 1;
        const int mrow = m0 + r * SEG;
        bool ok = h < AROWS && mrow < p.M;
        const Pix q = decode(ok ? mrow : 0, H, W);
        ok = ok && q.x + xl >= 0 && q.x + xl < W;
        acen[j] = ok ? mrow + xl : -1;
        ayr[j] = q.y;
        ace[j] = (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(h)) << 3);
    }
    const uint16_t* bsrc[BI];
    bool bok[BI];
#pragma unroll
    for (int j = 0; j < BI; ++j) {
        const int o = ((j * WAVES + wave) * 64 + lane) * 16;
        const int r = o / RB, w = o - r * RB;
        bok[j] = r < BN;
        bsrc[j] = p.bt16 + (size_t)(n0 + (bok[j] ? r : 0)) * rowb + (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(r)) << 3);
    }
    const uint16_t* zero = (const uint16_t*)p.zero16;
    const uint16_t* a16 = p.a16 + (size_t)p.aoff * 3;
    const int CC = C / BK;
    auto issue_a = [&](int g) {
        const int dy = (F & 2048) ? 1 : g / CC, c0 = (F & 2048) ? 0 : (g - dy * CC) * BK;  // 2048: L2-hot A
        char* base = smem + (g & 1) * AREG;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            if (F & 1) continue;
            const int yy = ayr[j] + dy - 1;
            const bool valid = acen[j] >= 0 && yy >= 0 && yy < H;
            const uint16_t* src = valid ? a16 + (size_t)(acen[j] + (dy - 1) * W) * rowa + c0 * 3 + ace[j] : zero;
            x3_dma16(src, base + (j * WAVES + wave) * 1024);
        }
    };
    auto issue_b = [&](int s) {
        const int g = s / 3, dx = s - g * 3;
        const int dy = g / CC, c0 = (g - dy * CC) * BK;
        const int k0 = (F & 1024) ? 0 : (dy * 3 + dx) * C + c0;  // 1024: always the same (L2-hot) B rows
        char* base = smem + 2 * AREG + (s & 1) * BREG;
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            if (F & 2) continue;
            x3_dma16(bok[j] ? bsrc[j] + k0 * 3 : zero, base + (j * WAVES + wave) * 1024);
        }
    };
    constexpr int AIX = (F & 1) ? 0 : AI;
    const int lh = lane >> 5, li = lane & 31;
    int ahb[MT], bro[NT], bfx[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int mo = wm * WM + mt * 32 + li;
        const int r = mo / SEG;
        ahb[mt] = r * HW + (mo - r * SEG);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int r = wn * WN + nt * 32 + li;
        bro[nt] = r * RB;
        bfx[nt] = swz(r);
    }
    bf16x8 xa;
#pragma unroll
    for (int j = 0; j < 8; ++j) xa[j] = (__bf16)(float)(lane + j);
    bf16x8 ha[MT][3], hb[NT][3];  // LAG: the previous sub-step's second k-step fragments
    bf16x8 pfa[MT][3];            // 128: the next sub-step's first k-step A fragments (same halo)
    const int ns = 9 * CC;
    issue_a(0);
    issue_b(0);
    for (int s = 0; s < ns; ++s) {
        const int g = s / 3, dx = s - g * 3;
        const bool nb = s + 1 < ns, na = dx == 0 && g + 1 < 3 * CC;
        const bool pa = dx == 1 && g + 1 < 3 * CC;
        if constexpr (!(F & 8)) {
            if (pa) x3_wait_vm<AIX>();
            else x3_wait_vm<0>();
            x3_barrier();
        }
        if constexpr (!(F & 32)) {
            if (nb) issue_b(s + 1);
            if (na) issue_a(g + 1);
        }
        if constexpr (LAG) {
            if (s > 0) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) mx3<F>(ha[mt], hb[nt], acc[mt][nt], acl[mt][nt]);
            }
        }
        const char* abase = smem + (g & 1) * AREG;
        const char* bbase = smem + 2 * AREG + (s & 1) * BREG;
        if constexpr (F & 256) {
            // explicit fragment pipeline: all k-step-0 fragments first, then the k-step-1 reads
            // interleaved one per MFMA with the k-step-0 MFMAs (sched_group_barrier), then the
            // k-step-1 MFMAs: the compiler's own order read ~8 fragments, drained lgkmcnt(0) and
            // ran a few MFMAs, seven times per sub-step
            bf16x8 fa[2][MT][3], fb[2][NT][3];
            auto rd = [&](int kk) {
                const int c = kk * 2 + lh;
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const int h = ahb[mt] + dx;
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        fa[kk][mt][q] = *(const bf16x8*)(abase + h * RB + q * 64 + ((c ^ swz(h)) << 4));
                }
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        fb[kk][nt][q] = *(const bf16x8*)(bbase + bro[nt] + q * 64 + ((c ^ bfx[nt]) << 4));
            };
            auto mm = [&](int kk) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) mx3<F>(fa[kk][mt], fb[kk][nt], acc[mt][nt], acl[mt][nt]);
            };
            rd(0);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (F & 32) {
                if (nb) issue_b(s + 1);
                if (na) issue_a(g + 1);
                __builtin_amdgcn_sched_barrier(0);
            }
            rd(1);
            mm(0);
#pragma unroll
            for (int i = 0; i < 3 * (MT + NT); ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one DS read
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 6 * MT * NT - 3 * (MT + NT), 0);
            __builtin_amdgcn_sched_barrier(0);
            mm(1);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int kk = 0; kk < ((F & 256) ? 0 : BK / 16); ++kk) {
            const int c = kk * 2 + lh;
            bf16x8 af[MT][3], bfr[NT][3];
            if constexpr (F & 4) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int q = 0; q < 3; ++q) af[mt][q] = xa;
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int q = 0; q < 3; ++q) bfr[nt][q] = xa;
            } else {
                if ((F & 128) && kk == 0 && dx > 0) {
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int q = 0; q < 3; ++q) af[mt][q] = pfa[mt][q];
                } else {
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        const int h = ahb[mt] + dx;
#pragma unroll
                        for (int q = 0; q < 3; ++q)
                            af[mt][q] = *(const bf16x8*)(abase + h * RB + q * 64 + ((c ^ swz(h)) << 4));
                    }
                }
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        bfr[nt][q] = *(const bf16x8*)(bbase + bro[nt] + q * 64 + ((c ^ bfx[nt]) << 4));
            }
            if constexpr (F & 32) {
                if (kk == 0) {
                    if (nb) issue_b(s + 1);
                    if (na) issue_a(g + 1);
                }
            }
            if ((F & 128) && kk == 1 && dx < 2) {  // the halo of this group stays: read ahead
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const int h = ahb[mt] + dx + 1;
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        pfa[mt][q] = *(const bf16x8*)(abase + h * RB + q * 64 + ((lh ^ swz(h)) << 4));
                }
            }
            if (LAG && kk == 1) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int q = 0; q < 3; ++q) ha[mt][q] = af[mt][q];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int q = 0; q < 3; ++q) hb[nt][q] = bfr[nt][q];
            } else {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) mx3<F>(af[mt], bfr[nt], acc[mt][nt], acl[mt][nt]);
            }
        }
        if constexpr (!(F & 8)) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if constexpr (LAG) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) mx3<F>(ha[mt], hb[nt], acc[mt][nt], acl[mt][nt]);
    }
    if constexpr (F & 8) x3_wait_vm<0>();
}

// 4096: only waves 0..3 issue LDS-DMA (twice the pieces each; the next group's halo spread over
// the current group's three sub-steps), so that waves 4..7 -- each sharing a SIMD with one
// loader -- keep the matrix pipe busy while their partner pays the DMA issue cost
// (MI355X_MICROARCH.md: 100-185 cycles per piece inside a busy phase).  With 64, waves 4..7 also
// run each sub-step's second k-step MFMAs after the next barrier (held fragments).
template <int BN, int F, bool LOADER, bool LAG>
__device__ __forceinline__ void halo_body_ld(const RowGemmArgs& p, char* smem, int wave, int lane,
                                             f32x16 (&acc)[2][BN / 64], f32x16 (&acl)[2][BN / 64], int m0,
                                             int n0) {
    constexpr int BM = 256, BK = 32, WM = 64, WN = BN / 2, WAVES_N = 2, WAVES = 8, LW = 4;
    constexpr int MT = WM / 32, NT = WN / 32;
    constexpr int RB = 192, AR = 288;
    constexpr int AI8 = (AR * RB + 1024 * WAVES - 1) / (1024 * WAVES);   // region sizes as the
    constexpr int BI8 = (BN * RB + 1024 * WAVES - 1) / (1024 * WAVES);   // 8-wave kernel (LDS map)
    constexpr int AREG = AI8 * WAVES * 1024, BREG = BI8 * WAVES * 1024;
    constexpr int AI = AREG / (1024 * LW), BI = BREG / (1024 * LW);      // pieces per loader wave
    constexpr int AC = (AI + 2) / 3;                                     // halo pieces per sub-step
    auto swz = [](int r) { return (r >> 2) & 3; };
    const int wm = wave / WAVES_N, wn = wave % WAVES_N;
    const int H = p.H, W = p.W, C = p.C, K = p.K;
    const int SEG = W < BM ? W : BM, HW = SEG + 2;
    const int AROWS = (BM / SEG) * HW;
    const size_t rowa = 3 * (size_t)p.lda, rowb = 3 * (size_t)K;
    int acen[LOADER ? AI : 1], ayr[LOADER ? AI : 1], ace[LOADER ? AI : 1];
    const uint16_t* bsrc[LOADER ? BI : 1];
    bool bok[LOADER ? BI : 1];
    if constexpr (LOADER) {
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            const int o = ((j * LW + wave) * 64 + lane) * 16;
            const int h = o / RB, w = o - h * RB;
            const int r = h / HW, xl = h - r * HW - 1;
            const int mrow = m0 + r * SEG;
            bool ok = h < AROWS && mrow < p.M;
            const Pix q = decode(ok ? mrow : 0, H, W);
            ok = ok && q.x + xl >= 0 && q.x + xl < W;
            acen[j] = ok ? mrow + xl : -1;
            ayr[j] = q.y;
            ace[j] = (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(h)) << 3);
        }
#pragma unroll
        for (int j = 0; j < BI; ++j) {
            const int o = ((j * LW + wave) * 64 + lane) * 16;
            const int r = o / RB, w = o - r * RB;
            bok[j] = r < BN;
            bsrc[j] = p.bt16 + (size_t)(n0 + (bok[j] ? r : 0)) * rowb + (w >> 6) * 32 + ((((w >> 4) & 3) ^ swz(r)) << 3);
        }
    }
    const uint16_t* zero = (const uint16_t*)p.zero16;
    const uint16_t* a16 = p.a16 + (size_t)p.aoff * 3;
    const int CC = C / BK;
    const int NG = 3 * CC;  // halo groups
    // halo pieces [j0, j1) of group g
    auto issue_a = [&](int g, int j0, int j1) {
        const int dy = g / CC, c0 = (g - dy * CC) * BK;
        char* base = smem + (g & 1) * AREG;
#pragma unroll
        for (int j = 0; j < AI; ++j) {
            if (j < j0 || j >= j1) continue;
            const int yy = ayr[j] + dy - 1;
            const bool valid = acen[j] >= 0 && yy >= 0 && yy < H;
            const uint16_t* src = valid ? a16 + (size_t)(acen[j] + (dy - 1) * W) * rowa + c0 * 3 + ace[j] : zero;
            x3_dma16(src, base + (j * LW + wave) * 1024);
        }
    };
    auto issue_b = [&](int s) {
        const int g = s / 3, dx = s - g * 3;
        const int dy = g / CC, c0 = (g - dy * CC) * BK;
        const int k0 = (dy * 3 + dx) * C + c0;
        char* base = smem + 2 * AREG + (s & 1) * BREG;
#pragma unroll
        for (int j = 0; j < BI; ++j) x3_dma16(bok[j] ? bsrc[j] + k0 * 3 : zero, base + (j * LW + wave) * 1024);
    };
    // per sub-step s (group g, tap dx): B(s + 1), then halo pieces [dx AC, (dx + 1) AC) of g + 1
    auto issue = [&](int s) {
        const int g = s / 3, dx = s - g * 3;
        if (s + 1 < 9 * CC) issue_b(s + 1);
        if (g + 1 < NG) issue_a(g + 1, dx * AC, dx * AC + AC);
    };
    const int lh = lane >> 5, li = lane & 31;
    int ahb[MT], bro[NT], bfx[NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int mo = wm * WM + mt * 32 + li;
        const int r = mo / SEG;
        ahb[mt] = r * HW + (mo - r * SEG);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int r = wn * WN + nt * 32 + li;
        bro[nt] = r * RB;
        bfx[nt] = swz(r);
    }
    bf16x8 ha[MT][3], hb[NT][3];
    const int ns = 9 * CC;
    if constexpr (LOADER) {
        issue_a(0, 0, AI);
        issue_b(0);
    }
    for (int s = 0; s < ns; ++s) {
        const int g = s / 3, dx = s - g * 3;
        if constexpr (LOADER) {
            // at s: B(s) and (dx = 0) the whole halo of g must have landed; the halo pieces of
            // g + 1 issued at s - 1 (dx >= 1, after B(s)) may stay in flight
            const int pend = (dx >= 1 && g + 1 < NG) ? 1 : 0;
            if (pend) x3_wait_vm<AC>();
            else x3_wait_vm<0>();
        }
        x3_barrier();
        if constexpr (LOADER && !(F & 32)) issue(s);
        if constexpr (LAG) {
            if (s > 0) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) mx3<F>(ha[mt], hb[nt], acc[mt][nt], acl[mt][nt]);
            }
        }
        const char* abase = smem + (g & 1) * AREG;
        const char* bbase = smem + 2 * AREG + (s & 1) * BREG;
#pragma unroll
        for (int kk = 0; kk < BK / 16; ++kk) {
            const int c = kk * 2 + lh;
            bf16x8 af[MT][3], bfr[NT][3];
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const int h = ahb[mt] + dx;
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    af[mt][q] = *(const bf16x8*)(abase + h * RB + q * 64 + ((c ^ swz(h)) << 4));
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    bfr[nt][q] = *(const bf16x8*)(bbase + bro[nt] + q * 64 + ((c ^ bfx[nt]) << 4));
            if constexpr (LOADER && (F & 32)) {
                if (kk == 0) issue(s);
            }
            if (LAG && kk == 1) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int q = 0; q < 3; ++q) ha[mt][q] = af[mt][q];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int q = 0; q < 3; ++q) hb[nt][q] = bfr[nt][q];
            } else {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) mx3<F>(af[mt], bfr[nt], acc[mt][nt], acl[mt][nt]);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if constexpr (LAG) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) mx3<F>(ha[mt], hb[nt], acc[mt][nt], acl[mt][nt]);
    }
}

template <int BN, int F>
__global__ __launch_bounds__(512, 1) void halo_exp_kernel(RowGemmArgs p) {
    constexpr int BM = 256, WM = 64, WN = BN / 2, MT = 2, NT = WN / 32;
    constexpr int RB = 192, AR = 288;
    constexpr int AI = (AR * RB + 8191) / 8192, BI = (BN * RB + 8191) / 8192;
    constexpr int SMEM = 2 * AI * 8192 + 2 * BI * 8192;
    __shared__ __attribute__((aligned(1024))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / 2, wn = wave % 2;
    const int ntn = p.N / BN;
    const int bid = p.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tile_m = bid / ntn, tile_n = bid - tile_m * ntn;
    const int m0 = tile_m * BM, n0 = tile_n * BN;
    f32x16 acc[MT][NT], acl[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = acl[i][j][r] = 0.f;
    if ((F & 16) && wave >= 4) __builtin_amdgcn_s_setprio(1);
    if constexpr (F & 4096) {
        if (wave >= 4)
            halo_body_ld<BN, F, false, (F & 64) != 0>(p, smem, wave, lane, acc, acl, m0, n0);
        else
            halo_body_ld<BN, F, true, false>(p, smem, wave, lane, acc, acl, m0, n0);
    } else if ((F & 64) && wave >= 4)
        halo_body<BN, F, true>(p, smem, wave, lane, acc, acl, m0, n0);
    else
        halo_body<BN, F, false>(p, smem, wave, lane, acc, acl, m0, n0);
    if (F & 16) __builtin_amdgcn_s_setprio(0);
    x3_barrier();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] += acl[mt][nt];
    row_epilogue<E_STORE, BM, BN, WM, WN, true>(p, acc, m0, n0, tile_m, wm, wn, lane, tid, (float*)smem);
}

template <int BN, int F>
int go(const RowGemmArgs& a) {
    hipLaunchKernelGGL((halo_exp_kernel<BN, F>), dim3(((a.M + 255) / 256) * (a.N / BN)), dim3(512), 0, 0, a);
    return (int)hipGetLastError();
}

#define FLAG_LIST(X) X(0) X(1) X(2) X(4) X(7) X(16) X(96) X(112) X(4096) X(4112) X(4128) X(4160) X(4176) X(4192) X(4208)

int run(const RowGemmArgs& a, int bn, int f) {
#define FCASE(v)                                       \
    if (f == v) return bn == 128 ? go<128, v>(a) : go<64, v>(a);
    FLAG_LIST(FCASE)
#undef FCASE
    return -2;
}

__global__ void fill_rand(float* p, size_t n, unsigned seed, float scale, int relu) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        float v = scale * ((x & 0xFFFFFF) / 16777216.0f - 0.5f);
        p[i] = relu ? fmaxf(v, 0.f) : v;
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    std::vector<int> flags = {0, 7, 15, 1, 2, 4, 8, 16, 32, 64, 80};
    if (argc > 2) {
        flags.clear();
        for (char* t = strtok(argv[2], ","); t; t = strtok(nullptr, ",")) flags.push_back(atoi(t));
    }
    struct Shape {
        const char* name;
        int N, H, W, Cin, Cout;
    } shapes[] = {
        {"L1 128->128 @128", 32, 128, 128, 128, 128}, {"L2 256->256 @64", 32, 64, 64, 256, 256},
        {"L3 512->512 @32", 32, 32, 32, 512, 512},    {"L4 1024->1024 @16", 32, 16, 16, 1024, 1024},
        {"L0 64->64 @256 (256x64)", 32, 256, 256, 64, 64},
    };
    void* zero;
    CK(hipMalloc(&zero, 256));
    CK(hipMemset(zero, 0, 256));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (const Shape& sh : shapes) {
        const int M = sh.N * sh.H * sh.W, N = sh.Cout, C = sh.Cin, K = 9 * C;
        const int bn = N % 128 == 0 ? 128 : 64;
        float *x, *w, *yref, *y;
        uint16_t *x3, *w3;
        CK(hipMalloc(&x, (size_t)M * C * 4));
        CK(hipMalloc(&w, (size_t)N * K * 4));
        CK(hipMalloc(&yref, (size_t)M * N * 4));
        CK(hipMalloc(&y, (size_t)M * N * 4));
        CK(hipMalloc(&x3, (size_t)M * C * 6));
        CK(hipMalloc(&w3, (size_t)N * K * 6));
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, x, (size_t)M * C, 17u, 4.f, 1);
        hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, w, (size_t)N * K, 91u, 2.f / sqrtf((float)K), 0);
        CK((hipError_t)k_to_x3(x, C, 0, C, nullptr, nullptr, 0, M, x3, C, 0, 0));
        CK((hipError_t)k_to_x3(w, K, 0, K, nullptr, nullptr, 0, N, w3, K, 0, 0));
        RowGemmArgs h{};
        h.H = sh.H; h.W = sh.W; h.M = M; h.N = N; h.K = K; h.lda = C; h.C = C; h.amode = G_CONV3;
        h.a16 = x3; h.bt16 = w3; h.zero16 = zero; h.ldo = N; h.emode = E_STORE; h.xcd = 1;
        const double fl = 2.0 * M * N * K;
        auto timeit = [&](auto fn) {
            CK((hipError_t)fn());
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < iters; ++i) fn();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            return ms / iters;
        };
        h.out = yref;
        const float tl = timeit([&] { return launch_rowgemm_x3(h, bn == 128 ? 4 : 5, 0); });
        printf("%-26s M=%d N=%d K=%d  library tile %d: %.3f ms %.1f TF/s\n", sh.name, M, N, K,
               bn == 128 ? 4 : 5, tl, fl / tl / 1e9);
        std::vector<float> r((size_t)M * N), q((size_t)M * N);
        CK(hipMemcpy(r.data(), yref, r.size() * 4, hipMemcpyDeviceToHost));
        h.out = y;
        if (bn == 64) {  // the 512 x 64 16-channel-group halo tile (tile 8), schedules 0 / 1
            for (int sc = 0; sc < 2; ++sc) {
                CK(hipMemset(y, 0, (size_t)M * N * 4));
                const float t = timeit([&] { return launch_rowgemm_x3(h, 8, 0, sc); });
                CK(hipMemcpy(q.data(), y, q.size() * 4, hipMemcpyDeviceToHost));
                double dmax = 0, rmx = 0;
                for (size_t i = 0; i < q.size(); ++i) {
                    dmax = std::max(dmax, (double)fabsf(q[i] - r[i]));
                    rmx = std::max(rmx, (double)fabsf(r[i]));
                }
                printf("    library tile 8 (512x64 k16) sched %d: %.3f ms %.1f TF/s  (max |diff| %.3g of %.3g)\n", sc,
                       t, fl / t / 1e9, dmax, rmx);
            }
        }
        if (bn == 64) {  // the 128 x 64 two-blocks-per-CU halo tile
            CK(hipMemset(y, 0, (size_t)M * N * 4));
            const float t = timeit([&] { return launch_rowgemm_x3(h, 6, 0, 0); });
            CK(hipMemcpy(q.data(), y, q.size() * 4, hipMemcpyDeviceToHost));
            const bool same = memcmp(q.data(), r.data(), q.size() * 4) == 0;
            printf("    library tile 6 (128x64, 2/CU): %.3f ms %.1f TF/s  %s\n", t, fl / t / 1e9,
                   same ? "bit-identical" : "DIFFERS");
        }
        const int scheds[] = {1, 9, 12};  // the library's schedules (8.. = 16x16x32)
        double rmax = 0;
        for (float v : r) rmax = std::max(rmax, (double)fabsf(v));
        for (int sc : scheds) {
            CK(hipMemset(y, 0, (size_t)M * N * 4));
            const float t = timeit([&] { return launch_rowgemm_x3(h, bn == 128 ? 4 : 5, 0, sc); });
            CK(hipMemcpy(q.data(), y, q.size() * 4, hipMemcpyDeviceToHost));
            const bool same = memcmp(q.data(), r.data(), q.size() * 4) == 0;
            double dmax = 0;
            for (size_t i = 0; i < q.size(); ++i) dmax = std::max(dmax, (double)fabsf(q[i] - r[i]));
            printf("    library sched %2d: %.3f ms %.1f TF/s  %s (max |diff| %.3g of max |y| %.3g)\n", sc, t,
                   fl / t / 1e9, same ? "bit-identical" : "differs", dmax, rmax);
            fflush(stdout);
        }
        for (int f : flags) {
            CK(hipMemset(y, 0, (size_t)M * N * 4));
            if (run(h, bn, f) == -2) {
                printf("    flags %3d: not built\n", f);
                continue;
            }
            const float t = timeit([&] { return run(h, bn, f); });
            CK(hipMemcpy(q.data(), y, q.size() * 4, hipMemcpyDeviceToHost));
            const bool same = memcmp(q.data(), r.data(), q.size() * 4) == 0;
            printf("    flags %3d: %.3f ms %.1f TF/s  %s\n", f, t, fl / t / 1e9,
                   (f & (3087 | 8192)) ? "(ablation)" : same ? "bit-identical" : "DIFFERS");
            fflush(stdout);
        }
        CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(yref)); CK(hipFree(y)); CK(hipFree(x3)); CK(hipFree(w3));
    }
    return 0;
}
