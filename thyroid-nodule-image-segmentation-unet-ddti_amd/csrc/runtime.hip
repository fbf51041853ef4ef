// Native runtime behind include/unet_hip.h: the layer graph of the reference UNets
// (models/model.py:UNet and models/mod.py:UNet), the workspace plan (NHWC activations,
// zero-copy concat buffers, packed weights, backward scratch) and the forward / backward /
// loss / optimizer orchestration on one HIP stream.
//
// Both reference networks are the same encoder / bottleneck / decoder topology over
// depth D levels of C_l = base << l channels:
//   block l < D      encoder at level l          (model.py encoder{l+1}; mod.py encoders.l)
//   block D          bottleneck at level D       (model.py middle.1;     mod.py bottleneck)
//   block D+1+j      decoder at level D-1-j      (model.py decoder*/final.0; mod.py decoders.j)
//   ConvT k          level D-k -> D-k-1, reads block D+k's output, feeds block D+1+k through
//                    the concat CAT_{D-k-1}      (model.py middle.2/decoder*.1; mod.py upconvs.k)
// and they differ in the order inside a block (model.py:36-41 Conv(+bias) -> ReLU -> BN;
// mod.py:45-50 Conv(no bias) -> BN -> ReLU), the concat order (model.py:64 [up, skip];
// mod.py:64 [skip, up]) and the parameter names / registration order.  mod.py:ResUNet
// (:71-131) has the same skeleton with residual blocks ReLU(conv(x) + skip(x)): there the
// block output is materialised by the 1x1 skip GEMM's epilogue (E_RESID) and every
// consumer reads it plainly.
#include <math.h>
#include <stdlib.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/unet_hip.h"
#include "kernels_misc.h"
#include "x3_split.h"

namespace {

constexpr float BN_EPS = 1e-5f;       // nn.BatchNorm2d default (models/model.py:38,41)
constexpr float BN_MOMENTUM = 0.1f;   // nn.BatchNorm2d default
constexpr int RED_G = 512;            // first-level blocks of the channel reductions
constexpr int WIDE_G = 2048;          // ... of the level-0 bandwidth passes (more loads in flight)
// blocks of a channel-reduction pass over P pixels: RED_G, up to WIDE_G on large levels (the
// partial buffers hold P/64 + 1 rows: p.stats / p.part per conv of the level, p.hpart WIDE_G)
inline int wide_g(int64_t P) { return (int)std::min<int64_t>(WIDE_G, std::max<int64_t>(RED_G, P / 64)); }
constexpr int STAT_G = 256;           // second level of the BN-stat reduction
constexpr int MAX_DEPTH = 6;

// A parameter tensor.  shape / off / numel describe the torch tensor in the caller's flat
// arena (what unet_param_info reports); poff / pshape the same tensor in the context's
// channel-padded arena (== the torch layout unless the network is padded, see
// unet_ctx::padded).  Padded dims are segmented: dim k holds nseg[k] segments of seg[k]
// real entries, each padded to pseg[k] (2 segments for a concat input [skip | up]).
struct ParamT {
    std::string name;
    int ndim;
    int64_t shape[4];
    int64_t off, numel;
    int stage;           // backward stage after which its gradient is final
    int64_t poff, pnumel;
    int64_t seg[4], pseg[4], nseg[4];
};

struct ConvL {
    int cin, cout, level, block, which;
    int64_t w, b;        // param offsets (b < 0: bias-free conv)
    int64_t pf, pd;      // packed weight offsets (floats) inside the pack region
};
struct BnL {
    int C;               // channels the kernels see (padded)
    int rC;              // channels of the torch module (running stats, gamma, beta)
    int64_t g, b;        // gamma / beta offsets in the (padded) parameter arena
    int64_t run;         // running_mean offset in the (padded) bn arena (var at run + C)
    int64_t rrun;        // ... in the caller's bn arena (var at rrun + rC)
    std::string name;
};
struct ConvTL {
    int cin, cout, in_level;
    int64_t w, b;
    int64_t pf, pd;
};

struct TimeRec {
    std::string label;
    hipEvent_t a, b;
    double flop;
};

// Kernel-schedule options of one context (unet_set_option).  The defaults are the
// measured-best schedules; the alternatives exist for A/B runs and tests and are chosen
// explicitly through the ABI (never from the environment).  None of them changes the
// numerics except where noted as bit-identical alternatives in DESIGN.md.
struct Options {
    int wgrad_row3 = 1;        // f32 3x3 wgrad on the one-row-of-taps kernel: 0 never,
                               // 1 every eligible layer (default: r02 A/B, conv wgrad
                               // 27.1 -> 24.4 ms/step), 2 layers with a 64-channel operand
    int wgrad_row3_tile = -1;  // its tile (>= 20), -1 = by channel counts
    int wgrad_blocks = 2048;       // split-K target (blocks) of the one-tap f32 weight gradients
    int rg16_bn_k = 0;             // rg16: E_STORE_BN GEMMs with K below this take the 128x128 tile
                                   // (8192 until the one-barrier halo kernel, r04: 0 is 1-1.5 %
                                   // faster on config 4, profiles/r04_c4_barrier_ab.txt)
    int wgrad16_blocks = 1536;     // split-K target (blocks) of the bf16 weight gradients
                                   // (config 4 A/B: 1536 +1.4 % over 2048, 1024 -4.7 %)
    int wgrad_row3_big = 21;       // row3 tile where Cin, Cout % 128 == 0 (-1 = 23)
    int wgrad_row3_n32 = 1;        // row3 weight gradients for 32-channel operands too (tiles 24..26,
                                   // one / two waves: the split-K target counts four-wave blocks)
    int wgrad_row3_blocks = 1536;  // split-K target (blocks) of the row3 weight gradients
                                   // (r02 sweep 512..2048: 1536 best, 391 vs 386 img/s)
    int wgrad_tile_w = 0;      // f32 wgrad tile, both channel counts multiples of 128
    int wgrad_tile_n = 7;      // ... 64-channel layers (64x64, 3 waves/SIMD)
    int tile_n128 = -1;        // f32 row-GEMM tile, N % 128 == 0 (-1 = pick_tile's default)
    int tile_n128_dgrad = -1;  // ... dgrad-type
    int tile_n64 = 19;         // ... N = 64 outputs (forward-type)
    int tile_n64_dgrad = 25;   // ... N = 64, dgrad-type (pipelined 128x64 at three blocks per
                               // CU: level-0 dgrads 1.50-1.55 -> 1.40-1.45 ms, r03)
    int tile_convt64 = 1;      // ConvT forward with 64 output channels (grid N = 256)
    int tile_n32 = 15;         // f32 row GEMMs with 32 outputs: 15 = 256 x 32 with operands
                               // straight from global memory (r04, ResUNet(32, 4) 263 -> 282
                               // img/s, (16, 4) 419 -> 478), 14 = the LDS-staged 256 x 32
    int tile_convt = -1;       // ConvT forward, >= 128 output channels (-1 = tile_n128's)
    int tile_convt_dgrad = 26; // ConvT input gradient (-1 = tile_n128_dgrad's; 26 = pipelined
                               // 128x64 at three blocks per CU: the K = 4 Cout short-K GEMMs
                               // with their BN-partials epilogue, 1.33 -> 1.15 ms per step)
    int rg16 = 1;              // bf16 row GEMMs on the LDS-DMA kernel (0: register-staged)
    int rg16_tile = -1;        // its tile (-1 = per GEMM, rg16_tile())
    int rg16_n128 = 20;        // rg16 tile of the GEMMs whose N is not a multiple of 256 (the
                               // 128-output layers; -1 = 128x128, 6 = 512x128, 20 = 512x128 tap-row
                               // halo for 3x3 convs, 6 elsewhere; r04 config 4: 122.7 -> 124.8
                               // img/s with 20, 121.9 with 6)
    int rg16_n128_bn = 0;      // ... also for the short-K E_STORE_BN GEMMs (else 128x128)
    int rg16_r3 = 1;           // 256x256 3x3-conv GEMMs (W >= 16) on the tap-row halo kernel (tile 19;
                               // config 4: +0.9..1.2 % over three A/B pairs, r03)
    int wg16 = 1;              // bf16 3x3 wgrad on the LDS-DMA transposed-read kernel
    int wg16_tile = 2;         // its tile (2 = 256x256)
    int convt16 = 1;           // bf16 training: the ConvT forward stores the up half of the
                               // decoder's concat straight into that conv's bf16 operand image
                               // (no f32 up half; its prep pass converts the skip half only)
    int wg16_r3 = 7;           // 3x3 layers with W % 64 == 0 on the tap-row bf16 weight gradient:
                               // 7 = 16x16x32 MFMAs with the re-read stagger (r06, config 4
                               // +1.3 % over 4, profiles/r06_c4_wg16_ab.txt; also at W = 32 / 16,
                               // +1.4 %, r06_c4_deep_wgrad_ab.txt), 4 = 32x32x16, four LDS stages
                               // (r04: 122.7 -> 125.2 img/s), 0 = off (one-tap kernel)
    int wg16t = 1;             // bf16 ConvT wgrad on the same kernel
    int xcd16 = 1;             // XCD-contiguous block order, LDS-DMA kernels
    int xcd_remap = 1;         // ... f32 GEMMs: 0 none, 1 both (default: r03 PMC, HBM bytes
                               // per launch rowgemm 128x128 2.21 -> 1.00 GB, row3 wgrad
                               // 2.02 -> 0.97 GB at equal time), 2 row GEMMs, 3 wgrad
    int dz_in_wgrad = 256;     // layers with Cin <= this form the BN-backward dz in the weight
                               // gradient's B' loader, which also stores it for the dgrad (no
                               // bn_dz pass; f32, both BN orders since r04; 0 = off).  Every A'-tile row of
                               // blocks re-reads do and y instead of dz, so the fusion pays
                               // where few A' tiles share a pixel slice (profiles/
                               // r03_tile_experiments.txt: Cin 64..256 gain, 512..1024 lose)
    int x3 = 1;                // f32 math: conv / ConvT GEMMs whose channel counts are multiples
                               // of 64 on the bf16 matrix cores through exact three-way operand
                               // splits (kernels_gemm_x3.hip; fp64 error below the f32 MFMA
                               // kernels'); 0 = the f32 MFMA kernels everywhere
    int x3_tile = -1;          // its row-GEMM tile (-1 = x3_tile())
    int x3_wtile = -1;         // its weight-gradient tile (-1 = by channel counts)
    int x3_wblocks = 1536;     // split-K target (blocks) of its 128x128 weight gradients
    int x3_n64 = 2;            // its row-GEMM tile for 64 outputs (2 = 128x64, 3 = 256x64)
    int x3_r3 = 1;             // its 256x128 3x3 GEMMs on the tap-row halo kernel (tile 4)
    int x3_wwaves = 3;         // tap-row x3 weight gradients: split-K so the grid is this many full
                               // waves of block slots (0 = the x3_wblocks target; r05,
                               // profiles/r05_wwaves_ab.txt)
    int x3_wwaves1 = 3;        // the same for the one-tap x3 weight gradients (ConvT, 8x8):
                               // +0.45 % (profiles/r05_wwaves_ab.txt)
    int pool_fuse = 1;         // x3 and (r06) bf16 paths: the encoder block's second conv recomputes its `do` from
                               // the max-pool backward's inputs instead of maxpool_bwd storing it
    int head_fuse = 1;         // x3 (r05) and bf16 (r06) paths, one output channel: the last conv's dz
                               // pass recomputes `do` from the head instead of head_bwd storing it
    int tile_group = 1;        // (r06) row-GEMM tile order of the LDS-DMA kernels (rg16, x3): 1 = grouped
                               // where the N tiles are many (tile_group_auto), 0 = M-major (r05);
                               // bit-identical
};
struct OptionDesc {
    const char* name;
    int Options::*field;
};
// (include/unet_hip.h lists these names; tests/test_lib_cpu.py checks the two agree)
const OptionDesc OPTION_TABLE[] = {
    {"wgrad_row3", &Options::wgrad_row3},
    {"wgrad_row3_tile", &Options::wgrad_row3_tile},
    {"wgrad_row3_big", &Options::wgrad_row3_big},
    {"wgrad_row3_blocks", &Options::wgrad_row3_blocks},
    {"wgrad_row3_n32", &Options::wgrad_row3_n32},
    {"wgrad_blocks", &Options::wgrad_blocks},
    {"wgrad16_blocks", &Options::wgrad16_blocks},
    {"wgrad_tile_w", &Options::wgrad_tile_w},
    {"wgrad_tile_n", &Options::wgrad_tile_n},
    {"tile_n128", &Options::tile_n128},
    {"tile_n128_dgrad", &Options::tile_n128_dgrad},
    {"tile_n64", &Options::tile_n64},
    {"tile_n64_dgrad", &Options::tile_n64_dgrad},
    {"tile_n32", &Options::tile_n32},
    {"tile_convt64", &Options::tile_convt64},
    {"tile_convt", &Options::tile_convt},
    {"tile_convt_dgrad", &Options::tile_convt_dgrad},
    {"rg16", &Options::rg16},
    {"rg16_tile", &Options::rg16_tile},
    {"rg16_bn_k", &Options::rg16_bn_k},
    {"rg16_r3", &Options::rg16_r3},
    {"rg16_n128", &Options::rg16_n128},
    {"rg16_n128_bn", &Options::rg16_n128_bn},
    {"wg16", &Options::wg16},
    {"wg16_tile", &Options::wg16_tile},
    {"wg16_r3", &Options::wg16_r3},
    {"convt16", &Options::convt16},
    {"wg16t", &Options::wg16t},
    {"xcd16", &Options::xcd16},
    {"xcd_remap", &Options::xcd_remap},
    {"dz_in_wgrad", &Options::dz_in_wgrad},
    {"x3", &Options::x3},
    {"x3_tile", &Options::x3_tile},
    {"x3_wtile", &Options::x3_wtile},
    {"x3_wblocks", &Options::x3_wblocks},
    {"x3_n64", &Options::x3_n64},
    {"x3_r3", &Options::x3_r3},
    {"head_fuse", &Options::head_fuse},
    {"pool_fuse", &Options::pool_fuse},
    {"x3_wwaves", &Options::x3_wwaves},
    {"x3_wwaves1", &Options::x3_wwaves1},
    {"tile_group", &Options::tile_group},
};

}  // namespace

struct unet_ctx {
    int device = 0;
    int cus = 256;  // compute units of the device (split-K sizing by whole waves of block slots)
    int in_ch = 1, out_ch = 1;
    int variant = UNET_VARIANT_MODEL;
    int base = 64, depth = 4;  // base: channels of level 0 as the kernels see them (padded)
    int rbase = 64;            // base_filters of the reference module (models/mod.py:13)
    // Narrow networks (base_filters 16 / 24 / 32 / 48 of the reference's model grid,
    // config/config.yaml) run with every level's channels zero-padded to the next power of
    // two >= 64, the widths the GEMM tiles and channel-quad kernels are built for.  The
    // caller's arenas keep the torch layouts; unet_forward / unet_backward expand them
    // into padded arenas in the workspace (zeros in the padding: zero weights, gamma,
    // beta, so padded channels stay exactly 0 through BN / ReLU / pooling / ConvT / the
    // head and add +0 to every real sum) and compact the running stats and gradients back.
    bool padded = false;
    bool bn_relu = false;    // BN -> ReLU (mod.py) instead of ReLU -> BN (model.py)
    bool skip_first = false; // concat [skip, up] (mod.py) instead of [up, skip] (model.py)
    bool bf16 = false;       // conv GEMMs on bf16 MFMA (f32 accumulate), BASELINE config 4
    bool res = false;        // residual blocks (mod.py:ResUNet): block outputs materialised
    std::vector<ParamT> params;
    int64_t n_param_floats = 0;   // caller's (torch-layout) arena
    int64_t n_pparam_floats = 0;  // padded arena (== n_param_floats unless padded)
    std::vector<ConvL> conv;
    std::vector<BnL> bn;
    std::vector<ConvTL> convt;
    std::vector<int64_t> skip_w, skip_pd;  // per block: 1x1 skip weight, its dgrad image
    int64_t head_w = 0, head_b = 0;
    int64_t n_bn_floats = 0;      // caller's running-stat arena
    int64_t n_pbn_floats = 0;     // padded
    int64_t pack_floats = 0;
    std::vector<PadDesc> pad_params, pad_bn;  // expand / compact tables (padded only)
    int64_t pad_max_numel = 0, pad_bn_max = 0;
    int cmax = 0;
    std::string err;
    // buckets (DP overlap): contiguous grad ranges, ready after backward stage bucket_stage
    std::vector<int64_t> bucket_off, bucket_len;
    std::vector<int> bucket_stage;
    std::vector<int> bucket_p0, bucket_p1;     // parameter tensors [p0, p1) of each bucket
    std::vector<int64_t> bucket_pmax;          // ... their largest padded numel
    std::vector<hipEvent_t> bucket_ev;
    // timing
    bool timing = false;
    std::string tfilter;  // time only launches whose label contains this (empty = all)
    std::vector<TimeRec> trec;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    Options opt;
    // the options of the last training forward: the workspace plan and which saved images
    // exist (x3, convt16, the bf16 kernels, ...) depend on them, so unet_backward refuses to
    // run under different ones (it would read saved activations at shifted offsets, or an
    // up half the forward never wrote)
    Options fwd_opt;
    bool fwd_opt_set = false;
    // (r06) weight images written by unet_adamw_repack (AdamW fused into the repack): device
    // buffers owned by the context, valid for the parameter arena `pp_src` until
    // unet_params_changed or another repack; pp_gen counts repacks, and a training forward that
    // read them records the generation its backward must still see
    float* pp = nullptr;
    uint16_t* pp3 = nullptr;
    // (r06) per-chunk loss statistics of unet_loss_stats (4 floats per chunk, grown on demand)
    float* lpart = nullptr;
    int64_t lpart_n = 0;
    const float* pp_src = nullptr;
    bool pp_ok = false;
    uint64_t pp_gen = 0;
    bool fwd_used_pp = false;
    uint64_t fwd_pp_gen = 0;

    int nconv() const { return (int)conv.size(); }
    int chl[MAX_DEPTH + 1] = {};                           // kernel (padded) channels per level
    int ch(int level) const { return chl[level]; }         // kernel (padded) channels
    int rch(int level) const { return rbase << level; }   // torch module channels
    int up_off(int l) const { return skip_first ? ch(l) : 0; }    // CAT_l channel offsets
    int skip_off(int l) const { return skip_first ? 0 : ch(l); }
};

namespace {

int fail(unet_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) {
        try {
            c->err = buf;
        } catch (...) {  // out of memory for the message itself: keep the code
        }
    }
    return code;
}

// Every extern "C" entry runs its body inside ABI_TRY / ABI_CATCH(ctx): no C++ exception
// (std::bad_alloc from the graph / plan / timing containers, ...) unwinds into the caller.
#define ABI_TRY try {
#define ABI_CATCH(ctx)                                                                      \
    }                                                                                       \
    catch (const std::bad_alloc&) {                                                         \
        return fail(const_cast<unet_ctx*>(ctx), UNET_ERR_NOMEM, "out of host memory");       \
    }                                                                                       \
    catch (const std::exception& e_) {                                                      \
        return fail(const_cast<unet_ctx*>(ctx), UNET_ERR_INTERNAL, "internal error: %s",     \
                    e_.what());                                                             \
    }                                                                                       \
    catch (...) {                                                                           \
        return fail(const_cast<unet_ctx*>(ctx), UNET_ERR_INTERNAL, "internal error");        \
    }

// Parameter table in the reference's named_parameters() order, layer tables, packing
// offsets and gradient buckets.
// One dimension of a parameter tensor: nseg segments of seg real entries, each padded to
// pseg entries (nseg = 2 for the [skip | up] concat input of a decoder block).
struct Dim {
    int64_t seg, pseg, nseg;
};

void build_graph(unet_ctx* c) {
    const int D = c->depth;
    const int nb = 2 * D + 1;
    c->conv.assign(2 * nb, ConvL{});
    c->bn.assign(2 * nb, BnL{});
    c->convt.assign(D, ConvTL{});
    c->params.clear();
    int64_t off = 0, poff = 0;
    // returns the tensor's offset in the padded arena (what the kernels index)
    auto add = [&](const std::string& name, std::initializer_list<Dim> dims, int stage) {
        ParamT p;
        p.name = name;
        p.ndim = (int)dims.size();
        p.numel = 1;
        p.pnumel = 1;
        int i = 0;
        for (const Dim& d : dims) {
            p.shape[i] = d.seg * d.nseg;
            p.seg[i] = d.seg;
            p.pseg[i] = d.pseg;
            p.nseg[i] = d.nseg;
            p.numel *= d.seg * d.nseg;
            p.pnumel *= d.pseg * d.nseg;
            ++i;
        }
        for (; i < 4; ++i) {
            p.shape[i] = 0;
            p.seg[i] = p.pseg[i] = p.nseg[i] = 1;
        }
        p.off = off;
        p.poff = poff;
        p.stage = stage;
        off += p.numel;
        poff += p.pnumel;
        c->params.push_back(p);
        return p.poff;
    };
    auto level_of = [&](int b) { return b <= D ? b : 2 * D - b; };
    auto lvl = [&](int l) { return Dim{c->rch(l), c->ch(l), 1}; };  // one level's channels
    auto block_cin = [&](int b) {  // kernel (padded) input channels of block b
        if (b == 0) return c->in_ch;
        if (b <= D) return c->ch(b - 1);
        return 2 * c->ch(level_of(b));
    };
    auto block_in_dim = [&](int b) {  // the same as a torch dimension
        if (b == 0) return Dim{c->in_ch, c->in_ch, 1};
        if (b <= D) return lvl(b - 1);
        return Dim{c->rch(level_of(b)), c->ch(level_of(b)), 2};  // concat of two halves
    };
    const Dim k3{3, 3, 1}, k2{2, 2, 1}, k1{1, 1, 1};
    // backward stage after which a block's gradients are final: 0 = head + last decoder,
    // then ConvT k together with block D+k (k = D-1 .. 0), then the encoders
    auto stage_of_block = [&](int b) { return 2 * D - b; };
    // 3x3 conv + BN pair `which` of block b; names per variant
    auto conv_pair = [&](int b, int which, const std::string& pfx) {
        const int i = 2 * b + which;
        ConvL& L = c->conv[i];
        L.cout = c->ch(level_of(b));
        L.cin = which == 0 ? block_cin(b) : L.cout;
        L.level = level_of(b);
        L.block = b;
        L.which = which;
        BnL& B = c->bn[i];
        B.C = L.cout;
        B.rC = c->rch(L.level);
        const Dim dout = lvl(L.level), din = which == 0 ? block_in_dim(b) : dout;
        const int st = stage_of_block(b);
        const std::string cp = c->res ? pfx + ".conv" : pfx;  // ResidualBlock.conv (mod.py:75)
        L.w = add(cp + (which ? ".3.weight" : ".0.weight"), {dout, din, k3, k3}, st);
        if (c->variant == UNET_VARIANT_MODEL) {  // model.py:33-43: 0 conv, 2 BN, 3 conv, 5 BN
            L.b = add(pfx + (which ? ".3.bias" : ".0.bias"), {dout}, st);
            B.name = pfx + (which ? ".5" : ".2");
        } else {  // mod.py:43-51 / :75-81: 0 conv (no bias), 1 BN, 3 conv, 4 BN
            L.b = -1;
            B.name = cp + (which ? ".4" : ".1");
        }
        B.g = add(B.name + ".weight", {dout}, st);
        B.b = add(B.name + ".bias", {dout}, st);
    };
    c->skip_w.assign(nb, -1);
    c->skip_pd.assign(nb, -1);
    auto block = [&](int b, const std::string& pfx) {
        conv_pair(b, 0, pfx);
        conv_pair(b, 1, pfx);
        if (c->res)  // ResidualBlock.skip, Conv2d(in, out, 1, bias=False) (mod.py:83)
            c->skip_w[b] = add(pfx + ".skip.weight", {lvl(level_of(b)), block_in_dim(b), k1, k1},
                               stage_of_block(b));
    };
    auto convT = [&](int k, const std::string& name) {
        ConvTL& T = c->convt[k];
        T.in_level = D - k;
        T.cin = c->ch(D - k);
        T.cout = c->ch(D - k - 1);
        const int st = stage_of_block(D + k);
        T.w = add(name + ".weight", {lvl(D - k), lvl(D - k - 1), k2, k2}, st);
        T.b = add(name + ".bias", {lvl(D - k - 1)}, st);
    };
    const Dim dout_head{c->out_ch, c->out_ch, 1};
    if (c->variant == UNET_VARIANT_MODEL) {
        // models/model.py:6-31 registration order (D = 4, base 64)
        const char* bname[9] = {"encoder1", "encoder2", "encoder3", "encoder4", "middle.1",
                                "decoder3.0", "decoder2.0", "decoder1.0", "final.0"};
        const char* tname[4] = {"middle.2", "decoder3.1", "decoder2.1", "decoder1.1"};
        for (int b = 0; b <= D; ++b) block(b, bname[b]);
        for (int k = 0; k < D; ++k) {
            convT(k, tname[k]);
            block(D + 1 + k, bname[D + 1 + k]);
        }
        c->head_w = add("final.1.weight", {dout_head, lvl(0), k1, k1}, 0);
        c->head_b = add("final.1.bias", {dout_head}, 0);
    } else {
        // models/mod.py:21-41: encoders, (pools), bottleneck, upconvs, decoders, final_conv
        for (int l = 0; l < D; ++l) block(l, "encoders." + std::to_string(l));
        block(D, "bottleneck");
        for (int k = 0; k < D; ++k) convT(k, "upconvs." + std::to_string(k));
        for (int k = 0; k < D; ++k) block(D + 1 + k, "decoders." + std::to_string(k));
        c->head_w = add("final_conv.weight", {dout_head, lvl(0), k1, k1}, 0);
        c->head_b = add("final_conv.bias", {dout_head}, 0);
    }
    c->n_param_floats = off;
    c->n_pparam_floats = poff;
    int64_t run = 0, rrun = 0;
    for (auto& B : c->bn) {  // named_buffers() order == conv order in both variants
        B.run = run;
        B.rrun = rrun;
        run += 2 * B.C;
        rrun += 2 * B.rC;
    }
    c->n_bn_floats = rrun;
    c->n_pbn_floats = run;
    // expand / compact tables (the bn arena: mean and var vectors of each layer)
    c->pad_params.clear();
    c->pad_bn.clear();
    c->pad_max_numel = c->pad_bn_max = 0;
    if (c->padded) {
        for (const ParamT& p : c->params) {
            PadDesc d{p.off, p.poff, p.numel, p.pnumel, {1, 1, 1, 1}, {1, 1, 1, 1}, {1, 1, 1, 1}};
            for (int k = 0; k < 4; ++k) {
                d.seg[k] = (int32_t)p.seg[k];
                d.pseg[k] = (int32_t)p.pseg[k];
                d.nseg[k] = (int32_t)p.nseg[k];
            }
            c->pad_params.push_back(d);
            c->pad_max_numel = std::max(c->pad_max_numel, p.pnumel);
        }
        for (const BnL& B : c->bn)
            for (int v = 0; v < 2; ++v) {
                PadDesc d{B.rrun + v * B.rC, B.run + v * B.C, B.rC, B.C,
                          {B.rC, 1, 1, 1}, {B.C, 1, 1, 1}, {1, 1, 1, 1}};
                c->pad_bn.push_back(d);
                c->pad_bn_max = std::max<int64_t>(c->pad_bn_max, B.C);
            }
    }
    c->cmax = 0;
    for (auto& L : c->conv) c->cmax = std::max(c->cmax, std::max(L.cin, L.cout));
    // packed weights (forward + dgrad images); conv 0 (Cin = in_channels) has its own kernel
    int64_t pk = 0;
    for (int i = 0; i < c->nconv(); ++i) {
        ConvL& L = c->conv[i];
        const int64_t n = (int64_t)L.cin * L.cout * 9;
        if (i == 0 && L.cin < 32) {
            L.pf = L.pd = -1;
            continue;
        }
        // (every image starts at a multiple of 32 floats: the x3 copy of the whole region,
        // converted as rows of 32, then holds each image's x3 image at 3x its offset)
        L.pf = pk;
        pk += (n + 31) / 32 * 32;
        L.pd = pk;
        pk += (n + 31) / 32 * 32;
    }
    for (auto& T : c->convt) {
        const int64_t n = (int64_t)T.cin * T.cout * 4;
        T.pf = pk;
        pk += (n + 31) / 32 * 32;
        T.pd = pk;
        pk += (n + 31) / 32 * 32;
    }
    for (int b = 1; b < nb && c->res; ++b) {  // transposed skip images for the dgrad
        c->skip_pd[b] = pk;
        pk += ((int64_t)c->conv[2 * b].cin * c->conv[2 * b].cout + 31) / 32 * 32;
    }
    c->pack_floats = pk;
    // gradient buckets: walk the arena from its end (what backward finishes first), open a
    // new bucket whenever a tensor finishes later than everything already in the current one
    // (so buckets become ready in order 0, 1, ...); tensors that finish earlier join it
    c->bucket_off.clear();
    c->bucket_len.clear();
    c->bucket_stage.clear();
    int64_t end = c->n_param_floats;
    int cur = -1;
    for (int t = (int)c->params.size() - 1; t >= 0; --t) {
        const ParamT& p = c->params[t];
        if (cur >= 0 && p.stage > cur) {
            c->bucket_off.push_back(p.off + p.numel);
            c->bucket_len.push_back(end - (p.off + p.numel));
            c->bucket_stage.push_back(cur);
            end = p.off + p.numel;
            cur = -1;
        }
        cur = std::max(cur, p.stage);
    }
    c->bucket_off.push_back(0);
    c->bucket_len.push_back(end);
    c->bucket_stage.push_back(cur);
    // the parameter tensors of each bucket (contiguous in arena order): a channel-padded
    // network compacts exactly these into the caller's arena before the bucket's event
    c->bucket_p0.assign(c->bucket_off.size(), 0);
    c->bucket_p1.assign(c->bucket_off.size(), 0);
    c->bucket_pmax.assign(c->bucket_off.size(), 0);
    for (size_t b = 0; b < c->bucket_off.size(); ++b) {
        int p0 = -1, p1 = -1;
        for (int t = 0; t < (int)c->params.size(); ++t) {
            const ParamT& q = c->params[t];
            if (q.off >= c->bucket_off[b] && q.off + q.numel <= c->bucket_off[b] + c->bucket_len[b]) {
                if (p0 < 0) p0 = t;
                p1 = t + 1;
                c->bucket_pmax[b] = std::max(c->bucket_pmax[b], q.pnumel);
            }
        }
        c->bucket_p0[b] = p0 < 0 ? 0 : p0;
        c->bucket_p1[b] = p1 < 0 ? 0 : p1;
    }
}

// ------------------------------------------------------------------------------------
// Workspace plan.  A bump allocator over the caller's buffer; the same function sizes and
// carves it so forward and backward agree on every pointer.
// ------------------------------------------------------------------------------------
struct Plan {
    int N, H, W;
    int64_t P[MAX_DEPTH + 1];  // pixels per level
    float* pack;
    float* x_nhwc;
    std::vector<float*> y;
    std::vector<int> ldy, offy;
    std::vector<float*> scale, shift, mean, invstd;
    float* cat[MAX_DEPTH];
    float* cat_scale[MAX_DEPTH];
    float* cat_shift[MAX_DEPTH];
    float* pool[MAX_DEPTH];
    uint8_t* idx[MAX_DEPTH];
    std::vector<float*> out;  // residual network: block outputs (ld, off)
    std::vector<int> ldout, offout;
    float* stats;
    float* stats2;
    // backward
    float* g[3];
    float* dcat[MAX_DEPTH];
    float* slab;
    float* part;   // BN-backward column partials [rows][2][C]
    float* part2;  // second-level reduction of part
    float* hpart;  // head / conv-first weight-gradient partials
    float* bslab;  // [splits][Nw] bias-gradient column sums from the wgrad kernels
    float* coef;
    float* gdz;    // option dz_in_wgrad: the dz the weight gradient stores for the dgrad
    // bf16 LDS-DMA GEMMs: prepared operand image (dense [pixels][C] bf16) and a zero page
    uint16_t* s16;
    void* zero16;
    std::vector<uint16_t*> x16;  // training, bf16: per-conv input images kept for the wgrad
    std::vector<uint16_t*> t16;  // training, bf16: per-ConvT input images kept for the wgrad
    // f32 GEMMs on split bf16 operands (option x3): x3 copy of the weight images, per-conv /
    // per-ConvT input images kept for the weight gradients, one scratch image
    uint16_t* pack3;
    uint16_t* s3;
    std::vector<uint16_t*> x3;
    std::vector<uint16_t*> t3;
    // channel-padded networks: padded parameter / running-stat / gradient arenas and the
    // device copies of the expand / compact tables
    float* pprm;
    float* pbn;
    float* pgrad;
    float* ugrad;  // padded network: the caller's (torch-layout) gradient arena
    PadDesc* ptab;
    PadDesc* btab;
    size_t bytes;
};

struct Bump {
    char* base;
    size_t off = 0;
    template <class T>
    T* take(int64_t n) {
        off = (off + 255) & ~(size_t)255;
        T* p = base ? (T*)(base + off) : nullptr;
        off += (size_t)n * sizeof(T);
        return p;
    }
};

struct WgradCfg {
    int tile, bm, bn, bkp, splits, pps;
};

// wgrad tile (kernels_gemm.hip WGRAD_TILES) + split-K over pixels so that every layer
// launches >= 2048 blocks; options wgrad_tile_{w,n} override (tuning runs).
// row_w: row width of a 3x3 conv's pixel grid (0 otherwise).  3x3 weight gradients on
// rows that are a multiple of 32 pixels take the one-row-of-taps tiles (ids 20..,
// wgrad_row3_kernel) when option wgrad_row3 selects them: 1 = every eligible layer,
// 2 = only layers with a 64-channel operand (the 256x256 / 128x128 levels), 0 = never.
// The split-K partition follows from the (default) tile dims; the bf16 LDS-DMA weight
// gradient (wg16_tile) reuses the register-staged tile's partition, so its tile choice
// never changes the summation order.
WgradCfg wgrad_cfg(const unet_ctx* c, int CA, int tapsA, int CB, int tapsB, int64_t P, bool bf16,
                   int row_w = 0) {
    const int r3 = c->opt.wgrad_row3, r3t = c->opt.wgrad_row3_tile;
    const int tw = c->opt.wgrad_tile_w, tn = c->opt.wgrad_tile_n;
    WgradCfg w;
    if (bf16) {  // kernels_gemm.hip WGRAD16_TILES
        w.tile = (CA % 128 == 0 && CB % 128 == 0) ? 0 : CA % 128 == 0 ? 3 : CB % 128 == 0 ? 4 : 2;
        wgrad16_tile_dims(w.tile, &w.bm, &w.bn, &w.bkp);
    } else {
        if (CA % 128 == 0 && CB % 128 == 0)
            w.tile = tw;
        else if (CA % 64 == 0 && CB % 64 == 0 && (CA % 128 || CB % 128) && tn >= 0)
            w.tile = (CA % 128 == 0) ? 5 : (CB % 128 == 0 ? 3 : tn);
        else if (CA % 64)  // 32-channel operands (narrow networks' level 0)
            w.tile = 9;
        else if (CB % 64)
            w.tile = 8;
        else
            w.tile = 7;
        const bool row3 = tapsA == 9 && tapsB == 1 && row_w > 0 && row_w % 32 == 0 &&
                          CA % 32 == 0 && CB % 32 == 0 &&
                          (r3 == 1 || (r3 == 2 && (CA == 64 || CB == 64)));
        const bool r3n = CA % 64 || CB % 64;  // a 32-channel operand (r04 tiles 24..26)
        if (row3 && r3n && c->opt.wgrad_row3_n32) {
            w.tile = CA % 64 ? (CB % 64 ? 24 : 26) : 25;
        } else if (row3 && !r3n) {
            w.tile = r3t >= 20 ? r3t
                               : (CA % 128 == 0 ? (CB % 128 == 0 ? 23 : 21) : (CB % 128 == 0 ? 22 : 20));
            // option wgrad_row3_big: the tile of the layers whose channel counts both divide
            // 128.  Default 128x64 (21) rather than 128x128 (23): the same GEMM time (126 TF/s)
            // but twice the tiles, so the 1536-block target needs half the split-K slices and
            // the slab reduction halves (r02 A/B: wgrad_reduce 1.09 -> 0.64 ms, 404 -> 408 img/s)
            if (r3t < 20 && c->opt.wgrad_row3_big >= 20 && CA % 128 == 0 && CB % 128 == 0)
                w.tile = c->opt.wgrad_row3_big;
        }
        wgrad_tile_dims(w.tile, &w.bm, &w.bn, &w.bkp);
    }
    const int64_t tiles =
        (int64_t)(tapsA * CA / (w.bm * wgrad_tile_taps(w.tile))) * (tapsB * CB / w.bn);
    // blocks to launch: 2048 one-tap blocks; a row3 block does the work of three, and every
    // extra split adds a full Mw x Nw slab to write and reduce
    const int64_t target = bf16 ? c->opt.wgrad16_blocks
                                : (w.tile >= 20 ? c->opt.wgrad_row3_blocks : c->opt.wgrad_blocks) *
                                      (w.tile == 24 ? 4 : (w.tile == 25 || w.tile == 26) ? 2 : 1);
    int64_t s = (target + tiles - 1) / tiles;
    const int64_t maxs = P / (8 * w.bkp) > 0 ? P / (8 * w.bkp) : 1;  // >= 8 chunks per split
    // (P need not be a multiple of the pixel chunk: the kernel zero-fills the tail)
    if (s > maxs) s = maxs;
    if (s < 1) s = 1;
    int64_t pps = (P + s - 1) / s;
    pps = (pps + 127) / 128 * 128;
    // (r06) bf16 3x3 weight gradients on the tap-row kernel (W % 64 == 0): the 1536-block target
    // above, counted in one-tap 128x128 tiles, launches (CA / 128) 3 (CB / 128) tap-row blocks
    // per split, i.e. 513-576 blocks on 256 one-block-per-CU slots -- a third wave holding 1-64
    // blocks, and the kernel took three block durations instead of two.  Instead pick the split
    // count s minimising waves(s) x chunks per block(s) + the slab traffic of s splits (the
    // one-tap kernel, option wg16_r3 = 0, gets the same partition: bit-identical).
    // (W = 32 / 16: the deep levels' tap-row instances, wg16_r3 = 7, r06)
    if (bf16 && tapsA == 9 && tapsB == 1 && row_w > 0 && (row_w % 64 == 0 || row_w == 32 || row_w == 16) &&
        CA % 128 == 0 && CB % 128 == 0 && P % 64 == 0) {
        const int64_t t3 = (int64_t)(CA / 128) * 3 * (CB / 128);
        const int64_t slots = c->cus;
        double best = -1;
        for (int64_t sc = 1; sc <= maxs; ++sc) {
            const int64_t waves = (t3 * sc + slots - 1) / slots;
            const int64_t chunks = (P + 64 * sc - 1) / (64 * sc);
            // ~1.2 us per 64-pixel chunk of a 128x128x3 block; slabs written and reduced at ~5 TB/s
            const double cost = waves * chunks * 1.2e-6 + sc * 9.0 * CA * CB * 8 / 5e12;
            if (best < 0 || cost < best) best = cost, s = sc;
        }
        pps = (P + s - 1) / s;
        pps = (pps + 63) / 64 * 64;
    }
    w.pps = (int)pps;
    w.splits = (int)((P + pps - 1) / pps);
    return w;
}

// bf16 math: conv / ConvT GEMMs whose K channels are a multiple of 64 and whose N is a
// multiple of 128 run on the LDS-DMA kernel (kernels_gemm16.hip) from a prepared bf16
// operand image; option rg16 = 0 keeps the register-staged bf16 kernel (A/B runs),
// rg16_tile picks its tile (kernels_gemm16.hip ROWGEMM16_TILES).
bool rg16_on(const unet_ctx* c, int C, int N) {
    return c->bf16 && c->opt.rg16 != 0 && C % 64 == 0 && N % 128 == 0;
}
// tile for one LDS-DMA row GEMM.  Option rg16_tile forces a tile (128x128 where N does not
// divide into it).  Every tile emits BN partials in 128-row groups, so the choice changes
// speed only.  Default: the 256x256 tile (8 waves, one block per CU) unless
//  * it would leave CUs idle: fewer than 256 blocks (the 16x16 / 32x32 levels of config 4:
//    bottleneck fwd 0.48 -> 0.37 ms, its dgrad 0.90 -> 0.48 ms on the 128x128 tile), or
//  * option rg16_bn_k > K for a BN-backward-partials GEMM (E_STORE_BN: reads the BN input,
//    writes f32 and reduces per-channel partials): with one block per CU nothing hides that
//    epilogue, while two co-resident 128x128 blocks overlap one's epilogue with the other's
//    MFMAs (r01: level-1 dgrad 1.15 -> 0.80 ms, profiles/r01_rg16_tile_sweep.txt; default 0
//    since the r04 one-barrier halo kernel made the 256x256 / 512x128 tiles faster overall).
int rg16_tile(const unet_ctx* c, const RowGemmArgs& g) {
    const int cout = g.emode == E_CONVT ? g.cout : 0;
    auto fits = [&](int t) {
        int bm = 0, bn = 0;
        if (rowgemm16_tile_dims(t, &bm, &bn) != 0) return false;
        if ((t == 19 || t == 20) && (g.amode != G_CONV3 || g.W < 16 || (bm % g.W && g.W % bm)))
            return false;
        return g.N % bn == 0 && (cout == 0 || cout % bn == 0);
    };
    if (c->opt.rg16_tile >= 0) return fits(c->opt.rg16_tile) ? c->opt.rg16_tile : 0;
    const int t0 = 0;
    int t4 = 4;
    if (c->opt.rg16_r3 && fits(19)) t4 = 19;  // option rg16_r3: the tap-row halo kernel
    if (!fits(4)) {
        // option rg16_n128: a 512-row tile for the 128-output GEMMs (halo kernel for 3x3 convs)
        // (rg16_r3 = 0 turns the halo kernel off here too: the one-tap 512x128 tile instead)
        int tn = c->opt.rg16_n128;
        if (tn == 20 && (!c->opt.rg16_r3 || !fits(20))) tn = 6;
        if (tn < 0 || !fits(tn)) return t0;
        if ((g.M + 511) / 512 * (g.N / 128) < 256) return t0;
        if (g.emode == E_STORE_BN && g.K < c->opt.rg16_bn_k && !c->opt.rg16_n128_bn) return t0;
        return tn;
    }
    const int64_t blocks = (g.M + 255) / 256 * (g.N / 256);
    // (r06) a grid too small for 256x256 that fills the CUs with 256x128 takes it (the 16^2
    // bottleneck's 4096-output GEMMs of config 4) instead of 128x128 at two blocks per CU
    if (blocks < 256) return (g.M + 255) / 256 * (g.N / 128) >= 256 && fits(2) ? 2 : t0;
    if (g.emode == E_STORE_BN && g.K < c->opt.rg16_bn_k) return t0;
    return t4;
}
// 3x3 weight gradients of layers with Cin, Cout multiples of 128 on the LDS-DMA
// transposed-read kernel (kernels_gemm16.hip wgrad16_kernel) from the forward's bf16 input
// image and the dz image; option wg16 = 0 keeps the register-staged bf16 wgrad, wg16_tile
// picks the tile.
bool wg16_on(const unet_ctx* c, int CA, int CB) {
    return c->bf16 && c->opt.wg16 != 0 && CA % 128 == 0 && CB % 128 == 0;
}
// XCD-contiguous block order for the LDS-DMA bf16 kernels: on by default (config 4 A/B:
// wgrad 718 -> 766 TF/s, forward 854 -> 871, dgrad -2 %, step +2 %); option xcd16 = 0 off
int xcd16_on(const unet_ctx* c) { return c->opt.xcd16 != 0 ? 1 : 0; }
// tile: option wg16_tile (default 256x256, tile 2) where both channel counts allow it
int wg16_tile(const unet_ctx* c, int CA = 128, int CB = 128) {
    const int t = c->opt.wg16_tile;
    int bm = 0, bn = 0;
    if (wgrad16g_tile_dims(t, &bm, &bn) != 0 || CA % bm || CB % bn) return 0;
    return t;
}
// ConvT weight gradient on the LDS-DMA transposed-read kernel (A' = the forward's bf16
// ConvT input image, B' = the bf16 image of the concat gradient's up half, G_UP2-gathered);
// the bias gradient then comes from k_up2_bias_partials.  Option wg16t = 0 keeps the
// register-staged kernel.
bool convt_wg16_on(const unet_ctx* c, int cin, int cout) {
    return c->opt.wg16t != 0 && wg16_on(c, cin, cout) && rg16_on(c, cin, 4 * cout) &&
           rg16_on(c, cout, cin);
}

// f32 math on the bf16 matrix cores (option x3, kernels_gemm_x3.hip): a 3x3 conv / ConvT
// whose in- and output channels are multiples of 64 runs its forward, input-gradient and
// weight-gradient GEMMs on x3 images (exact three-way bf16 splits of the f32 operands, six
// MFMA products, split f32 accumulators: fp64 error ~3x below the f32 MFMA kernels',
// profiles/r04_x3_probe_*.txt).  The residual network's 1x1 skip GEMMs keep the f32 kernels.
// (r05, removed in r06: option x3_n32, x3 for the 32-multiple channel counts of the reference
// grid's narrow widths on a 128 x 32 row tile and 32-wide weight-gradient tiles -- slower than the
// f32 MFMA kernels there, profiles/r05_x3_n32_ab.txt.)
bool x3_conv_on(const unet_ctx* c, int cin, int cout) {
    return c->opt.x3 && !c->bf16 && cin % 64 == 0 && cout % 64 == 0;
}
bool x3_convt_on(const unet_ctx* c, int cin, int cout) { return x3_conv_on(c, cin, cout); }

// row-GEMM tile: the tap-row halo kernel for 3x3 convs (4 = 256 x 128, one block of 8 waves per
// CU; 6 = 128 x 64 for the 64-output GEMMs, two blocks per CU); otherwise the one-tap tiles
// (0 = 256 x 128, 1 = 128 x 128 where the 256-row grid would leave CUs idle, 2 / 3 = 128 x 64 /
// 256 x 64: option x3_n64)
int x3_tile(const unet_ctx* c, const RowGemmArgs& g) {
    auto fits = [&](int t) {
        int bm = 0, bn = 0;
        if (rowgemm_x3_tile_dims(t, &bm, &bn) != 0 || g.N % bn) return false;
        return g.emode != E_CONVT || g.cout % bn == 0 || bn % g.cout == 0;
    };
    // the halo tiles: 3x3 convs on rows of 16 .. 256k pixels (option x3_r3)
    const bool r3ok = g.amode == G_CONV3 && g.W >= 16 && (256 % g.W == 0 || g.W % 256 == 0);
    const int ft = c->opt.x3_tile;
    if (ft >= 0 && fits(ft) && (ft < 4 || r3ok)) return ft;
    if (g.N % 128 == 0 && fits(0)) {
        const int64_t blocks = (int64_t)(g.M + 255) / 256 * (g.N / 128);
        if (blocks < 256) return 1;
        return c->opt.x3_r3 && r3ok ? 4 : 0;
    }
    // 64 outputs: the 128 x 64 halo tile where the 256-row grid fills the chip (r05: 0.2 % over
    // a 256 x 64 halo tile, 1.032 vs 1.103 ms for a 512 x 64 one, profiles/r05_halo_k16.txt)
    if (g.N % 64 == 0 && c->opt.x3_r3 && r3ok && (int64_t)(g.M + 255) / 256 >= 512) return 6;
    return fits(c->opt.x3_n64) ? c->opt.x3_n64 : -1;
}

// weight gradient: 128x128 tile where both channel counts allow it, else 64x64; split-K over
// pixels so the grid has >= x3_wblocks 128x128 blocks (4x that of 64x64 ones); pixels per
// split a multiple of 256
// 3x3 convs on rows of a multiple of 32 pixels (row_w): the tap-row kernel (tiles 2 = 64x128,
// 4 = 64x64 per tap, three taps per block)
WgradCfg x3_wgrad_cfg(const unet_ctx* c, int CA, int tapsA, int CB, int tapsB, int64_t P,
                      int row_w = 0, int row_h = 0) {
    WgradCfg w{};
    w.tile = (CA % 128 == 0 && CB % 128 == 0) ? 0 : 1;
    // tap-row kernel: rows of 32k pixels, or (r05) 16-pixel rows in pairs
    const bool w16 = row_w == 16 && row_h % 2 == 0 && CA % 64 == 0 && CB % 64 == 0;
    const bool r3 = tapsA == 9 && tapsB == 1 && ((row_w % 32 == 0 && row_w > 0) || w16);
    // (r06: 64 x 64 rather than 128 x 64 where only the input channels divide 128 -- config 2's
    // 128 -> 64 level-0 conv 1.53 -> 1.24 ms, profiles/r06_c2_wtile_ab.txt; tile 3 removed)
    if (r3 && CA % 64 == 0 && CB % 128 == 0) w.tile = 2;
    else if (r3 && CA % 64 == 0 && CB % 64 == 0) w.tile = 4;
    if (c->opt.x3_wtile >= 0) {
        int bm = 0, bn = 0;
        const int t = c->opt.x3_wtile;
        if (wgrad_x3_tile_dims(t, &bm, &bn) == 0 && CA % bm == 0 && CB % bn == 0 && (t < 2 || r3))
            w.tile = t;
    }
    wgrad_x3_tile_dims(w.tile, &w.bm, &w.bn);
    w.bkp = 32;
    const bool tap_row = w.tile == 2 || w.tile == 4;
    const int64_t tiles = tap_row ? (int64_t)(CA / w.bm) * 3 * (CB / w.bn)
                                  : (int64_t)(tapsA * CA / w.bm) * (tapsB * CB / w.bn);
    // blocks per 128x128 one-tap block of work: by area (one-tap), half that (tap-row)
    const int area = std::max(1, 16384 / (w.bm * w.bn));
    const int64_t target = (int64_t)c->opt.x3_wblocks *
                           (w.tile <= 1 ? area : tap_row ? std::max(1, area / 2) : area);
    int64_t splits = std::max<int64_t>(1, (target + tiles - 1) / tiles);
    int64_t pps = (P + splits - 1) / splits;
    pps = (pps + 255) / 256 * 256;
    const int ww = tap_row ? c->opt.x3_wwaves : c->opt.x3_wwaves1;
    if (w.tile <= 4 && ww > 0) {
        // (r05) exactly `ww` full waves of block slots (CUs x blocks per CU): at most that many
        // blocks, pixel splits in 32-pixel steps.  The 256-pixel rounding above can land a few
        // blocks past a wave boundary (1024: 2049 blocks on 2048 slots, -4 %)
        const int64_t slots = (int64_t)c->cus * (w.tile == 4 || w.tile == 1 ? 2 : 1) * ww;
        const int64_t s = std::max<int64_t>(1, slots / tiles);
        pps = (P + s - 1) / s;
        pps = (pps + 31) / 32 * 32;
    }
    w.pps = (int)pps;
    w.splits = (int)((P + pps - 1) / pps);
    return w;
}

// point g at x3 operands: A image `img` (lda = C channels), weights w3
void use_x3(const unet_ctx* c, const Plan& p, RowGemmArgs& g, const uint16_t* img, int C, const uint16_t* w3) {
    g.a = nullptr;
    g.a16 = img;
    g.lda = C;
    g.aoff = 0;
    g.ascale = g.ashift = nullptr;
    g.arelu = 0;
    g.acoef = nullptr;
    g.bt = nullptr;
    g.bt16 = w3;
    g.zero16 = p.zero16;
    g.xcd = 1;
    g.tgm = c->opt.tile_group ? -1 : 0;
}

std::string x3wlabel(const char* fam, const WgradCfg& w, int layer) {
    char b[112];
    snprintf(b, sizeof b, "%s/wx3%s_%dx%d|%d", fam, w.tile >= 2 ? "r3" : "", w.bm, w.bn, layer);
    return b;
}

std::string xlabel(const char* fam, int tile, int layer) {
    int bm = 0, bn = 0;
    rowgemm_x3_tile_dims(tile, &bm, &bn);
    char b[112];
    snprintf(b, sizeof b, "%s/x3%s_%dx%d|%d", fam, tile >= 4 ? "r3" : "", bm, bn, layer);
    return b;
}

void make_plan(unet_ctx* c, int N, int H, int W, bool training, char* base, Plan& p) {
    Bump b{base};
    const int D = c->depth, NC = c->nconv();
    p.N = N;
    p.H = H;
    p.W = W;
    for (int l = 0; l <= D; ++l) p.P[l] = (int64_t)N * (H >> l) * (W >> l);
    p.y.assign(NC, nullptr);
    p.ldy.assign(NC, 0);
    p.offy.assign(NC, 0);
    p.scale.assign(NC, nullptr);
    p.shift.assign(NC, nullptr);
    p.mean.assign(NC, nullptr);
    p.invstd.assign(NC, nullptr);
    p.pack = b.take<float>(c->pack_floats);
    p.pprm = p.pbn = p.pgrad = p.ugrad = nullptr;
    p.ptab = p.btab = nullptr;
    if (c->padded) {
        p.pprm = b.take<float>(c->n_pparam_floats);
        p.pbn = b.take<float>(c->n_pbn_floats);
        p.pgrad = training ? b.take<float>(c->n_pparam_floats) : nullptr;
        p.ptab = b.take<PadDesc>((int64_t)c->pad_params.size());
        p.btab = b.take<PadDesc>((int64_t)c->pad_bn.size());
    }
    p.x_nhwc = b.take<float>(p.P[0] * c->in_ch);  // NHWC copy of x (conv-0 wgrad input)
    for (int l = 0; l < D; ++l) {
        const int C = c->ch(l);
        p.cat[l] = b.take<float>(p.P[l] * 2 * C);
        p.cat_scale[l] = b.take<float>(2 * C);
        p.cat_shift[l] = b.take<float>(2 * C);
        p.pool[l] = b.take<float>(p.P[l + 1] * C);
        p.idx[l] = b.take<uint8_t>(p.P[l + 1] * C);
    }
    for (int i = 0; i < NC; ++i) {
        const ConvL& L = c->conv[i];
        if (L.block < D && L.which == 1 && !c->res) {
            // the encoder output lives in the skip half of its concat buffer, and its BN
            // affine is that half of the concat affine
            const int l = L.block, so = c->skip_off(l);
            p.y[i] = p.cat[l];
            p.ldy[i] = 2 * c->ch(l);
            p.offy[i] = so;
            p.scale[i] = p.cat_scale[l] ? p.cat_scale[l] + so : nullptr;
            p.shift[i] = p.cat_shift[l] ? p.cat_shift[l] + so : nullptr;
        } else {
            p.y[i] = b.take<float>(p.P[L.level] * L.cout);
            p.ldy[i] = L.cout;
            p.offy[i] = 0;
            p.scale[i] = b.take<float>(L.cout);
            p.shift[i] = b.take<float>(L.cout);
        }
        p.mean[i] = b.take<float>(L.cout);
        p.invstd[i] = b.take<float>(L.cout);
    }
    p.out.assign(2 * D + 1, nullptr);
    p.ldout.assign(2 * D + 1, 0);
    p.offout.assign(2 * D + 1, 0);
    for (int blk = 0; blk <= 2 * D && c->res; ++blk) {
        const ConvL& L = c->conv[2 * blk + 1];
        if (blk < D) {  // encoder output: the skip half of its concat buffer
            p.out[blk] = p.cat[blk];
            p.ldout[blk] = 2 * L.cout;
            p.offout[blk] = c->skip_off(blk);
        } else {
            p.out[blk] = b.take<float>(p.P[L.level] * L.cout);
            p.ldout[blk] = L.cout;
        }
    }
    // BN-stat partials: rows = M / 64 (smallest row tile) of the row GEMM, or RED_G for the
    // first conv
    int64_t srows = 0;
    for (int i = 0; i < NC; ++i) {
        const int64_t r = std::max<int64_t>((p.P[c->conv[i].level] + 63) / 64, RED_G);
        srows = std::max(srows, r * 2 * c->conv[i].cout);
    }
    p.stats = b.take<float>(srows);
    p.stats2 = b.take<float>((int64_t)STAT_G * 2 * c->cmax);
    p.s16 = nullptr;
    p.zero16 = b.take<char>(256);  // zeroed 16-B page: padding taps of the LDS-DMA GEMMs
    if (c->bf16) {
        int64_t n16 = 0;
        for (const ConvL& L : c->conv) n16 = std::max(n16, p.P[L.level] * std::max(L.cin, L.cout));
        for (const ConvTL& T : c->convt)
            n16 = std::max(n16, std::max(p.P[T.in_level] * T.cin, p.P[T.in_level - 1] * T.cout));
        p.s16 = b.take<uint16_t>(n16);
    }
    p.x16.assign(NC, nullptr);
    for (int i = 0; i < NC && training; ++i)
        if (wg16_on(c, c->conv[i].cin, c->conv[i].cout) && rg16_on(c, c->conv[i].cin, c->conv[i].cout))
            p.x16[i] = b.take<uint16_t>(p.P[c->conv[i].level] * c->conv[i].cin);
    p.t16.assign(c->convt.size(), nullptr);
    for (size_t k = 0; k < c->convt.size() && training; ++k) {
        const ConvTL& T = c->convt[k];
        if (!c->res && convt_wg16_on(c, T.cin, T.cout))
            p.t16[k] = b.take<uint16_t>(p.P[T.in_level] * T.cin);
    }
    // option x3: weight images, kept input images, one scratch image (dz, the concat
    // gradient's up half, and every input image of an inference pass)
    p.pack3 = p.s3 = nullptr;
    p.x3.assign(NC, nullptr);
    p.t3.assign(c->convt.size(), nullptr);
    {
        int64_t n3 = 0;
        for (int i = 0; i < NC; ++i) {
            const ConvL& L = c->conv[i];
            if (L.pf < 0 || !x3_conv_on(c, L.cin, L.cout)) continue;
            n3 = std::max(n3, p.P[L.level] * std::max(L.cin, L.cout));
            if (training) p.x3[i] = b.take<uint16_t>(3 * p.P[L.level] * L.cin);
        }
        for (size_t k = 0; k < c->convt.size(); ++k) {
            const ConvTL& T = c->convt[k];
            if (!x3_convt_on(c, T.cin, T.cout)) continue;
            n3 = std::max(n3, std::max(p.P[T.in_level] * T.cin, p.P[T.in_level - 1] * T.cout));
            if (training) p.t3[k] = b.take<uint16_t>(3 * p.P[T.in_level] * T.cin);
        }
        if (n3) {
            p.pack3 = b.take<uint16_t>(3 * c->pack_floats);
            p.s3 = b.take<uint16_t>(3 * n3);
        }
    }
    if (training) {
        int64_t gmax = p.P[0] * c->base;
        for (int i = 0; i < NC; ++i) {
            gmax = std::max(gmax, p.P[c->conv[i].level] * c->conv[i].cout);
            gmax = std::max(gmax, p.P[c->conv[i].level] * c->conv[i].cin);
        }
        p.g[0] = b.take<float>(gmax);
        p.g[1] = b.take<float>(gmax);
        p.g[2] = c->res ? b.take<float>(gmax) : nullptr;
        for (int l = 0; l < D; ++l) p.dcat[l] = b.take<float>(p.P[l] * 2 * c->ch(l));
        int64_t smax = 0, bmax = 0;
        for (int i = 1; i < NC; ++i) {
            const ConvL& L = c->conv[i];
            WgradCfg w = x3_conv_on(c, L.cin, L.cout)
                             ? x3_wgrad_cfg(c, L.cin, 9, L.cout, 1, p.P[L.level], W >> L.level, H >> L.level)
                             : wgrad_cfg(c, L.cin, 9, L.cout, 1, p.P[L.level], c->bf16, W >> L.level);
            smax = std::max(smax, (int64_t)w.splits * 9 * L.cin * L.cout);
            bmax = std::max(bmax, (int64_t)w.splits * L.cout);
        }
        for (int blk = 1; blk <= 2 * D && c->res; ++blk) {
            const ConvL& L = c->conv[2 * blk];
            WgradCfg w = wgrad_cfg(c, L.cin, 1, L.cout, 1, p.P[L.level], c->bf16);
            smax = std::max(smax, (int64_t)w.splits * L.cin * L.cout);
        }
        for (const ConvTL& T : c->convt) {
            WgradCfg w = x3_convt_on(c, T.cin, T.cout)
                             ? x3_wgrad_cfg(c, T.cin, 1, T.cout, 4, p.P[T.in_level])
                             : wgrad_cfg(c, T.cin, 1, T.cout, 4, p.P[T.in_level], c->bf16);
            smax = std::max(smax, (int64_t)w.splits * T.cin * 4 * T.cout);
            bmax = std::max(bmax, (int64_t)w.splits * 4 * T.cout);
        }
        p.slab = b.take<float>(smax);
        int64_t pmax = (int64_t)RED_G * 2 * c->cmax;
        for (int i = 0; i < NC; ++i)  // dgrad epilogues: ceil(P/64) rows of 2*C (BM >= 64)
            pmax = std::max(pmax, (p.P[c->conv[i].level] / 64 + 1) * 2 * c->conv[i].cout);
        p.part = b.take<float>(pmax);
        p.part2 = b.take<float>((int64_t)STAT_G * 2 * c->cmax);
        p.hpart = b.take<float>((int64_t)WIDE_G *
                                std::max<int64_t>(10 * c->base, (int64_t)c->out_ch * (c->base + 1)));
        p.bslab = b.take<float>(std::max<int64_t>(bmax, 1));
        p.coef = b.take<float>(4 * (int64_t)c->cmax);  // BN-backward dz coefficients [4][C]
        p.gdz = (c->opt.dz_in_wgrad && !c->bf16) ? b.take<float>(gmax) : nullptr;
    } else {
        p.gdz = nullptr;
        p.g[0] = p.g[1] = p.g[2] = p.slab = p.part = p.part2 = p.hpart = p.bslab = p.coef = nullptr;
        for (int l = 0; l < D; ++l) p.dcat[l] = nullptr;
    }
    p.bytes = b.off + 256;
}

// ------------------------------------------------------------------------------------
// launch bookkeeping (optional per-launch HIP-event timing)
// ------------------------------------------------------------------------------------
struct Launcher {
    unet_ctx* c;
    hipStream_t s;
    hipEvent_t ev() {
        if (c->ev_used == c->ev_pool.size()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            c->ev_pool.push_back(e);
        }
        return c->ev_pool[c->ev_used++];
    }
    template <class F>
    int run(const std::string& label, double flop, F&& f) {
        hipEvent_t a = nullptr, b = nullptr;
        const bool timed = c->timing && (c->tfilter.empty() || label.find(c->tfilter) != std::string::npos);
        if (timed) {
            a = ev();
            b = ev();
            (void)hipEventRecord(a, s);
        }
        int r = f();
        if (r != 0) return fail(c, UNET_ERR_HIP, "%s: launch failed (%d: %s)", label.c_str(), r,
                                r > 0 ? hipGetErrorString((hipError_t)r) : "bad shape");
        if (timed) {
            (void)hipEventRecord(b, s);
            c->trec.push_back(TimeRec{label, a, b, flop});
        }
        return 0;
    }
};

// Row-GEMM tile choice for an output width N (tile ids: kernels_gemm.hip ROWGEMM_TILES,
// 18, 19, 25, 26 = kernels_gemm_pipe.hip).
//  * f32, N % 128 == 0: the software-pipelined 128x128 kernel, forward with its global loads
//    two chunks ahead (18), dgrad too since r03 (one chunk ahead, tile 16, removed in r06).  r02
//    A/B (config 2):
//    401 img/s against 390 for the register-staged tiles (t7 / t4 / t0 by grid size), the
//    dominant kernel 128.9 vs 122.2 TF/s; the two schedules store identical bits
//    (tests/test_gpu_parity.py::test_pipe_gemm_bit_identical);
//  * f32, N = 64 outputs: the pipelined 128x64 with loads two chunks ahead (19) on the
//    forward GEMMs (level-0 128 -> 64 conv 112 -> 117 TF/s), the register-staged 128x64
//    (t1) on the ConvT forward and since r03 the three-blocks-per-CU 25 / 26 on the dgrads
//    (options tile_n64 / tile_n64_dgrad / tile_convt64; profiles/r02_pipe_exp.txt).
// bf16 MFMA (register-staged): a chunk of 64 K per barrier (4 MFMA k-steps) by default.
// Options tile_* override (tuning runs; -1 = automatic).
int pick_tile(const unet_ctx* c, int N, bool dgrad, bool bf16, bool convt = false) {
    const Options& o = c->opt;
    if (bf16) return N % 128 == 0 ? 6 : 1;  // register-staged bf16 tiles (kernels_gemm.hip)
    if (N % 64) return o.tile_n32;  // 32 outputs (narrow networks' level 0)
    if (N % 128) return convt && !dgrad ? o.tile_convt64 : (dgrad ? o.tile_n64_dgrad : o.tile_n64);
    if (convt && !dgrad && o.tile_convt >= 0) return o.tile_convt;
    if (convt && dgrad && o.tile_convt_dgrad >= 0) return o.tile_convt_dgrad;
    // dgrad on the two-chunks-ahead tile too since r03's prologue fence (loop waits vmcnt(2)
    // -> vmcnt(8)): conv dgrads 23.4 -> 23.0 ms per step
    if (dgrad) return o.tile_n128_dgrad >= 0 ? o.tile_n128_dgrad : 18;
    return o.tile_n128 >= 0 ? o.tile_n128 : 18;
}

std::string tlabel(const char* fam, int tile, int layer) {
    int bm = 0, bn = 0, bk = 0;
    rowgemm_tile_dims(tile, &bm, &bn, &bk);
    char b[112];
    const int db = rowgemm_tile_dbuf(tile);  // 1 = two LDS images, 2 = pipelined
    snprintf(b, sizeof b, "%s/rowgemm_%dx%dx%d%s|%d", fam, bm, bn, bk,
             db == 3 ? "g" : db == 2 ? "p" : (db ? "d" : ""), layer);
    return b;
}

std::string wlabel(const char* fam, const WgradCfg& w, int layer) {
    char b[112];
    snprintf(b, sizeof b, "%s/wgrad%s_%dx%dx%d|%d", fam, w.tile >= 20 ? "3" : "", w.bm, w.bn, w.bkp,
             layer);
    return b;
}

#define RUN(label, flop, expr)                            \
    do {                                                  \
        int rc_ = L.run(label, flop, [&]() { return (expr); }); \
        if (rc_) return rc_;                              \
    } while (0)

int stats_finalize(unet_ctx* c, Launcher& L, Plan& p, int i, int R, int64_t count, bool training,
                   const float* prm, float* bn_run, int64_t* bn_cnt) {
    const BnL& B = c->bn[i];
    const int C = B.C;
    hipStream_t s = L.s;
    if (!training) {
        RUN("bn_finalize", 0,
            k_bn_finalize_eval(C, prm + B.g, prm + B.b, bn_run + B.run, bn_run + B.run + C, BN_EPS,
                               p.scale[i], p.shift[i], s));
        return 0;
    }
    const float* part = p.stats;
    int G = R;
    if (R > STAT_G) {
        RUN("bn_stats_reduce", 0, k_reduce_rows(p.stats, R, 2 * C, p.stats2, STAT_G, s));
        part = p.stats2;
        G = STAT_G;
    }
    RUN("bn_finalize", 0,
        k_bn_finalize_train(part, G, C, (double)count, prm + B.g, prm + B.b,
                            bn_run ? bn_run + B.run : nullptr,
                            bn_run ? bn_run + B.run + C : nullptr, bn_cnt ? bn_cnt + i : nullptr,
                            BN_MOMENTUM, BN_EPS, p.scale[i], p.shift[i], p.mean[i], p.invstd[i],
                            s));
    return 0;
}

// Input operand of conv i: pointer, ld, offset, affine and the ReLU span (channels
// [0, relu) get ReLU after the affine: BN -> ReLU order).
struct Operand {
    const float* ptr;
    int ld, off;
    const float* scale;
    const float* shift;
    int relu;
};

Operand conv_input(unet_ctx* c, Plan& p, int i) {
    const ConvL& L = c->conv[i];
    const int D = c->depth;
    if (L.which == 1)
        return {p.y[i - 1], p.ldy[i - 1], p.offy[i - 1], p.scale[i - 1], p.shift[i - 1],
                c->bn_relu ? L.cin : 0};
    if (L.block >= 1 && L.block <= D)  // after a max-pool (already normalised + activated)
        return {p.pool[L.block - 1], L.cin, 0, nullptr, nullptr, 0};
    if (L.block > D) {  // concat: the skip half carries the encoder's BN (+ReLU) affine
        const int l = L.level;
        if (c->res) return {p.cat[l], 2 * c->ch(l), 0, nullptr, nullptr, 0};  // materialised
        return {p.cat[l], 2 * c->ch(l), 0, p.cat_scale[l], p.cat_shift[l],
                c->bn_relu ? c->ch(l) : 0};
    }
    return {nullptr, 0, 0, nullptr, nullptr, 0};  // conv 0: x
}

// BN partial rows a row GEMM emits: one per 128-row group, whatever its tile (gemm_common.h
// row_epilogue), so the BN statistics do not depend on the tile choice
int bn_groups(int64_t M) { return (int)((M + 127) / 128); }

const float* bias_ptr(const float* prm, int64_t off) { return off >= 0 ? prm + off : nullptr; }

// XCD-aware block order for the f32 GEMMs (option xcd_remap: 0 none, 1 both, 2 row GEMMs
// only, 3 wgrad only; A/B runs)
int xcd_remap_on(const unet_ctx* c) { return c->opt.xcd_remap == 1 || c->opt.xcd_remap == 2; }
int xcd_remap_wgrad(const unet_ctx* c) { return c->opt.xcd_remap == 1 || c->opt.xcd_remap == 3; }

// weight image of a row GEMM: f32, or bf16 packed into the same slot (half its size)
void set_weights(const unet_ctx* c, RowGemmArgs& g, const float* img) {
    g.xcd = xcd_remap_on(c);
    if (c->bf16)
        g.bt16 = (const uint16_t*)img;
    else
        g.bt = img;
}

std::string tlabel16(const char* fam, int tile, int layer) {
    int bm = 0, bn = 0, st = 0;
    rowgemm16_tile_dims(tile, &bm, &bn, &st);
    char b[112];
    snprintf(b, sizeof b, "%s/rg16%s_%dx%ds%d|%d", fam, (tile == 19 || tile == 20) ? "r3" : "",
             bm, bn, st, layer);
    return b;
}
// point g's A operand at the prepared bf16 image (lda = C channels)
void use_a16(const unet_ctx* c, const Plan& p, RowGemmArgs& g, int C) {
    g.a16 = p.s16;
    g.lda = C;
    g.aoff = 0;
    g.ascale = g.ashift = nullptr;
    g.arelu = 0;
    g.acoef = nullptr;
    g.zero16 = p.zero16;
    g.xcd = xcd16_on(c);
    g.tgm = c->opt.tile_group ? -1 : 0;
}

// device copies of the expand / compact tables (the host tables live in the context, so
// the asynchronous copy's source outlives it)
int upload_pad_tables(unet_ctx* c, Plan& p, hipStream_t s) {
    hipError_t e = hipMemcpyAsync(p.ptab, c->pad_params.data(), sizeof(PadDesc) * c->pad_params.size(),
                                  hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(p.btab, c->pad_bn.data(), sizeof(PadDesc) * c->pad_bn.size(),
                           hipMemcpyHostToDevice, s);
    return (int)e;
}

// the pack job table of every 3x3 conv (but the Cin = in_channels first conv) and ConvT weight
// (dgrad images too when `dgrad`); false when the table overflows
bool build_pack_jobs(const unet_ctx* c, bool dgrad, PackJobs& jobs) {
    jobs.n = 0;
    int blocks = 0;
    auto add = [&](int64_t w, int64_t f, int64_t d, int cin, int cout, int kind) {
        PackJob& J = jobs.j[jobs.n++];
        J.w = w;
        J.f = f;
        J.d = dgrad ? d : -1;
        J.cin = cin;
        J.cout = cout;
        J.kind = kind;
        J.tx = ((kind == 0 ? cin : cout) + 31) / 32;
        J.ty = ((kind == 0 ? cout : cin) + 31) / 32;
        J.block0 = blocks;
        blocks += J.tx * J.ty;
    };
    for (const ConvL& C : c->conv) {
        if (C.pf < 0) continue;
        if (jobs.n >= MAX_PACK_JOBS) return false;
        add(C.w, C.pf, C.pd, C.cin, C.cout, 0);
    }
    for (const ConvTL& T : c->convt) {
        if (jobs.n >= MAX_PACK_JOBS) return false;
        add(T.w, T.pf, T.pd, T.cin, T.cout, 1);
    }
    return true;
}

// whether the plan of this context carries x3 weight images (make_plan's pack3)
bool plan_has_pack3(const unet_ctx* c) {
    for (const ConvL& L : c->conv)
        if (L.pf >= 0 && x3_conv_on(c, L.cin, L.cout)) return true;
    for (const ConvTL& T : c->convt)
        if (x3_convt_on(c, T.cin, T.cout)) return true;
    return false;
}

int forward_impl(unet_ctx* c, const float* prm, float* bn_run, int64_t* bn_cnt, const float* x,
                 float* logits, Plan& p, bool training, hipStream_t s) {
    Launcher L{c, s};
    const int H = p.H, W = p.W, D = c->depth, NC = c->nconv();
    // 1. weight images for the row GEMMs: re-packed every call (params may have changed through
    //    the optimizer or load_state_dict; ~0.1 ms of HBM traffic per step at config 2) unless
    //    the fused AdamW of unet_adamw_repack wrote them for exactly these parameters (r06)
    const bool use_pp = c->pp_ok && c->pp_src == prm && c->pp && (!p.pack3 || c->pp3);
    if (training) {
        c->fwd_used_pp = use_pp;
        c->fwd_pp_gen = c->pp_gen;
    }
    if (use_pp) {
        p.pack = c->pp;
        if (p.pack3) p.pack3 = c->pp3;
    } else {
        PackJobs jobs{};
        if (!build_pack_jobs(c, training, jobs)) return fail(c, UNET_ERR_INTERNAL, "pack job table full");
        if (jobs.n) RUN("pack", 0, k_pack_all(jobs, prm, p.pack, c->bf16, s));
        // option x3: the whole region as rows of 32 floats (every image 32-aligned)
        if (p.pack3)
            RUN("pack", 0, k_to_x3(p.pack, 32, 0, 32, nullptr, nullptr, 0, c->pack_floats / 32, p.pack3,
                                   32, 0, s));
    }
    for (int b = 1; b <= 2 * D && c->res && training; ++b)
        RUN("pack", 0, k_pack_1x1_t(prm + c->skip_w[b], p.pack + c->skip_pd[b], c->conv[2 * b].cin,
                                    c->conv[2 * b].cout, s));
    // 2. concat affine: identity on the up-sampled half (no BN between ConvT and concat)
    for (int l = 0; l < D; ++l) {
        const int C = c->ch(l), uo = c->up_off(l);
        RUN("fill", 0, k_fill(p.cat_scale[l] + uo, C, 1.f, s));
        RUN("fill", 0, k_fill(p.cat_shift[l] + uo, C, 0.f, s));
    }
    if (p.zero16) RUN("fill", 0, (int)hipMemsetAsync(p.zero16, 0, 256, s));
    // in_channels == 1: NCHW == NHWC; keep a private copy for the conv-0 wgrad
    RUN("copy_x", 0, (int)hipMemcpyAsync(p.x_nhwc, x, sizeof(float) * p.P[0] * c->in_ch,
                                         hipMemcpyDeviceToDevice, s));
    const float* xin = p.x_nhwc;
    // decoder convs whose operand image already holds the ConvT's up half (option convt16)
    std::vector<char> up16(NC, 0);
    // x3: the max-pool wrote the next encoder conv's x3 operand image itself (no f32 pooled
    // tensor, no prep pass; r05)
    std::vector<char> pool3(NC, 0);
    // (r06) bf16: the max-pool wrote the next encoder conv's bf16 operand image (pool16); both
    // paths: the max-pool wrote the decoder conv's skip half of its kept image (skipimg)
    std::vector<char> pool16(NC, 0), skipimg(NC, 0);

    auto conv = [&](int i) -> int {
        const ConvL& C = c->conv[i];
        const int Hl = H >> C.level, Wl = W >> C.level;
        const int64_t M = p.P[C.level];
        int R;
        if (i == 0 && C.pf < 0) {
            R = wide_g(M);
            RUN("conv_first_fwd", 2.0 * M * 9 * C.cout,
                k_conv_first_fwd(xin, prm + C.w, bias_ptr(prm, C.b), p.y[0], (int)M, Hl, Wl, C.cout,
                                 c->bn_relu ? 0 : 1, p.stats, R, s));
        } else {
            Operand a = conv_input(c, p, i);
            RowGemmArgs g{};
            g.zero16 = p.zero16;
            g.H = Hl;
            g.W = Wl;
            g.M = (int)M;
            g.N = C.cout;
            g.K = 9 * C.cin;
            g.a = a.ptr;
            g.lda = a.ld;
            g.aoff = a.off;
            g.C = C.cin;
            g.amode = G_CONV3;
            g.ascale = a.scale;
            g.ashift = a.shift;
            g.arelu = a.relu;
            set_weights(c, g, p.pack + C.pf);
            g.out = p.y[i];
            g.ldo = p.ldy[i];
            g.ooff = p.offy[i];
            g.bias = bias_ptr(prm, C.b);
            g.stats = p.stats;
            g.emode = c->bn_relu ? E_STATS : E_BIAS_RELU_STATS;
            if (p.pack3 && x3_conv_on(c, C.cin, C.cout)) {
                uint16_t* img = p.x3[i] ? p.x3[i] : p.s3;
                if (pool3[i]) {
                    // (the max-pool already stored op(pooled) as this conv's x3 image)
                } else if (up16[i] && skipimg[i]) {
                    // (the ConvT stored the up half, the max-pool the skip half)
                } else if (up16[i]) {  // the ConvT stored the up half's x3 split: convert the skip half
                    const int l = C.level, so = c->skip_off(l), ch = c->ch(l);
                    const int rl = std::min(std::max(a.relu - so, 0), ch);
                    RUN("prep_x3", 0, k_to_x3(a.ptr, a.ld, a.off + so, ch, a.scale ? a.scale + so : nullptr,
                                              a.shift ? a.shift + so : nullptr, rl, M, img, C.cin, so, s));
                } else {
                    RUN("prep_x3", 0, k_to_x3(a.ptr, a.ld, a.off, C.cin, a.scale, a.shift, a.relu, M, img,
                                              C.cin, 0, s));
                }
                use_x3(c, p, g, img, C.cin, p.pack3 + 3 * C.pf);
                const int tile = x3_tile(c, g);
                R = bn_groups(M);
                RUN(xlabel("conv_fwd", tile, i), 2.0 * M * C.cout * 9 * C.cin, launch_rowgemm_x3(g, tile, s));
                return stats_finalize(c, L, p, i, R, M, training, prm, bn_run, bn_cnt);
            }
            if (rg16_on(c, C.cin, C.cout)) {
                uint16_t* img = p.x16[i] ? p.x16[i] : p.s16;
                if (pool16[i] || (up16[i] && skipimg[i])) {
                    // (the max-pool / the ConvT and the max-pool stored the whole image)
                } else if (up16[i]) {  // the ConvT stored the up half already: convert the skip half
                    const int l = C.level, so = c->skip_off(l);
                    RUN("prep16", 0, k_to_bf16(a.ptr, a.ld, a.off + so, c->ch(l), a.scale + so,
                                               a.shift + so, a.relu, M, img + so, s, C.cin));
                } else {
                    RUN("prep16", 0, k_to_bf16(a.ptr, a.ld, a.off, C.cin, a.scale, a.shift, a.relu, M,
                                               img, s));
                }
                use_a16(c, p, g, C.cin);
                g.a16 = img;
                const int tile = rg16_tile(c, g);
                R = bn_groups(M);
                RUN(tlabel16("conv_fwd", tile, i), 2.0 * M * C.cout * 9 * C.cin, launch_rowgemm16(g, tile, s));
                return stats_finalize(c, L, p, i, R, M, training, prm, bn_run, bn_cnt);
            }
            R = bn_groups(M);
            const int tile = pick_tile(c, C.cout, false, c->bf16);
            RUN(tlabel("conv_fwd", tile, i), 2.0 * M * C.cout * 9 * C.cin, launch_rowgemm(g, tile, s));
        }
        return stats_finalize(c, L, p, i, R, M, training, prm, bn_run, bn_cnt);
    };
    auto convT = [&](int k) -> int {
        const ConvTL& T = c->convt[k];
        const int src = 2 * (D + k) + 1;  // second conv of the bottleneck / decoder block
        const int lo = T.in_level - 1;
        RowGemmArgs g{};
        g.zero16 = p.zero16;
        g.H = H >> T.in_level;
        g.W = W >> T.in_level;
        g.M = (int)p.P[T.in_level];
        g.N = 4 * T.cout;
        g.K = T.cin;
        if (c->res) {  // the materialised output of block D+k
            g.a = p.out[D + k];
            g.lda = p.ldout[D + k];
            g.aoff = p.offout[D + k];
        } else {
            g.a = p.y[src];
            g.lda = p.ldy[src];
            g.aoff = p.offy[src];
            g.ascale = p.scale[src];
            g.ashift = p.shift[src];
            g.arelu = c->bn_relu ? T.cin : 0;
        }
        g.C = T.cin;
        g.amode = G_IDENT;
        set_weights(c, g, p.pack + T.pf);
        g.out = p.cat[lo];
        g.ldo = 2 * c->ch(lo);
        g.ooff = c->up_off(lo);
        g.bias = prm + T.b;
        g.cout = T.cout;
        g.emode = E_CONVT;
        if (p.pack3 && x3_convt_on(c, T.cin, T.cout)) {
            uint16_t* img = p.t3[k] ? p.t3[k] : p.s3;
            RUN("prep_x3", 0, k_to_x3(g.a, g.lda, g.aoff, T.cin, g.ascale, g.ashift, g.arelu, g.M, img,
                                      T.cin, 0, s));
            use_x3(c, p, g, img, T.cin, p.pack3 + 3 * T.pf);
            // option convt16 (x3 training): the up half of the decoder's concat goes straight
            // into that conv's kept x3 image, its only reader; the conv's prep pass then
            // converts the skip half only
            const int idec = 2 * (D + 1 + k);
            const ConvL& Cd = c->conv[idec];
            // (not in the residual network: its 1x1 skip GEMM reads the f32 concat as well)
            if (c->opt.convt16 && !c->res && p.x3[idec] && x3_conv_on(c, Cd.cin, Cd.cout)) {
                g.out3 = p.x3[idec];
                up16[idec] = true;
            }
            const int tile = x3_tile(c, g);
            RUN(xlabel("convT_fwd", tile, 100 + k), 2.0 * g.M * g.N * g.K, launch_rowgemm_x3(g, tile, s));
            return 0;
        }
        if (!c->res && rg16_on(c, T.cin, T.cout)) {
            uint16_t* img = p.t16[k] ? p.t16[k] : p.s16;
            RUN("prep16", 0, k_to_bf16(g.a, g.lda, g.aoff, T.cin, g.ascale, g.ashift, g.arelu, g.M,
                                       img, s));
            use_a16(c, p, g, T.cin);
            g.a16 = img;
            // option convt16: the up half goes to the decoder conv's kept bf16 image (the only
            // reader of that half in a bf16 training step; skip-first concat, identity affine)
            const int idec = 2 * (D + 1 + k);
            const ConvL& Cd = c->conv[idec];
            if (c->opt.convt16 && c->skip_first && p.x16[idec] && rg16_on(c, Cd.cin, Cd.cout)) {
                g.out16 = p.x16[idec];
                up16[idec] = true;
            }
            const int tile = rg16_tile(c, g);
            RUN(tlabel16("convT_fwd", tile, 100 + k), 2.0 * g.M * g.N * g.K,
                launch_rowgemm16(g, tile, s));
            return 0;
        }
        const int tile = pick_tile(c, T.cout, false, c->bf16, true);  // grid N = 4 cout
        RUN(tlabel("convT_fwd", tile, 100 + k), 2.0 * g.M * g.N * g.K, launch_rowgemm(g, tile, s));
        return 0;
    };

    // residual block b closes with out = ReLU(BN2(z2) + skip(x)) (mod.py:86)
    auto block_out = [&](int b) -> int {
        const ConvL& CL = c->conv[2 * b];
        const int i2 = 2 * b + 1;
        const int64_t M = p.P[CL.level];
        if (CL.pf < 0) {  // Cin = 1: the skip is a per-channel scale of the image
            RUN("res_out", 0, k_res_first_fwd(xin, prm + c->skip_w[b], p.y[i2], p.scale[i2],
                                              p.shift[i2], M, CL.cout, p.out[b], p.ldout[b],
                                              p.offout[b], s));
            return 0;
        }
        Operand a = conv_input(c, p, 2 * b);
        RowGemmArgs g{};
        g.zero16 = p.zero16;
        g.H = H >> CL.level;
        g.W = W >> CL.level;
        g.M = (int)M;
        g.N = CL.cout;
        g.K = CL.cin;
        g.a = a.ptr;
        g.lda = a.ld;
        g.aoff = a.off;
        g.C = CL.cin;
        g.amode = G_IDENT;
        g.bt = prm + c->skip_w[b];  // torch layout [co][ci] is already Bt[n][k]
        g.xcd = xcd_remap_on(c);
        g.out = p.out[b];
        g.ldo = p.ldout[b];
        g.ooff = p.offout[b];
        g.emode = E_RESID;
        g.ey = p.y[i2];
        g.ldey = p.ldy[i2];
        g.offey = p.offy[i2];
        g.escale = p.scale[i2];
        g.eshift = p.shift[i2];
        const int tile = pick_tile(c, CL.cout, false, false);
        RUN(tlabel("skip_fwd", tile, b), 2.0 * M * CL.cout * CL.cin, launch_rowgemm(g, tile, s));
        return 0;
    };

    int rc;
    for (int b = 0; b <= D; ++b) {
        if ((rc = conv(2 * b))) return rc;
        if ((rc = conv(2 * b + 1))) return rc;
        if (c->res && (rc = block_out(b))) return rc;
        if (b < D) {
            const int i = 2 * b + 1, C = c->ch(b);
            if (c->res)
                RUN("maxpool_fwd", 0,
                    k_maxpool_bn(p.out[b], p.ldout[b], p.offout[b], nullptr, nullptr, 0, p.N, H >> b,
                                 W >> b, C, p.pool[b], p.idx[b], s));
            else {
                const int j = 2 * (b + 1);  // the next encoder block's first conv
                const ConvL& Cj = c->conv[j];
                uint16_t* out3 = nullptr;
                uint16_t *o16 = nullptr, *s16 = nullptr, *s3 = nullptr;
                if (p.pack3 && x3_conv_on(c, Cj.cin, Cj.cout)) {
                    out3 = p.x3[j] ? p.x3[j] : p.s3;
                    pool3[j] = 1;
                } else if (p.x16[j] && rg16_on(c, Cj.cin, Cj.cout)) {  // (r06) training, bf16
                    o16 = p.x16[j];
                    pool16[j] = 1;
                }
                // (r06) the skip half of the decoder conv at this level (its ConvT stores the
                // up half, option convt16): op(BN(y)) as that conv's kept operand image
                const int idec = 2 * (2 * D - b);
                const ConvL& Cd = c->conv[idec];
                if (c->opt.convt16) {
                    if (p.pack3 && p.x3[idec] && x3_conv_on(c, Cd.cin, Cd.cout))
                        s3 = p.x3[idec];
                    else if (c->bf16 && c->skip_first && p.x16[idec] && rg16_on(c, Cd.cin, Cd.cout))
                        s16 = p.x16[idec];
                }
                skipimg[idec] = s3 || s16;
                RUN("maxpool_fwd", 0,
                    k_maxpool_bn(p.y[i], p.ldy[i], p.offy[i], p.scale[i], p.shift[i],
                                 c->bn_relu ? 1 : 0, p.N, H >> b, W >> b, C,
                                 out3 || o16 ? nullptr : p.pool[b],  // (its images are the only readers)
                                 p.idx[b], s, out3, o16, s16, s3, Cd.cin, c->skip_off(b)));
            }
        }
    }
    for (int k = 0; k < D; ++k) {
        if ((rc = convT(k))) return rc;
        const int b = D + 1 + k;
        if ((rc = conv(2 * b))) return rc;
        if ((rc = conv(2 * b + 1))) return rc;
        if (c->res && (rc = block_out(b))) return rc;
    }
    const int last = NC - 1;
    if (c->res)
        RUN("head_fwd", 2.0 * p.P[0] * c->base * c->out_ch,
            k_head_fwd(p.out[2 * D], c->base, nullptr, nullptr, 0, prm + c->head_w, prm + c->head_b,
                       c->out_ch, (int)p.P[0], H * W, logits, s));
    else
        RUN("head_fwd", 2.0 * p.P[0] * c->base * c->out_ch,
            k_head_fwd(p.y[last], c->base, p.scale[last], p.shift[last], c->bn_relu ? 1 : 0,
                       prm + c->head_w, prm + c->head_b, c->out_ch, (int)p.P[0], H * W, logits, s));
    return 0;
}

int backward_impl(unet_ctx* c, const float* prm, const float* dlogits, float* grads, Plan& p,
                  hipStream_t s) {
    Launcher L{c, s};
    const int H = p.H, W = p.W, D = c->depth, NC = c->nconv();
    int rc;
    // (weight gradients run on the same stream as the dgrad chain: a second stream measured
    // 1 % slower, every GEMM fills the chip on its own)
    // BatchNorm backward is fused: the producer of `do` (head_bwd, a dgrad epilogue,
    // maxpool_bwd) leaves {sum do, sum do*y} column partials in p.part (do already masked by
    // the following ReLU in BN -> ReLU order); this finalize turns them into dgamma, dbeta
    // and the per-channel coefficients of dz = A do + B (y - mean) + C (masked by [y > 0] in
    // ReLU -> BN order).
    auto bn_finalize = [&](int i, int R) -> int {
        const ConvL& C = c->conv[i];
        const BnL& B = c->bn[i];
        const float* part = p.part;
        int G = R;
        if (R > STAT_G) {
            RUN("bn_bwd_reduce", 0, k_reduce_rows(p.part, R, 2 * C.cout, p.part2, STAT_G, s));
            part = p.part2;
            G = STAT_G;
        }
        RUN("bn_bwd_finalize", 0,
            k_bn_bwd_finalize2(part, G, C.cout, (double)p.P[C.level], prm + B.g, p.mean[i],
                               p.invstd[i], p.coef, grads + B.g, grads + B.b, s));
        return 0;
    };
    // dz = A do + B (y - mean) + C as one elementwise pass over do, or (option dz_in_wgrad)
    // inside the weight gradient's B' loader, which also stores it for the dgrad
    const int dz_mask = c->bn_relu ? 0 : 1;
    // conv whose x3 dz pass recomputes `do` from the 1x1 head (set below when it applies)
    int head_src_conv = -1;
    // conv whose x3 dz pass recomputes `do` from the max-pool backward's inputs (option
    // pool_fuse, r05): the encoder block's second conv
    struct PoolSrc {
        int conv = -1;
        const float* dp = nullptr;
        const uint8_t* idx = nullptr;
        const float* dskip = nullptr;
        int ldskip = 0;
        const float *msc = nullptr, *msh = nullptr;
    } pool_src;
    // conv i backward from do_i (dense [P][cout]).
    // dgrad -> dx (ld ldx).  bn_next: dx is the `do` of BN layer i-1 (second conv of a
    // block), so the epilogue also emits that layer's partials; *rows = their count.
    auto conv_bwd = [&](int i, const float* dout, float* dx, int ldx, bool bn_next,
                        int* rows, bool accumulate = false) -> int {
        const ConvL& C = c->conv[i];
        const int Hl = H >> C.level, Wl = W >> C.level;
        const int64_t P = p.P[C.level];
        if (i == 0 && C.pf < 0) {
            RUN("conv_first_wgrad", 2.0 * P * 9 * C.cout,
                k_conv_first_wgrad(p.x_nhwc, dout, p.y[0], p.coef, (int)P, Hl, Wl, C.cout, dz_mask,
                                   p.hpart, wide_g(P), grads + C.w,
                                   C.b >= 0 ? grads + C.b : nullptr, s));
            return 0;
        }
        if (p.pack3 && x3_conv_on(c, C.cin, C.cout)) {
            // option x3: dz as an x3 image (and the conv bias's column partials), the weight
            // gradient from the forward's kept input image and dz, the input gradient from dz
            float* bp = C.b >= 0 ? p.part : nullptr;
            // (r05) the last conv's `do` straight from the 1x1 head (head_bwd stored none)
            const bool hsrc = i == head_src_conv;
            if (i == pool_src.conv) {  // (r05) do straight from the max-pool backward's inputs
                const PoolSrc& q = pool_src;
                RUN("bn_dz", 0, k_bn_dz_x3_pool(p.y[i], p.ldy[i], p.offy[i], P, C.cout, p.coef, dz_mask, p.s3,
                                                bp, q.dp, q.idx, q.dskip, q.ldskip, q.msc, q.msh, p.N, Hl,
                                                Wl, s));
            } else {
                RUN("bn_dz", 0, k_bn_dz_x3(dout, p.y[i], p.ldy[i], p.offy[i], P, C.cout, p.coef, dz_mask,
                                          p.s3, bp, s, hsrc ? dlogits : nullptr,
                                          hsrc ? prm + c->head_w : nullptr, hsrc ? p.scale[i] : nullptr,
                                          hsrc ? p.shift[i] : nullptr, c->bn_relu ? 1 : 0));
            }
            if (bp) {  // many 256-row partials: one two-level reduction (as the BN statistics)
                const int G = x3_dz_blocks(P);
                if (G > STAT_G) {
                    RUN("bias_grad", 0, k_reduce_rows(p.part, G, C.cout, p.part2, STAT_G, s));
                    RUN("bias_grad", 0, k_sum_partials(p.part2, STAT_G, C.cout, grads + C.b, s));
                } else {
                    RUN("bias_grad", 0, k_sum_partials(p.part, G, C.cout, grads + C.b, s));
                }
            }
            const WgradCfg wc = x3_wgrad_cfg(c, C.cin, 9, C.cout, 1, P, Wl, Hl);
            WgradArgs w{};
            w.xcd = 1;
            w.H = Hl;
            w.W = Wl;
            w.P = (int)P;
            w.a = (const float*)p.x3[i];
            w.lda = C.cin;
            w.CA = C.cin;
            w.amode = G_CONV3;
            w.b = (const float*)p.s3;
            w.ldb = C.cout;
            w.CB = C.cout;
            w.bmode = G_IDENT;
            w.Mw = 9 * C.cin;
            w.Nw = C.cout;
            w.pps = wc.pps;
            w.splits = wc.splits;
            w.slab = p.slab;
            w.zero16 = p.zero16;
            RUN(x3wlabel("conv_wgrad", wc, i), 2.0 * P * C.cout * 9 * C.cin, launch_wgrad_x3(w, wc.tile, s));
            RUN("wgrad_reduce", 0,
                k_slab_reduce(p.slab, wc.splits, w.Mw, w.Nw, 0, C.cin, C.cout, grads + C.w, s));
            if (!dx) return 0;
            RowGemmArgs g{};
            g.H = Hl;
            g.W = Wl;
            g.M = (int)P;
            g.N = C.cin;
            g.K = 9 * C.cout;
            g.C = C.cout;
            g.amode = G_CONV3;
            use_x3(c, p, g, p.s3, C.cout, p.pack3 + 3 * C.pd);
            g.out = dx;
            g.ldo = ldx;
            g.ooff = 0;
            g.emode = accumulate ? E_ADD : E_STORE;
            if (bn_next) {
                g.emode = E_STORE_BN;
                g.ey = p.y[i - 1];
                g.ldey = p.ldy[i - 1];
                g.offey = p.offy[i - 1];
                if (c->bn_relu) {
                    g.escale = p.scale[i - 1];
                    g.eshift = p.shift[i - 1];
                }
                g.stats = p.part;
            }
            const int tile = x3_tile(c, g);
            if (rows) *rows = bn_groups(P);
            RUN(xlabel("conv_dgrad", tile, i), 2.0 * P * C.cout * 9 * C.cin, launch_rowgemm_x3(g, tile, s));
            return 0;
        }
        // bf16 image of dz: A operand of the LDS-DMA dgrad, B' of the LDS-DMA wgrad; the f32
        // dz is still written when the register-staged kernel of either consumes it
        const bool dz16 = rg16_on(c, C.cout, C.cin) || p.x16[i];
        Operand a = conv_input(c, p, i);
        WgradCfg wc = wgrad_cfg(c, C.cin, 9, C.cout, 1, P, c->bf16, Wl);
        // option dz_in_wgrad: the weight gradient's B' loader forms dz from do and y (the
        // bn_dz pass disappears) and its first A'-tile blocks store it for the dgrad; f32
        // register-staged weight-gradient tiles only, with a dgrad to feed (r04: both BN orders;
        // BN -> ReLU forms dz unmasked, do already carries the ReLU mask)
        const bool dzw = p.gdz && C.cin <= c->opt.dz_in_wgrad && !dz16 && dx &&
                         (wc.tile < 10 || wc.tile >= 20);
        if (dzw) {
        } else if (dz16) {
            const bool f32 = !p.x16[i] || !(dx && rg16_on(c, C.cout, C.cin));
            if (i == pool_src.conv && !f32) {  // (r06) do straight from the max-pool backward's inputs
                const PoolSrc& q = pool_src;
                RUN("bn_dz", 0, k_bn_dz16_pool(p.y[i], p.ldy[i], p.offy[i], P, C.cout, p.coef, dz_mask, p.s16,
                                               q.dp, q.idx, q.dskip, q.ldskip, q.msc, q.msh, p.N, Hl, Wl, s));
            } else if (i == pool_src.conv) {
                return fail(c, UNET_ERR_INTERNAL, "pool_fuse: conv %d needs an f32 dz", i);
            } else if (i == head_src_conv) {  // (r06) do straight from the 1x1 head
                if (f32) return fail(c, UNET_ERR_INTERNAL, "head_fuse: conv %d needs an f32 dz", i);
                RUN("bn_dz", 0, k_bn_dz16(nullptr, p.y[i], p.ldy[i], p.offy[i], P, C.cout, p.coef, dz_mask,
                                          p.s16, 0, s, dlogits, prm + c->head_w, p.scale[i], p.shift[i],
                                          c->bn_relu ? 1 : 0));
            } else {
                RUN("bn_dz", 0, k_bn_dz16(const_cast<float*>(dout), p.y[i], p.ldy[i], p.offy[i], P, C.cout,
                                          p.coef, dz_mask, p.s16, f32 ? 1 : 0, s));
            }
        } else {
            RUN("bn_dz", 0, k_bn_dz(const_cast<float*>(dout), p.y[i], p.ldy[i], p.offy[i], P, C.cout,
                                    p.coef, dz_mask, s));
        }
        WgradArgs w{};
        w.xcd = xcd_remap_wgrad(c);
        w.H = Hl;
        w.W = Wl;
        w.P = (int)P;
        w.a = a.ptr;
        w.lda = a.ld;
        w.aoff = a.off;
        w.CA = C.cin;
        w.amode = G_CONV3;
        w.ascale = a.scale;
        w.ashift = a.shift;
        w.arelu = a.relu;
        w.b = dout;
        w.ldb = C.cout;
        w.boff = 0;
        w.CB = C.cout;
        w.bmode = G_IDENT;
        w.by = p.y[i];
        w.ldby = p.ldy[i];
        w.offby = p.offy[i];
        w.bcoef = dzw ? p.coef : nullptr;
        w.dzout = dzw ? p.gdz : nullptr;
        w.bdznomask = dz_mask ? 0 : 1;
        w.lddz = C.cout;
        w.bias_slab = C.b >= 0 ? p.bslab : nullptr;
        w.Mw = 9 * C.cin;
        w.Nw = C.cout;
        w.pps = wc.pps;
        w.splits = wc.splits;
        w.slab = p.slab;
        w.bf16 = c->bf16;
        if (p.x16[i]) {
            w.a = (const float*)p.x16[i];
            w.lda = C.cin;
            w.aoff = 0;
            w.ascale = w.ashift = nullptr;
            w.arelu = 0;
            w.b = (const float*)p.s16;
            w.by = nullptr;
            w.bcoef = nullptr;
            w.zero16 = p.zero16;
            w.xcd = xcd16_on(c);
            // (the split count, sized for >= 2048 128x128 tiles, gives >= 512 256x256 ones)
            int t = wg16_tile(c, C.cin, C.cout);
            // option wg16_r3: the tap-row kernel (three taps per block from one halo row)
            const int r3 = c->opt.wg16_r3;
            // (r06) tile 7 also at W = 32 / 16 (the 32^2 level and the 16^2 bottleneck)
            const bool deep = r3 == 7 && (Wl == 32 || Wl == 16) && (Hl * Wl) % 64 == 0 && P % 64 == 0;
            if ((r3 == 4 || r3 == 7) && (Wl % 64 == 0 || deep) && C.cin % 128 == 0 && C.cout % 128 == 0 &&
                wc.pps % 64 == 0)
                t = r3;
            int wbm = 0, wbn = 0, wst = 0;
            wgrad16g_tile_dims(t, &wbm, &wbn, &wst);
            char lb[96];
            snprintf(lb, sizeof lb, "conv_wgrad/wg16%s_%dx%ds%d|%d",
                     t == 4 ? "r3" : t == 7 ? "r3m" : "", wbm, wbn, wst, i);
            RUN(lb, 2.0 * P * C.cout * 9 * C.cin, launch_wgrad16(w, t, s));
        } else {
            RUN(wlabel("conv_wgrad", wc, i), 2.0 * P * C.cout * 9 * C.cin, launch_wgrad(w, wc.tile, s));
        }
        RUN("wgrad_reduce", 0,
            k_slab_reduce(p.slab, wc.splits, w.Mw, w.Nw, 0, C.cin, C.cout, grads + C.w, s));
        if (C.b >= 0) RUN("bias_grad", 0, k_bias_reduce(p.bslab, wc.splits, 1, C.cout, grads + C.b, s));
        if (dx) {
            RowGemmArgs g{};
            g.zero16 = p.zero16;
            g.H = Hl;
            g.W = Wl;
            g.M = (int)P;
            g.N = C.cin;
            g.K = 9 * C.cout;
            g.a = dzw ? p.gdz : dout;
            g.lda = C.cout;
            g.aoff = 0;
            g.C = C.cout;
            g.amode = G_CONV3;
            g.ay = p.y[i];
            g.lday = p.ldy[i];
            g.offay = p.offy[i];
            set_weights(c, g, p.pack + C.pd);
            g.out = dx;
            g.ldo = ldx;
            g.ooff = 0;
            g.emode = accumulate ? E_ADD : E_STORE;
            if (bn_next) {
                g.emode = E_STORE_BN;
                g.ey = p.y[i - 1];
                g.ldey = p.ldy[i - 1];
                g.offey = p.offy[i - 1];
                if (c->bn_relu) {
                    g.escale = p.scale[i - 1];
                    g.eshift = p.shift[i - 1];
                }
                g.stats = p.part;
            }
            if (dz16 && rg16_on(c, C.cout, C.cin)) {
                use_a16(c, p, g, C.cout);
                const int tile = rg16_tile(c, g);
                if (rows) *rows = bn_groups(P);
                RUN(tlabel16("conv_dgrad", tile, i), 2.0 * P * C.cout * 9 * C.cin,
                    launch_rowgemm16(g, tile, s));
                return 0;
            }
            if (rows) *rows = bn_groups(P);
            const int tile = pick_tile(c, C.cin, true, c->bf16);
            RUN(tlabel("conv_dgrad", tile, i), 2.0 * P * C.cout * 9 * C.cin, launch_rowgemm(g, tile, s));
        }
        return 0;
    };
    // ConvT k backward: dOut = up half of dcat[lo]; dx = `do` of its input's BN (partials ->
    // rows)
    auto convT_bwd = [&](int k, float* dx, int* rows) -> int {
        const ConvTL& T = c->convt[k];
        const int src = 2 * (D + k) + 1;
        const int lo = T.in_level - 1;
        const int ldo = 2 * c->ch(lo), uo = c->up_off(lo);
        const int Hi = H >> T.in_level, Wi = W >> T.in_level;
        const int64_t Pin = p.P[T.in_level];
        if (p.pack3 && x3_convt_on(c, T.cin, T.cout)) {
            // option x3: the up half of the concat gradient as an x3 image feeds the weight
            // gradient (B', gathered 2x2) and the input gradient (A)
            RUN("prep_x3", 0, k_to_x3(p.dcat[lo], ldo, uo, T.cout, nullptr, nullptr, 0, p.P[lo], p.s3,
                                      T.cout, 0, s));
            const WgradCfg wc = x3_wgrad_cfg(c, T.cin, 1, T.cout, 4, Pin);
            WgradArgs w{};
            w.xcd = 1;
            w.H = Hi;
            w.W = Wi;
            w.P = (int)Pin;
            w.a = (const float*)p.t3[k];
            w.lda = T.cin;
            w.CA = T.cin;
            w.amode = G_IDENT;
            w.b = (const float*)p.s3;
            w.ldb = T.cout;
            w.CB = T.cout;
            w.bmode = G_UP2;
            w.Mw = T.cin;
            w.Nw = 4 * T.cout;
            w.pps = wc.pps;
            w.splits = wc.splits;
            w.slab = p.slab;
            w.zero16 = p.zero16;
            RUN(x3wlabel("convT_wgrad", wc, 100 + k), 2.0 * Pin * T.cin * 4 * T.cout,
                launch_wgrad_x3(w, wc.tile, s));
            RUN("bias_grad", 0, k_up2_bias_partials(p.dcat[lo], ldo, uo, Hi, Wi, Pin, T.cout, wc.pps,
                                                    wc.splits, p.bslab, s));
            RUN("wgrad_reduce", 0,
                k_slab_reduce(p.slab, wc.splits, w.Mw, w.Nw, 1, T.cin, T.cout, grads + T.w, s));
            RUN("bias_grad", 0, k_bias_reduce(p.bslab, wc.splits, 4, T.cout, grads + T.b, s));
            RowGemmArgs g{};
            g.H = Hi;
            g.W = Wi;
            g.M = (int)Pin;
            g.N = T.cin;
            g.K = 4 * T.cout;
            g.C = T.cout;
            g.amode = G_UP2;
            use_x3(c, p, g, p.s3, T.cout, p.pack3 + 3 * T.pd);
            g.out = dx;
            g.ldo = T.cin;
            g.ooff = 0;
            if (c->res) {  // d(block output); the block's own backward entry masks it
                g.emode = E_STORE;
            } else {
                g.emode = E_STORE_BN;
                g.ey = p.y[src];
                g.ldey = p.ldy[src];
                g.offey = p.offy[src];
                if (c->bn_relu) {
                    g.escale = p.scale[src];
                    g.eshift = p.shift[src];
                }
                g.stats = p.part;
            }
            const int tile = x3_tile(c, g);
            *rows = bn_groups(Pin);
            RUN(xlabel("convT_dgrad", tile, 100 + k), 2.0 * Pin * T.cin * 4 * T.cout,
                launch_rowgemm_x3(g, tile, s));
            return 0;
        }
        WgradCfg wc = wgrad_cfg(c, T.cin, 1, T.cout, 4, Pin, c->bf16);
        WgradArgs w{};
        w.xcd = xcd_remap_wgrad(c);
        w.H = Hi;
        w.W = Wi;
        w.P = (int)Pin;
        if (c->res) {
            w.a = p.out[D + k];
            w.lda = p.ldout[D + k];
            w.aoff = p.offout[D + k];
        } else {
            w.a = p.y[src];
            w.lda = p.ldy[src];
            w.aoff = p.offy[src];
            w.ascale = p.scale[src];
            w.ashift = p.shift[src];
            w.arelu = c->bn_relu ? T.cin : 0;
        }
        w.CA = T.cin;
        w.amode = G_IDENT;
        w.b = p.dcat[lo];
        w.ldb = ldo;
        w.boff = uo;
        w.CB = T.cout;
        w.bmode = G_UP2;
        w.bias_slab = p.bslab;
        w.Mw = T.cin;
        w.Nw = 4 * T.cout;
        w.pps = wc.pps;
        w.splits = wc.splits;
        w.slab = p.slab;
        w.bf16 = c->bf16;
        const bool t16 = p.t16[k] != nullptr;
        if (t16) {
            // bf16 image of the up half of the concat gradient: B' here, A of the dgrad below
            RUN("prep16", 0, k_to_bf16(p.dcat[lo], ldo, uo, T.cout, nullptr, nullptr, 0, p.P[lo],
                                       p.s16, s));
            w.a = (const float*)p.t16[k];
            w.lda = T.cin;
            w.aoff = 0;
            w.ascale = w.ashift = nullptr;
            w.arelu = 0;
            w.b = (const float*)p.s16;
            w.ldb = T.cout;
            w.boff = 0;
            w.bias_slab = nullptr;
            w.zero16 = p.zero16;
            w.xcd = xcd16_on(c);
            const int t = wg16_tile(c, T.cin, T.cout);
            int wbm = 0, wbn = 0, wst = 0;
            wgrad16g_tile_dims(t, &wbm, &wbn, &wst);
            char lb[96];
            snprintf(lb, sizeof lb, "convT_wgrad/wg16_%dx%ds%d|%d", wbm, wbn, wst, 100 + k);
            RUN(lb, 2.0 * Pin * T.cin * 4 * T.cout, launch_wgrad16(w, t, s));
            RUN("bias_grad", 0, k_up2_bias_partials(p.dcat[lo], ldo, uo, Hi, Wi, Pin, T.cout, wc.pps,
                                                    wc.splits, p.bslab, s));
        } else {
            RUN(wlabel("convT_wgrad", wc, 100 + k), 2.0 * Pin * T.cin * 4 * T.cout,
                launch_wgrad(w, wc.tile, s));
        }
        RUN("wgrad_reduce", 0,
            k_slab_reduce(p.slab, wc.splits, w.Mw, w.Nw, 1, T.cin, T.cout, grads + T.w, s));
        RUN("bias_grad", 0, k_bias_reduce(p.bslab, wc.splits, 4, T.cout, grads + T.b, s));
        RowGemmArgs g{};
        g.zero16 = p.zero16;
        g.H = Hi;
        g.W = Wi;
        g.M = (int)Pin;
        g.N = T.cin;
        g.K = 4 * T.cout;
        g.a = p.dcat[lo];
        g.lda = ldo;
        g.aoff = uo;
        g.C = T.cout;
        g.amode = G_UP2;
        set_weights(c, g, p.pack + T.pd);
        g.out = dx;
        g.ldo = T.cin;
        g.ooff = 0;
        if (c->res) {  // d(block output); the block's own backward entry masks it
            g.emode = E_STORE;
        } else {
            g.emode = E_STORE_BN;
            g.ey = p.y[src];
            g.ldey = p.ldy[src];
            g.offey = p.offy[src];
            if (c->bn_relu) {
                g.escale = p.scale[src];
                g.eshift = p.shift[src];
            }
            g.stats = p.part;
        }
        if (!c->res && rg16_on(c, T.cout, T.cin)) {
            if (!t16) {
                RUN("prep16", 0, k_to_bf16(p.dcat[lo], ldo, uo, T.cout, nullptr, nullptr, 0, p.P[lo],
                                           p.s16, s));
            }
            use_a16(c, p, g, T.cout);
            const int tile = rg16_tile(c, g);
            *rows = bn_groups(Pin);
            RUN(tlabel16("convT_dgrad", tile, 100 + k), 2.0 * Pin * T.cin * 4 * T.cout,
                launch_rowgemm16(g, tile, s));
            return 0;
        }
        const int tile = pick_tile(c, T.cin, true, c->bf16, true);
        *rows = bn_groups(Pin);
        RUN(tlabel("convT_dgrad", tile, 100 + k), 2.0 * Pin * T.cin * 4 * T.cout, launch_rowgemm(g, tile, s));
        return 0;
    };
    // gradient bucket b is final once stage bucket_stage[b] is done: record its event (a
    // channel-padded network first compacts the bucket's tensors into the caller's arena,
    // so its all-reduce can overlap the rest of the backward as well)
    auto stage_done = [&](int st) -> int {
        for (size_t b = 0; b < c->bucket_stage.size(); ++b) {
            if (c->bucket_stage[b] != st) continue;
            if (c->padded && c->bucket_p1[b] > c->bucket_p0[b])
                RUN("pad_compact", 0,
                    k_pad_copy(p.ptab + c->bucket_p0[b], c->bucket_p1[b] - c->bucket_p0[b],
                               c->bucket_pmax[b], p.pgrad, p.ugrad, 0, s));
            (void)hipEventRecord(c->bucket_ev[b], s);
        }
        return 0;
    };

    float* G0 = p.g[0];
    float* G1 = p.g[1];
    int R = 0;
    if (c->res) {
        // Residual block b from d(out) in G0: du = d(out)[out > 0] (+ BN2 partials); the skip
        // conv's weight / input gradients from du; BN2 + conv2, then BN1-ReLU + conv1 whose
        // input gradient is ADDED to the skip's in dx (ld ldx; null for the first block).
        auto block_bwd = [&](int b, float* dx, int ldx) -> int {
            const ConvL& CL = c->conv[2 * b];
            const int i1 = 2 * b, i2 = 2 * b + 1;
            const int64_t P = p.P[CL.level];
            RUN("res_bwd_prep", 0, k_res_bwd_prep(G0, p.out[b], p.ldout[b], p.offout[b], p.y[i2], P,
                                                  CL.cout, p.part, RED_G, s));
            if (CL.pf < 0) {
                RUN("skip_wgrad", 2.0 * P * CL.cout,
                    k_res_first_wgrad(p.x_nhwc, G0, (int)P, CL.cout, p.hpart, RED_G,
                                      grads + c->skip_w[b], s));
            } else {
                Operand a = conv_input(c, p, i1);
                WgradCfg wc = wgrad_cfg(c, CL.cin, 1, CL.cout, 1, P, false);
                WgradArgs w{};
                w.xcd = xcd_remap_wgrad(c);
                w.H = H >> CL.level;
                w.W = W >> CL.level;
                w.P = (int)P;
                w.a = a.ptr;
                w.lda = a.ld;
                w.aoff = a.off;
                w.CA = CL.cin;
                w.amode = G_IDENT;
                w.b = G0;
                w.ldb = CL.cout;
                w.CB = CL.cout;
                w.bmode = G_IDENT;
                w.Mw = CL.cin;
                w.Nw = CL.cout;
                w.pps = wc.pps;
                w.splits = wc.splits;
                w.slab = p.slab;
                RUN(wlabel("skip_wgrad", wc, b), 2.0 * P * CL.cin * CL.cout, launch_wgrad(w, wc.tile, s));
                RUN("wgrad_reduce", 0, k_slab_reduce(p.slab, wc.splits, w.Mw, w.Nw, 2, CL.cin, CL.cout,
                                                     grads + c->skip_w[b], s));
                RowGemmArgs g{};
                g.zero16 = p.zero16;
                g.H = H >> CL.level;
                g.W = W >> CL.level;
                g.M = (int)P;
                g.N = CL.cin;
                g.K = CL.cout;
                g.a = G0;
                g.lda = CL.cout;
                g.C = CL.cout;
                g.amode = G_IDENT;
                g.bt = p.pack + c->skip_pd[b];
                g.xcd = xcd_remap_on(c);
                g.out = dx;
                g.ldo = ldx;
                g.emode = E_STORE;
                const int tile = pick_tile(c, CL.cin, true, false);
                RUN(tlabel("skip_dgrad", tile, b), 2.0 * P * CL.cin * CL.cout, launch_rowgemm(g, tile, s));
            }
            if ((rc = bn_finalize(i2, RED_G))) return rc;
            if ((rc = conv_bwd(i2, G0, G1, CL.cout, true, &R))) return rc;
            if ((rc = bn_finalize(i1, R))) return rc;
            return conv_bwd(i1, G1, dx, ldx, false, nullptr, dx != nullptr);
        };
        RUN("head_bwd", 2.0 * p.P[0] * c->base * c->out_ch * 2,
            k_head_bwd(p.out[2 * D], c->base, nullptr, nullptr, 0, prm + c->head_w, c->out_ch,
                       (int)p.P[0], H * W, dlogits, G0, p.hpart, nullptr, wide_g(p.P[0]), s));
        RUN("head_grad", 0, k_sum_partials(p.hpart, wide_g(p.P[0]), c->out_ch * c->base + c->out_ch,
                                           grads + c->head_w, s));
        if ((rc = block_bwd(2 * D, p.dcat[0], 2 * c->base))) return rc;
        if ((rc = stage_done(0))) return rc;
        for (int k = D - 1; k >= 0; --k) {
            const int b = D + k;
            if ((rc = convT_bwd(k, G0, &R))) return rc;
            const int l = c->conv[2 * b].level;
            if (b > D) {
                if ((rc = block_bwd(b, p.dcat[l], 2 * c->ch(l)))) return rc;
            } else if ((rc = block_bwd(b, p.g[2], c->conv[2 * b].cin))) {
                return rc;
            }
            if ((rc = stage_done(D - k))) return rc;
        }
        for (int b = D - 1; b >= 0; --b) {
            const int C = c->ch(b);
            RUN("maxpool_bwd", 0,
                k_maxpool_bwd(p.g[2], p.idx[b], p.dcat[b], 2 * C, c->skip_off(b), nullptr, 0, 0,
                              nullptr, nullptr, p.N, H >> b, W >> b, C, G0, nullptr, RED_G, s));
            if ((rc = block_bwd(b, b > 0 ? p.g[2] : nullptr, b > 0 ? c->conv[2 * b].cin : 0)))
                return rc;
            if ((rc = stage_done(2 * D - b))) return rc;
        }
        return 0;
    }
    // ---- head + last decoder block (stage 0) ----
    const int last = NC - 1;
    // (r05) one output channel on the x3 path (r06: and on the bf16 path's LDS-DMA GEMMs): the
    // last conv's dz pass recomputes `do` = mask * dl * w from the logit gradient, so head_bwd
    // stores no full-resolution f32 `do`
    const ConvL& CL = c->conv[last];
    const bool head_fuse = c->out_ch == 1 && CL.cout == c->base && c->opt.head_fuse &&
                           ((p.pack3 && x3_conv_on(c, CL.cin, CL.cout)) ||
                            (c->bf16 && p.x16[last] && rg16_on(c, CL.cout, CL.cin)));
    head_src_conv = head_fuse ? last : -1;
    RUN("head_bwd", 2.0 * p.P[0] * c->base * c->out_ch * 2,
        k_head_bwd(p.y[last], c->base, p.scale[last], p.shift[last], c->bn_relu ? 1 : 0,
                   prm + c->head_w, c->out_ch, (int)p.P[0], H * W, dlogits, head_fuse ? nullptr : G0,
                   p.hpart, p.part, wide_g(p.P[0]), s));
    RUN("head_grad", 0, k_sum_partials(p.hpart, wide_g(p.P[0]), c->out_ch * c->base + c->out_ch,
                                       grads + c->head_w, s));
    if ((rc = bn_finalize(last, wide_g(p.P[0])))) return rc;
    if ((rc = conv_bwd(last, G0, G1, c->base, true, &R))) return rc;
    if ((rc = bn_finalize(last - 1, R))) return rc;
    if ((rc = conv_bwd(last - 1, G1, p.dcat[0], 2 * c->base, false, nullptr))) return rc;
    if ((rc = stage_done(0))) return rc;
    // ---- ConvT k, then block D+k (the block whose output it up-samples) ----
    for (int k = D - 1; k >= 0; --k) {
        const int b = D + k;
        const int i1 = 2 * b + 1, i0 = 2 * b;
        if ((rc = convT_bwd(k, G0, &R))) return rc;
        if ((rc = bn_finalize(i1, R))) return rc;
        if ((rc = conv_bwd(i1, G0, G1, c->conv[i1].cin, true, &R))) return rc;
        if ((rc = bn_finalize(i0, R))) return rc;
        if (b > D) {
            const int l = c->conv[i0].level;  // input is CAT_l
            if ((rc = conv_bwd(i0, G1, p.dcat[l], 2 * c->ch(l), false, nullptr))) return rc;
        } else {
            // bottleneck: its input is pool[D-1]; G0 <- d pool[D-1]
            if ((rc = conv_bwd(i0, G1, G0, c->conv[i0].cin, false, nullptr))) return rc;
        }
        if ((rc = stage_done(D - k))) return rc;
    }
    // ---- encoders ----
    float* cur = G0;
    for (int b = D - 1; b >= 0; --b) {
        const int C = c->ch(b);
        const int i1 = 2 * b + 1, i0 = 2 * b;
        float* nxt = cur == G0 ? G1 : G0;
        // up to 2048 blocks on the large levels (512 left the pass at ~4.7 TB/s); the partial
        // rows fit: p.part holds P/64 + 1 rows of 2C for every conv of the level
        const int Gmp = wide_g(p.P[b]);
        const ConvL& C1 = c->conv[i1];
        // x3: the conv's x3 dz pass; bf16 (r06): its bf16 dz pass, where no f32 dz is needed
        // (the LDS-DMA dgrad and weight gradient read the bf16 image only)
        const bool pool_fuse =
            c->opt.pool_fuse && !c->res && C1.cout == C && p.P[b] < (1 << 24) &&
            ((p.pack3 && x3_conv_on(c, C1.cin, C1.cout)) ||
             (c->bf16 && p.x16[i1] && rg16_on(c, C1.cout, C1.cin)));
        pool_src = PoolSrc{};
        if (pool_fuse) {
            pool_src.conv = i1;
            pool_src.dp = cur;
            pool_src.idx = p.idx[b];
            pool_src.dskip = p.dcat[b] + c->skip_off(b);
            pool_src.ldskip = 2 * C;
            pool_src.msc = c->bn_relu ? p.scale[i1] : nullptr;
            pool_src.msh = c->bn_relu ? p.shift[i1] : nullptr;
        }
        RUN("maxpool_bwd", 0,
            k_maxpool_bwd(cur, p.idx[b], p.dcat[b], 2 * C, c->skip_off(b), p.y[i1], p.ldy[i1],
                          p.offy[i1], c->bn_relu ? p.scale[i1] : nullptr,
                          c->bn_relu ? p.shift[i1] : nullptr, p.N, H >> b, W >> b, C,
                          pool_fuse ? nullptr : nxt, p.part, Gmp, s));
        cur = nxt;
        nxt = cur == G0 ? G1 : G0;
        if ((rc = bn_finalize(i1, Gmp))) return rc;
        if ((rc = conv_bwd(i1, cur, nxt, C, true, &R))) return rc;
        cur = nxt;
        nxt = cur == G0 ? G1 : G0;
        if ((rc = bn_finalize(i0, R))) return rc;
        if (b > 0) {
            if ((rc = conv_bwd(i0, cur, nxt, c->conv[i0].cin, false, nullptr))) return rc;
            cur = nxt;
        } else {
            if ((rc = conv_bwd(0, cur, nullptr, 0, false, nullptr))) return rc;
        }
        if ((rc = stage_done(2 * D - b))) return rc;
    }
    return 0;
}

// Pillow's precompute_coeffs + normalize_coeffs_8bpc (libImaging/Resample.c) for the
// BILINEAR filter (support 1) over the full source extent [0, in_size): same double
// arithmetic in the same order, then the 22-bit fixed-point conversion.
int pil_resample_plan(int in_size, int out_size, int32_t* kk, int32_t* bounds) {
    const double in0 = 0.0, in1 = (double)(float)in_size;
    double filterscale, scale;
    filterscale = scale = (double)(in1 - in0) / out_size;
    if (filterscale < 1.0) filterscale = 1.0;
    const double support = 1.0 * filterscale;
    const int ksize = (int)ceil(support) * 2 + 1;
    if (!kk || !bounds) return ksize;
    std::vector<double> k(ksize);
    for (int xx = 0; xx < out_size; ++xx) {
        const double center = in0 + (xx + 0.5) * scale;
        double ww = 0.0;
        const double ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        int x = 0;
        for (; x < xmax; ++x) {
            double a = (x + xmin - center + 0.5) * ss;
            if (a < 0.0) a = -a;
            const double w = a < 1.0 ? 1.0 - a : 0.0;
            k[x] = w;
            ww += w;
        }
        for (x = 0; x < xmax; ++x)
            if (ww != 0.0) k[x] /= ww;
        for (; x < ksize; ++x) k[x] = 0;
        for (x = 0; x < ksize; ++x)
            kk[(int64_t)xx * ksize + x] = k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << (32 - 8 - 2)))
                                                   : (int32_t)(0.5 + k[x] * (1 << (32 - 8 - 2)));
        bounds[2 * xx] = xmin;
        bounds[2 * xx + 1] = xmax;
    }
    return ksize;
}

bool shape_ok(const unet_ctx* c, int N, int H, int W) {
    const int q = 1 << std::max(c->depth, 4);  // every level even; >= 16 (model.py contract)
    return N >= 1 && H >= q && W >= q && H % q == 0 && W % q == 0;
}

}  // namespace

// ====================================== C ABI ======================================
extern "C" {

int unet_create(const unet_cfg* cfg, int device, unet_ctx** out) {
    if (!out) return UNET_ERR_INVALID;
    *out = nullptr;
    try {
        std::unique_ptr<unet_ctx> c(new unet_ctx());
        c->device = device;
        int cus = 0;  // (no device in a CPU-only process: keep the MI355X's 256)
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
            c->cus = cus;
        else
            (void)hipGetLastError();
        if (cfg) {
            c->in_ch = cfg->in_channels;
            c->out_ch = cfg->out_channels;
            c->variant = cfg->variant;
            c->bf16 = cfg->math == UNET_MATH_BF16;
            if (cfg->math != UNET_MATH_F32 && cfg->math != UNET_MATH_BF16) return UNET_ERR_UNSUPPORTED;
            if (c->variant == UNET_VARIANT_MOD || c->variant == UNET_VARIANT_RES) {
                // mod.py:13-14 / :91-92 defaults base 64, depth 5
                c->base = cfg->base_filters > 0 ? cfg->base_filters : 64;
                c->depth = cfg->depth > 0 ? cfg->depth : 5;
            } else if ((cfg->base_filters > 0 && cfg->base_filters != 64) ||
                       (cfg->depth > 0 && cfg->depth != 4)) {
                return UNET_ERR_UNSUPPORTED;  // models/model.py:UNet has a fixed topology
            }
        }
        // The first conv kernel is specialised for a single input channel (every BASELINE
        // config); the GEMM tiles need 32-multiples of channels at every level (32-output
        // row tiles 13 / 14 and 32-channel wgrad tiles 8..10 for a 32-channel level 0) and the
        // channel-quad row kernels (pool, head, BN backward) a power-of-two channel count,
        // so the kernels run base 32, 64, 128 or 256.  Other base_filters (the reference
        // grid's 16 / 24 / 48, config/config.yaml; any multiple of 8 up to 256) run padded to
        // the next power of two >= 32 (unet_ctx::padded); the head's fused BN-partials path
        // handles up to 4 classes.
        // Per level: level 0 runs the next power of two >= 32 channels (the head and
        // first-conv kernels want a power-of-two channel-quad count), every deeper level the
        // next multiple of 32 of base_filters << l (a K-chunk is 32 channels of one tap), and
        // since r06 an odd multiple of 32 from 96 on the next multiple of 64 (below), so base
        // 16 pads level 0 only (16 -> 32, then 32, 64, ...: r03 padded every level 2x), base 48
        // levels 0 and 1 (48 -> 64, 96 -> 128, then 192, 384, ...), base 24 levels 0..2 (24 ->
        // 32, 48 -> 64, 96 -> 128).
        c->rbase = c->base;
        if (c->base < 8 || c->base > 256 || c->base % 8 || c->depth < 1 || c->depth > MAX_DEPTH)
            return UNET_ERR_UNSUPPORTED;
        c->padded = false;
        for (int l = 0; l <= c->depth; ++l) {
            int pc = 32;
            if (l == 0) {
                while (pc < c->rbase) pc <<= 1;
            } else {
                pc = ((c->rbase << l) + 31) / 32 * 32;
                // (r06) 96, 160, 224, ... channels run padded to the next multiple of 64: the
                // x3 GEMMs (f32 math on the bf16 matrix cores) take 64-multiples, and padded x3
                // beats the native f32 MFMA kernels (96 -> 128: 1.78x the FLOPs at ~2.2x the
                // rate; base 48's 96-channel level 1 and base 24's level 2)
                if (pc % 64 == 32 && pc >= 96) pc += 32;
            }
            c->chl[l] = pc;
            c->padded = c->padded || pc != (c->rbase << l);
        }
        c->base = c->chl[0];
        if ((c->variant != UNET_VARIANT_MODEL && c->variant != UNET_VARIANT_MOD &&
             c->variant != UNET_VARIANT_RES) || c->in_ch != 1 ||
            c->out_ch < 1 || c->out_ch > 4 || c->ch(c->depth) > 8192)
            return UNET_ERR_UNSUPPORTED;
        if ((c->padded || c->base < 64) && c->bf16)  // the bf16 kernels: 128-multiples of real channels
            return UNET_ERR_UNSUPPORTED;
        c->res = c->variant == UNET_VARIANT_RES;
        c->bn_relu = c->variant != UNET_VARIANT_MODEL;
        c->skip_first = c->bn_relu;
        if (c->bf16 && c->variant != UNET_VARIANT_MOD)  // bf16 GEMMs: mod.py UNet (config 4) only
            return UNET_ERR_UNSUPPORTED;
        build_graph(c.get());
        *out = c.release();
        return UNET_OK;
    } catch (const std::bad_alloc&) {
        return UNET_ERR_NOMEM;
    } catch (...) {
        return UNET_ERR_INTERNAL;
    }
}

int unet_destroy(unet_ctx* c) {
    ABI_TRY
    if (!c) return UNET_ERR_INVALID;
    for (auto e : c->bucket_ev) (void)hipEventDestroy(e);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->pp || c->pp3 || c->lpart) {
        (void)hipSetDevice(c->device);
        if (c->pp) (void)hipFree(c->pp);
        if (c->pp3) (void)hipFree(c->pp3);
        if (c->lpart) (void)hipFree(c->lpart);
    }
    delete c;
    return UNET_OK;
    ABI_CATCH(c)
}

const char* unet_last_error(const unet_ctx* c) { return c ? c->err.c_str() : "null context"; }

int unet_num_params(const unet_ctx* c, int* n, int64_t* nf) {
    if (!c) return UNET_ERR_INVALID;
    if (n) *n = (int)c->params.size();
    if (nf) *nf = c->n_param_floats;
    return UNET_OK;
}

int unet_param_info(const unet_ctx* c, int i, const char** name, int* ndim, int64_t shape[4],
                    int64_t* offset) {
    ABI_TRY
    if (!c || i < 0 || i >= (int)c->params.size()) return UNET_ERR_INVALID;
    const ParamT& p = c->params[i];
    if (name) *name = p.name.c_str();
    if (ndim) *ndim = p.ndim;
    if (shape)
        for (int k = 0; k < 4; ++k) shape[k] = p.shape[k];
    if (offset) *offset = p.off;
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_num_bn(const unet_ctx* c, int* n, int64_t* nf) {
    ABI_TRY
    if (!c) return UNET_ERR_INVALID;
    if (n) *n = c->nconv();
    if (nf) *nf = c->n_bn_floats;
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_bn_info(const unet_ctx* c, int i, const char** name, int* ch, int64_t* off) {
    ABI_TRY
    if (!c || i < 0 || i >= c->nconv()) return UNET_ERR_INVALID;
    if (name) *name = c->bn[i].name.c_str();
    if (ch) *ch = c->bn[i].rC;
    if (off) *off = c->bn[i].rrun;
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_workspace_size(unet_ctx* c, int N, int H, int W, int training, size_t* bytes) {
    ABI_TRY
    if (!c || !bytes) return UNET_ERR_INVALID;
    if (!shape_ok(c, N, H, W)) return fail(c, UNET_ERR_SHAPE, "bad shape N=%d H=%d W=%d", N, H, W);
    Plan p;
    make_plan(c, N, H, W, training != 0, nullptr, p);
    *bytes = p.bytes;
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_forward(unet_ctx* c, const float* params, float* bn_running, int64_t* bn_count,
                 const float* x, float* logits, void* ws, size_t ws_bytes, int N, int H, int W,
                 int training, unet_stream_t stream) {
    ABI_TRY
    if (!c || !params || !x || !logits || !ws) return c ? fail(c, UNET_ERR_INVALID, "null pointer") : UNET_ERR_INVALID;
    if (!shape_ok(c, N, H, W)) return fail(c, UNET_ERR_SHAPE, "bad shape N=%d H=%d W=%d", N, H, W);
    if (!training && !bn_running)
        return fail(c, UNET_ERR_INVALID, "eval forward needs running statistics");
    Plan p;
    make_plan(c, N, H, W, training != 0, nullptr, p);
    if (ws_bytes < p.bytes) return fail(c, UNET_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, p.bytes);
    make_plan(c, N, H, W, training != 0, (char*)ws, p);
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, UNET_ERR_HIP, "hipSetDevice");
    if (!c->timing) c->ev_used = 0;
    if (training) {
        c->fwd_opt = c->opt;
        c->fwd_opt_set = true;
    }
    const hipStream_t s = (hipStream_t)stream;
    if (!c->padded)
        return forward_impl(c, params, bn_running, bn_count, x, logits, p, training != 0, s);
    // narrow network: torch-layout arenas -> padded arenas, forward, running stats back
    int r = upload_pad_tables(c, p, s);
    if (!r) r = k_pad_copy(p.ptab, (int)c->pad_params.size(), c->pad_max_numel, params, p.pprm, 1, s);
    if (!r && bn_running)
        r = k_pad_copy(p.btab, (int)c->pad_bn.size(), c->pad_bn_max, bn_running, p.pbn, 1, s);
    if (r) return fail(c, UNET_ERR_HIP, "channel-padding expand: %d", r);
    r = forward_impl(c, p.pprm, bn_running ? p.pbn : nullptr, bn_count, x, logits, p,
                     training != 0, s);
    if (r) return r;
    if (training && bn_running &&
        k_pad_copy(p.btab, (int)c->pad_bn.size(), c->pad_bn_max, p.pbn, bn_running, 0, s))
        return fail(c, UNET_ERR_HIP, "channel-padding compact (running stats)");
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_backward(unet_ctx* c, const float* params, const float* dlogits, float* grads, void* ws,
                  size_t ws_bytes, int N, int H, int W, unet_stream_t stream) {
    ABI_TRY
    if (!c || !params || !dlogits || !grads || !ws) return c ? fail(c, UNET_ERR_INVALID, "null pointer") : UNET_ERR_INVALID;
    if (!shape_ok(c, N, H, W)) return fail(c, UNET_ERR_SHAPE, "bad shape N=%d H=%d W=%d", N, H, W);
    if (!c->fwd_opt_set) return fail(c, UNET_ERR_INVALID, "backward without a training forward");
    for (const OptionDesc& d : OPTION_TABLE)
        if (c->opt.*d.field != c->fwd_opt.*d.field)
            return fail(c, UNET_ERR_INVALID,
                        "option '%s' changed between the training forward (%d) and its backward "
                        "(%d): the workspace plan depends on it",
                        d.name, c->fwd_opt.*d.field, c->opt.*d.field);
    Plan p;
    make_plan(c, N, H, W, true, nullptr, p);
    if (ws_bytes < p.bytes) return fail(c, UNET_ERR_WORKSPACE, "workspace %zu < %zu", ws_bytes, p.bytes);
    make_plan(c, N, H, W, true, (char*)ws, p);
    if (c->fwd_used_pp) {  // (r06) the forward read the fused AdamW's weight images
        if (c->pp_gen != c->fwd_pp_gen || !c->pp_ok)
            return fail(c, UNET_ERR_INVALID,
                        "the weight images the training forward used were rewritten before its "
                        "backward (unet_adamw_repack / unet_params_changed in between)");
        p.pack = c->pp;
        if (p.pack3) p.pack3 = c->pp3;
    }
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, UNET_ERR_HIP, "hipSetDevice");
    if (c->bucket_ev.empty()) {
        c->bucket_ev.resize(c->bucket_off.size());
        for (auto& e : c->bucket_ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    }
    const hipStream_t s = (hipStream_t)stream;
    if (!c->padded) return backward_impl(c, params, dlogits, grads, p, s);
    // narrow network: the padded parameters expanded by the forward are still in the
    // workspace; each bucket's gradients are compacted into the caller's arena as soon as
    // they are final (backward_impl stage_done), then its event is recorded
    p.ugrad = grads;
    return backward_impl(c, p.pprm, dlogits, p.pgrad, p, s);
    ABI_CATCH(c)
}

int unet_loss_stats(unet_ctx* c, const float* logits, const float* targets, int N, int C, int H,
                    int W, float* stats, double* sums, unet_stream_t stream) {
    ABI_TRY
    if (!c || !logits || !targets || !stats || !sums) return UNET_ERR_INVALID;
    if (N < 1 || C < 1 || H < 1 || W < 1) return fail(c, UNET_ERR_SHAPE, "bad loss shape");
    const int64_t per = (int64_t)C * H * W, need = 4 * (int64_t)N * loss_groups(per);
    if (need > c->lpart_n) {
        if (hipSetDevice(c->device) != hipSuccess) return fail(c, UNET_ERR_HIP, "hipSetDevice");
        if (c->lpart) {  // a loss pass of an earlier call may still read it
            (void)hipDeviceSynchronize();
            (void)hipFree(c->lpart);
        }
        c->lpart_n = 0;
        if (hipMalloc((void**)&c->lpart, sizeof(float) * (size_t)need) != hipSuccess) {
            c->lpart = nullptr;
            return fail(c, UNET_ERR_HIP, "hipMalloc: loss partials: %lld floats", (long long)need);
        }
        c->lpart_n = need;
    }
    int r = k_loss_stats(logits, targets, N, per, stats, sums, c->lpart, (hipStream_t)stream);
    return r ? fail(c, UNET_ERR_HIP, "loss_stats launch %d", r) : UNET_OK;
    ABI_CATCH(c)
}

int unet_loss_finalize(unet_ctx* c, const double* sums, float* losses, float fa, float fb,
                       float fg, unet_stream_t stream) {
    ABI_TRY
    if (!c || !sums || !losses) return UNET_ERR_INVALID;
    int r = k_loss_finalize(sums, fa, fb, fg, losses, (hipStream_t)stream);
    return r ? fail(c, UNET_ERR_HIP, "loss_finalize launch %d", r) : UNET_OK;
    ABI_CATCH(c)
}

int unet_loss_fwd(unet_ctx* c, const float* logits, const float* targets, int N, int C, int H,
                  int W, float* stats, double* sums, float* losses, float fa, float fb, float fg,
                  unet_stream_t stream) {
    const int r = unet_loss_stats(c, logits, targets, N, C, H, W, stats, sums, stream);
    return r ? r : unet_loss_finalize(c, sums, losses, fa, fb, fg, stream);
}

int unet_loss_bwd(unet_ctx* c, const float* logits, const float* targets, int N, int C, int H,
                  int W, const float* stats, const double* sums, const float* w, float* dlogits,
                  float fa, float fb, float fg, unet_stream_t stream) {
    ABI_TRY
    if (!c || !logits || !targets || !stats || !sums || !w || !dlogits) return UNET_ERR_INVALID;
    if (N < 1 || C < 1 || H < 1 || W < 1) return fail(c, UNET_ERR_SHAPE, "bad loss shape");
    int r = k_loss_bwd(logits, targets, N, (int64_t)C * H * W, stats, sums, w, fa, fb, fg, dlogits,
                       (hipStream_t)stream);
    return r ? fail(c, UNET_ERR_HIP, "loss_bwd launch %d", r) : UNET_OK;
    ABI_CATCH(c)
}

int unet_adamw(unet_ctx* c, float* params, const float* grads, float* m, float* v, int64_t n,
               int step, double lr, double b1, double b2, double eps, double wd, double gscale,
               unet_stream_t stream) {
    ABI_TRY
    if (!c || !params || !grads || !m || !v || n < 0 || step < 1) return UNET_ERR_INVALID;
    // torch optim/adam.py _single_tensor_adam: every scalar is a Python float (double)
    // that ATen rounds to float once when it meets the fp32 tensor
    AdamwScalars a;
    a.decay = (float)(1.0 - lr * wd);                 // param.mul_(1 - lr * weight_decay)
    a.w1 = (float)(1.0 - b1);                         // exp_avg.lerp_(grad, 1 - beta1)
    a.lerp_small = fabs(1.0 - b1) < 0.5 ? 1 : 0;
    a.b2 = (float)b2;                                 // exp_avg_sq.mul_(beta2)
    a.w2 = (float)(1.0 - b2);                         // .addcmul_(grad, grad, value=1 - beta2)
    const double bc1 = 1.0 - pow(b1, (double)step);   // beta1 ** step (Python float pow)
    const double bc2 = 1.0 - pow(b2, (double)step);
    a.neg_step = (float)(-(lr / bc1));                // addcdiv_(..., value=-step_size)
    a.bc2_sqrt = (float)pow(bc2, 0.5);                // bias_correction2 ** 0.5
    a.eps = (float)eps;                               // .add_(eps)
    a.gscale = (float)gscale;
    int r = k_adamw(params, grads, m, v, n, a, (hipStream_t)stream);
    return r ? fail(c, UNET_ERR_HIP, "adamw launch %d", r) : UNET_OK;
    ABI_CATCH(c)
}

int unet_adamw_repack(unet_ctx* c, float* params, const float* grads, float* m, float* v, int64_t n,
                      int step, double lr, double b1, double b2, double eps, double wd, double gscale,
                      unet_stream_t stream) {
    ABI_TRY
    if (!c || !params || !grads || !m || !v || n < 0 || step < 1) return UNET_ERR_INVALID;
    // a narrow (channel-padded) network packs from its padded arena: the plain update, and the
    // next forward repacks
    if (n != c->n_param_floats || c->padded) {
        c->pp_ok = false;
        return unet_adamw(c, params, grads, m, v, n, step, lr, b1, b2, eps, wd, gscale, stream);
    }
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, UNET_ERR_HIP, "hipSetDevice");
    const bool x3 = plan_has_pack3(c);
    if (!c->pp && hipMalloc((void**)&c->pp, sizeof(float) * (size_t)std::max<int64_t>(c->pack_floats, 32)) != hipSuccess) {
        c->pp = nullptr;
        return fail(c, UNET_ERR_HIP, "hipMalloc: weight images: %lld floats", (long long)c->pack_floats);
    }
    if (x3 && !c->pp3 &&
        hipMalloc((void**)&c->pp3, 3 * sizeof(uint16_t) * (size_t)std::max<int64_t>(c->pack_floats, 32)) != hipSuccess) {
        c->pp3 = nullptr;
        return fail(c, UNET_ERR_HIP, "hipMalloc: x3 weight images: %lld floats", (long long)c->pack_floats);
    }
    PackJobs jobs{};
    if (!build_pack_jobs(c, true, jobs)) return fail(c, UNET_ERR_INTERNAL, "pack job table full");
    // the arena ranges the pack jobs do not cover, in order
    std::vector<std::pair<int64_t, int64_t>> wr;  // [begin, end) of the packed weight tensors
    for (int k = 0; k < jobs.n; ++k) {
        const PackJob& J = jobs.j[k];
        wr.push_back({J.w, J.w + (int64_t)J.cin * J.cout * (J.kind == 0 ? 9 : 4)});
    }
    std::sort(wr.begin(), wr.end());
    AdamRanges rest{};
    int64_t at = 0, cum = 0;
    auto gap = [&](int64_t b, int64_t e) -> bool {
        if (e <= b) return true;
        if (rest.n >= MAX_ADAM_RANGES) return false;
        rest.off[rest.n] = b;
        rest.cum[rest.n] = cum;
        cum += e - b;
        ++rest.n;
        return true;
    };
    for (auto& r : wr) {
        if (!gap(at, r.first)) return fail(c, UNET_ERR_INTERNAL, "adamw range table full");
        at = std::max(at, r.second);
    }
    if (!gap(at, n)) return fail(c, UNET_ERR_INTERNAL, "adamw range table full");
    rest.cum[rest.n] = cum;
    AdamwScalars a;  // (as unet_adamw)
    a.decay = (float)(1.0 - lr * wd);
    a.w1 = (float)(1.0 - b1);
    a.lerp_small = fabs(1.0 - b1) < 0.5 ? 1 : 0;
    a.b2 = (float)b2;
    a.w2 = (float)(1.0 - b2);
    const double bc1 = 1.0 - pow(b1, (double)step);
    const double bc2 = 1.0 - pow(b2, (double)step);
    a.neg_step = (float)(-(lr / bc1));
    a.bc2_sqrt = (float)pow(bc2, 0.5);
    a.eps = (float)eps;
    a.gscale = (float)gscale;
    const hipStream_t s = (hipStream_t)stream;
    c->pp_ok = false;
    ++c->pp_gen;
    int r = k_pack_adamw(jobs, rest, params, grads, m, v, a, c->pp, c->bf16 ? 1 : 0, s);
    if (!r && x3) r = k_to_x3(c->pp, 32, 0, 32, nullptr, nullptr, 0, c->pack_floats / 32, c->pp3, 32, 0, s);
    if (r) return fail(c, UNET_ERR_HIP, "adamw repack launch %d", r);
    c->pp_src = params;
    c->pp_ok = true;
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_params_changed(unet_ctx* c) {
    if (!c) return UNET_ERR_INVALID;
    c->pp_ok = false;
    return UNET_OK;
}

int unet_x3_split_host(const float* v, int64_t n, uint16_t* out) {
    if (!v || !out || n < 0 || n % 32) return UNET_ERR_INVALID;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t r = i / 32, j = i % 32;
        x3_split(v[i], X3CvtHost{}, out[96 * r + j], out[96 * r + 32 + j], out[96 * r + 64 + j]);
    }
    return UNET_OK;
}

int unet_x3_split_device(unet_ctx* c, const float* v, int64_t n, uint16_t* out, unet_stream_t stream) {
    ABI_TRY
    if (!c || !v || !out || n < 32 || n % 32) return c ? fail(c, UNET_ERR_INVALID, "x3 split: n") : UNET_ERR_INVALID;
    if (hipSetDevice(c->device) != hipSuccess) return fail(c, UNET_ERR_HIP, "hipSetDevice");
    const int r = k_to_x3(v, 32, 0, 32, nullptr, nullptr, 0, n / 32, out, 32, 0, (hipStream_t)stream);
    return r ? fail(c, UNET_ERR_HIP, "to_x3 launch %d", r) : UNET_OK;
    ABI_CATCH(c)
}

int unet_set_option(unet_ctx* c, const char* name, int64_t value) {
    ABI_TRY
    if (!c || !name) return UNET_ERR_INVALID;
    for (const OptionDesc& d : OPTION_TABLE)
        if (strcmp(d.name, name) == 0) {
            c->opt.*d.field = (int)value;
            return UNET_OK;
        }
    return fail(c, UNET_ERR_INVALID, "unknown option '%s'", name);
    ABI_CATCH(c)
}

int unet_get_option(const unet_ctx* c, const char* name, int64_t* value) {
    ABI_TRY
    if (!c || !name || !value) return UNET_ERR_INVALID;
    for (const OptionDesc& d : OPTION_TABLE)
        if (strcmp(d.name, name) == 0) {
            *value = c->opt.*d.field;
            return UNET_OK;
        }
    return UNET_ERR_INVALID;
    ABI_CATCH(c)
}

int unet_mask_counts(unet_ctx* c, const float* logits, const float* targets, int64_t n,
                     uint8_t* mask, int64_t* counts, unet_stream_t stream) {
    ABI_TRY
    if (!c || !logits || !targets || !counts || n < 0) return UNET_ERR_INVALID;
    int r = k_mask_counts(logits, targets, n, mask, counts, (hipStream_t)stream);
    return r ? fail(c, UNET_ERR_HIP, "mask_counts launch %d", r) : UNET_OK;
    ABI_CATCH(c)
}

int unet_num_buckets(const unet_ctx* c, int* n) {
    ABI_TRY
    if (!c || !n) return UNET_ERR_INVALID;
    *n = (int)c->bucket_off.size();
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_bucket_range(const unet_ctx* c, int b, int64_t* off, int64_t* len) {
    ABI_TRY
    if (!c || b < 0 || b >= (int)c->bucket_off.size()) return UNET_ERR_INVALID;
    if (off) *off = c->bucket_off[b];
    if (len) *len = c->bucket_len[b];
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_stream_wait_bucket(unet_ctx* c, int b, unet_stream_t stream) {
    ABI_TRY
    if (!c || b < 0 || b >= (int)c->bucket_ev.size()) return UNET_ERR_INVALID;
    if (hipStreamWaitEvent((hipStream_t)stream, c->bucket_ev[b], 0) != hipSuccess)
        return fail(c, UNET_ERR_HIP, "hipStreamWaitEvent");
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_bucket_event(unet_ctx* c, int b, void** hip_event) {
    ABI_TRY
    if (!c || !hip_event || b < 0 || b >= (int)c->bucket_ev.size()) return UNET_ERR_INVALID;
    *hip_event = (void*)c->bucket_ev[b];
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_option_name(int i, const char** name) {
    if (!name || i < 0 || i >= (int)(sizeof OPTION_TABLE / sizeof OPTION_TABLE[0]))
        return UNET_ERR_INVALID;
    *name = OPTION_TABLE[i].name;
    return UNET_OK;
}

int unet_timing_enable(unet_ctx* c, int en) {
    ABI_TRY
    if (!c) return UNET_ERR_INVALID;
    c->timing = en != 0;
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_timing_filter(unet_ctx* c, const char* substring) {
    ABI_TRY
    if (!c) return UNET_ERR_INVALID;
    c->tfilter = substring ? substring : "";
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_timing_reset(unet_ctx* c) {
    ABI_TRY
    if (!c) return UNET_ERR_INVALID;
    c->trec.clear();
    c->ev_used = 0;
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_timing_count(unet_ctx* c, int* n) {
    ABI_TRY
    if (!c || !n) return UNET_ERR_INVALID;
    *n = (int)c->trec.size();
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_timing_read(unet_ctx* c, int i, const char** family, int64_t* launches, double* total_ms,
                     double* flop) {
    ABI_TRY
    if (!c || i < 0 || i >= (int)c->trec.size()) return UNET_ERR_INVALID;
    TimeRec& t = c->trec[i];
    if (hipEventSynchronize(t.b) != hipSuccess) return fail(c, UNET_ERR_HIP, "event sync");
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, t.a, t.b);
    if (family) *family = t.label.c_str();
    if (launches) *launches = 1;
    if (total_ms) *total_ms = ms;
    if (flop) *flop = t.flop;
    return UNET_OK;
    ABI_CATCH(c)
}

int unet_resize_plan(int in_size, int out_size, int32_t* coeffs, int32_t* bounds, int* ksize) {
    ABI_TRY
    if (in_size < 1 || out_size < 1 || !ksize) return UNET_ERR_INVALID;
    *ksize = pil_resample_plan(in_size, out_size, coeffs, bounds);
    return UNET_OK;
    ABI_CATCH((unet_ctx*)nullptr)
}

int unet_resize_u8(unet_ctx* c, const uint8_t* src, int h, int w, float* dst, int oh, int ow,
                   const int32_t* kh, const int32_t* bh, int ksh, const int32_t* kv,
                   const int32_t* bv, int ksv, float divisor, unet_stream_t stream) {
    ABI_TRY
    if (!c || !src || !dst || h < 1 || w < 1 || oh < 1 || ow < 1 || !(divisor > 0.f))
        return UNET_ERR_INVALID;
    const int need_h = ow != w, need_v = oh != h;
    if ((need_h && (!kh || !bh || ksh < 1)) || (need_v && (!kv || !bv || ksv < 1)))
        return fail(c, UNET_ERR_INVALID, "resize: missing coefficient tables");
    int r = k_resize_u8(src, h, w, dst, oh, ow, kh, bh, ksh, kv, bv, ksv, need_h, need_v, divisor,
                        (hipStream_t)stream);
    return r ? fail(c, UNET_ERR_HIP, "resize launch %d", r) : UNET_OK;
    ABI_CATCH(c)
}

int unet_debug_view(unet_ctx* c, int N, int H, int W, int training, int kind, int index,
                    int64_t* byte_offset, int64_t* count, int* ld, int* off) {
    ABI_TRY
    if (!c || !byte_offset || !count) return UNET_ERR_INVALID;
    if (!shape_ok(c, N, H, W)) return fail(c, UNET_ERR_SHAPE, "bad shape");
    Plan p;
    char* const base = (char*)(uintptr_t)4096;  // fake base: offsets only
    make_plan(c, N, H, W, training != 0, base, p);
    const void* q = nullptr;
    int64_t n = 0;
    int l = 1, o = 0;
    if (kind <= 4) {
        if (index < 0 || index >= c->nconv()) return UNET_ERR_INVALID;
        const ConvL& L = c->conv[index];
        const int C = L.cout;
        if (kind == 0) {
            q = p.y[index];
            l = p.ldy[index];
            o = p.offy[index];
            n = p.P[L.level] * l;
        } else {
            q = kind == 1 ? p.scale[index] : kind == 2 ? p.shift[index] : kind == 3 ? p.mean[index] : p.invstd[index];
            n = C;
        }
    } else {
        if (index < 0 || index >= c->depth) return UNET_ERR_INVALID;
        const int C = c->ch(index);
        if (kind == 5) {
            // the x3 path's max-pool writes the next conv's x3 image instead (forward_impl):
            // the f32 pooled buffer is never written there
            const ConvL& Cj = c->conv[2 * (index + 1)];
            if (!c->res && p.pack3 && x3_conv_on(c, Cj.cin, Cj.cout))
                return fail(c, UNET_ERR_INVALID, "debug view 5: level %d pools into an x3 image", index);
            // (r06) ... and a bf16 training pass pools into the next conv's bf16 image
            if (!c->res && training && c->bf16 && wg16_on(c, Cj.cin, Cj.cout) && rg16_on(c, Cj.cin, Cj.cout))
                return fail(c, UNET_ERR_INVALID, "debug view 5: level %d pools into a bf16 image", index);
            q = p.pool[index];
            n = p.P[index + 1] * C;
            l = C;
        } else if (kind == 6) {
            q = p.cat[index];
            n = p.P[index] * 2 * C;
            l = 2 * C;
        } else if (kind == 7) {
            if (!training) return UNET_ERR_INVALID;
            q = p.dcat[index];
            n = p.P[index] * 2 * C;
            l = 2 * C;
        } else if (kind == 8) {  // max-pool winner index (uint8, window position 0..3)
            q = p.idx[index];
            n = p.P[index + 1] * C;
            l = C;
        } else {
            return UNET_ERR_INVALID;
        }
    }
    *byte_offset = (int64_t)((const char*)q - base);
    *count = n;
    if (ld) *ld = l;
    if (off) *off = o;
    return UNET_OK;
    ABI_CATCH(c)
}

}  // extern "C"
