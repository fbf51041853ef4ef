// Host launchers of kernels_misc.hip (internal).
#pragma once
#include "common.h"

// Weight images of the row GEMMs, every 3x3 conv (kind 0) and ConvTranspose (kind 1) of the
// network in one launch.  Offsets w (params), f / d (forward / dgrad images; d < 0: none)
// count floats; bf16 images (round to nearest even) are addressed at the same float offsets.
// A job covers tx x ty 32x32 tiles (conv3: x over cin, y over cout; ConvT: x over cout, y
// over cin) starting at block block0.
struct PackJob {
    int64_t w, f, d;
    int cin, cout, kind, tx, ty, block0;
};
constexpr int MAX_PACK_JOBS = 48;
struct PackJobs {
    int n;
    PackJob j[MAX_PACK_JOBS];
};
int k_pack_all(const PackJobs& jobs, const float* prm, float* pack, int bf16, hipStream_t s);
// (r06) AdamW fused into the weight repack (unet_adamw_repack): the pack jobs' weight tensors
// are updated in place and packed from the updated values; `rest` lists the other arena ranges
// (elementwise AdamW).  Bit-identical to k_adamw over the whole arena followed by k_pack_all.
constexpr int MAX_ADAM_RANGES = 120;
struct AdamRanges {
    int n;
    int64_t off[MAX_ADAM_RANGES];      // arena offset of range k
    int64_t cum[MAX_ADAM_RANGES + 1];  // elements before range k (cum[n] = total)
};
struct AdamwScalars;
int k_pack_adamw(const PackJobs& jobs, const AdamRanges& rest, float* p, const float* g, float* m, float* v,
                 const AdamwScalars& a, float* pack, int bf16, hipStream_t s);
// conv_first: relu = ReLU after (+bias) (model.py order); b may be null (mod.py, bias-free).
// wgrad: mask = dz masked by [y > 0] (ReLU before the BN, model.py order); gb may be null.
int k_conv_first_fwd(const float* x, const float* w, const float* b, float* y, int P, int H, int W,
                     int C, int relu, float* partial, int G, hipStream_t s);
int k_conv_first_wgrad(const float* x, const float* dout, const float* y, const float* coef, int P,
                       int H, int W, int C, int mask, float* partial, int G, float* gw, float* gb,
                       hipStream_t s);
int k_reduce_rows(const float* in, int R, int ncols, float* out, int G, hipStream_t s);
int k_bn_finalize_train(const float* part, int G, int C, double count, const float* gamma,
                        const float* beta, float* rmean, float* rvar, int64_t* nbt, float momentum,
                        float eps, float* scale, float* shift, float* mean, float* invstd,
                        hipStream_t s);
int k_bn_finalize_eval(int C, const float* gamma, const float* beta, const float* rmean,
                       const float* rvar, float eps, float* scale, float* shift, hipStream_t s);
// relu / mscale+mshift: BN -> ReLU order (mod.py:46-47), see the kernels.
// (r06) pool16: the pooled values as the next conv's bf16 image [pooled pixels][C]; skip16 / skip3:
// op(BN(y)) at full resolution as bf16 / x3 into the decoder conv's kept image (ldk channels per
// pixel, channel offset so) -- what k_to_bf16 / k_to_x3 would write there
int k_maxpool_bn(const float* y, int ld, int off, const float* scale, const float* shift, int relu,
                 int N, int H, int W, int C, float* out, uint8_t* idx, hipStream_t s,
                 uint16_t* out3 = nullptr, uint16_t* pool16 = nullptr, uint16_t* skip16 = nullptr,
                 uint16_t* skip3 = nullptr, int ldk = 0, int so = 0);
int k_maxpool_bwd(const float* dp, const uint8_t* idx, const float* dskip, int ldskip, int offskip,
                  const float* y, int ldy, int offy, const float* mscale, const float* mshift,
                  int N, int H, int W, int C, float* dout, float* partial, int G, hipStream_t s);
int k_bn_bwd_finalize2(const float* part, int G, int C, double count, const float* gamma,
                       const float* mean, const float* invstd, float* coef, float* dgamma,
                       float* dbeta, hipStream_t s);
int k_bn_dz(float* d, const float* y, int ld, int off, int64_t P, int C, const float* coef, int mask,
            hipStream_t s);
// bf16 image [P][dld] (dld 0 = C: dense) of op(src), channels [0, C), for the LDS-DMA GEMMs
// (affine if scale, ReLU on c < relu)
int k_to_bf16(const float* src, int ld, int off, int C, const float* scale, const float* shift,
              int relu, int64_t P, uint16_t* dst, hipStream_t s, int dld = 0);
// bn_dz writing the dense bf16 image of dz (and the f32 dz in place when f32 != 0)
// (r06) hdl != null (option head_fuse, one output channel): do = [hrelu: fma(y, hsc, hsh) > 0]
// hdl[m] hw[c] recomputed from the head (d unused, f32 must be 0)
int k_bn_dz16(float* d, const float* y, int ld, int off, int64_t P, int C, const float* coef,
              int mask, uint16_t* dz16, int f32, hipStream_t s, const float* hdl = nullptr,
              const float* hw = nullptr, const float* hsc = nullptr, const float* hsh = nullptr,
              int hrelu = 0);
// (r06) the same with `do` recomputed from the max-pool backward's inputs (option pool_fuse):
// do = [msc: fma(msc, y, msh) > 0] (dskip + [idx == window position] dp); no f32 dz
int k_bn_dz16_pool(const float* y, int ld, int off, int64_t P, int C, const float* coef, int mask,
                   uint16_t* dz16, const float* dp, const uint8_t* idx, const float* dskip, int ldskip,
                   const float* msc, const float* msh, int N, int H, int W, hipStream_t s);
int k_bias_reduce(const float* slab, int S, int taps, int C, float* out, hipStream_t s);
// ConvT bias partials [splits][4][C] from the up half of the concat gradient (LDS-DMA wgrad)
int k_up2_bias_partials(const float* d, int ld, int off, int H, int W, int64_t P, int C, int pps,
                        int splits, float* bslab, hipStream_t s);
int k_sum_partials(const float* part, int G, int ncols, float* out, hipStream_t s);
int k_slab_reduce(const float* slab, int S, int Mw, int Nw, int kind, int cin, int cout,
                  float* grad, hipStream_t s);
int k_head_fwd(const float* y, int C, const float* scale, const float* shift, int relu,
               const float* w, const float* b, int O, int P, int HW, float* logits, hipStream_t s);
int k_head_bwd(const float* y, int C, const float* scale, const float* shift, int relu,
               const float* w, int O, int P, int HW, const float* dlog, float* dout, float* partial,
               float* bnpart, int G, hipStream_t s);
int k_pack_1x1_t(const float* w, float* wt, int cin, int cout, hipStream_t s);
// Residual blocks (models/mod.py:ResUNet): first-block forward with the Cin = 1 skip,
// backward entry (ReLU mask + BN2 partials), first-block skip weight gradient.
int k_res_first_fwd(const float* x, const float* ws, const float* z, const float* sc,
                    const float* sh, int64_t P, int C, float* out, int ldo, int offo, hipStream_t s);
int k_res_bwd_prep(float* d, const float* out, int ldo, int offo, const float* z, int64_t P, int C,
                   float* partial, int G, hipStream_t s);
int k_res_first_wgrad(const float* x, const float* du, int P, int C, float* partial, int G,
                      float* gw, hipStream_t s);
// Pillow-exact 8-bit bilinear resize + scale (input pipeline, utils/transforms.py:143-156)
int k_resize_u8(const uint8_t* src, int H, int W, float* dst, int OH, int OW, const int* kh,
                const int* bh, int ksh, const int* kv, const int* bv, int ksv, int need_h,
                int need_v, float divisor, hipStream_t s);
// Channel padding (runtime.hip, unet_ctx::padded): one tensor of the caller's torch-layout
// arena (roff) and of the padded arena (poff).  Dim k holds nseg[k] segments of seg[k] real
// entries, each padded to pseg[k] entries (unused dims: 1, 1, 1).
struct PadDesc {
    int64_t roff, poff, rnumel, pnumel;
    int32_t seg[4], pseg[4], nseg[4];
};
// expand = 1: dst (padded) <- src (torch layout), zeros in the padding;
// expand = 0: dst (torch layout) <- src (padded).  table: device copy of n descriptors.
int k_pad_copy(const PadDesc* table, int n, int64_t max_numel, const float* src, float* dst,
               int expand, hipStream_t s);
// Losses: per-sample stats fp32[4N] + batch sums fp64[8] (see kernels_misc.hip)
// (r06) chunks per sample of loss_stats_kernel; part holds 4 * N * loss_groups(per) floats
int loss_groups(int64_t per);
int k_loss_stats(const float* x, const float* t, int N, int64_t per, float* stats, double* sums,
                 float* part, hipStream_t s);
int k_loss_finalize(const double* sums, float alpha, float beta, float gamma, float* losses,
                    hipStream_t s);
int k_loss_bwd(const float* x, const float* t, int N, int64_t per, const float* stats,
               const double* sums, const float* w, float alpha, float beta, float gamma, float* dx,
               hipStream_t s);
// AdamW scalars, each formed in double and rounded to float once (torch Scalar -> float)
struct AdamwScalars {
    float decay;     // 1 - lr * weight_decay
    float w1;        // 1 - beta1 (lerp weight)
    float b2;        // beta2
    float w2;        // 1 - beta2
    float neg_step;  // -lr / (1 - beta1^step)
    float bc2_sqrt;  // (1 - beta2^step) ** 0.5
    float eps;
    float gscale;    // gradient pre-scale (1 = none)
    int lerp_small;  // |w1| < 0.5 (ATen lerp branch)
};
int k_adamw(float* p, const float* g, float* m, float* v, int64_t n, const AdamwScalars& a,
            hipStream_t s);
int k_mask_counts(const float* x, const float* t, int64_t n, uint8_t* mask, int64_t* counts,
                  hipStream_t s);
int k_nchw_to_nhwc(const float* x, int N, int C, int HW, float* y, hipStream_t s);
int k_fill(float* p, int64_t n, float v, hipStream_t s);
