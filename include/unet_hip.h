/*
 * unet_hip.h - C ABI of libunet_hip.so, the MI355X-native (gfx950) UNet training /
 * inference path for the DDTI thyroid-nodule workload.
 *
 * The reference (WuJiaqiii/Thyroid-nodule-image-segmentation-UNet-DDTI) is pure Python;
 * its hot path is PyTorch autograd over models/model.py:UNet plus the losses and the
 * optimizer step driven by utils/trainer.py.  Each entry point below replaces one
 * call site of that path (file:line in the reference):
 *
 *   unet_create / unet_destroy      models/model.py:6-31   UNet.__init__ (topology only;
 *                                                           parameters stay torch-owned)
 *   unet_param_info / unet_bn_info  models/model.py:6-31   named_parameters()/named_buffers()
 *                                                           order, shapes and flat offsets
 *   unet_workspace_size             (new)                  device scratch the caller allocates
 *   unet_forward                    models/model.py:53-73  UNet.forward (train: batch-stat BN
 *                                                           + running-stat update; eval:
 *                                                           running-stat BN), called from
 *                                                           utils/trainer.py:84,139,216
 *   unet_backward                   utils/trainer.py:91    loss.backward() through the UNet
 *   unet_loss_stats / _finalize /   utils/trainer.py:85-87 BCEWithLogitsLoss, models/loss.py:13-24
 *   unet_loss_fwd                                           DiceLoss, models/loss.py:34-46
 *                                                           FocalTverskyLoss (two phases so DP
 *                                                           can all-reduce the batch sums)
 *   unet_loss_bwd                   utils/trainer.py:90-91 d(weighted loss)/d(logits)
 *   unet_adamw                      utils/trainer.py:41,92 AdamW.step (torch optim/adam.py
 *                                                           _single_tensor_adam, decoupled wd)
 *   unet_mask_counts                utils/trainer.py:217,236-242  sigmoid(x)>0.5 masks and
 *                                                           TP/FP/FN/TN counts
 *   unet_resize_plan / unet_resize_u8  utils/transforms.py:143-156 Resize + ToTensor of the
 *                                   data loader (data/data_loader.py:20-27), on the device
 *   unet_bucket_* / unet_stream_wait_bucket   utils/trainer.py:28-30 nn.DataParallel grad
 *                                   reduction -> per-bucket readiness for an RCCL all-reduce
 *                                   overlapped with the rest of the backward pass
 *
 * Conventions: every function returns 0 (UNET_OK) or a negative unet_status and never
 * throws across the ABI; unet_last_error() returns the text of the last failure on that
 * context.  All pointers are device pointers owned by the caller (PyTorch) unless noted;
 * the library only borrows them for the duration of the call.  Work is enqueued on the
 * caller's stream with no host synchronisation.  A context is not re-entrant.
 *
 * Tensor layouts at the boundary are the reference's: x (N, Cin, H, W), logits
 * (N, Cout, H, W), parameters in torch layout (Conv2d [Cout,Cin,kh,kw],
 * ConvTranspose2d [Cin,Cout,2,2]) packed back to back in named_parameters() order in one
 * flat fp32 arena (offsets from unet_param_info).  BN buffers: running_mean and
 * running_var in one fp32 arena (layer i: mean at bn_off[i], var at bn_off[i]+C_i) and
 * num_batches_tracked in an int64 array, one per BN layer.
 */
#ifndef UNET_HIP_H
#define UNET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct unet_ctx unet_ctx;
typedef void* unet_stream_t; /* hipStream_t (0 = legacy default stream) */

typedef enum {
    UNET_OK = 0,
    UNET_ERR_INVALID = -1,     /* null pointer / bad argument */
    UNET_ERR_SHAPE = -2,       /* H or W not divisible by 16, N < 1, ... */
    UNET_ERR_HIP = -3,         /* a HIP runtime call failed */
    UNET_ERR_WORKSPACE = -4,   /* workspace too small */
    UNET_ERR_UNSUPPORTED = -5, /* configuration not implemented */
    UNET_ERR_NOMEM = -6,       /* host allocation failed */
    UNET_ERR_INTERNAL = -7     /* unexpected internal failure (caught C++ exception) */
} unet_status;

/* Which reference network the context runs. */
typedef enum {
    UNET_VARIANT_MODEL = 0, /* models/model.py:UNet -- Conv(+bias) -> ReLU -> BN blocks,
                               concat [up, skip], depth 4, base 64 (fixed) */
    UNET_VARIANT_MOD = 1,   /* models/mod.py:9-66 UNet -- Conv(no bias) -> BN -> ReLU blocks,
                               concat [skip, up], base_filters / depth configurable */
    UNET_VARIANT_RES = 2    /* models/mod.py:71-131 ResUNet -- residual blocks
                               ReLU(Conv-BN-ReLU-Conv-BN(x) + Conv1x1(x)), otherwise as MOD
                               (the network main.py:122 builds) */
} unet_variant;

/* Arithmetic of the convolution GEMMs. */
typedef enum {
    UNET_MATH_F32 = 0,  /* f32 products (the reference's fp32): by default (option x3) the GEMMs
                           with 64-multiple channel counts run on v_mfma_f32_32x32x16_bf16 through
                           exact three-way bf16 splits of the f32 operands (six piece products,
                           split f32 accumulators: below the f32 MFMA's error against fp64), the
                           rest on v_mfma_f32_32x32x2_f32 */
    UNET_MATH_BF16 = 1  /* v_mfma_f32_32x32x16_bf16: operands rounded to bf16, f32 accumulate
                           (BASELINE config 4; models/mod.py variant only) */
} unet_math;

typedef struct {
    int in_channels;   /* models/model.py:6 / mod.py:11 in_channels (default 1; must be 1) */
    int out_channels;  /* models/model.py:6 / mod.py:12 out_channels (default 1; 1..4)   */
    int variant;       /* unet_variant (0 = models/model.py)                               */
    int base_filters;  /* mod.py:13 (0 = default 64); a multiple of 8, <= 256.  Channels are
                          padded per level inside the library (the caller's arenas keep the
                          torch layouts): level 0 runs the next power of two >= 32 of
                          base_filters, every deeper level the next multiple of 32 of
                          base_filters << level (base 16: 32, 32, 64, 128, 256 -- only level 0
                          padded; 24: 32, 64, 96, 192, ...; 48: 64, 96, 192, ...) */
    int depth;         /* mod.py:14 (0 = default 5 for mod, 4 for model); 1..6             */
    int math;          /* unet_math of the conv GEMMs (0 = f32)                            */
} unet_cfg;

/* models/model.py:6-31 / models/mod.py:10-41.  device = HIP ordinal the context will
 * launch on.  Zero-initialised fields take the reference defaults. */
int unet_create(const unet_cfg* cfg, int device, unet_ctx** out);
int unet_destroy(unet_ctx* ctx);
const char* unet_last_error(const unet_ctx* ctx);

/* Parameter table in named_parameters() order.  n_floats = size of the flat arena. */
int unet_num_params(const unet_ctx* ctx, int* n_tensors, int64_t* n_floats);
/* name: static string owned by the library; shape: up to 4 dims. */
int unet_param_info(const unet_ctx* ctx, int i, const char** name, int* ndim, int64_t shape[4],
                    int64_t* offset);
/* BN layer table: n_layers, total floats of the running-stat arena (mean|var per layer). */
int unet_num_bn(const unet_ctx* ctx, int* n_layers, int64_t* n_floats);
int unet_bn_info(const unet_ctx* ctx, int i, const char** name, int* channels, int64_t* offset);

/* Bytes of device workspace for one forward (+backward when training) at (N, H, W).
 * H and W must be multiples of max(16, 2**depth). */
int unet_workspace_size(unet_ctx* ctx, int N, int H, int W, int training, size_t* bytes);

/* Forward.  params: flat arena; bn_running: running-stat arena (updated when training);
 * bn_count: int64[n_bn] num_batches_tracked (incremented when training); x: (N,Cin,H,W);
 * logits: (N,Cout,H,W).  The workspace keeps what backward needs; pass the same one. */
int unet_forward(unet_ctx* ctx, const float* params, float* bn_running, int64_t* bn_count,
                 const float* x, float* logits, void* workspace, size_t ws_bytes, int N, int H,
                 int W, int training, unet_stream_t stream);

/* Backward of the last training forward run with this workspace.  dlogits: (N,Cout,H,W).
 * grads: flat arena laid out like params; every entry is overwritten (zero_grad -> None
 * semantics, utils/trainer.py:81). */
int unet_backward(unet_ctx* ctx, const float* params, const float* dlogits, float* grads,
                  void* workspace, size_t ws_bytes, int N, int H, int W, unet_stream_t stream);

/* Losses over logits/targets (N, C, H, W) (targets may be soft, e.g. mixup), in two
 * phases so that data parallelism can insert one collective between them:
 *   unet_loss_stats     per-sample partials stats (device fp32[4*N]) and the batch sums
 *                       sums (device fp64[8]) = {sum bce_elem, sum_n dice_n, TP, sum p,
 *                       sum t, samples, elements, 0}
 *   [DP: all-reduce(SUM) sums across ranks -- the loss of the gathered batch, exactly
 *        what nn.DataParallel evaluates (utils/trainer.py:28-30,85-90); FocalTversky's
 *        TP/FP/FN are batch-global (models/loss.py:41-45)]
 *   unet_loss_finalize  losses (device fp32[3]) <- {bce_mean, dice_loss, focal_tversky}
 * unet_loss_fwd = unet_loss_stats + unet_loss_finalize (single process).
 * focal uses (alpha, beta, gamma) of utils/trainer.py:38 / models/loss.py:27 defaults.
 * (r06) unet_loss_stats sums each sample in chunks into a context-owned scratch (grown on
 * demand, synchronising the device when it grows): one loss pass per context in flight at a
 * time, i.e. issue a context's loss calls on one stream. */
int unet_loss_stats(unet_ctx* ctx, const float* logits, const float* targets, int N, int C, int H,
                    int W, float* stats, double* sums, unet_stream_t stream);
int unet_loss_finalize(unet_ctx* ctx, const double* sums, float* losses, float focal_alpha,
                       float focal_beta, float focal_gamma, unet_stream_t stream);
int unet_loss_fwd(unet_ctx* ctx, const float* logits, const float* targets, int N, int C, int H,
                  int W, float* stats, double* sums, float* losses, float focal_alpha,
                  float focal_beta, float focal_gamma, unet_stream_t stream);
/* dlogits = w[0]*dBCE + w[1]*dDice + w[2]*dFocal of the batch described by `sums`
 * (w a device fp32[3]).  With all-reduced sums each rank writes its slice of the
 * gathered batch's dlogits, so the ranks' gradients SUM to the reference's. */
int unet_loss_bwd(unet_ctx* ctx, const float* logits, const float* targets, int N, int C, int H,
                  int W, const float* stats, const double* sums, const float* w, float* dlogits,
                  float focal_alpha, float focal_beta, float focal_gamma, unet_stream_t stream);

/* AdamW over flat arenas of n floats (one launch for all parameter tensors).
 * Hyper-parameters are the optimizer's Python floats (double); the library forms
 * 1 - lr*wd, 1 - beta1, 1 - beta2, -lr/(1 - beta1^step) and (1 - beta2^step)**0.5 in
 * double and rounds each to float once, as torch does (optim/adam.py _single_tensor_adam).
 * grads are multiplied by grad_scale first when it is not 1. */
int unet_adamw(unet_ctx* ctx, float* params, const float* grads, float* exp_avg,
               float* exp_avg_sq, int64_t n, int step, double lr, double beta1, double beta2,
               double eps, double weight_decay, double grad_scale, unet_stream_t stream);

/* (r06) The same AdamW step (utils/trainer.py:41,92 AdamW(...).step()) over the whole parameter
 * arena of this context (n == the unet_num_params float count), fused with the weight repack
 * the next forward needs: every 3x3 conv / ConvT weight tile is updated and packed into the
 * context's own GEMM images in one pass, the other tensors are updated elementwise.  Results
 * are bit-identical to unet_adamw.  The next unet_forward on the same `params` pointer reads
 * those images instead of repacking, until unet_params_changed (the caller changed the
 * parameters by other means: load_state_dict, another optimizer) or the next repack.  A
 * training forward that read them refuses its backward (UNET_ERR_INVALID) if they were rewritten
 * in between.  Another n, or a channel-padded network, runs the plain unet_adamw. */
int unet_adamw_repack(unet_ctx* ctx, float* params, const float* grads, float* exp_avg,
                      float* exp_avg_sq, int64_t n, int step, double lr, double beta1, double beta2,
                      double eps, double weight_decay, double grad_scale, unet_stream_t stream);
/* The caller changed the parameter arena outside unet_adamw_repack: the next forward repacks. */
int unet_params_changed(unet_ctx* ctx);

/* Mask readout + confusion counts, utils/trainer.py:101-107,217-242, utils/utils.py:225-251.
 * counts (device int64[6]) += {TP, FP, FN, TN} of (sigmoid(logits) > 0.5) vs targets cast to
 * an integer (== 1 is positive), then {|pred AND t!=0|, |pred OR t!=0|} (the bool cast of
 * calculate_iou).  mask (optional, may be null): uint8 (N,C,H,W). */
int unet_mask_counts(unet_ctx* ctx, const float* logits, const float* targets, int64_t n,
                     uint8_t* mask, int64_t* counts, unet_stream_t stream);

/* Gradient buckets for data-parallel overlap.  Bucket b covers grads[offset, offset+len)
 * and is complete once the event recorded by unet_backward for it has fired; buckets
 * become ready in order 0, 1, ... (decoder first). */
int unet_num_buckets(const unet_ctx* ctx, int* n);
int unet_bucket_range(const unet_ctx* ctx, int b, int64_t* offset, int64_t* len);
/* Make `stream` wait (device-side) until bucket b of the last backward is complete. */
int unet_stream_wait_bucket(unet_ctx* ctx, int b, unet_stream_t stream);
/* The hipEvent_t (returned as void*) that each unet_backward records on its stream when
 * bucket b is complete -- for a caller that drives RCCL (ncclAllReduce on its own
 * hipStream_t) without torch: hipStreamWaitEvent(comm_stream, ev, 0), then reduce
 * grads[offset, offset+len).  Owned by the context (valid until unet_destroy; created by
 * the first unet_backward, UNET_ERR_INVALID before it). */
int unet_bucket_event(unet_ctx* ctx, int b, void** hip_event);

/* Input pipeline (data/data_loader.py:20-27 + utils/transforms.py:143-156): the reference
 * resizes every PIL image and mask with TF.resize (= Pillow Image.resize(size, BILINEAR))
 * and scales with TF.to_tensor (float(u8) / 255).  unet_resize_plan is a HOST function:
 * Pillow's resampling coefficients (22-bit fixed point) and source bounds for one axis,
 * coeffs[out_size * ksize], bounds[2 * out_size] = {first, count}; pass coeffs = bounds =
 * NULL to get *ksize only.  unet_resize_u8 resizes one (h, w) uint8 image on the device
 * into dst (oh, ow) fp32, divided by `divisor` (255 for ToTensor), bit-identical to
 * Pillow + torch; kh/bh (width: w -> ow) and kv/bv (height: h -> oh) are device copies of the
 * plans (ignored for an axis whose size does not change). */
int unet_resize_plan(int in_size, int out_size, int32_t* coeffs, int32_t* bounds, int* ksize);
int unet_resize_u8(unet_ctx* ctx, const uint8_t* src, int h, int w, float* dst, int oh, int ow,
                   const int32_t* kh, const int32_t* bh, int ksh, const int32_t* kv,
                   const int32_t* bv, int ksv, float divisor, unet_stream_t stream);

/* Kernel-schedule options of a context (new; no reference counterpart).  The defaults are
 * the measured-best schedules; the named alternatives (tiles, LDS-DMA vs register-staged
 * bf16 kernels, XCD block order, ...) exist for A/B runs and the bit-identity tests.  The
 * library never reads the environment: an option changes only when set here.
 * Names (runtime.hip OPTION_TABLE, in this order; unet_option_name enumerates them):
 *   wgrad_row3 wgrad_row3_tile wgrad_row3_big wgrad_row3_blocks wgrad_row3_n32 wgrad_blocks
 *   wgrad16_blocks wgrad_tile_w wgrad_tile_n tile_n128 tile_n128_dgrad tile_n64 tile_n64_dgrad
 *   tile_n32 tile_convt64 tile_convt tile_convt_dgrad rg16 rg16_tile rg16_bn_k rg16_r3 rg16_n128
 *   rg16_n128_bn wg16 wg16_tile wg16_r3 convt16 wg16t xcd16 xcd_remap dz_in_wgrad x3 x3_tile
 *   x3_wtile x3_wblocks x3_n64 x3_r3 head_fuse pool_fuse x3_wwaves x3_wwaves1 tile_group
 * Set them between steps, not between a forward and its backward: the workspace plan and
 * which saved images exist depend on them (x3, convt16, the bf16 kernel choices, ...), so
 * unet_backward returns UNET_ERR_INVALID when any option differs from the last training
 * unet_forward's (or when no training forward ran on this context). */
int unet_set_option(unet_ctx* ctx, const char* name, int64_t value);
int unet_get_option(const unet_ctx* ctx, const char* name, int64_t* value);
/* i-th option name (0 ..), UNET_ERR_INVALID past the last one; *name is static. */
int unet_option_name(int i, const char** name);

/* Per-kernel timing: when enabled, unet_forward/unet_backward bracket every launch with
 * HIP events; unet_timing_read synchronises and returns, per kernel family, the launch
 * count, total ms and algorithmic FLOP of the last call(s) since the last reset. */
int unet_timing_enable(unet_ctx* ctx, int enable);
/* Time only the launches whose label ("family/kernel|layer") contains `substring`
 * (NULL or "" = every launch): keeps the event overhead off the rest of the step. */
int unet_timing_filter(unet_ctx* ctx, const char* substring);
int unet_timing_reset(unet_ctx* ctx);
int unet_timing_count(unet_ctx* ctx, int* n_families);
int unet_timing_read(unet_ctx* ctx, int i, const char** family, int64_t* launches,
                     double* total_ms, double* flop);

/* Debug/test view into a workspace: byte offset of an intermediate tensor.
 * kind: 0 y[i] (post-ReLU conv output, NHWC, channel stride *ld, channel offset *off),
 *       1 BN scale[i], 2 BN shift[i], 3 BN batch mean[i], 4 BN invstd[i],
 *       5 pooled[l] (NHWC dense; not written when the next conv runs on the x3 kernels:
 *       the max-pool then stores that conv's x3 operand image instead), 6 concat buffer[l]
 *       (NHWC, 2*64<<l channels),
 *       7 d(concat)[l] of the last backward, 8 max-pool winner index[l] (uint8 NHWC dense,
 *       window position 0..3 in torch's scan order).  *count = elements (pixels*ld for NHWC). */
int unet_debug_view(unet_ctx* ctx, int N, int H, int W, int training, int kind, int index,
                    int64_t* byte_offset, int64_t* count, int* ld, int* off);

/* Test hooks of the exact three-way bf16 split the x3 GEMMs use (csrc/x3_split.h; no
 * reference counterpart).  n f32 values (n a multiple of 32) become the x3 image the kernels
 * stream, bf16 bit patterns [n / 32][3][32]: for v = v[32 r + j], out[96 r + j] = h,
 * out[96 r + 32 + j] = m, out[96 r + 64 + j] = l, with v = h + m + l exactly for normal and
 * huge finite v; +-inf / NaN keep h = v, m = l = 0.  unet_x3_split_host runs the shared source on the host (bit-level RNE);
 * unet_x3_split_device runs the device pass (to_x3_kernel, hardware bf16 conversion) on n
 * device floats into a device buffer, enqueued on `stream`. */
int unet_x3_split_host(const float* v, int64_t n, uint16_t* out);
int unet_x3_split_device(unet_ctx* ctx, const float* v, int64_t n, uint16_t* out,
                         unet_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* UNET_HIP_H */
