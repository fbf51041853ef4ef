"""Python handle on a native UNet context (libunet_hip.so).

One ``UNetRuntime`` per (device, network configuration).  It exposes the native
parameter / BN-buffer tables (so the ``nn.Module`` can lay its tensors out in the flat
arenas the kernels read) and thin, shape-checked wrappers of the C entry points that
take torch tensors and enqueue on torch's current stream.
"""
import ctypes

import torch

from . import _lib

_RUNTIMES = {}


class UNetRuntime:
    def __init__(self, device, in_channels=1, out_channels=1, variant=_lib.VARIANT_MODEL,
                 base_filters=0, depth=0, math=_lib.MATH_F32):
        lib = _lib.load()
        self.lib = lib
        self.device = torch.device(device)
        cfg = _lib.UnetCfg(in_channels, out_channels, variant, base_filters, depth, math)
        h = ctypes.c_void_p()
        _lib.check(lib.unet_create(ctypes.byref(cfg), self.device.index or 0, ctypes.byref(h)),
                   None, "unet_create")
        self.ctx = h
        n, nf = ctypes.c_int(), ctypes.c_int64()
        lib.unet_num_params(h, ctypes.byref(n), ctypes.byref(nf))
        self.n_param_floats = nf.value
        self.params = []  # (name, shape, offset)
        for i in range(n.value):
            name, nd, off = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_int64()
            shape = (ctypes.c_int64 * 4)()
            lib.unet_param_info(h, i, ctypes.byref(name), ctypes.byref(nd), shape, ctypes.byref(off))
            self.params.append((name.value.decode(), tuple(shape[k] for k in range(nd.value)),
                                off.value))
        lib.unet_num_bn(h, ctypes.byref(n), ctypes.byref(nf))
        self.n_bn_floats = nf.value
        self.bn = []  # (name, channels, offset)
        for i in range(n.value):
            name, ch, off = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_int64()
            lib.unet_bn_info(h, i, ctypes.byref(name), ctypes.byref(ch), ctypes.byref(off))
            self.bn.append((name.value.decode(), ch.value, off.value))
        nb = ctypes.c_int()
        lib.unet_num_buckets(h, ctypes.byref(nb))
        self.buckets = []
        for b in range(nb.value):
            o, l = ctypes.c_int64(), ctypes.c_int64()
            lib.unet_bucket_range(h, b, ctypes.byref(o), ctypes.byref(l))
            self.buckets.append((o.value, l.value))
        # the context's schedule options as created (reset_options restores them)
        self._default_options = {k: self.get_option(k) for k in _lib.option_names()}

    def __del__(self):
        try:
            if getattr(self, "ctx", None):
                self.lib.unet_destroy(self.ctx)
        except Exception:
            pass

    @staticmethod
    def get(device, in_channels=1, out_channels=1, variant=_lib.VARIANT_MODEL, base_filters=0,
            depth=0, math=_lib.MATH_F32):
        key = (str(torch.device(device)), in_channels, out_channels, variant, base_filters, depth,
               math)
        rt = _RUNTIMES.get(key)
        if rt is None:
            rt = UNetRuntime(device, in_channels, out_channels, variant, base_filters, depth, math)
            _RUNTIMES[key] = rt
        return rt

    # ------------------------------------------------------------------ entry points
    def workspace_bytes(self, N, H, W, training):
        b = ctypes.c_size_t()
        _lib.check(self.lib.unet_workspace_size(self.ctx, N, H, W, int(training), ctypes.byref(b)),
                   self.ctx, "unet_workspace_size")
        return b.value

    def forward(self, params, bn_running, bn_count, x, training, workspace=None):
        N, _, H, W = x.shape
        nb = self.workspace_bytes(N, H, W, training)
        if workspace is None or workspace.numel() < nb:
            workspace = torch.empty(nb, dtype=torch.uint8, device=x.device)
        logits = torch.empty((N, self.out_channels(), H, W), dtype=torch.float32, device=x.device)
        rc = self.lib.unet_forward(self.ctx, _lib.ptr(params), _lib.ptr(bn_running), _lib.ptr(bn_count),
                                   _lib.ptr(x), _lib.ptr(logits), _lib.ptr(workspace),
                                   workspace.numel(), N, H, W, int(training), _lib.stream_ptr(x.device))
        _lib.check(rc, self.ctx, "unet_forward")
        return logits, workspace

    def backward(self, params, dlogits, grads, workspace):
        N, _, H, W = dlogits.shape
        rc = self.lib.unet_backward(self.ctx, _lib.ptr(params), _lib.ptr(dlogits), _lib.ptr(grads),
                                    _lib.ptr(workspace), workspace.numel(), N, H, W,
                                    _lib.stream_ptr(dlogits.device))
        _lib.check(rc, self.ctx, "unet_backward")

    def out_channels(self):
        return self.params[-1][1][0]

    def loss_stats(self, logits, targets):
        """Per-sample partials fp32[4N] and the batch sums fp64[8] (unet_loss_stats)."""
        N, C, H, W = logits.shape
        stats = torch.empty(4 * N, dtype=torch.float32, device=logits.device)
        sums = torch.empty(8, dtype=torch.float64, device=logits.device)
        rc = self.lib.unet_loss_stats(self.ctx, _lib.ptr(logits), _lib.ptr(targets), N, C, H, W,
                                      _lib.ptr(stats), _lib.ptr(sums), _lib.stream_ptr(logits.device))
        _lib.check(rc, self.ctx, "unet_loss_stats")
        return stats, sums

    def loss_finalize(self, sums, alpha=0.4, beta=0.6, gamma=2.0):
        losses = torch.empty(3, dtype=torch.float32, device=sums.device)
        rc = self.lib.unet_loss_finalize(self.ctx, _lib.ptr(sums), _lib.ptr(losses), alpha, beta,
                                         gamma, _lib.stream_ptr(sums.device))
        _lib.check(rc, self.ctx, "unet_loss_finalize")
        return losses

    def loss_fwd(self, logits, targets, alpha=0.4, beta=0.6, gamma=2.0):
        stats, sums = self.loss_stats(logits, targets)
        return self.loss_finalize(sums, alpha, beta, gamma), stats, sums

    def loss_bwd(self, logits, targets, stats, sums, w, alpha=0.4, beta=0.6, gamma=2.0):
        N, C, H, W = logits.shape
        d = torch.empty_like(logits)
        rc = self.lib.unet_loss_bwd(self.ctx, _lib.ptr(logits), _lib.ptr(targets), N, C, H, W,
                                    _lib.ptr(stats), _lib.ptr(sums), _lib.ptr(w), _lib.ptr(d), alpha,
                                    beta, gamma, _lib.stream_ptr(logits.device))
        _lib.check(rc, self.ctx, "unet_loss_bwd")
        return d

    def adamw(self, params, grads, m, v, step, lr, beta1, beta2, eps, wd, grad_scale=1.0):
        rc = self.lib.unet_adamw(self.ctx, _lib.ptr(params), _lib.ptr(grads), _lib.ptr(m), _lib.ptr(v),
                                 params.numel(), step, float(lr), float(beta1), float(beta2),
                                 float(eps), float(wd), float(grad_scale),
                                 _lib.stream_ptr(params.device))
        _lib.check(rc, self.ctx, "unet_adamw")

    def adamw_repack(self, params, grads, m, v, step, lr, beta1, beta2, eps, wd, grad_scale=1.0):
        """AdamW over this context's whole parameter arena fused with the next forward's weight
        repack (unet_adamw_repack; bit-identical to adamw)."""
        rc = self.lib.unet_adamw_repack(self.ctx, _lib.ptr(params), _lib.ptr(grads), _lib.ptr(m),
                                        _lib.ptr(v), params.numel(), step, float(lr), float(beta1),
                                        float(beta2), float(eps), float(wd), float(grad_scale),
                                        _lib.stream_ptr(params.device))
        _lib.check(rc, self.ctx, "unet_adamw_repack")

    def params_changed(self):
        """The parameter arena changed outside adamw_repack: the next forward repacks."""
        _lib.check(self.lib.unet_params_changed(self.ctx), self.ctx, "unet_params_changed")

    # ------------------------------------------------------------------ schedule options
    def set_option(self, name, value):
        """Kernel-schedule option (include/unet_hip.h unet_set_option); A/B runs and tests."""
        _lib.check(self.lib.unet_set_option(self.ctx, name.encode(), int(value)), self.ctx,
                   f"unet_set_option({name})")

    def reset_options(self):
        """Every schedule option back to its value at creation (this runtime is shared by
        every model of its configuration on the device)."""
        for k, v in self._default_options.items():
            if self.get_option(k) != v:
                self.set_option(k, v)

    def get_option(self, name):
        v = ctypes.c_int64()
        _lib.check(self.lib.unet_get_option(self.ctx, name.encode(), ctypes.byref(v)), self.ctx,
                   f"unet_get_option({name})")
        return v.value

    def mask_counts(self, logits, targets, counts, mask=None):
        rc = self.lib.unet_mask_counts(self.ctx, _lib.ptr(logits), _lib.ptr(targets), logits.numel(),
                                       _lib.ptr(mask), _lib.ptr(counts), _lib.stream_ptr(logits.device))
        _lib.check(rc, self.ctx, "unet_mask_counts")

    def stream_wait_bucket(self, b, stream):
        rc = self.lib.unet_stream_wait_bucket(self.ctx, b, ctypes.c_void_p(stream.cuda_stream))
        _lib.check(rc, self.ctx, "unet_stream_wait_bucket")

    def bucket_event(self, b):
        """The hipEvent_t (as an int handle) the last backward recorded for bucket b -- what a
        caller driving RCCL without torch streams waits on (hipStreamWaitEvent)."""
        e = ctypes.c_void_p()
        _lib.check(self.lib.unet_bucket_event(self.ctx, b, ctypes.byref(e)), self.ctx,
                   "unet_bucket_event")
        return e.value

    # ------------------------------------------------------------------ timing
    def timing(self, enable, only=None):
        """Per-launch HIP-event timing; `only`: time just the labels containing it."""
        self.lib.unet_timing_enable(self.ctx, int(enable))
        self.lib.unet_timing_filter(self.ctx, only.encode() if only else None)
        self.lib.unet_timing_reset(self.ctx)

    def timing_records(self):
        n = ctypes.c_int()
        self.lib.unet_timing_count(self.ctx, ctypes.byref(n))
        out = []
        for i in range(n.value):
            fam, cnt, ms, fl = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
            _lib.check(self.lib.unet_timing_read(self.ctx, i, ctypes.byref(fam), ctypes.byref(cnt),
                                                 ctypes.byref(ms), ctypes.byref(fl)), self.ctx, "timing")
            out.append((fam.value.decode(), ms.value, fl.value))
        self.lib.unet_timing_reset(self.ctx)
        return out

    # ------------------------------------------------------------------ debug views
    def debug_view(self, workspace, N, H, W, training, kind, index):
        """A tensor view (NHWC pixels x channels, or a vector) of an intermediate buffer."""
        bo, cnt, ld, off = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.unet_debug_view(self.ctx, N, H, W, int(training), kind, index,
                                            ctypes.byref(bo), ctypes.byref(cnt), ctypes.byref(ld),
                                            ctypes.byref(off)), self.ctx, "unet_debug_view")
        if kind == 8:  # uint8 max-pool winner index
            return workspace[bo.value:bo.value + cnt.value].view(-1, ld.value), off.value
        flat = workspace[bo.value:bo.value + 4 * cnt.value].view(torch.float32)
        if kind in (1, 2, 3, 4):
            return flat
        return flat.view(-1, ld.value), off.value
