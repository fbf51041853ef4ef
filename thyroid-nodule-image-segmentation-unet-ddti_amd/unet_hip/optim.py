"""``HipAdamW``: torch.optim.AdamW semantics (utils/trainer.py:41,92) as one native launch.

Same hyper-parameters and defaults as ``torch.optim.AdamW`` (lr, betas=(0.9, 0.999),
eps=1e-8, weight_decay=1e-2) and the same update as torch's ``_single_tensor_adam`` with
decoupled weight decay.  When every parameter is a view into one flat arena (the HIP
``UNet`` after its first forward) and every grad is a view into one flat grad arena
laid out the same way, the whole step is ONE kernel over 31M floats; otherwise it runs
one native launch per parameter tensor.  ``grad_scale`` (e.g. 1/world_size after an
RCCL sum) is folded into the same pass.

``self.state[p]["exp_avg"] / ["exp_avg_sq"]`` stay the source of truth, as in any
``torch.optim.Optimizer``: on the flat path they are views of the two moment arenas, and
when they are not (``load_state_dict`` replaced them, or a parameter had no state yet) the
arenas are rebuilt from them before the step, so a resumed optimizer continues from the
loaded moments.
"""
import torch

from ._lib import HipUnavailable
from .runtime import UNetRuntime


def _flat_base(tensors):
    """(base tensor, [offsets]) if all tensors are contiguous views of one storage laid out
    back to back in order, else None."""
    if not tensors:
        return None
    t0 = tensors[0]
    base_ptr = t0.data_ptr()
    off = 0
    offs = []
    for t in tensors:
        if not t.is_contiguous() or t.data_ptr() != base_ptr + 4 * off:
            return None
        offs.append(off)
        off += t.numel()
    base = t0.untyped_storage()
    flat = torch.empty(0, dtype=torch.float32, device=t0.device).set_(
        base, t0.storage_offset(), (off,), (1,))
    return flat


class HipAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.grad_scale = 1.0
        self._flat = {}

    def _views_of(self, params, m, v):
        """True if every param's exp_avg / exp_avg_sq is the slice of arenas m / v."""
        off = 0
        for p in params:
            s = self.state.get(p, {})
            ea, eq = s.get("exp_avg"), s.get("exp_avg_sq")
            if ea is None or eq is None or ea.data_ptr() != m.data_ptr() + 4 * off \
                    or eq.data_ptr() != v.data_ptr() + 4 * off:
                return False
            off += p.numel()
        return True

    def _rebuild_flat(self, params, fp):
        """Fresh moment arenas holding each param's current state (zeros where none), with
        the state re-pointed at their slices."""
        m = torch.zeros_like(fp)
        v = torch.zeros_like(fp)
        off = 0
        for p in params:
            s = self.state[p]
            n = p.numel()
            for k, arena in (("exp_avg", m), ("exp_avg_sq", v)):
                view = arena[off:off + n].view_as(p)
                if k in s:
                    view.copy_(s[k].reshape(p.shape))
                s[k] = view
            off += n
        return m, v

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            if params[0].device.type != "cuda":
                raise HipUnavailable("HipAdamW runs on the HIP path only")
            rt = UNetRuntime.get(params[0].device)
            b1, b2 = group["betas"]
            lr, eps, wd = group["lr"], group["eps"], group["weight_decay"]
            # per-group step counter kept in every param state (torch keeps it per param)
            st0 = self.state[params[0]]
            step = int(st0.get("step", torch.tensor(0.0)).item()) + 1
            fp = _flat_base(params)
            fg = _flat_base([p.grad for p in params]) if fp is not None else None
            if fp is not None and fg is not None:
                key = (gi, fp.data_ptr(), fp.numel())
                m, v = self._flat.get(key, (None, None))
                if m is None or not self._views_of(params, m, v):
                    m, v = self._rebuild_flat(params, fp)
                    self._flat = {key: (m, v)}
                # (r06) the whole arena of a HIP model: AdamW fused with its next forward's
                # weight repack (unet_adamw_repack, bit-identical to unet_adamw)
                from .module import arena_owner
                st = arena_owner(fp)
                if st is not None and fg.numel() == fp.numel():
                    st.rt.adamw_repack(fp, fg, m, v, step, lr, b1, b2, eps, wd, self.grad_scale)
                    st.native_version = st.version()  # the images match the parameters
                else:
                    rt.adamw(fp, fg, m, v, step, lr, b1, b2, eps, wd, self.grad_scale)
            else:
                for p in params:
                    s = self.state[p]
                    if "exp_avg" not in s:
                        s["exp_avg"] = torch.zeros_like(p)
                        s["exp_avg_sq"] = torch.zeros_like(p)
                    g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                    rt.adamw(p, g, s["exp_avg"], s["exp_avg_sq"], step, lr, b1, b2, eps, wd,
                             self.grad_scale)
            for p in params:
                self.state[p]["step"] = torch.tensor(float(step))
        return loss
