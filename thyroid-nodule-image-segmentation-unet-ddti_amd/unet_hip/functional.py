"""autograd bridges from PyTorch to the native kernels.

* ``UNetFunction``  - forward/backward of the whole encoder-decoder
  (models/model.py:53-73 forward, utils/trainer.py:91 backward).  Gradients land in one
  flat arena laid out like the parameter arena; autograd receives views of it.
* ``SegLossFunction`` - the fused BCEWithLogits (mean) + Dice + FocalTversky statistics
  kernel (utils/trainer.py:85-87, models/loss.py:13-46).  It returns the 3-vector
  ``[bce, dice, focal]``; its backward takes the incoming gradient of that vector as the
  per-term weights, so ``bce_ratio*l[0] + dice_ratio*l[1] + ...`` (utils/trainer.py:90)
  differentiates into ONE dlogits kernel with no host synchronisation.
"""
import torch

from ._lib import HipUnavailable


class UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, state, *params):
        logits, ws = state.rt.forward(state.param_arena, state.bn_arena, state.nbt_arena, x,
                                      training=True)
        ctx.state = state
        ctx.ws = ws
        ctx.n_params = len(params)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        st = ctx.state
        grads = st.grad_arena_for_backward()
        st.rt.backward(st.param_arena, dlogits.contiguous(), grads, ctx.ws)
        ctx.ws = None
        return (None, None) + tuple(st.grad_views(grads))


class SegLossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, rt, alpha, beta, gamma):
        logits = logits.contiguous()
        targets = targets.contiguous().float()
        losses, stats = rt.loss_fwd(logits, targets, alpha, beta, gamma)
        ctx.save_for_backward(logits, targets, stats)
        ctx.rt, ctx.abg = rt, (alpha, beta, gamma)
        return losses

    @staticmethod
    def backward(ctx, g):
        logits, targets, stats = ctx.saved_tensors
        w = g.contiguous().float()
        d = ctx.rt.loss_bwd(logits, targets, stats, w, *ctx.abg)
        return d, None, None, None, None, None


def seg_losses(logits, targets, alpha=0.4, beta=0.6, gamma=2.0):
    """[bce_mean, dice_loss, focal_tversky] of logits vs targets on the HIP path."""
    if logits.device.type != "cuda":
        raise HipUnavailable("seg_losses runs on the HIP path only (got a CPU tensor)")
    from .runtime import UNetRuntime
    rt = UNetRuntime.get(logits.device)
    if targets.shape != logits.shape:
        raise ValueError(f"targets {tuple(targets.shape)} != logits {tuple(logits.shape)}")
    return SegLossFunction.apply(logits, targets, rt, float(alpha), float(beta), float(gamma))
