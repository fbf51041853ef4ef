"""autograd bridges from PyTorch to the native kernels.

* ``UNetFunction``  - forward/backward of the whole encoder-decoder
  (models/model.py:53-73 forward, utils/trainer.py:91 backward).  Gradients land in one
  flat arena laid out like the parameter arena; autograd receives views of it.
* ``SegLossFunction`` - the fused BCEWithLogits (mean) + Dice + FocalTversky statistics
  kernel (utils/trainer.py:85-87, models/loss.py:13-46), with an optional all-reduce of
  the 8 batch sums between the statistics and the finalize (data parallelism = the loss of
  the gathered batch, as nn.DataParallel computes it).  It returns the 3-vector
  ``[bce, dice, focal]``; its backward takes the incoming gradient of that vector as the
  per-term weights, so ``bce_ratio*l[0] + dice_ratio*l[1] + ...`` (utils/trainer.py:90)
  differentiates into ONE dlogits kernel with no host synchronisation.
"""
import torch
import torch.distributed as dist

from ._lib import HipUnavailable


class UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, state, *params):
        state.sync_params()
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
    def forward(ctx, logits, targets, rt, alpha, beta, gamma, group):
        logits = logits.contiguous()
        targets = targets.contiguous().float()
        stats, sums = rt.loss_stats(logits, targets)
        if group is not None:
            # nn.DataParallel evaluates the losses on the gathered batch (utils/trainer.py:
            # 28-30,85-90): summing the 8 batch sums over the ranks makes every rank's
            # finalize see exactly that batch (incl. FocalTversky's global TP/FP/FN)
            dist.all_reduce(sums, group=group)
        losses = rt.loss_finalize(sums, alpha, beta, gamma)
        ctx.save_for_backward(logits, targets, stats, sums)
        ctx.rt, ctx.abg = rt, (alpha, beta, gamma)
        return losses

    @staticmethod
    def backward(ctx, g):
        logits, targets, stats, sums = ctx.saved_tensors
        w = g.contiguous().float()
        d = ctx.rt.loss_bwd(logits, targets, stats, sums, w, *ctx.abg)
        return d, None, None, None, None, None, None


def seg_losses(logits, targets, alpha=0.4, beta=0.6, gamma=2.0, group=None):
    """[bce_mean, dice_loss, focal_tversky] of logits vs targets on the HIP path.

    group: a torch.distributed process group whose ranks each hold one shard of the batch.
    The losses (and their gradients) are then those of the GATHERED batch, as with the
    reference's nn.DataParallel: every rank returns the same three values, its dlogits are
    its slice of the gathered batch's dlogits, and the ranks' parameter gradients must be
    SUMMED (``DistributedUNet`` does that).  Unequal shards are handled exactly."""
    if logits.device.type != "cuda":
        raise HipUnavailable("seg_losses runs on the HIP path only (got a CPU tensor)")
    from .runtime import UNetRuntime
    rt = UNetRuntime.get(logits.device)
    if targets.shape != logits.shape:
        raise ValueError(f"targets {tuple(targets.shape)} != logits {tuple(logits.shape)}")
    return SegLossFunction.apply(logits, targets, rt, float(alpha), float(beta), float(gamma),
                                 group)
