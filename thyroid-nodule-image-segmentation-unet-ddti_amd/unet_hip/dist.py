"""Data-parallel training: one process per GPU, RCCL all-reduce of the flat gradient arena.

Replaces the reference's single-process ``nn.DataParallel`` (utils/trainer.py:28-30), which
re-broadcasts all 124 MB of parameters every forward, gathers the logits on GPU 0, takes the
loss of the gathered batch there and reduce-adds the replicas' gradients.  Here every rank
holds a full replica, parameters are broadcast ONCE from rank 0, each rank runs its shard of
the batch with its own train-mode BatchNorm statistics (exactly DataParallel's per-replica
BN), and the two exchanges DataParallel implies are made explicit:

* the loss: ``DistributedUNet.losses`` all-reduces the 8 batch sums of the fused loss
  statistics (Σbce, Σdice_n, TP, Σp, Σt, samples, elements) before the finalize, so every
  rank evaluates the loss of the gathered batch -- including FocalTversky, whose TP/FP/FN
  are global (models/loss.py:41-45) -- and its dlogits are its slice of the gathered
  batch's dlogits (any shard sizes);
* the gradients: the ranks' gradient arenas are SUMMED with ``torch.distributed``
  all-reduce (backend "nccl" == RCCL on ROCm, over xGMI), DataParallel's reduce-add.

A caller that takes a per-rank LOCAL loss instead (plain ``seg_losses`` without a group)
passes ``average=True``: the sum is then scaled by 1/world inside the AdamW pass
(``grad_scale``), which equals the gathered-batch gradient for equal shards and
shard-decomposable losses (BCE-mean, per-sample Dice), not for FocalTversky.  With
``average=False`` (the default) ``reduce_gradients`` refuses a step whose loss did not
come from ``losses`` (or ``empty_step``): summing gradients of per-rank local losses would
silently train with world-times-larger gradients.

BatchNorm buffers: DataParallel re-broadcasts replica 0's parameters AND buffers before
every forward (torch nn/parallel/replicate.py), so every shard is evaluated with GPU 0's
running statistics and only replica 0's running-stat updates survive a training step.
Train-mode forwards never read the running statistics, so here they may drift per rank
during training; ``sync_buffers`` broadcasts rank 0's running-stat and counter arenas
(2 x 5,888 floats + 18 int64 for models/model.py) and the Trainer calls it before every
validate / test pass (utils/trainer.py:130,210 -> eval forwards at :139,216).

Overlap: the native backward records one event per gradient bucket (decoder first,
unet_bucket_range); ``reduce_gradients`` enqueues, on a side stream, "wait for bucket b"
followed by the all-reduce of bucket b, for b = 0..B-1.  Because the host enqueues the
whole backward before the GPU has finished it, the all-reduce of the decoder buckets runs
while the encoder's dgrad/wgrad kernels are still executing.

On CPU tensors (gloo, tests) the same bucket walk runs without stream waits.
"""
import torch
import torch.distributed as dist


class BucketReducer:
    """Sums a flat gradient arena across ranks bucket by bucket.

    buckets: [(offset, length)] in readiness order.  wait_fn(b, stream) makes `stream`
    wait until bucket b is complete (native event) -- None on CPU.
    """

    def __init__(self, buckets, group=None, wait_fn=None):
        self.buckets = list(buckets)
        self.group = group
        self.wait_fn = wait_fn
        self.stream = None

    def reduce(self, arena, wait_native=True):
        """Sum `arena` over the ranks in place; returns the world size.  wait_native=False:
        the arena was not written by a native backward this step (an empty shard)."""
        ws = dist.get_world_size(self.group)
        if ws == 1:
            return 1
        works = []
        if arena.is_cuda:
            if self.stream is None:
                self.stream = torch.cuda.Stream(device=arena.device)
            main = torch.cuda.current_stream(arena.device)
            with torch.cuda.stream(self.stream):
                for b, (off, n) in enumerate(self.buckets):
                    if self.wait_fn is not None and wait_native:
                        self.wait_fn(b, self.stream)
                    else:
                        self.stream.wait_stream(main)
                    works.append(dist.all_reduce(arena[off:off + n], group=self.group,
                                                 async_op=True))
            for w in works:
                w.wait()  # makes the current (compute) stream wait for the collective
            main.wait_stream(self.stream)
        else:
            for off, n in self.buckets:
                works.append(dist.all_reduce(arena[off:off + n], group=self.group, async_op=True))
            for w in works:
                w.wait()
        return ws


def broadcast_module(module, src=0, group=None):
    """Rank src's parameters and buffers to every rank (once, at setup)."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)


class DistributedUNet:
    """Wraps the HIP ``UNet`` for one-process-per-GPU data parallelism.

    ``losses(logits, targets)`` -> the [bce, dice, focal] of the GATHERED batch (same value
    on every rank); after ``backward``, ``reduce_gradients()`` sums the gradient arenas.
    ``average=True`` is for per-rank local losses (see the module docstring)."""

    def __init__(self, model, optimizer=None, group=None, average=False):
        self.model = model
        self.group = group
        self.average = average
        st = model.flatten_()
        broadcast_module(model, 0, group)
        rt = st.rt
        self.reducer = BucketReducer(rt.buckets, group, wait_fn=rt.stream_wait_bucket)
        self.optimizer = optimizer
        self._gathered_loss = False  # set by losses() / empty_step(), consumed by reduce_gradients

    def _src(self):
        return 0 if self.group is None else dist.get_global_rank(self.group, 0)

    def sync_buffers(self):
        """Every rank takes rank 0's BN running statistics and num_batches_tracked (the
        buffers nn.DataParallel evaluates every shard with).  One broadcast per arena."""
        st = self.model.flatten_()
        dist.broadcast(st.bn_arena, src=self._src(), group=self.group)
        dist.broadcast(st.nbt_arena, src=self._src(), group=self.group)

    def gather_batch(self, images, masks, device):
        """The gathered global batch (DataParallel's input before its scatter) on every
        rank, plus this rank's (offset, count) in it.  images / masks: this rank's shard or
        None for an empty shard.  Used by mixup, which the reference applies to the whole
        batch before DataParallel scatters it (utils/trainer.py:62-78)."""
        ws = dist.get_world_size(self.group)
        n = 0 if images is None else int(images.shape[0])
        shape = [0, 0, 0, 0] if images is None else list(images.shape)
        mshape = [0, 0, 0, 0] if masks is None else list(masks.shape)
        meta = torch.tensor([n] + shape[1:] + mshape[1:], dtype=torch.int64, device=device)
        metas = [torch.zeros_like(meta) for _ in range(ws)]
        dist.all_gather(metas, meta, group=self.group)
        metas = [m.tolist() for m in metas]
        counts = [m[0] for m in metas]
        full = next((m for m in metas if m[0] > 0), None)
        if full is None:
            return None, None, 0, 0
        ishape, mshp = full[1:4], full[4:7]
        cap = max(counts)
        out = []
        for t, shp in ((images, ishape), (masks, mshp)):
            pad = torch.zeros([cap] + shp, dtype=torch.float32, device=device)
            if n:
                pad[:n].copy_(t)
            parts = [torch.empty_like(pad) for _ in range(ws)]
            dist.all_gather(parts, pad, group=self.group)
            out.append(torch.cat([p[:c] for p, c in zip(parts, counts)]))
        rank = dist.get_rank(self.group)
        return out[0], out[1], sum(counts[:rank]), n

    def __call__(self, x):
        return self.model(x)

    def losses(self, logits, targets, alpha=0.4, beta=0.6, gamma=2.0):
        from .functional import seg_losses
        grp = self.group if self.group is not None else dist.group.WORLD
        if torch.is_grad_enabled() and logits.requires_grad:
            # only a differentiable (training) loss licenses the next gradient sum; an
            # eval / no_grad pass in between (validate) must not
            self._gathered_loss = True
        return seg_losses(logits, targets, alpha, beta, gamma, group=grp)

    def empty_step(self, extra_scalar_reduces=0):
        """This rank's shard of the batch is empty (a last batch with fewer samples than
        ranks, data.data_loader.DataParallelShardSampler): join the step's collectives -- the
        loss sums, `extra_scalar_reduces` single-value all-reduces (the trainer's boundary
        loss), the gradient buckets -- with zero contributions, so that every rank then
        applies the same summed gradients."""
        st = self.model.flatten_()
        dev = st.param_arena.device
        sums = torch.zeros(8, dtype=torch.float64, device=dev)
        dist.all_reduce(sums, group=self.group)  # SegLossFunction.forward's collective
        for _ in range(extra_scalar_reduces):
            z = torch.zeros(1, device=dev)
            dist.all_reduce(z, group=self.group)
        if st.grad_arena is None:
            st.grad_arena = torch.zeros_like(st.param_arena)
        else:
            st.grad_arena.zero_()
        for (p, _, _), g in zip(st.params, st.grad_views(st.grad_arena)):
            p.grad = g
        self._gathered_loss = True
        return self.reduce_gradients(wait_native=False)

    def empty_losses(self, extra_scalar_reduces=0):
        """Eval-mode counterpart of empty_step: only the loss collectives."""
        dev = self.model.flatten_().param_arena.device
        sums = torch.zeros(8, dtype=torch.float64, device=dev)
        dist.all_reduce(sums, group=self.group)
        for _ in range(extra_scalar_reduces):
            z = torch.zeros(1, device=dev)
            dist.all_reduce(z, group=self.group)

    def reduce_gradients(self, wait_native=True):
        """Sum (or, with average=True, average) the flat gradient arena over the ranks.
        Returns the scale the optimizer applies to the summed gradients."""
        if not self.average and not self._gathered_loss:
            raise RuntimeError("reduce_gradients() SUMS the ranks' gradients, which is the "
                               "gathered-batch gradient only when the loss came from "
                               "DistributedUNet.losses() this step; for per-rank local losses "
                               "construct DistributedUNet(..., average=True)")
        self._gathered_loss = False
        st = self.model._state
        p0 = st.params[0][0]
        arena = st.grad_arena
        if p0.grad is None or p0.grad.data_ptr() != arena.data_ptr():
            raise RuntimeError("gradients are not in the flat grad arena (accumulated grads are "
                               "not supported by the bucketed reducer)")
        ws = self.reducer.reduce(arena, wait_native)
        scale = 1.0 / ws if self.average else 1.0
        if self.optimizer is not None and hasattr(self.optimizer, "grad_scale"):
            self.optimizer.grad_scale = scale
        elif scale != 1.0:
            arena.mul_(scale)
        return scale
