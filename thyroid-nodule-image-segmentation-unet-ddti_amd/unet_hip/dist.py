"""Data-parallel training: one process per GPU, RCCL all-reduce of the flat gradient arena.

Replaces the reference's single-process ``nn.DataParallel`` (utils/trainer.py:28-30), which
re-broadcasts all 124 MB of parameters every forward and reduces gradients to GPU 0.
Here every rank holds a full replica, parameters are broadcast ONCE from rank 0, each
rank runs its shard of the batch with its own train-mode BatchNorm statistics (exactly
DataParallel's per-replica BN), and after backward the gradient arena is summed with
``torch.distributed.all_reduce`` (backend "nccl" == RCCL on ROCm, over xGMI).  The sum
is turned into the mean (= the gradient of the full-batch loss with equal shards, since
BCE-mean and the per-sample Dice mean are averages over the shards) inside the AdamW
pass via ``grad_scale = 1 / world_size``.

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

    def reduce(self, arena):
        ws = dist.get_world_size(self.group)
        if ws == 1:
            return 1.0
        works = []
        if arena.is_cuda:
            if self.stream is None:
                self.stream = torch.cuda.Stream(device=arena.device)
            main = torch.cuda.current_stream(arena.device)
            with torch.cuda.stream(self.stream):
                for b, (off, n) in enumerate(self.buckets):
                    if self.wait_fn is not None:
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
        return 1.0 / ws


def broadcast_module(module, src=0, group=None):
    """Rank src's parameters and buffers to every rank (once, at setup)."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src=src, group=group)


class DistributedUNet:
    """Wraps the HIP ``UNet`` for one-process-per-GPU data parallelism."""

    def __init__(self, model, optimizer=None, group=None):
        self.model = model
        self.group = group
        st = model.flatten_()
        broadcast_module(model, 0, group)
        rt = st.rt
        self.reducer = BucketReducer(rt.buckets, group, wait_fn=rt.stream_wait_bucket)
        self.optimizer = optimizer

    def __call__(self, x):
        return self.model(x)

    def reduce_gradients(self):
        st = self.model._state
        p0 = st.params[0][0]
        arena = st.grad_arena
        if p0.grad is None or p0.grad.data_ptr() != arena.data_ptr():
            raise RuntimeError("gradients are not in the flat grad arena (accumulated grads are "
                               "not supported by the bucketed reducer)")
        scale = self.reducer.reduce(arena)
        if self.optimizer is not None and hasattr(self.optimizer, "grad_scale"):
            self.optimizer.grad_scale = scale
        elif scale != 1.0:
            arena.mul_(scale)
        return scale
