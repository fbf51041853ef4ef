"""Multi-process data-parallel path on CPU (gloo, world_size 2).

The per-rank compute is the CPU oracle; the code under test is the product's bucket
reducer (unet_hip/dist.py: BucketReducer over the native gradient-bucket table) and the
two DP semantics it implements, pinned against fixtures produced by the reference itself
under nn.DataParallel (utils/trainer.py:28-30):

* per-rank local losses (``DistributedUNet(average=True)``): the summed gradients times
  1/world equal the gathered batch's gradient for BCE + Dice on equal shards
  (tests/golden/unet_dp2_64.npz);
* the gathered-batch loss (the default; what ``DistributedUNet.losses`` / the native
  unet_loss_stats -> all-reduce -> unet_loss_finalize sequence computes): each rank
  all-reduces the 8 batch sums of the loss statistics, differentiates the loss of the
  gathered batch w.r.t. its own logits, and the SUMMED gradients equal DataParallel's --
  with FocalTversky's global TP/FP/FN and with unequal shards (tests/golden/unet_dpf_64.npz).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "thyroid-nodule-image-segmentation-unet-ddti_amd")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (REPO, PKG):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    try:
        from oracle import unet_ref_cpu as O
        from oracle import weights as Wt
        from unet_hip.dist import BucketReducer
        from unet_hip.runtime import UNetRuntime
        rt = UNetRuntime("cuda:0")  # host-side tables only (no device work)
        P = O.make_params(42)
        x = torch.from_numpy(Wt.make_input(3, 4, 1, 64, 64))
        t = torch.from_numpy(Wt.make_target(3, 4, 64, 64))
        xs, ts = torch.chunk(x, world)[rank], torch.chunk(t, world)[rank]
        r = O.train_step(P, O.init_buffers(), None, xs, ts)
        arena = torch.empty(rt.n_param_floats)
        for name, shape, off in rt.params:
            arena[off:off + int(np.prod(shape))] = r["grads"][name].reshape(-1)
        ws = BucketReducer(rt.buckets).reduce(arena)
        scale = 1.0 / ws
        arena.mul_(scale)
        loss = r["loss"].clone()
        dist.all_reduce(loss)
        loss /= world
        if rank == 0:
            norms = [float(arena[off:off + int(np.prod(shape))].double().norm())
                     for name, shape, off in rt.params]
            q.put((float(loss), norms, scale))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_dp2_gloo_matches_dataparallel_golden(golden_dir):
    f = np.load(os.path.join(golden_dir, "unet_dp2_64.npz"), allow_pickle=False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    loss, norms, scale = q.get(timeout=500)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert scale == 0.5
    assert abs(loss - float(f["loss"])) < 1e-5
    np.testing.assert_allclose(norms, f["grad_norm"], rtol=1e-4)


def _bucket_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, PKG)
        from unet_hip.dist import BucketReducer
        buckets = [(70, 30), (20, 50), (0, 20)]
        arena = torch.arange(100, dtype=torch.float32) * (rank + 1)
        s = BucketReducer(buckets).reduce(arena)
        if rank == 0:
            q.put((s, arena.tolist()))
    finally:
        dist.destroy_process_group()


def test_bucket_reducer_sums_every_bucket():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    s, vals = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert s == 2
    assert vals == [3.0 * i for i in range(100)]


def _batch_sums(logits, t):
    """The 7 batch sums of the native loss statistics (kernels_misc.hip loss_sums_kernel),
    differentiable: {sum bce_elem, sum_n dice_n, TP, sum p, sum t, samples, elements}."""
    import torch.nn.functional as F
    n = logits.shape[0]
    p = torch.sigmoid(logits)
    bce = F.binary_cross_entropy_with_logits(logits, t, reduction="sum")
    pf, tf = p.reshape(n, -1), t.reshape(n, -1)
    inter = (pf * tf).sum(1)
    dice = ((2 * inter + 1) / (pf.sum(1) + tf.sum(1) + 1)).sum()
    one = torch.ones((), dtype=logits.dtype)
    return torch.stack([bce, dice, inter.sum(), pf.sum(), tf.sum(), n * one, logits.numel() * one])


def _losses_from_sums(S, alpha=0.4, beta=0.6, gamma=2.0):
    """kernels_misc.hip loss_finalize_kernel (models/loss.py:13-46 on the gathered batch)."""
    tp, fp, fn = S[2], S[3] - S[2], S[4] - S[2]
    ti = (tp + 1e-6) / (tp + alpha * fp + beta * fn + 1e-6)
    return S[0] / S[6], 1 - S[1] / S[5], (1 - ti) ** gamma


def _gathered_worker(rank, world, port, q, tag, B, seed, ratios):
    import sys
    for p in (REPO, PKG):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    try:
        from oracle import unet_ref_cpu as O
        from oracle import weights as Wt
        from unet_hip.dist import BucketReducer
        from unet_hip.runtime import UNetRuntime
        rt = UNetRuntime("cuda:0")  # host-side tables only (no device work)
        P = O.make_params(42)
        x = torch.from_numpy(Wt.make_input(seed, B, 1, 64, 64))
        t = torch.from_numpy(Wt.make_target(seed, B, 64, 64))
        xs, ts = torch.chunk(x, world)[rank], torch.chunk(t, world)[rank]  # DP scatter
        Pg = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
        logits = O.forward(xs, Pg, O.init_buffers(), True).double()
        s_loc = _batch_sums(logits, ts.double())
        S = s_loc.detach().clone()
        dist.all_reduce(S)  # the one loss collective (DistributedUNet.losses)
        S_glob = s_loc + (S - s_loc.detach())  # other ranks' sums are constants here
        lb, ld, lf = _losses_from_sums(S_glob)
        loss = ratios[0] * lb + ratios[1] * ld + ratios[2] * lf
        loss.backward()
        arena = torch.empty(rt.n_param_floats, dtype=torch.float64)
        for name, shape, off in rt.params:
            arena[off:off + int(np.prod(shape))] = Pg[name].grad.double().reshape(-1)
        ws = BucketReducer(rt.buckets).reduce(arena)  # DataParallel's reduce-add: a SUM
        if rank == 0:
            norms = [float(arena[off:off + int(np.prod(shape))].norm())
                     for name, shape, off in rt.params]
            q.put((float(lb), float(ld), float(lf), float(loss), norms, ws))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("tag,B,seed", [("eq_", 4, 22), ("uneq_", 3, 23)])
def test_gathered_batch_loss_matches_dataparallel_focal(golden_dir, tag, B, seed):
    f = np.load(os.path.join(golden_dir, "unet_dpf_64.npz"), allow_pickle=False)
    ratios = [float(v) for v in f[tag + "ratios"]]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gathered_worker, args=(r, 2, port, q, tag, B, seed, ratios))
             for r in range(2)]
    for p in procs:
        p.start()
    lb, ld, lf, loss, norms, ws = q.get(timeout=500)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert ws == 2
    for v, k in ((lb, "bce"), (ld, "dice"), (lf, "focal"), (loss, "loss")):
        assert abs(v - float(f[tag + k])) < 1e-5, k
    # per-rank fp32 forward (each shard's own BN, as DataParallel) -> grads to the
    # reference's fp32 error (~4e-3 norm-relative is the reference's own
    # fp32 vs fp64 spread; the loss here is evaluated in fp64)
    np.testing.assert_allclose(norms, f[tag + "grad_norm"], rtol=2e-3)


def _config3_worker(rank, world, port, q, n, bs):
    """One rank of config 3's data-parallel step arithmetic: its DataParallelShardSampler
    shard of every global batch, a per-rank 'gradient' arena built from its samples, the
    product's BucketReducer over the real 31M-float bucket table of models/model.py."""
    import sys
    for p in (REPO, PKG):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    try:
        from data.data_loader import DataParallelShardSampler
        from unet_hip.dist import BucketReducer
        from unet_hip.runtime import UNetRuntime
        rt = UNetRuntime("cuda:0")  # host-side tables only (no device work)
        base = (torch.arange(rt.n_param_floats) % 13).float()
        samp = DataParallelShardSampler(n, bs, True, rank, world, seed=7)
        out = []
        for shard in samp:
            # every per-sample contribution is an exact small integer multiple of `base`,
            # so the summed arena is exact whatever the reduction order
            w = float(sum(i + 1 for i in shard))
            arena = base * w
            ws = BucketReducer(rt.buckets).reduce(arena)
            ok = torch.equal(arena[:1000], base[:1000] * arena[1] / max(base[1].item(), 1.0))
            out.append((len(shard), float(arena[1]), float(arena[-1]), ok, ws,
                        bool(torch.equal(arena, base * float(arena[1])))))
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,n,bs", [(4, 256 + 5, 256), (8, 2 * 256 + 3, 256)])
def test_config3_shards_and_bucket_sum(world, n, bs):
    """Config 3 (bs 256 = 8 x 32 over 8 ranks; 4 x 64 over 4) with a ragged last batch
    smaller than the rank count (some shards empty): every rank's BucketReducer result
    equals the single-process sum over the GLOBAL batch, for every bucket of the real
    models/model.py gradient table."""
    from data.data_loader import DataParallelShardSampler
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config3_worker, args=(r, world, port, q, n, bs)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=500)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    glob = DataParallelShardSampler(n, bs, True, 0, world, seed=7).global_batches()
    assert len(out) == len(glob)
    for (n0, v1, vlast, ok, ws, whole), gb in zip(out, glob):
        want = float(sum(int(i) + 1 for i in gb))
        assert ws == world and ok and whole
        assert v1 == want * 1.0, (v1, want)   # base[1] == 1
        assert n0 == len(torch.chunk(gb, world)[0])
    assert out[0][0] == bs // world                 # 32 per GPU at 8 ranks
    assert len(torch.chunk(glob[-1], world)) < world  # the ragged batch left shards empty


def _gather_worker(rank, world, port, q, sizes):
    import sys
    from types import SimpleNamespace
    sys.path.insert(0, PKG)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from unet_hip.dist import DistributedUNet
        off = sum(sizes[:rank])
        n = sizes[rank]
        full = torch.arange(sum(sizes) * 2 * 3 * 3, dtype=torch.float32).view(-1, 2, 3, 3)
        mfull = -full[:, :1]
        imgs = full[off:off + n] if n else None
        msks = mfull[off:off + n] if n else None
        gi, gm, o, c = DistributedUNet.gather_batch(SimpleNamespace(group=None), imgs, msks, "cpu")
        q.put((rank, torch.equal(gi, full), torch.equal(gm, mfull), o, c))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [(2, 2, 1), (1, 0, 0), (3, 3, 2)])
def test_gather_batch_rebuilds_the_global_batch(sizes):
    """DistributedUNet.gather_batch (the trainer's DataParallel mixup: the reference mixes
    the whole batch before the scatter, utils/trainer.py:62-78) rebuilds the gathered batch
    on every rank from ragged and empty shards, with each rank's offset and count."""
    world = len(sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q, list(sizes))) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r, ok_i, ok_m, o, c in res:
        assert ok_i and ok_m
        assert (o, c) == (sum(sizes[:r]), sizes[r])
