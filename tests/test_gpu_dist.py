"""The data-parallel product path on a real GPU: two ranks (gloo, both on cuda:0 -- the
pool's boxes have one GPU, and RCCL refuses two ranks on one device) run the HIP UNet
through ``unet_hip.dist.DistributedUNet``: parameters broadcast from rank 0, per-rank
train-mode BN on its shard (DataParallel's torch.chunk scatter), the loss of the GATHERED
batch (``DistributedUNet.losses``: native loss statistics -> all-reduce of the 8 batch
sums -> native finalize), the native per-bucket events gating the side-stream all-reduce
that SUMS the gradients.  Loss values and summed gradients must match the reference's own
nn.DataParallel fixtures -- BCE + Dice (tests/golden/unet_dp2_64.npz) and the default
FocalTversky mix on equal and unequal shards (tests/golden/unet_dpf_64.npz) -- and both
ranks must hold identical parameters after the AdamW step."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "thyroid-nodule-image-segmentation-unet-ddti_amd")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, seed, B, ratios, average):
    import sys
    for p in (REPO, PKG, os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import unet_hip
        from _helpers import hip_model
        from oracle import unet_ref_cpu as O
        from oracle import weights as Wt
        from unet_hip.dist import DistributedUNet
        dev = torch.device("cuda:0")
        # rank 1 starts from different weights: the broadcast must replace them
        m = hip_model(O.make_params(42 if rank == 0 else 7), dev)
        opt = unet_hip.HipAdamW(m.parameters(), lr=1e-5)
        ddp = DistributedUNet(m, opt, average=average)
        x = torch.from_numpy(Wt.make_input(seed, B, 1, 64, 64))
        t = torch.from_numpy(Wt.make_target(seed, B, 64, 64))
        xs, ts = torch.chunk(x, world)[rank].to(dev), torch.chunk(t, world)[rank].to(dev)
        opt.zero_grad(set_to_none=True)
        logits = ddp(xs)
        if average:  # per-rank local losses, averaged gradients
            losses = unet_hip.seg_losses(logits, ts)
        else:        # the gathered batch's losses, summed gradients
            losses = ddp.losses(logits, ts)
        loss = ratios[0] * losses[0] + ratios[1] * losses[1] + ratios[2] * losses[2]
        loss.backward()
        scale = ddp.reduce_gradients()
        grads = m._state.grad_arena.detach().clone() * scale
        opt.step()
        params = m._state.param_arena.detach().clone()
        vals = torch.cat([losses.detach().double(), loss.detach().double().reshape(1)]).cpu()
        if average:
            dist.all_reduce(vals)
            vals /= world
        pd = params.cpu()
        dist.broadcast(pd, src=0)
        same = bool(torch.equal(pd, params.cpu()))
        if rank == 0:
            rt = m._state.rt
            norms = [float(grads[off:off + int(np.prod(shape))].double().norm())
                     for name, shape, off in rt.params]
            q.put((vals.tolist(), norms, scale, same))
        else:
            q.put(("rank1", vals.tolist(), same))
    finally:
        dist.destroy_process_group()


def _run(seed, B, ratios, average):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, seed, B, ratios, average))
             for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=500), q.get(timeout=500)]
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    r0 = [r for r in res if r[0] != "rank1"][0]
    r1 = [r for r in res if r[0] == "rank1"][0]
    return r0, r1


@pytest.mark.timeout(600)
def test_dp2_on_gpu_matches_dataparallel_golden(golden_dir):
    """BCE + Dice, equal shards, both DP modes: the gathered-batch loss with summed
    gradients (default) and per-rank local losses with averaged gradients."""
    f = np.load(os.path.join(golden_dir, "unet_dp2_64.npz"), allow_pickle=False)
    for average in (False, True):
        (vals, norms, scale, same0), r1 = _run(3, 4, (1.0, 1.0, 0.0), average)
        assert scale == (0.5 if average else 1.0)
        assert same0 and r1[2], "ranks diverged after the AdamW step"
        assert abs(vals[3] - float(f["loss"])) < 1e-5, (average, vals[3], float(f["loss"]))
        if not average:
            assert vals == r1[1], "ranks disagree on the gathered-batch loss"
        np.testing.assert_allclose(norms, f["grad_norm"], rtol=1e-2)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("tag,B,seed", [("eq_", 4, 22), ("uneq_", 3, 23)])
def test_dp2_focal_on_gpu_matches_dataparallel_golden(golden_dir, tag, B, seed):
    """FocalTversky in the DP loss (global TP/FP/FN of the gathered batch): the CLI default
    ratios on equal shards, 1/1/1 on DataParallel's unequal scatter (3 -> 2 + 1)."""
    f = np.load(os.path.join(golden_dir, "unet_dpf_64.npz"), allow_pickle=False)
    ratios = tuple(float(v) for v in f[tag + "ratios"])
    (vals, norms, scale, same0), r1 = _run(seed, B, ratios, False)
    assert scale == 1.0
    assert same0 and r1[2], "ranks diverged after the AdamW step"
    assert vals == r1[1], "ranks disagree on the gathered-batch loss"
    for v, k in zip(vals, ("bce", "dice", "focal", "loss")):
        assert abs(v - float(f[tag + k])) < 1e-5, (k, v, float(f[tag + k]))
    np.testing.assert_allclose(norms, f[tag + "grad_norm"], rtol=1e-2)
