#!/usr/bin/env python3
"""Gradient-bucket readiness timeline of one config-2 backward (bs 32, 256x256) on one GPU:
the overlap budget of the data-parallel all-reduce.

For every bucket b of the native table (unet_bucket_range, decoder first) a side stream
waits on the library's bucket event (unet_stream_wait_bucket) and records a timing event, so
its timestamp is when the bucket's gradients are complete.  Printed: bucket sizes, ready
time after the backward starts, and the backward's end, as JSON (profiles/r03_buckets.json).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "thyroid-nodule-image-segmentation-unet-ddti_amd")]

import torch  # noqa: E402

import unet_hip  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(42)
    m = unet_hip.UNet(1, 1).to(dev).train()
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-5)
    g = torch.Generator().manual_seed(1000)
    x = torch.rand(32, 1, 256, 256, generator=g).to(dev)
    t = (torch.rand(32, 1, 256, 256, generator=g) > 0.5).float().to(dev)
    rt = m.flatten_().rt
    side = torch.cuda.Stream(device=dev)
    res = []
    for it in range(4):
        opt.zero_grad(set_to_none=True)
        logits = m(x)
        losses = unet_hip.seg_losses(logits, t)
        loss = losses[0] + losses[1]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        loss.backward()
        e1.record()
        evs = []
        with torch.cuda.stream(side):
            for b in range(len(rt.buckets)):
                rt.stream_wait_bucket(b, side)
                e = torch.cuda.Event(enable_timing=True)
                e.record(side)
                evs.append(e)
        torch.cuda.current_stream().wait_stream(side)
        opt.step()
        torch.cuda.synchronize()
        if it:  # first iteration warms up
            res.append(([e0.elapsed_time(e) for e in evs], e0.elapsed_time(e1)))
    n = len(res)
    ready = [sum(r[0][b] for r in res) / n for b in range(len(rt.buckets))]
    bwd = sum(r[1] for r in res) / n
    out = {"workload": "models/model.py UNet bs=32 256x256 backward (config 2/3 per rank)",
           "backward_ms": round(bwd, 3),
           "buckets": [{"bucket": b, "mbytes": round(4 * ln / 1e6, 2), "ready_ms": round(ready[b], 3)}
                       for b, (off, ln) in enumerate(rt.buckets)]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
