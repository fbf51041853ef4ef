#!/usr/bin/env python3
"""Overlap budget of the data-parallel gradient all-reduce on one GPU:
bucket readiness of one config-2 backward (bs 32, 256x256) and the step-time cost of
communication-like traffic running beside the backward.

1. Timeline.  For every bucket b of the native table (unet_bucket_range, decoder first) a side
   stream waits on the library's bucket event (unet_stream_wait_bucket) and records a timing
   event, so its timestamp is when the bucket's gradients are complete.

2. Interference (--interfere).  After each bucket event a side stream runs an elementwise
   device pass that reads and writes 2 * 7/8 of that bucket's bytes -- the per-rank ring
   volume of an 8-rank all-reduce -- while the remaining backward runs.  Modes: none, side
   stream at default priority, side stream at high priority (torch.cuda.Stream(priority=-1)).
   Whole training steps (forward, loss, backward, AdamW) are timed with HIP events, the modes
   interleaved round by round so box drift cancels; the inflation is each mode's median step
   over the no-traffic median.

   The stand-in is not RCCL: an RCCL ring kernel holds a few CUs (one block per channel) for
   the collective's whole duration, bounded by xGMI; this pass spreads short blocks over every
   CU and finishes at HBM speed.  Both contend with the GEMMs only where a CU frees up: the x3
   GEMMs run one block per CU with 160 KB of LDS, so nothing co-resides with them.

Prints JSON (profiles/r05_buckets.json).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "thyroid-nodule-image-segmentation-unet-ddti_amd")]

import torch  # noqa: E402

import unet_hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5, help="steps per mode per round")
    ap.add_argument("--ranks", type=int, default=8, help="ring size the traffic emulates")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(42)
    m = unet_hip.UNet(1, 1).to(dev).train()
    opt = unet_hip.HipAdamW(m.parameters(), lr=1e-5)
    g = torch.Generator().manual_seed(1000)
    x = torch.rand(32, 1, 256, 256, generator=g).to(dev)
    t = (torch.rand(32, 1, 256, 256, generator=g) > 0.5).float().to(dev)
    rt = m.flatten_().rt
    frac = 2.0 * (args.ranks - 1) / args.ranks
    nmax = max(int(frac * ln) for _, ln in rt.buckets)
    src = torch.rand(nmax, device=dev)
    dst = torch.empty(nmax, device=dev)
    streams = {"side": torch.cuda.Stream(device=dev),
               "side_high_priority": torch.cuda.Stream(device=dev, priority=-1)}

    def step(mode, timeline=False):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        opt.zero_grad(set_to_none=True)
        logits = m(x)
        losses = unet_hip.seg_losses(logits, t)
        loss = losses[0] + losses[1]
        eb = torch.cuda.Event(enable_timing=True)
        eb.record()
        loss.backward()
        ebe = torch.cuda.Event(enable_timing=True)
        ebe.record()
        evs = []
        if mode != "none" or timeline:
            side = streams.get(mode, streams["side"])
            with torch.cuda.stream(side):
                for b, (_, ln) in enumerate(rt.buckets):
                    rt.stream_wait_bucket(b, side)
                    if timeline:
                        e = torch.cuda.Event(enable_timing=True)
                        e.record(side)
                        evs.append(e)
                    if mode != "none":
                        n = int(frac * ln)
                        torch.mul(src[:n], 1.0000001, out=dst[:n])
            torch.cuda.current_stream().wait_stream(side)
        opt.step()
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        return e0, eb, ebe, evs, e1

    for _ in range(3):
        step("none")
    torch.cuda.synchronize()
    # 1. bucket timeline (ready time after the backward's first launch)
    tl = []
    for _ in range(4):
        e0, eb, ebe, evs, e1 = step("none", timeline=True)
        torch.cuda.synchronize()
        tl.append(([eb.elapsed_time(e) for e in evs], eb.elapsed_time(ebe)))
    nb = len(rt.buckets)
    ready = [sum(r[0][b] for r in tl) / len(tl) for b in range(nb)]
    bwd = sum(r[1] for r in tl) / len(tl)
    # 2. interference: interleaved rounds of whole steps per mode
    modes = ["none", "side", "side_high_priority"]
    times = {k: [] for k in modes}
    for _ in range(args.rounds):
        for mode in modes:
            for _ in range(2):  # settle
                step(mode)
            recs = [step(mode) for _ in range(args.steps)]
            torch.cuda.synchronize()
            times[mode] += [r[0].elapsed_time(r[4]) for r in recs]

    def med(v):
        v = sorted(v)
        return v[len(v) // 2]
    base = med(times["none"])
    moved = sum(2 * 4 * int(frac * ln) for _, ln in rt.buckets)
    out = {"workload": "models/model.py UNet bs=32 256x256 train step (config 2/3 per rank), one MI355X",
           "backward_ms": round(bwd, 3),
           "buckets": [{"bucket": b, "mbytes": round(4 * ln / 1e6, 2), "ready_ms": round(ready[b], 3),
                        "before_backward_end_ms": round(bwd - ready[b], 3)}
                       for b, (off, ln) in enumerate(rt.buckets)],
           "interference": {
               "traffic": (f"after each bucket event: torch.mul over 2*{args.ranks - 1}/{args.ranks} of the "
                           f"bucket's floats (read + write), {moved / 1e6:.0f} MB per step in total"),
               "steps_per_mode": len(times["none"]),
               "step_ms_median": {k: round(med(v), 3) for k, v in times.items()},
               "inflation_pct": {k: round(100 * (med(v) / base - 1), 2) for k, v in times.items() if k != "none"},
               "step_ms_all": {k: [round(a, 3) for a in v] for k, v in times.items()}}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
