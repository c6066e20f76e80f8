"""Diagnostic: does running the 256-clip batch as G concurrent clip groups (one StyleEngine and
one stream each, the persistent block kernels limited to 256/G CUs) beat one engine?  While one
group runs its HBM-bound Gram kernels, the other's MFMA-bound block kernels use the other CUs.

  python tools/groups_probe.py [steps] [offset_ms]

Prints ms per 256-clip step for: one engine; G = 2 groups started together (lock-step);
G = 2 groups with the second delayed by offset_ms (a torch.cuda._sleep on its stream, counted
in the timed region)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from audio_style_transfer_amd.engine import AdamLoop, StyleEngine
from audio_style_transfer_amd.shard import clip_range


def setup(G, B=256, T=16384):
    dev = torch.device('cuda', 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    loops, streams = [], []
    for g in range(G):
        eng = StyleEngine(B // G, T, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
        if G > 1:
            eng.set_cu_limit(ncu // G)
        x = bench.make_problem(eng, list(range(g * B // G, (g + 1) * B // G)), T, dev)
        loops.append(AdamLoop(eng, x, lr=2.0, graph=True))
        streams.append(torch.cuda.Stream(device=dev))
    return loops, streams


def timed(loops, streams, steps, offset_ms=0.0):
    for lp, s in zip(loops, streams):
        with torch.cuda.stream(s):
            lp.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for g, (lp, s) in enumerate(zip(loops, streams)):
        with torch.cuda.stream(s):
            if g and offset_ms > 0:
                torch.cuda._sleep(int(offset_ms * 1e-3 * 2.1e9 * g))
            for _ in range(steps):
                lp.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    off = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
    t_sleep = time.perf_counter()
    torch.cuda._sleep(int(0.05 * 2.1e9))
    torch.cuda.synchronize()
    print('sleep calibration: 50 ms requested -> %.1f ms' % ((time.perf_counter() - t_sleep) * 1e3), flush=True)
    loops, streams = setup(1)
    print('one engine: %.2f ms/step' % timed(loops, streams, steps), flush=True)
    del loops, streams
    torch.cuda.empty_cache()
    loops, streams = setup(2)
    print('2 groups lock-step: %.2f ms/step' % timed(loops, streams, steps), flush=True)
    for o in (off, off / 2, 1.5 * off):
        print('2 groups offset %.0f ms: %.2f ms/step (incl. the offset)' % (o, timed(loops, streams, steps, o)), flush=True)


if __name__ == '__main__':
    main()
