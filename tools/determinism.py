"""Diagnostic: is ast_loss_grad deterministic?  The same x evaluated N times (eager, then as one
captured graph replayed N times, then two engines' graphs interleaved); every evaluation's loss
parts and gradient are compared bitwise with the first.

  python tools/determinism.py [B] [N]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from audio_style_transfer_amd.engine import StyleEngine


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device('cuda', 0)
    engs, xs = [], []
    for g in range(2):
        e = StyleEngine(B, 16384, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
        engs.append(e)
        xs.append(bench.make_problem(e, list(range(g * B, (g + 1) * B)), 16384, dev))
    ref = []
    for e, x in zip(engs, xs):
        p, gr = e.loss_grad(x)
        ref.append((p.clone(), gr.clone()))
    torch.cuda.synchronize()

    def cmp(tag, k, p, gr):
        rp, rg = ref[k]
        dp = (p != rp).any(dim=1)
        dg = (gr != rg).any(dim=1)
        if dp.any() or dg.any():
            print('%s engine %d: parts differ on clips %s, grad on clips %s; max |dparts| %.3g max |dgrad| %.3g'
                  % (tag, k, dp.nonzero().flatten().tolist(), dg.nonzero().flatten().tolist(),
                     float((p - rp).abs().max()), float((gr - rg).abs().max())), flush=True)
            return 1
        return 0

    bad = 0
    for i in range(N):
        for k, (e, x) in enumerate(zip(engs, xs)):
            p, gr = e.loss_grad(x)
            bad += cmp('eager %d' % i, k, p, gr)
    print('eager: %d mismatches in %d' % (bad, 2 * N), flush=True)
    outs, graphs = [], []
    for k, (e, x) in enumerate(zip(engs, xs)):
        gr = torch.empty_like(x)
        p = torch.empty(B, 4, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            e.loss_grad(x, gr, p)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            e.loss_grad(x, gr, p)
        outs.append((p, gr))
        graphs.append(g)
    bad = 0
    for i in range(N):
        graphs[0].replay()
        torch.cuda.synchronize()
        bad += cmp('graph0 alone %d' % i, 0, *outs[0])
    print('graph engine 0 alone: %d mismatches in %d' % (bad, N), flush=True)
    bad = 0
    for i in range(N):
        for k in range(2):
            graphs[k].replay()
        torch.cuda.synchronize()
        for k in range(2):
            bad += cmp('graphs interleaved %d' % i, k, *outs[k])
    print('graphs interleaved: %d mismatches in %d' % (bad, 2 * N), flush=True)
    bad = 0
    for i in range(N):
        for k in range(2):
            graphs[k].replay()
            torch.cuda.synchronize()
            bad += cmp('graphs interleaved+sync %d' % i, k, *outs[k])
    print('graphs interleaved with syncs: %d mismatches in %d' % (bad, 2 * N), flush=True)


if __name__ == '__main__':
    main()
