"""Diagnostic: which half of ast_loss_grad goes wrong on graph replay.  Against the eager result
of the same x: (a) the whole call captured; (b) both phases captured as two graphs; (c) phase 1
eager, phase 2 captured; (d) the whole call with the block kernels on 128 CUs.  4 replays each.

  python tools/determinism2.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from audio_style_transfer_amd.engine import StyleEngine


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device('cuda', 0)
    e = StyleEngine(B, 16384, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
    x = bench.make_problem(e, list(range(B)), 16384, dev)
    rp, rg = e.loss_grad(x)
    rp, rg = rp.clone(), rg.clone()
    g = torch.empty_like(x)
    p = torch.empty(B, 4, device=dev)

    def report(tag):
        torch.cuda.synchronize()
        dp = (p != rp).any(dim=1)
        dg = (g != rg).any(dim=1)
        return '%s parts clips %s grad clips %s' % (tag, dp.nonzero().flatten().tolist(),
                                                     dg.nonzero().flatten().tolist())

    ph = lambda k: (lambda: e.loss_grad_phase(x, g, p, k))
    def warm(*fns):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for f in fns:
                f()
        torch.cuda.current_stream().wait_stream(s)

    def cap(fn):
        gg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gg):
            fn()
        return gg

    for mode in ('a', 'b', 'c', 'd'):
        out = []
        if mode in ('a', 'd'):
            if mode == 'd':
                e.set_cu_limit(128)
            warm(ph(0))
            gr = cap(ph(0))
            for i in range(4):
                gr.replay()
                out.append(report('r%d' % i))
            e.set_cu_limit(0)
        elif mode == 'b':
            warm(ph(1), ph(2))
            gr = cap(ph(1))
            g2 = cap(ph(2))      # (the host side saw phase 1 captured just before)
            for i in range(4):
                gr.replay()
                g2.replay()
                out.append(report('r%d' % i))
            del g2
        else:
            warm(ph(1), ph(2))
            e.loss_grad_phase(x, g, p, 1)
            gr = cap(ph(2))
            for i in range(4):
                e.loss_grad_phase(x, g, p, 1)
                gr.replay()
                out.append(report('r%d' % i))
        del gr
        print('mode %s: %s' % (mode, ' | '.join(out)), flush=True)


if __name__ == '__main__':
    main()
