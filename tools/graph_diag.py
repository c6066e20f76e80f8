"""Diagnostic: AdamLoop graph replay vs eager at bench length (T = 16384): per-step losses of a
4-clip batch with and without a host synchronisation between steps, and the Adam step counter.

  python tools/graph_diag.py [T] [steps] [lr]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from audio_style_transfer_amd.engine import AdamLoop, StyleEngine


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    lr = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
    dev = torch.device('cuda', 0)
    e = StyleEngine(4, T, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
    x0 = bench.make_problem(e, list(range(4)), T, dev).clone()
    for mode in ('eager-sync', 'graph-sync', 'graph-nosync', 'eager-nosync'):
        lp = AdamLoop(e, x0.clone(), lr=lr, graph=mode.startswith('graph'))
        rows = []
        for _ in range(steps):
            lp.step()
            if mode.endswith('-sync'):
                torch.cuda.synchronize()
                rows.append((float(lp.parts[:, 0].mean()), int(lp.step_dev.item()),
                             float(lp.x.abs().max()), float(lp.grad.abs().max())))
        torch.cuda.synchronize()
        rows.append(('end', float(lp.parts[:, 0].mean()), int(lp.step_dev.item()), float(lp.x.abs().max())))
        print(mode, rows, flush=True)
        del lp


if __name__ == '__main__':
    main()
