"""Diagnostic: the same clips' Adam trajectories in engines of different batch size (each clip is
an independent problem, so clip c's losses must not depend on B): per-step losses of clips 0..3
for B = 16 and B = 256, graph and eager.

  python tools/batch_diag.py [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from audio_style_transfer_amd.engine import AdamLoop, StyleEngine


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device('cuda', 0)
    T = 16384
    for B, graph in ((16, True), (16, False), (256, True)):
        e = StyleEngine(B, T, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
        x = bench.make_problem(e, list(range(B)), T, dev)
        lp = AdamLoop(e, x, lr=2.0, graph=graph)
        rows = []
        for _ in range(steps):
            lp.step()
            torch.cuda.synchronize()
            rows.append([round(float(v), 5) for v in lp.parts[:4, 0].cpu()])
        print('B %d graph %d: clips 0..3 loss per step %s | mean %s' % (B, graph, rows, float(lp.parts[:, 0].mean())), flush=True)
        del lp, x, e
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
