"""Diagnostic: engine.AdamGroups at bench scale -- concurrent vs serialized replay (same graphs,
same phase offsets) and vs one AdamLoop per group run alone, per-step max |x| difference.

  python tools/groups_diag.py [clips_per_group] [T] [steps] [groups]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from audio_style_transfer_amd.engine import AdamGroups, AdamLoop, StyleEngine


def engines(G, Bg, T, dev):
    engs, xs = [], []
    for g in range(G):
        e = StyleEngine(Bg, T, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
        engs.append(e)
        xs.append(bench.make_problem(e, list(range(g * Bg, (g + 1) * Bg)), T, dev))
    return engs, xs


def main():
    Bg = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    G = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    dev = torch.device('cuda', 0)
    runs = {}
    for mode in ('alone', 'serial', 'concurrent'):
        engs, xs = engines(G, Bg, T, dev)
        traj, parts = [], []
        if mode == 'alone':
            loops = [AdamLoop(e, x, lr=2.0, graph=True) for e, x in zip(engs, xs)]
            for _ in range(steps):
                for lp in loops:
                    lp.step()
                torch.cuda.synchronize()
                traj.append(torch.cat([lp.x for lp in loops]).cpu())
                parts.append(torch.cat([lp.parts for lp in loops]).cpu())
        else:
            grp = AdamGroups(engs, xs, lr=2.0, serial=mode == 'serial')
            for _ in range(steps):
                grp.step()
                torch.cuda.synchronize()
                traj.append(torch.cat(grp.xs).cpu())
                parts.append(torch.cat(grp.parts).cpu())
        runs[mode] = (traj, parts)
        print(mode, 'loss per step', [round(float(p[:, 0].mean()), 5) for p in parts], flush=True)
        del engs, xs
        torch.cuda.empty_cache()
    for mode in ('serial', 'concurrent'):
        d = [float((a - b).abs().max()) for a, b in zip(runs['alone'][0], runs[mode][0])]
        print(mode, 'vs alone: max |dx| per step', ['%.3g' % v for v in d], flush=True)


if __name__ == '__main__':
    main()
