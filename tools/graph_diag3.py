"""Diagnostic: which clips blow up when two engines of 8 clips live in one process.  Cases (each
in a fresh process): one engine of clips 0..7 / 8..15 / 0..15 alone; two engines stepped
alternately, graph and eager; two engines with only the first stepped.  Prints per-clip loss of
step 2 and the mean per step.

  python tools/graph_diag3.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, torch
sys.path.insert(0, sys.argv[1])
import bench
from audio_style_transfer_amd.engine import AdamLoop, StyleEngine
sets = [list(map(int, s.split('-'))) for s in sys.argv[2].split(',')]
graph, stepped = int(sys.argv[3]), int(sys.argv[4])
dev = torch.device('cuda', 0)
loops = []
for lo, hi in sets:
    e = StyleEngine(hi - lo, 16384, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
    x = bench.make_problem(e, list(range(lo, hi)), 16384, dev)
    loops.append(AdamLoop(e, x, lr=2.0, graph=bool(graph)))
means, per = [], None
for k in range(4):
    for lp in loops[:stepped]:
        lp.step()
    torch.cuda.synchronize()
    p = torch.cat([lp.parts[:, 0] for lp in loops[:stepped]]).cpu()
    means.append(round(float(p.mean()), 3))
    if k == 1:
        per = [round(float(v), 2) for v in p]
print('%s graph %d stepped %d: means %s step2 %s' % (sys.argv[2], graph, stepped, means, per), flush=True)
'''
for sets, graph, stepped in (('0-8', 1, 1), ('8-16', 1, 1), ('0-16', 1, 1), ('0-8,8-16', 1, 2),
                             ('0-8,8-16', 0, 2), ('0-8,8-16', 1, 1), ('8-16,0-8', 1, 1)):
    r = subprocess.run([sys.executable, '-c', CHILD, ROOT, sets, str(graph), str(stepped)],
                       capture_output=True, text=True, timeout=240)
    print(r.stdout.strip() or r.stderr[-1500:], flush=True)
