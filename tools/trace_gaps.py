"""Per-kernel durations and the idle gap in front of each launch from a rocprofv3 kernel trace
(diagnostic): python tools/trace_gaps.py <kernel_trace.csv> [name-substring ...]"""
import csv
import sys
from collections import defaultdict

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'],
                     int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])))
rows.sort()
want = sys.argv[2:] or ['']
dur, gap = defaultdict(list), defaultdict(list)
for i, (s, e, n, g) in enumerate(rows):
    key = (n.split('(')[0][-60:], g)
    dur[key].append((e - s) / 1e3)
    if i:
        gap[key].append((s - rows[i - 1][1]) / 1e3)
for key in sorted(dur, key=lambda k: -sum(dur[k])):
    if not any(w in key[0] for w in want):
        continue
    d, gp = dur[key], gap[key]
    d_s = sorted(d)
    print('%-60s grid %8d  n %5d  mean %8.1f us  median %8.1f  gap mean %6.1f us' % (
        key[0], key[1], len(d), sum(d) / len(d), d_s[len(d_s) // 2], sum(gp) / max(1, len(gp))))
