"""Per-layer durations (median over the trace's launches) of the bench-sized block kernels in a
rocprofv3 kernel-trace CSV: forward launch i = layer i, backward launch i = layer 29 - i.
usage: trace_layers.py <kernel_trace.csv> [grid_threads]"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
grid = sys.argv[2] if len(sys.argv) > 2 else '65536'
for nk in ('k_block_fwd_s', 'k_block_bwd_s'):
    ks = sorted((r for r in rows if nk in r['Kernel_Name'] and r['Grid_Size_X'] == grid),
                key=lambda r: int(r['Start_Timestamp']))
    if not ks:
        continue
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in ks]
    per = collections.defaultdict(list)
    for i, v in enumerate(d):
        per[i % 30].append(v)
    m = [statistics.median(per[i]) for i in range(30)]
    if 'bwd' in nk:
        m = m[::-1]
    print('%s launches %d mean %.1f us' % (nk, len(d), sum(d) / len(d)))
    print('  ' + ' '.join('%d:%.0f' % (l, m[l]) for l in range(30)))
