"""Reads a rocprofv3 kernel-trace CSV and prints the mean duration of each block-kernel launch
position (launch i of every forward / backward: dilation 2^(i % 10) for the forward)."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
for name_key in ('k_block_fwd_s', 'k_block_bwd_s'):
    ks = [r for r in rows if name_key in r['Kernel_Name']]
    if not ks:
        continue
    ks.sort(key=lambda r: int(r['Start_Timestamp']))
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in ks]
    per = collections.defaultdict(list)
    for i, v in enumerate(d):
        per[i % 30].append(v)
    print(name_key, 'launches', len(d), 'mean us', sum(d) / len(d))
    print(' '.join('%d:%.0f' % (i, sum(v) / len(v)) for i, v in sorted(per.items())))
