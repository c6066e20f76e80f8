"""Sums rocprofv3 --pmc counters per kernel family (k_block_fwd_s / k_block_bwd_s / gram) over
one or more run_counter_collection.csv files; prints per-launch means.
usage: pmc_sum.py <csv> [<csv> ...]"""
import csv, sys, collections
fams = ('k_block_fwd_s', 'k_block_bwd_s', 'k_gram_fwd_s', 'k_gram_bwd_s')
for path in sys.argv[1:]:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row['Kernel_Name']
            fam = next((x for x in fams if x in k), None)
            if fam is None or int(row['Grid_Size']) < 65536:
                continue
            per[fam][row['Counter_Name']] += float(row['Counter_Value'])
            disp[fam].add(row['Dispatch_Id'])
    for fam in fams:
        if fam in per:
            n = len(disp[fam])
            print(fam, 'launches', n, ' '.join('%s=%.4g' % (c, v / n) for c, v in sorted(per[fam].items())))
