"""Summarise tools/sqpmc.sh output: mean counter value per kernel (block kernels)."""
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
with open(sys.argv[1]) as f:
    for row in csv.DictReader(f):
        if 'block' in row['Kernel_Name']:
            acc[row['Kernel_Name']][row['Counter_Name']].append(float(row['Counter_Value']))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print('   %-24s %14.4g' % (c, sum(v) / len(v)))
