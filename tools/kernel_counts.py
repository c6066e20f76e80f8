"""Per-kernel launch counts and mean durations of a rocprofv3 kernel trace (usage: kernel_counts.py <csv>)."""
import collections, csv, sys
c = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    c[r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for k, v in sorted(c.items(), key=lambda kv: -sum(kv[1])):
    print('%-60s %5d %8.3f ms' % (k[:60], len(v), sum(v) / len(v)))
