"""Summarise tools/doop_probe.sh output: per process, k_gram_bwd_s / k_gram_fwd_s durations
(kernel trace, evaluations 2.. only) and the TCC counters of k_gram_bwd_s per launch
(FETCH_SIZE in KB x2 on gfx950, WRITE_SIZE in KB, MI355X_MICROARCH.md)."""
import csv, glob, os, re, statistics, sys
D = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/doop'
rows = []
for log in sorted(glob.glob(os.path.join(D, 'r*.log')), key=lambda p: int(re.findall(r'r(\d+)', os.path.basename(p))[0])):
    tag = os.path.basename(log)[:-4]
    txt = open(log).read()
    m = re.search(r'DOOP=(\d)', txt)
    kt = os.path.join(D, tag, 'run_kernel_trace.csv')
    if not m or not os.path.isfile(kt):
        continue
    dur = {'bwd': [], 'fwd': []}
    for r in csv.DictReader(open(kt)):
        n = r['Kernel_Name']
        for k, key in (('k_gram_bwd_s', 'bwd'), ('k_gram_fwd_s', 'fwd')):
            if k in n:
                dur[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
    cnt = {}
    cc = os.path.join(D, tag, 'run_counter_collection.csv')
    if os.path.isfile(cc):
        per = {}
        for r in csv.DictReader(open(cc)):
            if 'k_gram_bwd_s' in r['Kernel_Name']:
                per.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
        for k, v in per.items():
            v = v[1:] if len(v) > 1 else v
            val = statistics.mean(v)
            if k == 'FETCH_SIZE':
                cnt['fetch_GB'] = round(val * 2 * 1024 / 1e9, 1)
            elif k == 'WRITE_SIZE':
                cnt['write_GB'] = round(val * 1024 / 1e9, 1)
            else:
                cnt[k.replace('TCC_EA0_', '').replace('_sum', '')] = '%.3g' % val
        if 'RDREQ_LEVEL' in cnt and 'RDREQ' in cnt:   # mean outstanding-read residency (cycles)
            cnt['rd_lat'] = '%.0f' % (float(cnt['RDREQ_LEVEL']) / float(cnt['RDREQ']))
        if 'WRREQ_LEVEL' in cnt and 'WRREQ' in cnt:
            cnt['wr_lat'] = '%.0f' % (float(cnt['WRREQ_LEVEL']) / float(cnt['WRREQ']))
    b = dur['bwd'][1:] or dur['bwd']
    f = dur['fwd'][1:] or dur['fwd']
    print('%-4s DOOP=%s gram_bwd %s ms  gram_fwd %.2f ms  %s' % (tag, m.group(1), ' '.join('%.1f' % x for x in b),
          statistics.mean(f) if f else 0, cnt))
