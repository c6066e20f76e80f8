"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats, verbatim) and
profiles/<tag>_summary.json: per kernel and grid size (from the kernel trace, so the bench's
small side-check launches do not dilute the bench-sized ones), average duration and HBM
traffic per launch from the separate FETCH_SIZE / WRITE_SIZE passes.  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE counts half the bytes of a wide (16 B/lane) coalesced read, so fetched bytes =
2 * FETCH_SIZE * 1024; WRITE_SIZE reads exactly for 16-B stores: written = WRITE_SIZE * 1024.
Also (re)writes profiles/traffic.json (traffic_gatys.json for a --gatys profile) for bench.py's
roofline.traffic field.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, name):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row['Counter_Name'] == name:
                per[(row['Kernel_Name'], int(row['Grid_Size']))].append(float(row['Counter_Value']))
    return per


def launches(path):
    """Per (kernel, grid size in threads) durations from the kernel trace: the bench's side
    checks launch the same kernels on small batches, which the --stats averages mix in."""
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            grid = int(row['Grid_Size_X']) * int(row['Grid_Size_Y']) * int(row['Grid_Size_Z'])
            per[(row['Kernel_Name'], grid)].append(
                (int(row['End_Timestamp']) - int(row['Start_Timestamp'])) / 1e6)
    return per


def main(tag, precision, clips, T):
    src = os.path.join(ROOT, 'gpurun_out', 'prof_' + tag)
    dst = os.path.join(ROOT, 'profiles')
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, 'trace', 'run_kernel_stats.csv'),
                os.path.join(dst, tag + '_kernel_stats.csv'))
    stats = {}
    for (name, grid), ds in launches(os.path.join(src, 'trace', 'run_kernel_trace.csv')).items():
        stats['%s@%d' % (name, grid)] = {'name': name, 'grid_threads': grid, 'calls': len(ds),
                                         'avg_ms': sum(ds) / len(ds), 'total_ms': sum(ds),
                                         'min_ms': min(ds), 'max_ms': max(ds)}
    fetch = counters(os.path.join(src, 'fetch', 'run_counter_collection.csv'), 'FETCH_SIZE')
    write = counters(os.path.join(src, 'write', 'run_counter_collection.csv'), 'WRITE_SIZE')
    for v in stats.values():
        k = (v['name'], v['grid_threads'])
        if k in fetch:
            v['fetch_bytes_raw'] = sum(fetch[k]) / len(fetch[k]) * 1024
            v['fetch_bytes_corrected'] = 2 * v['fetch_bytes_raw']
        if k in write:
            v['write_bytes'] = sum(write[k]) / len(write[k]) * 1024
        if 'fetch_bytes_corrected' in v and 'write_bytes' in v:
            v['hbm_bytes_per_launch'] = v['fetch_bytes_corrected'] + v['write_bytes']
            v['hbm_GBs'] = v['hbm_bytes_per_launch'] / (v['avg_ms'] * 1e-3) / 1e9
    summary = {'tag': tag, 'precision': precision, 'clips': clips, 'T': T, 'kernels': stats}
    with open(os.path.join(dst, tag + '_summary.json'), 'w') as f:
        json.dump(summary, f, indent=1)
    def pick(name):   # the bench-sized launches (largest grid) of every template variant
        ks = [k for k in stats if name in k and 'hbm_bytes_per_launch' in stats[k]]
        big = max((stats[k]['grid_threads'] for k in ks), default=0)
        ks = [k for k in ks if stats[k]['grid_threads'] == big]
        n = sum(stats[k]['calls'] for k in ks)
        if not n:
            return {}
        return {'hbm_bytes_per_launch': sum(stats[k]['hbm_bytes_per_launch'] * stats[k]['calls']
                                            for k in ks) / n,
                'avg_ms': sum(stats[k]['avg_ms'] * stats[k]['calls'] for k in ks) / n, 'calls': n}
    fw, bw = pick('k_block_fwd'), pick('k_block_bwd')
    gatys = any('k_gatys' in k for k in stats)
    gf, gb = (pick('k_gatys_fwd'), pick('k_gatys_bwd')) if gatys else (pick('k_gram_fwd'), pick('k_gram_bwd'))
    if 'hbm_bytes_per_launch' in fw and 'hbm_bytes_per_launch' in bw:
        # the library the profiled runs loaded (tools/profile.sh records its sha256)
        with open(os.path.join(src, 'lib.sha256')) as f:
            sha = f.read().split()[0][:16]
        tj = {'precision': precision, 'clips': clips, 'T': T, 'gatys': gatys, 'source': tag,
              'lib_sha16': sha,
              'fwd_bytes_per_launch': fw['hbm_bytes_per_launch'],
              'bwd_bytes_per_launch': bw['hbm_bytes_per_launch'],
              'fwd_ms': fw['avg_ms'], 'bwd_ms': bw['avg_ms'],
              'gram_fwd_bytes_per_launch': gf.get('hbm_bytes_per_launch'),
              'gram_bwd_bytes_per_launch': gb.get('hbm_bytes_per_launch'),
              'gram_fwd_ms': gf.get('avg_ms'), 'gram_bwd_ms': gb.get('avg_ms')}
        with open(os.path.join(dst, 'traffic_gatys.json' if gatys else 'traffic.json'), 'w') as f:
            json.dump(tj, f, indent=1)
    for k, v in sorted(stats.items(), key=lambda kv: -kv[1]['total_ms'])[:10]:
        print('%-40s calls %4d avg %8.3f ms  hbm/launch %s' % (
            k[:40], v['calls'], v['avg_ms'],
            '%.3f GB (%.0f GB/s)' % (v['hbm_bytes_per_launch'] / 1e9, v['hbm_GBs'])
            if 'hbm_bytes_per_launch' in v else '-'))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
