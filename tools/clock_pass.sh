#!/bin/bash
# Effective shader clock per kernel (MI355X_MICROARCH.md 'DVFS give-back': GRBM_GUI_ACTIVE / 8 XCDs / kernel time)
# usage: tools/clock_pass.sh <tag> [env assignments...]   -> gpurun_out/clock_<tag>/
set -euo pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/clock_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
env "$@" timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE -T --output-format csv -d "$OUT" -o run -- python3 bench.py --cpu-baseline-seconds 0 --side-steps 0 > "$OUT/bench.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = defaultdict(lambda: [0.0, 0.0, 0])
for r in csv.DictReader(open(f)):
    if r['Counter_Name'] != 'GRBM_GUI_ACTIVE':
        continue
    g = int(r['Grid_Size']) if 'Grid_Size' in r else 0
    k = (r['Kernel_Name'].split('(')[0][-40:], g)
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) if 'End_Timestamp' in r else 0
    a = acc[k]; a[0] += float(r['Counter_Value']); a[1] += dur; a[2] += 1
for k, (c, d, n) in sorted(acc.items(), key=lambda x: -x[1][1])[:8]:
    if d:
        print('%-40s grid %8d n %4d  clock %6.0f MHz' % (k[0], k[1], n, c / 8 / d * 1e3))
PY
