#!/bin/bash
# The bare split GEMM-1 loop (tools/diag/mfma_shape) under one GRBM_GUI_ACTIVE pass: its TF/s
# and the shader clock it holds (the power-limited ceiling of the block kernels' MFMA stream).
set -euo pipefail
OUT=gpurun_out/mfma_clock; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE -T --output-format csv -d $OUT -o run -- ./tools/diag/mfma_shape > $OUT/out.log 2>&1
cat $OUT/out.log | grep -v amdgpu.ids
python3 - $OUT <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = defaultdict(lambda: [0.0, 0.0, 0])
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0][-30:]
    a = acc[k]; a[0] += float(r['Counter_Value']); a[1] += int(r['End_Timestamp']) - int(r['Start_Timestamp']); a[2] += 1
for k, (c, d, n) in acc.items():
    print('%-30s n %4d  mean %8.1f us  clock %6.0f MHz' % (k, n, d / n / 1e3, c / 8 / d * 1e3))
PY
