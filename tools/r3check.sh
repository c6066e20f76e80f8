#!/bin/bash
# Round-3 iteration loop on the GPU box: split parity tests, stamps of the split block kernels
# at B = 256, a quick bench.  usage: tools/r3check.sh [tests] [stamps] [quick]
set -o pipefail
mkdir -p gpurun_out
for step in "$@"; do
  case $step in
    tests) timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_tests.log; exit 1; }
           tail -2 gpurun_out/r3_tests.log ;;
    stamps) timeout -k 10 200 python tools/stamps.py 256 fwd > gpurun_out/r3_stamps_fwd.log 2>&1 && \
            timeout -k 10 200 python tools/stamps.py 256 bwd > gpurun_out/r3_stamps_bwd.log 2>&1 || { echo "stamps failed"; tail gpurun_out/r3_stamps_*.log; exit 1; }
            grep -v amdgpu.ids gpurun_out/r3_stamps_fwd.log; grep -v amdgpu.ids gpurun_out/r3_stamps_bwd.log | grep bwd ;;
    quick) timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/r3_quick.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/r3_quick.log; exit 1; }
           python -c "import json;d=json.loads(open('gpurun_out/r3_quick.log').read().strip().splitlines()[-1]);print('value %.3f ms/step %.1f'%(d['value'],d['ms_per_step']), d['kernels_ms_per_step'], 'fwd %.3f bwd %.3f ms/launch'%(d['roofline']['fwd']['launch_ms'], d['roofline']['bwd']['launch_ms']), 'grad', d.get('grad_rel_l2'))" ;;
  esac
done
