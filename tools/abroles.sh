#!/bin/bash
# A/B of the role-split block kernels on the GPU box: split + parity tests, then quick benches
# with the role-split kernels (default) and with the one-wave kernels (ASTYLE_*_ROLES=0).
# usage: tools/abroles.sh [tests] [bench]
set -o pipefail
mkdir -p gpurun_out
q() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'value %.3f ms/step %.1f'%(d['value'],d['ms_per_step']), {k:round(v,2) for k,v in d['kernels_ms_per_step'].items()}, 'fwd %.3f bwd %.3f ms/launch'%(d['roofline']['fwd']['launch_ms'], d['roofline']['bwd']['launch_ms']), 'grad', d.get('grad_rel_l2'))" "$1" "$2"; }
for step in "$@"; do
  case $step in
    tests) timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/roles_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/roles_tests.log; exit 1; }
           tail -2 gpurun_out/roles_tests.log ;;
    bench) timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/roles_quick.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/roles_quick.log; exit 1; }
           q gpurun_out/roles_quick.log roles
           ASTYLE_FWD_ROLES=0 ASTYLE_BWD_ROLES=0 timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/roles_off_quick.log 2>&1 || { echo "bench (off) failed"; tail -30 gpurun_out/roles_off_quick.log; exit 1; }
           q gpurun_out/roles_off_quick.log one-wave ;;
  esac
done
