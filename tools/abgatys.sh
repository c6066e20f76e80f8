#!/bin/bash
# --gatys quick benches of library variants (libastyle_<name>.so; base = libastyle.so)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  lib=audio_style_transfer_amd/libastyle_$v.so; [ "$v" = base ] && lib=audio_style_transfer_amd/libastyle.so
  ASTYLE_LIB=$lib timeout -k 10 300 python bench.py --gatys --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/gvar_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/gvar_$v.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'value %.3f ms/step %.1f'%(d['value'],d['ms_per_step']), {k:round(v,2) for k,v in d['kernels_ms_per_step'].items()}, 'grad', d.get('grad_rel_l2'))" gpurun_out/gvar_$v.log $v
done
