#!/bin/bash
# quick benches of library variants: tools/abvar.sh name1 name2 ... (libastyle_<name>.so; "base" = libastyle.so;
# "onewave" = libastyle.so with the one-wave-per-SIMD block kernels; "db" = ASTYLE_FWD_DB=1)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  lib=audio_style_transfer_amd/libastyle_$v.so; [ "$v" = base ] && lib=audio_style_transfer_amd/libastyle.so
  envs=""; [ "$v" = onewave ] && { lib=audio_style_transfer_amd/libastyle.so; envs="ASTYLE_FWD_ROLES=0 ASTYLE_BWD_ROLES=0"; }
  [ "$v" = db ] && { lib=audio_style_transfer_amd/libastyle.so; envs="ASTYLE_FWD_DB=1"; }
  env $envs ASTYLE_LIB=$lib timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/var_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/var_$v.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'value %.3f ms/step %.1f'%(d['value'],d['ms_per_step']), {k:round(v,2) for k,v in d['kernels_ms_per_step'].items()}, 'fwd %.3f bwd %.3f ms/launch'%(d['roofline']['fwd']['launch_ms'], d['roofline']['bwd']['launch_ms']), 'grad', d.get('grad_rel_l2'))" gpurun_out/var_$v.log $v
done
