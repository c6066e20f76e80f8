#!/bin/bash
# timing variants of the double-buffered forward kernel (ASTYLE_FWD_DB=1): tools/abdb.sh lib1 lib2 ...
# ("base" = libastyle.so; "one" = libastyle.so with the default kernel)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  lib=audio_style_transfer_amd/libastyle_$v.so; db=1
  [ "$v" = base ] && lib=audio_style_transfer_amd/libastyle.so
  [ "$v" = one ] && { lib=audio_style_transfer_amd/libastyle.so; db=0; }
  ASTYLE_FWD_DB=$db ASTYLE_LIB=$lib timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 > gpurun_out/abdb_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/abdb_$v.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], 'value %.3f'%d['value'], 'fwd %.3f bwd %.3f ms/launch'%(d['roofline']['fwd']['launch_ms'], d['roofline']['bwd']['launch_ms']))" gpurun_out/abdb_$v.log $v
done
