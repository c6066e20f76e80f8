mkdir -p gpurun_out
for v in base cur base2 cur2; do
  case $v in base*) L=audio_style_transfer_amd/libastyle_base.so;; *) L=audio_style_transfer_amd/libastyle.so;; esac
  ASTYLE_LIB=$L timeout -k 10 200 python bench.py --clips 1 --steps 60 --warmup 3 --side-steps 0 --cpu-baseline-seconds 0 > gpurun_out/c1_$v.log 2>&1 || { tail -20 gpurun_out/c1_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/c1_$v.log').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$v', round(d['value']*256,1), 'clip-iters/s', round(d['ms_per_step'],3), 'ms', {a: round(b,3) for a,b in k.items()})"
done
