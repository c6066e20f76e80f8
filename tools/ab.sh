mkdir -p gpurun_out
for V in "$@"; do
  if [ $V = base ]; then L=audio_style_transfer_amd/libastyle.so; else L=audio_style_transfer_amd/libastyle_$V.so; fi
  ASTYLE_LIB=$L timeout -k 10 200 python bench.py --cpu-baseline-seconds 0 --fp32-steps 0 > gpurun_out/ab_$V.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$V.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$V', round(d['value'],3), round(r['fwd_launch_ms'],4), round(r['bwd_launch_ms'],4))"
done
