#!/bin/bash
# Round-4 GPU check: the GPU suite, then the default bench, clip groups (--groups 2) and the
# Gram-stage A/B, each step under its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/gputest.log; exit 1; }
tail -2 gpurun_out/gputest.log
for v in "g1:--groups 1" "g2:--groups 2" "g4:--groups 4" "st2:--groups 1:ASTYLE_GRAM_STAGES=2" "bs3:--groups 1:ASTYLE_GRAM_BWD_STAGES=3" "vb:--groups 1:ASTYLE_LIB=audio_style_transfer_amd/libastyle_fwdvariants.so" "wp:--groups 1:ASTYLE_LIB=audio_style_transfer_amd/libastyle_fwdvariants.so ASTYLE_FWD_WINOPROBE=1" "bwp:--groups 1:ASTYLE_LIB=audio_style_transfer_amd/libastyle_fwdvariants.so ASTYLE_BWD_WINOPROBE=1" "gy1:--gatys --groups 1" "gy2:--gatys --groups 1:ASTYLE_GATYS_BWD=2"; do
  tag=${v%%:*}; rest=${v#*:}; args=${rest%%:*}; envs=""; [ "$rest" != "$args" ] && envs=${rest#*:}
  env $envs timeout -k 10 300 python bench.py --cpu-baseline-seconds 0 --side-steps 0 --steps 10 $args > gpurun_out/r4_$tag.log 2>&1 || { echo "bench $tag failed"; tail -30 gpurun_out/r4_$tag.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r4_$tag.log').read().strip().splitlines()[-1]); r=d['roofline']; k=d['kernels_ms_per_step']; print('$tag', round(d['value'],3), round(d['ms_per_step'],2), 'fwd', round(r['fwd']['launch_ms'],4), 'bwd', round(r['bwd']['launch_ms'],4), 'gram', round(k['gram_fwd'],2), round(k['gram_bwd'],2), 'other', round(k['other'],2), 'grad', d['grad_rel_l2'], 'flagged', d.get('range_flagged_clips'))"
done
