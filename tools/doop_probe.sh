#!/bin/bash
# Gram backward in place vs out of place, several processes each:
# kernel traces for the per-process duration, then TCC counter passes (one rocprofv3 --pmc pass
# per process, kernel trace on, so every pass carries its own duration).
# Usage (GPU box, repo root): tools/doop_probe.sh            (traces + the default counter sets)
#                             tools/doop_probe.sh "<set>" ...  (only these counter sets)
set -o pipefail
OUT=gpurun_out/doop
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
run() {   # run <doop> <counters or ->
  i=$((i+1))
  local pm=()
  [ "$2" != "-" ] && pm=(--pmc $2)
  ASTYLE_DOOP=$1 timeout -s KILL 120 rocprofv3 "${pm[@]}" --kernel-trace -T --output-format csv -d $OUT/r$i -o run -- python3 tools/gram_probe.py > $OUT/r$i.log 2>&1 || { echo "run $i failed"; tail -5 $OUT/r$i.log; return 1; }
  echo "r$i DOOP=$1 pmc=$2 $(grep 'step ms' $OUT/r$i.log)"
}
SETS=("$@")
if [ ${#SETS[@]} -eq 0 ]; then
  for d in 0 0 0 1 1 0 0; do run $d - || exit 1; done
  SETS=("FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum" "TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
else
  i=100
fi
for c in "${SETS[@]}"; do
  for d in 0 0 0 0 1 1; do run $d "$c" || exit 1; done
done
echo "doop probe done"
