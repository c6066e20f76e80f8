set -o pipefail
for envs in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "AMD_SERIALIZE_KERNEL=3" "DEBUG_HIP_GRAPH_BATCH_SIZE=1"; do
  echo "== $envs"
  env $envs timeout -k 10 200 python tools/determinism.py 8 4 2>&1 | grep -E "mismatches" || exit 1
done
