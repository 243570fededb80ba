set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  for c in 65536 131072 262144; do
    echo "{\"chunk\": $c, \"t\": $(SCT_SPECTRAL_CHUNK=$c timeout -k 10 120 python3 tools/spectral_time.py 2 8)}" >> gpurun_out/chunk_ab.jsonl || exit $?
  done
done
