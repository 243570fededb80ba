# SPECTRAL count time vs chunk size (slices per seed/tile pass): does a chunk that fits the
# Infinity Cache (256 MB = 16,384 int8 slices) beat HBM round trips?
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in 65536 32768 16384 8192 4096 16384 65536; do
  echo -n "{\"chunk\": $c, \"r\": " >> gpurun_out/chunk_sweep.jsonl
  SCT_SPECTRAL_CHUNK=$c timeout -k 10 120 python3 tools/spectral_time.py 2 8 >> gpurun_out/chunk_sweep.jsonl 2>>gpurun_out/chunk_sweep.err || exit $?
  sed -i '$ s/$/}/' gpurun_out/chunk_sweep.jsonl
done
exit 0
