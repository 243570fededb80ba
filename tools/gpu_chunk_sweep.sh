# SPECTRAL count time vs chunk size (slices per seed/tile pass), with the histogram checked.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${VARIANTS:-65536 131072 262144 65536 131072 262144}; do
  echo -n "{\"chunk\": $c, \"r\": " >> gpurun_out/chunk_sweep.jsonl
  SCT_SPECTRAL_CHUNK=$c timeout -k 10 120 python3 tools/spectral_time.py 2 8 >> gpurun_out/chunk_sweep.jsonl 2>>gpurun_out/chunk_sweep.err || exit $?
  echo -n ", \"k\": " >> gpurun_out/chunk_sweep.jsonl
  sed -i '$ s/\n$//' gpurun_out/chunk_sweep.jsonl
  SCT_SPECTRAL_CHUNK=$c timeout -k 10 120 python3 tools/spectral_kernels.py 2 1 | tr -d '\n' >> gpurun_out/chunk_sweep.jsonl 2>>gpurun_out/chunk_sweep.err || exit $?
  echo "}" >> gpurun_out/chunk_sweep.jsonl
done
exit 0
