# Overlapped seed/tile schedule (SCT_SPECTRAL_OVERLAP = tile workgroups per CU) vs serial.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for o in ${VARIANTS:-0 1 2 3 0 2}; do
  echo -n "{\"overlap\": $o, \"t\": " >> gpurun_out/overlap.jsonl
  SCT_SPECTRAL_OVERLAP=$o timeout -k 10 120 python3 tools/spectral_time.py 2 8 >> gpurun_out/overlap.jsonl 2>>gpurun_out/overlap.err || exit $?
  sed -i '$ s/$/, "k": /' gpurun_out/overlap.jsonl
  SCT_SPECTRAL_OVERLAP=$o timeout -k 10 120 python3 tools/spectral_kernels.py 2 1 >> gpurun_out/overlap.jsonl 2>>gpurun_out/overlap.err || exit $?
  sed -i '$ s/$/}/' gpurun_out/overlap.jsonl
done
exit 0
