# Seed / tile overlap over two streams (SCT_SPECTRAL_OVERLAP=1) x seed kernel: parity, then
# whole-count times on the 737K headline.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spectral_kernel_variants or column_sizes or 737k" > gpurun_out/overlap2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/overlap2.log; [ $rc -ne 0 ] && exit $rc
O=gpurun_out/overlap2.jsonl
for rep in 1 2; do
  for sv in walk mx; do
    for ov in 0 1; do
      t=$(SCT_SPECTRAL_SEED=$sv SCT_SPECTRAL_OVERLAP=$ov timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
      echo "{\"seed\": \"$sv\", \"overlap\": $ov, \"count\": $t}" >> $O
    done
  done
done
exit 0
