# MFMA seed kernel (default for int8 seeds; SCT_SPECTRAL_SEED=walk = the Gray-walk seed):
# SPECTRAL parity, then seed/tile times and whole-count times beside the walk seed.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spectral or 737k or config5" > gpurun_out/seed_mx.log 2>&1
rc=$?; echo "mx pytest rc=$rc"; tail -3 gpurun_out/seed_mx.log; [ $rc -ne 0 ] && exit $rc
O=gpurun_out/seed_mx_ab.jsonl
for rep in 1 2; do
  for sv in mx walk; do
    r=$(SCT_SPECTRAL_SEED=$sv timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
    t=$(SCT_SPECTRAL_SEED=$sv timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
    echo "{\"seed\": \"$sv\", \"k\": $r, \"count\": $t}" >> $O
  done
done
exit 0
