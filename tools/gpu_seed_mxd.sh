# Direct MFMA seed + 4-slice interleaved intermediate (SCT_SPECTRAL_SEED=mxd): SPECTRAL parity
# tests under it, then seed / tile / count times beside the shipped walk seed + reg_qp tile.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  SCT_SPECTRAL_SEED=mxd timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread -m gpu -k "spectral" > gpurun_out/seed_mxd_pytest.log 2>&1
  rc=$?; echo "mxd pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
fi
O=gpurun_out/seed_mxd_ab.jsonl
for rep in 1 2 3; do
  for v in ${AB_SEEDS:-walk mxd}; do
    r=$(SCT_SPECTRAL_SEED=$v timeout -k 10 120 python3 tools/spectral_kernels.py 2 5) || exit $?
    t=$(SCT_SPECTRAL_SEED=$v timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
    echo "{\"seed\": \"$v\", \"k\": $r, \"count\": $t}" >> $O
  done
done
exit 0
