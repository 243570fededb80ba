# Register-resident tile kernel variants (SCT_SPECTRAL_TILE=reg|reg_np|reg_w3): SPECTRAL parity
# tests under each, then seed/tile kernel times beside the shipped two-stage kernel.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in reg reg_np reg_w3; do
  SCT_SPECTRAL_TILE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spectral" > gpurun_out/tile_reg_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
done
O=gpurun_out/tile_reg_ab.jsonl
for rep in 1 2; do
  for v in mfma2 reg reg_np reg_w3; do
    r=$(SCT_SPECTRAL_TILE=$v timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
    t=$(SCT_SPECTRAL_TILE=$v timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
    echo "{\"tile\": \"$v\", \"k\": $r, \"count\": $t}" >> $O
  done
done
exit 0
