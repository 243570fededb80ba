# Register tile micro-variants (SCT_SPECTRAL_TILE=reg1|reg2|reg3: plane sum on the matrix
# pipe / cvt_pk byte split / both): parity on each, then tile/count times beside reg.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in reg1 reg2 reg3; do
  SCT_SPECTRAL_TILE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spectral_scheme or 737k_spectral" > gpurun_out/tile_opt_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
O=gpurun_out/tile_opt_ab.jsonl
for rep in 1 2; do
  for v in reg reg1 reg2 reg3; do
    r=$(SCT_SPECTRAL_TILE=$v timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
    t=$(SCT_SPECTRAL_TILE=$v timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
    echo "{\"tile\": \"$v\", \"k\": $r, \"count\": $t}" >> $O
  done
done
exit 0
