# Register-tile variants (SCT_SPECTRAL_TILE=...): SPECTRAL parity tests under TEST_VARIANTS,
# then seed / tile kernel times (tools/spectral_kernels.py, 737K) for AB_VARIANTS, 3 rounds.
# (Round 2 used it for reg / reg_qp / reg_qp2 / reg_p16 / reg_q16w3 and the since-removed
# fast-square variants: profiles/ab_tile_*_r02.jsonl.)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
for v in ${TEST_VARIANTS:-reg_p16}; do
SCT_SPECTRAL_TILE=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread -m gpu -k "spectral" > gpurun_out/tile_${v}_pytest.log 2>&1
rc=$?; echo "$v pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
done
fi
O=gpurun_out/tile_ab.jsonl
for rep in 1 2 3; do
  for v in ${AB_VARIANTS:-reg_qp reg_p16}; do
    r=$(SCT_SPECTRAL_TILE=$v timeout -k 10 120 python3 tools/spectral_kernels.py 2 5) || exit $?
    echo "{\"tile\": \"$v\", \"k\": $r}" >> $O
  done
done
exit 0
