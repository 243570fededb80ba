# Fast-square register tile variants (SCT_SPECTRAL_TILE=reg_fs / reg_fs2; reg_fs3 = no energy
# test, ablation library, timing only): SPECTRAL parity tests, then kernel times beside reg.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
for v in ${TEST_VARIANTS:-reg_fs2}; do
SCT_SPECTRAL_TILE=$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread -m gpu -k "spectral" > gpurun_out/tile_${v}_pytest.log 2>&1
rc=$?; echo "$v pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
done
fi
O=gpurun_out/tile_fs_ab.jsonl
for rep in 1 2 3; do
  for v in ${AB_VARIANTS:-reg reg_fs reg_fs2 reg_fs3}; do
    lib=""
    [ "$v" = "reg_fs3" ] && lib=sctools_amd/libsctools_hip_abl.so
    r=$(SCTOOLS_HIP_LIB=$lib SCT_SPECTRAL_TILE=$v timeout -k 10 120 python3 tools/spectral_kernels.py 2 5) || exit $?
    echo "{\"tile\": \"$v\", \"k\": $r}" >> $O
  done
done
exit 0
