# Seed variants on config 2 and config 5 (int16 seeds): parity tests for $TESTS, then kernel
# times (tools/spectral_kernels.py) for the seeds in $AB on both configs.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sd in ${TESTS:-}; do
  SCT_SPECTRAL_SEED=$sd timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -m gpu -k "spectral" > gpurun_out/seed_cfg_${sd}_pytest.log 2>&1
  rc=$?; echo "$sd pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
done
O=gpurun_out/seed_cfg.jsonl
for rep in 1 2; do
  for cfg in 2 5; do
    for sd in ${AB:-walk}; do
      r=$(SCT_SPECTRAL_SEED=$sd timeout -k 10 200 python3 tools/spectral_kernels.py $cfg 3) || exit $?
      echo "{\"seed\": \"$sd\", \"cfg\": $cfg, \"k\": $r}" >> $O
    done
  done
done
exit 0
