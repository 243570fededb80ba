# Spread-store seed kernel (SCT_SPECTRAL_SEED=spread): SPECTRAL parity, then seed/tile times
# and whole-count times beside the shipped kernels, and walks per workgroup (ablation lib).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
SCT_SPECTRAL_SEED=spread SCT_SPECTRAL_TILE=reg timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spectral or 737k" > gpurun_out/seed_spread.log 2>&1
rc=$?; echo "spread pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
O=gpurun_out/seed_spread_ab.jsonl
for rep in 1 2; do
  for sv in old spread; do
    for tv in mfma2 reg; do
      r=$(SCT_SPECTRAL_SEED=$sv SCT_SPECTRAL_TILE=$tv timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
      t=$(SCT_SPECTRAL_SEED=$sv SCT_SPECTRAL_TILE=$tv timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
      echo "{\"seed\": \"$sv\", \"tile\": \"$tv\", \"k\": $r, \"count\": $t}" >> $O
    done
  done
done
for w in 4 8 16 32; do
  r=$(SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_abl.so SCT_SEED_WALKS=$w SCT_SPECTRAL_SEED=spread timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
  echo "{\"seed\": \"spread\", \"walks\": $w, \"k\": $r}" >> $O
done
exit 0
