# Ablations of the SPECTRAL kernels (ablation library; wrong results by design): tile
# (SCT_SPECTRAL_ABL 31 no loads, 32 no squares, 33 no LDS exchange, 34 no stage-2 MFMA,
# 35 no barriers) and seed (SCT_SEED_ABL 1 no stores, 2 no walk, 3 no LDS staging), each
# beside the unablated kernel in the same process order, twice.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/abl_r2.jsonl
export SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_abl.so
for rep in 1 2; do
  for a in 0 31 32 33 34 35; do
    r=$(SCT_SPECTRAL_ABL=$a timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
    echo "{\"tile_abl\": $a, \"r\": $r}" >> $O
  done
  for a in 0 1 2 3; do
    r=$(SCT_SEED_ABL=$a timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
    echo "{\"seed_abl\": $a, \"r\": $r}" >> $O
  done
done
exit 0
