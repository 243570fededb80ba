# Tile/seed kernel ablations (ablation library) + instruction-rate microbenchmarks.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/valu_peak > gpurun_out/valu_peak.jsonl 2>&1 || exit $?
export SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_abl.so
for a in 0 11 12 13 14 15; do
  SCT_SPECTRAL_ABL=$a timeout -k 10 120 python3 tools/spectral_kernels.py 2 5 >> gpurun_out/tile_abl.jsonl 2>>gpurun_out/tile_abl.err || exit $?
done
for a in 1 2 3; do
  SCT_SEED_ABL=$a timeout -k 10 120 python3 tools/spectral_kernels.py 2 5 >> gpurun_out/tile_abl.jsonl 2>>gpurun_out/tile_abl.err || exit $?
done
exit 0
