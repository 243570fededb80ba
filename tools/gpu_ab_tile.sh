# A/B of tile variants (ablation library, SCT_SPECTRAL_ABL), hist printed for a correctness comparison.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
export SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_abl.so
for a in ${VARIANTS:-0 16 0 16}; do
  SCT_SPECTRAL_ABL=$a timeout -k 10 120 python3 tools/spectral_kernels.py ${CFG:-2} 5 >> gpurun_out/ab_tile.jsonl 2>>gpurun_out/ab_tile.err || exit $?
done
exit 0
