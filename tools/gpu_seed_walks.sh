# Seed walks per workgroup sweep (ablation library, SCT_SEED_WALKS).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
export SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_abl.so
for w in ${WALKS:-8 2 4 16 32 8 4 16}; do
  SCT_SEED_WALKS=$w timeout -k 10 120 python3 tools/spectral_kernels.py 2 5 >> gpurun_out/seed_walks.jsonl 2>>gpurun_out/seed_walks.err || exit $?
done
exit 0
