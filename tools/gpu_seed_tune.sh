set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/seed_tune.jsonl
export SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_abl.so
for rep in 1 2; do
for w in 8 16 32; do
for a in 0 4 9 10; do
  r=$(SCT_SEED_ABL=$a SCT_SEED_WALKS=$w timeout -k 10 120 python3 tools/spectral_kernels.py 2 5 2>/dev/null) || exit $?
  echo "{\"abl\": $a, \"walks\": $w, \"r\": $r}" >> gpurun_out/seed_tune.jsonl
done; done; done
exit 0
