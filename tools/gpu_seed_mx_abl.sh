# MFMA seed ablations (ablation lib, SCT_MX_ABL): see seed_mx_kernel's ABL list; 10/12 =
# 4-wave workgroups (normal / no stores).  Beside the walk seed.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/seed_mx_abl.jsonl
AB=$PWD/sctools_amd/libsctools_hip_abl.so
for rep in 1 2; do
  r=$(SCTOOLS_HIP_LIB=$AB SCT_SPECTRAL_SEED=walk timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
  echo "{\"v\": \"walk\", \"k\": $r}" >> $O
  for v in 0 2 5 10 12 15; do
    r=$(SCTOOLS_HIP_LIB=$AB SCT_MX_ABL=$v timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
    echo "{\"v\": \"mx$v\", \"k\": $r}" >> $O
  done
done
exit 0
