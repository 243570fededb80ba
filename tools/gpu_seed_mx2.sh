# MFMA seed workgroup forms (SCT_SPECTRAL_MX_FORM 0 = 64-column paired workgroups,
# 1 = 16-column waves x 8, 2 = 8-column waves x 16): parity on each, then seed / count times
# beside the walk seed, and two ablations of form 0 (ablation lib).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in 0 1 2; do
  SCT_SPECTRAL_SEED=mx SCT_SPECTRAL_MX_FORM=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spectral_scheme or column_sizes or 737k_spectral or crowded" > gpurun_out/seed_mx2_$f.log 2>&1
  rc=$?; echo "form $f pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
O=gpurun_out/seed_mx2_ab.jsonl
AB=$PWD/sctools_amd/libsctools_hip_abl.so
for rep in 1 2; do
  for v in walk mx0 mx1 mx2; do
    case $v in walk) e="SCT_SPECTRAL_SEED=walk";; mx*) e="SCT_SPECTRAL_SEED=mx SCT_SPECTRAL_MX_FORM=${v#mx}";; esac
    r=$(env $e timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
    t=$(env $e timeout -k 10 120 python3 tools/spectral_time.py 2 8) || exit $?
    echo "{\"v\": \"$v\", \"k\": $r, \"count\": $t}" >> $O
  done
  for a in 2 5; do
    r=$(SCTOOLS_HIP_LIB=$AB SCT_SPECTRAL_SEED=mx SCT_MX_ABL=$a timeout -k 10 120 python3 tools/spectral_kernels.py 2 3) || exit $?
    echo "{\"v\": \"mx0_abl$a\", \"k\": $r}" >> $O
  done
done
exit 0
