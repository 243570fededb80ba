# Seed kernel times, current library vs $OLD_LIB, configs 2 and 5 (tools/spectral_kernels.py),
# after the SPECTRAL parity tests on the current library.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -m gpu -k "spectral" > gpurun_out/seed_lib_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
O=gpurun_out/seed_lib_ab.jsonl
for rep in 1 2; do
  for cfg in 2 5; do
    r=$(timeout -k 10 200 python3 tools/spectral_kernels.py $cfg 3) || exit $?
    echo "{\"lib\": \"new\", \"cfg\": $cfg, \"k\": $r}" >> $O
    r=$(SCTOOLS_HIP_LIB=$PWD/${OLD_LIB:-sctools_amd/libsctools_hip_old.so} timeout -k 10 200 python3 tools/spectral_kernels.py $cfg 3) || exit $?
    echo "{\"lib\": \"old\", \"cfg\": $cfg, \"k\": $r}" >> $O
  done
done
exit 0
