# Seed column-chunk order A/B: SPECTRAL parity tests, then seed/tile kernel times with the
# current library and with SCTOOLS_HIP_LIB=$OLD_LIB alternately.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spectral or scheme or allpairs" > gpurun_out/pytest_spectral.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python3 tools/spectral_kernels.py 2 5 >> gpurun_out/order_new.jsonl 2>>gpurun_out/order_ab.err || exit $?
  SCTOOLS_HIP_LIB=$PWD/${OLD_LIB:-sctools_amd/libsctools_hip_old.so} timeout -k 10 120 python3 tools/spectral_kernels.py 2 5 >> gpurun_out/order_old.jsonl 2>>gpurun_out/order_ab.err || exit $?
done
timeout -k 10 120 python3 tools/spectral_kernels.py 5 3 >> gpurun_out/order_new.jsonl 2>>gpurun_out/order_ab.err || exit $?
exit 0
