# One GPU call: the SPECTRAL parity tests (-k spectral or config5), then seed / tile kernel
# times of config 5 and config 2 (tools/spectral_kernels.py).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu -k "${PYTEST_K:-spectral or config5}" > gpurun_out/pytest_s16.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/spectral_kernels.py 5 5 > gpurun_out/s16_k5.json 2> gpurun_out/s16_k5.err || exit $?
timeout -k 10 200 python -u tools/spectral_kernels.py 2 5 > gpurun_out/s16_k2.json 2> gpurun_out/s16_k2.err || exit $?
exit 0
