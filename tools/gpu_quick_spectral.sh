# SPECTRAL parity tests, per-rank step emulation and kernel times (one GPU call).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "spectral or scheme or allpairs" > gpurun_out/pytest_spectral.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/rank_step.py 2 20 > gpurun_out/rank_step.jsonl 2>gpurun_out/rank_step.err || exit $?
timeout -k 10 120 python3 tools/spectral_kernels.py 2 5 > gpurun_out/kernels.jsonl 2>gpurun_out/kernels.err || exit $?
exit 0
