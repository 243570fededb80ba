# One GPU call: 16-bit-column parity tests, then the interleaved A/B of 14- vs 16-bit columns on
# config ${AB_CONFIG:-2} and config 5's kernels (tools/ab_seed_tune.py).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu -k "${PYTEST_K:-16bit or config5}" > gpurun_out/pytest_s16.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/ab_seed_tune.py ${AB_CONFIG:-2} ${AB_ROUNDS:-5} spectral_columns=14 spectral_columns=16 > gpurun_out/ab_s16_c2.json 2> gpurun_out/ab_s16_c2.err || exit $?
timeout -k 10 300 python -u tools/ab_seed_tune.py 5 3 spectral_columns=16 spectral_columns=14 > gpurun_out/ab_s16_c5.json 2> gpurun_out/ab_s16_c5.err || exit $?
exit 0
