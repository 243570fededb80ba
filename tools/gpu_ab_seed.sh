# One GPU call: SPECTRAL parity tests (-k ${PYTEST_K:-step_major}), then the interleaved seed A/B
# on config ${AB_CONFIG:-2} (tools/ab_seed_tune.py) of ${AB_VARIANTS}.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -v --timeout 180 --timeout-method thread -m gpu -k "${PYTEST_K:-step_major}" > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_seed_tune.py ${AB_CONFIG:-2} ${AB_ROUNDS:-5} ${AB_VARIANTS:-spectral_seed=0 spectral_seed=1} > gpurun_out/ab_seed.json 2> gpurun_out/ab_seed.err
