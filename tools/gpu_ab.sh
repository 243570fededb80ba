# One GPU call: the all-pairs parity tests (-k allpairs), then an interleaved A/B of
# count-kernel variants (tools/ab_allpairs.py) on config ${AB_CONFIG:-2}.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${AB_TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests -x -v --timeout 180 --timeout-method thread -m gpu -k "${PYTEST_K:-allpairs}" > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
SCTOOLS_HIP_LIB=${AB_LIB:-} timeout -k 10 300 python -u tools/ab_allpairs.py --config ${AB_CONFIG:-2} --rounds ${AB_ROUNDS:-7} --variants ${AB_VARIANTS:-"v=2,s=0" "v=2,s=1"} > gpurun_out/ab.json 2> gpurun_out/ab.err
