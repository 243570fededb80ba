# Round 6, first box: the new device-split / workspace / destroy-contract tests, the changed
# from_iterable_strings test and the plan-cache test, smoke, then the drop-in path both ways.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6a
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_devices.py \
  "tests/test_gpu_parity.py::test_from_iterable_strings_items_golden" \
  "tests/test_gpu_parity.py::test_plan_cache_reuse_and_release" > $P/pytest.log 2>&1
rc=$?
tail -5 $P/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || exit 3
timeout -k 10 300 python3 tools/run_paths.py dropin > $P/dropin.json 2> $P/dropin.err || exit 3
echo done
