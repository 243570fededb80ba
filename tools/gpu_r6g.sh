# Round 6: the one-block arena for workspace-freeing one-shot plans: the SPECTRAL / plan-cache /
# device-split tests, then the drop-in path both ways.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6g
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_devices.py \
  tests/test_gpu_parity.py -k "allpairs or spectral or plan_cache or distinct or summary or whitelist_1k or first50 or small_sets or config1 or negative_keys" > $P/pytest.log 2>&1
rc=$?
tail -3 $P/pytest.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 tools/run_paths.py dropin > $P/dropin.json 2> $P/dropin.err || exit 3
echo done
