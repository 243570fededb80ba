# Round 5: where the pipelined step builds (side stream vs in line): the pipelined-step tests in
# both modes, then the same-box A/B at W = 1 and rank 0's W = 8 share.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5o
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "pipelined" --timeout 120 --timeout-method thread > $P/pytest_sel.log 2>&1
rc=$?
tail -3 $P/pytest_sel.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 400 python3 tools/build_on_ab.py > $P/ab_build_on.jsonl 2> $P/ab_build_on.err || exit 3
cat $P/ab_build_on.jsonl
echo done
