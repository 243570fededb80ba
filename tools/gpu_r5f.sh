# Round 5: the whole GPU suite (one-read whitelist ingest with multi-limb rows, the nearest tables
# back to round 4's), then one default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5f
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -le 1 ] || exit 3
timeout -k 10 500 python3 bench.py > $P/bench.log 2> $P/bench.err || exit 3
echo done
