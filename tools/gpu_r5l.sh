# Round 5: host stream stages from the stream-ordered pool and >= 4 chunks per call: the stream /
# pool / release tests, the FASTQ -> nearest flow, then one default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5l
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "encode_stream or pinned or release or stream_pipeline or fastq" --timeout 120 --timeout-method thread > $P/pytest_sel.log 2>&1
rc=$?
tail -3 $P/pytest_sel.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 tools/fastq_flow_breakdown.py > $P/fastq_flow.json 2> $P/fastq_flow.err || exit 3
cat $P/fastq_flow.json
timeout -k 10 500 python3 bench.py > $P/bench.log 2> $P/bench.err || exit 3
echo done
