# Round 5: parallel positional reads of plain FASTQ files (3 workers) with the next piece staged on
# the device: the FASTQ tests, the FASTQ -> nearest flow twice, then the whole GPU suite and one
# default bench line.
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5u
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fastq.py -m gpu -x -v --timeout 120 --timeout-method thread > $P/pytest_fastq.log 2>&1
rc=$?
tail -3 $P/pytest_fastq.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 tools/fastq_flow_breakdown.py > $P/fastq_flow.json 2> $P/fastq_flow.err || exit 3
cat $P/fastq_flow.json
timeout -k 10 300 python3 tools/fastq_flow_breakdown.py > $P/fastq_flow2.json 2> $P/fastq_flow2.err || exit 3
cat $P/fastq_flow2.json
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 500 python3 bench.py > $P/bench.log 2> $P/bench.err || exit 3
echo done
