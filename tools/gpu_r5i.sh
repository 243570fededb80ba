# Round 5: host stream paths on page-locked pool arrays (FASTQ pieces read into a pinned buffer and
# DMAed in place, rows / codes / nearest results in pool blocks): the FASTQ -> nearest flow, the
# whole GPU suite (any failure ends the call), then one default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5i
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/fastq_flow_breakdown.py > $P/fastq_flow.json 2> $P/fastq_flow.err || exit 3
cat $P/fastq_flow.json
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 500 python3 bench.py > $P/bench.log 2> $P/bench.err || exit 3
echo done
