# Round 5: WhitelistCorrector (one device index, host batches): its tests, the FASTQ -> nearest
# flow, then the whole GPU suite (any failure ends the call).
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5m
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "corrector" --timeout 120 --timeout-method thread > $P/pytest_sel.log 2>&1
rc=$?
tail -3 $P/pytest_sel.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python3 tools/fastq_flow_breakdown.py > $P/fastq_flow.json 2> $P/fastq_flow.err || exit 3
cat $P/fastq_flow.json
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -eq 0 ] || exit 3
echo done
