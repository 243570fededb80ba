# Round 6: rank 0's W = 8 share of the headline step, emulated on one GPU, plain and under a trace
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6p
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/w8_share.py 8 40 > $P/plain.json 2> $P/plain.err || { tail $P/plain.err; exit 3; }
cat $P/plain.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 tools/w8_share.py 8 40 > $P/trace.log 2>&1 || exit 3
tail -1 $P/trace.log
echo done
