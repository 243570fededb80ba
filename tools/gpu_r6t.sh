# Round 6: kernel trace of the emulated W = 8 share with the build in line on the main stream
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6t
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $P/trace -o run --output-format csv -- python3 tools/w8_share.py 8 40 main > $P/trace.log 2>&1 || exit 3
grep '^{' $P/trace.log
echo done
