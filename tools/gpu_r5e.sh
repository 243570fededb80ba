# Round 5 (one box): the whole GPU suite; the one-read whitelist ingest A/B (round-4 library / one
# read / one read off); then one default bench line (with the host-resident stream paths).
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5e
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -le 1 ] || exit 3
timeout -k 10 300 python3 tools/ab_libs.py --path whitelist --variant base=sctools_amd/libsctools_hip_base.so \
  --variant spec= --variant nospec=:ingest_spec=0 --rounds 3 > $P/ab_whitelist.jsonl 2> $P/ab_whitelist.err || exit 3
tail -1 $P/ab_whitelist.jsonl
timeout -k 10 400 python3 bench.py > $P/bench.log 2> $P/bench.err || exit 3
echo done
