# Round 5: the 14-bit column probe without global atomics for large sets: the whole GPU suite (the
# layout decisions at every column width), then a same-box A/B of the drop-in summary call.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5q
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $P/pytest_gpu.log 2>&1
rc=$?
tail -3 $P/pytest_gpu.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 python3 tools/ab_libs.py --path dropin --variant base=sctools_amd/libsctools_hip_base.so --variant hist= --rounds 4 > $P/ab_probe.jsonl 2> $P/ab_probe.err || exit 3
tail -1 $P/ab_probe.jsonl
echo done
