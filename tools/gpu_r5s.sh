# Round 5: seed columns to lanes by group count (a stable three-class partition per block): the
# SPECTRAL parity tests (both column widths, config 5 bin for bin), then same-box A/Bs of config 5's
# all-pairs path and config 2's pipelined step against the previous library.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5s
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -k "spectral or allpairs or summar or sharded or multirank or config3" --timeout 240 --timeout-method thread > $P/pytest_sel.log 2>&1
rc=$?
tail -3 $P/pytest_sel.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 500 python3 tools/ab_libs.py --path config5_allpairs --variant base=sctools_amd/libsctools_hip_base.so --variant cls= --rounds 3 > $P/ab_cls5.jsonl 2> $P/ab_cls5.err || exit 3
tail -1 $P/ab_cls5.jsonl
timeout -k 10 500 python3 tools/ab_libs.py --path headline --variant base=sctools_amd/libsctools_hip_base.so --variant cls= --rounds 3 > $P/ab_cls2.jsonl 2> $P/ab_cls2.err || exit 3
tail -1 $P/ab_cls2.jsonl
echo done
