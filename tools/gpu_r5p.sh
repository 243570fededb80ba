# Round 5: whitelist ingest without the flag memset (a generation per call) and with a resident-slot
# count grid: the ingest tests, then a same-box A/B against the previous library.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5p
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "whitelist or lines or ingest" --timeout 120 --timeout-method thread > $P/pytest_sel.log 2>&1
rc=$?
tail -3 $P/pytest_sel.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 python3 tools/ab_libs.py --path whitelist --variant base=sctools_amd/libsctools_hip_base.so --variant gen= --rounds 4 > $P/ab_wl_gen.jsonl 2> $P/ab_wl_gen.err || exit 3
tail -1 $P/ab_wl_gen.jsonl
echo done
