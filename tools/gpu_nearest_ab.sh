# Nearest-whitelist key filter A/B: nearest parity tests, then config 4 (100M queries) with
# the filter (default) and without (SCT_NEAREST_FILTER=0), alternately.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -m gpu -k "nearest" > gpurun_out/pytest_nearest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
A="--reads 0 --stream-reads 0 --fastq-records 0 --skip-allpairs5"
for i in 1 2; do
  echo "{\"filter\": 1, \"r\": $(timeout -k 10 200 python -u tools/bench_paths.py $A)}" >> gpurun_out/nearest_ab.jsonl || exit $?
  echo "{\"filter\": 0, \"r\": $(SCT_NEAREST_FILTER=0 timeout -k 10 200 python -u tools/bench_paths.py $A)}" >> gpurun_out/nearest_ab.jsonl || exit $?
done
exit 0
