# Nearest-whitelist A/B: nearest parity tests under the variant, then config 4 (100M
# queries) with the shipped kernel (SCT_NEAREST_SPEC=0) and the variant (=1), alternately.
# (The all-tables-at-once variant behind SCT_NEAREST_SPEC was removed after this A/B,
# profiles/ab_nearest_spec_r02.jsonl; re-add a switch before reusing the script.)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/nearest_ab.jsonl
SCT_NEAREST_SPEC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -m gpu -k "nearest" > gpurun_out/pytest_nearest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
A="--reads 0 --stream-reads 0 --fastq-records 0 --skip-allpairs5"
for i in 1 2 3; do
  echo "{\"spec\": 0, \"r\": $(SCT_NEAREST_SPEC=0 timeout -k 10 200 python -u tools/bench_paths.py $A)}" >> gpurun_out/nearest_ab.jsonl || exit $?
  echo "{\"spec\": 1, \"r\": $(SCT_NEAREST_SPEC=1 timeout -k 10 200 python -u tools/bench_paths.py $A)}" >> gpurun_out/nearest_ab.jsonl || exit $?
done
exit 0
