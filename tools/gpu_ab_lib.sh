# One GPU call: same-box A/B of two builds of the library (SCTOOLS_HIP_LIB), alternating
# processes: ${AB_CMD} (default: the FASTQ path of tools/bench_paths.py) run ${AB_ROUNDS:-3} times
# per build; then the FASTQ tests on the current build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD=${AB_CMD:-"python -u tools/bench_paths.py --reads 0 --stream-reads 0 --queries 0 --skip-allpairs5"}
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu -k "${PYTEST_K:-fastq}" > gpurun_out/pytest_ablib.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/ab_lib.jsonl
for r in $(seq ${AB_ROUNDS:-3}); do
  for lib in sctools_amd/libsctools_hip_prev.so sctools_amd/libsctools_hip.so; do
    echo "{\"lib\": \"$lib\", \"round\": $r}" >> gpurun_out/ab_lib.jsonl
    SCTOOLS_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 $CMD >> gpurun_out/ab_lib.jsonl 2>> gpurun_out/ab_lib.err || exit $?
  done
done
