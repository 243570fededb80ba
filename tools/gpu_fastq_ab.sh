# FASTQ extraction A/B: FASTQ + encode tests, then the 20M-record extraction timed with the
# current library and with SCTOOLS_HIP_LIB=$OLD_LIB alternately.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "fastq or encode" > gpurun_out/pytest_fastq.log 2>&1 || exit $?
A="--reads 0 --stream-reads 0 --queries 0 --skip-allpairs5"
for i in 1 2; do
  timeout -k 10 120 python -u tools/bench_paths.py $A >> gpurun_out/fastq_new.jsonl 2>>gpurun_out/fastq_ab.err || exit $?
  SCTOOLS_HIP_LIB=$PWD/${OLD_LIB:-sctools_amd/libsctools_hip_old.so} timeout -k 10 120 python -u tools/bench_paths.py $A >> gpurun_out/fastq_old.jsonl 2>>gpurun_out/fastq_ab.err || exit $?
done
exit 0
