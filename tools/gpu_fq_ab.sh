# FASTQ extraction A/B: FASTQ tests on the current library, then tools/fq_experiment.py
# (index and extraction times, 20M records): current library (extract2), the same library
# with SCT_FASTQ_EXTRACT=1 (extract_kernel), and $OLD_LIB -- or, with AB_ENV="VAR=value",
# the current library under that environment.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "fastq or whitelist" > gpurun_out/pytest_fastq.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
for i in 1 2 3; do
  echo "{\"lib\": \"new\", \"t\": $(timeout -k 10 120 python -u tools/fq_experiment.py)}" >> gpurun_out/fq_ab.jsonl || exit $?

  if [ -n "${AB_ENV:-}" ]; then
    echo "{\"lib\": \"$AB_ENV\", \"t\": $(env $AB_ENV timeout -k 10 120 python -u tools/fq_experiment.py)}" >> gpurun_out/fq_ab.jsonl || exit $?
  else
    echo "{\"lib\": \"old\", \"t\": $(SCTOOLS_HIP_LIB=$PWD/${OLD_LIB:-sctools_amd/libsctools_hip_old.so} timeout -k 10 120 python -u tools/fq_experiment.py)}" >> gpurun_out/fq_ab.jsonl || exit $?
  fi
done
exit 0
