# Round 6: FASTQ range kernel with the span table (and the output pointers) staged in LDS instead
# of kernel-argument SGPRs (55 -> 48 / 28 SGPR spills): FASTQ GPU tests per variant, then the A/B
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6z
mkdir -p $P
export TMPDIR=/tmp
for v in ldsp ldsto; do
  SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_$v.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 \
    --timeout-method thread -k "fastq or ingest or embedded" > $P/pytest_$v.log 2>&1 || { tail -30 $P/pytest_$v.log; exit 3; }
  echo $v $(tail -1 $P/pytest_$v.log)
done
timeout -k 10 600 python3 tools/ab_libs.py --path fastq --rounds 3 --variant base=sctools_amd/libsctools_hip_base.so \
  --variant ldsp=sctools_amd/libsctools_hip_ldsp.so --variant ldsto=sctools_amd/libsctools_hip_ldsto.so > $P/ab.jsonl 2> $P/ab.err || { tail $P/ab.err; exit 3; }
tail -1 $P/ab.jsonl
echo done
