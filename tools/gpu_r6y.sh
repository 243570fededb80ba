# Round 6: FASTQ count pass with 2 / 4 tiles per workgroup (all loads issued first): the FASTQ GPU
# tests on each variant library, then the fastq path A/B against HEAD's library
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6y
mkdir -p $P
export TMPDIR=/tmp
for v in tpw2 tpw4; do
  SCTOOLS_HIP_LIB=$PWD/sctools_amd/libsctools_hip_$v.so timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 \
    --timeout-method thread -k "fastq or ingest or embedded" > $P/pytest_$v.log 2>&1 || { tail -30 $P/pytest_$v.log; exit 3; }
  echo $v $(tail -1 $P/pytest_$v.log)
done
timeout -k 10 600 python3 tools/ab_libs.py --path fastq --rounds 3 --variant base=sctools_amd/libsctools_hip_base.so \
  --variant tpw2=sctools_amd/libsctools_hip_tpw2.so --variant tpw4=sctools_amd/libsctools_hip_tpw4.so > $P/ab.jsonl 2> $P/ab.err || { tail $P/ab.err; exit 3; }
tail -1 $P/ab.jsonl
echo done
