# Round 6: nearest bucket scans from the bucket's dword (not its 16-B chunk) and the invalid-digit
# mask folded into the XOR: nearest GPU tests on the working tree, then config 4 A/B vs HEAD
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6s
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "nearest or corrector or whitelist" > $P/pytest.log 2>&1 || { tail -30 $P/pytest.log; exit 3; }
tail -2 $P/pytest.log
timeout -k 10 600 python3 tools/ab_libs.py --path config4 --rounds 3 --variant base=sctools_amd/libsctools_hip_base.so \
  --variant align2=sctools_amd/libsctools_hip_v1.so --variant both=sctools_amd/libsctools_hip_v2.so > $P/ab.jsonl 2> $P/ab.err || { tail $P/ab.err; exit 3; }
tail -4 $P/ab.jsonl
echo done
