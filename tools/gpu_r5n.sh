# Round 5: base_frequency grid A/B (1,024 workgroups at >= 8 codes per lane vs 512 at >= 32 vs 256
# at >= 64), the whitelist path (which also times the ingest) in interleaved rounds.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5n
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_libs.py --path whitelist --variant base=sctools_amd/libsctools_hip_base.so --variant g512= --variant g256=sctools_amd/libsctools_hip_v256.so --rounds 3 > $P/ab_basefreq.jsonl 2> $P/ab_basefreq.err || exit 3
tail -2 $P/ab_basefreq.jsonl
echo done
