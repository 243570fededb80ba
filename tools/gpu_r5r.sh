# Round 5: the build's counting-sort workgroups (64 / 128 / 256): same-box A/B of config 2's
# pipelined step at W = 1 and rank 0's W = 8 share.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r5r
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 800 python3 tools/ab_libs.py --path headline --variant w128=sctools_amd/libsctools_hip_base.so --variant w64=sctools_amd/libsctools_hip_w64.so --variant w256=sctools_amd/libsctools_hip_w256.so --rounds 3 > $P/ab_sortwgs.jsonl 2> $P/ab_sortwgs.err || exit 3
cat $P/ab_sortwgs.jsonl
echo done
