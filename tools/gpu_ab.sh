set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_allpairs.py --rounds 7 --variants ${AB_VARIANTS:-"unroll=2" "unroll=1"} > gpurun_out/ab.json 2> gpurun_out/ab.err
