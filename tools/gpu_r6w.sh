# Round 6: the headline with the clock-settle steps (default) against none, interleaved on one box
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6w
mkdir -p $P
export TMPDIR=/tmp
for i in 1 2 3; do
  for st in 30 0; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-paths --no-cpu --settle-steps $st > $P/b_${st}_$i.json 2> $P/err || { tail $P/err; exit 3; }
    python3 -c "
import json; d=json.loads(open('$P/b_${st}_$i.json').read().strip().splitlines()[-1]); print($st, d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['other_kernel']['ms'])"
  done
done
echo done
