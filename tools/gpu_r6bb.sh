# Round 6: the driver's bench command twice on one box (run-to-run spread of the final line)
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6bb
mkdir -p $P
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench_$i.log 2> $P/bench_$i.err || { tail $P/bench_$i.err; exit 3; }
  python3 -c "
import json; d=json.loads(open('$P/bench_$i.log').read().strip().splitlines()[-1]); print($i, d['ms_per_step'], d['value'], d['roofline']['frac'], d['paths']['config4_nearest']['ms'], d['paths']['fastq_ingest']['ms'])"
done
echo done
