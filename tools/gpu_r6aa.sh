# Round 6: bench.py's multi-rank path (run_rank at world 2 and 4, gloo, ranks sharing the box's one
# GPU) with the clock-settle steps: the line forms and the histograms agree
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6aa
mkdir -p $P
export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n \
    bench.py --gpus $n --backend gloo --allow-shared-gpu --steps 5 --warmup 2 --no-paths --no-cpu > $P/b$n.log 2> $P/b$n.err || { tail -20 $P/b$n.err; exit 3; }
  python3 -c "
import json; d=json.loads([l for l in open('$P/b$n.log') if l.startswith('{')][-1]); print($n, d['n_gpus'], d['settle_steps'], d['ms_per_step'], d['config'].get('parallelism'), str(d.get('summary'))[:200])"
done
echo done
