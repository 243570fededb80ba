# Round 6: the driver's bench command on the final tree (bench line assembly check)
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r6x
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.log 2> $P/bench.err || { tail $P/bench.err; exit 3; }
python3 -c "
import json; d=json.loads(open('$P/bench.log').read().strip().splitlines()[-1])
r=d['roofline']; print('ms_per_step', d['ms_per_step'], 'frac', r['frac'], 'kernel_ms', r['kernel_ms'])
print(json.dumps(r.get('rocprof') or r.get('kernels', {}).get('tile', {}).get('rocprof'))[:600])"
echo done
