"""Run selected bench.py side paths alone: python tools/run_paths.py config4 dropin whitelist fastq
config5_encode config5_allpairs pipeline host_arrays scalar.  One JSON line {name: result}."""
import json
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

import bench  # noqa: E402
from sctools_amd import _lib, synthetic  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
names = sys.argv[1:] or ["config4", "dropin"]
copy = bench.copy_ceiling_gbs(dev)
threads, _ = bench.host_threads()
out = {"copy_ceiling_gbs": copy}
for name in names:
    if name == "config4":
        out[name] = bench._guarded(bench.path_config4, dev, 5, copy, threads)
    elif name == "dropin":
        n, L, seed = synthetic.CONFIGS[2]
        h = _lib.hamming_hist_allpairs(synthetic.whitelist_codes(n, L, seed), 2 * L)
        out[name] = bench._guarded(bench.path_dropin, dev, 7, _lib.summary_from_hist(h))
    elif name == "whitelist":
        out[name] = bench._guarded(bench.path_whitelist, dev, 5, copy)
    elif name == "fastq":
        out[name] = bench._guarded(bench.path_fastq, dev, 5, copy)
    elif name == "pipeline":
        out[name] = bench._guarded(bench.path_pipeline, dev, 5, copy, threads)
    elif name == "config5_encode":
        out[name] = bench._guarded(bench.path_config5_encode, dev, 3, copy)
    elif name == "host_arrays":
        out[name] = bench._guarded(bench.path_host_arrays, dev, bench.pcie_ceiling_gbs(dev))
    elif name == "scalar":
        out[name] = bench._guarded(bench.path_scalar_calls, dev)
    elif name == "config5_allpairs":
        out[name] = bench._guarded(bench.path_config5_allpairs, dev, 5, copy)
    print(json.dumps({name: out.get(name)}), file=sys.stderr, flush=True)
print(json.dumps(out))
