"""Run one bench.py side path on cuda:0 and print its JSON (for rocprofv3 traces of a path).
  python tools/run_path.py whitelist|fastq|config4|config5_encode [reps]"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402

name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
fn = {"whitelist": lambda: bench.path_whitelist(dev, reps, 5000.0),
      "fastq": lambda: bench.path_fastq(dev, reps, 5000.0),
      "config4": lambda: bench.path_config4(dev, reps, 5000.0, 16),
      "config5_encode": lambda: bench.path_config5_encode(dev, reps, 5000.0)}[name]
print(json.dumps(fn()))
