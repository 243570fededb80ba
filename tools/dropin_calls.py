"""Five default-policy drop-in calls (config 2 dict) after one warm call: a target for
`rocprofv3 --hip-trace --stats` (which runtime calls the workspace-freeing policy adds)."""
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from sctools_amd import _lib, barcode, synthetic  # noqa: E402

n, L, seed = synthetic.CONFIGS[2]
codes = synthetic.whitelist_codes(n, L, seed)
b = barcode.Barcodes(dict.fromkeys((int(c) for c in codes), 1), L)
keep = len(sys.argv) > 1 and sys.argv[1] == "keep"
_lib.keep_workspace(keep)
r = b.summarize_hamming_distances()
for _ in range(5):
    assert b.summarize_hamming_distances() == r
print("ok", keep)
