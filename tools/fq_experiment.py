import sys, time, json
sys.path.insert(0, '.')
import numpy as np, torch
from sctools_amd import _lib
dev = torch.device('cuda'); s = torch.cuda.current_stream()
n_rec = 20_000_000
g = torch.Generator(device=dev).manual_seed(6)
acgt = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
rec = torch.empty((n_rec, 69), dtype=torch.uint8, device=dev)
rec[:, 0] = ord("@"); rec[:, 1:12] = ord("r"); rec[:, 12] = 10
rec[:, 13:39] = acgt[torch.randint(0, 4, (n_rec, 26), device=dev, generator=g)]
rec[:, 39] = 10; rec[:, 40] = ord("+"); rec[:, 41] = 10; rec[:, 42:68] = ord("F"); rec[:, 68] = 10
buf = rec.reshape(-1); nb = buf.numel()
seqs = torch.empty(n_rec * 24, dtype=torch.uint8, device=dev); quals = torch.empty_like(seqs)
ix = _lib.FastqIndex(buf.data_ptr(), nb, [nb], False, s.cuda_stream)
out = {}
for name, spans, q in (("nospan", [], 0), ("cb_seq", [(0, 16)], 0), ("cb_umi_seq", [(0, 16), (16, 24)], 0), ("all", [(0, 16), (16, 24)], 1)):
    ts = []
    for it in range(6):
        torch.cuda.synchronize(); t = time.perf_counter()
        ix.extract_spans(buf.data_ptr(), spans, seqs.data_ptr(), quals.data_ptr() if q else 0, stream=s.cuda_stream)
        torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    out[name] = round(float(np.median(ts[1:])) * 1e3, 3)
ts = []
for it in range(6):
    torch.cuda.synchronize(); t = time.perf_counter()
    ix2 = _lib.FastqIndex(buf.data_ptr(), nb, [nb], False, s.cuda_stream); ix2.close()
    torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
out["index"] = round(float(np.median(ts[1:])) * 1e3, 3)
print(json.dumps(out))
