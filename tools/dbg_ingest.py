import sys; sys.path.insert(0, "/root/repo")
import numpy as np, torch
from sctools_amd import _lib
from oracle import oracle as O
rng = np.random.default_rng(12)
lines = [bytes(rng.choice(list(b"ACGTacgt"), size=int(rng.integers(1, 40))).tolist()) + b"\n" for _ in range(5000)]
lines[10] = b"\n"; lines[4999] = lines[4999][:-1]
data = b"".join(lines)
for words in (1, 2):
    codes, starts, lens, flags = _lib.whitelist_encode(data, 2) if words == 2 else (None,)*4
    if codes is None: continue
    want_st, pos = [], 0
    for ln in lines: want_st.append(pos); pos += len(ln)
    want_len = [len(l) - 1 for l in lines]
    print("n", len(starts), len(lines), "words", codes.shape)
    bad = [i for i in range(len(lines)) if starts[i] != want_st[i] or lens[i] != want_len[i]]
    print("span mismatches", len(bad), bad[:5])
    if bad:
        i = bad[0]; print(i, starts[i-2:i+3], want_st[i-2:i+3], lens[i-2:i+3], want_len[i-2:i+3])
    w = [O.two_bit_encode(l[:-1]) if l.endswith(b"\n") else O.two_bit_encode(l[:-1]) for l in lines]
    got = _lib.limbs_to_ints(codes)
    cb = [i for i in range(len(lines)) if got[i] != w[i]]
    print("code mismatches", len(cb), cb[:5], [ (lens[i], flags[i]) for i in cb[:5]])
