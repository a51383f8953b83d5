"""Debug helper (GPU): bisect the merge prefix at which device encode diverges from the oracle."""
import sys, os
sys.path.insert(0, 'zig-bpe_amd'); sys.path.insert(0, 'oracle')
import numpy as np, zbpe, oracle as O
e = zbpe.Engine(0)
text = zbpe.synth_corpus("words_utf8", 41, 400000)
m, _, _ = e.train(text, 900)
def same(k):
    return np.array_equal(e.encode(m[:k], text), O.encode(m[:k], text))
lo, hi = 0, len(m)
print("full same:", same(hi))
while hi - lo > 1:
    mid = (lo + hi) // 2
    if same(mid): lo = mid
    else: hi = mid
print("first bad prefix", hi, "merge", m[hi-1].tolist())
g = e.encode(m[:hi], text); o = O.encode(m[:hi], text)
print(len(g), len(o))
d = np.nonzero(g[:min(len(g),len(o))] != o[:min(len(g),len(o))])[0]
print("ndiff", len(d), d[:10])
if len(d):
    i = d[0]; print("gpu", g[max(0,i-5):i+6].tolist()); print("ora", o[max(0,i-5):i+6].tolist())
g1 = e.encode(m[:hi-1], text); print("prefix-1 equal:", np.array_equal(g1, O.encode(m[:hi-1], text)))
print(g1[max(0,d[0]-5):d[0]+8].tolist() if len(d) else '')
