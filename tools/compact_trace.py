"""Where compactions happen (slot count drops) in a C4 train, per compaction threshold:
  python tools/compact_trace.py [den ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
import numpy as np  # noqa: E402
import zbpe  # noqa: E402

text = zbpe.synth_corpus("words_utf8", 0x5EED0004, 1 << 30, threads=16)
C = {k: i for i, k in enumerate(zbpe.TRACE_COLUMNS)}
for den in [int(x) for x in sys.argv[1:]] or [8]:
    e = zbpe.Engine(0)
    e.set_option("compact_den", den)
    e.set_option("trace", 1)
    e.set_option("print_runtime", 0)
    e.upload(text)
    m, c, st = e.train_resident(32000)
    T = e.trace()
    slots, live = T[:, C["slots"]], T[:, C["live"]]
    drops = np.nonzero(np.diff(slots) < 0)[0] + 1
    L = e.merge_log()
    first_list = int(np.argmax(L[:, 4] != 0))
    print(f"den {den}: compactions {st.compactions} at merges {drops.tolist()[:12]}; first list scan at {first_list}; "
          f"holes/slots before them {[round(float(1 - live[d - 1] / slots[d - 1]), 4) for d in drops[:12]]}", flush=True)
    e.close()
