"""Stream-form slots read against live tokens for compaction thresholds (the holes streamed):
  python tools/compact_probe.py [den ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
import numpy as np  # noqa: E402
import zbpe  # noqa: E402

text = zbpe.synth_corpus("words_utf8", 0x5EED0004, 1 << 30, threads=16)
for den in [int(x) for x in sys.argv[1:]] or [8]:
    e = zbpe.Engine(0)
    e.set_option("compact_den", den)
    e.set_option("print_runtime", 0)
    e.upload(text)
    m, c, st = e.train_resident(32000)
    L = e.merge_log()
    stream = L[:, 4] == 0
    print(f"den {den}: compactions {st.compactions}, stream launches {int(stream.sum())}, scan_read/alg "
          f"{st.scan_read_bytes / max(1, 2 * L[stream, 2].astype(np.float64).sum()):.4f}, scan_kernel_s {st.scan_kernel_s:.4f}, "
          f"total {st.total_s:.3f}", flush=True)
    e.close()
