"""Debug helper (GPU): multi-rank run with per-merge recount checks on small corpora."""
import sys, os
sys.path.insert(0, 'tests'); sys.path.insert(0, 'zig-bpe_amd'); sys.path.insert(0, 'oracle')
from dist_worker import run, train_worker
if __name__ != '__main__':
    raise SystemExit
for case in [dict(kind="runs", seed=62, n=60000, vocab=400, options={"debug_checks": 1}),
             dict(kind="runs", seed=65, n=3000, vocab=400, options={"debug_checks": 1})]:
    for world in (2, 3):
        try:
            out = run(train_worker, world, case)
            print(case['kind'], case['n'], world, 'ok', len(out[0][1]))
        except Exception as e:
            print(case['kind'], case['n'], world, 'FAIL', str(e)[-1500:])
