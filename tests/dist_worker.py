"""Worker processes for the multi-rank tests (spawned, one per rank; gloo on 127.0.0.1)."""
import ctypes
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))


def _init(rank, world, port):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    return dist


def collective_worker(rank, world, port, q):
    """CPU: exercise zbpe.torch_collective (the host collective the GPU engine calls)."""
    try:
        import numpy as np
        import zbpe

        dist = _init(rank, world, port)
        cb = zbpe.torch_collective(rank, world)
        a = np.array([rank + 1, 10 * rank, 0xFFFFFFFF - rank], dtype=np.uint32)
        assert cb(None, 0, a.ctypes.data, 3) == 0
        m = np.array([5 + rank, 7 - rank, 123], dtype=np.uint32)
        assert cb(None, 1, m.ctypes.data, 3) == 0
        g = np.zeros(4 * world, dtype=np.uint8)
        g[4 * rank:4 * rank + 4] = [rank, rank + 1, rank + 2, 200]
        assert cb(None, 2, g.ctypes.data, 4) == 0
        q.put((rank, a.tolist(), m.tolist(), g.tolist()))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "ERROR", traceback.format_exc()))


def train_worker(rank, world, port, q, case):
    """GPU: `world` ranks share cuda:0, collectives through gloo; rank 0 reports the merges."""
    try:
        import zbpe

        dist = _init(rank, world, port)
        if "text" in case:
            text = case["text"]
        elif "parts" in case:
            text = b"".join(zbpe.synth_corpus(k, s, n) for k, s, n in case["parts"])
        else:
            text = zbpe.synth_corpus(case["kind"], case["seed"], case["n"])
        e = zbpe.Engine(0, rank=rank, world=world, collective=zbpe.torch_collective(rank, world))
        for k, v in case.get("options", {}).items():
            e.set_option(k, v)
        e.upload(text)
        del text
        m, c, st = e.train_resident(case["vocab"])
        q.put((rank, m.tolist(), c.tolist(), st.as_dict(), e.compaction_log().tolist()))
        e.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "ERROR", traceback.format_exc()))


def run(target, world, *args, timeout=600):
    import multiprocessing as mp
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(world):
            item = q.get(timeout=timeout)
            out[item[0]] = item
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r, item in out.items():
        if item[1] == "ERROR":
            raise RuntimeError(f"rank {r} failed:\n{item[2]}")
    return out


def big_worker(rank, world, port, q, case):
    """GPU: a corpus past 2^32 bytes sharded over `world` ranks on cuda:0 (gloo collectives); saves this
    rank's token stream before the last merge to case["dir"], then trains case["vocab"] - 256 merges."""
    try:
        import numpy as np
        import zbpe

        dist = _init(rank, world, port)
        text = zbpe.synth_corpus(case["kind"], case["seed"], case["n"], threads=8)
        e = zbpe.Engine(0, rank=rank, world=world, collective=zbpe.torch_collective(rank, world))
        e.upload(text)
        del text
        e.train_resident(case["vocab"] - 1)  # the stream before the last merge, for the oracle's iteration
        np.save(os.path.join(case["dir"], f"tok{rank}.npy"), e.tokens())
        m, c, st = e.train_resident(case["vocab"])
        q.put((rank, m.tolist(), c.tolist(), st.as_dict()))
        e.close()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "ERROR", traceback.format_exc()))


def bench_setup_worker(rank, world, port, q, case):
    """CPU: bench.py's N>1 engine set-up (make_engine) over a real gloo group with a stand-in zbpe
    module: the unique id rank 0 makes reaches every rank, each rank gets its GPU and rank; an RCCL
    init failure falls back to host collectives."""
    try:
        import types

        sys.path.insert(0, ROOT)
        import bench

        dist = _init(rank, world, port)
        made = []

        class ZbpeError(Exception):
            pass

        class Engine:
            def __init__(self, device=0, rank=0, world=1, unique_id=None, collective=None):
                if unique_id is not None and case.get("rccl_fails"):
                    raise ZbpeError("ncclCommInitRank failed")
                made.append(dict(device=device, rank=rank, world=world, unique_id=unique_id,
                                 collective=collective is not None))

        fake = types.SimpleNamespace(Engine=Engine, ZbpeError=ZbpeError, comm_unique_id=lambda: b"uid-of-rank-0" + bytes(115),
                                     torch_collective=lambda r, w: ("collective", r, w))
        eng, backend = bench.make_engine(fake, case.get("share_gpu", False), rank, world, rank, dist)
        q.put((rank, made, backend))
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "ERROR", traceback.format_exc()))
