"""Multi-rank sharding path (scatter PCM -> per-rank transcribe -> gather ids) with
the gloo backend on CPU, world_size 2 (the bench runs the same code over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Out:
    def __init__(self, tokens):
        self.tokens = tokens


class EchoEngine:
    """Tokens derived from the clip bytes, so misrouted shards are detected."""

    def transcribe_batch(self, clips, cfg, device_pcm=None, offsets=None):
        return [_Out([int(c[0]), int(c[-1]), int(np.int64(c.astype(np.int64).sum()) % 50000)]) for c in clips]

    def sibling(self):
        return EchoEngine()

    def close(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, S, q, lanes=1, steps=1):
    import sys
    sys.path.insert(0, ROOT)
    import osw_path
    osw_path.load()
    from open_speech_amd.distributed import DataParallelTranscriber
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dp = DataParallelTranscriber(EchoEngine(), None, dist=dist, clips_per_rank=B, n_samples=S, ctx=16,
                                     lanes=lanes)
        allpcm = None
        if rank == 0:
            rng = np.random.default_rng(5)
            allpcm = torch.from_numpy(rng.integers(-30000, 30000, size=(world * B, S), dtype=np.int16))
        if steps == 1 and lanes == 1:
            outs, gathered = dp.step(allpcm)
            res = [gathered]
        else:
            res = [g for _, g in dp.run_steps(allpcm, steps)]
        dp.close()
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,lanes,steps", [(2, 1, 1), (2, 2, 3)])
def test_scatter_transcribe_gather_gloo(world, lanes, steps):
    B, S = 3, 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, S, q, lanes, steps)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(5)
    allpcm = rng.integers(-30000, 30000, size=(world * B, S), dtype=np.int16)
    want = EchoEngine().transcribe_batch(list(allpcm), None)
    assert got == [[w.tokens for w in want]] * steps


def test_single_rank_path():
    import osw_path
    osw_path.load()
    from open_speech_amd.distributed import DataParallelTranscriber
    dp = DataParallelTranscriber(EchoEngine(), None, dist=None, clips_per_rank=2, n_samples=10, ctx=8)
    pcm = torch.arange(20, dtype=torch.int16).reshape(2, 10)
    outs, g = dp.step(pcm)
    assert g == [[0, 9, 45], [10, 19, 145]]


def test_single_rank_lanes_run_steps():
    import osw_path
    osw_path.load()
    from open_speech_amd.distributed import DataParallelTranscriber
    dp = DataParallelTranscriber(EchoEngine(), None, dist=None, clips_per_rank=2, n_samples=10, ctx=8, lanes=2)
    assert len(dp.lanes) == 2 and len(dp.shards) == 3
    pcm = torch.arange(20, dtype=torch.int16).reshape(2, 10)
    res = dp.run_steps(pcm, 5)
    dp.close()
    assert [g for _, g in res] == [[[0, 9, 45], [10, 19, 145]]] * 5


class SleepyEngine(EchoEngine):
    """Rank r takes (r + 1) * 40 ms per step and decodes r + 1 tokens per clip."""

    def __init__(self, rank):
        self.rank = rank

    def transcribe_batch(self, clips, cfg, device_pcm=None, offsets=None):
        import time
        time.sleep(0.04 * (self.rank + 1))
        return [_Out(list(range(self.rank + 1))) for _ in clips]

    def sibling(self):
        return SleepyEngine(self.rank)


def _bench_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import osw_path
    osw_path.load()
    import bench
    from open_speech_amd.distributed import DataParallelTranscriber
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B, S, k = 3, 100, 4
        dp = DataParallelTranscriber(SleepyEngine(rank), None, dist=dist, clips_per_rank=B, n_samples=S, ctx=8)
        allpcm = torch.zeros((world * B, S), dtype=torch.int16) if rank == 0 else None
        el, ntok, res = bench.timed_steps(dp, allpcm, k, dist, torch.device("cpu"))
        q.put((rank, el, ntok, len(res)))
    finally:
        dist.destroy_process_group()


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                               "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p, [json.loads(ln) for ln in lines]


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` without a torchrun environment starts the two ranks itself
    (BASELINE configs[3]'s launch): one JSON line, from rank 0, with n_gpus 2, the
    global batch of both ranks, and the slow rank's time (max over ranks: rank 1 takes
    80 ms per step in the stand-in)."""
    p, lines = _run_bench(["--gpus", "2", "--standin", "--batch", "3", "--steps", "3", "--warmup", "1"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1, p.stdout
    ln = lines[0]
    assert ln["n_gpus"] == 2
    assert ln["config"]["global_batch"] == 6 and ln["config"]["parallelism"] == "dp2"
    assert ln["ms_per_step"] >= 80.0
    assert ln["tokens_per_clip"] == 1.5            # rank 0 decodes 1 token per clip, rank 1 decodes 2
    assert abs(ln["value"] - 6 * 3 * 30.0 / (ln["ms_per_step"] * 3 / 1e3)) / ln["value"] < 0.01


def test_bench_world_size_mismatch_exits_nonzero():
    """Under a launcher whose WORLD_SIZE disagrees with --gpus the bench refuses to run
    rather than measure a different number of GPUs than it reports."""
    p, lines = _run_bench(["--gpus", "4", "--standin"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"},
                          timeout=120)
    assert p.returncode != 0 and not lines
    assert "WORLD_SIZE=2" in p.stderr


def test_bench_accounting_gloo():
    """bench.py's timed region over ranks: the time is the MAX over ranks (the slow rank
    sets it) and tokens are summed over ranks, so `value` = all ranks' audio / that time."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, el0, n0, k0), (_, el1, n1, k1) = got
    assert el0 == el1                      # every rank reports the same (max) time
    assert el0 >= 4 * 0.04 * 2             # at least the slow rank's 4 steps x 80 ms
    assert n0 == n1 == 4 * 3 * (1 + 2)     # tokens summed over both ranks
    assert k0 == k1 == 4
