"""Data-parallel clip sharding over ranks (one process per GPU, torch.distributed).

Independent 30 s clips are the unit: rank r transcribes clips
[r·B, (r+1)·B).  The only exchanges are the ones the workload really has — the
PCM arrives at rank 0 and is scattered, the token ids are gathered back — and they
run as RCCL collectives over xGMI when the backend is "nccl" (gloo on CPU for the
tests).  int16 PCM travels viewed as int32 (RCCL has no int16 type; the bytes are
unchanged).  No collective touches the compute path itself.
"""
from __future__ import annotations

import numpy as np

N_SAMPLES = 480000


class DataParallelTranscriber:
    def __init__(self, engine, cfg, dist=None, device=None, clips_per_rank: int = 64, n_samples: int = N_SAMPLES,
                 ctx: int = 448):
        import torch

        self.torch = torch
        self.engine, self.cfg, self.dist = engine, cfg, dist
        self.world = dist.get_world_size() if dist else 1
        self.rank = dist.get_rank() if dist else 0
        self.device = device if device is not None else torch.device("cpu")
        self.B, self.S, self.ctx = clips_per_rank, n_samples, ctx
        assert n_samples % 2 == 0, "int16 PCM travels as int32 pairs"
        self.shard = torch.empty((self.B, self.S), dtype=torch.int16, device=self.device)
        self.tok = torch.empty((self.B, ctx + 1), dtype=torch.int32, device=self.device)
        self.offsets = np.arange(self.B + 1, dtype=np.int64) * self.S

    def scatter(self, all_pcm) -> None:
        """all_pcm: [world*B, S] int16 tensor on rank 0 (ignored elsewhere)."""
        if self.world == 1:
            self.shard.copy_(all_pcm)
            return
        chunks = list(all_pcm.view(self.torch.int32).chunk(self.world)) if self.rank == 0 else None
        self.dist.scatter(self.shard.view(self.torch.int32), chunks, src=0)

    def run_local(self):
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)
            return self.engine.transcribe_batch(None, self.cfg, device_pcm=self.shard.data_ptr(),
                                                offsets=self.offsets)
        return self.engine.transcribe_batch(list(self.shard.numpy()), self.cfg)

    def gather(self, outs):
        """Token ids of every clip on rank 0: list of lists in global clip order."""
        t = np.full((self.B, self.ctx + 1), -1, np.int32)
        for i, o in enumerate(outs):
            n = min(len(o.tokens), self.ctx)
            t[i, 0] = n
            t[i, 1:1 + n] = o.tokens[:n]
        self.tok.copy_(self.torch.from_numpy(t))
        if self.world == 1:
            parts = [self.tok]
        else:
            parts = [self.torch.empty_like(self.tok) for _ in range(self.world)] if self.rank == 0 else None
            self.dist.gather(self.tok, parts, dst=0)
        if self.rank != 0:
            return None
        allt = self.torch.cat(parts).cpu().numpy()
        return [row[1:1 + row[0]].tolist() for row in allt]

    def step(self, all_pcm=None):
        self.scatter(all_pcm)
        outs = self.run_local()
        return outs, self.gather(outs)
