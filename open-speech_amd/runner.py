"""Dynamic batcher + per-GPU workers behind ``transcribe()``.

The reference calls ``transcribe`` concurrently from the default executor (REST,
``src/main.py:305``), a 4-thread streaming pool (``src/streaming.py:50-52``), a
4-thread Realtime pool (``src/realtime/server.py:33-35``) and Wyoming.  Each call
here becomes a request on a queue; one worker thread per GPU drains up to
``max_batch`` requests (waiting at most ``max_wait_ms`` for company once the first
arrives, and at most ``gap_ms`` after the latest arrival), runs them as one batched seek loop on its engine, and completes each
caller's future.  Requests are routed to the worker with the shortest queue
(multi-GPU serving: independent clips, no collective).  A worker whose GPU fails
marks every worker of that GPU (its sibling lanes) dead and re-queues the requests
it held that are still unanswered on the workers of the other GPUs.
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass

import numpy as np

from .segments import ClipResult, TranscribeOptions, transcribe_clips
from .tokenizer import WhisperTokenizer, get_suppressed_tokens


@dataclass
class _Req:
    pcm: np.ndarray
    opts: TranscribeOptions
    fut: Future


class _Worker(threading.Thread):
    def __init__(self, pool: "BatchRunner", engine, idx: int):
        super().__init__(daemon=True, name=f"osw-worker-{idx}")
        self.pool, self.engine, self.idx = pool, engine, idx
        self.q: "queue.Queue[_Req | None]" = queue.Queue()
        self.alive = True
        self.inflight = 0

    def load(self) -> int:
        return self.q.qsize() + self.inflight

    def run(self) -> None:
        while True:
            first = self.q.get()
            if first is None:
                return
            batch = [first]
            now = time.monotonic()
            deadline = now + self.pool.max_wait_ms / 1000.0
            gap = self.pool.gap_ms / 1000.0 if self.pool.gap_ms is not None else None
            last = now
            while len(batch) < self.engine.max_batch:
                # wait for company until max_wait after the first request, or gap after the
                # latest one (callers released together by the previous batch arrive within
                # a fraction of a millisecond; waiting the whole max_wait for a 5th that the
                # 4-thread streaming pool can never send cost ~4 ms per call)
                end = deadline if gap is None else min(deadline, last + gap)
                left = end - time.monotonic()
                try:
                    nxt = self.q.get(timeout=max(0.0, left)) if left > 0 else self.q.get_nowait()
                except queue.Empty:
                    break
                if nxt is None:
                    self.q.put(None)
                    break
                batch.append(nxt)
                last = time.monotonic()
            self.inflight = len(batch)
            try:
                self._run_batch(batch)
            except Exception as e:  # noqa: BLE001 - forwarded to callers
                if self.pool.is_device_error(e) and self.pool.fail_device(self):
                    # requests of earlier opts-groups of this batch are already answered
                    for r in batch:
                        if not r.fut.done():
                            self.pool.submit_req(r)
                    return
                for r in batch:
                    if not r.fut.done():
                        r.fut.set_exception(e)
            finally:
                self.inflight = 0

    def _run_batch(self, batch: list) -> None:
        groups: dict = {}
        for r in batch:
            groups.setdefault(r.opts.key(), []).append(r)
        for reqs in groups.values():
            res = transcribe_clips(self.engine, [r.pcm for r in reqs], reqs[0].opts, self.pool.tokenizer,
                                   self.pool.suppress_for(reqs[0].opts))
            for r, out in zip(reqs, res):
                if not r.fut.done():
                    r.fut.set_result(out)


class BatchRunner:
    def __init__(self, engines: list, tokenizer: WhisperTokenizer, max_wait_ms: float = 5.0,
                 gap_ms: float | None = None):
        self.tokenizer = tokenizer
        self.max_wait_ms = max_wait_ms
        self.gap_ms = gap_ms
        self._sup_cache: dict = {}
        self._lock = threading.Lock()
        self.workers = [_Worker(self, e, i) for i, e in enumerate(engines)]
        for w in self.workers:
            w.start()

    def suppress_for(self, opts: TranscribeOptions) -> tuple:
        key = tuple(opts.suppress_tokens)
        if key not in self._sup_cache:
            self._sup_cache[key] = get_suppressed_tokens(self.tokenizer, list(opts.suppress_tokens))
        return self._sup_cache[key]

    @staticmethod
    def is_device_error(e: Exception) -> bool:
        from ._lib import OswDeviceError
        if isinstance(e, OswDeviceError):
            return True
        s = str(e)
        return "hipError" in s or "(-100)" in s

    @staticmethod
    def _device_of(w: _Worker):
        return getattr(w.engine, "device", None)

    def fail_device(self, failed: _Worker) -> bool:
        """Mark every worker on `failed`'s GPU dead (lanes share the device) and move their
        queued requests to the survivors.  False when no other GPU's worker is alive
        (the error then goes to the callers)."""
        dev = self._device_of(failed)
        same = [w for w in self.workers if w is failed or (dev is not None and self._device_of(w) == dev)]
        with self._lock:
            if not any(w.alive and w not in same for w in self.workers):
                return False
            for w in same:
                w.alive = False
        for w in same:
            self.drain_dead(w)
            if w is not failed:
                w.q.put(None)   # its thread exits after the batch it may be running
        return True

    def submit_req(self, r: _Req, exclude=None) -> None:
        with self._lock:
            live = [w for w in self.workers if w.alive and w is not exclude]
            if not live:
                if not r.fut.done():
                    r.fut.set_exception(RuntimeError("no live GPU worker"))
                return
            w = min(live, key=lambda x: x.load())
            w.q.put(r)

    def drain_dead(self, dead: _Worker) -> None:
        while True:
            try:
                r = dead.q.get_nowait()
            except queue.Empty:
                return
            if r is not None and not r.fut.done():
                self.submit_req(r, exclude=dead)

    def submit(self, pcm: np.ndarray, opts: TranscribeOptions) -> Future:
        f: Future = Future()
        self.submit_req(_Req(np.ascontiguousarray(pcm, dtype=np.int16), opts, f))
        return f

    def transcribe(self, pcm: np.ndarray, opts: TranscribeOptions, timeout: float | None = None) -> ClipResult:
        return self.submit(pcm, opts).result(timeout=timeout)

    def close(self) -> None:
        for w in self.workers:
            if w.is_alive():
                w.q.put(None)
        for w in self.workers:
            w.join(timeout=30)
        for w in self.workers:
            close = getattr(w.engine, "close", None)
            if close:
                close()
