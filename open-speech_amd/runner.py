"""Dynamic batcher + per-GPU lanes behind ``transcribe()``.

The reference calls ``transcribe`` concurrently from the default executor (REST,
``src/main.py:305``), a 4-thread streaming pool (``src/streaming.py:50-52``), a
4-thread Realtime pool (``src/realtime/server.py:33-35``) and Wyoming.  Each call
here becomes a request on its GPU's queue (requests go to the GPU with the fewest
queued + running requests; multi-GPU serving shards independent clips, no
collective).  The lanes of a GPU (contexts sharing one weight copy, one host thread
each) pull batches from that queue: a free lane that finds the queue non-empty waits
for company (at most ``max_wait_ms`` after the oldest request, ``gap_ms`` after the
latest), takes up to ``max_batch`` requests and runs them as one batched seek loop.

Pipelining (``split``): a GPU runs one encoder at a time (a lane's ``engine.encode`` is
synchronous, and it is tracked per GPU).  A free lane that finds requests queued while
another lane of its GPU is encoding waits for that encoder to finish and then takes
everything queued (up to ``max_batch``); when the encoder is idle and no other lane is
running a batch, it takes half of the queue (rounded up) and leaves the rest to the next
free lane, which then waits for this lane's encoder.  Under the streaming pool's closed
loop (4 calls in flight, each session waiting for its call) this turns lock-step batches
of 4 — encode 4, decode 4, nothing overlapping — into staggered batches that take turns
on the encoder while the other batches decode.  With a deep queue (REST load) the
batches are ``max_batch`` anyway.

Continuous batching (``continuous``, the backend's default): every lane drives a decode
session instead (``_SessionLane``, osw_session_*): a request's windows are queued into
the session one at a time as its seek loop advances, free decoder slots are refilled
between chunks of 4 decoder steps (OSW_SESSION_CHUNK), so a request arriving mid-batch starts within a chunk
and a batch costs what its windows' own lengths cost.  Lanes take turns on the encoder
the same way (a session's admission is an encoder call counted on the GPU's queue).

A lane whose GPU fails marks every lane of that GPU dead, moves the GPU's queued
requests to the other GPUs and re-queues there the requests of its batch that are
still unanswered.
"""
from __future__ import annotations

import threading
import time
from collections import deque
from concurrent.futures import Future
from dataclasses import dataclass, field

import numpy as np

from .segments import ClipResult, TranscribeOptions, session_supported, transcribe_clips
from .tokenizer import WhisperTokenizer, get_suppressed_tokens


@dataclass(eq=False)   # identity: a request holds a numpy clip (deque.remove compares)
class _Req:
    pcm: np.ndarray
    opts: TranscribeOptions
    fut: Future
    t_enq: float = field(default=0.0)


class _DevQueue:
    """The request queue of one GPU, shared by its lanes."""

    def __init__(self, device):
        self.device = device
        self.items: deque = deque()
        self.cv = threading.Condition()
        self.lanes: list = []
        self.collecting = False     # a lane is waiting for company for its batch
        self.encoding = 0           # lanes inside engine.encode (synchronous) on this GPU
        self.alive = True
        self.closing = False

    def load(self) -> int:
        return len(self.items) + sum(w.inflight for w in self.lanes)

    def put(self, r: _Req) -> None:
        with self.cv:
            r.t_enq = time.monotonic()
            self.items.append(r)
            self.cv.notify_all()


class _LaneEngine:
    """The lane's engine, with its encoder calls counted on the GPU's queue."""

    def __init__(self, engine, dq: _DevQueue):
        self._e, self._dq = engine, dq

    def __getattr__(self, k):
        return getattr(self._e, k)

    def encode(self, windows):
        with self._dq.cv:
            self._dq.encoding += 1
        try:
            return self._e.encode(windows)
        finally:
            with self._dq.cv:
                self._dq.encoding -= 1
                self._dq.cv.notify_all()


class _Worker(threading.Thread):
    def __init__(self, pool: "BatchRunner", engine, idx: int, dq: _DevQueue):
        super().__init__(daemon=True, name=f"osw-lane-{idx}")
        self.pool, self.engine, self.idx, self.dq = pool, _LaneEngine(engine, dq), idx, dq
        self.alive = True
        self.inflight = 0

    @property
    def q(self) -> _DevQueue:
        return self.dq

    def _take(self) -> list | None:
        """Block until a batch is ready for this lane; None when the runner closes."""
        dq, pool = self.dq, self.pool
        with dq.cv:
            while True:
                if dq.closing or not self.alive:
                    return None
                if dq.items and not dq.collecting:
                    break
                dq.cv.wait()
            dq.collecting = True
            try:
                gap = pool.gap_ms / 1000.0 if pool.gap_ms is not None else None
                cap = self.engine.max_batch
                while len(dq.items) < cap and not dq.closing and self.alive:
                    # wait for company until max_wait after the oldest request, or gap after the
                    # latest one (callers released together by the previous batch arrive within
                    # a fraction of a millisecond; waiting the whole max_wait for a 5th that the
                    # 4-thread streaming pool can never send cost ~4 ms per call)
                    end = dq.items[0].t_enq + pool.max_wait_ms / 1000.0
                    if gap is not None:
                        end = min(end, dq.items[-1].t_enq + gap)
                    left = end - time.monotonic()
                    if left <= 0:
                        break
                    dq.cv.wait(timeout=left)
                if pool.split:
                    # another lane's encoder is running: wait for it (bounded), then take
                    # everything that queued meanwhile
                    end = time.monotonic() + pool.max_pace_ms / 1000.0
                    while dq.encoding and not dq.closing and self.alive:
                        left = end - time.monotonic()
                        if left <= 0:
                            break
                        dq.cv.wait(timeout=left)
                if dq.closing or not self.alive or not dq.items:
                    return None if (dq.closing or not self.alive) else []
                k = min(cap, len(dq.items))
                others_busy = any(w.inflight for w in dq.lanes if w is not self)
                idle_sibling = any(w.alive and not w.inflight for w in dq.lanes if w is not self)
                if pool.split and not others_busy and idle_sibling and not dq.encoding:
                    k = min(k, (len(dq.items) + 1) // 2)
                batch = [dq.items.popleft() for _ in range(k)]
                self.inflight = len(batch)
                return batch
            finally:
                dq.collecting = False
                dq.cv.notify_all()

    def run(self) -> None:
        while True:
            batch = self._take()
            if batch is None:
                return
            if not batch:
                continue
            try:
                self._run_batch(batch)
            except Exception as e:  # noqa: BLE001 - forwarded to callers
                if self.pool.is_device_error(e) and self.pool.fail_device(self):
                    # requests of earlier opts-groups of this batch are already answered
                    for r in batch:
                        if not r.fut.done():
                            self.pool.submit_req(r)
                    self.inflight = 0
                    return
                for r in batch:
                    if not r.fut.done():
                        r.fut.set_exception(e)
            finally:
                with self.dq.cv:
                    self.inflight = 0
                    self.dq.cv.notify_all()

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


class _SessionLane(_Worker):
    """A lane driving one decode session (osw_session_*, ``continuous`` runners).

    Every request's seek loop advances on its own: its first window is queued into the
    lane's session when the request is taken, and each finished window is consumed
    (segments.consume_window) and the clip's next window queued at once, so windows of
    different requests and different seek positions decode side by side and a finished
    window's slot is refilled between chunks of 4 decoder steps instead of waiting for
    the batch's longest window.  A session holds one decode configuration
    (``TranscribeOptions.key()``): a lane admits only requests of its session's key, and
    opens a session for another key once its own has drained.  Requests a session cannot
    hold (segments.session_supported: temperature > 0, max_new_tokens, beam_size > 5)
    run through the batched seek loop of an idle lane.
    """

    def _admit(self, key, room: int, idle: bool):
        """('sess', key, reqs) — requests to add to the session (key: the session's, or a
        new one when idle); ('batch', reqs); None when the runner closes."""
        dq, pool = self.dq, self.pool
        deadline = None     # an idle lane waits for another lane's encoder at most max_pace_ms per call
        with dq.cv:
            while True:
                if not self.alive:
                    return None
                if dq.closing:
                    # admit nothing more; a lane with windows in flight finishes them first
                    return None if idle else ("sess", key, [])
                if dq.items and room > 0:
                    if pool.split and dq.encoding:
                        # another lane's encoder is running: a busy lane keeps decoding, an
                        # idle one waits for that encoder (at most max_pace_ms over this
                        # call) and then takes everything that queued meanwhile — the lanes
                        # take turns on the encoder
                        if not idle:
                            # a busy lane keeps decoding — unless a request has waited
                            # max_pace_ms already (then it is admitted beside the encoder)
                            waited = time.monotonic() - dq.items[0].t_enq
                            if not pool.busy_admit or waited < pool.max_pace_ms / 1000.0:
                                return ("sess", key, [])
                        elif deadline is None:
                            deadline = time.monotonic() + pool.max_pace_ms / 1000.0
                        if idle:
                            left = deadline - time.monotonic()
                            if left > 0:
                                dq.cv.wait(timeout=left)
                                continue
                        # waited max_pace_ms: take requests beside the running encoder
                    if idle:
                        head = dq.items[0]
                        if not session_supported(head.opts):
                            k = head.opts.key()
                            batch = [r for r in dq.items if r.opts.key() == k][:self.engine.max_batch]
                            for r in batch:
                                dq.items.remove(r)
                            self.inflight = len(batch)
                            return ("batch", batch)
                        key = head.opts.key()
                    else:
                        now = time.monotonic()
                        # a request of another key waited max_pace_ms: admit nothing more, so
                        # this session drains and the lane can switch
                        if any(r.opts.key() != key and now - r.t_enq > pool.max_pace_ms / 1000.0
                               for r in dq.items):
                            return ("sess", key, [])
                        # spread_ms: an idle sibling takes what waited less than that (a fresh
                        # session on an idle lane runs beside this one instead of growing it)
                        idle_sibling = any(w.alive and not w.inflight for w in dq.lanes if w is not self)
                        if (pool.spread_ms is not None and idle_sibling
                                and all(now - r.t_enq < pool.spread_ms / 1000.0 for r in dq.items)):
                            return ("sess", key, [])
                    take = [r for r in dq.items if r.opts.key() == key][:room]
                    for r in take:
                        dq.items.remove(r)
                    self.inflight += len(take)
                    if take:
                        dq.cv.notify_all()
                    return ("sess", key, take)
                if not idle:
                    return ("sess", key, [])
                dq.cv.wait()

    def run(self) -> None:
        from .segments import clip_state, consume_window, finish_clip, next_window, session_config
        pool, eng, tok = self.pool, self.engine, self.pool.tokenizer
        flights: dict = {}      # tag -> [req, clip state, window]
        key, is_open, tag = None, False, 0
        added = False           # windows queued since the last admission

        def answer(t, exc=None):
            req, s, w = flights.pop(t)
            if w is not None and is_open:
                try:
                    eng.session_release_clip(t)   # the request's resident log-mel
                except Exception:  # noqa: BLE001 - best effort; session_end frees it anyway
                    pass
            if not req.fut.done():
                if exc is None and s is not None:
                    req.fut.set_result(finish_clip(s, req.opts, tok))
                else:
                    req.fut.set_exception(exc if exc is not None else RuntimeError("request state lost"))

        def queue_window(t):
            req, s, _ = flights[t]
            if s.done:
                answer(t)
                return
            w = next_window(s, req.opts, tok)
            # the request's clip key is its tag: the first window brings the PCM (its log-mel
            # is computed once and stays on the device), later windows only the key
            w.update(tag=t, clip=t, pcm=req.pcm if flights[t][2] is None else None)
            flights[t][2] = w
            eng.session_add([w])
            nonlocal added
            added = True

        while True:
            idle = not flights
            if idle and is_open:
                eng.session_end()
                is_open = False
            got = self._admit(key, eng.max_batch - len(flights), idle)
            if got is None:
                break
            try:
                if got[0] == "batch":
                    try:
                        self._run_batch(got[1])
                    finally:
                        with self.dq.cv:
                            self.inflight = 0
                            self.dq.cv.notify_all()
                    continue
                _, k, reqs = got
                if reqs and not is_open:
                    eng.session_begin(session_config(reqs[0].opts, pool.suppress_for(reqs[0].opts)))
                    key, is_open = k, True
                for r in reqs:
                    tag += 1
                    flights[tag] = [r, None, None]
                    try:
                        flights[tag][1] = clip_state(0, r.pcm, r.opts, tok)
                        queue_window(tag)
                    except Exception as e:  # noqa: BLE001 - this request (its options or window) was refused
                        if pool.is_device_error(e):
                            raise
                        answer(tag, e)
                if not flights:
                    continue
                if added:
                    # admission on its own (the encoder, waited for), counted on the GPU's
                    # queue so that the other lanes take turns with it
                    added = False
                    with self.dq.cv:
                        self.dq.encoding += 1
                    try:
                        eng.session_step(max_chunks=0, refill_min=pool.refill_min)
                    finally:
                        with self.dq.cv:
                            self.dq.encoding -= 1
                            self.dq.cv.notify_all()
                done, _, _ = eng.session_step(max_chunks=1, refill_min=pool.refill_min)
                for t, out in done:
                    req, s, w = flights[t]
                    try:
                        consume_window(s, w, out, req.opts, tok)
                        queue_window(t)
                    except Exception as e:  # noqa: BLE001
                        if pool.is_device_error(e):
                            raise
                        if t in flights:
                            answer(t, e)
                with self.dq.cv:
                    self.inflight = len(flights)
                    self.dq.cv.notify_all()
            except Exception as e:  # noqa: BLE001 - forwarded to callers
                # the requests in flight and the ones taken this round (not all in flights yet)
                reqs = [f[0] for f in flights.values()]
                for r in (got[1] if got[0] == "batch" else got[2]):
                    if not any(r is q for q in reqs):
                        reqs.append(r)
                flights.clear()
                added = False
                if is_open:
                    try:
                        eng.session_end()
                    except Exception:  # noqa: BLE001
                        pass
                    is_open = False
                with self.dq.cv:
                    self.inflight = 0
                    self.dq.cv.notify_all()
                if pool.is_device_error(e) and pool.fail_device(self):
                    for r in reqs:
                        if not r.fut.done():
                            pool.submit_req(r)
                    return
                for r in reqs:
                    if not r.fut.done():
                        r.fut.set_exception(e)
        if is_open:
            try:
                eng.session_end()
            except Exception:  # noqa: BLE001
                pass
        # (closing: the loop above drained the flights.)  A lane marked dead because a
        # sibling lane of its GPU failed hands its unanswered requests to the surviving GPUs
        # (they restart there: a request's answer is only produced at its end)
        for req, _, _ in flights.values():
            if not req.fut.done():
                if not self.alive:
                    pool.submit_req(req)
                else:
                    req.fut.set_exception(RuntimeError("runner closed"))


class BatchRunner:
    def __init__(self, engines: list, tokenizer: WhisperTokenizer, max_wait_ms: float = 5.0,
                 gap_ms: float | None = None, split: bool = True, max_pace_ms: float = 100.0,
                 continuous: bool = False, refill_min: int = 1, spread_ms: float | None = None):
        self.tokenizer = tokenizer
        self.max_wait_ms = max_wait_ms
        self.gap_ms = gap_ms
        self.split = split
        self.max_pace_ms = max_pace_ms
        self.continuous = continuous
        self.refill_min = refill_min
        self.spread_ms = spread_ms
        # a busy session lane admits a request that waited max_pace_ms even while another lane
        # encodes; STT_HIP_BUSY_ADMIT=0: never (the round-5 pacing, for A/B runs)
        import os
        self.busy_admit = os.environ.get("STT_HIP_BUSY_ADMIT", "1") != "0"
        self._sup_cache: dict = {}
        self._lock = threading.Lock()
        self.queues: list[_DevQueue] = []
        by_dev: dict = {}
        self.workers = []
        for i, e in enumerate(engines):
            dev = getattr(e, "device", None)
            key = ("dev", dev) if dev is not None else ("engine", i)
            if key not in by_dev:
                by_dev[key] = _DevQueue(dev)
                self.queues.append(by_dev[key])
            dq = by_dev[key]
            w = (_SessionLane if continuous else _Worker)(self, e, i, dq)
            dq.lanes.append(w)
            self.workers.append(w)
        for w in self.workers:
            w.start()

    def suppress_for(self, opts: TranscribeOptions) -> tuple:
        key = tuple(opts.suppress_tokens)
        if key not in self._sup_cache:
            self._sup_cache[key] = get_suppressed_tokens(self.tokenizer, list(opts.suppress_tokens))
        return self._sup_cache[key]

    @staticmethod
    def is_device_error(e: Exception) -> bool:
        """A fault of the GPU itself (its lanes are failed over).  A refused or invalidated
        stream capture (OSW_ECAPTURE) is not one: the context and the GPU stay usable, so
        only the requests of that call fail."""
        from ._lib import OswCaptureError, OswDeviceError
        if isinstance(e, OswCaptureError):
            return False
        if isinstance(e, OswDeviceError):
            return True
        s = str(e)
        if "capture" in s.lower():
            return False
        return "hipError" in s or "(-100)" in s

    def fail_device(self, failed: _Worker) -> bool:
        """Mark every lane of `failed`'s GPU dead (lanes share the device) and move that
        GPU's queued requests to the survivors.  False when no other GPU is alive (the
        error then goes to the callers)."""
        dq = failed.dq
        with self._lock:
            if not any(q.alive for q in self.queues if q is not dq):
                return False
            dq.alive = False
        with dq.cv:
            for w in dq.lanes:
                w.alive = False
            moved = list(dq.items)
            dq.items.clear()
            dq.cv.notify_all()
        for r in moved:
            if not r.fut.done():
                self.submit_req(r)
        return True

    def submit_req(self, r: _Req) -> None:
        with self._lock:
            live = [q for q in self.queues if q.alive]
            if not live:
                if not r.fut.done():
                    r.fut.set_exception(RuntimeError("no live GPU worker"))
                return
            q = min(live, key=lambda x: x.load())
        q.put(r)

    def submit(self, pcm: np.ndarray, opts: TranscribeOptions) -> Future:
        f: Future = Future()
        self.submit_req(_Req(np.ascontiguousarray(pcm, dtype=np.int16), opts, f))
        return f

    def transcribe(self, pcm: np.ndarray, opts: TranscribeOptions, timeout: float | None = None) -> ClipResult:
        return self.submit(pcm, opts).result(timeout=timeout)

    def close(self) -> None:
        for q in self.queues:
            with q.cv:
                q.closing = True
                q.cv.notify_all()
        # a lane finishes what it is running (a session lane: its windows in flight, each
        # request to its end, as the reference's in-flight WhisperModel.transcribe calls
        # keep their model alive past unload_model)
        for w in self.workers:
            w.join(timeout=300)
        for q in self.queues:
            for r in q.items:
                if not r.fut.done():
                    r.fut.set_exception(RuntimeError("runner closed"))
            q.items.clear()
        for w in self.workers:
            if w.is_alive():
                continue   # (a lane still inside a call keeps its context: never destroyed under it)
            close = getattr(w.engine._e, "close", None)
            if close:
                close()
