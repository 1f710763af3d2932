"""Host logic of the drop-in backend (no GPU): STTBackend surface, lifecycle dicts,
response shapes, the faster-whisper seek loop / segment split, batching under
concurrency, and WAV ingest.  The engine is a scripted stand-in with the
WhisperEngine interface (the same seam style as the reference's FakeSTTBackend,
tests/test_model_manager.py:14-47)."""
import asyncio
import io
import threading
import time
import wave

import numpy as np
import pytest

from open_speech_amd import dims as D
from open_speech_amd import synth
from open_speech_amd.audio import decode_audio_bytes, pcm16_from_wav
from open_speech_amd.backend import HipWhisperBackend, install
from open_speech_amd.engine import WindowOutput
from open_speech_amd.segments import split_segments_by_timestamps, to_srt, to_vtt

ST = D.SpecialTokens.for_vocab(51866)
TB = ST.timestamp_begin


class FakeEngine:
    """Scripted engine: `script(window, call_index, prefix, language) -> WindowOutput`."""

    def __init__(self, dims, gpu, max_batch, script=None):
        self.dims, self.gpu, self.max_batch = dims, gpu, max_batch
        self.script = script or (lambda w, i, p, l: WindowOutput([TB, 1000, 1001, TB + 100], -1.0, 0.01, ST.first_lang))
        self.calls, self.batches, self.closed = [], [], False
        self._nf = []
        self._wins = []
        self.lock = threading.Lock()

    def init_random(self, seed=0):
        pass

    def load_weights(self, w):
        pass

    def log_mel(self, clips):
        self._nf = [(len(c) + 160) // 160 for c in clips]
        return self._nf

    def encode(self, wins):
        self._wins = list(wins)

    def decode(self, n, cfg, prefix=None, dump_steps=0, languages=None):
        assert n == len(self._wins)
        self.batches.append(n)
        outs = []
        for k, w in enumerate(self._wins):
            lang = None if languages is None else languages[k]
            self.calls.append((w, prefix[k] if prefix else [], lang, cfg.task))
            outs.append(self.script(w, len(self.calls) - 1, prefix[k] if prefix else [], lang))
        return outs

    # decode sessions (runner._SessionLane): a window finishes 1-3 steps after admission
    def session_begin(self, cfg):
        assert getattr(self, "_sess", None) is None
        self._sess = dict(cfg=cfg, q=[], active=[])
        self.sessions = getattr(self, "sessions", 0) + 1

    def session_add(self, wins):
        clips = self._sess.setdefault("clips", {})
        for w in wins:
            if w.get("pcm") is not None and w.get("clip") not in clips:
                clips[w.get("clip")] = len(w["pcm"])
            n = clips[w["clip"]] if w.get("clip") is not None else len(w["pcm"])
            if w["seek"] >= n // 160 + 1:
                raise ValueError("window seek out of range")
            self._sess["q"].append(w)

    def session_release_clip(self, clip):
        self._sess.get("clips", {}).pop(clip, None)
        self.released = getattr(self, "released", 0) + 1

    def session_step(self, max_chunks=1, refill_min=1):
        time.sleep(getattr(self, "step_sleep", 0.0))
        s = self._sess
        while s["q"] and len(s["active"]) < self.max_batch:
            w = s["q"].pop(0)
            win = (0, w["seek"], w["segment_size"])
            prefix = list(w.get("prefix") or [])
            lang = w.get("language_token")
            self.calls.append((win, prefix, lang, s["cfg"].task))
            out = self.script(win, len(self.calls) - 1, prefix, lang)
            s["active"].append([1 + len(self.calls) % 3, w["tag"], out])
        if max_chunks == 0:   # admission only
            return [], len(s["active"]), len(s["q"])
        self.batches.append(len(s["active"]))
        done = []
        for a in s["active"]:
            a[0] -= 1
            if a[0] == 0:
                done.append((a[1], a[2]))
        s["active"] = [a for a in s["active"] if a[0] > 0]
        return done, len(s["active"]), len(s["q"])

    def session_end(self):
        self._sess = None

    def close(self):
        self.closed = True


def make_backend(script=None, holder=None):
    def factory(dims, gpu, mb):
        e = FakeEngine(dims, gpu, mb, script)
        if holder is not None:
            holder.append(e)
        return e
    return HipWhisperBackend(engine_factory=factory)


def wav(seconds=30.0, i=0):
    return synth.to_wav_bytes(synth.chirp_clip(i, seconds))


MID = "random:micro-test"


# --------------------------------------------------------------------------- segment split
def test_split_pairs_single_ending():
    toks = [TB, 10, 11, TB + 50, TB + 50, 12, TB + 120]
    segs, seek, single = split_segments_by_timestamps(toks, TB, 0.0, 3000, 30.0, 0)
    assert single and seek == 3000
    assert [(s["start"], s["end"]) for s in segs] == [(0.0, 1.0), (1.0, 2.4)]
    assert segs[0]["tokens"] == [TB, 10, 11, TB + 50]


def test_split_unfinished_seeks_to_last_timestamp():
    toks = [TB, 10, TB + 40, TB + 40, 11, 12]
    segs, seek, single = split_segments_by_timestamps(toks, TB, 5.0, 3000, 30.0, 500)
    assert not single
    assert len(segs) == 1 and segs[0]["start"] == 5.0 and abs(segs[0]["end"] - 5.8) < 1e-9
    assert seek == 500 + 40 * 2


def test_split_no_pairs_uses_last_timestamp_duration():
    toks = [TB, 10, 11, TB + 75]
    segs, seek, _ = split_segments_by_timestamps(toks, TB, 0.0, 2000, 20.0, 0)
    assert len(segs) == 1 and abs(segs[0]["end"] - 1.5) < 1e-9 and seek == 2000
    segs, seek, _ = split_segments_by_timestamps([10, 11], TB, 3.0, 1000, 10.0, 300)
    assert segs[0]["end"] == 13.0 and seek == 1300


def test_srt_vtt_format():
    class S:
        def __init__(self, a, b, t):
            self.start, self.end, self.text = a, b, t
    s = [S(0.0, 1.5, " hi"), S(3661.25, 3662.0, " there ")]
    assert to_srt(s) == "1\n00:00:00,000 --> 00:00:01,500\nhi\n\n2\n01:01:01,250 --> 01:01:02,000\nthere\n"
    assert to_vtt(s).startswith("WEBVTT\n\n00:00:00.000 --> 00:00:01.500\nhi\n")


# --------------------------------------------------------------------------- backend surface
def test_protocol_surface_and_lifecycle():
    b = make_backend()
    assert b.name == "faster-whisper"
    for m in ("load_model", "unload_model", "loaded_models", "is_model_loaded", "transcribe", "translate",
              "list_cached_models", "delete_cached_model", "is_model_cached"):
        assert callable(getattr(b, m))
    assert not b.is_model_loaded(MID)
    b.load_model(MID)
    t0 = b._loaded_at[MID]
    b.load_model(MID)                      # idempotent
    assert b._loaded_at[MID] == t0
    assert b.is_model_loaded(MID) and MID in b._models and MID in b._last_used
    info = b.loaded_models()[0]
    get = (lambda k: info[k]) if isinstance(info, dict) else (lambda k: getattr(info, k))
    assert get("model") == MID and get("backend") == "faster-whisper" and get("compute_type") == "float16"
    assert get("device").startswith("rocm:")
    b.unload_model(MID)
    assert not b.is_model_loaded(MID) and MID not in b._last_used and MID not in b._loaded_at
    b.unload_model(MID)                    # no-op


def test_autoload_and_last_used_refresh():
    b = make_backend()
    r = b.transcribe(wav(2.0), MID)
    assert b.is_model_loaded(MID)
    lu = b._last_used[MID]
    time.sleep(0.01)
    b.transcribe(wav(2.0), MID)
    assert b._last_used[MID] > lu
    assert set(r) == {"text"}
    b.unload_model(MID)


@pytest.mark.parametrize("fmt", ["json", "verbose_json", "text", "srt", "vtt"])
def test_response_shapes(fmt):
    b = make_backend()
    r = b.transcribe(wav(5.0), MID, response_format=fmt)
    if fmt == "verbose_json":
        assert set(r) == {"task", "language", "duration", "text", "segments"}
        assert r["task"] == "transcribe" and r["language"] == "en" and abs(r["duration"] - 5.0) < 1e-6
        seg = r["segments"][0]
        assert set(seg) == {"id", "seek", "start", "end", "text", "tokens", "temperature", "avg_logprob",
                            "compression_ratio", "no_speech_prob"}
        assert seg["id"] == 0 and seg["tokens"] == [TB, 1000, 1001, TB + 100]
        assert abs(seg["avg_logprob"] - (-1.0 / 5)) < 1e-6 and seg["end"] == 2.0
    elif fmt in ("text", "srt", "vtt"):
        assert r["raw_text"] is True and isinstance(r["text"], str)
    else:
        assert set(r) == {"text"}
    b.unload_model(MID)


def test_translate_detects_language_and_uses_translate_task():
    holder = []
    b = make_backend(holder=holder)
    r = b.translate(wav(3.0), MID, response_format="verbose_json")
    assert r["task"] == "translate"
    e = holder[0]
    assert all(c[3] == "translate" for c in e.calls)
    assert all(c[2] is None for c in e.calls)  # language detected, never forced
    b.unload_model(MID)


def test_language_forwarded_for_transcribe():
    holder = []
    b = make_backend(holder=holder)
    b.transcribe(wav(3.0), MID, language="de")
    assert holder[0].calls[0][2] == ST.first_lang + 2  # "de" is the 3rd language token
    b.unload_model(MID)


def test_seek_loop_conditions_on_previous_text():
    """First window ends mid-segment -> second window starts at the last timestamp,
    with <|startofprev|> + previous tokens as prompt prefix."""
    def script(w, i, prefix, lang):
        clip, seek, size = w
        if seek == 0:
            return WindowOutput([TB, 500, 501, TB + 600, TB + 600, 502], -0.5, 0.01, ST.first_lang)
        return WindowOutput([TB, 600, TB + 30], -0.5, 0.01, ST.first_lang)
    holder = []
    b = make_backend(script, holder)
    r = b.transcribe(wav(30.0), MID, response_format="verbose_json")
    calls = holder[0].calls
    assert calls[0][0] == (0, 0, 3000) and calls[0][1] == []
    assert calls[1][0] == (0, 1200, 3000 - 1200)
    assert calls[1][1] == [ST.sot_prev, TB, 500, 501, TB + 600]
    assert calls[1][2] == ST.first_lang      # language fixed after detection
    assert [s["seek"] for s in r["segments"]] == [0, 1200]
    assert abs(r["segments"][1]["start"] - 12.0) < 1e-9 and abs(r["segments"][1]["end"] - 12.6) < 1e-9
    b.unload_model(MID)


def test_no_speech_window_skipped():
    b = make_backend(lambda w, i, p, l: WindowOutput([TB, 5, TB + 10], -9.0, 0.95, ST.first_lang))
    r = b.transcribe(wav(4.0), MID, response_format="verbose_json")
    assert r["segments"] == [] and r["text"] == ""
    b.unload_model(MID)


def test_concurrent_calls_are_batched():
    holder = []
    b = make_backend(holder=holder)
    b.load_model(MID)
    holder[0].step_sleep = 0.01   # (continuous default: a session step takes time, so calls overlap)
    res = [None] * 16

    def call(i):
        res[i] = b.transcribe(wav(1.0 + 0.1 * i, i), MID)

    ts = [threading.Thread(target=call, args=(i,)) for i in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert all(r is not None and "text" in r for r in res)
    assert max(holder[0].batches) > 1          # at least one multi-request batch
    b.unload_model(MID)


def test_asyncio_executor_seam():
    """main.transcribe runs the backend via loop.run_in_executor (src/main.py:305-315)."""
    b = make_backend()

    async def go():
        loop = asyncio.get_running_loop()
        return await asyncio.gather(*[loop.run_in_executor(None, lambda: b.transcribe(wav(1.0), MID))
                                      for _ in range(4)])
    out = asyncio.run(go())
    assert len(out) == 4
    b.unload_model(MID)


def test_errors_propagate():
    b = make_backend()
    with pytest.raises(Exception):
        b.transcribe(b"not audio at all", MID)
    with pytest.raises(FileNotFoundError):
        b.load_model("nonexistent-org/nonexistent-model")
    b.unload_model(MID)


class RouterStandIn:
    """Mirror of BackendRouter's fields and dispatch (src/router.py:16-72)."""

    def __init__(self):
        self._backends = {"faster-whisper": object()}
        self._default_backend = self._backends["faster-whisper"]

    def get_backend(self, model_id):
        return self._default_backend

    def transcribe(self, audio, model, **kw):
        return self.get_backend(model).transcribe(audio, model, **kw)


def test_install_into_router_seam():
    r = RouterStandIn()
    b = install(r, make_backend())
    assert r._backends["faster-whisper"] is b and r._default_backend is b
    out = r.transcribe(wav(1.0), MID, language=None, response_format="json", temperature=0.0)
    assert "text" in out
    b.unload_model(MID)


# --------------------------------------------------------------------------- audio ingest
def _wav(x, sr, ch=1, width=2):
    buf = io.BytesIO()
    with wave.open(buf, "wb") as wf:
        wf.setnchannels(ch)
        wf.setsampwidth(width)
        wf.setframerate(sr)
        wf.writeframes(x.tobytes())
    return buf.getvalue()


def test_wav_16k_mono_exact():
    pcm = synth.chirp_clip(3, 2.0)
    assert np.array_equal(pcm16_from_wav(_wav(pcm, 16000)), pcm)


def test_wav_stereo_and_resample():
    x = (np.sin(np.arange(44100) * 2 * np.pi * 440 / 44100) * 8000).astype(np.int16)
    st = np.stack([x, x], 1).reshape(-1)
    y = pcm16_from_wav(_wav(st, 44100, ch=2))
    assert abs(len(y) - 16000) <= 1 and y.dtype == np.int16
    assert abs(np.abs(y).max() - 8000) < 400


def test_non_wav_rejected_or_converted():
    with pytest.raises(ValueError):
        decode_audio_bytes(b"RIFF" + b"\x00" * 100)   # the reference tests' fake upload


# --------------------------------------------------------------------------- failover
def test_device_error_fails_over_to_other_gpu():
    """A HIP error in the second opts-group of a batch: the first group's answers stand,
    only the unanswered requests move, and they skip the failed GPU's sibling lane
    (runner.py re-queued answered requests onto a lane of the same GPU).
    Both lanes of GPU 0 fail on their second decode; whichever takes the batch fails,
    and the other never decodes."""
    from open_speech_amd._lib import OswDeviceError
    from open_speech_amd.runner import BatchRunner
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    class Eng(FakeEngine):
        def __init__(self, device, tag, fail_on_call=None):
            super().__init__(D.MICRO_TEST, device, 8,
                             lambda w, i, p, l: WindowOutput([TB, 1000 + tag, TB + 50], -1.0, 0.01, ST.first_lang))
            self.device, self.tag, self.fail_on_call, self.n_decode = device, tag, fail_on_call, 0

        def decode(self, n, cfg, prefix=None, dump_steps=0, languages=None):
            self.n_decode += 1
            if self.n_decode == self.fail_on_call:
                raise OswDeviceError("osw_decode_windows failed (-100): hipErrorLaunchFailure", -100)
            return super().decode(n, cfg, prefix, dump_steps, languages)

    a, a2, b = Eng(0, 1, fail_on_call=2), Eng(0, 1, fail_on_call=2), Eng(1, 3)
    runner = BatchRunner([a, a2, b], WhisperTokenizer(51866), max_wait_ms=300, split=False)
    try:
        from concurrent.futures import Future
        from open_speech_amd.runner import _Req
        reqs = []
        for i in range(4):
            opts = TranscribeOptions(beam_size=1, language="en" if i < 2 else "de")
            reqs.append(_Req(synth.chirp_clip(i, 4.0), opts, Future()))
        for r in reqs:
            runner.workers[0].q.put(r)   # GPU 0's queue
        res = [r.fut.result(timeout=30) for r in reqs]
        assert [sg.tokens for sg in res[0].segments] == [[TB, 1001, TB + 50]]   # group 1 answered by GPU 0
        assert all(sg.tokens == [TB, 1003, TB + 50] for r in res[2:] for sg in r.segments)  # moved to GPU 1
        assert not runner.workers[0].alive and not runner.workers[1].alive and runner.workers[2].alive
        assert a.n_decode + a2.n_decode == 2   # one batch: group 1 answered, group 2 failed
        # new work avoids the failed GPU
        assert [sg.tokens for sg in runner.transcribe(synth.chirp_clip(9, 3.0), TranscribeOptions(beam_size=1,
                language="en")).segments] == [[TB, 1003, TB + 50]]
    finally:
        runner.close()


def test_cache_listing_with_stt_model_dir(tmp_path, monkeypatch):
    """STT_MODEL_DIR holds HF-style and plainly named model dirs (reference
    src/backends/faster_whisper.py:122-195): both are listed, found and deletable."""
    (tmp_path / "models--Systran--faster-whisper-base" / "snapshots" / "x").mkdir(parents=True)
    (tmp_path / "models--Systran--faster-whisper-base" / "snapshots" / "x" / "model.bin").write_bytes(b"\0" * 2048)
    (tmp_path / "my-turbo").mkdir()
    (tmp_path / "my-turbo" / "model.bin").write_bytes(b"\0" * 4096)
    (tmp_path / ".hidden").mkdir()
    monkeypatch.setenv("STT_MODEL_DIR", str(tmp_path))
    b = make_backend()
    ids = {m["model"] for m in b.list_cached_models()}
    assert ids == {"Systran/faster-whisper-base", "my-turbo"}
    assert b.is_model_cached("Systran/faster-whisper-base") and b.is_model_cached("org/my-turbo")
    assert b.delete_cached_model("my-turbo") and not (tmp_path / "my-turbo").exists()
    monkeypatch.delenv("STT_MODEL_DIR")
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path))
    b2 = make_backend()
    assert {m["model"] for m in b2.list_cached_models()} == {"Systran/faster-whisper-base"}


def test_batcher_gap_ends_collection_early():
    """The batcher stops waiting gap_ms after the latest arrival instead of max_wait_ms
    after the first: requests queued together still form one batch, a lone request is
    not held for the whole max_wait."""
    import time as _t
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    class Eng(FakeEngine):
        def __init__(self):
            super().__init__(D.MICRO_TEST, 0, 8,
                             lambda w, i, p, l: WindowOutput([TB, 1000, TB + 50], -1.0, 0.01, ST.first_lang))
            self.batches = []

        def decode(self, n, cfg, prefix=None, dump_steps=0, languages=None):
            self.batches.append(n)
            return super().decode(n, cfg, prefix, dump_steps, languages)

    e = Eng()
    runner = BatchRunner([e], WhisperTokenizer(51866), max_wait_ms=2000, gap_ms=50)
    try:
        reqs = [_Req(synth.chirp_clip(i, 3.0), TranscribeOptions(beam_size=1, language="en"), Future())
                for i in range(3)]
        t0 = _t.monotonic()
        for r in reqs:
            runner.workers[0].q.put(r)
        for r in reqs:
            r.fut.result(timeout=30)
        assert e.batches and set(e.batches) == {3}   # every seek-loop call carries all three
        assert _t.monotonic() - t0 < 1.5   # not the 2 s max_wait
    finally:
        runner.close()


@pytest.mark.parametrize("split,want", [(True, [2, 2]), (False, [4])])
def test_split_pipelines_lanes(split, want):
    """Pipelined lanes (runner.py): 4 requests queued together on a GPU with 3 idle lanes
    go out as two batches of 2 (the first lane takes half, the next free lane the rest at
    once), so one batch can encode while the other decodes; without split, one batch."""
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    class Eng(FakeEngine):
        def __init__(self):
            super().__init__(D.MICRO_TEST, 0, 8,
                             lambda w, i, p, l: WindowOutput([TB, 1000, TB + 50], -1.0, 0.01, ST.first_lang))
            self.device = 0

        def decode(self, n, cfg, prefix=None, dump_steps=0, languages=None):
            time.sleep(0.05)
            return super().decode(n, cfg, prefix, dump_steps, languages)

    es = [Eng(), Eng(), Eng()]
    runner = BatchRunner(es, WhisperTokenizer(51866), max_wait_ms=500, gap_ms=30, split=split)
    try:
        assert len(runner.queues) == 1
        reqs = [_Req(synth.chirp_clip(i, 3.0), TranscribeOptions(beam_size=1, language="en"), Future())
                for i in range(4)]
        for r in reqs:
            runner.submit_req(r)
        for r in reqs:
            assert r.fut.result(timeout=30).segments
        assert sorted(b for e in es for b in e.batches) == want
    finally:
        runner.close()


def test_lanes_take_turns_on_the_encoder():
    """Pipelined lanes: while one lane encodes, a free lane waits for that encoder and
    then takes everything that queued meanwhile (one batch), instead of starting a
    one-request batch whose encoder would only queue behind it."""
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    class Eng(FakeEngine):
        def __init__(self):
            super().__init__(D.MICRO_TEST, 0, 8,
                             lambda w, i, p, l: WindowOutput([TB, 1000, TB + 50], -1.0, 0.01, ST.first_lang))
            self.device = 0
            self.enc_windows = []

        def encode(self, wins):
            self.enc_windows.append(len(wins))
            time.sleep(0.15)
            return super().encode(wins)

        def decode(self, n, cfg, prefix=None, dump_steps=0, languages=None):
            time.sleep(0.1)   # lane A still decodes when lane B takes its batch
            return super().decode(n, cfg, prefix, dump_steps, languages)

    es = [Eng(), Eng(), Eng()]
    runner = BatchRunner(es, WhisperTokenizer(51866), max_wait_ms=500, gap_ms=5, split=True)
    try:
        opts = TranscribeOptions(beam_size=1, language="en")
        reqs = [_Req(synth.chirp_clip(i, 3.0), opts, Future()) for i in range(5)]
        runner.submit_req(reqs[0])
        time.sleep(0.05)                  # lane A is encoding request 0
        for r in reqs[1:]:
            runner.submit_req(r)
        for r in reqs:
            assert r.fut.result(timeout=30).segments
        assert sorted(n for e in es for n in e.enc_windows) == [1, 4]
    finally:
        runner.close()


# --------------------------------------------------------------------------- session lanes
@pytest.fixture
def continuous(monkeypatch):
    monkeypatch.setenv("STT_HIP_CONTINUOUS", "1")


def test_session_lane_seek_loop(continuous):
    """The seek loop on a session lane: the second window of the clip starts at the last
    timestamp with <|startofprev|> + previous tokens and the detected language, as on the
    batch path (test_seek_loop_conditions_on_previous_text)."""
    def script(w, i, prefix, lang):
        clip, seek, size = w
        if seek == 0:
            return WindowOutput([TB, 500, 501, TB + 600, TB + 600, 502], -0.5, 0.01, ST.first_lang)
        return WindowOutput([TB, 600, TB + 30], -0.5, 0.01, ST.first_lang)
    holder = []
    b = make_backend(script, holder)
    r = b.transcribe(wav(30.0), MID, response_format="verbose_json")
    calls = holder[0].calls
    assert holder[0].batches and not any(c[0] is None for c in calls)
    assert calls[0][0] == (0, 0, 3000) and calls[0][1] == []
    assert calls[1][0] == (0, 1200, 3000 - 1200)
    assert calls[1][1] == [ST.sot_prev, TB, 500, 501, TB + 600]
    assert calls[1][2] == ST.first_lang
    assert [s["seek"] for s in r["segments"]] == [0, 1200]
    b.unload_model(MID)


def test_session_lane_matches_batch_path(monkeypatch):
    """Many concurrent multi-window requests: the continuous runner's transcripts equal the
    batch runner's for a script that depends only on the window and its prompt."""
    def script(w, i, prefix, lang):
        _, seek, size = w
        k = (seek // 7 + len(prefix)) % 5
        toks = [TB, 300 + k, 301 + k, TB + 200 + 50 * k]
        if k % 2:
            toks += [TB + 200 + 50 * k, 310 + k]   # unfinished segment: the next window seeks back
        return WindowOutput(toks, -0.3, 0.01, ST.first_lang + k % 3)

    def run(cont):
        if cont:
            monkeypatch.setenv("STT_HIP_CONTINUOUS", "1")
        else:
            monkeypatch.delenv("STT_HIP_CONTINUOUS", raising=False)
        b = make_backend(script)
        b.load_model(MID)
        res = [None] * 12

        def call(i):
            res[i] = b.transcribe(wav(20.0 + 9.0 * i, i), MID, response_format="verbose_json")
        ts = [threading.Thread(target=call, args=(i,)) for i in range(12)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        b.unload_model(MID)
        return res
    a, c = run(False), run(True)
    assert a == c
    assert sum(len(r["segments"]) for r in a) > 24


def test_session_lane_concurrent_and_fallback(continuous):
    """Concurrent requests share a lane's session (several windows decode at once);
    temperature > 0 goes through the batched seek loop of an idle lane."""
    holder = []
    b = make_backend(holder=holder)
    b.load_model(MID)
    holder[0].step_sleep = 0.01
    res = [None] * 16

    def call(i):
        res[i] = b.transcribe(wav(1.0 + 0.1 * i, i), MID, temperature=0.7 if i % 5 == 0 else 0.0)
    ts = [threading.Thread(target=call, args=(i,)) for i in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert all(r is not None and "text" in r for r in res)
    e = holder[0]
    assert max(e.batches) > 1
    assert any(c[0] is not None and c[3] == "transcribe" for c in e.calls)
    b.unload_model(MID)


def test_session_lane_bad_window_fails_only_its_request():
    """A window the session refuses fails its own request; the others complete."""
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    class Eng(FakeEngine):
        def session_add(self, wins):
            if len(wins[0]["pcm"]) == 16000 * 2:
                raise ValueError("refused")
            return super().session_add(wins)

    e = Eng(D.MICRO_TEST, 0, 4)
    runner = BatchRunner([e], WhisperTokenizer(51866), continuous=True)
    try:
        opts = TranscribeOptions(beam_size=5, language="en")
        reqs = [_Req(synth.chirp_clip(i, 2.0 if i == 3 else 3.0), opts, Future()) for i in range(6)]
        for r in reqs:
            runner.submit_req(r)
        for i, r in enumerate(reqs):
            if i == 3:
                with pytest.raises(ValueError):
                    r.fut.result(timeout=30)
            else:
                assert r.fut.result(timeout=30).segments
        assert e.sessions >= 1
    finally:
        runner.close()


def test_session_lane_device_error_fails_over():
    """A HIP error in a session step moves the lane's in-flight requests to the other GPU."""
    from concurrent.futures import Future
    from open_speech_amd._lib import OswDeviceError
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    class Eng(FakeEngine):
        def __init__(self, device, tag, fail=False):
            super().__init__(D.MICRO_TEST, device, 8,
                             lambda w, i, p, l: WindowOutput([TB, 1000 + tag, TB + 50], -1.0, 0.01, ST.first_lang))
            self.device, self.fail = device, fail

        def session_step(self, max_chunks=1, refill_min=1):
            if self.fail:
                raise OswDeviceError("osw_session_step failed (-100): hipErrorLaunchFailure", -100)
            return super().session_step(max_chunks, refill_min)

    a, b = Eng(0, 1, fail=True), Eng(1, 3)
    runner = BatchRunner([a, b], WhisperTokenizer(51866), continuous=True)
    try:
        reqs = [_Req(synth.chirp_clip(i, 3.0), TranscribeOptions(language="en"), Future()) for i in range(3)]
        for r in reqs:
            runner.workers[0].q.put(r)
        for r in reqs:
            assert [sg.tokens for sg in r.fut.result(timeout=30).segments] == [[TB, 1003, TB + 50]]
        assert not runner.workers[0].alive and runner.workers[1].alive
    finally:
        runner.close()


def test_session_lane_device_error_two_lanes_per_gpu():
    """GPU 0 has two lanes, both with windows in flight; one fails with a device
    error.  fail_device marks both dead; the healthy sibling's unanswered requests go to
    GPU 1 instead of failing with 'runner closed'.  Every request is answered."""
    from concurrent.futures import Future
    from open_speech_amd._lib import OswDeviceError
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    armed, fired = threading.Event(), []
    lock = threading.Lock()

    class Eng(FakeEngine):
        def __init__(self, device, tag, max_batch):
            super().__init__(D.MICRO_TEST, device, max_batch,
                             lambda w, i, p, l: WindowOutput([TB, 1000 + tag, TB + 50], -1.0, 0.01, ST.first_lang))
            self.device, self.step_sleep = device, 0.02
            self.began = threading.Event()

        def session_step(self, max_chunks=1, refill_min=1):
            if max_chunks:
                self.began.set()
            with lock:
                fire = self.device == 0 and armed.is_set() and not fired
                if fire:
                    fired.append(self)
            if fire:
                raise OswDeviceError("osw_session_step failed (-100): hipErrorLaunchFailure", -100)
            return super().session_step(max_chunks, refill_min)

    l0, l1, b = Eng(0, 1, 2), Eng(0, 1, 2), Eng(1, 3, 8)
    runner = BatchRunner([l0, l1, b], WhisperTokenizer(51866), continuous=True, split=False)
    try:
        opts = TranscribeOptions(language="en")
        # long clips (many windows each): two requests per lane of GPU 0 (max_batch 2)
        reqs = [_Req(synth.chirp_clip(i, 120.0), opts, Future()) for i in range(4)]
        with runner.queues[0].cv:
            for r in reqs:
                r.t_enq = time.monotonic()
                runner.queues[0].items.append(r)
            runner.queues[0].cv.notify_all()
        assert l0.began.wait(10) and l1.began.wait(10)
        assert all(not r.fut.done() for r in reqs)
        armed.set()
        for r in reqs:
            res = r.fut.result(timeout=60)
            assert res.segments and all(sg.tokens in ([TB, 1001, TB + 50], [TB, 1003, TB + 50]) for sg in res.segments)
        assert fired and not runner.workers[0].alive and not runner.workers[1].alive and runner.workers[2].alive
        # the sibling that did not fail had requests in flight: they finished on GPU 1
        sib = l1 if fired[0] is l0 else l0
        assert sib.calls and b.calls
        assert sum(any(sg.tokens == [TB, 1003, TB + 50] for sg in r.fut.result().segments) for r in reqs) >= 3
    finally:
        runner.close()


def test_capture_error_is_not_a_device_fault():
    """an OSW_ECAPTURE error (a refused / invalidated stream capture) fails the
    requests of that call only; the GPU is not marked dead and keeps serving."""
    from concurrent.futures import Future
    from open_speech_amd._lib import OswCaptureError
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    assert not BatchRunner.is_device_error(OswCaptureError("osw_decode_windows failed (-102): x", -102))
    assert not BatchRunner.is_device_error(RuntimeError(
        "osw_decode_windows failed (-100): hipGetLastError(): operation failed due to a previous error during capture"))

    class Eng(FakeEngine):
        def __init__(self, device):
            super().__init__(D.MICRO_TEST, device, 4)
            self.device, self.n = device, 0

        def session_step(self, max_chunks=1, refill_min=1):
            self.n += 1
            if self.n == 2:
                raise OswCaptureError("osw_session_step failed (-102): operation would make the legacy stream "
                                      "depend on a capturing blocking stream", -102)
            return super().session_step(max_chunks, refill_min)

    a, b = Eng(0), Eng(1)
    runner = BatchRunner([a, b], WhisperTokenizer(51866), continuous=True)
    try:
        r1 = _Req(synth.chirp_clip(1, 3.0), TranscribeOptions(language="en"), Future())
        runner.workers[0].q.put(r1)
        with pytest.raises(OswCaptureError):
            r1.fut.result(timeout=10)
        assert runner.workers[0].alive and runner.queues[0].alive
        r2 = _Req(synth.chirp_clip(2, 3.0), TranscribeOptions(language="en"), Future())
        runner.workers[0].q.put(r2)
        assert r2.fut.result(timeout=10).segments
        assert not b.calls    # nothing moved to the other GPU
    finally:
        runner.close()


@pytest.mark.parametrize("busy_admit", ["1", "0"])
def test_busy_lane_admits_a_request_that_waited(monkeypatch, busy_admit):
    """while another lane of the GPU encodes, a busy session lane keeps decoding
    instead of admitting — but a request that has waited max_pace_ms is admitted by the
    busy lane beside the running encoder (STT_HIP_BUSY_ADMIT=0: it waits for the encoder)."""
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    monkeypatch.setenv("STT_HIP_BUSY_ADMIT", busy_admit)
    slow_admit = threading.Event()

    class Eng(FakeEngine):
        def session_step(self, max_chunks=1, refill_min=1):
            if max_chunks == 0 and self.tag == "slow" and slow_admit.is_set():
                time.sleep(0.6)          # a long encoder on this lane
            return super().session_step(max_chunks, refill_min)

    busy, slow = Eng(D.MICRO_TEST, 0, 4), Eng(D.MICRO_TEST, 0, 4)
    busy.device = slow.device = 0                # two lanes of one GPU: one queue, one encoder count
    busy.tag, slow.tag = "busy", "slow"
    busy.step_sleep = slow.step_sleep = 0.005
    # spread_ms: the busy lane leaves a fresh request to the idle sibling (which then encodes)
    runner = BatchRunner([busy, slow], WhisperTokenizer(51866), continuous=True, max_pace_ms=50, spread_ms=1000)
    try:
        opts = TranscribeOptions(language="en")
        long_req = _Req(synth.chirp_clip(1, 300.0), opts, Future())   # keeps one lane busy (10 windows)
        runner.submit_req(long_req)
        deadline = time.monotonic() + 5
        while not (busy.batches or slow.batches) and time.monotonic() < deadline:
            time.sleep(0.002)
        busy_eng = busy if busy.batches else slow
        other = slow if busy_eng is busy else busy
        other.tag, busy_eng.tag = "slow", "busy"
        busy_eng.step_sleep = 0.1                # its 10 windows keep it busy for seconds
        slow_admit.set()
        first = _Req(synth.chirp_clip(2, 3.0), opts, Future())
        runner.submit_req(first)                 # the idle lane takes it and encodes slowly
        time.sleep(0.05)
        t0 = time.monotonic()
        late = _Req(synth.chirp_clip(3, 3.0), opts, Future())
        runner.submit_req(late)
        late.fut.result(timeout=10)
        waited = time.monotonic() - t0
        busy_still = not long_req.fut.done()
        if busy_admit == "1":
            assert waited < 0.45, waited          # admitted by the busy lane after ~max_pace_ms
        else:
            assert waited > 0.45, waited          # only after the slow encoder finished
        first.fut.result(timeout=10)
        assert busy_still                        # the other lane was busy throughout
        long_req.fut.result(timeout=30)
    finally:
        runner.close()


def test_session_lane_close_drains_flights():
    """closing the runner (unload_model) lets a session lane finish the requests
    it is decoding instead of failing them with 'runner closed'."""
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    e = FakeEngine(D.MICRO_TEST, 0, 4)
    e.step_sleep = 0.01
    runner = BatchRunner([e], WhisperTokenizer(51866), continuous=True)
    reqs = [_Req(synth.chirp_clip(i, 60.0), TranscribeOptions(language="en"), Future()) for i in range(2)]
    for r in reqs:
        runner.submit_req(r)
    deadline = time.monotonic() + 10
    while not e.batches and time.monotonic() < deadline:
        time.sleep(0.005)
    assert e.batches, "the lane never started decoding"
    runner.close()
    for r in reqs:
        assert r.fut.result(timeout=1).segments
    assert e.closed


def test_session_lane_error_before_flight_fails_taken_requests():
    """An error while opening the session (before the taken requests are in flight) fails
    those requests instead of dropping them (a request is never left unanswered)."""
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    class Eng(FakeEngine):
        def session_begin(self, cfg):
            raise ValueError("cannot open")

    runner = BatchRunner([Eng(D.MICRO_TEST, 0, 4)], WhisperTokenizer(51866), continuous=True)
    try:
        reqs = [_Req(synth.chirp_clip(i, 3.0), TranscribeOptions(language="en"), Future()) for i in range(3)]
        for r in reqs:
            runner.submit_req(r)
        for r in reqs:
            with pytest.raises(ValueError, match="cannot open"):
                r.fut.result(timeout=10)
    finally:
        runner.close()


def test_session_lane_switches_keys():
    """Requests of two decode configurations on one lane: the lane's session takes its own
    key's requests, stops admitting once a request of the other key waited max_pace_ms,
    drains and opens a session for the other key; every request is answered."""
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    class Eng(FakeEngine):
        def __init__(self):
            super().__init__(D.MICRO_TEST, 0, 4)
            self.cfgs = []
            self.step_sleep = 0.002

        def session_begin(self, cfg):
            self.cfgs.append(cfg.beam_size)
            return super().session_begin(cfg)

    e = Eng()
    runner = BatchRunner([e], WhisperTokenizer(51866), continuous=True, max_pace_ms=20)
    try:
        reqs = [_Req(synth.chirp_clip(i, 3.0), TranscribeOptions(language="en", beam_size=5 if i % 2 else 1), Future())
                for i in range(12)]
        for r in reqs:
            runner.submit_req(r)
        for r in reqs:
            assert r.fut.result(timeout=30).segments
        assert set(e.cfgs) == {1, 5} and len(e.cfgs) >= 2
    finally:
        runner.close()


def test_session_lane_bad_option_fails_only_its_request():
    """An unsupported language fails its own request; the lane's other requests, already
    decoding in the same session, complete."""
    from concurrent.futures import Future
    from open_speech_amd.runner import BatchRunner, _Req
    from open_speech_amd.segments import TranscribeOptions
    from open_speech_amd.tokenizer import WhisperTokenizer

    e = FakeEngine(D.MICRO_TEST, 0, 4)
    e.step_sleep = 0.005
    runner = BatchRunner([e], WhisperTokenizer(51866), continuous=True)
    try:
        good = [_Req(synth.chirp_clip(i, 3.0), TranscribeOptions(language="en"), Future()) for i in range(3)]
        bad = _Req(synth.chirp_clip(9, 3.0), TranscribeOptions(language="en"), Future())
        bad.opts.language = "xx"   # same key as the good ones is not required: key() includes language
        for r in good[:2]:
            runner.submit_req(r)
        time.sleep(0.02)
        runner.submit_req(bad)
        runner.submit_req(good[2])
        for r in good:
            assert r.fut.result(timeout=30).segments
        with pytest.raises(ValueError, match="unsupported language"):
            bad.fut.result(timeout=30)
    finally:
        runner.close()
