"""End-to-end through the drop-in backend on the GPU (real engine, random weights)."""
import threading
import time

import numpy as np
import pytest

from open_speech_amd import synth
from open_speech_amd.backend import HipWhisperBackend

pytestmark = pytest.mark.gpu
MID = "random:tiny-test:1234"


@pytest.fixture(scope="module")
def backend():
    import os
    os.environ["STT_HIP_MAX_BATCH"] = "4"
    b = HipWhisperBackend()
    b.load_model(MID)
    yield b
    b.unload_model(MID)


def test_verbose_json_end_to_end(backend):
    r = backend.transcribe(synth.to_wav_bytes(synth.chirp_clip(2, 30.0)), MID, response_format="verbose_json")
    assert r["task"] == "transcribe" and abs(r["duration"] - 30.0) < 1e-6
    assert isinstance(r["language"], str) and len(r["language"]) >= 2
    for s in r["segments"]:
        # timestamps are window-relative offsets (not clamped to the duration, as upstream)
        assert 0.0 <= s["start"] <= s["end"]
        assert all(0 <= t < 51866 for t in s["tokens"])
        assert s["temperature"] == 0.0 and 0.0 <= s["no_speech_prob"] <= 1.0


def test_concurrent_equals_sequential(backend):
    wavs = [synth.to_wav_bytes(synth.chirp_clip(30 + i, 7.0 + 5 * i)) for i in range(5)]
    seq = [backend.transcribe(w, MID, response_format="verbose_json") for w in wavs]
    par = [None] * len(wavs)

    def go(i):
        par[i] = backend.transcribe(wavs[i], MID, response_format="verbose_json")
    ts = [threading.Thread(target=go, args=(i,)) for i in range(len(wavs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for a, b in zip(seq, par):
        assert [s["tokens"] for s in a["segments"]] == [s["tokens"] for s in b["segments"]]
        assert a["language"] == b["language"]


def test_silence_and_short_clips(backend):
    for pcm in (synth.silence_clip(2.0), synth.tone_clip(0.2), np.zeros(1600, np.int16)):
        r = backend.transcribe(synth.to_wav_bytes(pcm), MID, response_format="verbose_json")
        assert "segments" in r


@pytest.mark.parametrize("variant", ["greedy", "tokenizer_prompt"])
def test_backend_verbose_json_matches_oracle_seek_loop(monkeypatch, tmp_path, variant):
    """SURVEY §8a rows a1/a5 through the boundary: HipWhisperBackend.transcribe (WAV bytes
    in, the reference's verbose_json out, src/backends/faster_whisper.py:249-270) on a 75 s
    clip, greedy, with every window the backend's runner encoded and decoded checked
    against the oracle's generate_segments restatement (oracle/seek.py) decoding the GPU's
    own encoder output, and the returned segments equal to the oracle's.
    "tokenizer_prompt": the model is a transformers-layout directory (config.json,
    model.safetensors, tokenizer.json: tests/tokfix.py) at micro dims, the request carries
    a prompt (faster-whisper initial_prompt): the first window's prompt is
    [<|startofprev|>] + encode(" " + prompt), the non-speech set comes from the
    tokenizer, and every segment's text / compression_ratio are the tokenizer's."""
    import zlib

    import tokfix
    from oracle import decode as odec
    from oracle import seek as oseek
    from oracle.model import WhisperOracle
    from open_speech_amd import dims as D
    from open_speech_amd import model_store, weights
    from open_speech_amd.engine import WhisperEngine
    from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens

    class Recorder:  # the engine seam the runner drives; records encoder outputs and decode calls
        def __init__(self, eng):
            self.eng, self.enc, self.calls, self._wins = eng, {}, [], []

        def __getattr__(self, k):
            return getattr(self.eng, k)

        def encode(self, wins):
            self._wins = list(wins)
            self.eng.encode(wins)
            for k, (_c, seek, size) in enumerate(wins):
                self.enc[(seek, size)] = self.eng.encoder_output(k)

        def decode(self, n, cfg, prefix=None, dump_steps=0, languages=None):
            outs = self.eng.decode(n, cfg, prefix=prefix, languages=languages)
            for k, w in enumerate(self._wins):
                self.calls.append((w[1], w[2], list(prefix[k]) if prefix else [], outs[k]))
            return outs

    recs = []

    def factory(dims, gpu, max_batch):
        r = Recorder(WhisperEngine(dims, device=gpu, max_batch=max_batch))
        recs.append(r)
        return r

    if variant == "greedy":
        mid, prompt = MID, None
    else:
        mid, prompt = tokfix.make_hf_model_dir(str(tmp_path / "micro_hf"), D.MICRO_TEST), "  Budget review, part two. "
    monkeypatch.setenv("STT_HIP_BEAM_SIZE", "1")
    monkeypatch.setenv("STT_HIP_CONTINUOUS", "0")  # batch at a time: the recorder sees encode/decode
    monkeypatch.setenv("STT_HIP_MAX_BATCH", "2")
    monkeypatch.setenv("STT_HIP_GPUS", "0")
    monkeypatch.setenv("STT_HIP_LANES", "1")  # one lane: every window goes through the recorder
    b = HipWhisperBackend(engine_factory=factory)
    b.load_model(mid)
    try:
        pcm = synth.chirp_clip(41, 75.0)
        r = b.transcribe(synth.to_wav_bytes(pcm), mid, response_format="verbose_json", prompt=prompt)
    finally:
        b.unload_model(mid)
    assert len(recs) == 1
    rec = recs[0]
    assert len(rec.calls) >= 3, "a 75 s clip needs at least three 30 s windows"
    if variant == "greedy":
        d = D.TINY_TEST
        w = weights.random_weights(d, seed=1234)  # the values init_random(seed=1234) writes on the device
        tok = WhisperTokenizer(d.n_vocab)
    else:
        src = model_store.resolve(mid)
        d, w = src.dims, model_store.load_weights(src)
        tok = WhisperTokenizer(d.n_vocab, src.tokenizer_json)
        assert tok.has_text
    st = tok.special
    sup = get_suppressed_tokens(tok, [-1])
    init = tok.encode(" " + prompt.strip()) if prompt else []
    orc = WhisperOracle(d, w, fp16=True)
    gpu = {(s, z): (p, o) for s, z, p, o in rec.calls}
    lang = {}

    def decode_window(seek, size, prompt_toks):
        enc = rec.enc[(seek, size)]
        o = odec.greedy_from_encoder(orc, orc.cross_kv(enc), st, language=lang.get("tok"),
                                     prev_tokens=prompt_toks[1:], opts=odec.DecodeOptions(suppress_tokens=sup))
        lang.setdefault("tok", o.language)
        gp, go = gpu[(seek, size)]
        assert gp == prompt_toks, f"window {seek}: prompt differs"
        assert go.tokens == o.tokens, f"window {seek}: ids differ from the oracle's"
        return go.tokens, go.sum_logprob, go.no_speech_prob

    nf = (len(pcm) + 160) // 160
    wins = oseek.seek_loop(decode_window, nf, st, tok.decode, initial_tokens=init)
    if prompt:
        assert wins[0].prompt == [st.sot_prev] + init
    want = [(a, b_, t) for x in wins for a, b_, t in x.segments]
    got = [(s["start"], s["end"], s["tokens"]) for s in r["segments"]]
    assert [(round(a, 6), round(e, 6), t) for a, e, t in got] == [(round(a, 6), round(e, 6), t) for a, e, t in want]
    assert r["task"] == "transcribe" and r["duration"] == pytest.approx(75.0)
    assert [s["id"] for s in r["segments"]] == list(range(len(r["segments"])))
    # text fields: the tokenizer's decode of each segment, the window text's compression ratio
    for s in r["segments"]:
        assert s["text"] == tok.decode(s["tokens"])
        wt = tok.decode(gpu[(s["seek"], next(z for sk, z in gpu if sk == s["seek"]))][1].tokens).strip().encode()
        assert s["compression_ratio"] == (len(wt) / len(zlib.compress(wt)) if wt else 0.0)
    assert r["text"] == "".join(s["text"] for s in r["segments"]).strip()


def test_backend_default_config_matches_oracle_seek_loop(monkeypatch, tmp_path):
    """The batch-at-a-time backend (STT_HIP_CONTINUOUS=0), its defaults otherwise (STT_HIP_BEAM_SIZE 5 = the reference's
    beam_size, src/backends/faster_whisper.py:237; 3 lanes per GPU; max batch 16; the
    batcher's 1 ms gap), three concurrent requests (75, 61 and 47 s WAVs) so the batcher
    spreads windows over the lanes and batches windows of different clips.  Every lane is
    recorded; each request's windows are replayed through the oracle's seek loop with the
    oracle's CTranslate2-BeamSearch restatement (width 5) decoding the GPU's own encoder
    output: every prompt and every window's ids must equal the oracle's, and each response's
    segments the oracle's.  Model: micro dims with the synthetic tokenizer (tests/tokfix.py),
    so the numpy beam oracle stays fast over full 448-position windows."""
    import hashlib

    import tokfix
    from oracle import decode as odec
    from oracle import seek as oseek
    from oracle.model import WhisperOracle
    from open_speech_amd import dims as D
    from open_speech_amd import model_store
    from open_speech_amd.engine import WhisperEngine
    from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens

    for k in ("STT_HIP_BEAM_SIZE", "STT_HIP_LANES", "STT_HIP_MAX_BATCH", "STT_HIP_BATCH_GAP_MS",
              "STT_HIP_BATCH_WAIT_MS"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("STT_HIP_GPUS", "0")
    monkeypatch.setenv("STT_HIP_CONTINUOUS", "0")  # batch at a time (the continuous form: below)

    calls = []              # (clip hash, seek, size, prompt, output, encoder output) over every lane
    lock = threading.Lock()

    class Recorder:
        def __init__(self, eng):
            self.eng, self._clips, self._wins = eng, [], []

        def __getattr__(self, k):
            return getattr(self.eng, k)

        def sibling(self, max_batch=None):
            return Recorder(self.eng.sibling(max_batch))

        def log_mel(self, clips, *a, **kw):
            self._clips = [hashlib.sha1(np.asarray(c, np.int16).tobytes()).hexdigest() for c in clips]
            return self.eng.log_mel(clips, *a, **kw)

        def encode(self, wins):
            self._wins = list(wins)
            self.eng.encode(wins)
            self._enc = [self.eng.encoder_output(k) for k in range(len(wins))]

        def decode(self, n, cfg, prefix=None, dump_steps=0, languages=None):
            assert cfg.beam_size == 5, "the backend's default decoding is beam search width 5"
            outs = self.eng.decode(n, cfg, prefix=prefix, languages=languages)
            with lock:
                for k, (c, seek, size) in enumerate(self._wins):
                    calls.append((self._clips[c], seek, size, list(prefix[k]) if prefix else [], outs[k],
                                  self._enc[k]))
            return outs

    def factory(dims, gpu, max_batch):
        return Recorder(WhisperEngine(dims, device=gpu, max_batch=max_batch))

    mid = tokfix.make_hf_model_dir(str(tmp_path / "micro_hf"), D.MICRO_TEST)
    b = HipWhisperBackend(engine_factory=factory)
    b.load_model(mid)
    clips = [synth.chirp_clip(51 + i, s) for i, s in enumerate((75.0, 61.0, 47.0))]
    res = [None] * len(clips)
    try:
        def go(i):
            res[i] = b.transcribe(synth.to_wav_bytes(clips[i]), mid, response_format="verbose_json")
        engines = list(b._models[mid].engines)
        ts = [threading.Thread(target=go, args=(i,)) for i in range(len(clips))]
        for t in ts:
            t.start()
            time.sleep(0.05)    # later requests arrive while the first lane is busy: other lanes take them
        for t in ts:
            t.join(timeout=600)
    finally:
        b.unload_model(mid)
    assert len(engines) == 3 and all(r is not None for r in res)
    src = model_store.resolve(mid)
    d, w = src.dims, model_store.load_weights(src)
    tok = WhisperTokenizer(d.n_vocab, src.tokenizer_json)
    st = tok.special
    sup = get_suppressed_tokens(tok, [-1])
    orc = WhisperOracle(d, w, fp16=True)
    by_key = {}
    for h, seek, size, p, o, enc in calls:
        by_key.setdefault((h, seek, size), []).append((p, o, enc))
    for pcm, r in zip(clips, res):
        h = hashlib.sha1(pcm.tobytes()).hexdigest()
        lang = {}

        def decode_window(seek, size, prompt_toks):
            (gp, go, enc), = by_key[(h, seek, size)]
            o = odec.beam_from_encoder(orc, orc.cross_kv(enc), st, language=lang.get("tok"),
                                       prev_tokens=prompt_toks[1:], opts=odec.DecodeOptions(suppress_tokens=sup),
                                       beam=odec.BeamOptions(beam_size=5))
            lang.setdefault("tok", o.language)
            assert gp == prompt_toks, f"{len(pcm)} samples, window {seek}: prompt differs"
            assert go.tokens == o.tokens, f"{len(pcm)} samples, window {seek}: ids differ from the oracle's"
            return go.tokens, go.sum_logprob, go.no_speech_prob

        wins = oseek.seek_loop(decode_window, (len(pcm) + 160) // 160, st, tok.decode)
        want = [(round(a, 6), round(e, 6), t) for x in wins for a, e, t in x.segments]
        got = [(round(s["start"], 6), round(s["end"], 6), s["tokens"]) for s in r["segments"]]
        assert got == want
    # the three requests' windows went through more than one lane
    assert sum(1 for e in engines if e._wins) >= 2


def test_backend_continuous_matches_oracle_seek_loop(monkeypatch, tmp_path):
    """Continuous batching as deployed (the default, STT_HIP_CONTINUOUS=1, runner._SessionLane):
    the backend's defaults (beam 5, 3 lanes, max batch 16), four concurrent requests
    (75, 61, 47 and 12 s WAVs) arriving while earlier ones decode, so windows of different
    requests and seek positions share a lane's decode session and join it between chunks
    of steps.  Every window a session admitted is recorded (prompt, result); its encoder
    output is recomputed on a separate context (a window's encoder output does not depend
    on its batch: test_tile_sizes_bit_identical) and each request's windows are replayed
    through the oracle's seek loop with the oracle's beam search (width 5): every prompt
    and every window's ids must equal the oracle's, each response's segments the
    oracle's."""
    import hashlib

    import tokfix
    from oracle import decode as odec
    from oracle import seek as oseek
    from oracle.model import WhisperOracle
    from open_speech_amd import dims as D
    from open_speech_amd import model_store
    from open_speech_amd.engine import WhisperEngine
    from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens

    for k in ("STT_HIP_BEAM_SIZE", "STT_HIP_LANES", "STT_HIP_MAX_BATCH", "STT_HIP_BATCH_GAP_MS",
              "STT_HIP_BATCH_WAIT_MS", "STT_HIP_SPREAD_MS", "STT_HIP_REFILL_MIN"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("STT_HIP_GPUS", "0")
    monkeypatch.setenv("STT_HIP_CONTINUOUS", "1")

    added, done, shared = {}, {}, []
    lock = threading.Lock()

    class Recorder:
        def __init__(self, eng):
            self.eng = eng
            self.tags = {}
            self.clip_hash = {}

        def __getattr__(self, k):
            return getattr(self.eng, k)

        def sibling(self, max_batch=None):
            return Recorder(self.eng.sibling(max_batch))

        def session_begin(self, cfg):
            assert cfg.beam_size == 5, "the backend's default decoding is beam search width 5"
            return self.eng.session_begin(cfg)

        def session_add(self, wins):
            with lock:
                for w in wins:
                    # a request's first window brings its PCM; later ones only its clip key
                    if w.get("pcm") is not None:
                        self.clip_hash[w["clip"]] = hashlib.sha1(np.asarray(w["pcm"], np.int16).tobytes()).hexdigest()
                    h = self.clip_hash[w["clip"]]
                    self.tags[w["tag"]] = (h, w["seek"], w["segment_size"])
                    added[(h, w["seek"], w["segment_size"])] = list(w["prefix"] or [])
            return self.eng.session_add(wins)

        def session_step(self, max_chunks=1, refill_min=1):
            res, active, queued = self.eng.session_step(max_chunks, refill_min)
            with lock:
                shared.append(active + len(res))
                for tag, out in res:
                    done[self.tags[tag]] = out
            return res, active, queued

    def factory(dims, gpu, max_batch):
        return Recorder(WhisperEngine(dims, device=gpu, max_batch=max_batch))

    mid = tokfix.make_hf_model_dir(str(tmp_path / "micro_hf"), D.MICRO_TEST)
    b = HipWhisperBackend(engine_factory=factory)
    b.load_model(mid)
    clips = [synth.chirp_clip(61 + i, s) for i, s in enumerate((75.0, 61.0, 47.0, 12.0))]
    res = [None] * len(clips)
    try:
        def go(i):
            res[i] = b.transcribe(synth.to_wav_bytes(clips[i]), mid, response_format="verbose_json")
        ts = [threading.Thread(target=go, args=(i,)) for i in range(len(clips))]
        for t in ts:
            t.start()
            time.sleep(0.02)
        for t in ts:
            t.join(timeout=600)
    finally:
        b.unload_model(mid)
    assert all(r is not None for r in res)
    assert max(shared) >= 2, "windows of different requests decoded in one session"
    src = model_store.resolve(mid)
    d, w = src.dims, model_store.load_weights(src)
    tok = WhisperTokenizer(d.n_vocab, src.tokenizer_json)
    st = tok.special
    sup = get_suppressed_tokens(tok, [-1])
    orc = WhisperOracle(d, w, fp16=True)
    eng = WhisperEngine(d, device=0, max_batch=1)
    try:
        eng.load_weights(w)
        for pcm, r in zip(clips, res):
            h = hashlib.sha1(pcm.tobytes()).hexdigest()
            eng.log_mel([pcm])
            lang = {}

            def decode_window(seek, size, prompt_toks):
                key = (h, seek, size)
                assert key in done, f"{len(pcm)} samples, window {seek}: not decoded by a session"
                eng.encode([(0, seek, size)])
                enc = eng.encoder_output(0)
                o = odec.beam_from_encoder(orc, orc.cross_kv(enc), st, language=lang.get("tok"),
                                           prev_tokens=prompt_toks[1:], opts=odec.DecodeOptions(suppress_tokens=sup),
                                           beam=odec.BeamOptions(beam_size=5))
                lang.setdefault("tok", o.language)
                go_ = done[key]
                assert added[key] == prompt_toks, f"{len(pcm)} samples, window {seek}: prompt differs"
                assert go_.tokens == o.tokens, f"{len(pcm)} samples, window {seek}: ids differ from the oracle's"
                return go_.tokens, go_.sum_logprob, go_.no_speech_prob

            wins = oseek.seek_loop(decode_window, (len(pcm) + 160) // 160, st, tok.decode)
            want = [(round(a, 6), round(e, 6), t) for x in wins for a, e, t in x.segments]
            got = [(round(s["start"], 6), round(s["end"], 6), s["tokens"]) for s in r["segments"]]
            assert got == want
    finally:
        eng.close()
