"""The C ABI's concurrency contract (include/osw.h) under a stream capture in progress.

GPUTEST_r05 recorded a sibling lane's synchronous legacy-stream hipMemcpy
(osw_get_encoder_output) invalidating another lane's decode-graph capture.  These tests
hold a capture open deterministically (osw_debug_hold_capture: the same locks as a
decode-graph capture, for a fixed time) while another thread calls the entry points the
reference's serving pattern reaches concurrently (src/main.py:305, src/streaming.py:50-52)
and the on-demand model load (src/backends/faster_whisper.py:210-215): every call must
succeed, the held capture must not be invalidated, and the results must equal the same
calls made with no capture in progress.  Each test runs once; nothing is repeated."""
import threading
import time

import numpy as np
import pytest

from open_speech_amd import dims as D
from open_speech_amd import ingest, synth
from open_speech_amd.engine import DecodeConfig, WhisperEngine

pytestmark = pytest.mark.gpu

HOLD_MS = 1500


def _holder(eng, hold_ms, box):
    def run():
        box["t0"] = time.monotonic()
        try:
            eng.hold_capture(hold_ms)
        except Exception as e:  # noqa: BLE001 - reported by the test
            box["err"] = e
        box["t1"] = time.monotonic()
    t = threading.Thread(target=run)
    t.start()
    return t


def test_calls_beside_a_held_capture():
    d = D.TINY_TEST
    eng = WhisperEngine(d, device=0, max_batch=2)
    try:
        eng.init_random(seed=1234)
        sib = eng.sibling()
        clip_a, clip_b = synth.chirp_clip(3, 30.0), synth.chirp_clip(4, 12.0)
        cfg = DecodeConfig(max_length=64)
        # reference results, nothing capturing
        sib.log_mel([clip_a])
        sib.encode([(0, 0, 3000)])
        enc_ref = sib.encoder_output(0)
        w_ref = sib.get_weight("dec.l0.fc1.w")
        sib.log_mel([clip_b])
        sib.encode([(0, 0, 1201)])
        dec_ref = sib.decode(1, cfg)
        pcm = synth.chirp_clip(5, 2.0)
        gain_ref = ingest.normalize_pcm16(pcm)
        sib.log_mel([clip_a])
        sib.encode([(0, 0, 3000)])

        box = {}
        t = _holder(eng, HOLD_MS, box)
        time.sleep(0.3)   # the holder is inside its capture
        t_start = time.monotonic()
        # ungated calls run during the capture (own non-blocking stream)
        assert np.array_equal(sib.encoder_output(0), enc_ref)
        assert np.array_equal(sib.get_weight("dec.l0.fc1.w"), w_ref)
        during = time.monotonic() - t_start
        # gated calls (a larger clip than any before: log_mel grows its buffers; the first
        # decode of a new key captures a graph; a new context; weight upload; ingest)
        sib.log_mel([synth.chirp_clip(6, 95.0)])
        sib.log_mel([clip_b])
        sib.encode([(0, 0, 1201)])
        out = sib.decode(1, cfg)
        other = WhisperEngine(D.MICRO_TEST, device=0, max_batch=1)
        other.init_random(seed=7)
        other.set_weight("dec.pos", np.zeros((D.MICRO_TEST.n_text_ctx, D.MICRO_TEST.n_text_state), np.float32))
        other.close()
        gain = ingest.normalize_pcm16(pcm)
        t.join(timeout=60)
        assert not t.is_alive()
        assert "err" not in box, f"the held capture failed: {box.get('err')}"
        assert during < HOLD_MS / 1000.0 - 0.3, f"ungated calls waited for the capture ({during:.3f} s)"
        assert [o.tokens for o in out] == [o.tokens for o in dec_ref]
        assert np.array_equal(gain, gain_ref)
        sib.close()
    finally:
        eng.close()


def test_backend_loads_a_second_model_while_serving(monkeypatch):
    """The on-demand load (src/backends/faster_whisper.py:210-215 auto-loads a model id on
    its first transcribe) of a second model while the first serves concurrent requests
    through its 3 lanes (beam 5, continuous batching: decode graphs are being captured).
    Every request succeeds and equals the same request made alone."""
    from open_speech_amd.backend import HipWhisperBackend

    for k in ("STT_HIP_BEAM_SIZE", "STT_HIP_LANES", "STT_HIP_CONTINUOUS", "STT_HIP_MAX_BATCH"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("STT_HIP_GPUS", "0")
    m1, m2 = "random:micro-test:11", "random:micro-test:12"
    b = HipWhisperBackend()
    b.load_model(m1)
    try:
        wavs = [synth.to_wav_bytes(synth.chirp_clip(70 + i, 8.0 + 6 * i)) for i in range(4)]
        res, errs = [None] * len(wavs), []

        def go(i):
            try:
                res[i] = b.transcribe(wavs[i], m1, response_format="verbose_json")
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        ts = [threading.Thread(target=go, args=(i,)) for i in range(len(wavs))]
        for t in ts:
            t.start()
        time.sleep(0.05)
        r2 = b.transcribe(wavs[0], m2, response_format="verbose_json")   # auto-loads m2 meanwhile
        for t in ts:
            t.join(timeout=300)
        assert not errs, errs
        alone = [b.transcribe(w, m1, response_format="verbose_json") for w in wavs]
        assert [[s["tokens"] for s in r["segments"]] for r in res] == [[s["tokens"] for s in r["segments"]]
                                                                      for r in alone]
        assert r2["segments"] is not None
        assert [s["tokens"] for s in b.transcribe(wavs[0], m2, response_format="verbose_json")["segments"]] == \
            [s["tokens"] for s in r2["segments"]]
    finally:
        for m in list(b._models):
            b.unload_model(m)
