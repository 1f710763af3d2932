"""BASELINE configs[4] (/v1/audio/stream) as a GPU test: concurrent streaming sessions
driven through the reference's control flow against the drop-in backend on the
benchmarked model, and every call's result checked against a cold single call.

The session driver is bench.stream_sessions (the same code the bench's `streaming`
figure comes from): 100 ms chunks arriving in real time, the scripted VAD of the
reference's own tests (tests/test_streaming_session_runtime.py:53-58: speech, then
silence), the growing utterance re-transcribed on every chunk while speech is active
(_transcribe_utterance, src/streaming.py:357-420: response_format json, temperature
0, utterances < 0.1 s skipped), the final call after 300 ms of silence
(_finalize_utterance :422-481), all through a 4-thread executor like
_streaming_executor (:50-52).  The backend batches the concurrent calls on the GPU;
what a session gets back must not depend on that batching."""
import pytest

from open_speech_amd.backend import HipWhisperBackend

pytestmark = pytest.mark.gpu
MID = "random:large-v3-turbo"


@pytest.mark.parametrize("sessions,speech_s,max_batch", [(8, 2.0, "8"), (32, 6.0, None)])
def test_streaming_sessions_equal_cold_single_calls(monkeypatch, sessions, speech_s, max_batch):
    """(8, 2 s, max batch 8): a quick form.  (32, 6 s, backend defaults): BASELINE
    configs[4] at its stated size, ~2000 calls, every one re-checked cold."""
    import bench
    if max_batch:
        monkeypatch.setenv("STT_HIP_MAX_BATCH", max_batch)
    else:
        monkeypatch.delenv("STT_HIP_MAX_BATCH", raising=False)
    monkeypatch.setenv("STT_HIP_GPUS", "0")
    be = HipWhisperBackend(length_control=bench.LENGTH_CONTROL_TPS)  # random weights never emit <|endoftext|>
    try:
        rec = []
        stats = bench.stream_sessions(sessions, speech_s, model=MID, backend=be, record=rec)
        print("streaming", sessions, "sessions:", stats)
        assert stats["transcriptions"] == len(rec) > sessions
        assert {i for i, _, _ in rec} == set(range(sessions))     # every session was served
        assert stats["final_transcript_lag_p50_s"] is not None
        # the reference's beam_size 5 (backend default), same bytes, nothing else in flight
        for i, wav, got in rec:
            cold = be.transcribe(audio=wav, model=MID, language=None, response_format="json", temperature=0.0)
            assert cold == got, (i, len(wav))
            assert set(got) == {"text"}
    finally:
        be.unload_model(MID)
