#!/usr/bin/env python3
"""Throughput bench: whisper-large-v3-turbo transcription on MI355X.

A "step" = one pass of the hot path (log-mel -> encoder -> cross-K/V -> greedy
decode with Whisper's logits rules) over one batch of `--batch` synthetic 30 s
16 kHz clips per GPU (BASELINE.json configs[2]; configs[3] is the same per-GPU shard
at N=8).  With N>1 ranks (torchrun, one process per GPU) rank 0 holds every clip
in HBM and the step starts with an RCCL scatter of the int16 PCM and ends with an
RCCL gather of the token ids.  ``--gpus N`` alone starts the N
ranks itself (torch.distributed.run on 127.0.0.1, before this process touches the
GPU); under torchrun, WORLD_SIZE must equal ``--gpus`` or the bench exits non-zero.

Prints ONE JSON line (rank 0).  value = audio seconds transcribed per wall second
over all ranks (max-over-ranks time).  Weights are random (no checkpoint is
available offline) and decoding runs to <|endoftext|> or max_length, so tokens
per clip are reported beside the number.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth  # noqa: E402
from open_speech_amd.distributed import REFILL_MIN  # noqa: E402
from open_speech_amd.engine import DecodeConfig, WhisperEngine  # noqa: E402
from open_speech_amd.tokenizer import WhisperTokenizer, get_suppressed_tokens  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X spec (MI355X_MICROARCH.md)
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense fp16 MFMA spec
VALU_F32_PEAK_TFLOPS = 157.3   # fp32 vector spec (MI355X_MICROARCH.md)
# VALU flops of mel_logmel_kernel per frame (csrc/mel.hip): stage 1, 25 real 16-point DFTs
# (16 window mults, 9 bins x 16 x 2 FMA, 16 complex twiddles) = 25 x 688; stage 2, 201 bins x
# 25 complex MACs x 8 + 201 x 3 (power); stage 3, the slaney bank's 394 taps (128 mels) x 2 +
# 128 log10 + 128 max
MEL_FLOPS_PER_FRAME = 25 * 688 + 201 * 25 * 8 + 201 * 3 + 394 * 2 + 2 * 128


# length control of the serving benches (HipWhisperBackend(length_control=...)): random
# weights never emit <|endoftext|>, so each window ends after 4 tokens per second of audio
LENGTH_CONTROL_TPS = 4.0

def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20,
                    help="timed 64-clip steps; the first ~3 fill the lanes' pipeline (measured, r03_ac: "
                         "6 steps 4942, 12 steps 5043, 24 steps 5099 audio-s/s)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=64, help="30 s clips per GPU per step")
    ap.add_argument("--lanes", type=int, default=3,
                    help="contexts per GPU sharing one weight copy; consecutive steps overlap on them "
                         "(measured, 12 steps x 2 runs: 2 lanes 4023, 3 lanes 4234, 4 lanes 4057 audio-s/s)")
    ap.add_argument("--model", default="large-v3-turbo", choices=sorted(D.PRESETS))
    ap.add_argument("--max-length", type=int, default=448)
    ap.add_argument("--latency-repeats", type=int, default=50,
                    help="batch-1 latency (BASELINE configs[1]): timed repeats after --latency-warmup (SURVEY §8d: 50 + 5)")
    ap.add_argument("--latency-warmup", type=int, default=5)
    ap.add_argument("--beam5-latency-repeats", type=int, default=20,
                    help="batch-1 latency with the reference's beam_size=5 (after --latency-warmup)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--beam5", type=int, default=1, help="also time one isolated beam-5 step (the reference default)")
    ap.add_argument("--beam5-steps", type=int, default=3,
                    help="also time this many beam-5 steps on the lanes (after the greedy timed region)")
    ap.add_argument("--cpu-decode-steps", type=int, default=0,
                    help="decoder steps of the CPU baseline; 0 = the whole per-clip decode of the GPU run")
    ap.add_argument("--stream-sessions", type=int, default=32,
                    help="BASELINE configs[4]: concurrent /v1/audio/stream sessions simulated through the backend "
                         "(0 = skip)")
    ap.add_argument("--rest-callers", type=int, default=16,
                    help="mixed-length REST load, continuous vs batch-at-a-time (0: skip)")
    ap.add_argument("--rest-calls", type=int, default=8, help="calls per REST caller")
    ap.add_argument("--stream-speech-s", type=float, default=6.0, help="seconds of speech per streaming session")
    ap.add_argument("--refill-min", type=int, default=REFILL_MIN,
                    help="row refill (realistic lengths): admit queued clips once this many rows are free")
    ap.add_argument("--realistic-steps", type=int, default=9,
                    help="also time this many steps with realistic output lengths (random weights never emit "
                         "<|endoftext|>: each clip's length is forced from a seeded distribution)")
    ap.add_argument("--pmc-summary", default=os.path.join(ROOT, "profiles", "r06_s2j_pmc.json"),
                    help="per-kernel HBM bytes from a rocprofv3 --pmc pass (tools/pmc_summary.py)")
    ap.add_argument("--standin", action="store_true",
                    help="launcher test only: ranks run a CPU stand-in engine over gloo (no GPU, no HIP library)")
    return ap.parse_args(argv)


def spawn_ranks(n: int, argv: list) -> int:
    """``--gpus N`` (N > 1) outside a torchrun environment: start the N rank processes
    here, one per GPU, as children of torch.distributed.run on 127.0.0.1, and return
    their exit status.  Called before this process imports the HIP library or makes
    any torch.cuda call (a process that has touched the GPU must not exec or hand its
    device over).  Only rank 0 prints the JSON line, so the children's stdout is this
    process's stdout."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


class StandInEngine:
    """--standin: rank r takes (r + 1) x 40 ms per batch and decodes r + 1 tokens per
    clip, so the launcher test sees the slow rank set the max-over-ranks time."""

    def __init__(self, rank: int):
        self.rank = rank

    def transcribe_batch(self, clips, cfg, device_pcm=None, offsets=None):
        class _Out:
            tokens = list(range(self.rank + 1))
        time.sleep(0.04 * (self.rank + 1))
        return [_Out() for _ in clips]

    def sibling(self):
        return StandInEngine(self.rank)

    def close(self):
        pass


def make_clips(n: int, offset: int = 0, unique: int = 32) -> np.ndarray:
    """n synthetic clips; at most `unique` distinct ones (cycled) to bound host time."""
    base = [synth.chirp_clip(offset + i, 30.0) for i in range(min(n, unique))]
    return np.stack([base[i % len(base)] for i in range(n)])


def cpu_baseline(dims, n_tokens_per_clip: float, decode_steps: int) -> dict:
    """The oracle (numpy restatement, fp32) on the host cores: one clip's log-mel +
    encoder + decoder steps, as audio-s/s.  decode_steps <= 0 (the default): the whole
    decode the GPU run did per clip (3 prompt steps + its mean tokens), every step timed
    with its growing self-K/V cache; > 0: that many steps, scaled.  Test infrastructure
    used only as the reported CPU baseline."""
    from oracle import mel as omel
    from oracle.model import WhisperOracle
    from open_speech_amd import weights

    try:
        from threadpoolctl import threadpool_info
        cores = max((i.get("num_threads", 1) for i in threadpool_info()), default=1)
    except Exception:
        cores = os.cpu_count() or 1
    # same shapes/dtypes as the GPU run; values from a fast RNG (timing only)
    rng = np.random.default_rng(0)
    w = {}
    for sp in weights.canonical_specs(dims):
        shp = weights.spec_shape(sp, dims)
        w[sp.name] = (rng.standard_normal(shp, dtype=np.float32) * 0.02).astype(
            np.float16 if sp.dtype == weights.F16 else np.float32)
    orc = WhisperOracle(dims, w, fp16=False)
    del w
    st = D.SpecialTokens.for_vocab(dims.n_vocab)
    pcm = synth.chirp_clip(0, 30.0)
    t0 = time.perf_counter()
    mel = omel.log_mel(omel.pcm16_to_float(pcm), dims.n_mels)
    t1 = time.perf_counter()
    enc = orc.encode(mel[:, :3000].astype(np.float32))
    xkv = orc.cross_kv(enc)
    t2 = time.perf_counter()
    full = decode_steps <= 0
    if full:
        decode_steps = int(round(3 + n_tokens_per_clip))
    cache = orc.new_cache()
    toks = [st.sot, st.first_lang, st.transcribe] + [st.timestamp_begin] * max(0, decode_steps - 3)
    for p, t in enumerate(toks[:decode_steps]):
        orc.decoder_step(t, p, cache, xkv)
    t3 = time.perf_counter()
    per_step = (t3 - t2) / max(1, decode_steps)
    per_clip = (t1 - t0) + (t2 - t1) + per_step * (3 + n_tokens_per_clip)
    how = (f"all {decode_steps} decoder steps (the GPU run's per-clip mean), {t3 - t2:.2f}s, not extrapolated"
           if full else f"{decode_steps} decoder steps ({per_step * 1e3:.0f} ms/step), scaled to "
                        f"{3 + n_tokens_per_clip:.0f} decoder steps per clip (the GPU run's mean)")
    return {"value": round(30.0 / per_clip, 4), "unit": "audio-sec/sec", "cores": int(cores), "kind": "port",
            "sample": f"oracle (numpy fp32) on 1 x 30 s clip: log-mel {t1 - t0:.2f}s + encoder+crossKV "
                      f"{t2 - t1:.2f}s + {how}"}


def rest_mixed(callers: int, calls: int, model: str = "random:large-v3-turbo") -> dict:
    """Mixed-length REST load on the drop-in backend (tools/rest_probe.py ... mix): `callers`
    threads each post `calls` WAVs of 4-75 s (1-3 windows) through transcribe() with
    exponentially distributed think time (mean 40 ms), once with continuous batching (the
    default, runner._SessionLane) and once batch at a time (STT_HIP_CONTINUOUS=0), so the
    line shows what continuous batching buys on the load it is for (src/main.py:305 calls
    transcribe() from the default executor).  Beam 5, 4 tokens/s length control."""
    import threading

    from open_speech_amd.audio import pcm_to_wav
    from open_speech_amd.backend import HipWhisperBackend

    lens = (4.0, 12.0, 30.0, 45.0, 75.0, 20.0, 8.0, 60.0)
    wavs = [pcm_to_wav(synth.chirp_clip(800 + i, x).tobytes(), 16000) for i, x in enumerate(lens)]
    out = {"callers": callers, "calls_per_caller": calls, "clip_s": list(lens), "think_ms_mean": 40}
    prev = os.environ.get("STT_HIP_CONTINUOUS")
    for mode, flag in (("continuous", "1"), ("batch_at_a_time", "0")):
        os.environ["STT_HIP_CONTINUOUS"] = flag
        be = HipWhisperBackend(length_control=LENGTH_CONTROL_TPS)
        be.load_model(model)
        be.transcribe(audio=wavs[0], model=model, language=None, response_format="json")   # warm
        lat, lock = [], threading.Lock()

        def caller(i):
            rng = np.random.default_rng(i)
            for k in range(calls):
                time.sleep(rng.exponential(0.040))
                t = time.perf_counter()
                be.transcribe(audio=wavs[(i + k) % len(wavs)], model=model, language=None, response_format="json")
                with lock:
                    lat.append(time.perf_counter() - t)

        ts = [threading.Thread(target=caller, args=(i,)) for i in range(callers)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        wall = time.perf_counter() - t0
        be.unload_model(model)
        audio = sum(lens[(i + k) % len(lens)] for i in range(callers) for k in range(calls))
        out[mode] = {"calls_per_s": round(len(lat) / wall, 2), "audio_sec_per_sec": round(audio / wall, 1),
                     "latency_p50_ms": round(1e3 * float(np.median(lat)), 1),
                     "latency_p95_ms": round(1e3 * float(np.percentile(lat, 95)), 1)}
    if prev is None:
        os.environ.pop("STT_HIP_CONTINUOUS", None)
    else:
        os.environ["STT_HIP_CONTINUOUS"] = prev
    return out


def stream_sessions(n_sessions: int, speech_s: float, model: str = "random:large-v3-turbo", backend=None,
                    record: list | None = None) -> dict:
    """BASELINE configs[4]: n concurrent streaming sessions against the drop-in backend,
    following src/streaming.py's control flow with a scripted VAD (the reference's own
    test stand-in, tests/test_streaming_session_runtime.py:53-58): 100 ms chunks arrive in
    real time; while speech is active every chunk re-transcribes the whole utterance so
    far (_transcribe_utterance, src/streaming.py:357-420: json, temperature 0, utterances
    < 0.1 s skipped) and the session awaits the call before its next chunk; 300 ms of
    silence finalises (_finalize_utterance :422-481).  Calls go through a 4-thread
    executor like _streaming_executor (:50-52), so at most 4 are in flight and the
    backend batches them across sessions.  Random weights never emit <|endoftext|>: the
    backend cuts each window at 4 tokens per second of audio (its bench-only
    ``length_control``; a backend passed in must have been built with it).  The reference's default beam_size 5 is used."""
    import asyncio
    from concurrent.futures import ThreadPoolExecutor

    from open_speech_amd.audio import pcm_to_wav
    from open_speech_amd.backend import HipWhisperBackend

    own = backend is None
    be = HipWhisperBackend(length_control=LENGTH_CONTROL_TPS) if own else backend
    be.load_model(model)
    ex = ThreadPoolExecutor(max_workers=4, thread_name_prefix="stream-transcribe")
    chunk = 1600
    silence_s, endpoint = 0.5, int(16000 * 300 / 1000)
    lat, finals = [], []

    async def session(i, t0):
        loop = asyncio.get_running_loop()
        pcm = synth.chirp_clip(500 + i, speech_s + silence_s).tobytes()
        utter, active, silence = bytearray(), False, 0

        async def call():
            if len(utter) < 3200:
                return
            wav = pcm_to_wav(bytes(utter), 16000)
            ts = time.perf_counter()
            r = await loop.run_in_executor(ex, lambda: be.transcribe(audio=wav, model=model, language=None,
                                                                     response_format="json", temperature=0.0))
            lat.append(time.perf_counter() - ts)
            if record is not None:
                record.append((i, wav, r))

        n = len(pcm) // (2 * chunk)
        for c in range(n):
            await asyncio.sleep(max(0.0, t0 + (c + 1) * 0.1 - loop.time()))   # real-time arrival
            data = pcm[c * 2 * chunk:(c + 1) * 2 * chunk]
            if c * 0.1 < speech_s:                                            # scripted VAD: speech
                if not active:
                    active, utter = True, bytearray()
                utter.extend(data)
                await call()
            elif active:
                silence += chunk
                utter.extend(data)
                if silence >= endpoint:
                    await call()
                    finals.append(loop.time() - (t0 + n * 0.1))   # lag of the final transcript
                    active, utter, silence = False, bytearray(), 0
                else:
                    await call()

    async def main():
        loop = asyncio.get_running_loop()
        t0 = loop.time() + 0.2
        await asyncio.gather(*[session(i, t0 + 1.0 * i / max(1, n_sessions)) for i in range(n_sessions)])

    wall0 = time.perf_counter()
    asyncio.run(main())
    wall = time.perf_counter() - wall0
    ex.shutdown(wait=True)
    if own:
        be.unload_model(model)
    audio = n_sessions * (speech_s + silence_s)
    return {"sessions": n_sessions, "speech_s_per_session": speech_s, "chunk_ms": 100, "executor_threads": 4,
            "transcriptions": len(lat), "transcriptions_per_s": round(len(lat) / wall, 1),
            "call_latency_p50_ms": round(1e3 * float(np.median(lat)), 1) if lat else None,
            "call_latency_p95_ms": round(1e3 * float(np.percentile(lat, 95)), 1) if lat else None,
            "final_transcript_lag_p50_s": round(float(np.median(finals)), 3) if finals else None,
            "final_transcript_lag_max_s": round(float(np.max(finals)), 3) if finals else None,
            "audio_seconds": audio, "wall_s": round(wall, 2),
            "realtime_factor": round(audio / wall, 2),
            "note": "scripted VAD (speech then 0.5 s silence), 4 tokens/s length control, beam 5, random weights"}


def ingest_timing(repeats: int = 30, device: int = 0) -> dict:
    """The GPU ingest drop-ins (open_speech_amd/ingest.py) against the host numpy / scipy
    operations the reference runs for the same calls (src/audio/preprocessing.py:53-63
    for a 30 s upload, src/streaming.py:55-91 for one 100 ms 48 kHz client chunk), both
    timed here with bytes in and bytes out (median of `repeats` after 3 warm-ups).  The
    host side is written out inline for timing only."""
    import io
    import wave

    from scipy.signal import resample_poly

    from open_speech_amd import ingest

    wav30 = synth.to_wav_bytes(synth.chirp_clip(7, 30.0))
    t = np.arange(4800) / 48000.0
    chunk = (np.sin(2 * np.pi * 1000.0 * t) * 0.5 * 32767).astype(np.int16).tobytes()

    def host_pre(wav):
        with wave.open(io.BytesIO(wav), "rb") as wf:
            sr, raw = wf.getframerate(), wf.readframes(wf.getnframes())
        a = np.frombuffer(raw, np.int16).astype(np.float32) / 32768.0
        rms = np.sqrt(np.mean(np.square(a)))
        if rms > 1e-8:
            a = np.clip(a * 10 ** ((-18.0 - 20 * np.log10(rms)) / 20), -1.0, 1.0)
        return synth.to_wav_bytes((np.clip(a, -1.0, 1.0) * 32767.0).astype(np.int16), sr)

    def host_rs(pcm):
        x = np.frombuffer(pcm, np.int16).astype(np.float32)
        return np.clip(resample_poly(x, 1, 3), -32768, 32767).astype(np.int16).tobytes()

    def med(f, arg):
        for _ in range(3):
            f(arg)
        ts = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            f(arg)
            ts.append((time.perf_counter() - t0) * 1e3)
        return round(float(np.median(ts)), 3)

    gpu_pre = lambda w: ingest.preprocess_stt_audio(w, noise_reduce=False, normalize=True, device=device)  # noqa
    gpu_rs = lambda p: ingest.resample_pcm16(p, 48000, 16000, device=device)  # noqa: E731
    return {"preprocess_30s_wav": {"gpu_ms": med(gpu_pre, wav30), "host_numpy_ms": med(host_pre, wav30)},
            "resample_100ms_48k_chunk": {"gpu_ms": med(gpu_rs, chunk), "host_scipy_ms": med(host_rs, chunk)},
            "repeats": repeats, "note": "bytes in, bytes out; host = the reference's numpy/scipy ops, one thread"}


def timed_steps(dp, allpcm, k: int, dist=None, dev=None, runner=None):
    """The bench contract's timed region: barrier + device sync on both sides of exactly
    k steps, then the MAX of the elapsed time over ranks and the SUM of tokens decoded.
    Returns (seconds, total tokens over all ranks, per-step results of this rank)."""
    import torch

    def sync():
        if dev is not None and dev.type == "cuda":
            torch.cuda.synchronize(dev)

    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    res = (runner or dp.run_steps)(allpcm, k)
    sync()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    ntok = sum(len(o.tokens) for outs, _ in res for o in outs)
    if dist:
        t = torch.tensor([el, float(ntok)], dtype=torch.float64, device=dev)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        el, ntok = float(mx[0].item()), int(t[1].item())
    return el, ntok, res


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        # one process per GPU: start the ranks ourselves (nothing here has touched the GPU)
        sys.exit(spawn_ranks(a.gpus, argv))
    world = int(env_world or "1")
    if world != a.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}; launch one rank per GPU with matching counts")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if a.standin:
        dev = torch.device("cpu")
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
    else:
        if world > 1:
            import torch.distributed as dist
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(0)
        dev = torch.device("cuda", local if world > 1 else 0)
    dims = D.PRESETS[a.model]
    B = a.batch
    sup = get_suppressed_tokens(WhisperTokenizer(dims.n_vocab), [-1])
    cfg = DecodeConfig(suppress_tokens=sup, max_length=a.max_length)
    if a.standin:
        eng = StandInEngine(rank)
    else:
        eng = WhisperEngine(dims, device=dev.index, max_batch=B)
        eng.init_random(seed=0)

    n_total = B * world
    from open_speech_amd.distributed import DataParallelTranscriber

    dp = DataParallelTranscriber(eng, cfg, dist=dist, device=dev, clips_per_rank=B, ctx=dims.n_text_ctx,
                                 lanes=1 if a.standin else a.lanes)
    # inputs resident in HBM before timing: rank 0 holds every clip
    allpcm = torch.from_numpy(make_clips(n_total)).to(dev) if rank == 0 else None

    # warm-up: every lane captures its decode graph
    dp.run_steps(allpcm, max(a.warmup, len(dp.lanes)) if a.warmup > 0 else 0)
    el, ntok, res = timed_steps(dp, allpcm, a.steps, dist, dev)

    audio_s = n_total * a.steps * 30.0
    value = audio_s / el
    tokens_per_clip = ntok / (n_total * a.steps)
    if a.standin:
        if rank == 0:
            print(json.dumps({
                "metric": "audio-sec/sec (launcher test: CPU stand-in engine, not a measurement)",
                "value": round(value, 2), "unit": "audio-sec/sec", "n_gpus": world, "steps": a.steps,
                "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 2), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "none", "data": "stand-in engine over gloo",
                "config": {"workload": "stand-in", "clips_per_gpu": B, "global_batch": n_total,
                           "parallelism": f"dp{world}"},
                "tokens_per_clip": round(tokens_per_clip, 3)}), flush=True)
        dp.close()
        if dist:
            dist.destroy_process_group()
        return
    profs = [e.profile() for e in dp.lanes]

    # Realistic output lengths: real speech gives ~2-6 tokens per second of audio (text +
    # timestamp pairs), so each clip's greedy decode is cut at a length drawn from
    # N(130, 40) clipped to [16, 440] (seeded; the same lengths on every rank) by the
    # decoder's token budget.  Finished rows skip their self / cross-attention; with row
    # refill (the default, WhisperEngine.transcribe_refill) a finished window's row takes
    # the next queued clip, so a lane's rows stay full across its steps instead of every
    # batch waiting for its longest window.  The plain per-batch path is timed beside it.
    realistic = None
    if a.realistic_steps > 0:
        lens = np.clip(np.round(np.random.default_rng(77).normal(130, 40, B)), 16, 440).astype(int)
        import dataclasses
        dp.cfg = dataclasses.replace(cfg, token_budget=tuple(int(x) for x in lens))
        dp.run_steps(allpcm, len(dp.lanes))
        rel0, rtok0, _ = timed_steps(dp, allpcm, a.realistic_steps, dist, dev)
        refill = lambda pcm, k: dp.run_steps_refill(pcm, k, refill_min=a.refill_min)  # noqa: E731
        refill(allpcm, len(dp.lanes))  # every lane captures its refill graph
        rel, rtok_all, _ = timed_steps(dp, allpcm, a.realistic_steps, dist, dev, runner=refill)
        rtok = rtok_all / (n_total * a.realistic_steps)
        realistic = {"value": round(n_total * a.realistic_steps * 30.0 / rel, 2), "unit": "audio-sec/sec",
                     "steps": a.realistic_steps, "ms_per_step": round(rel / a.realistic_steps * 1e3, 2),
                     "tokens_per_clip": round(rtok, 1), "max_tokens_per_clip": int(lens.max()),
                     "lengths": "N(130, 40) clipped to [16, 440], seed 77",
                     "row_refill": {"refill_min": a.refill_min,
                                    "steps_per_lane_call": -(-a.realistic_steps // len(dp.lanes))},
                     "no_refill": {"value": round(n_total * a.realistic_steps * 30.0 / rel0, 2),
                                   "ms_per_step": round(rel0 / a.realistic_steps * 1e3, 2),
                                   "tokens_per_clip": round(rtok0 / (n_total * a.realistic_steps), 1)}}
        dp.cfg = cfg

    # The reference's own decoding (beam_size=5, src/backends/faster_whisper.py:237) on the
    # same lanes: warm-up steps let every lane capture its beam graph, then K_b timed steps.
    beam5_lanes = None
    if a.beam5_steps > 0:
        dp.cfg = DecodeConfig(suppress_tokens=sup, max_length=a.max_length, beam_size=5)
        dp.run_steps(allpcm, len(dp.lanes))
        bel, btok_all, _ = timed_steps(dp, allpcm, a.beam5_steps, dist, dev)
        btok = btok_all / (n_total * a.beam5_steps)
        beam5_lanes = {"value": round(n_total * a.beam5_steps * 30.0 / bel, 2), "unit": "audio-sec/sec",
                       "steps": a.beam5_steps, "ms_per_step": round(bel / a.beam5_steps * 1e3, 2),
                       "lanes_per_gpu": len(dp.lanes), "tokens_per_clip": round(btok, 1)}
        dp.cfg = cfg

    if rank == 0:
        # Roofline pass, after the timed region: lane 0 alone runs one more step of the
        # same workload with per-kernel HIP-event timers on its stream and the decode
        # steps launched eagerly (inside the timed region the lanes overlap, so a
        # kernel's duration there is inflated by the other lane's kernels).
        eng.set_profiling(True, eager_decode=True)
        eng.transcribe_batch(None, cfg, device_pcm=allpcm.data_ptr(),
                             offsets=np.arange(B + 1, dtype=np.int64) * allpcm.shape[-1])
        prof = eng.profile()
        eng.set_profiling(False)
        cands = {
            "encoder_gemm": (prof["enc_gemm_ms"], prof["enc_gemm_flops"], prof["enc_gemm_launches"], "mfma"),
            "encoder_attention": (prof["enc_attn_ms"], prof["enc_attn_flops"], prof["enc_attn_launches"], "mfma"),
            "decoder_cross_attention": (prof["xattn_ms"], prof["xattn_bytes"], prof["xattn_launches"], "hbm"),
            "log_mel": (prof["mel_kernel_ms"], prof["mel_kernel_bytes"], prof["mel_kernel_launches"], "hbm"),
        }
        try:
            with open(a.pmc_summary) as fh:
                pmc_classes = json.load(fh)["classes"]
        except (OSError, KeyError, ValueError):
            pmc_classes = {}

        def roofline(name):
            ms, work, nl, bound = cands[name]
            if bound == "mfma":
                ach, peak, unit = work / (ms * 1e-3) / 1e12, MFMA_F16_PEAK_TFLOPS, "TFLOP/s"
            else:
                ach, peak, unit = work / (ms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s"
            r = {"kernel": name, "bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit,
                 "frac": round(ach / peak, 4), "traffic": None, "avg_launch_ms": round(ms / max(1, nl), 4),
                 "work_per_launch": work / max(1, nl), "launches": int(nl)}
            pmc = pmc_classes.get(name)
            if pmc:
                r["traffic"] = round(pmc["hbm_bytes_per_launch"])
                r["traffic_source"] = os.path.relpath(a.pmc_summary, ROOT)
            return r

        live = [k for k in cands if cands[k][2] > 0]
        roofs = {k: roofline(k) for k in live}
        if "log_mel" in roofs:
            # the log-mel kernel's arithmetic against the VALU fp32 peak (its bytes are ~1 % of
            # HBM time): MEL_FLOPS_PER_FRAME x 3001 frames per 30 s clip
            ms, _, nl, _ = cands["log_mel"]
            fl = MEL_FLOPS_PER_FRAME * 3001 * B * nl
            ach = fl / (ms * 1e-3) / 1e12
            roofs["log_mel"]["valu"] = {
                "bound": "valu", "achieved": round(ach, 2), "peak": VALU_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / VALU_F32_PEAK_TFLOPS, 4), "flop_per_frame": MEL_FLOPS_PER_FRAME,
                "frac_of_unpacked": round(ach / (VALU_F32_PEAK_TFLOPS / 2), 4),
                "note": "spec vector peak counts packed fp32 (v_pk_fma_f32); this library is built without "
                        "packed fp32 (csrc/Makefile NOPK), whose ceiling is half of it"}
        roof = dict(roofs[max(live, key=lambda k: cands[k][0])])
        roof["measured"] = "isolated roofline pass after the timed region (1 lane, HIP events on the lane's stream)"
        stages = {k: {"ms": round(v[0], 2), "launches": int(v[2])} for k, v in cands.items()}

        # the reference's own decoding (beam_size=5, src/backends/faster_whisper.py:237): one
        # isolated 64-clip step on lane 0, reported beside the greedy headline
        beam5 = None
        if a.beam5:
            bcfg = DecodeConfig(suppress_tokens=sup, max_length=a.max_length, beam_size=5)
            torch.cuda.synchronize(dev)
            tb = time.perf_counter()
            eng.transcribe_batch(None, bcfg, device_pcm=allpcm.data_ptr(),
                                 offsets=np.arange(B + 1, dtype=np.int64) * allpcm.shape[-1])
            beam5 = round(B * 30.0 / (time.perf_counter() - tb), 2)

        # latency of one 30 s clip at batch 1 (BASELINE configs[1]): warm-ups, then timed repeats
        one = torch.from_numpy(make_clips(1, offset=999)).to(dev)
        offs1 = np.array([0, 480000], np.int64)

        def latency(c, repeats):
            for _ in range(a.latency_warmup if repeats else 0):
                eng.transcribe_batch(None, c, device_pcm=one.data_ptr(), offsets=offs1)
            lat = []
            for _ in range(repeats):
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                eng.transcribe_batch(None, c, device_pcm=one.data_ptr(), offsets=offs1)
                lat.append((time.perf_counter() - t1) * 1e3)
            if not lat:
                return None
            return {"p50_ms": round(float(np.median(lat)), 2), "p95_ms": round(float(np.percentile(lat, 95)), 2),
                    "repeats": repeats, "warmup": a.latency_warmup}

        lat_greedy = latency(cfg, a.latency_repeats)
        lat_beam = latency(DecodeConfig(suppress_tokens=sup, max_length=a.max_length, beam_size=5),
                           a.beam5_latency_repeats)
        p50 = lat_greedy["p50_ms"] if lat_greedy else None

        stream = None
        if a.stream_sessions > 0 and world == 1:
            stream = stream_sessions(a.stream_sessions, a.stream_speech_s)

        rest = None
        if a.rest_callers > 0 and world == 1:
            rest = rest_mixed(a.rest_callers, a.rest_calls)

        ingest_t = None
        if world == 1:
            ingest_t = ingest_timing(device=dev.index)

        cpu = None
        if not a.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(dims, tokens_per_clip, a.cpu_decode_steps)

        line = {
            "metric": "audio-sec/sec (whisper-large-v3-turbo, 30 s clips, greedy)",
            "value": round(value, 2), "unit": "audio-sec/sec", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f16", "data": "synthetic (chirps+noise, random weights)",
            "config": {"workload": f"{a.model}: {B} x 30 s clips per GPU per step, mel+encoder+greedy decode "
                                   f"(max_length {a.max_length})" + (", RCCL scatter/gather" if world > 1 else ""),
                       "clips_per_gpu": B, "global_batch": n_total, "parallelism": f"dp{world}",
                       "lanes_per_gpu": len(dp.lanes)},
            "tokens_per_clip": round(tokens_per_clip, 1),
            "p50_latency_ms_b1": p50,
            "latency_b1": {"greedy": lat_greedy, "beam5": lat_beam},
            "beam5": beam5_lanes,
            "realistic_lengths": realistic,
            "streaming": stream,
            "rest_mixed": rest,
            "ingest": ingest_t,
            "beam5_audio_sec_per_sec_1lane": beam5,
            "realtime_factor": round(value, 1),
            "roofline": roof,
            "rooflines": {k: {kk: v[kk] for kk in ("achieved", "unit", "frac", "avg_launch_ms", "valu") if kk in v}
                          for k, v in roofs.items()},
            "stages_ms_roofline_pass": stages,
            "decode_steps_last_call": int(profs[0]["decode_steps"]),
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    dp.close()
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
