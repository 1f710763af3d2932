#!/usr/bin/env python3
"""Which fp16 storage point dominates the logits error at whisper-large-v3-turbo dims?

CPU only (the oracle in numpy): the fp32 oracle is the reference; each variant rounds
activations to fp16 at a subset of the HIP path's storage points (oracle.model
ROUND_POINTS).  Decoding is teacher-forced on the fp32 greedy tokens so every variant
sees the same history; the error is max |log_softmax(variant) - log_softmax(fp32)| over
the whole vocabulary per step (the norm the north-star "logits within 1e-3" check uses).

Usage: python tools/precision_study.py [--steps 12] [--seed 0]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import osw_path  # noqa: E402

osw_path.load()
from open_speech_amd import dims as D  # noqa: E402
from open_speech_amd import synth, weights  # noqa: E402
from oracle import decode as odec  # noqa: E402
from oracle import mel as omel  # noqa: E402
from oracle.model import ROUND_POINTS, WhisperOracle  # noqa: E402

ENC_POINTS = ("mel", "conv1", "enc_ln", "enc_qkv", "enc_p", "enc_attn", "enc_fc1", "enc_out")
DEC_POINTS = ("xkv", "dec_ln", "dec_qkv", "dec_attn", "dec_q", "dec_fc1", "dec_final_ln")


def lsm(x):
    return odec.log_softmax(np.asarray(x, np.float64))


def forced(orc, xkv, st, toks):
    """Raw logits at each sampled step for a fixed token history."""
    cache = orc.new_cache()
    prompt = [st.sot, st.first_lang, st.transcribe]
    out, pos = [], 0
    for t in prompt:
        lg = orc.decoder_step(t, pos, cache, xkv)
        pos += 1
    out.append(lg)
    for t in toks:
        lg = orc.decoder_step(t, pos, cache, xkv)
        pos += 1
        out.append(lg)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--emb-std", type=float, default=0.02)
    ap.add_argument("--dec-combos", action="store_true",
                    help="decoder-only subsets of rounding points (fp32 encoder output)")
    a = ap.parse_args()
    d = D.LARGE_V3_TURBO
    st = D.SpecialTokens.for_vocab(d.n_vocab)
    t0 = time.time()
    w = weights.random_weights(d, seed=a.seed, emb_std=a.emb_std)
    print(f"weights {time.time() - t0:.0f}s", flush=True)
    mel = omel.window(omel.log_mel(omel.pcm16_to_float(synth.chirp_clip(0, 30.0)), d.n_mels), 0, 3000)
    ref = WhisperOracle(d, w, fp16=False)
    t0 = time.time()
    enc32 = ref.encode(mel)
    print(f"fp32 encode {time.time() - t0:.0f}s", flush=True)
    xkv32 = ref.cross_kv(enc32)
    r = odec.greedy_from_encoder(ref, xkv32, st, opts=odec.DecodeOptions(max_length=3 + a.steps), keep_logits=a.steps)
    toks = r.tokens[:a.steps - 1]
    base = [lsm(x) for x in forced(ref, xkv32, st, toks)]
    print("fp32 greedy ids", r.tokens, "lsm range", float(base[0].min()), float(base[0].max()), flush=True)

    def report(name, orc, enc=None):
        e = orc.encode(mel) if enc is None else enc
        lg = forced(orc, orc.cross_kv(e), st, toks)
        err = [float(np.abs(lsm(x) - b).max()) for x, b in zip(lg, base)]
        ee = float(np.abs(e - enc32).max())
        print(f"{name:28s} enc max|d| {ee:.3e}  lsm max|d| per step max {max(err):.3e} mean {np.mean(err):.3e}",
              flush=True)
        return e

    if a.dec_combos:
        combos = {
            "GEMM inputs fp32 (keep qkv,q,attn fp16)": ("xkv", "dec_qkv", "dec_q", "dec_attn"),
            "GEMM inputs+attn out fp32 (keep qkv,q)": ("xkv", "dec_qkv", "dec_q"),
            "only xkv+K/V cache fp16": ("xkv", "dec_qkv"),
            "only xkv fp16": ("xkv",),
            "all but final_ln+fc1": ("xkv", "dec_ln", "dec_qkv", "dec_attn", "dec_q"),
            "all but ln+final_ln": ("xkv", "dec_qkv", "dec_attn", "dec_q", "dec_fc1"),
            "fp32 ln,attn,fc1 (final_ln,q,K/V fp16)": ("xkv", "dec_qkv", "dec_q", "dec_final_ln"),
            "fp32 ln,attn,fc1,final_ln (q,K/V fp16)": ("xkv", "dec_qkv", "dec_q"),
            "fp32 ln,fc1,final_ln (attn,q,K/V fp16)": ("xkv", "dec_qkv", "dec_q", "dec_attn"),
            "fp32 all but K/V cache, xkv": ("xkv", "dec_qkv"),
        }
        only = os.environ.get("PREC_ONLY")
        for nm, pts in combos.items():
            if only and only not in nm:
                continue
            report(nm, WhisperOracle(d, w, fp16=pts), enc=enc32)
        return
    encs = {}
    encs["all"] = report("all points (round-1 GPU)", WhisperOracle(d, w, fp16=ROUND_POINTS))
    report("GPU points (hi/lo decoder)", WhisperOracle(d, w, fp16=True))
    report("encoder points only", WhisperOracle(d, w, fp16=ENC_POINTS))
    report("decoder points only", WhisperOracle(d, w, fp16=DEC_POINTS), enc=enc32)
    for p in ENC_POINTS:
        report(f"all but {p}", WhisperOracle(d, w, fp16=ROUND_POINTS - {p}))
    for p in DEC_POINTS:
        report(f"all but {p}", WhisperOracle(d, w, fp16=ROUND_POINTS - {p}), enc=encs["all"] if p != "xkv" else None)


if __name__ == "__main__":
    main()
