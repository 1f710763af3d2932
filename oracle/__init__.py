"""ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU (numpy) restatement of the arithmetic the reference delegates to
faster-whisper 1.2.1 + CTranslate2 (pinned at /root/reference/requirements.lock:7;
neither package is vendored in /root/reference nor installed in this image).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker / CPU baseline.  The product path
(``open-speech_amd/``) never imports it and fails loudly when the HIP library is
missing.

Parity pinning: the reference's own tests pin no numbers for this path
(SURVEY.md §8c).  This restatement is pinned against golden vectors produced by
an independent implementation of the same published algorithm — transformers
5.15.0's ``WhisperFeatureExtractor`` and ``WhisperForConditionalGeneration`` — by
``tools/make_golden.py`` (fixtures in ``tests/golden/``).  Against faster-whisper
itself parity is UNPINNED (the package cannot be run here).
"""
