"""Test infrastructure shared by tools/make_hf_longform_pin.py and
tests/test_oracle_hf_longform.py: the position-scheduled logit bias that gives a
random-weight Whisper a varied long-form transcript.

Random hash weights collapse to one repeated token and never emit <|endoftext|> or a
second timestamp, so a seek loop over them only ever takes one path (one segment per
window, seek += window).  Both decoders under comparison (transformers' long-form
``generate`` and the oracle's seek loop) add the same bias to the model's logits at
every decoder position p: a +12 pull toward <|endoftext|> (p % 17 == 9), toward a
timestamp (p % 6 == 4) or toward a hashed text token (otherwise).  The Whisper logits
rules still apply on top, so windows end in timestamp pairs, single timestamp endings,
<|endoftext|> and max_length, and the seek moves by partial windows."""
import numpy as np

BIAS = 12.0


def bias_row(p: int, st, n_vocab: int) -> np.ndarray:
    b = np.zeros(n_vocab, np.float32)
    h = (p * 2654435761) % 1000003
    if p % 17 == 9:
        b[st.eot] = BIAS
    elif p % 6 == 4:
        b[st.timestamp_begin + (p * 7) % 1200] = BIAS
    else:
        b[200 + h % 20000] = BIAS
    return b
