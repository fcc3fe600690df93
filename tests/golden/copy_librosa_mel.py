"""Copy the librosa mel filterbanks the reference ships as data into tests/golden/librosa_mel_filters.npz.

The reference's qwen_tts/core/tokenizer_25hz/vq/assets/mel_filters.npz holds the output of
librosa.filters.mel(sr=16000, n_fft=400, n_mels=80 / 128) (defaults: htk=False, norm="slaney", fmin=0, fmax=sr/2;
its generating call is quoted at qwen_tts/core/tokenizer_25hz/vq/whisper_encoder.py:47-53).  librosa is absent
offline, so these two matrices are the only librosa-made vectors available: they pin the slaney mel filterbank that
the speaker encoder front end restates (M:435-437).  Loaded with allow_pickle=False; arrays are re-saved as-is.
"""
import os
import sys

import numpy as np

SRC = "/root/reference/qwen_tts/core/tokenizer_25hz/vq/assets/mel_filters.npz"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librosa_mel_filters.npz")

if __name__ == "__main__":
    src = sys.argv[1] if len(sys.argv) > 1 else SRC
    with np.load(src, allow_pickle=False) as f:
        arrs = {k: f[k] for k in ("mel_80", "mel_128")}
    np.savez_compressed(DST, **arrs)
    print(DST, {k: v.shape for k, v in arrs.items()})
