"""Real-speech fixture: the vendored pyannote `sample.wav` (30 s, 16 kHz, 2 speakers; MIT licence, pyannote-audio,
egs/mlc_slm/dicow/pyannote-audio/LICENSE in the reference) and its `sample.rttm`, stored as DATA so the GPU box
(which has no /root/reference) can run the frontend parity tests on real speech.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_sample_fixture.py
"""
import os
import wave

import numpy as np

REF = os.environ.get("SDIAR_REFERENCE", "/root/reference")
SRC = os.path.join(REF, "egs/mlc_slm/dicow/pyannote-audio/pyannote/audio/sample")
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    with wave.open(os.path.join(SRC, "sample.wav")) as w:
        assert (w.getnchannels(), w.getsampwidth(), w.getframerate()) == (1, 2, 16000)
        pcm = np.frombuffer(w.readframes(w.getnframes()), dtype="<i2").copy()
    rttm = open(os.path.join(SRC, "sample.rttm")).read()
    np.savez_compressed(os.path.join(HERE, "sample_wav.npz"), pcm16=pcm, sample_rate=np.int64(16000),
                        rttm=np.array(rttm), source=np.array("pyannote-audio sample.wav / sample.rttm (MIT licence)"))
    print("sample_wav.npz", pcm.shape, pcm.dtype)


if __name__ == "__main__":
    main()
