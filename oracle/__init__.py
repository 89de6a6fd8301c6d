"""CPU oracle — TEST INFRASTRUCTURE ONLY.

A restatement of the reference algorithms (shanguanma/speaker_diarization) on
the host CPU, used as the parity checker by tests/, by __graft_entry__.smoke()
and as the cpu_baseline leg of bench.py.  Nothing in speaker_diarization_amd/
imports this package; the product path runs only the HIP library.

Pinning: tests/golden/ holds outputs of the reference modules themselves
(imported from /root/reference in the build container by
tests/golden/make_golden.py) on seeded inputs/weights; tests/test_oracle.py
checks this restatement against them.  Components whose reference arithmetic
lives in a package absent from the container (torchaudio 2.5.1 kaldi.fbank and
models.Conformer, librosa 0.10.2) are restated from their published algorithms
and marked "parity unpinned" where they are used.
"""
