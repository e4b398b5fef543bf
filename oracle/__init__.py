"""CPU oracle for the Whisper contextual-biasing hot path — TEST INFRASTRUCTURE ONLY.

This package is the checker, never the product: only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import it. The shipped path (`whisper_context_biasing_amd`)
never imports anything from here and fails loudly when its HIP library is missing.

Contents (each function cites the reference / [tf] file:line it restates):
  * `whisper_np`  — numpy float32 restatement of log-mel, encoder, KV-cached decoder, greedy
                    generate (HF semantics), bias-list Aho-Corasick boost, beam search.
  * `bias_ref`    — pure-Python Aho-Corasick automaton defining the boost operator (A8).
  * `wce_ref`     — numpy restatement of the bias-weighted cross entropy (`whisper_medical.py:113-156`).
  * `metric_ref`  — pure-Python WER / bias-WER restatement of `utils/compute_metric.py`.

Pinning: `whisper_np` is checked against golden vectors produced by importing the reference model
class (`models/whisper_medical.py`) and HF's feature extractor in the survey container
(`tests/golden/make_golden.py`); `metric_ref` against the reference's own `results/*.txt` dumps.
The A8 boost for λ > 0 has no reference implementation: parity unpinned.
"""
